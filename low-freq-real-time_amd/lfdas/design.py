"""Filter design on the host, as DASCore's ``pass_filter`` does it
*(DASCore, external: dascore/proc/filter.py ``_get_sos``)*: a Butterworth
``scipy.signal.iirfilter(corners, Wn, btype, ftype='butter', output='zpk')``
converted with ``zpk2sos`` (SciPy's default 'nearest' pairing).  Design is a
one-off host computation; the filtering runs in liblfdas.so."""
from __future__ import annotations

import numpy as np
import scipy.signal as _sig


class FilterValueError(ValueError):
    """Corner frequencies outside (0, Nyquist) — DASCore's error type name."""


def pass_filter_sos(fs: float, lo, hi, corners: int = 4) -> np.ndarray:
    """SOS of ``Patch.pass_filter(time=(lo, hi), corners=corners)``: low-pass
    when ``lo`` is None, high-pass when ``hi`` is None, else band-pass."""
    nyq = 0.5 * float(fs)
    lo = None if lo is None or (isinstance(lo, float) and np.isnan(lo)) else float(lo)
    hi = None if hi is None or (isinstance(hi, float) and np.isnan(hi)) else float(hi)
    if lo is None and hi is None:
        raise FilterValueError("pass_filter needs at least one corner frequency")
    for v in (lo, hi):
        if v is not None and not (0.0 < v < nyq):
            raise FilterValueError(
                f"filter corner {v} Hz must be in (0, Nyquist={nyq} Hz)")
    if lo is not None and hi is not None and lo >= hi:
        raise FilterValueError("low corner must be below the high corner")
    if lo is None:
        z, p, k = _sig.iirfilter(corners, hi / nyq, btype="lowpass", ftype="butter", output="zpk")
    elif hi is None:
        z, p, k = _sig.iirfilter(corners, lo / nyq, btype="highpass", ftype="butter", output="zpk")
    else:
        z, p, k = _sig.iirfilter(corners, [lo / nyq, hi / nyq], btype="bandpass", ftype="butter",
                                 output="zpk")
    return _sig.zpk2sos(z, p, k)


def lowpass_sos(fs: float, fc: float, corners: int = 4) -> np.ndarray:
    return pass_filter_sos(fs, None, fc, corners)


def default_padlen(sos) -> int:
    """scipy/signal/_signaltools.py:4811-4813."""
    sos = np.asarray(sos)
    ntaps = 2 * sos.shape[0] + 1 - min(int((sos[:, 2] == 0).sum()), int((sos[:, 5] == 0).sum()))
    return 3 * ntaps
