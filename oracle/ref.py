"""ORACLE restatements (test infrastructure only — see oracle/__init__.py).

Every function cites the reference (``lf_das.py``), SciPy (``scipy/...``, under
``/usr/local/lib/python3.10/dist-packages``) or DASCore (external, absent from
this container: restated from its public API, marked *(DASCore, external)*)
code it follows.  Nothing here is imported by the product package.
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess

import numpy as np

__all__ = [
    "buttap", "lp2lp_zpk", "lp2hp_zpk", "bilinear_zpk", "iirfilter_butter_zpk",
    "zpk2sos", "butter_sos", "sosfilt_zi", "odd_ext", "sosfilt", "sosfiltfilt",
    "sosfiltfilt_ref_padlen", "interp1d_linear", "dascore_pass_filter_sos",
    "pass_filter", "interpolate", "rolling_mean", "rolling_out_times",
    "get_patch_time", "lfproc_time_grid", "lfproc_schedule", "lfproc_process",
    "down_sample_processing", "get_edge_effect_time", "have_c_oracle",
    "sosfiltfilt_rows_c", "edge_loop", "lp2bp_zpk", "cheb1ap", "cheby1_sos", "decimate_iir", "firwin_hamming", "decimate_fir",
    "median_filter", "demean_scale",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def _load_c():
    """Load (building on first use if gcc is present) the C restatement of
    SciPy's ``_sosfilt`` (oracle/csrc/sosfilt.c)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    so = os.path.join(_HERE, "_build", "liboracle.so")
    if not os.path.exists(so):
        try:
            subprocess.run(["make", "-s", "-C", _HERE], check=True,
                           capture_output=True, timeout=120)
        except Exception:  # pragma: no cover - no compiler: numpy fallback
            _LIB = False
            return _LIB
    lib = ctypes.CDLL(so)
    i64, dp, fp, ci = ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int
    lib.oracle_sosfilt_f64.argtypes = [dp, ci, dp, i64, i64, dp]
    lib.oracle_sosfilt_f64.restype = None
    lib.oracle_sosfiltfilt_rows_f32.argtypes = [dp, ci, dp, ci, fp, i64, i64, i64, dp, dp]
    lib.oracle_sosfiltfilt_rows_f32.restype = None
    _LIB = lib
    return lib


def have_c_oracle() -> bool:
    return bool(_load_c())


# ---------------------------------------------------------------------------
# Filter design (SciPy, restated)
# ---------------------------------------------------------------------------
def buttap(N: int):
    """Analog Butterworth prototype — scipy/signal/_filter_design.py:4361."""
    if abs(int(N)) != N:
        raise ValueError("Filter order must be a nonnegative integer")
    z = np.array([])
    m = np.arange(-N + 1, N, 2)
    p = -np.exp(1j * np.pi * m / (2 * N))
    return z, p, 1


def _relative_degree(z, p):
    """scipy/signal/_filter_design.py:2684."""
    degree = len(p) - len(z)
    if degree < 0:
        raise ValueError("Improper transfer function. Must have at least as many poles as zeros.")
    return degree


def lp2lp_zpk(z, p, k, wo=1.0):
    """scipy/signal/_filter_design.py:2780."""
    z = np.atleast_1d(z)
    p = np.atleast_1d(p)
    wo = float(wo)
    degree = _relative_degree(z, p)
    return wo * z, wo * p, k * wo ** degree


def lp2hp_zpk(z, p, k, wo=1.0):
    """scipy/signal/_filter_design.py:2826 (lp2hp_zpk)."""
    z = np.atleast_1d(z)
    p = np.atleast_1d(p)
    wo = float(wo)
    degree = _relative_degree(z, p)
    z_hp = wo / z
    p_hp = wo / p
    z_hp = np.append(z_hp, np.zeros(degree))
    k_hp = k * np.real(np.prod(-z) / np.prod(-p))
    return z_hp, p_hp, k_hp


def bilinear_zpk(z, p, k, fs):
    """scipy/signal/_filter_design.py:2696."""
    z = np.atleast_1d(z)
    p = np.atleast_1d(p)
    degree = _relative_degree(z, p)
    fs2 = 2.0 * fs
    z_z = (fs2 + z) / (fs2 - z)
    p_z = (fs2 + p) / (fs2 - p)
    z_z = np.append(z_z, -np.ones(degree))
    k_z = k * np.real(np.prod(fs2 - z) / np.prod(fs2 - p))
    return z_z, p_z, k_z


def lp2bp_zpk(z, p, k, wo=1.0, bw=1.0):
    """scipy/signal/_filter_design.py lp2bp_zpk: low-pass prototype → band-pass
    centred on ``wo`` with bandwidth ``bw``."""
    z = np.atleast_1d(z)
    p = np.atleast_1d(p)
    wo = float(wo)
    bw = float(bw)
    degree = _relative_degree(z, p)
    z_lp = (z * bw / 2).astype(complex)
    p_lp = (p * bw / 2).astype(complex)
    z_bp = np.concatenate((z_lp + np.sqrt(z_lp ** 2 - wo ** 2), z_lp - np.sqrt(z_lp ** 2 - wo ** 2)))
    p_bp = np.concatenate((p_lp + np.sqrt(p_lp ** 2 - wo ** 2), p_lp - np.sqrt(p_lp ** 2 - wo ** 2)))
    z_bp = np.append(z_bp, np.zeros(degree))
    return z_bp, p_bp, k * bw ** degree


def cheb1ap(N: int, rp: float):
    """scipy/signal/_filter_design.py cheb1ap: analog Chebyshev type I
    prototype (``rp`` dB ripple)."""
    if N == 0:
        return np.array([]), np.array([]), 10 ** (-rp / 20)
    z = np.array([])
    eps = np.sqrt(10 ** (0.1 * rp) - 1.0)
    mu = 1.0 / N * np.arcsinh(1 / eps)
    m = np.arange(-N + 1, N, 2)
    theta = np.pi * m / (2 * N)
    p = -np.sinh(mu + 1j * theta)
    k = np.prod(-p, axis=0).real
    if N % 2 == 0:
        k = k / np.sqrt(1 + eps * eps)
    return z, p, k


def cheby1_sos(N: int, rp: float, Wn: float):
    """``scipy.signal.cheby1(N, rp, Wn, output='sos')`` (digital low-pass):
    iirfilter's digital branch (fs = 2, prewarp) → lp2lp → bilinear → zpk2sos."""
    z, p, k = cheb1ap(N, rp)
    fs = 2.0
    warped = 2 * fs * np.tan(np.pi * float(Wn) / fs)
    z, p, k = lp2lp_zpk(z, p, k, wo=warped)
    z, p, k = bilinear_zpk(z, p, k, fs=fs)
    return zpk2sos(z, p, k)


def decimate_iir(x, q: int, axis: int = -1):
    """``scipy.signal.decimate(x, q, ftype='iir', axis=axis, zero_phase=True)``
    (scipy/signal/_signaltools.py decimate): 8th-order Chebyshev I at
    ``0.8/q``, ``sosfiltfilt``, then every q-th sample.  (DASCore's
    ``Patch.decimate(filter_type='iir')`` is restated as this call; the
    wrapper itself is external and unpinned.)  float64 data."""
    sos = cheby1_sos(8, 0.05, 0.8 / q)
    y = sosfiltfilt(sos, np.asarray(x, dtype=np.float64), axis=axis)
    sl = [slice(None)] * y.ndim
    sl[axis] = slice(None, None, q)
    return y[tuple(sl)]


def firwin_hamming(numtaps: int, cutoff: float):
    """``scipy.signal.firwin(numtaps, cutoff, window='hamming')`` (low-pass,
    scale=True; scipy/signal/_fir_filter_design.py firwin): windowed sinc
    ``cutoff * sinc(cutoff * m)``, m = n - (numtaps - 1)/2, times the
    symmetric Hamming window ``0.54 - 0.46 cos(2 pi n / (numtaps - 1))``,
    normalised to unit DC gain."""
    n = np.arange(numtaps, dtype=np.float64)
    m = n - 0.5 * (numtaps - 1)
    h = cutoff * np.sinc(cutoff * m)
    h = h * (0.54 - 0.46 * np.cos(2.0 * np.pi * n / (numtaps - 1)))
    return h / np.sum(h)


def decimate_fir(x, q: int, axis: int = -1):
    """``scipy.signal.decimate(x, q, ftype='fir', axis=axis, zero_phase=True)``
    (scipy/signal/_signaltools.py decimate) = ``resample_poly(x, 1, q,
    window=firwin(20q+1, 1/q, 'hamming'))`` (_signaltools.py resample_poly,
    padtype 'constant'): the filter is pre-padded with n_pre = q - half % q
    zeros (half = 10q), the full convolution is taken every q-th sample from
    index n_pre_remove q (n_pre_remove = (half + n_pre) // q), ceil(n/q)
    outputs; samples outside the record are zeros.  float64."""
    x = np.moveaxis(np.asarray(x, dtype=np.float64), axis, -1)
    h = firwin_hamming(20 * q + 1, 1.0 / q)
    half = (h.size - 1) // 2
    n_pre = q - half % q
    n_pre_remove = (half + n_pre) // q
    hp = np.concatenate([np.zeros(n_pre), h])
    n = x.shape[-1]
    n_out = -(-n // q)
    flat = x.reshape(-1, n)
    out = np.empty((flat.shape[0], n_out))
    idx = (n_pre_remove + np.arange(n_out)) * q
    for r in range(flat.shape[0]):
        full = np.convolve(flat[r], hp)
        full = np.concatenate([full, np.zeros(max(0, int(idx[-1]) + 1 - full.size))])
        out[r] = full[idx]
    return np.moveaxis(out.reshape(x.shape[:-1] + (n_out,)), -1, axis)


def median_filter(a, size):
    """``scipy.ndimage.median_filter(a, size=size)`` (mode 'reflect' =
    half-sample symmetric, origin 0, rank = window // 2) —
    scipy/ndimage/_filters.py median_filter → _rank_filter."""
    a = np.asarray(a)
    k = (int(size),) * a.ndim if np.ndim(size) == 0 else tuple(int(v) for v in size)
    pad = [(kk // 2, kk - 1 - kk // 2) for kk in k]
    padded = np.pad(a, pad, mode="symmetric")
    win = np.lib.stride_tricks.sliding_window_view(padded, k)
    flat = win.reshape(a.shape + (-1,))
    n = flat.shape[-1]
    return np.partition(flat, n // 2, axis=-1)[..., n // 2]


def demean_scale(data, ch_start: int, ch_end: int, scale: float):
    """low_pass_dascore.ipynb cells 14/18/22 on (time, distance) data:
    ``(data - mean(data[:, c0:c1], axis=1).reshape(-1, 1)) * scale_iDAS``."""
    data = np.asarray(data, dtype=np.float64)
    return (data - np.mean(data[:, ch_start:ch_end], axis=1).reshape(-1, 1)) * scale


def iirfilter_butter_zpk(N: int, Wn: float, btype: str = "lowpass"):
    """Digital Butterworth zpk, as scipy.signal.iirfilter(N, Wn, btype=...,
    ftype='butter', output='zpk') — scipy/signal/_filter_design.py:2443-2680
    (digital branch: fs = 2, prewarp ``warped = 2*fs*tan(pi*Wn/fs)``)."""
    z, p, k = buttap(N)
    fs = 2.0
    warped = 2 * fs * np.tan(np.pi * np.asarray(Wn, dtype=float) / fs)
    if btype in ("lowpass", "low"):
        z, p, k = lp2lp_zpk(z, p, k, wo=float(warped))
    elif btype in ("highpass", "high"):
        z, p, k = lp2hp_zpk(z, p, k, wo=float(warped))
    elif btype in ("bandpass", "band"):
        bw = warped[1] - warped[0]
        wo = np.sqrt(warped[0] * warped[1])
        z, p, k = lp2bp_zpk(z, p, k, wo=wo, bw=bw)
    else:
        raise NotImplementedError(btype)
    return bilinear_zpk(z, p, k, fs=fs)


def _cplxreal(z, tol=None):
    """scipy/signal/_filter_design.py:876 (conjugate pairing)."""
    z = np.atleast_1d(z)
    if z.size == 0:
        return z, z
    if tol is None:
        tol = 100 * np.finfo((1.0 * z).dtype).eps
    z = z[np.lexsort((abs(z.imag), z.real))]
    real_indices = abs(z.imag) <= tol * abs(z)
    zr = z[real_indices].real
    if len(zr) == len(z):
        return np.array([]), zr
    z = z[~real_indices]
    zp = z[z.imag > 0]
    zn = z[z.imag < 0]
    if len(zp) != len(zn):
        raise ValueError("Array contains complex value with no matching conjugate.")
    same_real = np.diff(zp.real) <= tol * abs(zp[:-1])
    diffs = np.diff(np.concatenate(([0], same_real, [0])))
    run_starts = np.nonzero(diffs > 0)[0]
    run_stops = np.nonzero(diffs < 0)[0]
    for i in range(len(run_starts)):
        start = run_starts[i]
        stop = run_stops[i] + 1
        for chunk in (zp[start:stop], zn[start:stop]):
            chunk[...] = chunk[np.lexsort([abs(chunk.imag)])]
    zc = (zp + zn.conj()) / 2
    return zc, zr


def _single_zpksos(z, p, k):
    """scipy/signal/_filter_design.py:1367 via zpk2tf (:1135)."""
    sos = np.zeros(6)
    b = k * np.real(np.poly(z)) if len(z) else np.array([float(k)])
    a = np.real(np.poly(p)) if len(p) else np.array([1.0])
    sos[3 - len(b):3] = b
    sos[6 - len(a):6] = a
    return sos


def _nearest_real_complex_idx(fro, to, which):
    """scipy/signal/_filter_design.py:1354."""
    order = np.argsort(np.abs(fro - to))
    if which == "any":
        return order[0]
    mask = np.isreal(fro[order])
    if which == "complex":
        mask = ~mask
    return order[np.nonzero(mask)[0][0]]


def zpk2sos(z, p, k):
    """Digital zpk → sos with SciPy's default 'nearest' pairing —
    scipy/signal/_filter_design.py:1376-1661.  The pole closest to the unit
    circle goes into the LAST section; the gain multiplies section 0."""
    z = np.asarray(z)
    p = np.asarray(p)
    if len(z) == len(p) == 0:
        return np.array([[k, 0.0, 0.0, 1.0, 0.0, 0.0]])
    p = np.concatenate((p, np.zeros(max(len(z) - len(p), 0))))
    z = np.concatenate((z, np.zeros(max(len(p) - len(z), 0))))
    n_sections = (max(len(p), len(z)) + 1) // 2
    if len(p) % 2 == 1:
        p = np.concatenate((p, [0.0]))
        z = np.concatenate((z, [0.0]))
    z = np.concatenate(_cplxreal(z))
    p = np.concatenate(_cplxreal(p))
    k = float(np.real(k))

    def idx_worst(pp):
        return np.argmin(np.abs(1 - np.abs(pp)))

    sos = np.zeros((n_sections, 6))
    for si in range(n_sections - 1, -1, -1):
        p1_idx = idx_worst(p)
        p1 = p[p1_idx]
        p = np.delete(p, p1_idx)
        if np.isreal(p1) and np.isreal(p).sum() == 0:
            z1_idx = _nearest_real_complex_idx(z, p1, "real")
            z1 = z[z1_idx]
            z = np.delete(z, z1_idx)
            sos[si] = _single_zpksos([z1, 0], [p1, 0], 1)
        elif (len(p) + 1 == len(z) and not np.isreal(p1)
              and np.isreal(p).sum() == 1 and np.isreal(z).sum() == 1):
            z1_idx = _nearest_real_complex_idx(z, p1, "complex")
            z1 = z[z1_idx]
            z = np.delete(z, z1_idx)
            sos[si] = _single_zpksos([z1, z1.conj()], [p1, p1.conj()], 1)
        else:
            if np.isreal(p1):
                prealidx = np.flatnonzero(np.isreal(p))
                p2_idx = prealidx[idx_worst(p[prealidx])]
                p2 = p[p2_idx]
                p = np.delete(p, p2_idx)
            else:
                p2 = p1.conj()
            if len(z) > 0:
                z1_idx = _nearest_real_complex_idx(z, p1, "any")
                z1 = z[z1_idx]
                z = np.delete(z, z1_idx)
                if not np.isreal(z1):
                    sos[si] = _single_zpksos([z1, z1.conj()], [p1, p2], 1)
                elif len(z) > 0:
                    z2_idx = _nearest_real_complex_idx(z, p1, "real")
                    z2 = z[z2_idx]
                    z = np.delete(z, z2_idx)
                    sos[si] = _single_zpksos([z1, z2], [p1, p2], 1)
                else:
                    sos[si] = _single_zpksos([z1], [p1, p2], 1)
            else:
                sos[si] = _single_zpksos([], [p1, p2], 1)
    sos[0][:3] *= k
    return sos


def butter_sos(N: int, Wn: float, btype: str = "lowpass"):
    """``zpk2sos(iirfilter(N, Wn, btype, ftype='butter', output='zpk'))``."""
    return zpk2sos(*iirfilter_butter_zpk(N, Wn, btype))


def sosfilt_zi(sos):
    """scipy/signal/_signaltools.py:4103-4175 with lfilter_zi (:3967-4100)."""
    sos = np.asarray(sos, dtype=float)
    n_sections = sos.shape[0]
    zi = np.empty((n_sections, 2))
    scale = 1.0
    for s in range(n_sections):
        b = sos[s, :3]
        a = sos[s, 3:]
        if a[0] != 1.0:
            b = b / a[0]
            a = a / a[0]
        companion_t = np.array([[-a[1], 1.0], [-a[2], 0.0]])
        iminus_a = np.eye(2) - companion_t
        bb = b[1:] - a[1:] * b[0]
        zi[s] = scale * np.linalg.solve(iminus_a, bb)
        scale *= b.sum() / a.sum()
    return zi


# ---------------------------------------------------------------------------
# Filtering (SciPy, restated)
# ---------------------------------------------------------------------------
def odd_ext(x, n, axis=-1):
    """scipy/signal/_arraytools.py:57-107 (computed in x's dtype)."""
    if n < 1:
        return x
    x = np.moveaxis(np.asarray(x), axis, -1)
    if n > x.shape[-1] - 1:
        raise ValueError(f"The extension length n ({n}) is too big. It must not exceed x.shape[axis]-1, which is {x.shape[-1] - 1}.")
    left_end = x[..., :1]
    left_ext = x[..., n:0:-1]
    right_end = x[..., -1:]
    right_ext = x[..., -2:-(n + 2):-1]
    ext = np.concatenate((2 * left_end - left_ext, x, 2 * right_end - right_ext), axis=-1)
    return np.moveaxis(ext, -1, axis)


def sosfilt(sos, x, zi):
    """Restated ``scipy.signal.sosfilt(sos, x, axis=-1, zi=zi)``: float64
    rows (n_sig, n_t), zi (n_sig, n_sec, 2).  Uses the C restatement of
    ``_sosfilt`` (bit-exact) when built, else a NumPy loop over time that
    performs the same operations in the same order."""
    sos = np.ascontiguousarray(sos, dtype=np.float64)
    y = np.array(x, dtype=np.float64, order="C", ndmin=2)
    z = np.array(zi, dtype=np.float64, order="C").reshape(y.shape[0], sos.shape[0], 2)
    lib = _load_c()
    if lib:
        lib.oracle_sosfilt_f64(sos.ctypes.data, sos.shape[0], y.ctypes.data,
                               y.shape[0], y.shape[1], z.ctypes.data)
        return y, z
    for n in range(y.shape[1]):  # pragma: no cover
        xc = y[:, n].copy()
        for s in range(sos.shape[0]):
            b0, b1, b2, _, a1, a2 = sos[s]
            xn = b0 * xc + z[:, s, 0]
            z[:, s, 0] = b1 * xc - a1 * xn + z[:, s, 1]
            z[:, s, 1] = b2 * xc - a2 * xn
            xc = xn
        y[:, n] = xc
    return y, z


def sosfiltfilt_ref_padlen(sos) -> int:
    """Default edge of sosfiltfilt — scipy/signal/_signaltools.py:4811-4813."""
    sos = np.asarray(sos)
    ntaps = 2 * sos.shape[0] + 1
    ntaps -= min(int((sos[:, 2] == 0).sum()), int((sos[:, 5] == 0).sum()))
    return 3 * ntaps


def sosfiltfilt(sos, x, axis=-1, padlen=None):
    """scipy/signal/_signaltools.py:4718-4828, padtype='odd'."""
    sos = np.asarray(sos, dtype=np.float64)
    x = np.moveaxis(np.asarray(x), axis, -1)
    edge = sosfiltfilt_ref_padlen(sos) if padlen is None else int(padlen)
    if x.shape[-1] <= edge:
        raise ValueError("The length of the input vector x must be greater than padlen, which is %d." % edge)
    shp = x.shape
    x2 = x.reshape(-1, shp[-1])
    ext = odd_ext(x2, edge) if edge > 0 else x2
    zi = sosfilt_zi(sos)
    n_sig = ext.shape[0]
    x0 = ext[:, :1].astype(np.float64)
    zi0 = zi[None, :, :] * x0[:, :, None]
    y, _ = sosfilt(sos, ext, zi0)
    y0 = y[:, -1:]
    y, _ = sosfilt(sos, y[:, ::-1], zi[None, :, :] * y0[:, :, None])
    y = y[:, ::-1]
    if edge > 0:
        y = y[:, edge:-edge]
    y = y.reshape(shp[:-1] + (y.shape[-1],))
    return np.moveaxis(y, -1, axis)


def sosfiltfilt_rows_c(sos, x_f32_rows, padlen=None):
    """The C channel-block driver (oracle/csrc/sosfilt.c) — same semantics as
    ``sosfiltfilt`` for float32 rows; used as bench.py's CPU baseline."""
    lib = _load_c()
    if not lib:
        raise RuntimeError("C oracle not built (oracle/Makefile)")
    sos = np.ascontiguousarray(sos, dtype=np.float64)
    x = np.asarray(x_f32_rows)
    assert x.dtype == np.float32 and x.strides[1] == 4
    edge = sosfiltfilt_ref_padlen(sos) if padlen is None else int(padlen)
    zi = np.ascontiguousarray(sosfilt_zi(sos))
    n_sig, n_t = x.shape
    y = np.empty((n_sig, n_t), dtype=np.float64)
    work = np.empty(n_t + 2 * edge, dtype=np.float64)
    lib.oracle_sosfiltfilt_rows_f32(sos.ctypes.data, sos.shape[0], zi.ctypes.data, edge,
                                    x.ctypes.data, n_sig, n_t, x.strides[0] // 4,
                                    y.ctypes.data, work.ctypes.data)
    return y


def interp1d_linear(t, y, t_new, axis=-1):
    """``scipy.interpolate.interp1d(t, y, axis=axis, kind='linear')(t_new)`` —
    scipy/interpolate/_interpolate.py:457-484 (searchsorted, clip to
    [1, n-1], slope*(x_new-x_lo)+y_lo)."""
    t = np.asarray(t, dtype=np.float64)
    t_new = np.asarray(t_new, dtype=np.float64)
    y = np.moveaxis(np.asarray(y), axis, 0)
    idx = np.searchsorted(t, t_new).clip(1, len(t) - 1).astype(int)
    lo = idx - 1
    hi = idx
    x_lo = t[lo]
    x_hi = t[hi]
    y_lo = y[lo]
    y_hi = y[hi]
    shape = (-1,) + (1,) * (y.ndim - 1)
    slope = (y_hi - y_lo) / (x_hi - x_lo).reshape(shape)
    out = slope * (t_new - x_lo).reshape(shape) + y_lo
    return np.moveaxis(out, 0, axis)


# ---------------------------------------------------------------------------
# DASCore wrapper semantics (external, restated)
# ---------------------------------------------------------------------------
def dascore_pass_filter_sos(fs: float, lo, hi, corners: int = 4):
    """*(DASCore, external)* ``dascore/proc/filter.py`` ``_get_sos``: Butterworth
    zpk via iirfilter → zpk2sos; low-pass when the lower corner is None."""
    nyquist = 0.5 * fs
    if lo is None and hi is not None:
        if hi >= nyquist:
            raise ValueError("filter corner must be below the Nyquist frequency")
        return butter_sos(corners, hi / nyquist, "lowpass")
    if hi is None and lo is not None:
        return butter_sos(corners, lo / nyquist, "highpass")
    return butter_sos(corners, [lo / nyquist, hi / nyquist], "bandpass")


def pass_filter(data, axis: int, fs: float, lo, hi, corners: int = 4):
    """*(DASCore, external)* ``Patch.pass_filter(time=(lo, hi), corners,
    zerophase=True)`` → ``sosfiltfilt(sos, data, axis)`` (float64 out).
    Called at lf_das.py:40 and lf_das.py:223."""
    sos = dascore_pass_filter_sos(fs, lo, hi, corners)
    return sosfiltfilt(sos, data, axis=axis)


def interpolate(data, axis: int, t_ns, t_new_ns):
    """*(DASCore, external)* ``Patch.interpolate(time=array, kind='linear')`` →
    interp1d on numeric coordinates (lf_das.py:42, :223-225).  Coordinates
    are taken relative to the first sample (exact integer ns → float)."""
    t_ns = np.asarray(t_ns, dtype=np.int64)
    t0 = t_ns[0]
    return interp1d_linear((t_ns - t0).astype(np.float64), data,
                           (np.asarray(t_new_ns, dtype=np.int64) - t0).astype(np.float64), axis=axis)


def rolling_mean(x, W: int, S: int, axis: int = -1):
    """*(DASCore, external)* ``Patch.rolling(time=w, step=s, engine='numpy')
    .mean()`` (rolling_mean_dascore.ipynb:148): pandas-compatible
    right-aligned windows, ``out[k] = mean(x[kS-W+1 : kS+1])`` when
    ``kS >= W-1`` else NaN, ``n_out = ceil(N/S)`` (pinned against
    ``pandas.Series.rolling(W, step=S).mean()``).  Accumulates in float64 and
    returns x's dtype (np.mean keeps float32)."""
    x = np.moveaxis(np.asarray(x), axis, -1)
    n = x.shape[-1]
    n_out = -(-n // S)
    out = np.full(x.shape[:-1] + (n_out,), np.nan, dtype=np.float64)
    for k in range(n_out):
        e = k * S
        if e >= W - 1:
            seg = x[..., e - W + 1:e + 1].astype(np.float64)
            out[..., k] = seg.sum(axis=-1) / W
    return np.moveaxis(out.astype(x.dtype if x.dtype.kind == "f" else np.float64), -1, axis)


def rolling_out_times(t0_ns: int, dt_ns: int, n: int, S: int):
    """Output coordinate of the rolling op: ``t0 + k*S*dt`` for k < ceil(n/S)."""
    return t0_ns + np.arange(-(-n // S), dtype=np.int64) * (S * dt_ns)


# ---------------------------------------------------------------------------
# lf_das.py (restated)
# ---------------------------------------------------------------------------
def get_patch_time(memory_size, sampling_rate, num_ch, bytes_per_element=8,
                   processing_factor=5, memory_safety_factor=1.2):
    """lf_das.py:90-107."""
    mem = sampling_rate * num_ch * bytes_per_element * processing_factor * memory_safety_factor / 1e6
    return memory_size / mem


def lfproc_time_grid(t1_ns: int, t2_ns: int, dt_s: float):
    """lf_das.py:252-256: ``np.arange(t1, t2, timedelta64(int(dt*1000), 'ms'))``."""
    step = int(dt_s * 1000) * 1_000_000
    return np.arange(int(t1_ns), int(t2_ns), step, dtype=np.int64)


def lfproc_schedule(n_grid: int, patch_size: int, buff_size: int):
    """The chunk loop of LFProc.process_time_range (lf_das.py:258-290) as
    pure index arithmetic.  Returns a list of
    ``(read_first, read_last, out_begin, out_end)`` grid indices: chunk k is
    ``spool.select(time=(tg[read_first], tg[read_last]))`` (inclusive) and
    writes ``tg[out_begin:out_end]``."""
    P = int(patch_size)
    B = int(buff_size)
    L = int(n_grid)
    if L <= P:
        P = L - 1
    sched = [(0, P, B, P - B)]
    data_end = P
    new_data_end = data_end + P - 2 * B
    if P - 2 * B <= 0 and new_data_end < L:
        raise ValueError("process_patch_size must exceed 2*edge_buff_size")
    while new_data_end < L:
        sched.append((data_end - 2 * B, new_data_end, data_end - B, new_data_end - B))
        data_end = new_data_end
        new_data_end = data_end + P - 2 * B
    if (L - data_end) > 1:
        new_data_end = L - 1
        sched.append((data_end - 2 * B, new_data_end, data_end - B, new_data_end - B))
    return sched


def lfproc_process(data, t0_ns: int, dt_ns: int, t1_ns: int, t2_ns: int,
                   dt_out: float, patch_size: int, buff_size: int,
                   corners: int = 4, time_axis: int = -1):
    """The reference path of ``LFProc.process_time_range`` (lf_das.py:219-290)
    over one contiguous in-memory spool whose samples sit at
    ``t0 + i*dt_ns``.  Per chunk: inclusive ``select`` (lf_das.py:236-240,
    264-266), ``pass_filter(time=(None, 1/dt/2*0.9))`` then
    ``interpolate(time=tg[a:b])`` (lf_das.py:223-225).  Returns a list of
    ``(out_times_ns, out_data_float64)`` in chunk order."""
    data = np.moveaxis(np.asarray(data), time_axis, -1)
    n = data.shape[-1]
    t = t0_ns + np.arange(n, dtype=np.int64) * dt_ns
    tg = lfproc_time_grid(t1_ns, t2_ns, dt_out)
    fs = 1.0 / (dt_ns / 1e9)
    fc = 1 / dt_out / 2 * 0.9
    out = []
    for (ra, rb, oa, ob) in lfproc_schedule(len(tg), patch_size, buff_size):
        sel = (t >= tg[ra]) & (t <= tg[rb])
        idx = np.nonzero(sel)[0]
        chunk = data[..., idx[0]:idx[-1] + 1]
        y = pass_filter(chunk, -1, fs, None, fc, corners)
        yi = interpolate(y, -1, t[idx[0]:idx[-1] + 1], tg[oa:ob])
        out.append((tg[oa:ob].copy(), np.moveaxis(yi, -1, time_axis)))
    return out


def down_sample_processing(data, time_axis: int, t_ns, freq=5, nqfreq_ratio=0.8):
    """lf_das.py:34-44 on raw arrays: low-pass at ``freq*0.5*ratio`` then
    interpolate onto ``arange(time_min, time_max, 1/freq s)``."""
    t_ns = np.asarray(t_ns, dtype=np.int64)
    dt = np.int64(int(1 / freq * 1e9))
    fs = 1.0 / ((t_ns[1] - t_ns[0]) / 1e9)
    y = pass_filter(data, time_axis, fs, None, freq * 0.5 * nqfreq_ratio)
    new_t = np.arange(t_ns[0], t_ns[-1], dt, dtype=np.int64)
    return new_t, interpolate(y, time_axis, t_ns, new_t)


def get_edge_effect_time(sampling_interval, total_T, tol=1e-6, freq=5, nqfreq_ratio=0.8):
    """lf_das.py:47-87 (impulse response of the downsampling chain)."""
    N = int(total_T / sampling_interval)
    taxis = (np.arange(N) - N // 2) * sampling_interval
    data = np.zeros_like(taxis)
    data[N // 2] = 1
    step_ns = int(round(sampling_interval * 1e9))
    t_ns = (np.arange(N, dtype=np.int64) - N // 2) * step_ns
    new_t, out = down_sample_processing(data.reshape(-1, 1), 0, t_ns, freq=freq,
                                        nqfreq_ratio=nqfreq_ratio)
    d = out[:, 0]
    max_val = np.max(np.abs(d))
    ind = np.abs(d) > max_val * tol
    ind_1 = np.where(ind)[0][0]
    ind_2 = np.where(ind)[0][-1]
    new_taxis = (new_t - new_t[0]) / 1e9 - N // 2 * sampling_interval
    edge_t = max(abs(new_taxis[ind_1]), abs(new_taxis[ind_2]))
    if int(math.ceil(edge_t * freq)) * 2 >= int(total_T * freq):
        raise ValueError(f"edge_t value ({edge_t} sec) is too close to half of the processing chunk size ({total_T} sec).")
    return edge_t


def edge_loop(data, t0_ns: int, dt_ns: int, push_len: int, t_start_ns: int, dt_out: float,
              patch_size: int, buff_size: int, resume_back_ns: int, corners: int = 4):
    """The real-time loop of low_pass_dascore_edge.ipynb cell 11 (:199-235)
    with one new file of ``push_len`` samples per iteration: run k sees the
    data of files 0..k and calls ``process_time_range(t_1, t_2)`` with
    ``t_2`` = newest sample time (``sub_sp[-1].attrs['time_max']``) and
    ``t_1`` = ``t_start`` on the first run, else ``get_last_processed_time()``
    (lf_das.py:214-217: the last output time) minus ``resume_back_ns``
    (``int((ceil(edge/d_t)-1)*d_t)`` s).  A run whose time grid holds
    ``<= 2*buff_size + 1`` points cannot produce an output (the reference
    indexes out of range there) and is skipped until more data arrives.
    Returns, per push, the list of ``(out_times_ns, out_data)`` chunks."""
    data = np.asarray(data)
    n = data.shape[-1]
    res = []
    last_out = None
    for end in range(push_len, n + 1, push_len):
        t2 = t0_ns + (end - 1) * dt_ns
        t1 = t_start_ns if last_out is None else last_out - resume_back_ns
        tg = lfproc_time_grid(t1, t2, dt_out)
        if len(tg) < 2 or len(tg) <= 2 * buff_size + 1:
            res.append([])
            continue
        out = lfproc_process(data[..., :end], t0_ns, dt_ns, t1, t2, dt_out, patch_size,
                             buff_size, corners)
        out = [(t, y) for t, y in out if len(t)]
        if out:
            last_out = int(out[-1][0][-1])
        res.append(out)
    return res
