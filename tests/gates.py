"""Parity gates of the low-pass + decimate path (float64 outputs, like
SciPy's sosfiltfilt result, scipy/signal/_signaltools.py:4684, which
lf_das.py:223-232 interpolates and writes).

north_star's bar is relRMS 1e-4.  Every check here is tighter: its gate is
10x the relRMS that exact check measured (``tests/golden/gates_measured.json``,
made from a GPU run's log by ``tests/golden/make_gates.py``), so a
regression of one order of magnitude — a wrong tap row, a mis-indexed run
constant — fails.  The measured values span 1e-14 (cfg1, Wn = 0.008) to
~1e-9 (dt = 10 s grids at 1-2 kHz: poles within 3e-4 of the unit circle and
a DC offset), so one constant per category would be 10^5 too loose for the
well-conditioned cases.  A check missing from the table (a new case) falls
back to its category's constant:

* ``MFMA``    device path (fp64-MFMA block taps K1 + run scan) vs the oracle
              or a SciPy golden on the same float32 samples;
* ``REC``     the recurrence K1 (float32 FIR taps on non-negative-tap
              cascades, fp64 all-pole) vs the oracle;
* ``PATHS``   two device kernels on the same plan (same algebra, other
              summation order / kernel);
* ``STREAM``  the streaming arena (edge / continuous);
* ``DC``      max relative error of a constant input, which comes back as
              itself;
* ``Q32``     vs SciPy on the float64 data the float32 samples were rounded
              from (the input quantisation bounds it);
* ``ROLL``    rolling means (float32 like numpy's mean of float32 windows,
              summed in float64): the oracle rounds the same float64 window
              sums, so most checks measure 0 and are held bit-exact;
* ``EMU_*``   the NumPy model of the kernels (tests/emulate.py) on CPU.

``LFD_GATE_LOG=<file>`` appends every measured value (one JSON line per
check); ``LFD_GATE_MEASURE=1`` holds every check to north_star's 1e-4 only
(the run that re-derives the table after a kernel change).
"""
from __future__ import annotations

import json
import os

import numpy as np

MFMA = 1e-8
REC = 1e-7
PATHS = 1e-8
STREAM = 1e-8
DC = 1e-10
Q32 = 1e-6
ROLL = 1e-6
EMU_TAPS = 1e-8
EMU_REC = 5e-8

NORTH_STAR = 1e-4
FACTOR = 10.0  # gate = FACTOR x the measured value of the same check
FLOOR = 1e-15  # (a check that measured exactly 0 is held to FACTOR x FLOOR)

_TABLE_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "gates_measured.json")
try:
    with open(_TABLE_PATH) as _f:
        MEASURED = json.load(_f)["measured"]
except FileNotFoundError:  # pragma: no cover
    MEASURED = {}


def relrms(a, b) -> float:
    """relRMS of ``a`` against ``b`` over the entries finite in ``b``."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    m = np.isfinite(b)
    den = float(np.sum(b[m] ** 2))
    return float(np.sqrt(np.sum((a[m] - b[m]) ** 2) / den)) if den > 0 else float(np.sqrt(np.sum(a[m] ** 2)))


def gate(tag: str, fallback: float) -> float:
    if os.environ.get("LFD_GATE_MEASURE"):
        return NORTH_STAR
    if tag in MEASURED:
        return FACTOR * max(float(MEASURED[tag]), FLOOR)
    return fallback


def check(tag: str, value: float, fallback: float) -> None:
    tol = gate(tag, fallback)
    log = os.environ.get("LFD_GATE_LOG")
    if log:
        with open(log, "a") as f:
            f.write(json.dumps({"tag": tag, "rel": float(value), "tol": tol}) + "\n")
    assert value < tol, f"{tag}: relRMS {value:.3e} >= gate {tol:.1e}"
