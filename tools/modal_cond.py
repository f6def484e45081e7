"""Condition numbers of the eigenvector matrices of the full-rate path's
32-sample state transition (SciPy TDF-II cascade states, Phi = P^32) for
representative Butterworth designs: the bound on the precision a modal
(block-diagonal) basis for the row scans would lose (CPU only).

    python tools/modal_cond.py
"""
import numpy as np
from scipy import signal


def tdf2_transition(sos):
    """One-sample homogeneous transition of SciPy's sosfilt states."""
    ns = len(sos)
    n = 2 * ns
    P = np.zeros((n, n))
    for k in range(n):
        z = np.zeros(n)
        z[k] = 1.0
        zn = z.copy()
        v = 0.0
        for s in range(ns):
            b0, b1, b2, _, a1, a2 = sos[s]
            yv = b0 * v + z[2 * s]
            zn[2 * s] = b1 * v - a1 * yv + z[2 * s + 1]
            zn[2 * s + 1] = b2 * v - a2 * yv
            v = yv
        P[:, k] = zn
    return P


def main():
    cases = {
        "butter(4, 0.02) low-pass": signal.butter(4, 0.02, output="sos"),
        "band-pass 1-10 Hz @ 1 kHz (bench)": signal.butter(4, [1.0, 10.0], btype="band", fs=1000.0, output="sos"),
        "low-pass 0.45 Hz @ 500 Hz (cfg3)": signal.butter(4, 0.45, fs=500.0, output="sos"),
        "band-pass 0.2-30 Hz @ 250 Hz": signal.butter(4, [0.2, 30.0], btype="band", fs=250.0, output="sos"),
        "low-pass 1 Hz @ 500 Hz": signal.butter(4, 1.0, fs=500.0, output="sos"),
        "high-pass 2 Hz @ 250 Hz": signal.butter(4, 2.0, btype="high", fs=250.0, output="sos"),
    }
    for name, sos in cases.items():
        P32 = np.linalg.matrix_power(tdf2_transition(sos), 32)
        w, V = np.linalg.eig(P32)
        print(f"{name:36s} states {P32.shape[0]}  max|eig| {np.abs(w).max():.6f}  cond(V) {np.linalg.cond(V):.2e}")


if __name__ == "__main__":
    main()
