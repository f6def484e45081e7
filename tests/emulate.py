"""Test-side NumPy model of the two device kernels (k_block_functionals and
k_chunk_scan), driven by the constants a host-only plan computed in C++
(``lfd_debug_plan_constants``).  It lets the CPU suite check the plan's host
math (state-space matrices, zi, chunk geometry) against the oracle without a
GPU.  Not product code."""
import numpy as np


def emulate(plan, x, padlen):
    bc, sc, cg = plan.constants()
    ns = plan.n_sec; n = 2*ns; L = plan.block_len
    n_ch, n_t = x.shape
    f = dict(b0=bc['b0'][:ns], b1=bc['b1'][:ns], b2=bc['b2'][:ns], a1=bc['a1'][:ns], a2=bc['a2'][:ns])
    def fstep(z, v):
        for i in range(ns):
            vi = f['b0'][i]*v + z[2*i]
            z[2*i] = f['b1'][i]*v - f['a1'][i]*vi + z[2*i+1]
            z[2*i+1] = f['b2'][i]*v - f['a2'][i]*vi
            v = vi
        return v
    def istep(u, y):
        g = 0.0
        for i in range(ns):
            t0, t1 = u[2*i], u[2*i+1]
            if i > 0: t0 = t0 - bc['beta0'][i]*g; t1 = t1 - bc['beta1'][i]*g
            w0 = -bc['ia2'][i]*t1; w1 = t0 - bc['ra'][i]*t1
            if i+1 < ns: g = w0 if i == 0 else bc['b0'][i]*g + w0
            u[2*i] = bc['Bv'][2*i]*y + w0; u[2*i+1] = bc['Bv'][2*i+1]*y + w1
    # K1 (vectorised over channels and blocks)
    nb = plan.n_blocks; base = None
    # recover base from chunk geometry: head_end = base + kb*L
    base = cg[0]['head_end'] - cg[0]['kb']*L
    X = np.stack([x[:, base + k*L: base + (k+1)*L] for k in range(nb)], 1).astype(np.float64)  # ch, nb, L
    z = np.zeros((n,)+X.shape[:2]); u = np.zeros((n,)+X.shape[:2])
    yf0 = None
    for m in range(L):
        yv = fstep(z, X[:, :, m])
        if m == 0: yf0 = yv.copy()
        istep(u, yv)
    T = bc['T'][:n, :n]; er0 = np.einsum('ij,jab->iab', T, u)
    p0 = bc['d0']*yf0 + np.einsum('j,jab->ab', bc['cp'][:n], u)
    # K2
    y = np.full((n_ch, plan.n_grid), np.nan, np.float32)
    E = padlen
    Phi = sc['Phi'][:n,:n]; M = sc['M'][:n,:n]; zi = sc['zi'][:n]
    for G in cg:
        s0, s1 = G['s0'], G['s1']
        xl = x[:, s0]
        e0 = (2*xl - x[:, s0+E]).astype(np.float32).astype(np.float64)
        s = zi[:, None]*e0[None]
        for i in range(E):
            fstep(s, (2*xl - x[:, s0+E-i]).astype(np.float32).astype(np.float64))
        tp = []
        for t in range(s0, G['head_end']): tp.append(fstep(s, x[:, t].astype(np.float64)))
        nhead = len(tp)
        SF = {}
        for k in range(G['kb'], G['ke']):
            SF[k] = s.copy(); s = Phi@s + z[:, :, k]
        for t in range(G['tail_begin'], s1+1): tp.append(fstep(s, x[:, t].astype(np.float64)))
        xr = x[:, s1]
        for i in range(E): tp.append(fstep(s, (2*xr - x[:, s1-1-i]).astype(np.float32).astype(np.float64)))
        r = zi[:, None]*tp[-1][None]
        for i in range(len(tp)-1, nhead-1, -1):
            v = fstep(r, tp[i])
            if G['tail_out_j'] >= 0 and G['tail_begin'] + (i-nhead) == G['tail_out_pos']: y[:, G['tail_out_j']] = v
        for k in range(G['ke']-1, G['kb']-1, -1):
            if G['kout0'] <= k < G['kout1']:
                y[:, G['jout0'] + k - G['kout0']] = p0[:, k] + sc['H0'][:n]@r + sc['G0'][:n]@SF[k]
            r = Phi@r + er0[:, :, k] + M@SF[k]
        if G['head_out_j'] >= 0:
            for i in range(nhead-1, -1, -1):
                v = fstep(r, tp[i])
                if s0 + i == G['head_out_pos']: y[:, G['head_out_j']] = v; break
    return y

