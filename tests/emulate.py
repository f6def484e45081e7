"""Test-side NumPy model of the two device kernels (k_block_functionals_* and
k_chunk_scan, realization R of csrc/lfd_internal.h), driven by the constants
a host-only plan computed in C++ (``lfd_debug_plan_constants``).  It lets the
CPU suite check the plan's host math (state-space matrices, p0 coefficients,
FIR-history correction, chunk geometry) against SciPy's golden vectors
without a GPU.  Not product code."""
import numpy as np


def block_functionals_taps(plan, x):
    """Model of k_block_functionals_mfma: F[c, ch, k] = sum_p Kx[c, p]
    x[ch, base + k L - J + p] (samples before the channel start are 0),
    accumulated in float64."""
    Kx = plan.block_taps()
    _, _, cg = plan.constants()
    L, nb, J = plan.block_len, plan.n_blocks, 2 * plan.n_sec
    base = int(cg[0]["head_end"] - cg[0]["kb"] * L)
    n_ch = x.shape[0]
    pad = np.zeros((n_ch, J), np.float64)
    xe = np.concatenate([pad, x.astype(np.float64)], 1)  # xe[:, i + J] = x[:, i]
    rows = np.stack([xe[:, base + k * L: base + k * L + L + J] for k in range(nb)], 1)
    return np.einsum("cp,akp->cak", Kx, rows)


def emulate(plan, x, padlen, fir32=True, k1="recurrence"):
    bc, sc, cg = plan.constants()
    ns = plan.n_sec
    n = 2 * ns
    J = 2 * ns
    L = plan.block_len
    r = bc["r"]
    na1, na2, nia2, nra = r["na1"][:ns], r["na2"][:ns], r["nia2"][:ns], r["nra"][:ns]
    c64 = r["c64"][:J + 1]
    c32 = r["c32"][:J + 1]
    G = float(r["G"])
    n_ch, n_t = x.shape
    nb = plan.n_blocks
    base = int(cg[0]["head_end"] - cg[0]["kb"] * L)
    # ---------------- K1 (vectorised over channels x blocks)
    X = np.stack([x[:, base + k * L: base + (k + 1) * L] for k in range(nb)], 1)
    H = np.zeros((J, n_ch, nb), np.float32)
    for k in range(nb):
        for j in range(J):
            t = base + k * L - 1 - j
            H[j, :, k] = x[:, t] if t >= 0 else 0.0
    S = np.zeros((n, n_ch, nb))
    u = np.zeros((n, n_ch, nb))
    y0 = np.zeros((J + 1, n_ch, nb))
    for m in range(L):
        xm = X[:, :, m]
        if fir32:
            w = xm.astype(np.float32)
            for j in range(1, J + 1):
                w = (np.float32(c32[j]) * H[j - 1] + w).astype(np.float32)
            w = w.astype(np.float64)
        else:
            w = xm.astype(np.float64) + sum(c64[j] * H[j - 1].astype(np.float64) for j in range(1, J + 1))
        H[1:] = H[:-1].copy()
        H[0] = xm
        v = w
        for s in range(ns):
            vn = na1[s] * S[2 * s] + na2[s] * S[2 * s + 1] + v
            S[2 * s + 1] = S[2 * s].copy()
            S[2 * s] = vn
            v = vn
        if m <= J:
            y0[m] = v
        t = u.copy()
        for s in range(ns):
            d = t[0] if s == 0 else t[2 * s] - t[2 * s - 2]
            u[2 * s] = t[2 * s + 1] + v
            u[2 * s + 1] = nra[s] * t[2 * s + 1] + nia2[s] * d
    ef = S
    er0 = np.einsum("ij,jab->iab", bc["T"][:n, :n], u)
    p0 = np.einsum("j,jab->ab", bc["cp"][:n], u) + np.einsum("m,mab->ab", bc["dp"][:J + 1], y0)
    if k1 in ("taps", "runs"):
        F = block_functionals_taps(plan, x)
        ef, er0, p0 = F[:n], F[n:2 * n], F[2 * n]
    if k1 == "runs":  # model of k_block_runs_mfma: fold blocks into runs
        run_ks, run_len, rc = plan.runs()
        rPhiF, rM, rPhiR = (rc[k].reshape(4, 4) for k in ("PhiF", "M", "PhiR"))
        rG0, rH0 = rc["G0"], rc["H0"]
        Y0 = np.zeros((n_ch, nb))
        AG = np.zeros((len(run_ks), 8, n_ch))
        for ri, (ks, ln) in enumerate(zip(run_ks, run_len)):
            S0 = np.zeros((4, n_ch))
            pg, vv = [], []
            for p in range(ln):
                k = ks + p
                pg.append(p0[:, k] + rG0 @ S0)
                vv.append(er0[:, :, k] + rM @ S0)
                S0 = rPhiF @ S0 + ef[:, :, k]
            T0 = np.zeros((4, n_ch))
            for p in range(ln - 1, -1, -1):
                Y0[:, ks + p] = pg[p] + rH0 @ T0
                T0 = rPhiR @ T0 + vv[p]
            AG[ri, :4], AG[ri, 4:] = S0, T0
    # ---------------- K2
    PhiF, PhiR, M = sc["PhiF"][:n, :n], sc["PhiR"][:n, :n], sc["M"][:n, :n]
    G0, H0, Kc = sc["G0"][:n], sc["H0"][:n], sc["Kc"][: 2 * n + 1, :J]
    y = np.full((n_ch, plan.n_grid), np.nan, np.float64)
    E = padlen

    def fwd(Sf, h, xv):
        w = xv + sum(c64[j] * h[j - 1] for j in range(1, J + 1))
        h[1:] = h[:-1].copy()
        h[0] = xv
        v = w
        for s in range(ns):
            vn = na1[s] * Sf[2 * s] + na2[s] * Sf[2 * s + 1] + v
            Sf[2 * s + 1] = Sf[2 * s].copy()
            Sf[2 * s] = vn
            v = vn
        return G * v

    def rev(T, yv):
        v = yv
        for s in range(ns):
            qn = na1[s] * T[2 * s] + na2[s] * T[2 * s + 1] + v
            T[2 * s + 1] = T[2 * s].copy()
            T[2 * s] = qn
            v = qn
        return v

    def steady(c, with_fir):
        v = c * float(r["csum"]) if with_fir else c
        St = np.zeros((n,) + np.shape(c))
        for s in range(ns):
            v = v * r["dcg"][s]
            St[2 * s] = v
            St[2 * s + 1] = v
        return St, v

    for Gc in cg:
        s0, s1 = int(Gc["s0"]), int(Gc["s1"])
        kb, ke = int(Gc["kb"]), int(Gc["ke"])
        xl = x[:, s0]
        e0 = (2 * xl - x[:, s0 + E]).astype(np.float32).astype(np.float64)
        Sf, _ = steady(e0, True)
        h = np.stack([e0] * J, 0)
        he = int(Gc["head_end"])
        hs = k1 == "runs" and int(Gc["hskip"]) != 0 and E > 0
        lo_h = he - L
        n_pad = E - (s0 - lo_h) if hs else E
        for i in range(n_pad):
            fwd(Sf, h, (2 * xl - x[:, s0 + E - i]).astype(np.float32).astype(np.float64))
        if hs:
            # head skip: K1's one-block run kb-1 summed the head; correct the
            # row samples before s0 (pad instead of raw) with the e_f taps
            rh = int(Gc["r0"]) - 1
            assert run_ks[rh] == kb - 1 and run_len[rh] == 1
            Sf = rc["PhiFp"][1].reshape(4, 4) @ Sf + AG[rh, :4]
            for pq in range(s0 - lo_h + J):
                pos = lo_h - J + pq
                u = (2 * xl - x[:, 2 * s0 - pos]).astype(np.float32).astype(np.float64)
                rv = x[:, pos].astype(np.float64) if pos >= 0 else np.zeros(n_ch)
                if pos < lo_h:
                    rv = np.where(np.isfinite(rv), rv, 0.0)
                Sf = Sf + np.outer(rc["KfH"][:, pq], u - rv)
            h = np.stack([x[:, he - 1 - j] for j in range(J)], 0).astype(np.float64)
        else:
            for t in range(s0, he):
                fwd(Sf, h, x[:, t].astype(np.float64))
        raw = np.stack([x[:, he - 1 - j] if he - 1 - j >= 0 else np.zeros(n_ch) for j in range(J)], 0)
        dh = h - raw.astype(np.float64)
        dw = np.stack([sum(c64[jj] * dh[jj - m - 1] for jj in range(m + 1, J + 1)) for m in range(J)], 0)
        corr = Kc @ dw
        SFs = {}
        if k1 == "runs":
            r0, r1 = int(Gc["r0"]), int(Gc["r1"])
            assert run_ks[r0] == kb and run_len[r0] == 1 and (r1 == len(run_ks) or run_ks[r1] == ke)
            for ri in range(r0, r1):
                SFs[ri] = Sf.copy()
                Sf = rc["PhiFp"][run_len[ri]].reshape(4, 4) @ Sf + AG[ri, :4] + (corr[:n] if ri == r0 else 0)
        for k in range(kb, ke if k1 != "runs" else kb):
            SFs[k] = Sf.copy()
            Sf = PhiF @ Sf + ef[:, :, k] + (corr[:n] if k == kb else 0)
        tb = int(Gc["tail_begin"])
        h = np.stack([x[:, tb - 1 - j] for j in range(J)], 0).astype(np.float64)
        tp = [fwd(Sf, h, x[:, t].astype(np.float64)) for t in range(tb, s1 + 1)]
        xr = x[:, s1]
        for i in range(E):
            tp.append(fwd(Sf, h, (2 * xr - x[:, s1 - 1 - i]).astype(np.float32).astype(np.float64)))
        T, qss = steady(tp[-1], False)
        qw = [qss] * J
        y_next = 0.0
        for i in range(len(tp) - 1, -1, -1):
            q = rev(T, tp[i])
            if Gc["tail_out_j"] >= 0 and tb + i in (Gc["tail_out_pos"], Gc["tail_out_pos"] + 1):
                yv = G * (q + sum(c64[j] * qw[j - 1] for j in range(1, J + 1)))
                if tb + i == Gc["tail_out_pos"] + 1:
                    y_next = yv
                else:  # interp1d between the two samples (the grid's w)
                    y[:, Gc["tail_out_j"]] = yv + float(sc["ow"]) * (y_next - yv)
            qw = [q] + qw[:-1]
        kst = int(Gc["kstep"])

        def is_out(k):
            return Gc["kout0"] <= k < Gc["kout1"] and (k - Gc["kout0"]) % kst == 0

        def out_j(k):
            return Gc["jout0"] + (k - Gc["kout0"]) // kst
        if k1 == "runs":
            for ri in range(r1 - 1, r0 - 1, -1):
                sin, ks, ln = SFs[ri], int(run_ks[ri]), int(run_len[ri])
                for p in range(ln):
                    k = ks + p
                    if is_out(k):
                        yk = Y0[:, k] + (corr[2 * n] if k == kb else 0)
                        yk = yk + rc["A"][ln][p] @ sin + rc["B"][ln - 1 - p] @ T
                        y[:, out_j(k)] = yk
                T = (rc["PhiRp"][ln].reshape(4, 4) @ T + AG[ri, 4:] + (corr[n:2 * n] if ri == r0 else 0)
                     + rc["C"][ln].reshape(4, 4) @ sin)
            continue
        for k in range(ke - 1, kb - 1, -1):
            sf = SFs[k]
            if is_out(k):
                pk = p0[:, k] + (corr[2 * n] if k == kb else 0)
                y[:, out_j(k)] = pk + H0 @ T + G0 @ sf
            T = PhiR @ T + er0[:, :, k] + (corr[n:2 * n] if k == kb else 0) + M @ sf
    return y


def fir_decimate_mfma_model(x, taps, q, delay, dm=6):
    """NumPy model of k_fir_decimate_mfma's arithmetic (lfd_kernels.hip): the
    polyphase sum y[o] = sum_v sum_u h_v[u] X_v[o - u] evaluated as 4 x 4
    Toeplitz pieces A_{v,d}[i][k] = h_v[4d + i - k] (o = 4G + i, index
    n = 4(G - d) + k, d < dm) plus the row-0 epilogue tap h[21 q] X_0[o - 21]
    that dm = 6 steps do not reach.  X_v[n] = x[n q + delay - v], zero outside
    the record.  Returns float64 (n_ch, ceil(n_t / q))."""
    x = np.asarray(x, np.float64)
    h = np.asarray(taps, np.float64)
    n_ch, n_t = x.shape
    n_out = -(-n_t // q)
    o = np.arange(n_out)
    G, i = o // 4, o % 4

    def X(v, n):
        t = n * q + delay - v
        ok = (t >= 0) & (t < n_t)
        out = np.zeros((n_ch, len(n)))
        out[:, ok] = x[:, t[ok]]
        return out

    y = np.zeros((n_ch, n_out))
    for v in range(q):
        for d in range(dm):
            for k in range(4):
                u = 4 * d + i - k
                ti = u * q + v
                a = np.where((u >= 0) & (ti < h.size), h[np.clip(ti, 0, h.size - 1)], 0.0)
                y += a * X(v, 4 * (G - d) + k)
    if 21 * q < h.size:
        y += np.where(i == 0, h[21 * q], 0.0) * X(0, o - 21)
    return y
