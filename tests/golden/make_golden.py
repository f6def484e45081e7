"""Generate the committed golden vectors with SciPy / pandas (the libraries
the reference path's arithmetic lives in: DASCore → scipy.signal.sosfiltfilt,
scipy.interpolate.interp1d; pandas-compatible rolling).  Run in the dev
container only:  python tests/golden/make_golden.py

Nothing here imports the repo's oracle or product code: these vectors are the
independent pin for both.  LFProc chunking follows lf_das.py:252-290; the
chunk loop is written out here directly from the reference's index
arithmetic."""
import json
import os
import sys

import numpy as np
import pandas as pd
import scipy
import scipy.signal as ss
from scipy.interpolate import interp1d

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import synth  # noqa: E402


def chunks_ref(L, P, B):
    # lf_das.py:258-290
    if L <= P:
        P = L - 1
    out = [(0, P, B, P - B)]
    de = P
    nde = de + P - 2 * B
    while nde < L:
        out.append((de - 2 * B, nde, de - B, nde - B))
        de = nde
        nde = de + P - 2 * B
    if L - de > 1:
        nde = L - 1
        out.append((de - 2 * B, nde, de - B, nde - B))
    return out


def lfproc_scipy(x, fs, dt_out, P, B, t0=synth.T0_NS):
    n = x.shape[1]
    dt_ns = int(round(1e9 / fs))
    t = t0 + np.arange(n, dtype=np.int64) * dt_ns
    tg = np.arange(t0, t0 + n * dt_ns, int(dt_out * 1000) * 1_000_000, dtype=np.int64)
    nyq = 0.5 * fs
    z, p, k = ss.iirfilter(4, (1 / dt_out / 2 * 0.9) / nyq, btype="lowpass", ftype="butter", output="zpk")
    sos = ss.zpk2sos(z, p, k)
    outs = []
    for a, b, oa, ob in chunks_ref(len(tg), P, B):
        sel = (t >= tg[a]) & (t <= tg[b])
        i = np.nonzero(sel)[0]
        y = ss.sosfiltfilt(sos, x[:, i[0]:i[-1] + 1], axis=-1)
        tt = (t[i[0]:i[-1] + 1] - t0).astype(np.float64)
        yi = interp1d(tt, y, kind="linear", axis=-1)((tg[oa:ob] - t0).astype(np.float64))
        outs.append((oa, ob, yi))
    return tg, sos, outs


def save_lfproc(name, x, fs, dt_out, P, B, recipe):
    tg, sos, outs = lfproc_scipy(x, fs, dt_out, P, B)
    y = np.full((x.shape[0], len(tg)), np.nan)
    sched = []
    for oa, ob, yi in outs:
        y[:, oa:ob] = yi
        sched.append((oa, ob))
    np.savez_compressed(os.path.join(HERE, name), y=y, tg=tg, sos=sos, sched=np.array(sched),
                        fs=fs, dt_out=dt_out, P=P, B=B, x_sha256=synth.digest(x),
                        recipe=json.dumps(recipe))


def main():
    meta = {"scipy": scipy.__version__, "numpy": np.__version__, "pandas": pd.__version__}
    # 1) filter design + sosfilt_zi (iirfilter zpk → zpk2sos)
    cases, soss, zis = [], [], []
    for N in (2, 4, 5, 8):
        for Wn in (0.008, 0.0018, 4.5e-4, 0.3):
            for bt in ("lowpass", "highpass"):
                z, p, k = ss.iirfilter(N, Wn, btype=bt, ftype="butter", output="zpk")
                sos = ss.zpk2sos(z, p, k)
                cases.append((N, Wn, bt))
                soss.append(np.pad(sos, ((0, 4 - sos.shape[0]), (0, 0))))
                zis.append(np.pad(ss.sosfilt_zi(sos), ((0, 4 - sos.shape[0]), (0, 0))))
    np.savez_compressed(os.path.join(HERE, "design.npz"), cases=json.dumps(cases),
                        sos=np.array(soss), zi=np.array(zis), meta=json.dumps(meta))
    # 2) sosfilt with zi (the _sosfilt kernel)
    rng = np.random.default_rng(2024)
    x = rng.standard_normal((3, 257))
    sos = ss.butter(4, 0.0018, output="sos")
    zi = rng.standard_normal((3, 2, 2)) * 1e-3
    y, zf = ss.sosfilt(sos, x, axis=-1, zi=np.moveaxis(zi, 0, 1))
    np.savez_compressed(os.path.join(HERE, "sosfilt_small.npz"), x=x, sos=sos, zi=zi, y=y,
                        zf=np.moveaxis(zf, 1, 0))
    # 3) sosfiltfilt full-rate, float32 input (odd padding computed in float32)
    x32 = synth.noise_sine(4, 3000, 250.0, seed=5, dc=3.0)
    sos = ss.butter(4, 0.008, output="sos")
    np.savez_compressed(os.path.join(HERE, "sosfiltfilt_small.npz"), x=x32, sos=sos,
                        y=ss.sosfiltfilt(sos, x32, axis=-1))
    # 4) LFProc chunk path
    save_lfproc("lfproc_cfg1.npz", synth.random_das_spool_data().astype(np.float32), 250.0, 0.2, 40, 6,
                {"data": "random_das x3 (RandomState(42).random((300,2000)) per patch), float32"})
    save_lfproc("lfproc_cfg3_slice.npz", synth.noise_sine(4, 750_000, 500.0, seed=3), 500.0, 1.0, 600, 7,
                {"data": "noise_sine(4, 750000, 500.0, seed=3)"})
    save_lfproc("lfproc_cfg5_slice.npz", synth.noise_sine(4, 600_000, 200.0, seed=5, dc=1000.0),
                200.0, 10.0, 100, 7, {"data": "noise_sine(4, 600000, 200.0, seed=5, dc=1000.0)"})
    # 5) rolling mean (pandas right-aligned rolling with step)
    rr = {}
    for n, W, S in [(20, 5, 5), (20, 5, 3), (1003, 7, 13), (5000, 1000, 1000), (50, 1, 1), (999, 100, 37)]:
        xr = synth.noise_sine(1, n, 1000.0, seed=n + W)[0]
        rr[f"x_{n}_{W}_{S}"] = xr
        rr[f"y_{n}_{W}_{S}"] = pd.Series(xr).rolling(W, step=S).mean().to_numpy()
    np.savez_compressed(os.path.join(HERE, "rolling.npz"), **rr)
    # 6) the LFProc chunk table of SURVEY §3.1 (cfg1) and cfg3
    tables = {"cfg1": chunks_ref(120, 40, 6), "cfg3": chunks_ref(3600, 600, 7),
              "short": chunks_ref(30, 40, 6), "exact": chunks_ref(96, 40, 6)}
    with open(os.path.join(HERE, "schedule.json"), "w") as f:
        json.dump(tables, f, indent=1)
    print("golden vectors written to", HERE)


def main_next_rows():
    """band-pass design, decimate(ftype='iir'), and the
    notebook post-processing (scipy.ndimage.median_filter, demean + scale)."""
    import scipy.ndimage as nd
    band = {}
    for i, (N, W) in enumerate([(4, (0.01, 0.1)), (2, (0.2, 0.4)), (4, (4.5e-4, 0.02))]):
        z, p, k = ss.iirfilter(N, list(W), btype="bandpass", ftype="butter", output="zpk")
        band[f"sos_{i}"] = ss.zpk2sos(z, p, k)
        band[f"case_{i}"] = np.array([N, W[0], W[1]])
    x = synth.noise_sine(3, 4000, 250.0, seed=21, dc=2.0).astype(np.float64)
    band["x"] = x
    band["y_bp0"] = ss.sosfiltfilt(band["sos_0"], x, axis=-1)
    for q in (2, 5, 10, 50):
        band[f"cheby_{q}"] = ss.cheby1(8, 0.05, 0.8 / q, output="sos")
        band[f"dec_{q}"] = ss.decimate(x, q, ftype="iir", axis=-1)
        band[f"firwin_{q}"] = ss.firwin(20 * q + 1, 1.0 / q, window="hamming")
        band[f"decfir_{q}"] = ss.decimate(x, q, ftype="fir", axis=-1)
    np.savez_compressed(os.path.join(HERE, "band_decimate.npz"), **band)
    rng = np.random.default_rng(77)
    post = {"x2": rng.standard_normal((40, 23)), "x1": rng.standard_normal(200)}
    for k in (5, (3, 7), 4, (9, 3), 11):
        tag = "x".join(str(v) for v in np.atleast_1d(k))
        post[f"med2_{tag}"] = nd.median_filter(post["x2"], size=k)
    for k in (9, 5, 4):
        post[f"med1_{k}"] = nd.median_filter(post["x1"], size=k)
    d = rng.standard_normal((50, 30)) * 1e-3 + 5.0
    post["d"] = d
    post["demean"] = (d - np.mean(d[:, 5:17], axis=1).reshape(-1, 1)) * float((116 * 500.0 / 10.0) / 1e9)
    np.savez_compressed(os.path.join(HERE, "post.npz"), **post)
    print("next-row golden vectors written to", HERE)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "next":
        main_next_rows()
    else:
        main()
        main_next_rows()
