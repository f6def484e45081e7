"""SURVEY §8(f) rows beside the hot path, each to the same bar:
band-/high-pass ``pass_filter`` through the same device kernels, DASCore
``decimate(filter_type='iir' | 'fir')`` (restated as scipy.signal.decimate), and the
notebook post-processing (demean + strain-rate scale, scipy.ndimage
median_filter) on device.

CPU: the oracle restatements against the SciPy goldens (tests/golden/
make_golden.py main_next_rows).  GPU: device results against the oracle —
median filter bit-exact (the output is an input value), demean/scale and
filters within relRMS 1e-9 / 1e-4 (float64 / float32-sample paths)."""
import os

import numpy as np
import pytest

import gates
import oracle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
T0 = np.datetime64("2023-03-22T03:00:00", "ns")


def _g(name):
    return np.load(os.path.join(GOLD, name))


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(np.sum((a - b) ** 2) / np.sum(b ** 2)))


# ---------------------------------------------------------------- CPU ---
def test_bandpass_design_matches_golden():
    g = _g("band_decimate.npz")
    for i in range(3):
        N, w0, w1 = g[f"case_{i}"]
        np.testing.assert_allclose(oracle.butter_sos(int(N), [w0, w1], "bandpass"), g[f"sos_{i}"],
                                   rtol=0, atol=1e-15)
    assert _rel(oracle.sosfiltfilt(g["sos_0"], g["x"]), g["y_bp0"]) < 1e-13


@pytest.mark.parametrize("q", [2, 5, 10, 50])
def test_decimate_iir_matches_golden(q):
    g = _g("band_decimate.npz")
    np.testing.assert_allclose(oracle.cheby1_sos(8, 0.05, 0.8 / q), g[f"cheby_{q}"], rtol=0, atol=1e-15)
    assert _rel(oracle.decimate_iir(g["x"], q), g[f"dec_{q}"]) < 1e-13


@pytest.mark.parametrize("q", [2, 5, 10, 50])
def test_decimate_fir_matches_golden(q):
    """decimate(ftype='fir'): firwin(20q+1, 1/q, 'hamming') and resample_poly
    restated; the device design helper uses the same taps and centring."""
    from lfdas.proc import fir_decimate_design
    g = _g("band_decimate.npz")
    np.testing.assert_allclose(oracle.firwin_hamming(20 * q + 1, 1.0 / q), g[f"firwin_{q}"], rtol=0, atol=1e-16)
    assert _rel(oracle.decimate_fir(g["x"], q), g[f"decfir_{q}"]) < 1e-13
    taps, delay = fir_decimate_design(q)
    np.testing.assert_array_equal(taps[taps.size - 20 * q - 1:], g[f"firwin_{q}"])
    assert not np.any(taps[:taps.size - 20 * q - 1])
    # y[k] = sum_i taps[i] x[k q + delay - i]: the restated kernel formula
    x = g["x"]
    xp = np.concatenate([np.zeros((x.shape[0], taps.size)), x, np.zeros((x.shape[0], delay + q))], axis=1)
    n_out = -(-x.shape[1] // q)
    k = np.arange(n_out)
    y = np.stack([xp[:, taps.size + k * q + delay - i] for i in range(taps.size)], 0)
    assert _rel(np.einsum("i,irk->rk", taps, y), g[f"decfir_{q}"]) < 1e-13


def test_median_and_demean_match_golden():
    g = _g("post.npz")
    for k in (5, (3, 7), 4, (9, 3), 11):
        tag = "x".join(str(v) for v in np.atleast_1d(k))
        np.testing.assert_array_equal(oracle.median_filter(g["x2"], k), g[f"med2_{tag}"])
    for k in (9, 5, 4):
        np.testing.assert_array_equal(oracle.median_filter(g["x1"], k), g[f"med1_{k}"])
    np.testing.assert_allclose(oracle.demean_scale(g["d"], 5, 17, (116 * 500.0 / 10.0) / 1e9), g["demean"],
                               rtol=1e-12, atol=0)


def test_scale_iDAS():
    from lfdas.post import scale_iDAS
    assert scale_iDAS(500.0, 10.0) == float((116 * 500.0 / 10.0) / 1e9)


# ---------------------------------------------------------------- GPU ---
def _patch(x, fs):
    import lfdas.dc as dc
    t = T0 + np.arange(x.shape[1]) * np.timedelta64(int(round(1e9 / fs)), "ns")
    return dc.Patch(data=x, coords={"distance": np.arange(float(x.shape[0])), "time": t},
                    dims=("distance", "time"))


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["row", "col"])
def test_median_filter_device_bit_exact(layout):
    from lfdas.post import median_filter
    rng = np.random.default_rng(5)
    x = rng.standard_normal((137, 61))
    if layout == "col":
        x = np.asfortranarray(x)
    for k in (5, (3, 7), 4, (9, 3), 11, 1, (1, 9)):
        np.testing.assert_array_equal(median_filter(x, k), oracle.median_filter(x, k))
    tr = rng.standard_normal(300)
    for k in (9, 5, 4):
        np.testing.assert_array_equal(median_filter(tr, k), oracle.median_filter(tr, k))
    # the notebook's 2-D use on a (time, distance) low-passed result (cell 20)
    big = rng.standard_normal((1400, 96))
    np.testing.assert_array_equal(median_filter(big, 5), oracle.median_filter(big, 5))


@pytest.mark.gpu
def test_demean_scale_device():
    from lfdas.post import demean_scale, scale_iDAS
    g = _g("post.npz")
    s = scale_iDAS(500.0, 10.0)
    y = demean_scale(g["d"], 5, 17, s)
    assert _rel(y, g["demean"]) < 1e-12
    x = np.random.default_rng(6).standard_normal((3000, 955)) * 1e-6 + 1e-4
    assert _rel(demean_scale(x, 0, 200, s), oracle.demean_scale(x, 0, 200, s)) < 1e-12
    with pytest.raises(ValueError):
        demean_scale(x, 10, 10, s)


@pytest.mark.gpu
@pytest.mark.parametrize("band", [(1.0, 10.0), (None, 10.0), (2.0, None), (0.2, 30.0)])
def test_pass_filter_band_and_high_full_rate(band):
    fs = 250.0
    x = np.random.default_rng(8).standard_normal((7, 5000)).astype(np.float32) + 3.0
    y = _patch(x, fs).pass_filter(time=band).data
    ref = oracle.sosfiltfilt(oracle.dascore_pass_filter_sos(fs, band[0], band[1]), x)
    assert y.dtype == np.float64 and _rel(y, ref) < 1e-9


@pytest.mark.gpu
def test_bandpass_interpolate_uses_block_path():
    fs = 250.0
    x = np.random.default_rng(9).standard_normal((9, 6000)).astype(np.float32)
    p = _patch(x, fs)
    grid = p.coords["time"][::25][1:-2]
    out = p.pass_filter(time=(0.5, 4.0)).interpolate(time=grid)
    ref = oracle.sosfiltfilt(oracle.dascore_pass_filter_sos(fs, 0.5, 4.0), x)[:, 25::25][:, :len(grid)]
    assert out.data.dtype == np.float64
    gates.check("bandpass_interpolate", _rel(out.data, ref), gates.REC)


@pytest.mark.gpu
@pytest.mark.parametrize("q", [2, 5, 10, 50])
def test_decimate_iir_device(q):
    g = _g("band_decimate.npz")
    x = g["x"]
    p = _patch(x, 250.0)
    out = p.decimate(time=q, filter_type="iir")
    ref = oracle.decimate_iir(x.astype(np.float32).astype(np.float64), q)
    assert out.data.shape == ref.shape
    np.testing.assert_array_equal(out.coords["time"], p.coords["time"][::q])
    gates.check(f"decimate_iir q={q}", _rel(out.data, ref), gates.REC)
    # SciPy on the float64 data: the float32 sample quantisation (~3e-8 of
    # the samples) bounds this one
    gates.check(f"decimate_iir_golden q={q}", _rel(out.data, g[f"dec_{q}"]), gates.Q32)
    with pytest.raises(ValueError):
        p.decimate(time=q, filter_type="kaiser")


@pytest.mark.gpu
@pytest.mark.parametrize("q", [2, 5, 10, 50])
@pytest.mark.parametrize("layout", ["row", "col"])
def test_decimate_fir_device(q, layout):
    """decimate(filter_type='fir') on device (lfd_fir_decimate_f32): float64
    FIR at the kept samples vs the oracle on the same float32 samples
    (relRMS 1e-12) and vs SciPy on the float64 data (1e-6); a NaN poisons
    exactly the outputs whose window holds it."""
    import lfdas.dc as dc
    g = _g("band_decimate.npz")
    x = g["x"]
    x32 = x.astype(np.float32)
    if layout == "row":
        p = _patch(x, 250.0)
    else:
        t = T0 + np.arange(x.shape[1]) * np.timedelta64(4_000_000, "ns")
        p = dc.Patch(data=np.ascontiguousarray(x.T), coords={"time": t, "distance": np.arange(float(x.shape[0]))},
                     dims=("time", "distance"))
    out = p.decimate(time=q, filter_type="fir")
    d = out.data if layout == "row" else out.data.T
    ref = oracle.decimate_fir(x32.astype(np.float64), q)
    assert d.dtype == np.float64 and d.shape == ref.shape
    np.testing.assert_array_equal(out.coords["time"], p.coords["time"][::q])
    assert _rel(d, ref) < 1e-12
    assert _rel(d, g[f"decfir_{q}"]) < 1e-6
    xn = x32.copy()
    xn[1, 1234] = np.nan
    dn = _patch(xn, 250.0).decimate(time=q, filter_type="fir").data
    refn = oracle.decimate_fir(xn.astype(np.float64), q)
    np.testing.assert_array_equal(np.isnan(dn), np.isnan(refn))
    assert np.isnan(dn).sum() > 0
    if 4 <= q <= 10 and layout == "row":  # time-contiguous rows, firwin(20q+1) pieces fit the matrix-core kernel
        from lfdas._lib import load
        assert load().lfd_fir_decimate_last_kernel() == 1


@pytest.mark.parametrize("q", [4, 5, 6, 8, 10])
def test_fir_mfma_toeplitz_model_matches_oracle(q):
    """CPU model of the matrix-core FIR kernel's decomposition (4 x 4 Toeplitz
    pieces over the polyphase rows, 6 steps + the row-0 epilogue tap) equals
    scipy.signal.decimate(ftype='fir') as restated by the oracle (1e-13)."""
    from emulate import fir_decimate_mfma_model
    from lfdas.proc import fir_decimate_design
    rng = np.random.default_rng(q)
    x = rng.standard_normal((3, 40 * q + 7))
    taps, delay = fir_decimate_design(q)
    assert taps.size == 21 * q + 1
    y = fir_decimate_mfma_model(x, taps, q, delay)
    assert _rel(y, oracle.decimate_fir(x, q)) < 1e-13
    # any filter of 21 q + 1 taps (firwin's end taps are ~1e-18, so random
    # taps exercise the row-0 epilogue tap h[21 q]) vs the direct sum
    h = rng.standard_normal(21 * q + 1)
    n_out = -(-x.shape[1] // q)
    ref = np.zeros((3, n_out))
    for o in range(n_out):
        for i in range(h.size):
            t = o * q + delay - i
            if 0 <= t < x.shape[1]:
                ref[:, o] += h[i] * x[:, t]
    assert _rel(fir_decimate_mfma_model(x, h, q, delay), ref) < 1e-13


@pytest.mark.gpu
@pytest.mark.parametrize("q", [4, 10])
@pytest.mark.parametrize("aligned", [False, True])
def test_decimate_fir_device_nulls_and_ragged(q, aligned):
    """Matrix-core FIR decimation on a ragged array (6 channels: one
    partial 4-channel group; several 256-output tiles) with NaN / +-inf
    samples at tile edges, inside the zero pre-pad taps' reach and in the
    Toeplitz corners: the NaN / inf footprint and every finite value match
    the oracle (relRMS 1e-12 over finite outputs).  Odd record lengths stage
    every tile through registers; aligned ones (16-B rows) by LDS-DMA except
    at the record's edges."""
    import torch
    from lfdas._lib import load
    from lfdas.plan import fir_decimate_device
    from lfdas.proc import fir_decimate_design
    rng = np.random.default_rng(7 + q)
    n_ch, n_t = 6, (256 * q * 5 if aligned else 256 * q * 3 + 17 * q + 5)
    x = rng.standard_normal((n_ch, n_t)).astype(np.float32)
    tile = 256 * q
    x[0, tile - 1] = np.nan
    x[1, tile] = np.inf
    x[2, 2 * tile + 3] = -np.inf
    x[3, 5] = np.nan
    x[4, n_t - 1] = np.nan
    x[5, 1000] = np.inf
    x[5, 1000 + q] = -np.inf  # +inf and -inf in one window -> NaN
    taps, delay = fir_decimate_design(q)
    y = fir_decimate_device(torch.from_numpy(x).cuda(), taps, q, delay).cpu().numpy()
    assert load().lfd_fir_decimate_last_kernel() == 1
    ref = oracle.decimate_fir(x.astype(np.float64), q)
    assert y.shape == ref.shape
    np.testing.assert_array_equal(np.isnan(y), np.isnan(ref))
    np.testing.assert_array_equal(np.isposinf(y), np.isposinf(ref))
    np.testing.assert_array_equal(np.isneginf(y), np.isneginf(ref))
    f = np.isfinite(ref)
    assert _rel(y[f], ref[f]) < 1e-12
    # a random filter of 21 q + 1 taps (firwin's end taps are ~1e-18): the
    # row-0 epilogue tap h[21 q] and every Toeplitz slot carry weight
    from emulate import fir_decimate_mfma_model
    h = rng.standard_normal(21 * q + 1)
    xf = np.nan_to_num(x, nan=0.0, posinf=0.0, neginf=0.0)
    y2 = fir_decimate_device(torch.from_numpy(xf).cuda(), h, q, delay).cpu().numpy()
    assert load().lfd_fir_decimate_last_kernel() == 1
    assert _rel(y2, fir_decimate_mfma_model(xf.astype(np.float64), h, q, delay)) < 1e-12


def _layout(x, kind):
    import torch
    if kind == "row":
        return torch.from_numpy(x).cuda()
    if kind == "col":
        return torch.from_numpy(np.ascontiguousarray(x.T)).cuda().t()
    full = torch.from_numpy(np.concatenate([np.zeros((x.shape[0], 1), np.float32), x], 1)).cuda()
    return full[:, 1:]  # rows 4 B past 16-B alignment


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(10))
def test_fullrate_random_geometry(seed):
    """Ten seeded random full-rate zero-phase filters (Patch.pass_filter(...)
    .data: low / high / band-pass, 2 - 8 corners, rates 50 Hz - 2 kHz,
    records from just past padlen to 120,000 samples, SciPy's or a random
    padlen, three row layouts) against the oracle's sosfiltfilt, gated per
    geometry at 10x its measured relRMS."""
    from lfdas.plan import sosfiltfilt_device
    rng = np.random.default_rng(3000 + seed)
    fs = float(rng.choice([50.0, 100.0, 250.0, 500.0, 1000.0, 2000.0]))
    kind = str(rng.choice(["low", "high", "band"]))
    corners = int(rng.choice([2, 4])) if kind == "band" else int(rng.choice([2, 4, 6, 8]))
    f1 = float(fs * rng.uniform(0.002, 0.2))
    f2 = float(min(fs * 0.45, f1 * rng.uniform(1.5, 8.0)))
    lo, hi = {"low": (None, f1), "high": (f1, None), "band": (f1, f2)}[kind]
    sos = oracle.dascore_pass_filter_sos(fs, lo, hi, corners)
    pad_ref = oracle.sosfiltfilt_ref_padlen(sos)
    padlen = None if rng.random() < 0.6 else int(rng.integers(0, 3 * pad_ref + 1))
    pl = pad_ref if padlen is None else padlen
    n_t = int(rng.integers(pl + 2, pl + 200)) if rng.random() < 0.3 else int(rng.integers(2_000, 120_001))
    n_ch = int(rng.integers(1, 17))
    layout = str(rng.choice(["row", "col", "row_unaligned"]))
    x = (rng.standard_normal((n_ch, n_t)) + 2.0).astype(np.float32)
    y = sosfiltfilt_device(_layout(x, layout), sos, -1 if padlen is None else padlen).cpu().numpy()
    ref = oracle.sosfiltfilt(sos, x, padlen=padlen)
    assert y.shape == ref.shape and np.isfinite(y).all()
    gates.check(f"fullrate_random seed={seed} {(fs, kind, corners, lo, hi, padlen, n_t, n_ch, layout)}",
                _rel(y, ref), gates.PATHS)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(10))
def test_fir_decimate_random_geometry(seed):
    """Ten seeded random FIR decimations (decimate(q, ftype='fir'): q 2 - 12,
    records of 3 - 200,000 samples, 1 - 16 channels, three row layouts, a
    NaN in some) against the oracle on the same float32 samples: identical
    NaN footprint, relRMS gated per geometry at 10x its measured value."""
    from lfdas.plan import fir_decimate_device
    from lfdas.proc import fir_decimate_design
    rng = np.random.default_rng(4000 + seed)
    q = int(rng.integers(2, 13))
    n_t = int(rng.integers(3, 400)) if rng.random() < 0.3 else int(rng.integers(1_000, 200_001))
    n_ch = int(rng.integers(1, 17))
    layout = str(rng.choice(["row", "col", "row_unaligned"]))
    x = (rng.standard_normal((n_ch, n_t)) + 1.0).astype(np.float32)
    if rng.random() < 0.4:
        x[int(rng.integers(0, n_ch)), int(rng.integers(0, n_t))] = np.nan
    taps, delay = fir_decimate_design(q)
    y = fir_decimate_device(_layout(x, layout), taps, q, delay).cpu().numpy()
    ref = oracle.decimate_fir(x.astype(np.float64), q)
    assert y.shape == ref.shape
    np.testing.assert_array_equal(np.isnan(y), np.isnan(ref))
    m = np.isfinite(ref)
    gates.check(f"fir_random seed={seed} {(q, n_t, n_ch, layout)}", _rel(y[m], ref[m]), gates.PATHS)
