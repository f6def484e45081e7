"""GPU parity of the chunked low-pass + decimate path (liblfdas.so) against
the oracle (restated LFProc.process_time_range → sosfiltfilt → interp1d).
Outputs are float64 (SciPy's dtype); gates (tests/gates.py) sit at <= 10x
the measured relRMS, far inside north_star's 1e-4; identical output
times/shapes."""
import numpy as np
import pytest

import gates
import oracle
from lfdas import schedule as S
from lfdas._lib import kernel_options

pytestmark = pytest.mark.gpu

T0 = 1_505_692_800_000_000_000  # 2017-09-18T00:00:00 (DASCore random_das)


def _relrms(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(np.sum((a - b) ** 2) / np.sum(b ** 2)))


def _run(x, fs, dt_out, P, B, layout="tc", off_ns=0):
    """off_ns > 0: the samples start off_ns after the whole second on which
    the output grid starts (a real archive's bgtime; every grid point then
    lies the same fraction w of a sample past a sample)."""
    import torch
    from lfdas.plan import LowpassPlan
    n_ch, n = x.shape
    dt_ns = int(round(1e9 / fs))
    t0 = T0 + off_ns
    t1 = T0 if off_ns == 0 else T0 + 1_000_000_000
    tg = S.time_grid(t1, t0 + n * dt_ns, dt_out)
    sched = S.lfproc_chunks(len(tg), P, B)
    lo, w = S.grid_positions(t0, dt_ns, tg)
    chunks = [(*S.select_range(t0, dt_ns, n, tg[a], tg[b]), oa, ob) for a, b, oa, ob in sched]
    sos = oracle.butter_sos(4, (1 / dt_out / 2 * 0.9) / (fs / 2))
    plan = LowpassPlan(sos, n_ch, n, lo, w, chunks)
    if layout == "tc":
        xd = torch.from_numpy(x).cuda()
    else:  # channel-contiguous (time, distance) storage, viewed as (ch, t)
        xd = torch.from_numpy(np.ascontiguousarray(x.T)).cuda().t()
    yd = torch.full((n_ch, len(tg)), float("nan"), dtype=torch.float64, device="cuda")
    plan.execute(xd, yd, plan.alloc_workspace())
    torch.cuda.synchronize()
    _run.last_kernel = plan.last_kernel()
    _run.last_scan = plan.last_scan()
    _run.lattice = plan.lattice()[:2]
    y = yd.cpu().numpy()
    ref = oracle.lfproc_process(x, t0, dt_ns, tg[0], tg[-1] + 1, dt_out, P, B)
    _run.w = w
    return y, ref, sched


@pytest.mark.parametrize("layout", ["tc", "cc"])
@pytest.mark.parametrize("cfg", [
    (250.0, 0.2, 40, 6, 24, 24.0),     # cfg1 geometry (R = 50)
    (500.0, 1.0, 600, 7, 16, 1500.0),  # cfg3 parameters (R = 500, Wn = 1.8e-3)
    (200.0, 10.0, 100, 7, 8, 3000.0),  # cfg5 parameters (R = 2000 = 4 sub-blocks, Wn = 4.5e-4)
    (1000.0, 1.0, 30, 3, 70, 100.0),   # ragged channel count, short chunks
])
@pytest.mark.parametrize("dc,off_ns", [(0.0, 0), (1000.0, 0), (0.0, 370_000), (0.0, 1_900_000)])
def test_lfproc_parity(cfg, dc, layout, off_ns):
    fs, dt_out, P, B, n_ch, dur = cfg
    n = int(dur * fs)
    rng = np.random.default_rng(11)
    t = np.arange(n) / fs
    x = (rng.standard_normal((n_ch, n)) + np.sin(2 * np.pi * 0.01 * t) + dc).astype(np.float32)
    y, ref, sched = _run(x, fs, dt_out, P, B, layout, off_ns=off_ns)
    assert np.all(_run.w == _run.w[0]) and (_run.w[0] != 0) == (off_ns % int(round(1e9 / fs)) != 0)
    produced = np.zeros(y.shape[1], bool)
    num = den = 0.0
    for (tt, r), (a, b, oa, ob) in zip(ref, sched):
        assert r.shape == (n_ch, ob - oa)
        num += float(np.sum((y[:, oa:ob] - r) ** 2))
        den += float(np.sum(r ** 2))
        produced[oa:ob] = True
    gates.check(f"lfproc_parity {cfg} dc={dc} {layout} off={off_ns}", (num / den) ** 0.5, gates.MFMA)
    assert np.all(np.isnan(y[:, ~produced]))  # trimmed edges untouched
    # contiguous rows run the fp64-MFMA block taps; strided rows the recurrence;
    # both fold into runs (in registers where the MFMA kernel's LDS fits the
    # run buffers, else by the separate fold kernel: L = 2000, recurrence)
    # (off-sample grids stay on the block plan: the blended output functional)
    assert _run.last_kernel == ("mfma_runs" if layout == "tc" else "mfma_runs_tm")


@pytest.mark.parametrize("cfg", [
    (250.0, 0.2, 40, 6, 1, 24.0),      # one channel
    (250.0, 0.2, 1000, 6, 5, 24.0),    # process_patch_size beyond the grid: one chunk
    (250.0, 0.2, 13, 6, 3, 24.0),      # P = 2B + 1 (the smallest the reference terminates on): 1 output per chunk
    (250.0, 0.2, 40, 6, 3, 6.0),       # a record barely longer than the edge buffers
    (500.0, 1.0, 20, 2, 65, 40.0),     # 65 channels (one past a 64-channel group), B = 2
])
def test_lfproc_parity_degenerate(cfg):
    """Degenerate LFProc geometries (lf_das.py:252-290): a single channel, a
    single chunk, one output per chunk, a record barely longer than the edge
    buffers, a ragged 64-channel group — identical chunk shapes and outputs
    within the gate of the regular cases."""
    fs, dt_out, P, B, n_ch, dur = cfg
    n = int(dur * fs)
    rng = np.random.default_rng(23)
    x = (rng.standard_normal((n_ch, n)) + 3.0).astype(np.float32)
    y, ref, sched = _run(x, fs, dt_out, P, B)
    assert len(ref) == len(sched) and len(sched) >= 1
    num = den = 0.0
    for (tt, r), (a, b, oa, ob) in zip(ref, sched):
        assert r.shape == (n_ch, ob - oa)
        num += float(np.sum((y[:, oa:ob] - r) ** 2))
        den += float(np.sum(r ** 2))
    gates.check(f"lfproc_parity_degenerate {cfg}", (num / den) ** 0.5, gates.MFMA)


def _random_geometry(seed):
    """A seeded random LFProc geometry: sampling rate, output interval
    (R = fs dt_out >= 10 samples per output), edge buffer, patch size, grid
    length, channel count, start offset and storage layout."""
    rng = np.random.default_rng(1000 + seed)
    while True:
        fs = float(rng.choice([100.0, 200.0, 250.0, 500.0, 1000.0, 2000.0]))
        dt_out = float(rng.choice([0.2, 0.5, 1.0, 2.0, 5.0, 10.0]))
        if abs(fs * dt_out - round(fs * dt_out)) < 1e-9 and fs * dt_out >= 10:
            break
    B = int(rng.integers(1, 9))
    P = int(rng.integers(2 * B + 1, 2 * B + 61))
    n_grid = int(rng.integers(P, 4 * P + 1))
    n = int(n_grid * dt_out * fs) + int(rng.integers(1, int(fs) + 2))
    n_ch = int(rng.integers(1, 81))
    while n_ch * n > 30_000_000 and n_ch > 1:
        n_ch //= 2
    dt_ns = int(round(1e9 / fs))
    off_ns = 0 if rng.random() < 0.4 else int(rng.integers(1, dt_ns))
    layout = "tc" if rng.random() < 0.7 else "cc"
    return fs, dt_out, P, B, n_ch, n, off_ns, layout


@pytest.mark.parametrize("seed", range(12))
def test_lfproc_parity_random_geometry(seed):
    """Twelve seeded random LFProc geometries (rates 100 Hz - 2 kHz, output
    intervals 0.2 - 10 s, edge buffers 1 - 8, patch sizes 2B + 1 .. 2B + 60,
    1 - 80 channels, on- and off-sample starts, both layouts) against the
    oracle: identical chunk shapes, NaN-free produced outputs, and relRMS
    gated per geometry at 10x its measured value."""
    fs, dt_out, P, B, n_ch, n, off_ns, layout = _random_geometry(seed)
    rng = np.random.default_rng(seed)
    t = np.arange(n) / fs
    x = (rng.standard_normal((n_ch, n)) + np.sin(2 * np.pi * 0.5 / dt_out * 0.3 * t) + 2.0).astype(np.float32)
    y, ref, sched = _run(x, fs, dt_out, P, B, layout, off_ns=off_ns)
    num = den = 0.0
    for (tt, r), (a, b, oa, ob) in zip(ref, sched):
        assert r.shape == (n_ch, ob - oa)
        assert not np.isnan(y[:, oa:ob]).any()
        num += float(np.sum((y[:, oa:ob] - r) ** 2))
        den += float(np.sum(r ** 2))
    gates.check(f"lfproc_parity_random seed={seed} {(fs, dt_out, P, B, n_ch, n, off_ns, layout)}",
                (num / den) ** 0.5, gates.MFMA)


@pytest.mark.parametrize("phases", [False, True])
@pytest.mark.parametrize("layout,off_ns,null", [("tc", 0, False), ("tc", 123_457, False), ("cc", 123_457, False),
                                                ("tc", 0, True)])
def test_lfproc_parity_lattice_grid(layout, off_ns, null, phases):
    """3 kHz data on integer-ns sample times (333,333 ns): the 1 s output grid
    drifts against the samples, so the fraction w varies from point to point
    and the spacing is 3,000 or 3,001 samples.  The plan decomposes the grid
    into lattice phases and still runs the block-plan kernels: for
    (channel, time) rows one K1 pass forms every phase's outputs (MFMA rows
    8 + d, the one-pass form), otherwise (time-major rows, or option
    lattice_phases) one uniform block sub-plan per phase; then the interp1d
    blend.  Outputs match the oracle (gates.MFMA) with identical shapes."""
    fs, dt_out, P, B, n_ch, dur = 3000.0, 1.0, 120, 7, 20, 1300.0
    n = int(dur * fs)
    rng = np.random.default_rng(5)
    t = np.arange(n) / fs
    x = (rng.standard_normal((n_ch, n)) + np.sin(2 * np.pi * 0.02 * t) + 50.0).astype(np.float32)
    if null:  # a NaN in one channel: NaN in every output of the chunks holding it
        x[3, n // 2] = np.nan
    with kernel_options(lattice_phases=1 if phases else 0):
        y, ref, sched = _run(x, fs, dt_out, P, B, layout, off_ns=off_ns)
    assert _run.lattice == ((0 if phases else _run.lattice[0]), layout == "tc" and not phases)
    assert phases or 2 <= _run.lattice[0] <= 8
    w = _run.w
    assert len(np.unique(w)) > 100  # a varying fraction
    num = den = 0.0
    for (tt, r), (a, b, oa, ob) in zip(ref, sched):
        assert r.shape == (n_ch, ob - oa)
        np.testing.assert_array_equal(np.isnan(y[:, oa:ob]), np.isnan(r))
        f = np.isfinite(r)
        num += float(np.sum((y[:, oa:ob][f] - r[f]) ** 2))
        den += float(np.sum(r[f] ** 2))
    # (the phase outputs and the blend are float64: no extra rounding)
    gates.check(f"lattice {layout} off={off_ns} null={null} phases={phases}", (num / den) ** 0.5, gates.MFMA)
    assert _run.last_kernel == ("mfma_runs" if layout == "tc" else "mfma_runs_tm")


@pytest.mark.parametrize("seed", range(6))
def test_lfproc_parity_lattice_random(seed):
    """Six seeded random drifting grids: rates whose integer-ns sample
    interval does not divide the output interval (750 Hz - 6 kHz), 300 -
    1,400 s, random start offset, edge buffer, patch size and layout, the
    one-pass or the per-phase lattice plan — against the oracle, gated per
    geometry at 10x its measured value."""
    rng = np.random.default_rng(6000 + seed)
    fs = float(rng.choice([750.0, 1200.0, 1500.0, 2400.0, 3000.0, 6000.0]))
    dt_out = float(rng.choice([1.0, 2.0]))
    B = int(rng.integers(2, 8))
    P = int(rng.integers(2 * B + 5, 2 * B + 120))
    dur = float(rng.integers(300, 1401))
    n_ch = int(rng.integers(1, 9))
    n = int(dur * fs)
    dt_ns = int(round(1e9 / fs))
    off_ns = int(rng.integers(0, dt_ns))
    layout = "tc" if rng.random() < 0.7 else "cc"
    phases = bool(rng.random() < 0.3)
    t = np.arange(n) / fs
    x = (rng.standard_normal((n_ch, n)) + np.sin(2 * np.pi * 0.02 * t) + 20.0).astype(np.float32)
    with kernel_options(lattice_phases=1 if phases else 0):
        y, ref, sched = _run(x, fs, dt_out, P, B, layout, off_ns=off_ns)
    num = den = 0.0
    for (tt, r), (a, b, oa, ob) in zip(ref, sched):
        assert r.shape == (n_ch, ob - oa)
        assert not np.isnan(y[:, oa:ob]).any()
        num += float(np.sum((y[:, oa:ob] - r) ** 2))
        den += float(np.sum(r ** 2))
    gates.check(f"lattice_random seed={seed} {(fs, dt_out, P, B, n_ch, n, off_ns, layout, phases)} {_run.lattice}",
                (num / den) ** 0.5, gates.MFMA)


def _plan_cfg(fs, dt_out, P, B, n_ch, n):
    from lfdas.plan import LowpassPlan
    dt_ns = int(round(1e9 / fs))
    tg = S.time_grid(T0, T0 + n * dt_ns, dt_out)
    sched = S.lfproc_chunks(len(tg), P, B)
    lo, w = S.grid_positions(T0, dt_ns, tg)
    chunks = [(*S.select_range(T0, dt_ns, n, tg[a], tg[b]), oa, ob) for a, b, oa, ob in sched]
    sos = oracle.butter_sos(4, (1 / dt_out / 2 * 0.9) / (fs / 2))
    return LowpassPlan(sos, n_ch, n, lo, w, chunks), len(tg)


@pytest.mark.parametrize("cfg", [
    (250.0, 0.2, 40, 6, 37, 6000),      # L = 50: four row-shift tap tables
    (500.0, 1.0, 600, 7, 33, 750_000),  # L = 500
    (200.0, 10.0, 100, 7, 5, 600_000),  # R = 2000: 4 sub-blocks of 500
    (1000.0, 0.5, 40, 4, 18, 100_003),  # L = 500, odd n_t (channel stride % 4 != 0: rows 4-B aligned)
])
def test_k1_mfma_matches_recurrence(cfg):
    """Both block-functional kernels feed the same scan: outputs agree to the
    recurrence K1's float32-FIR rounding; the dispatch picks MFMA for every time-contiguous row
    stride (odd record lengths load 4-B aligned 16-B pieces)."""
    import torch
    fs, dt_out, P, B, n_ch, n = cfg
    rng = np.random.default_rng(7)
    x = (rng.standard_normal((n_ch, n)) + 300.0).astype(np.float32)
    plan, n_grid = _plan_cfg(fs, dt_out, P, B, n_ch, n)
    xd = torch.from_numpy(x).cuda()
    ws = plan.alloc_workspace()
    out = {}
    opts = {"default": {}, "noruns": {"no_runs": 1}, "rec": {"no_runs": 1, "k1_recurrence": 1},
            "recfold": {"k1_recurrence": 1}}
    for mode in ("default", "noruns", "rec", "recfold"):
        yd = torch.full((n_ch, n_grid), float("nan"), dtype=torch.float64, device="cuda")
        with kernel_options(**opts[mode]):
            plan.execute(xd, yd, ws)
        torch.cuda.synchronize()
        out[mode] = (yd.cpu().numpy(), plan.last_kernel())
    assert out["default"][1] == "mfma_runs"
    assert out["noruns"][1] == "mfma"
    assert out["rec"][1] == "recurrence"
    assert out["recfold"][1] == "recurrence_fold"
    b = out["rec"][0]
    m = ~np.isnan(b)
    for mode in ("default", "noruns", "recfold"):
        a = out[mode][0]
        assert np.array_equal(np.isnan(a), ~m)
        gates.check(f"k1_vs_rec {cfg} {mode}", _relrms(a[m], b[m]), gates.PATHS if mode == "recfold" else gates.REC)


def test_k1_unaligned_base_pointer():
    """A view starting one sample in (rows not 16-B aligned) runs the same
    MFMA run kernel as an aligned copy of the same rows — bit-identical
    outputs — and matches the recurrence kernel."""
    import torch
    fs, dt_out, P, B = 500.0, 1.0, 60, 7
    n_ch, n = 9, 40_000
    rng = np.random.default_rng(2)
    x = (rng.standard_normal((n_ch, n + 4)) + 1.0).astype(np.float32)
    plan, n_grid = _plan_cfg(fs, dt_out, P, B, n_ch, n)
    full = torch.from_numpy(x).cuda()
    xd = full[:, 1:n + 1]
    yd = torch.full((n_ch, n_grid), float("nan"), dtype=torch.float64, device="cuda")
    plan.execute(xd, yd, plan.alloc_workspace())
    assert plan.last_kernel() == "mfma_runs"
    y_ok = yd.cpu().numpy()
    yr = torch.full((n_ch, n_grid), float("nan"), dtype=torch.float64, device="cuda")
    with kernel_options(k1_recurrence=1):
        plan.execute(xd, yr, plan.alloc_workspace())
    assert plan.last_kernel() == "recurrence_fold"
    y_rec = yr.cpu().numpy()
    xa = torch.from_numpy(np.ascontiguousarray(x[:, 1:n + 1])).cuda()
    yd2 = torch.full((n_ch, n_grid), float("nan"), dtype=torch.float64, device="cuda")
    plan.execute(xa, yd2, plan.alloc_workspace())
    assert plan.last_kernel() == "mfma_runs"
    y2 = yd2.cpu().numpy()
    m = ~np.isnan(y2)
    np.testing.assert_array_equal(y_ok, y2)
    gates.check("k1_unaligned_vs_rec", _relrms(y_rec[m], y2[m]), gates.REC)


def test_cfg1_random_das():
    """cfg1: 3 random_das patches (300 ch x 2000 @ 250 Hz) merged, dt=0.2 s."""
    x = np.concatenate([np.random.RandomState(42).random((300, 2000))] * 3, axis=1).astype(np.float32)
    y, ref, sched = _run(x, 250.0, 0.2, 40, 6)
    for (tt, r), (a, b, oa, ob) in zip(ref, sched):
        gates.check(f"cfg1_random_das {oa}", _relrms(y[:, oa:ob], r), gates.MFMA)


@pytest.mark.parametrize("cfg", [
    (1000.0, 10.0, 30, 6, 8, 1200.0),   # the batch notebook's d_t = 10 s at 1 kHz: R = 10,000
    (2000.0, 10.0, 30, 6, 5, 900.0),    # ... at 2 kHz: R = 20,000
    (2000.0, 1.0, 125, 7, 12, 400.0),   # cfg4 parameters: R = 2000
])
@pytest.mark.parametrize("off_ns", [0, 370_000])
def test_long_grid_spacing_runs_mfma(cfg, off_ns):
    """Grid spacings far beyond one LDS tap table run as sub-blocks of <= 504
    samples (outputs at every kstep-th block start) on the MFMA run kernel."""
    fs, dt_out, P, B, n_ch, dur = cfg
    n = int(dur * fs)
    rng = np.random.default_rng(17)
    t = np.arange(n) / fs
    x = (rng.standard_normal((n_ch, n)) + np.sin(2 * np.pi * 0.004 * t) + 20.0).astype(np.float32)
    y, ref, sched = _run(x, fs, dt_out, P, B, "tc", off_ns=off_ns)
    assert _run.last_kernel == "mfma_runs"
    num = den = 0.0
    for (tt, r), (a, b, oa, ob) in zip(ref, sched):
        assert r.shape == (n_ch, ob - oa)
        num += float(np.sum((y[:, oa:ob] - r) ** 2))
        den += float(np.sum(r ** 2))
    gates.check(f"long_grid {cfg} off={off_ns}", (num / den) ** 0.5, gates.MFMA)


@pytest.mark.parametrize("W,S_", [(1000, 1), (1000, 250), (1000, 1000), (1000, 3), (999, 7), (64, 1),
                                  (4000, 7),  # W + 512 > 4096: x[t - W] re-read, no LDS ring
                                  # gcd(W, S) >= 16: segment prefix sums (k_rolling_seg)
                                  (1000, 200), (1000, 400), (2500, 1000), (4096, 64), (48, 16), (1000, 500)])
def test_rolling_mean_window_step(W, S_):
    """Overlapping windows (step < window) run the running-sum scan kernel
    (every sample read once), or segment prefix sums when gcd(W, S) >= 16;
    step >= window sums each window directly."""
    import torch
    from lfdas.plan import rolling_mean_device
    rng = np.random.default_rng(W + S_)
    n_ch, n = 5, 12_345
    x = (rng.standard_normal((n_ch, n)) + 3.0).astype(np.float32)
    ref = oracle.rolling_mean(x, W, S_)
    for layout in ("tc", "cc", "tc_unaligned"):
        if layout == "tc":
            xd = torch.from_numpy(x).cuda()
        elif layout == "cc":
            xd = torch.from_numpy(np.ascontiguousarray(x.T)).cuda().t()
        else:
            full = torch.from_numpy(np.concatenate([np.zeros((n_ch, 1), np.float32), x], 1)).cuda()
            xd = full[:, 1:]
        y = rolling_mean_device(xd, W, S_).cpu().numpy()
        assert y.shape == ref.shape
        m = ~np.isnan(ref)
        assert np.array_equal(np.isnan(y), ~m), layout
        gates.check(f"rolling_window_step W={W} S={S_} {layout}", _relrms(y[m], ref[m]), gates.ROLL)


@pytest.mark.parametrize("seed", range(12))
def test_rolling_mean_random_geometry(seed):
    """Twelve seeded random rolling-mean geometries (window 1 - 5,000, step 1 -
    2 x window, 1 - 40 channels, contiguous / strided / 4-B offset rows, a
    NaN and an inf in some) against the oracle: identical null footprint, and
    relRMS gated per geometry at 10x its measured value (most are 0)."""
    import torch
    from lfdas.plan import rolling_mean_device
    rng = np.random.default_rng(2000 + seed)
    W = int(rng.integers(1, 5001))
    S_ = int(rng.integers(1, 2 * W + 1)) if rng.random() < 0.5 else int(rng.choice([1, max(1, W // 4), W]))
    n = int(rng.integers(W, 40 * W + 2)) if W > 100 else int(rng.integers(W, 4000 + W))
    n_ch = int(rng.integers(1, 41))
    while n_ch * n > 20_000_000 and n_ch > 1:
        n_ch //= 2
    x = (rng.standard_normal((n_ch, n)) + 1.5).astype(np.float32)
    if rng.random() < 0.5:
        x[int(rng.integers(0, n_ch)), int(rng.integers(0, n))] = np.nan
        x[int(rng.integers(0, n_ch)), int(rng.integers(0, n))] = np.inf
    layout = str(rng.choice(["tc", "cc", "tc_unaligned"]))
    if layout == "tc":
        xd = torch.from_numpy(x).cuda()
    elif layout == "cc":
        xd = torch.from_numpy(np.ascontiguousarray(x.T)).cuda().t()
    else:
        full = torch.from_numpy(np.concatenate([np.zeros((n_ch, 1), np.float32), x], 1)).cuda()
        xd = full[:, 1:]
    ref = oracle.rolling_mean(x, W, S_)
    y = rolling_mean_device(xd, W, S_).cpu().numpy()
    assert y.shape == ref.shape
    np.testing.assert_array_equal(np.isnan(y), np.isnan(ref))
    np.testing.assert_array_equal(np.isposinf(y), np.isposinf(ref))
    m = np.isfinite(ref)
    gates.check(f"rolling_random seed={seed} {(W, S_, n, n_ch, layout)}",
                _relrms(y[m], ref[m]) if m.any() else 0.0, gates.ROLL)


@pytest.mark.parametrize("W,S_,n", [
    (320, 16, 12_345),     # 80 outputs per unit: a batch of 64 leaves mid-unit, the rest at its end
    (2032, 1008, 50_000),  # Q = 63: the prefix ring only fits batches of 8 (9 outputs per unit)
    (4096, 64, 40_000),    # batches of 64 inside 256-output units
])
def test_rolling_seg_output_batches(W, S_, n):
    """k_rolling_seg emits its outputs in batches (64, or fewer when the
    prefix ring of 1,024 entries would not hold a batch's windows): batch
    boundaries inside a unit and the ring bound give the oracle's means, with
    nulls spread across batches."""
    import torch
    from lfdas.plan import rolling_mean_device
    rng = np.random.default_rng(W + S_ + n)
    n_ch = 3
    x = (rng.standard_normal((n_ch, n)) + 3.0).astype(np.float32)
    x[1, n // 3] = np.nan
    x[2, n // 2] = np.inf
    ref = oracle.rolling_mean(x, W, S_)
    y = rolling_mean_device(torch.from_numpy(x).cuda(), W, S_).cpu().numpy()
    assert y.shape == ref.shape
    np.testing.assert_array_equal(np.isnan(y), np.isnan(ref))
    np.testing.assert_array_equal(np.isposinf(y), np.isposinf(ref))
    m = np.isfinite(ref)
    gates.check(f"rolling_seg_batches W={W} S={S_} n={n}", _relrms(y[m], ref[m]), gates.ROLL)


@pytest.mark.parametrize("S_", [1, 250, 200])
def test_rolling_mean_overlapping_nulls(S_):
    """step < window: a NaN / inf sample turns exactly the windows holding it
    into NaN / inf (the running sum, or the segment prefix ring, carries a
    count of nulls), the rest stay exact, also right after the null leaves
    the window."""
    import torch
    from lfdas.plan import rolling_mean_device
    rng = np.random.default_rng(8)
    n_ch, n, W = 5, 20_000, 1000
    x = (rng.standard_normal((n_ch, n)) + 0.5).astype(np.float32)
    x[0, 2999] = np.nan
    x[1, 5000] = np.inf
    x[2, 7001] = -np.inf
    x[2, 7002] = np.inf    # +inf and -inf in one window: NaN
    x[3, 0] = np.nan       # inside the leading NaN windows and the first full one
    x[4, n - 1] = np.nan   # last window only
    ref = oracle.rolling_mean(x, W, S_)
    for layout in ("tc", "cc"):
        xd = torch.from_numpy(x).cuda() if layout == "tc" else torch.from_numpy(np.ascontiguousarray(x.T)).cuda().t()
        y = rolling_mean_device(xd, W, S_).cpu().numpy()
        assert np.array_equal(np.isnan(y), np.isnan(ref)), layout
        assert np.array_equal(np.isposinf(y), np.isposinf(ref)), layout
        assert np.array_equal(np.isneginf(y), np.isneginf(ref)), layout
        m = np.isfinite(ref)
        gates.check(f"rolling_overlapping_nulls S={S_} {layout}", _relrms(y[m], ref[m]), gates.ROLL)


def test_rolling_mean_parity():
    import torch
    from lfdas.plan import rolling_mean_device
    rng = np.random.default_rng(3)
    for (n_ch, n, W, S_) in [(7, 10000, 1000, 1000), (5, 1003, 7, 13), (3, 20, 5, 3), (64, 4096, 100, 50), (2, 50, 1, 1)]:
        x = (rng.standard_normal((n_ch, n)) + 0.5).astype(np.float32)
        ref = oracle.rolling_mean(x, W, S_)
        for layout in ("tc", "cc"):
            xd = torch.from_numpy(x).cuda() if layout == "tc" else torch.from_numpy(np.ascontiguousarray(x.T)).cuda().t()
            y = rolling_mean_device(xd, W, S_).cpu().numpy()
            assert y.shape == ref.shape
            m = ~np.isnan(ref)
            assert np.array_equal(np.isnan(y), ~m)
            gates.check(f"rolling_parity {(n_ch, n, W, S_)} {layout}", _relrms(y[m], ref[m]), gates.ROLL)


def test_rolling_mean_nulls():
    """A NaN / inf sample affects exactly the windows that contain it (per-window
    mean over the raw values, like DASCore's numpy engine); window edges next to
    it stay exact."""
    import torch
    from lfdas.plan import rolling_mean_device
    rng = np.random.default_rng(4)
    n_ch, n, W, S_ = 6, 10000, 1000, 1000
    x = (rng.standard_normal((n_ch, n)) + 0.5).astype(np.float32)
    x[1, 2999] = np.nan   # inside window k = 3 (samples 2001..3000)
    x[2, 3000] = np.inf   # first sample after window k = 3
    x[3, 4001] = -np.inf
    x[4, 0] = np.nan      # only in the leading (NaN) window
    ref = oracle.rolling_mean(x, W, S_)
    for layout in ("tc", "cc"):
        xd = torch.from_numpy(x).cuda() if layout == "tc" else torch.from_numpy(np.ascontiguousarray(x.T)).cuda().t()
        y = rolling_mean_device(xd, W, S_).cpu().numpy()
        assert np.array_equal(np.isnan(y), np.isnan(ref))
        assert np.array_equal(np.isposinf(y), np.isposinf(ref))
        assert np.array_equal(np.isneginf(y), np.isneginf(ref))
        m = np.isfinite(ref)
        gates.check(f"rolling_nulls {layout}", _relrms(y[m], ref[m]), gates.ROLL)


def test_full_rate_filtfilt_parity():
    import torch
    from lfdas.plan import sosfiltfilt_device
    rng = np.random.default_rng(5)
    x = (rng.standard_normal((33, 3000)) + 5).astype(np.float32)
    sos = oracle.butter_sos(4, 0.02)
    y = sosfiltfilt_device(torch.from_numpy(x).cuda(), sos).cpu().numpy()
    assert _relrms(y, oracle.sosfiltfilt(sos, x)) < 1e-10


@pytest.mark.parametrize("case", [
    # (fs, lo, hi, n_t, padlen): band-pass with heavily damped poles
    # (|p| = 0.48), a low-pass with poles at |p| = 0.9988, 2nd/6th-order
    # cascades, padlen 0 / long, tails of 1..2048 samples (big blocks of 2048)
    (250.0, 0.2, 30.0, 20000, None),
    (500.0, None, 1.0, 9000, None),
    (1000.0, 1.0, 10.0, 2 * 2048 + 1, None),
    (1000.0, 1.0, 10.0, 2 * 2048, None),
    (1000.0, 1.0, 10.0, 3 * 2048 + 5, 0),
    (250.0, 2.0, None, 6000, 700),
    # medium-block path (512): one medium block past the last big block with a
    # 1-sample tail, three past it, a 512-sample tail
    (1000.0, 1.0, 10.0, 9 * 512 + 1, None),
    (1000.0, 1.0, 10.0, 11 * 512 + 77, None),
    (1000.0, 1.0, 10.0, 9 * 512, None),
])
@pytest.mark.parametrize("bigblock", [0, 1])
def test_full_rate_blocked_parity(case, bigblock):
    """lfd_sosfiltfilt_f32's blocked paths against SciPy's sosfiltfilt
    restatement, relRMS < 1e-10 per channel: the medium-block path (matrix-core
    functionals -> k_fullrate_scan_seg -> row-scan output pass, the default
    for time-contiguous rows of any stride: the odd n_t cases run it on rows
    that are not 16-B aligned) and the big-block path (k_fullrate_wave
    functionals -> k_fullrate_scan -> k_fullrate_wave outputs)."""
    import torch
    from lfdas._lib import kernel_options
    from lfdas.plan import sosfiltfilt_device
    fs, lo, hi, n_t, padlen = case
    sos = oracle.dascore_pass_filter_sos(fs, lo, hi)
    rng = np.random.default_rng(n_t)
    x = (rng.standard_normal((5, n_t)) + 3).astype(np.float32)
    pl = -1 if padlen is None else padlen
    with kernel_options(fullrate_bigblock=bigblock):
        y = sosfiltfilt_device(torch.from_numpy(x).cuda(), sos, pl).cpu().numpy()
        ref = oracle.sosfiltfilt(sos, x, padlen=padlen)
        for c in range(x.shape[0]):
            assert _relrms(y[c], ref[c]) < 1e-10, c
        for order in (2, 6):  # other cascade lengths (n_sec = 1, 3)
            sos2 = oracle.butter_sos(order, 0.05)
            y2 = sosfiltfilt_device(torch.from_numpy(x).cuda(), sos2, pl).cpu().numpy()
            assert _relrms(y2, oracle.sosfiltfilt(sos2, x, padlen=padlen)) < 1e-10


def test_full_rate_blocked_strides_and_nan():
    """Strided input (a column view of a (time, channel) array) and a channel
    holding a NaN: the NaN channel is all-NaN like SciPy's, the others are
    unaffected."""
    import torch
    from lfdas.plan import sosfiltfilt_device
    sos = oracle.dascore_pass_filter_sos(500.0, 0.5, 20.0)
    rng = np.random.default_rng(77)
    xt = rng.standard_normal((7000, 6)).astype(np.float32)
    xt[3000, 2] = np.nan
    xd = torch.from_numpy(xt).cuda().t()  # (channel, time) view, s_t = 6
    y = sosfiltfilt_device(xd, sos).cpu().numpy()
    ref = oracle.sosfiltfilt(sos, xt.T)
    assert np.isnan(y[2]).all() and np.isnan(ref[2]).all()
    m = [0, 1, 3, 4, 5]
    assert _relrms(y[m], ref[m]) < 1e-10


def test_execute_is_graph_capturable():
    """lfd_lowpass_execute allocates nothing and never synchronises, so a
    whole chunked low-pass (K1 + scan) can be captured once as a HIP graph and
    replayed (lfdas.h: "hipGraph-capturable")."""
    import torch
    from lfdas.plan import LowpassPlan
    fs, dt_out, P, B, n_ch, dur = 500.0, 1.0, 120, 7, 48, 900.0
    n = int(dur * fs)
    dt_ns = int(round(1e9 / fs))
    tg = S.time_grid(T0, T0 + n * dt_ns, dt_out)
    sched = S.lfproc_chunks(len(tg), P, B)
    lo, w = S.grid_positions(T0, dt_ns, tg)
    chunks = [(*S.select_range(T0, dt_ns, n, tg[a], tg[b]), oa, ob) for a, b, oa, ob in sched]
    sos = oracle.butter_sos(4, (1 / dt_out / 2 * 0.9) / (fs / 2))
    plan = LowpassPlan(sos, n_ch, n, lo, w, chunks)
    x = torch.randn((n_ch, n), device="cuda") + 4.0
    y_eager = torch.zeros((n_ch, len(tg)), dtype=torch.float64, device="cuda")
    y_graph = torch.zeros_like(y_eager)
    ws = plan.alloc_workspace()
    plan.execute(x, y_eager, ws)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            plan.execute(x, y_graph, ws, stream=s)
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(y_graph, y_eager)
    x.mul_(2.0)  # replay sees the new input in place
    g.replay()
    torch.cuda.synchronize()
    assert torch.allclose(y_graph, 2.0 * y_eager, rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("layout", ["tc", "cc"])
@pytest.mark.parametrize("where", ["interior", "before_chunk_start", "after_chunk_end"])
def test_nonfinite_samples_poison_their_chunk_only(where, layout):
    """SciPy semantics for nulls: a NaN or inf sample turns every output of
    its (chunk, channel) into NaN (forward pass, then the reverse pass from
    its NaN end), and nothing else.  Samples right beside a chunk boundary
    (FIR history of the next chunk's first block; zero-tap padding read past
    the previous chunk's last block) must not leak into the neighbour."""
    fs, dt_out, P, B, n_ch, dur = 500.0, 1.0, 600, 7, 8, 1500.0
    n = int(dur * fs)
    x = np.random.default_rng(1).standard_normal((n_ch, n)).astype(np.float32)
    # chunks: samples [0, 600 s], [586 s, 1186 s], [1172 s, 1499 s]
    pos = {"interior": (300.0, 900.0),
           "before_chunk_start": (586.0 - 1 / fs, 1172.0 - 2 / fs),
           "after_chunk_end": (600.0 + 1 / fs, 1186.0 + 3 / fs)}[where]
    x[3, int(round(pos[0] * fs))] = np.nan
    x[5, int(round(pos[1] * fs))] = np.inf
    y, ref, sched = _run(x, fs, dt_out, P, B, layout)
    for (tt, r), (a, b, oa, ob) in zip(ref, sched):
        yy = y[:, oa:ob]
        assert np.array_equal(np.isnan(yy), np.isnan(r)), (where, a, b)
        m = ~np.isnan(r)
        gates.check(f"nonfinite {where} {layout} {a}", _relrms(yy[m], r[m]), gates.MFMA)


@pytest.mark.parametrize("cfg", [
    (250.0, 0.2, 40, 6, 37, 6000, 37),      # L = 50
    (500.0, 1.0, 600, 7, 33, 750_001, 40),  # L = 500, channel subset of a wider (time, ch) array
    (1000.0, 0.5, 40, 4, 18, 100_003, 18),  # odd n_t
    (250.0, 0.2, 40, 6, 70, 6000, 72),      # even channels (channel-pair loads), ragged last wave
])
def test_k1_time_major_fold_matches_blocks(cfg):
    """(time, channel) storage viewed as (channel, time) (s_ch = 1, s_t =
    row width): the time-major MFMA run kernel and the recurrence K1 + run
    fold agree with the per-block scan and with the oracle, nulls included."""
    import torch
    fs, dt_out, P, B, n_ch, n, width = cfg
    rng = np.random.default_rng(9)
    xt = (rng.standard_normal((n, width)) + 30.0).astype(np.float32)
    xt[n // 3, 2] = np.nan  # a null: its chunks' outputs of channel 2 are NaN
    plan, n_grid = _plan_cfg(fs, dt_out, P, B, n_ch, n)
    xd = torch.from_numpy(xt).cuda()[:, :n_ch].t()
    assert xd.stride() == (1, width)
    ws = plan.alloc_workspace()
    out = {}
    # nox2: one dword load per channel instead of channel pairs
    opts = {"default": {}, "nox2": {"tm_no_pairs": 1}, "recfold": {"tm_no_pairs": 1, "k1_recurrence": 1},
            "blocks": {"tm_no_pairs": 1, "k1_recurrence": 1, "no_runs": 1}}
    for mode in ("default", "nox2", "recfold", "blocks"):
        yd = torch.full((n_ch, n_grid), float("nan"), dtype=torch.float64, device="cuda")
        with kernel_options(**opts[mode]):
            plan.execute(xd, yd, ws)
        torch.cuda.synchronize()
        out[mode] = (yd.cpu().numpy(), plan.last_kernel())
    assert out["default"][1] == "mfma_runs_tm"
    assert out["nox2"][1] == "mfma_runs_tm"
    # both load shapes feed the same products; the channel-pair loads group
    # the MFMA accumulations differently (float64 last bits)
    assert np.array_equal(np.isnan(out["default"][0]), np.isnan(out["nox2"][0]))
    fm = np.isfinite(out["nox2"][0])
    gates.check(f"tm_pairs_vs_nox2 {cfg}", _relrms(out["default"][0][fm], out["nox2"][0][fm]), gates.PATHS)
    assert out["recfold"][1] == "recurrence_fold"
    assert out["blocks"][1] == "recurrence"
    b = out["blocks"][0]
    m = ~np.isnan(b)
    for mode in ("default", "recfold"):
        a = out[mode][0]
        assert np.array_equal(np.isnan(a), np.isnan(b)), mode
        gates.check(f"tm_fold {cfg} {mode}", _relrms(a[m], b[m]), gates.REC if mode == "default" else gates.PATHS)
    a = out["default"][0]
    # oracle on the same channels
    x = np.ascontiguousarray(xt[:, :n_ch].T)
    dt_ns = int(round(1e9 / fs))
    tg = S.time_grid(T0, T0 + n * dt_ns, dt_out)
    sched = S.lfproc_chunks(len(tg), P, B)
    ref = oracle.lfproc_process(x, T0, dt_ns, tg[0], tg[-1] + 1, dt_out, P, B)
    for (tt, r), (_, _, oa, ob) in zip(ref, sched):
        yy = a[:, oa:ob]
        assert np.array_equal(np.isnan(yy), np.isnan(r))
        mm = ~np.isnan(r)
        gates.check(f"tm_fold_oracle {cfg}", _relrms(yy[mm], r[mm]), gates.MFMA)


@pytest.mark.parametrize("off_ns", [0, 1_900_000])
def test_scan_deferred_outputs_bit_identical(off_ns):
    """Run-mode scan with the outputs inside the backward chain
    (option scan_defer=1) and deferred to k_run_outputs (=2): same
    arithmetic, bit-identical outputs, both against the oracle."""
    fs, dt_out, P, B, n_ch, dur = 500.0, 1.0, 60, 7, 70, 400.0
    x = (np.random.default_rng(3).standard_normal((n_ch, int(dur * fs))) + 5.0).astype(np.float32)
    out = {}
    for mode in ("0", "1"):
        with kernel_options(scan_defer=1 + int(mode)):
            out[mode] = _run(x, fs, dt_out, P, B, "tc", off_ns=off_ns)
        assert _run.last_kernel == "mfma_runs"
        assert _run.last_scan == ("in_chain" if mode == "0" else "deferred")
    np.testing.assert_array_equal(out["0"][0], out["1"][0])
    y, ref, sched = out["1"]
    for (tt, r), (a, b, oa, ob) in zip(ref, sched):
        gates.check(f"scan_deferred off={off_ns} {oa}", _relrms(y[:, oa:ob], r), gates.MFMA)


@pytest.mark.parametrize("cfg", [
    (500.0, 1.0, 60, 7, 70, 400.0, 0, False),          # short chains (~8 runs per chunk)
    (500.0, 1.0, 600, 7, 33, 1500.0, 123_457, False),  # off-sample grid, head skip
    (1000.0, 10.0, 30, 6, 20, 3000.0, 0, True),        # dt = 10 s: long chains (sub-blocks), a null
])
def test_scan_segmented_chains_match_deferred(cfg):
    """Segmented run chains (option scan_defer = 3: head, per-segment
    forward aggregates + combine, tail, per-segment backward; chosen
    automatically for chunks of >= 128 runs) against the unsegmented deferred
    scan (= 2): the same states up to summation order (gates.PATHS),
    identical NaN footprint — and both against the oracle (gates.MFMA)."""
    fs, dt_out, P, B, n_ch, dur, off_ns, null = cfg
    x = (np.random.default_rng(9).standard_normal((n_ch, int(dur * fs))) + 3.0).astype(np.float32)
    if null:
        x[4, int(dur * fs) // 3] = np.nan
    out = {}
    for mode in (2, 3):
        with kernel_options(scan_defer=mode):
            out[mode] = _run(x, fs, dt_out, P, B, "tc", off_ns=off_ns)
        assert _run.last_kernel == "mfma_runs"
        assert _run.last_scan == {2: "deferred", 3: "segmented"}[mode]
    a, b = out[2][0], out[3][0]
    np.testing.assert_array_equal(np.isnan(a), np.isnan(b))
    f = np.isfinite(a)
    gates.check(f"seg_vs_deferred {cfg}", _relrms(b[f], a[f]), gates.PATHS)
    y, ref, sched = out[3]
    for (tt, r), (lo, hi, oa, ob) in zip(ref, sched):
        fr = np.isfinite(r)
        np.testing.assert_array_equal(np.isnan(y[:, oa:ob]), ~fr)
        gates.check(f"seg_oracle {cfg} {oa}", _relrms(y[:, oa:ob][fr], r[fr]), gates.MFMA)


@pytest.mark.parametrize("cfg", [
    (500.0, 1.0, 60, 7, 70, 400.0, 0, False, "tc"),          # short chains (~8 runs per chunk), ragged 64-groups
    (500.0, 1.0, 600, 7, 130, 1500.0, 123_457, False, "tc"),  # off-sample grid, head skip, 3 x 64-groups
    (500.0, 1.0, 600, 7, 19, 1500.0, 123_457, True, "tc"),    # the same with a null (the right edge's map)
    (1000.0, 10.0, 30, 6, 20, 3000.0, 0, True, "tc"),        # dt = 10 s: long chains (sub-blocks), a null
    (500.0, 1.0, 600, 7, 64, 1200.0, 0, True, "cc"),         # (time, channel) storage, one full 64-group
    (250.0, 0.2, 40, 6, 24, 24.0, 0, False, "tc"),           # cfg1 geometry: 1-run chunks
    (250.0, 0.2, 40, 6, 37, 24.0, 0, False, "fold"),         # recurrence K1 + fold (padding channels unwritten)
])
def test_scan_fused_matches_deferred(cfg):
    """The fused one-launch segmented scan (option scan_defer = 4:
    k_scan_fused, one 256-thread workgroup per chunk x 16 channels, one
    segment of the run chain per 16 lanes, the outputs formed in the backward
    walk) against the deferred two-launch scan (= 2): the same states up to
    summation order (gates.PATHS, identical NaN footprint), and both against
    the oracle (gates.MFMA).  Chunks whose run chains exceed the fused scan's
    segment table fall back to the default choice (lfd_lowpass_last_scan
    says which ran; every case here fits it)."""
    fs, dt_out, P, B, n_ch, dur, off_ns, null, layout = cfg
    x = (np.random.default_rng(19).standard_normal((n_ch, int(dur * fs))) + 3.0).astype(np.float32)
    if null:
        x[3, int(dur * fs) // 3] = np.nan
    out = {}
    fold = layout == "fold"
    for mode in (2, 4):
        with kernel_options(scan_defer=mode, k1_recurrence=int(fold)):
            out[mode] = _run(x, fs, dt_out, P, B, "tc" if fold else layout, off_ns=off_ns)
        assert _run.last_kernel == {"tc": "mfma_runs", "cc": "mfma_runs_tm", "fold": "recurrence_fold"}[layout]
        assert _run.last_scan == ("deferred" if mode == 2 else "fused"), mode
    a, b = out[2][0], out[4][0]
    np.testing.assert_array_equal(np.isnan(a), np.isnan(b))
    f = np.isfinite(a)
    gates.check(f"fused_vs_deferred {cfg}", _relrms(b[f], a[f]), gates.PATHS)
    y, ref, sched = out[4]
    for (tt, r), (lo, hi, oa, ob) in zip(ref, sched):
        fr = np.isfinite(r)
        np.testing.assert_array_equal(np.isnan(y[:, oa:ob]), ~fr)
        gates.check(f"fused_oracle {cfg} {oa}", _relrms(y[:, oa:ob][fr], r[fr]), gates.REC if fold else gates.MFMA)


@pytest.mark.parametrize("which", ["lo", "head_first", "head_last", "fir_history"])
def test_offsample_head_skip_nulls(which):
    """Off-sample grids skip the chunk head with K1's one-block run kb-1
    (ChunkGeom::hskip).  A null at the sample before the chunk start (inside
    block kb-1 but outside the chunk) makes that (chunk, channel) walk its
    head instead; nulls in the head or the FIR history must poison exactly
    what SciPy's chunked sosfiltfilt poisons."""
    fs, dt_out, P, B, n_ch, dur, off = 500.0, 1.0, 120, 7, 6, 400.0, 1_900_000
    n = int(dur * fs)
    dt_ns = int(round(1e9 / fs))
    x = (np.random.default_rng(4).standard_normal((n_ch, n)) + 2.0).astype(np.float32)
    t0, t1 = T0 + off, T0 + 1_000_000_000
    tg = S.time_grid(t1, t0 + n * dt_ns, dt_out)
    sched = S.lfproc_chunks(len(tg), P, B)
    s0 = S.select_range(t0, dt_ns, n, tg[sched[1][0]], tg[sched[1][1]])[0]  # chunk 1's first sample
    L = int(round(fs * dt_out))
    pos = {"lo": s0 - 1, "head_first": s0, "head_last": s0 + L - 2, "fir_history": s0 - 3}[which]
    x[2, pos] = np.nan
    x[4, pos] = -np.inf
    y, ref, sched2 = _run(x, fs, dt_out, P, B, "tc", off_ns=off)
    assert _run.last_kernel == "mfma_runs"
    for (tt, r), (a, b, oa, ob) in zip(ref, sched2):
        yy = y[:, oa:ob]
        assert np.array_equal(np.isnan(yy), np.isnan(r)), (which, a, b)
        m = ~np.isnan(r)
        gates.check(f"head_skip {which} {oa}", _relrms(yy[m], r[m]), gates.MFMA)


@pytest.mark.parametrize("cfg", [
    (500.0, 1.0, 600, 7, 40, 1500.0, "tc"),   # cfg3 parameters, narrow: the fused scan
    (250.0, 0.2, 40, 6, 37, 24.0, "cc"),      # cfg1 geometry, (time, channel) rows
    (3000.0, 1.0, 120, 7, 6, 300.0, "tc"),    # lattice grid (one-pass K1 + scan + blend)
])
def test_pipeline_matches_execute(cfg):
    """lfdas.plan.LowpassPipeline (lfd_lowpass_execute_split: each batch's
    scan on a scan stream beside the next batch's block pass, two
    workspaces) gives every batch exactly plan.execute's outputs, for
    batches submitted back to back without host synchronisation."""
    import torch
    from lfdas.plan import LowpassPipeline, LowpassPlan
    fs, dt_out, P, B, n_ch, dur, layout = cfg
    n = int(dur * fs)
    dt_ns = int(round(1e9 / fs))
    tg = S.time_grid(T0, T0 + n * dt_ns, dt_out)
    sched = S.lfproc_chunks(len(tg), P, B)
    lo, w = S.grid_positions(T0, dt_ns, tg)
    chunks = [(*S.select_range(T0, dt_ns, n, tg[a], tg[b]), oa, ob) for a, b, oa, ob in sched]
    sos = oracle.butter_sos(4, (1 / dt_out / 2 * 0.9) / (fs / 2))
    plan = LowpassPlan(sos, n_ch, n, lo, w, chunks)
    rng = np.random.default_rng(23)
    xs = []
    for i in range(5):
        x = (rng.standard_normal((n_ch, n)) + 10.0 * i).astype(np.float32)
        if i == 2:
            x[1, n // 3] = np.nan
        xd = torch.from_numpy(x).cuda() if layout == "tc" else torch.from_numpy(np.ascontiguousarray(x.T)).cuda().t()
        xs.append(xd)
    ws = plan.alloc_workspace()
    ref = []
    for xd in xs:
        y = torch.full((n_ch, len(tg)), float("nan"), dtype=torch.float64, device="cuda")
        plan.execute(xd, y, ws)
        ref.append(y)
    torch.cuda.synchronize()
    pipe = LowpassPipeline(plan)
    ys = [torch.full((n_ch, len(tg)), float("nan"), dtype=torch.float64, device="cuda") for _ in xs]
    for xd, y in zip(xs, ys):
        pipe.submit(xd, y)
    pipe.wait()
    torch.cuda.synchronize()
    for a, b in zip(ref, ys):
        assert torch.equal(torch.nan_to_num(a, 7.0), torch.nan_to_num(b, 7.0))
    assert np.isnan(ys[2].cpu().numpy()[1]).any() and not np.isnan(ys[1].cpu().numpy()[1, 50:-50]).any()
    plan.close()
