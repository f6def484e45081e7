"""Streaming low-pass (lfd_stream_*): the real-time edge loop of
low_pass_dascore_edge.ipynb cell 11 and out-of-core process_time_range, with
the overlap held in HBM.

CPU tests drive the native bookkeeping in dry-run mode (no device) and check
output times, chunk (file) boundaries and retention against the oracle's
restatement of the notebook loop; GPU tests check the values (relRMS <= 1e-4,
north_star) for both host layouts and for pinned / pageable pushes."""
import numpy as np
import pytest

import gates
import oracle
from lfdas import stream as ST

T0 = 1_505_692_800_000_000_000  # 2017-09-18T00:00:00


def _relrms(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(np.sum((a - b) ** 2) / np.sum(b ** 2)))


# ---------------------------------------------------------------- CPU ---
@pytest.mark.parametrize("L", [2, 3, 5, 14, 15, 16, 17, 40, 41, 100, 120, 601, 3600])
@pytest.mark.parametrize("P,B", [(40, 6), (600, 7), (100, 10), (15, 7), (30, 3)])
def test_native_schedule_matches_oracle(L, P, B):
    try:
        ref = oracle.lfproc_schedule(L, P, B)
    except ValueError:
        with pytest.raises(ValueError):
            ST.lfproc_schedule(L, P, B)
        return
    assert ST.lfproc_schedule(L, P, B) == [tuple(r) for r in ref]


def _edge_cfg_cases():
    # (fs, dt_out, P, B, push seconds, n pushes, t_start offset s)
    return [
        (250.0, 1.0, 125, 7, 30.0, 6, 0.0),    # cfg4 cadence at a small fs
        (250.0, 0.2, 40, 6, 8.0, 6, 0.0),      # cfg1 geometry, file = 8 s
        (200.0, 10.0, 30, 6, 125.0, 5, 0.0),   # d_t = 10 s (notebook default)
        (100.0, 1.0, 20, 3, 7.3, 9, 2.0),      # ragged files, late start
        (250.0, 1.0, 40, 6, 20.0, 5, 0.0005),  # grid between samples: blended output functional
        (3000.0, 1.0, 60, 6, 30.0, 5, 0.0),    # 333,333 ns samples: drifting fraction (lattice plans)
    ]


def _edge_ref(x, fs, dt_out, P, B, push_s, t_start):
    dt_ns = int(round(1e9 / fs))
    push = int(round(push_s * fs))
    back = int((B - 1) * dt_out) * 1_000_000_000
    return oracle.edge_loop(x, T0, dt_ns, push, T0 + int(t_start * 1e9), dt_out, P, B, back), push, dt_ns


@pytest.mark.parametrize("case", _edge_cfg_cases())
def test_edge_dry_run_times_match_notebook_loop(case):
    fs, dt_out, P, B, push_s, n_push, t_start = case
    push = int(round(push_s * fs))
    x = np.random.default_rng(3).standard_normal((2, push * n_push)).astype(np.float32)
    ref, push, dt_ns = _edge_ref(x, fs, dt_out, P, B, push_s, t_start)
    s = ST.LowpassStream(2, dt_ns, dt_out, P, B, mode="edge", t_start=T0 + int(t_start * 1e9),
                         dry_run=True)
    all_t = []
    for k in range(n_push):
        o = s.push(x[:, k * push:(k + 1) * push], T0 + k * push * dt_ns)
        want = ref[k]
        assert o.chunk_counts == [len(t) for t, _ in want] or (not want and o.n_out == 0)
        exp_t = np.concatenate([t for t, _ in want]) if want else np.zeros(0, np.int64)
        np.testing.assert_array_equal(o.times_ns, exp_t)
        all_t.append(o.times_ns)
        # retention: only what the next run selects stays in the arena
        cap, held, t_held = s.info()
        assert held <= push + int((2 * B + 2) * dt_out * fs) + 4 or not np.concatenate(all_t).size
    t = np.concatenate(all_t)
    assert np.all(np.diff(t) == int(dt_out * 1000) * 1_000_000)  # contiguous, no duplicates
    s.close()


@pytest.mark.parametrize("push_s", [7.0, 30.0, 61.3])
def test_continuous_dry_run_matches_process_time_range(push_s):
    fs, dt_out, P, B = 100.0, 1.0, 40, 5
    n = int(600 * fs)
    dt_ns = int(1e9 / fs)
    t2 = T0 + (n - 1) * dt_ns
    tg = oracle.lfproc_time_grid(T0, t2, dt_out)
    sched = oracle.lfproc_schedule(len(tg), P, B)
    s = ST.LowpassStream(3, dt_ns, dt_out, P, B, mode="continuous", t_start=T0, t_end=t2, dry_run=True)
    push = int(push_s * fs)
    got, counts = [], []
    for k0 in range(0, n, push):
        k1 = min(n, k0 + push)
        o = s.push(np.zeros((3, k1 - k0), np.float32), T0 + k0 * dt_ns)
        got.append(o.times_ns)
        counts += o.chunk_counts
        _, held, _ = s.info()
        assert held <= (P + 1) * dt_out * fs + push + 4
    o = s.flush()
    got.append(o.times_ns)
    counts += o.chunk_counts
    assert counts == [ob - oa for _, _, oa, ob in sched]
    np.testing.assert_array_equal(np.concatenate(got), tg[sched[0][2]:sched[-1][3]])


def test_stream_gap_and_config_errors():
    s = ST.LowpassStream(2, 4_000_000, 1.0, 40, 6, dry_run=True, t_start=T0)
    s.reserve(100)
    assert s.info()[0] >= 400
    s.push(np.zeros((2, 100), np.float32), T0)
    with pytest.raises(ValueError, match="patch merge failed! Gap in data exists"):
        s.push(np.zeros((2, 100), np.float32), T0 + 101 * 4_000_000)
    with pytest.raises(ValueError, match="channels"):
        s.push(np.zeros((3, 100), np.float32), T0 + 100 * 4_000_000)
    with pytest.raises(ValueError, match="2\\*edge_buff_size"):
        ST.LowpassStream(2, 4_000_000, 1.0, 12, 6, dry_run=True)
    with pytest.raises(ValueError, match="t_start and t_end"):
        ST.LowpassStream(2, 4_000_000, 1.0, 40, 6, mode="continuous", dry_run=True)


def test_stream_merge_rule_matches_chunk_merge():
    """Pushes follow Spool.chunk(time=None)'s merge rule (tolerance 1.5
    samples): a duplicated boundary sample is dropped, a first sample up to
    1.5 intervals after the last one continues the sample grid, more is a gap."""
    dt = 4_000_000
    s = ST.LowpassStream(2, dt, 1.0, 40, 6, dry_run=True, t_start=T0)
    s.push(np.zeros((2, 100), np.float32), T0)
    assert s.info()[1] == 100
    s.push(np.zeros((2, 100), np.float32), T0 + 99 * dt)  # first sample duplicates the last
    assert s.info()[1] == 199
    s.push(np.zeros((2, 100), np.float32), T0 + 199 * dt + dt // 5)  # 1.2-sample gap: merged
    assert s.info()[1] == 299
    s.push(np.zeros((2, 10), np.float32), T0 + 298 * dt + 3 * dt // 2)  # exactly 1.5: merged
    assert s.info()[1] == 309
    with pytest.raises(ValueError, match="patch merge failed! Gap in data exists"):
        s.push(np.zeros((2, 10), np.float32), T0 + 308 * dt + 3 * dt // 2 + 1)
    with pytest.raises(ValueError, match="patch merge failed! Gap in data exists"):
        s.push(np.zeros((2, 10), np.float32), T0 + 300 * dt)  # overlap
    s.close()


# ---------------------------------------------------------------- GPU ---
def _edge_gpu(x, case, time_axis=1, pinned=False):
    import torch
    fs, dt_out, P, B, push_s, n_push, t_start = case
    ref, push, dt_ns = _edge_ref(x, fs, dt_out, P, B, push_s, t_start)
    s = ST.LowpassStream(x.shape[0], dt_ns, dt_out, P, B, mode="edge",
                         t_start=T0 + int(t_start * 1e9))
    worst = 0.0
    for k in range(n_push):
        blk = x[:, k * push:(k + 1) * push]
        if time_axis == 0:
            blk = np.ascontiguousarray(blk.T)
        if pinned:
            blk = torch.from_numpy(np.ascontiguousarray(blk)).pin_memory()
        o = s.push(blk, T0 + k * push * dt_ns, time_axis=time_axis)
        y = s.fetch()
        want = ref[k]
        assert o.chunk_counts == [len(t) for t, _ in want] or (not want and o.n_out == 0)
        if want:
            r = np.concatenate([d for _, d in want], axis=1)
            np.testing.assert_array_equal(o.times_ns, np.concatenate([t for t, _ in want]))
            assert y.shape == r.shape
            worst = max(worst, _relrms(y, r))
    s.close()
    return worst


@pytest.mark.gpu
@pytest.mark.parametrize("case", _edge_cfg_cases())
@pytest.mark.parametrize("time_axis,pinned", [(1, False), (0, False), (1, True), (0, True)])
def test_edge_stream_parity(case, time_axis, pinned):
    fs, dt_out, P, B, push_s, n_push, t_start = case
    push = int(round(push_s * fs))
    rng = np.random.default_rng(5)
    n_ch = 19
    t = np.arange(push * n_push) / fs
    x = (rng.standard_normal((n_ch, push * n_push)) + np.sin(2 * np.pi * 0.01 * t) + 3.0).astype(np.float32)
    worst = _edge_gpu(x, case, time_axis, pinned)
    gates.check(f"edge_stream {case} ax={time_axis} pinned={pinned}", worst, gates.STREAM)


@pytest.mark.gpu
def test_continuous_stream_parity_and_reuse():
    import torch
    fs, dt_out, P, B = 200.0, 1.0, 60, 7
    n_ch, n = 37, int(900 * fs)
    dt_ns = int(1e9 / fs)
    rng = np.random.default_rng(9)
    x = (rng.standard_normal((n_ch, n)) + 50.0).astype(np.float32)
    t2 = T0 + (n - 1) * dt_ns
    ref = oracle.lfproc_process(x, T0, dt_ns, T0, t2, dt_out, P, B)
    r = np.concatenate([d for _, d in ref], axis=1)
    rt = np.concatenate([t for t, _ in ref])
    s = ST.LowpassStream(n_ch, dt_ns, dt_out, P, B, mode="continuous", t_start=T0, t_end=t2,
                         capacity=int(150 * fs))
    push = int(40 * fs)
    ys, ts = [], []
    host = torch.empty((n_ch, push), dtype=torch.float32).pin_memory()
    for k0 in range(0, n, push):
        k1 = min(n, k0 + push)
        host[:, :k1 - k0] = torch.from_numpy(x[:, k0:k1])
        o = s.push(host[:, :k1 - k0], T0 + k0 * dt_ns)
        ys.append(s.fetch())  # waits for the push: the pinned buffer is free again
        ts.append(o.times_ns)
    o = s.flush()
    ys.append(s.fetch())
    ts.append(o.times_ns)
    y = np.concatenate(ys, axis=1)
    np.testing.assert_array_equal(np.concatenate(ts), rt)
    assert y.dtype == np.float64
    gates.check("continuous_stream", _relrms(y, r), gates.STREAM)
    cap, held, _ = s.info()
    assert cap <= 4 * push + 64  # the arena did not grow with the spool
    s.close()


@pytest.mark.gpu
def test_3khz_edge_stream_reuses_lattice_plans():
    """3 kHz on integer-ns times (333,333 ns): every run's grid drifts
    against the samples (lattice plans).  Plans are cached by the grid's
    structure and the blend fractions computed on device per run, so 36
    pushes of 30 s build only a few plans (not one per push) and
    the outputs still match the notebook loop (gates.STREAM)."""
    case = (3000.0, 1.0, 60, 6, 30.0, 36, 0.0)
    fs, dt_out, P, B, push_s, n_push, t_start = case
    push = int(round(push_s * fs))
    rng = np.random.default_rng(21)
    t = np.arange(push * n_push) / fs
    x = (rng.standard_normal((6, push * n_push)) + np.sin(2 * np.pi * 0.02 * t) + 7.0).astype(np.float32)
    ref, push, dt_ns = _edge_ref(x, fs, dt_out, P, B, push_s, t_start)
    s = ST.LowpassStream(x.shape[0], dt_ns, dt_out, P, B, mode="edge", t_start=T0)
    worst, runs = 0.0, 0
    for k in range(n_push):
        o = s.push(x[:, k * push:(k + 1) * push], T0 + k * push * dt_ns)
        y = s.fetch()
        want = ref[k]
        if want:
            runs += 1
            r = np.concatenate([d for _, d in want], axis=1)
            np.testing.assert_array_equal(o.times_ns, np.concatenate([t for t, _ in want]))
            worst = max(worst, _relrms(y, r))
    created, hits = s.plan_stats()
    s.close()
    gates.check("3khz_edge_stream", worst, gates.STREAM)
    assert runs >= n_push - 2
    assert created + hits >= runs
    assert created <= runs // 3, (created, hits, runs)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(8))
def test_continuous_stream_random_pushes(seed):
    """Eight seeded random out-of-core streams (rates 100 Hz - 1 kHz, output
    intervals 0.5 - 5 s, edge buffers 1 - 7, patch sizes 2B + 2 .. 2B + 40,
    pushes of random lengths, an arena a few pushes deep so it compacts)
    against the oracle's process_time_range over the whole range: identical
    output times, relRMS gated per stream at 10x its measured value."""
    rng = np.random.default_rng(5000 + seed)
    while True:
        fs = float(rng.choice([100.0, 200.0, 250.0, 500.0, 1000.0]))
        dt_out = float(rng.choice([0.5, 1.0, 2.0, 5.0]))
        if fs * dt_out >= 20:
            break
    B = int(rng.integers(1, 8))
    P = int(rng.integers(2 * B + 2, 2 * B + 41))
    n_ch = int(rng.integers(1, 40))
    n_grid = int(rng.integers(2 * P, 6 * P + 1))
    n = int(n_grid * dt_out * fs)
    dt_ns = int(round(1e9 / fs))
    x = (rng.standard_normal((n_ch, n)) + 10.0).astype(np.float32)
    t2 = T0 + (n - 1) * dt_ns
    ref = oracle.lfproc_process(x, T0, dt_ns, T0, t2, dt_out, P, B)
    r = np.concatenate([d for _, d in ref], axis=1)
    rt = np.concatenate([t for t, _ in ref])
    mean_push = max(8, int(n / rng.integers(4, 30)))
    s = ST.LowpassStream(n_ch, dt_ns, dt_out, P, B, mode="continuous", t_start=T0, t_end=t2,
                         capacity=int(3 * mean_push + (2 * B + P + 2) * dt_out * fs))
    ys, ts = [], []
    k0 = 0
    while k0 < n:
        k1 = min(n, k0 + int(rng.integers(max(1, mean_push // 3), 2 * mean_push)))
        o = s.push(np.ascontiguousarray(x[:, k0:k1]), T0 + k0 * dt_ns)
        ys.append(s.fetch())
        ts.append(o.times_ns)
        k0 = k1
    o = s.flush()
    ys.append(s.fetch())
    ts.append(o.times_ns)
    s.close()
    y = np.concatenate(ys, axis=1)
    np.testing.assert_array_equal(np.concatenate(ts), rt)
    gates.check(f"continuous_random seed={seed} {(fs, dt_out, P, B, n_ch, n, mean_push)}", _relrms(y, r),
                gates.STREAM)
