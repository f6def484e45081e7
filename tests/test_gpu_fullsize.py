"""Parity at BASELINE.json's full sizes.  The oracle cannot process 72 GB in
seconds, so every check here is size-independent: a sample of channels of the
full-size device result against the oracle (tests/gates.py, identical output
times), and closed-form properties over every channel (a constant input comes
back exactly; linearity of the filter across two inputs)."""
import numpy as np
import pytest

import gates
import oracle

pytestmark = pytest.mark.gpu

T0 = 1_505_692_800_000_000_000


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(np.sum((a - b) ** 2) / np.sum(b ** 2)))


def _cfg3_plan(n_ch=10_000, n=1_800_000, fs=500.0, dt_out=1.0, P=600, B=7):
    import bench
    plan, sched, sos, t0, dt_ns, tg = bench.build_plan(n_ch, n, fs, dt_out, P, B)
    return plan, sched, dt_ns, tg


def test_cfg3_full_size_sampled_channels_and_dc():
    import torch

    import bench
    n_ch, n = 10_000, 1_800_000
    plan, sched, dt_ns, tg = _cfg3_plan(n_ch, n)
    x = torch.empty((n_ch, n), dtype=torch.float32, device="cuda")
    bench.synth_fill(x, 500.0, 2024)
    y = torch.full((n_ch, plan.n_grid), float("nan"), dtype=torch.float64, device="cuda")
    ws = plan.alloc_workspace()
    plan.execute(x, y, ws)
    torch.cuda.synchronize()
    assert plan.last_kernel() == "mfma_runs"
    rows = [0, 1, 15, 16, 4999, 9983, 9998, 9999]
    xs = x[rows].cpu().numpy()
    ys = y[rows].cpu().numpy()
    ref = oracle.lfproc_process(xs, T0, dt_ns, tg[0], tg[-1] + 1, 1.0, 600, 7)
    got = np.concatenate([ys[:, oa:ob] for _, _, oa, ob in sched], axis=1)
    want = np.concatenate([r for _, r in ref], axis=1)
    assert got.shape == want.shape == (len(rows), 3585)
    gates.check("cfg3_full", _rel(got, want), gates.MFMA)
    produced = np.zeros(plan.n_grid, bool)
    for _, _, oa, ob in sched:
        produced[oa:ob] = True
    assert not torch.isnan(y[:, torch.as_tensor(produced, device="cuda")]).any()
    # every channel: a constant comes back as itself (DC gain 1, odd padding
    # of a constant is the constant, zi starts it steady)
    x.fill_(0.0)
    x += torch.arange(n_ch, device="cuda", dtype=torch.float32)[:, None] * 0.5 + 100.0
    plan.execute(x, y, ws)
    torch.cuda.synchronize()
    yc = y[:, torch.as_tensor(produced, device="cuda")]
    expect = (torch.arange(n_ch, device="cuda", dtype=torch.float32) * 0.5 + 100.0)[:, None].double()
    gates.check("cfg3_full_dc (max rel)", float(((yc - expect).abs() / expect).max()), gates.DC)
    del x, y, ws
    torch.cuda.empty_cache()


def test_cfg3_full_size_linearity():
    """f(x1 + 3 x2) == f(x1) + 3 f(x2) over all 10,000 channels."""
    import torch

    import bench
    n_ch, n = 10_000, 1_800_000
    plan, sched, dt_ns, tg = _cfg3_plan(n_ch, n)
    ws = plan.alloc_workspace()
    x = torch.empty((n_ch, n), dtype=torch.float32, device="cuda")
    outs = []
    for seed in (1, 2):
        bench.synth_fill(x, 500.0, seed)
        y = torch.empty((n_ch, plan.n_grid), dtype=torch.float64, device="cuda")
        plan.execute(x, y, ws)
        outs.append(y)
    # x1 + 3 x2 regenerated in place (the generator is seeded)
    bench.synth_fill(x, 500.0, 2)
    x *= 3.0
    g = torch.empty((n_ch, plan.n_grid), dtype=torch.float64, device="cuda")
    # add x1 slice by slice to keep memory at 2 x 72 GB
    x_full1 = torch.empty((n_ch, n), dtype=torch.float32, device="cuda")
    bench.synth_fill(x_full1, 500.0, 1)
    x += x_full1
    del x_full1
    plan.execute(x, g, ws)
    torch.cuda.synchronize()
    lhs = g[:, sched[0][2]:sched[-1][3]].double()
    rhs = (outs[0] + 3.0 * outs[1])[:, sched[0][2]:sched[-1][3]].double()
    rel = float(torch.sqrt(((lhs - rhs) ** 2).sum() / (rhs ** 2).sum()))
    gates.check("cfg3_full_linearity", rel, gates.PATHS)
    del x, g, outs, ws
    torch.cuda.empty_cache()


def test_cfg2_rolling_full_size_sampled_channels():
    import torch

    import bench
    from lfdas.plan import rolling_mean_device
    x = torch.empty((5000, 600_000), dtype=torch.float32, device="cuda")
    bench.synth_fill(x, 1000.0, 99)
    y = rolling_mean_device(x, 1000, 1000)
    torch.cuda.synchronize()
    assert tuple(y.shape) == (5000, 600)
    rows = [0, 17, 2500, 4999]
    ref = oracle.rolling_mean(x[rows].cpu().numpy(), 1000, 1000)
    got = y[rows].cpu().numpy()
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    m = ~np.isnan(ref)
    gates.check("cfg2_rolling_full_size", _rel(got[m], ref[m]), gates.ROLL)
    assert bool(torch.isnan(y[:, 0]).all()) and not bool(torch.isnan(y[:, 1:]).any())
    del x, y
    torch.cuda.empty_cache()


CFG5_ROWS = [0, 15, 16, 24_999, 49_999]


def cfg5_push_block(k, n_ch, push, fs, rows, dev):
    """Push k of the cfg5 check spool, generated on the device: every channel
    holds its own constant 100 + ch/1000, the sampled rows carry noise + a
    slow sine on top (seeded per push)."""
    import torch
    x = (torch.arange(n_ch, device=dev, dtype=torch.float32) * 1e-3 + 100.0)[:, None].repeat(1, push)
    g = torch.Generator(device=dev)
    g.manual_seed(5000 + k)
    t = (torch.arange(push, device=dev, dtype=torch.float64) + k * push) / fs
    sig = torch.sin(2 * np.pi * 0.002 * t).float()
    idx = torch.as_tensor(rows, device=dev)
    x[idx] += torch.randn((len(rows), push), device=dev, generator=g) + sig[None, :]
    return x


def test_cfg5_out_of_core_stream_full_width():
    """cfg5 geometry through the continuous (out-of-core) stream: 50,000 ch @
    200 Hz in 60 s pinned pushes, dt = 10 s, P = 120, B = 6, 45 min (3 LFProc
    chunks).  Sampled channels against the oracle's process_time_range, every
    other channel's constant back as itself, identical output times."""
    import torch

    from lfdas.stream import LowpassStream
    n_ch, fs, push_s, dur = 50_000, 200.0, 60.0, 2700.0
    push, n = int(push_s * fs), int(dur * fs)
    dt_ns = int(1e9 / fs)
    t_end = T0 + (n - 1) * dt_ns
    dev = torch.device("cuda")
    rows = CFG5_ROWS
    st = LowpassStream(n_ch, dt_ns, 10.0, 120, 6, mode="continuous", t_start=T0, t_end=t_end,
                       capacity=int(1300 * fs) + 2 * push)
    st.reserve(push)
    host = [torch.empty((n_ch, push), dtype=torch.float32).pin_memory() for _ in range(2)]
    xs = np.empty((len(rows), n), np.float32)
    ys, ts = [], []
    for k in range(n // push):
        h = host[k % 2]
        h.copy_(cfg5_push_block(k, n_ch, push, fs, rows, dev))
        xs[:, k * push:(k + 1) * push] = h[rows].numpy()
        o = st.push(h, T0 + k * push * dt_ns)
        if o.n_out:
            ys.append(st.fetch())  # also frees the pinned buffer
            ts.append(o.times_ns)
        else:
            st.wait_copy()
    o = st.flush()
    if o.n_out:
        ys.append(st.fetch())
        ts.append(o.times_ns)
    st.close()
    y = np.concatenate(ys, axis=1)
    ref = oracle.lfproc_process(xs, T0, dt_ns, T0, t_end, 10.0, 120, 6)
    np.testing.assert_array_equal(np.concatenate(ts), np.concatenate([t for t, _ in ref]))
    want = np.concatenate([r for _, r in ref], axis=1)
    assert y.shape == (n_ch, want.shape[1]) and want.shape[1] == 257
    gates.check("cfg5_stream_full", _rel(y[rows], want), gates.STREAM)
    mask = np.ones(n_ch, bool)
    mask[rows] = False
    expect = (np.arange(n_ch, dtype=np.float32) * np.float32(1e-3) + np.float32(100.0)).astype(np.float64)
    dc = y[mask]
    gates.check("cfg5_stream_dc (max rel)", float(np.max(np.abs(dc - expect[mask, None]) / expect[mask, None])), gates.DC)
    torch.cuda.empty_cache()


def test_cfg4_edge_full_width_sampled_channels():
    """cfg4 (2,000 ch @ 2 kHz, 30 s pushes) through the edge stream, a sample
    of channels against the oracle's notebook loop."""
    import torch

    from lfdas.stream import LowpassStream
    n_ch, fs, push = 2000, 2000.0, 60_000
    dt_ns = 500_000
    n_push = 4
    rng = np.random.default_rng(4)
    rows = [0, 777, 1999]
    st = LowpassStream(n_ch, dt_ns, 1.0, 125, 7, mode="edge", t_start=T0)
    st.reserve(push)
    xs = np.empty((len(rows), push * n_push), np.float32)
    got = []
    for k in range(n_push):
        blk = torch.empty((n_ch, push), dtype=torch.float32).pin_memory()
        blk.copy_(torch.from_numpy((rng.standard_normal((n_ch, push)) + 2.0).astype(np.float32)))
        xs[:, k * push:(k + 1) * push] = blk[rows].numpy()
        st.push(blk, T0 + k * push * dt_ns)
        got.append(st.fetch()[rows])
    st.close()
    ref = oracle.edge_loop(xs, T0, dt_ns, push, T0, 1.0, 125, 7, 6_000_000_000)
    for g, r in zip(got, ref):
        want = np.concatenate([d for _, d in r], axis=1) if r else np.zeros((len(rows), 0))
        assert g.shape == want.shape
        if want.size:
            gates.check("cfg4_edge_full", _rel(g, want), gates.STREAM)


@pytest.mark.parametrize("variant", ["time_major", "off_sample"])
def test_cfg3_full_size_layouts_sampled_channels(variant):
    """cfg3 at full size through the other two production K1 paths: stored
    (time, channel) like the real files (k_block_runs_mfma_tm, channel-pair
    buffer loads) and an archive whose samples start 1.9 ms after the output
    grid's second (blended output functional + scan head skip).  Sampled
    channels against the oracle (gates.MFMA, identical output times), no
    NaN in any produced output."""
    import torch

    import bench
    n_ch, n, fs = 10_000, 1_800_000, 500.0
    off = 1_900_000 if variant == "off_sample" else 0
    plan, sched, sos, t0, dt_ns, tg = bench.build_plan(n_ch, n, fs, 1.0, 600, 7, off)
    if variant == "time_major":
        xs_t = torch.empty((n, n_ch), dtype=torch.float32, device="cuda")
        bench.synth_fill_time_major(xs_t, fs, 11)
        x = xs_t.t()
    else:
        x = torch.empty((n_ch, n), dtype=torch.float32, device="cuda")
        bench.synth_fill(x, fs, 11)
    y = torch.full((n_ch, plan.n_grid), float("nan"), dtype=torch.float64, device="cuda")
    ws = plan.alloc_workspace()
    plan.execute(x, y, ws)
    torch.cuda.synchronize()
    assert plan.last_kernel() == ("mfma_runs_tm" if variant == "time_major" else "mfma_runs")
    rows = [0, 1, 31, 32, 5001, 9998, 9999]
    xs = x[rows].cpu().numpy()
    ys = y[rows].cpu().numpy()
    ref = oracle.lfproc_process(xs, t0, dt_ns, tg[0], tg[-1] + 1, 1.0, 600, 7)
    assert len(ref) == len(sched)
    for (tt, r), (_, _, oa, ob) in zip(ref, sched):
        np.testing.assert_array_equal(tt, tg[oa:ob])
    got = np.concatenate([ys[:, oa:ob] for _, _, oa, ob in sched], axis=1)
    want = np.concatenate([r for _, r in ref], axis=1)
    assert got.shape == want.shape
    gates.check(f"cfg3_full_{variant}", _rel(got, want), gates.MFMA)
    produced = np.zeros(plan.n_grid, bool)
    for _, _, oa, ob in sched:
        produced[oa:ob] = True
    assert not torch.isnan(y[:, torch.as_tensor(produced, device="cuda")]).any()
    del x, y, ws
    torch.cuda.empty_cache()
