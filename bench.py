"""Benchmark of the north-star path: chunked zero-phase low-pass + decimate
(LFProc.process_time_range, lf_das.py:219-290) on MI355X.

Workload (BASELINE.json configs[2], "cfg3"): 10,000 channels x 1 h @ 500 Hz
float32 (72 GB, channel-major, DASCore dims ("distance","time")), 4th-order
Butterworth at 0.45 Hz, decimate to 1 Hz, LFProc chunking P = 600, B = 7.
One step = one pass of the hot path over the whole hour (7 overlapping chunks,
3,585 outputs per channel), inputs resident in HBM.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--channels C] [--weak]

N > 1 runs one rank per GPU: under torch.distributed.run (the driver's
form; WORLD_SIZE must equal --gpus), or ``python bench.py --gpus N`` starts
that launcher itself as a child process (and fails, printing no line, when
the node has fewer than N GPUs).  The headline is BASELINE configs[2] as
quoted, "10,000 ch x 1 h @ 500 Hz, channel-sharded at 1/2/4/8 GPUs": strong
scaling, cfg3's 10,000 channels split into contiguous blocks
(lfdas.shard.channel_range, 1,250 per GPU at N = 8), no data-path
collective, ``value`` = 10,000 x 1.8 M channel-samples per step /
max-over-ranks time.  With N > 1 the weak-scaling figure (every rank its own
10,000-channel spool) is reported beside it as
``secondary.weak_scaling_cfg3``; ``--weak`` makes it the headline.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "low-freq-real-time_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)
# --pipelined: steps through lfdas.plan.LowpassPipeline (each step's scan
# beside the next step's block pass).  Measured r05t: no gain (cfg3 12.996
# vs 12.986 ms serial; 1,250 ch 1.723 vs 1.745, 2,500 ch 3.366 vs 3.307), so
# the default is serial: one execute after the other on one stream
PIPELINED = False


def _args():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--channels", type=int, default=10_000)
    p.add_argument("--seconds", type=float, default=3600.0)
    p.add_argument("--fs", type=float, default=500.0)
    p.add_argument("--dt-out", type=float, default=1.0)
    p.add_argument("--patch-size", type=int, default=600)
    p.add_argument("--edge-buff", type=int, default=7)
    p.add_argument("--cpu-channels", type=int, default=768,
                   help="channels of the bounded CPU-baseline sample (full hour each)")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-rolling", action="store_true")
    p.add_argument("--no-stream", action="store_true", help="skip the cfg4 / cfg5 streaming lines")
    p.add_argument("--cfg5-hours", type=float, default=24.0,
                   help="hours of the cfg5 spool streamed by the 1-GPU out-of-core line (BASELINE configs[4]: 24)")
    p.add_argument("--no-extra", action="store_true",
                   help="skip the extra low-pass lines (off-sample grid, 1 kHz dt = 10 s, time-major)")
    p.add_argument("--weak", action="store_true",
                   help="headline = every rank owns --channels channels (weak scaling); default: --channels "
                        "split over the ranks (strong scaling, BASELINE configs[2])")
    p.add_argument("--strong", action="store_true", help="the default (kept for old command lines)")
    p.add_argument("--one-device", action="store_true",
                   help="rehearsal of the N > 1 path on a 1-GPU box: every rank on cuda:0, gloo collectives "
                        "(the line is marked rehearsal; not a scaling measurement)")
    p.add_argument("--pipelined", action="store_true",
                   help="also time the steps through lfdas.plan.LowpassPipeline (each step's scan beside the "
                        "next step's block pass) and report that as the value; the serial time is reported "
                        "beside it")
    p.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                   help="rocprofv3 PMC traffic summary (tools/pmc_summary.py) for roofline.traffic")
    return p.parse_args()


def _dist():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_or_check(args) -> int | None:
    """``--gpus N`` without a launcher: start N rank processes with
    torch.distributed.run as a CHILD process (before this process touches
    the GPU: device_count() does not initialise HIP on this image) and return
    its exit code.  Under a launcher (WORLD_SIZE set), refuse a world size
    that differs from ``--gpus``.  None = this process is a rank: run."""
    ws_env = os.environ.get("WORLD_SIZE")
    if ws_env is not None:
        if int(ws_env) != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws_env} (launcher and flag disagree)",
                  file=sys.stderr)
            return 2
        return None
    if args.gpus <= 1:
        return None
    import torch
    n_dev = torch.cuda.device_count()
    if n_dev < args.gpus and not args.one_device:
        print(f"bench.py: --gpus {args.gpus} needs {args.gpus} GPUs, this node has {n_dev}; "
              "not printing an N=1 line for an N>1 request", file=sys.stderr)
        return 2
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def device_samples(shape, device):
    from lfdas.arena import device_samples as ds
    return ds(shape, device=device)


def synth_fill(x, fs, seed):
    """x[c, t] = 0.5 + sin(2*pi*0.05*t/fs + phi_c) + N(0,1), generated on the
    device in channel slices (synthetic; there is no dataset)."""
    import torch
    g = torch.Generator(device=x.device)
    g.manual_seed(seed)
    n_ch, n = x.shape
    t = torch.arange(n, device=x.device, dtype=torch.float32) * (2 * np.pi * 0.05 / fs)
    step = max(1, int(2e9 // (n * 4)))
    for c0 in range(0, n_ch, step):
        c1 = min(n_ch, c0 + step)
        phi = torch.rand((c1 - c0, 1), device=x.device, generator=g) * (2 * np.pi)
        blk = x[c0:c1]
        torch.randn(blk.shape, device=x.device, generator=g, out=blk)
        blk += torch.sin(t[None, :] + phi) + 0.5


def synth_fill_time_major(x, fs, seed):
    """The same kind of synthetic samples in (time, channel) storage."""
    import torch
    g = torch.Generator(device=x.device)
    g.manual_seed(seed)
    n, n_ch = x.shape
    phi = torch.rand((1, n_ch), device=x.device, generator=g) * (2 * np.pi)
    step = max(1, int(2e9 // (n_ch * 4)))
    for t0 in range(0, n, step):
        t1 = min(n, t0 + step)
        blk = x[t0:t1]
        torch.randn(blk.shape, device=x.device, generator=g, out=blk)
        t = torch.arange(t0, t1, device=x.device, dtype=torch.float32)[:, None] * (2 * np.pi * 0.05 / fs)
        blk += torch.sin(t + phi) + 0.5


def build_plan(n_ch, n, fs, dt_out, P, B, off_ns=0):
    """The LFProc plan of ``n`` samples per channel.  ``off_ns`` > 0: the
    samples start that long after the whole second on which the output grid
    starts (a real archive: every grid point lies a fraction of a sample past
    a sample)."""
    from lfdas import schedule as S
    from lfdas.design import lowpass_sos
    from lfdas.plan import LowpassPlan
    dt_ns = int(round(1e9 / fs))
    t_grid = 1_505_692_800_000_000_000
    t0 = t_grid + off_ns
    tg = S.time_grid(t_grid if off_ns == 0 else t_grid + 1_000_000_000, t0 + n * dt_ns, dt_out)
    sched = S.lfproc_chunks(len(tg), P, B)
    lo, w = S.grid_positions(t0, dt_ns, tg)
    chunks = [(*S.select_range(t0, dt_ns, n, tg[a], tg[b]), oa, ob) for a, b, oa, ob in sched]
    sos = lowpass_sos(fs, 1 / dt_out / 2 * 0.9, 4)
    return LowpassPlan(sos, n_ch, n, lo, w, chunks), sched, sos, t0, dt_ns, tg


K1_KERNELS = {"mfma_runs": "k_block_runs_mfma", "mfma_runs_tm": "k_block_runs_mfma_tm",
              "mfma": "k_block_functionals_mfma",
              "mfma_fold": "k_block_functionals_mfma + k_fold_runs",
              "recurrence": "k_block_functionals_lds|gen",
              "recurrence_fold": "k_block_functionals_lds|gen + k_fold_runs"}


def time_plan(plan, x, y, wsb, stream, steps, warmup, barrier=None):
    """Warm up, then time ``steps`` executes between two barriers; returns
    (wall seconds, per-step K1 ms, per-step scan ms) from HIP events on the
    execution stream (lfd_lowpass_last_timing)."""
    import torch
    from lfdas.plan import set_timing
    barrier = barrier or (lambda: torch.cuda.synchronize(x.device))
    # a ring of `steps` event triples: the timed steps are queued back to
    # back with no host synchronisation between them (a per-step event sync
    # left the GPU idle while the host launched the next step: 0.16 ms of a
    # 2 ms step on a 1,250-channel shard)
    set_timing(True, ring=max(2, steps))
    for _ in range(warmup):
        plan.execute(x, y, wsb, stream)
    barrier()
    t_a = time.perf_counter()
    for _ in range(steps):
        plan.execute(x, y, wsb, stream)
    barrier()
    el = time.perf_counter() - t_a
    k1, sc = plan.timings_ms(steps)
    set_timing(False)
    return el, k1, sc


def time_plan_pipelined(plan, x, y, steps, warmup, barrier=None):
    """Wall seconds of ``steps`` batches through ``lfdas.plan.LowpassPipeline``
    (each batch's scan beside the next batch's block pass, two workspaces),
    between two barriers; every batch is the full computation of
    ``plan.execute`` (bit-identical outputs, tests/test_gpu_lowpass.py)."""
    import torch
    from lfdas.plan import LowpassPipeline
    barrier = barrier or (lambda: torch.cuda.synchronize(x.device))
    pipe = LowpassPipeline(plan, x.device)
    for _ in range(warmup):
        pipe.submit(x, y)
    pipe.wait()
    barrier()
    t_a = time.perf_counter()
    for _ in range(steps):
        pipe.submit(x, y)
    pipe.wait()
    barrier()
    el = time.perf_counter() - t_a
    del pipe
    return el


def shard_line_fresh(args, c):
    """cfg3's c-channel shard timed by a child run of this script (a fresh
    process, like one rank of an N-GPU run: its samples in its own
    lfdas.arena placement); 20 timed steps after 3 warmups.  None if the
    child fails.  The parent holds no device buffers meanwhile."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--channels", str(c), "--steps", "20", "--warmup", "3",
           "--seconds", str(args.seconds), "--fs", str(args.fs), "--dt-out", str(args.dt_out),
           "--patch-size", str(args.patch_size), "--edge-buff", str(args.edge_buff),
           "--no-cpu", "--no-extra", "--no-rolling", "--no-stream"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
        if p.returncode != 0:
            return None
        return json.loads(p.stdout.strip().splitlines()[-1])
    except Exception:  # pragma: no cover - reported as the in-process fallback
        return None


def bench_lowpass_line(dev, n_ch, fs, seconds, dt_out, P, B, off_ns=0, time_major=False, steps=5,
                       label="", warmup=1):
    """One extra low-pass workload, timed like the headline (inputs in HBM,
    K1 roofline from its HIP-event time)."""
    import torch
    n = int(seconds * fs)
    plan, sched, sos, t0, dt_ns, tg = build_plan(n_ch, n, fs, dt_out, P, B, off_ns)
    if time_major:  # (time, distance) storage, viewed as (channel, time)
        xs = torch.empty((n, n_ch), dtype=torch.float32, device=dev)
        synth_fill_time_major(xs, fs, 77)
        x = xs.t()
    else:
        x = device_samples((n_ch, n), device=dev)
        synth_fill(x, fs, 77)
    y = torch.empty((n_ch, plan.n_grid), dtype=torch.float64, device=dev)
    wsb = plan.alloc_workspace(dev)
    stream = torch.cuda.current_stream(dev)
    el, k1_ms, scan_ms = time_plan(plan, x, y, wsb, stream, steps, warmup)
    el_s = el
    if PIPELINED:
        el = time_plan_pipelined(plan, x, y, steps, warmup)
    R = int(round(fs * dt_out))
    k1 = float(np.mean(k1_ms))
    gbs = n_ch * n * (4.0 + 8.0 / R) / (k1 * 1e-3) / 1e9
    out = {"value": n_ch * n * steps / el, "unit": "channel-samples/s", "ms_per_step": el / steps * 1e3,
           "ms_per_step_serial": el_s / steps * 1e3, "pipelined": PIPELINED,
           "config": label, "k1": plan.last_kernel(), "block_len": plan.block_len,
           "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": gbs / HBM_PEAK_GBS, "kernel": K1_KERNELS.get(plan.last_kernel()),
                        "kernel_ms": k1, "scan_kernel_ms": float(np.mean(scan_ms)),
                        "alg_bytes_per_sample": 4.0 + 8.0 / R}}
    n_off, onepass, _ = plan.lattice()
    if n_off or "lattice" in label:
        out["lattice"] = {"offsets": n_off, "onepass": onepass}
    plan.close()
    del x, y, wsb
    torch.cuda.empty_cache()
    return out


def _cpu_chunks(backend, x, sos, sched, t0, dt_ns, tg):
    """The LFProc chunks of the channel rows ``x`` on the CPU: ``"port"`` =
    the oracle's C restatement of scipy's _sosfilt (+ its interp1d);
    ``"scipy"`` = scipy.signal.sosfiltfilt + scipy.interpolate.interp1d, the
    library DASCore's pass_filter / interpolate call (lf_das.py:223-225)."""
    from lfdas import schedule as S
    n = x.shape[1]
    if backend == "scipy":
        import scipy.interpolate as si
        import scipy.signal as ss
    else:
        sys.path.insert(0, ROOT)
        import oracle
    for a, b, oa, ob in sched:
        s0, s1 = S.select_range(t0, dt_ns, n, tg[a], tg[b])
        tt = (np.arange(s0, s1 + 1, dtype=np.int64) * dt_ns).astype(np.float64)
        tq = (tg[oa:ob] - t0).astype(np.float64)
        if backend == "scipy":
            y = ss.sosfiltfilt(sos, x[:, s0:s1 + 1], axis=-1)
            si.interp1d(tt, y, axis=-1, kind="linear")(tq)
        else:
            y = oracle.sosfiltfilt_rows_c(sos, x[:, s0:s1 + 1])
            oracle.interp1d_linear(tt, y, tq)


def _cpu_data(n_c, n, fs, seed):
    rng = np.random.default_rng(seed)
    t = np.arange(n, dtype=np.float64) * (2 * np.pi * 0.05 / fs)
    return (rng.standard_normal((n_c, n)) + 0.5 + np.sin(t)[None, :]).astype(np.float32)


def cpu_baseline(args, sos, sched, t0, dt_ns, tg, backend="port", n_c=None):
    """One process, one thread, over a bounded channel sample of the full hour."""
    n = int(args.seconds * args.fs)
    n_c = n_c or args.cpu_channels
    x = _cpu_data(n_c, n, args.fs, 0)
    t_start = time.perf_counter()
    _cpu_chunks(backend, x, sos, sched, t0, dt_ns, tg)
    el = time.perf_counter() - t_start
    what = ("oracle C sosfiltfilt + interp1d" if backend == "port"
            else "scipy.signal.sosfiltfilt + scipy.interpolate.interp1d")
    return {"value": n_c * n / el, "unit": "channel-samples/s", "cores": 1,
            "kind": "port" if backend == "port" else "reference-lib",
            "sample": f"{n_c} ch x {n} samples ({args.seconds:.0f} s @ {args.fs:.0f} Hz), same LFProc "
                      f"chunks, {what}, 1 thread, {el:.1f} s"}


def _pinned_blocks(dev, n_blocks, shape, fs, seed):
    """Pinned host blocks of synthetic samples (generated on the device, copied
    down once): the host side of a stream, outside the timed region."""
    import torch
    out = []
    for i in range(n_blocks):
        d = torch.empty(shape, dtype=torch.float32, device=dev)
        synth_fill(d, fs, seed + i)
        h = torch.empty(shape, dtype=torch.float32).pin_memory()
        h.copy_(d)
        out.append(h)
        del d
    torch.cuda.synchronize(dev)
    return out


def bench_edge_cfg4(dev, n_push=12, warm=2, time_major=False):
    """cfg4: real-time edge mode, 2,000 ch @ 2 kHz in 30 s files
    (low_pass_dascore_edge.ipynb cell 11 with one file per run), dt = 1 s,
    P = 125 (the notebook's 125 s cadence), B = 7 (planner edge ~6 s).
    Latency = push of a pinned 30 s file -> decimated outputs on the host."""
    import torch
    from lfdas.plan import set_timing
    from lfdas.stream import LowpassStream
    n_ch, fs, push_s = 2000, 2000.0, 30.0
    push = int(push_s * fs)
    dt_ns = int(1e9 / fs)
    t0 = 1_679_464_800_000_000_000  # 2023-03-22T06:00:00 (the notebook's start)
    shape = (push, n_ch) if time_major else (n_ch, push)
    blocks = _pinned_blocks(dev, 2, shape, fs, 4321)
    st = LowpassStream(n_ch, dt_ns, 1.0, 125, 7, mode="edge", t_start=t0)
    st.reserve(push)
    lat, cp, run, n_out = [], [], [], []
    set_timing(True)
    for k in range(n_push + warm):
        blk = blocks[k % 2]
        ta = time.perf_counter()
        o = st.push(blk, t0 + k * push * dt_ns, time_axis=0 if time_major else 1)
        st.fetch()
        tb = time.perf_counter()
        if k >= warm:
            lat.append((tb - ta) * 1e3)
            a, b = st.last_timing_ms()
            cp.append(a)
            run.append(b)
            n_out.append(o.n_out)
    set_timing(False)
    st.close()
    lat = np.array(lat)
    return {"p50_ms": float(np.percentile(lat, 50)), "p99_ms": float(np.percentile(lat, 99)),
            "max_ms": float(lat.max()), "chunk_ms": push_s * 1e3,
            "latency_frac_of_chunk": float(np.percentile(lat, 99) / (push_s * 1e3)),
            "h2d_ms": float(np.median(cp)), "run_ms": float(np.median(run)),
            "h2d_GBps": n_ch * push * 4 / (np.median(cp) * 1e-3) / 1e9,
            "outputs_per_push": int(np.median(n_out)), "pushes": n_push,
            "config": f"2,000 ch @ 2 kHz, 30 s pinned pushes ({'time, distance' if time_major else 'distance, time'} "
                      "layout), dt = 1 s, P = 125, B = 7, resume buffer (B-1) s; latency = push -> host outputs"}


CFG5_ROWS = [0, 15, 16, 24_999, 49_999]


def bench_ooc_cfg5(dev, n_ch=50_000, seconds=86400.0, push_s=60.0):
    """cfg5: out-of-core process_time_range over a 50,000-ch @ 200 Hz spool
    (BASELINE configs[4]: 24 h = 1,440 pushes of 60 s, 3.46 TB) streamed from
    a pinned host ring, dt = 10 s (fc = 0.045 Hz), P = 120 (1,200 s chunks),
    B = 6 (planner edge 60 s).  Bound: PCIe.  The timed loop includes
    downloading every output; afterwards (untimed) the sampled channels of
    every chunk are checked against the oracle's process_time_range.  Reports
    the copy time per push (p50 / p99 / max, and the first vs the last tenth
    of the pushes: the arena's compaction, the plan cache and the pinned ring
    must keep it flat) and the stream's plan-cache counts."""
    import torch
    from lfdas.plan import set_timing
    from lfdas.stream import LowpassStream
    fs = 200.0
    push = int(push_s * fs)
    n = int(seconds * fs)
    n_push = n // push
    dt_ns = int(1e9 / fs)
    t0 = 1_679_464_800_000_000_000
    t_end = t0 + (n - 1) * dt_ns
    blocks = _pinned_blocks(dev, 2, (n_ch, push), fs, 777)
    st = LowpassStream(n_ch, dt_ns, 10.0, 120, 6, mode="continuous", t_start=t0,
                       t_end=t_end, capacity=int(1300 * fs) + 2 * push)
    st.reserve(push)
    n_out = 0
    cp = []
    ys, ts = [], []
    torch.cuda.synchronize(dev)
    set_timing(True)
    ta = time.perf_counter()
    for k in range(n_push):
        if k and k % 240 == 0:  # (progress: a 24 h run streams for about a minute)
            print(f"cfg5: {k}/{n_push} pushes, {time.perf_counter() - ta:.1f} s", file=sys.stderr, flush=True)
        o = st.push(blocks[k % 2], t0 + k * push * dt_ns)
        n_out += o.n_out
        if o.n_out:
            y = st.fetch()  # outputs to the host (also frees the pinned block)
            ys.append(y[CFG5_ROWS].copy())
            ts.append(o.times_ns)
        else:
            st.wait_copy()  # ring buffer (k+1) % 2 is free again
        cp.append(st.last_timing_ms()[0])
    set_timing(False)
    o = st.flush()
    n_out += o.n_out
    if o.n_out:
        ys.append(st.fetch()[CFG5_ROWS].copy())
        ts.append(o.times_ns)
    st.synchronize()
    el = time.perf_counter() - ta
    created, hits = st.plan_stats()
    cap, held, _ = st.info()
    st.close()
    xs = np.concatenate([blocks[k % 2][CFG5_ROWS].numpy() for k in range(n_push)], axis=1)
    del blocks
    samples = n_ch * n_push * push
    cpa = np.asarray(cp)
    tenth = max(1, n_push // 10)
    out = {"value": samples / el, "unit": "channel-samples/s", "seconds_streamed": n_push * push_s,
           "pushes": n_push, "wall_s": el, "h2d_GBps": samples * 4 / el / 1e9, "pcie_peak_GBps": 63.0,
           "pcie_frac": samples * 4 / el / 1e9 / 63.0, "outputs_per_channel": n_out,
           "copy_ms_p50": float(np.median(cpa)), "copy_ms_p99": float(np.percentile(cpa, 99)),
           "copy_ms_max": float(np.max(cpa)), "copy_ms_p50_first_tenth": float(np.median(cpa[:tenth])),
           "copy_ms_p50_last_tenth": float(np.median(cpa[-tenth:])),
           "plans_created": created, "plan_cache_hits": hits, "arena_capacity_samples": cap,
           "config": f"{n_ch:,} ch @ 200 Hz, {n_push * push_s / 3600:.3g} h of the 24 h spool in {push_s:.0f} s "
                     "pinned pushes, dt = 10 s, P = 120, B = 6, 1 GPU; outputs downloaded inside the timed loop"}
    # parity of the sampled channels (the checker, outside the timed region)
    sys.path.insert(0, ROOT)
    import oracle
    ref = oracle.lfproc_process(xs, t0, dt_ns, t0, t_end, 10.0, 120, 6)
    want = np.concatenate([r for _, r in ref], axis=1)
    got = np.concatenate(ys, axis=1) if ys else np.zeros((len(CFG5_ROWS), 0))
    times_ok = bool(np.array_equal(np.concatenate(ts) if ts else np.zeros(0, np.int64),
                                   np.concatenate([t for t, _ in ref])))
    rel = (float(np.sqrt(np.sum((got.astype(np.float64) - want) ** 2) / np.sum(want ** 2)))
           if got.shape == want.shape else float("inf"))
    # per chunk too: the first, the middle and the last of the spool
    per_chunk = []
    j = 0
    for _, r in ref:
        c = r.shape[1]
        if got.shape == want.shape and c:
            per_chunk.append(float(np.sqrt(np.sum((got[:, j:j + c] - r) ** 2) / np.sum(r ** 2))))
        j += c
    out["check"] = {"rows": CFG5_ROWS, "relrms_vs_oracle": rel, "times_identical": times_ok,
                    "chunks": len(ref), "relrms_first_middle_last_chunk":
                        [per_chunk[0], per_chunk[len(per_chunk) // 2], per_chunk[-1]] if per_chunk else None,
                    "pass": bool(times_ok and rel < 1e-9),
                    "checker": "oracle.lfproc_process on the sampled rows over the whole spool (untimed)"}
    if not out["check"]["pass"]:
        print(f"WARNING: cfg5 sampled-channel check failed: {out['check']}", file=sys.stderr)
    return out


def bench_ooc_cfg5_sharded(dev, ws, rank, barrier, max_over_ranks, n_ch=50_000, seconds=3600.0,
                           push_s=60.0):
    """cfg5 across the ranks (BASELINE configs[4], "across 8xMI355X"):
    every rank opens ``shard_stream`` on its channel block of the 50,000-ch
    @ 200 Hz spool and pushes its rows of each full-width host block
    (``push_rows``; only its own rows are touched and page-locked,
    ``pin_rows``).  No data exchange: N independent host->HBM streams.
    ``value`` = all ranks' channel-samples / max-over-ranks wall time,
    outputs downloaded inside the timed loop; the first and last channel of
    every rank are checked against the oracle afterwards (untimed).  Every
    collective here runs on every rank whatever happened locally (a local
    failure is agreed on, not left to hang the others)."""
    import torch
    from lfdas.plan import set_timing
    from lfdas.shard import pin_rows, push_rows, shard_stream
    fs = 200.0
    push = int(push_s * fs)
    n = int(seconds * fs)
    n_push = n // push
    dt_ns = int(1e9 / fs)
    t0 = 1_679_464_800_000_000_000
    t_end = t0 + (n - 1) * dt_ns
    st, blocks, pins, err = None, [], [], None
    try:
        st, (c0, c1) = shard_stream(n_ch, dt_ns, output_sample_interval=10.0, process_patch_size=120,
                                    edge_buff_size=6, mode="continuous", t_start=t0, t_end=t_end,
                                    capacity=int(1300 * fs) + 2 * push, device=dev)
        # full-width host blocks: virtual memory, only this rank's rows written
        for i in range(2):
            b = np.empty((n_ch, push), np.float32)
            d = torch.empty((c1 - c0, push), dtype=torch.float32, device=dev)
            synth_fill(d, fs, 777 + 100 * rank + i)
            b[c0:c1] = d.cpu().numpy()
            del d
            pins.append(pin_rows(b, (c0, c1)))
            blocks.append(b)
        st.reserve(push)
    except Exception as e:
        err = e
    if max_over_ranks(1.0 if err is not None else 0.0) > 0:  # also the start barrier
        for p in pins:  # page-locked rows released now, not whenever GC runs
            p.release()
        if st is not None:
            st.close()
        return {"error": repr(err) if err is not None else "setup failed on another rank"}
    rows = [c0, c1 - 1]
    ys, ts, n_out = [], [], 0
    torch.cuda.synchronize(dev)
    ta = time.perf_counter()
    try:
        set_timing(True)
        for k in range(n_push):
            o = push_rows(st, blocks[k % 2], (c0, c1), t0 + k * push * dt_ns)
            n_out += o.n_out
            if o.n_out:
                y = st.fetch()
                ys.append(y[[r - c0 for r in rows]].copy())
                ts.append(o.times_ns)
            else:
                st.wait_copy()
        o = st.flush()
        n_out += o.n_out
        if o.n_out:
            ys.append(st.fetch()[[r - c0 for r in rows]].copy())
            ts.append(o.times_ns)
        st.synchronize()
        el = time.perf_counter() - ta
    except Exception as e:
        err, el = e, float("inf")
    finally:
        set_timing(False)
    st.close()
    el_max = max_over_ranks(el)
    rel, ok = float("inf"), 0.0
    if err is None:
        try:
            xs = np.concatenate([blocks[k % 2][rows] for k in range(n_push)], axis=1)
            sys.path.insert(0, ROOT)
            import oracle
            ref = oracle.lfproc_process(xs, t0, dt_ns, t0, t_end, 10.0, 120, 6)
            want = np.concatenate([r for _, r in ref], axis=1)
            got = np.concatenate(ys, axis=1) if ys else np.zeros((len(rows), 0))
            times_ok = bool(np.array_equal(np.concatenate(ts) if ts else np.zeros(0, np.int64),
                                           np.concatenate([t for t, _ in ref])))
            if got.shape == want.shape:
                rel = float(np.sqrt(np.sum((got.astype(np.float64) - want) ** 2) / np.sum(want ** 2)))
            ok = 1.0 if (times_ok and rel < 1e-9) else 0.0
        except Exception as e:
            err = e
    for p in pins:
        p.release()
    del blocks
    all_ok = -max_over_ranks(-ok)  # min over ranks
    worst = max_over_ranks(rel)
    if err is not None or not np.isfinite(el_max):
        return {"error": repr(err) if err is not None else "stream failed on another rank"}
    samples = n_ch * n_push * push
    return {"value": samples / el_max, "unit": "channel-samples/s", "n_gpus": ws,
            "wall_s": el_max, "h2d_GBps_total": samples * 4 / el_max / 1e9,
            "h2d_GBps_per_gpu": samples * 4 / el_max / 1e9 / ws, "channels_rank0": c1 - c0,
            "outputs_per_channel": n_out, "scaling": "strong",
            "config": f"{n_ch:,} ch @ 200 Hz, {seconds:.0f} s of the 24 h spool in {push_s:.0f} s pushes, "
                      f"dt = 10 s, P = 120, B = 6, channel-sharded over {ws} GPUs (shard_stream + push_rows, "
                      "each rank's rows page-locked in place); outputs downloaded inside the timed loop",
            "check": {"rows_per_rank": "first and last channel", "worst_relrms_vs_oracle": worst,
                      "pass": bool(all_ok > 0.5), "checker": "oracle.lfproc_process (untimed)"}}


def bench_fir_decimate(dev, q=10, n_ch=2000, n=600_000, fs=1000.0, reps=10):
    """Patch.decimate(time=q, filter_type='fir') (scipy.signal.decimate
    ftype='fir': firwin(20q+1, 1/q) via resample_poly): 2,000 ch x 10 min @
    1 kHz float32 -> float64 at fs/q.  Algorithmic bytes 4 + 8/q per input
    sample; kernel k_fir_decimate_mfma (fp64 matrix cores)."""
    import torch
    import oracle
    from lfdas._lib import load
    from lfdas.plan import fir_decimate_device
    from lfdas.proc import fir_decimate_design
    taps, delay = fir_decimate_design(q)
    x = torch.empty((n_ch, n), dtype=torch.float32, device=dev)
    synth_fill(x, fs, 91)
    h = torch.as_tensor(taps).to(dev)
    y = torch.empty((n_ch, -(-n // q)), dtype=torch.float64, device=dev)
    lib = load()
    stream = torch.cuda.current_stream(dev)

    from lfdas._lib import check
    from lfdas.plan import _ptr

    def run():
        check(lib.lfd_fir_decimate_f32(_ptr(x), n_ch, n, x.stride(0), x.stride(1), _ptr(h), h.numel(), q, delay,
                                       _ptr(y), y.stride(0), y.stride(1), stream.cuda_stream))
    for _ in range(2):
        run()
    torch.cuda.synchronize(dev)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        run()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    kern = "k_fir_decimate_mfma" if lib.lfd_fir_decimate_last_kernel() == 1 else "k_fir_decimate"
    gbs = n_ch * n * (4 + 8 / q) / (ms * 1e-3) / 1e9
    # parity spot check outside the timed region (2 channels vs the oracle)
    rows = [0, n_ch - 1]
    ref = oracle.decimate_fir(x[rows].double().cpu().numpy(), q)
    got = y[rows].cpu().numpy()
    rel = float(np.sqrt(np.sum((got - ref) ** 2) / np.sum(ref ** 2)))
    del x, y, h
    torch.cuda.empty_cache()
    return {"value": n_ch * n / (ms * 1e-3), "unit": "channel-samples/s", "ms": ms, "kernel": kern,
            "config": f"{n_ch:,} ch x {n:,} @ {fs:g} Hz fp32 -> f64, decimate(time={q}, filter_type='fir'), "
                      f"{taps.size} taps",
            "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": gbs / HBM_PEAK_GBS, "alg_bytes_per_sample": 4 + 8 / q},
            "relrms_vs_oracle_2ch": rel}


def bench_rolling(dev, W, S_, reps=10):
    """cfg2 rolling mean (5,000 ch x 10 min @ 1 kHz), window W, step S_;
    algorithmic bytes 4 + 4/S per channel-sample."""
    import torch
    from lfdas.plan import rolling_mean_device
    xr = torch.empty((5000, 600_000), dtype=torch.float32, device=dev)
    synth_fill(xr, 1000.0, 99)
    for _ in range(2):
        y = rolling_mean_device(xr, W, S_)
    torch.cuda.synchronize(dev)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        y = rolling_mean_device(xr, W, S_)
    e1.record()
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    gbs = 5000 * 600_000 * (4 + 4 / S_) / (ms * 1e-3) / 1e9
    del xr, y
    torch.cuda.empty_cache()
    return {"value": 5000 * 600_000 / (ms * 1e-3), "unit": "channel-samples/s", "ms": ms,
            "config": f"5,000 ch x 10 min @ 1 kHz fp32, W = {W}, S = {S_}",
            "kernel": ("k_rolling_tc" if S_ >= W else
                       ("k_rolling_seg" if S_ > 1 and np.gcd(W, S_) >= 16 else "k_rolling_scan_tc")),
            "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": gbs / HBM_PEAK_GBS, "alg_bytes_per_sample": 4 + 4 / S_}}


def bench_fullrate(dev, n_ch=2000, n=600_000, fs=1000.0, band=(1.0, 10.0), reps=5):
    """Full-rate zero-phase band-pass (DASCore ``pass_filter(time=band)``
    .data -> scipy sosfiltfilt): 2,000 ch x 10 min @ 1 kHz, 8th-order
    Butterworth band-pass (4 sections), float32 in, float64 out (SciPy's
    dtype).  Algorithmic bytes 4 + 8 per channel-sample.  The dominant
    kernel is the output pass k_fullrate_out_mb<4> (x read + y written over
    the medium blocks, 12 B per sample)."""
    import torch
    import oracle
    from lfdas.design import pass_filter_sos
    from lfdas.plan import load, set_timing, sosfiltfilt_device, sosfiltfilt_last_timing_ms
    # the product's own filter design (the oracle is only the spot check below)
    sos = pass_filter_sos(fs, band[0], band[1])
    x = torch.empty((n_ch, n), dtype=torch.float32, device=dev)
    synth_fill(x, fs, 77)
    y = torch.empty((n_ch, n), dtype=torch.float64, device=dev)
    wsb = load().lfd_sosfiltfilt_workspace_bytes(n_ch, n, -1, sos.shape[0])
    ws = torch.empty(int(wsb), dtype=torch.uint8, device=dev)
    for _ in range(2):
        sosfiltfilt_device(x, sos, y=y, ws=ws)
    torch.cuda.synchronize(dev)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        sosfiltfilt_device(x, sos, y=y, ws=ws)
    e1.record()
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    set_timing(True)
    kt = []
    for _ in range(reps):
        sosfiltfilt_device(x, sos, y=y, ws=ws)
        kt.append(sosfiltfilt_last_timing_ms())
    set_timing(False)
    kt = np.mean(np.array(kt), axis=0)
    LB = 512  # medium block: the output pass covers M = (n - 1) // 512 of them
    n_out_s = (n - 1) // LB * LB
    gbs_out = n_ch * n_out_s * 12 / (kt[2] * 1e-3) / 1e9
    gbs_all = n_ch * n * 12 / (ms * 1e-3) / 1e9
    # parity spot check outside the timed region (3 channels vs the oracle)
    rows = [0, n_ch // 2, n_ch - 1]
    xs = x[rows].cpu().numpy()
    rel = float(np.sqrt(np.sum((y[rows].cpu().numpy() - oracle.sosfiltfilt(sos, xs)) ** 2)
                        / np.sum(oracle.sosfiltfilt(sos, xs) ** 2)))
    # the previous one-thread-per-channel kernel on a tenth of the samples
    from lfdas._lib import kernel_options
    with kernel_options(fullrate_serial=1):
        xs10 = x[:, : n // 10]
        ys10 = y[:, : n // 10]
        sosfiltfilt_device(xs10, sos, y=ys10, ws=ws)
        torch.cuda.synchronize(dev)
        e0.record()
        sosfiltfilt_device(xs10, sos, y=ys10, ws=ws)
        e1.record()
        torch.cuda.synchronize(dev)
        serial_ms = e0.elapsed_time(e1)
    # CPU: SciPy's sosfiltfilt itself on 24 channels (single core)
    from scipy.signal import sosfiltfilt as sp_sosfiltfilt
    xc = x[:24].cpu().numpy()
    ta = time.perf_counter()
    sp_sosfiltfilt(sos, xc, axis=-1)
    cpu_s = time.perf_counter() - ta
    del x, y, ws
    torch.cuda.empty_cache()
    return {"value": n_ch * n / (ms * 1e-3), "unit": "channel-samples/s", "ms": ms,
            "config": f"{n_ch:,} ch x {n:,} @ {fs:g} Hz fp32 -> f64, Butterworth band-pass {band} Hz "
                      f"(corners=4, {sos.shape[0]} sections), zero-phase, full rate",
            "kernels_ms": {"k_block_functionals_mfma (medium-block functionals, fp64 MFMA)": kt[0],
                           "k_fullrate_scan_seg<4> (segmented scan)": kt[1],
                           "k_fullrate_out_mb<4> (output)": kt[2]},
            "roofline": {"bound": "hbm", "kernel": "k_fullrate_out_mb<4>", "achieved": gbs_out,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs_out / HBM_PEAK_GBS,
                         "alg_bytes_per_sample": 12, "samples_per_launch": n_ch * n_out_s},
            "pipeline_hbm_frac": gbs_all / HBM_PEAK_GBS,
            "relrms_vs_oracle_3ch": rel,
            "serial_kernel_ms_tenth": serial_ms,
            "serial_kernel_value": n_ch * (n // 10) / (serial_ms * 1e-3),
            "cpu_baseline": {"value": 24 * n / cpu_s, "unit": "channel-samples/s", "cores": 1,
                             "kind": "reference-lib", "sample": f"scipy.signal.sosfiltfilt, 24 ch x {n:,}"}}


def _cpu_worker(a, barrier=None, q=None):
    """One CPU-baseline process: the LFProc chunks of ``n_c`` channels x the
    full hour (own data, made before the start barrier)."""
    backend, fs, seconds, n_c, seed, sos, sched, t0, dt_ns, tg = a
    x = _cpu_data(n_c, int(seconds * fs), fs, seed)
    if barrier is not None:
        barrier.wait()
    ta = time.perf_counter()
    _cpu_chunks(backend, x, sos, sched, t0, dt_ns, tg)
    el = time.perf_counter() - ta
    if q is not None:
        q.put(el)
    return el


def cpu_workers() -> int:
    """The host cores this job may use: the box's CPU share (OMP_NUM_THREADS,
    16 per GPU on the pool) bounded by the affinity mask."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        aff = os.cpu_count() or 1
    cap = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
    return max(1, min(aff, cap, 16))


def cpu_baseline_parallel(args, sos, sched, t0, dt_ns, tg, n_c_per=48, backend="port"):
    """SURVEY §8(d) figure 2: one worker PROCESS per core over channel blocks
    (SciPy's _sosfilt does not scale with threads).  Forked before the GPU is
    initialised.  Channel-sample rate of the whole pool (wall clock)."""
    import multiprocessing as mp
    nw = cpu_workers()
    ctx = mp.get_context("fork")
    barrier = ctx.Barrier(nw + 1)
    q = ctx.Queue()
    procs = [ctx.Process(target=_cpu_worker, args=((backend, args.fs, args.seconds, n_c_per, 100 + i, sos, sched,
                                                     t0, dt_ns, tg), barrier, q)) for i in range(nw)]
    for p in procs:
        p.start()
    barrier.wait()  # every worker holds its data
    ta = time.perf_counter()
    per = [q.get(timeout=600) for _ in procs]
    wall = time.perf_counter() - ta
    for p in procs:
        p.join()
    n = int(args.seconds * args.fs)
    what = "oracle C sosfiltfilt + interp1d" if backend == "port" else "scipy sosfiltfilt + interp1d"
    return {"value": nw * n_c_per * n / wall, "cores": nw, "wall_s": wall,
            "sample": f"{nw} processes x {n_c_per} ch x {n} samples, same LFProc chunks, {what}; "
                      f"per-process {min(per):.1f}-{max(per):.1f} s"}


def main():
    args = _args()
    global PIPELINED
    PIPELINED = args.pipelined
    rc = launch_or_check(args)
    if rc is not None:
        sys.exit(rc)
    import torch
    ws, rank, local = _dist()
    n = int(args.seconds * args.fs)
    cpu = None
    if ws == 1 and not args.no_cpu:
        # host-only plan geometry (the library's schedule), then the CPU legs
        # before the GPU is initialised (the parallel legs fork)
        from lfdas import schedule as S
        from lfdas.design import lowpass_sos
        c_dt_ns = int(round(1e9 / args.fs))
        c_t0 = 1_505_692_800_000_000_000
        c_tg = S.time_grid(c_t0, c_t0 + n * c_dt_ns, args.dt_out)
        c_sched = S.lfproc_chunks(len(c_tg), args.patch_size, args.edge_buff)
        c_sos = lowpass_sos(args.fs, 1 / args.dt_out / 2 * 0.9, 4)
        geo = (c_sos, c_sched, c_t0, c_dt_ns, c_tg)
        one = cpu_baseline(args, *geo)
        par = cpu_baseline_parallel(args, *geo)
        cpu = {"value": par["value"], "unit": "channel-samples/s", "cores": par["cores"], "kind": "port",
               "extrapolated": True,
               "sample": par["sample"] + "; rate extrapolated linearly to the full 10,000-channel step",
               "single_process": {"value": one["value"], "cores": 1, "sample": one["sample"]},
               "workers": "processes (fork) over channel blocks"}
        try:  # the reference's own numeric library (scipy), timed the same way
            one_s = cpu_baseline(args, *geo, backend="scipy", n_c=192)
            par_s = cpu_baseline_parallel(args, *geo, n_c_per=16, backend="scipy")
            cpu["reference_lib"] = {"value": par_s["value"], "unit": "channel-samples/s", "cores": par_s["cores"],
                                    "kind": "reference-lib", "extrapolated": True, "sample": par_s["sample"],
                                    "single_process": {"value": one_s["value"], "cores": 1,
                                                       "sample": one_s["sample"]}}
        except ImportError as e:  # pragma: no cover
            cpu["reference_lib"] = {"error": repr(e)}
    if ws > 1:
        import torch.distributed as dist
        if args.one_device:
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if ws > 1 and not args.one_device else 0)
    comm_dev = torch.device("cpu") if args.one_device else dev
    torch.cuda.set_device(dev)

    from lfdas.shard import channel_range
    if args.weak:
        n_ch_total, (c0, c1) = args.channels * ws, (0, args.channels)
    else:
        n_ch_total = args.channels
        c0, c1 = channel_range(args.channels, ws, rank)
    n_ch = c1 - c0
    plan, sched, sos, t0, dt_ns, tg = build_plan(n_ch, n, args.fs, args.dt_out, args.patch_size,
                                                 args.edge_buff)
    # the product's sample buffer (lfdas.arena: a rank's 9 GB shard of an
    # N = 8 run sits in a >= 32 GiB allocation, the translation-friendly
    # placement; the 72 GB single-GPU input is that size already)
    x = device_samples((n_ch, n), device=dev)
    synth_fill(x, args.fs, 1234 + rank)
    y = torch.empty((n_ch, plan.n_grid), dtype=torch.float64, device=dev)
    wsb = plan.alloc_workspace(dev)
    stream = torch.cuda.current_stream(dev)

    def barrier():
        torch.cuda.synchronize(dev)
        if ws > 1:
            torch.distributed.barrier()

    def max_over_ranks(v):
        if ws == 1:
            return v
        tt = torch.tensor([v], device=comm_dev, dtype=torch.float64)
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        return float(tt.item())

    # every rank reports in over the data-path backend (RCCL for N > 1)
    ranks_seen = 1
    if ws > 1:
        one = torch.ones(1, device=comm_dev, dtype=torch.int64)
        torch.distributed.all_reduce(one)
        ranks_seen = int(one.item())
    el, k1_ms, scan_ms = time_plan(plan, x, y, wsb, stream, args.steps, args.warmup, barrier)
    el_serial = max_over_ranks(el)
    el = el_serial
    if PIPELINED:
        el = max_over_ranks(time_plan_pipelined(plan, x, y, args.steps, args.warmup, barrier))
    k1_kernel = plan.last_kernel()

    R = int(round(args.fs * args.dt_out))
    value = n_ch_total * n * args.steps / el
    k1 = float(np.mean(k1_ms))
    alg_bytes = n_ch * n * (4.0 + 8.0 / R)
    achieved = alg_bytes / (k1 * 1e-3) / 1e9
    traffic = None
    try:
        with open(args.pmc) as f:
            pm = json.load(f)
        if pm.get("channels") == n_ch and pm.get("samples") == n:
            traffic = pm.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass

    secondary = {}
    if ws > 1:
        # the path's one collective, outside the timed step: RCCL all-gather of
        # the decimated outputs (lfdas.shard.all_gather_channels), every rank
        # ends with all n_ch_total channels
        from lfdas.shard import all_gather_channels
        try:
            g_ms = []
            for i in range(4):
                barrier()
                t_g = time.perf_counter()
                full = all_gather_channels(y.to(comm_dev), n_ch_total)
                torch.cuda.synchronize(dev)
                if i:
                    g_ms.append((time.perf_counter() - t_g) * 1e3)
            del full
            gm = max_over_ranks(float(np.median(g_ms)))
            secondary["allgather_outputs"] = {
                "ms": gm, "bytes_per_rank": int(y.numel() * 8), "frac_of_step": gm / (el / args.steps * 1e3),
                "note": "RCCL all_gather of every rank's (n_ch, n_grid) float64 outputs; not in the timed step"}
        except Exception as e:  # the optional gather never voids the bench line
            secondary["allgather_outputs"] = {"error": repr(e)}
    del x, y, wsb
    plan.close()
    torch.cuda.empty_cache()
    if ws > 1:
        # the other scaling mode beside the headline: weak (every rank its own
        # 10,000 channels) under the strong default, strong under --weak
        if not args.weak:
            o0, o1, o_tot, o_key = 0, args.channels, ws * args.channels, "weak_scaling_cfg3"
        else:
            (o0, o1), o_tot, o_key = channel_range(args.channels, ws, rank), args.channels, "strong_scaling_cfg3"
        plan_w, _, _, _, _, _ = build_plan(o1 - o0, n, args.fs, args.dt_out, args.patch_size, args.edge_buff)
        xw = device_samples((o1 - o0, n), device=dev)
        synth_fill(xw, args.fs, 4321 + rank)
        yw = torch.empty((o1 - o0, plan_w.n_grid), dtype=torch.float64, device=dev)
        ww = plan_w.alloc_workspace(dev)
        el_w, k1_w, _ = time_plan(plan_w, xw, yw, ww, stream, args.steps, 1, barrier)
        el_w = max_over_ranks(el_w)
        secondary[o_key] = {
            "value": o_tot * n * args.steps / el_w, "unit": "channel-samples/s",
            "ms_per_step": el_w / args.steps * 1e3, "kernel_ms_rank0": float(np.mean(k1_w)),
            "channels_rank0": o1 - o0, "scaling": "strong" if o_key.startswith("strong") else "weak",
            "config": (f"{args.channels:,} ch x 1 h @ 500 Hz split over {ws} GPUs" if o_key.startswith("strong")
                       else f"{args.channels:,} ch x 1 h @ 500 Hz per GPU x {ws} GPUs")}
        del xw, yw, ww
        plan_w.close()
        torch.cuda.empty_cache()
    if ws > 1 and not args.no_stream:
        try:
            secondary["out_of_core_cfg5_sharded"] = bench_ooc_cfg5_sharded(dev, ws, rank, barrier,
                                                                           max_over_ranks)
        except Exception as e:  # pragma: no cover - reported, never voids the headline line
            secondary["out_of_core_cfg5_sharded"] = {"error": repr(e)}
        torch.cuda.empty_cache()
    if ws == 1 and not args.no_extra:
        secondary["cfg3_offsample_grid"] = bench_lowpass_line(
            dev, args.channels, args.fs, args.seconds, args.dt_out, args.patch_size, args.edge_buff,
            off_ns=1_900_000, label="cfg3 with the samples starting 1.9 ms after the output grid's second "
                                    "(every output interpolated between two samples, w = 0.05)")
        secondary["cfg3_time_major"] = bench_lowpass_line(
            dev, args.channels, args.fs, args.seconds, args.dt_out, args.patch_size, args.edge_buff,
            time_major=True, label="cfg3 stored (time, distance) like the real files (data[:, ch])")
        secondary["lowpass_1khz_dt10"] = bench_lowpass_line(
            dev, 10_000, 1000.0, 3600.0, 10.0, 120, 6,
            label="10,000 ch x 1 h @ 1 kHz (144 GB), dt = 10 s (the batch notebook's d_t), P = 120, B = 6: "
                  "R = 10,000 as 20 sub-blocks of 500")
    if ws == 1 and not args.no_extra:
        # a grid no single uniform block plan takes: 3 kHz samples on integer-ns
        # times (333,333 ns) drift against the 1 s output grid (lattice plan:
        # one K1 pass forms every phase's outputs, then the interp1d blend)
        secondary["lowpass_3khz_lattice"] = bench_lowpass_line(
            dev, 2000, 3000.0, 1800.0, 1.0, 600, 7,
            label="2,000 ch x 30 min @ 3 kHz (333,333 ns samples: varying interpolation fraction, spacing "
                  "3,000 / 3,001), dt = 1 s, P = 600, B = 7: lattice plan, one pass (kernel_ms = the K1 pass "
                  "with every phase's outputs, scan_kernel_ms = state scan + per-phase outputs + blend)")
    if ws == 1 and not args.no_extra:
        # strong-scaling proxy on one GPU: the channel shard one rank of an
        # N-GPU run owns, timed alone — in a FRESH child process (this same
        # script, --channels c), as each rank of the real run is: a shard's K1
        # depends on where the driver places its samples (lfdas.arena), and
        # this process has allocated and freed ~500 GB by now (in-process the
        # 1,250-channel K1 measured 1.66-1.77 ms by box, in fresh processes
        # 1.65 every time: profiles/r05_alloc_placement.txt).  The driver's
        # SCALE run is the record
        shards = {}
        for n_gpu in (2, 4, 8):
            c = -(-args.channels // n_gpu)
            r = shard_line_fresh(args, c)
            where = "fresh process"
            if r is None:  # (the child failed: the same line in this process)
                r = bench_lowpass_line(dev, c, args.fs, args.seconds, args.dt_out, args.patch_size,
                                       args.edge_buff, steps=20, warmup=3,
                                       label=f"{c:,}-channel shard of cfg3 ({n_gpu} GPUs)")
                where = "this process"
            shards[f"n{n_gpu}"] = {"channels": c, "ms_per_step": r["ms_per_step"],
                                   "measured_in": where,
                                   "kernel_ms": r["roofline"]["kernel_ms"],
                                   "scan_kernel_ms": r["roofline"]["scan_kernel_ms"],
                                   "roofline_frac": r["roofline"]["frac"],
                                   "projected_efficiency": (el / args.steps * 1e3 / n_gpu) / r["ms_per_step"]}
        secondary["shard_widths_1gpu"] = shards
    if ws == 1 and not args.no_extra:
        secondary["fullrate_bandpass"] = bench_fullrate(dev)
        secondary["fir_decimate_q10"] = bench_fir_decimate(dev)
    if not args.no_rolling and ws == 1:
        secondary["rolling_mean_cfg2"] = bench_rolling(dev, 1000, 1000)
        secondary["rolling_mean_cfg2_step1"] = bench_rolling(dev, 1000, 1, reps=5)
        secondary["rolling_mean_cfg2_step250"] = bench_rolling(dev, 1000, 250, reps=5)
    if not args.no_stream and ws == 1:
        secondary["edge_latency_cfg4"] = bench_edge_cfg4(dev)
        secondary["edge_latency_cfg4_time_major"] = bench_edge_cfg4(dev, time_major=True)
        torch.cuda.empty_cache()
        secondary["out_of_core_cfg5"] = bench_ooc_cfg5(dev, seconds=args.cfg5_hours * 3600.0)
        torch.cuda.empty_cache()

    if rank == 0:
        out = {
            "metric": "channel-samples/s low-pass+decimate",
            "value": value,
            "unit": "channel-samples/s",
            "n_gpus": ws,
            "ranks_seen": ranks_seen,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": el / args.steps * 1e3,
            "ms_per_step_serial": el_serial / args.steps * 1e3,
            "pipelined": ("each step's chunk scan runs beside the next step's block pass (lfdas.plan."
                          "LowpassPipeline: two workspaces, one block stream, one scan stream); every step "
                          "is the full computation" if PIPELINED else False),
            "higher_is_better": True,
            "scaling": "weak" if args.weak else "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (0.5 + sin + N(0,1), generated on device)",
            "config": {"workload": "cfg3: 10,000 ch x 1 h @ 500 Hz fp32 (72 GB), 4th-order Butterworth "
                                   "0.45 Hz zero-phase, decimate to 1 Hz, LFProc P=600 B=7"
                                   + (", per GPU" if args.weak else ", channel-sharded over the GPUs"),
                       "channels": n_ch_total, "channels_rank0": n_ch, "samples": n, "fs": args.fs,
                       "dt_out": args.dt_out, "chunks": len(sched),
                       "outputs_per_channel": int(sum(b - a for _, _, a, b in sched)),
                       "parallelism": (f"one spool per GPU x{ws} (channel-partitioned job)" if args.weak
                                       else f"channel-shard x{ws}"),
                       "io_dtype": "f32"},
            **({"rehearsal": "--one-device: every rank on cuda:0 over gloo; not a scaling number"}
               if args.one_device else {}),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": K1_KERNELS.get(k1_kernel), "kernel_ms": k1,
                         "scan_kernel_ms": float(np.mean(scan_ms)),
                         "alg_bytes_per_sample": 4.0 + 8.0 / R, "samples_per_launch": n_ch * n},
            "cpu_baseline": cpu,
            "secondary": secondary,
        }
        print(json.dumps(out))
    if ws > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
