"""Benchmark of the north-star path: chunked zero-phase low-pass + decimate
(LFProc.process_time_range, lf_das.py:219-290) on MI355X.

Workload (BASELINE.json configs[2], "cfg3"): 10,000 channels x 1 h @ 500 Hz
float32 (72 GB, channel-major, DASCore dims ("distance","time")), 4th-order
Butterworth at 0.45 Hz, decimate to 1 Hz, LFProc chunking P = 600, B = 7.
One step = one pass of the hot path over the whole hour (7 overlapping chunks,
3,585 outputs per channel), inputs resident in HBM.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--channels C]

N > 1 is launched by torch.distributed.run (one rank per GPU); channels shard
across ranks with no data-path collective (weak scaling: every rank owns a
10,000-channel spool).  Rank 0 prints ONE JSON line.
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
    p.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                   help="rocprofv3 PMC traffic summary (tools/pmc_summary.py) for roofline.traffic")
    return p.parse_args()


def _dist():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


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


def build_plan(n_ch, n, fs, dt_out, P, B):
    from lfdas import schedule as S
    from lfdas.design import lowpass_sos
    from lfdas.plan import LowpassPlan
    dt_ns = int(round(1e9 / fs))
    t0 = 1_505_692_800_000_000_000
    tg = S.time_grid(t0, t0 + n * dt_ns, dt_out)
    sched = S.lfproc_chunks(len(tg), P, B)
    lo, w = S.grid_positions(t0, dt_ns, tg)
    chunks = [(*S.select_range(t0, dt_ns, n, tg[a], tg[b]), oa, ob) for a, b, oa, ob in sched]
    sos = lowpass_sos(fs, 1 / dt_out / 2 * 0.9, 4)
    return LowpassPlan(sos, n_ch, n, lo, w, chunks), sched, sos, t0, dt_ns, tg


def cpu_baseline(args, sos, sched, t0, dt_ns, tg):
    """Oracle C restatement of scipy's sosfiltfilt (+ interp) over the same
    LFProc chunks, 1 process / 1 thread, on a bounded channel sample."""
    sys.path.insert(0, ROOT)
    import oracle
    n = int(args.seconds * args.fs)
    rng = np.random.default_rng(0)
    n_c = args.cpu_channels
    t = np.arange(n, dtype=np.float64) * (2 * np.pi * 0.05 / args.fs)
    x = (rng.standard_normal((n_c, n)) + 0.5 + np.sin(t)[None, :]).astype(np.float32)
    from lfdas import schedule as S
    t_start = time.perf_counter()
    for a, b, oa, ob in sched:
        s0, s1 = S.select_range(t0, dt_ns, n, tg[a], tg[b])
        y = oracle.sosfiltfilt_rows_c(sos, x[:, s0:s1 + 1])
        tt = (np.arange(s0, s1 + 1, dtype=np.int64) * dt_ns).astype(np.float64)
        oracle.interp1d_linear(tt, y, (tg[oa:ob] - t0).astype(np.float64))
    el = time.perf_counter() - t_start
    return {"value": n_c * n / el, "unit": "channel-samples/s", "cores": 1, "kind": "port",
            "sample": f"{n_c} ch x {n} samples ({args.seconds:.0f} s @ {args.fs:.0f} Hz), same LFProc "
                      f"chunks, oracle C sosfiltfilt + interp1d, 1 thread, {el:.1f} s"}


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


def bench_ooc_cfg5(dev, n_ch=50_000, seconds=3600.0, push_s=60.0):
    """cfg5 (bounded sample): out-of-core process_time_range over a 50,000-ch
    @ 200 Hz spool streamed from a pinned host ring, dt = 10 s (fc = 0.045 Hz),
    P = 120 (1,200 s chunks), B = 6 (planner edge 60 s).  Bound: PCIe."""
    import torch
    from lfdas.stream import LowpassStream
    fs = 200.0
    push = int(push_s * fs)
    n = int(seconds * fs)
    dt_ns = int(1e9 / fs)
    t0 = 1_679_464_800_000_000_000
    blocks = _pinned_blocks(dev, 2, (n_ch, push), fs, 777)
    st = LowpassStream(n_ch, dt_ns, 10.0, 120, 6, mode="continuous", t_start=t0,
                       t_end=t0 + (n - 1) * dt_ns, capacity=int(1300 * fs) + 2 * push)
    from lfdas.plan import set_timing
    st.reserve(push)
    n_out = 0
    cp = []
    torch.cuda.synchronize(dev)
    set_timing(True)
    ta = time.perf_counter()
    for k in range(n // push):
        o = st.push(blocks[k % 2], t0 + k * push * dt_ns)
        n_out += o.n_out
        st.wait_copy()  # ring buffer (k+1) % 2 is free again
        cp.append(st.last_timing_ms()[0])
    set_timing(False)
    o = st.flush()
    n_out += o.n_out
    st.synchronize()
    el = time.perf_counter() - ta
    st.close()
    del blocks
    samples = n_ch * (n // push) * push
    return {"value": samples / el, "unit": "channel-samples/s", "seconds_streamed": seconds,
            "wall_s": el, "h2d_GBps": samples * 4 / el / 1e9, "pcie_peak_GBps": 63.0,
            "pcie_frac": samples * 4 / el / 1e9 / 63.0, "outputs_per_channel": n_out,
            "copy_ms_p50": float(np.median(cp)), "copy_ms_max": float(np.max(cp)),
            "config": f"{n_ch:,} ch @ 200 Hz, {seconds:.0f} s of the 24 h spool in {push_s:.0f} s pinned "
                      "pushes, dt = 10 s, P = 120, B = 6, 1 GPU"}


def _cpu_worker(a, barrier=None, q=None):
    """One CPU-baseline process: the LFProc chunks of ``n_c`` channels x the
    full hour through the oracle C sosfiltfilt + interp1d (own data, made
    before the start barrier)."""
    fs, seconds, n_c, seed, sos, sched, t0, dt_ns, tg = a
    sys.path.insert(0, ROOT)
    import oracle
    from lfdas import schedule as S
    n = int(seconds * fs)
    rng = np.random.default_rng(seed)
    t = np.arange(n, dtype=np.float64) * (2 * np.pi * 0.05 / fs)
    x = (rng.standard_normal((n_c, n)) + 0.5 + np.sin(t)[None, :]).astype(np.float32)
    if barrier is not None:
        barrier.wait()
    ta = time.perf_counter()
    for a_, b_, oa, ob in sched:
        s0, s1 = S.select_range(t0, dt_ns, n, tg[a_], tg[b_])
        y = oracle.sosfiltfilt_rows_c(sos, x[:, s0:s1 + 1])
        tt = (np.arange(s0, s1 + 1, dtype=np.int64) * dt_ns).astype(np.float64)
        oracle.interp1d_linear(tt, y, (tg[oa:ob] - t0).astype(np.float64))
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


def cpu_baseline_parallel(args, sos, sched, t0, dt_ns, tg, n_c_per=48):
    """SURVEY §8(d) figure 2: one worker PROCESS per core over channel blocks
    (SciPy's _sosfilt does not scale with threads).  Forked before the GPU is
    initialised.  Channel-sample rate of the whole pool (wall clock)."""
    import multiprocessing as mp
    nw = cpu_workers()
    ctx = mp.get_context("fork")
    barrier = ctx.Barrier(nw + 1)
    q = ctx.Queue()
    procs = [ctx.Process(target=_cpu_worker, args=((args.fs, args.seconds, n_c_per, 100 + i, sos, sched,
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
    return {"value": nw * n_c_per * n / wall, "cores": nw, "wall_s": wall,
            "sample": f"{nw} processes x {n_c_per} ch x {n} samples, same LFProc chunks, oracle C "
                      f"sosfiltfilt + interp1d; per-process {min(per):.1f}-{max(per):.1f} s"}


def main():
    args = _args()
    import torch
    ws, rank, local = _dist()
    if ws > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if ws > 1 else 0)
    torch.cuda.set_device(dev)

    from lfdas.plan import set_timing
    n_ch = args.channels
    n = int(args.seconds * args.fs)
    cpu = None
    if ws == 1 and not args.no_cpu:
        # host-only plan geometry (the library's schedule), then the CPU legs
        # before the GPU is initialised (the parallel leg forks)
        from lfdas import schedule as S
        from lfdas.design import lowpass_sos
        c_dt_ns = int(round(1e9 / args.fs))
        c_t0 = 1_505_692_800_000_000_000
        c_tg = S.time_grid(c_t0, c_t0 + n * c_dt_ns, args.dt_out)
        c_sched = S.lfproc_chunks(len(c_tg), args.patch_size, args.edge_buff)
        c_sos = lowpass_sos(args.fs, 1 / args.dt_out / 2 * 0.9, 4)
        one = cpu_baseline(args, c_sos, c_sched, c_t0, c_dt_ns, c_tg)
        par = cpu_baseline_parallel(args, c_sos, c_sched, c_t0, c_dt_ns, c_tg)
        cpu = {"value": par["value"], "unit": "channel-samples/s", "cores": par["cores"], "kind": "port",
               "extrapolated": True,
               "sample": par["sample"] + "; rate extrapolated linearly to the full 10,000-channel step",
               "single_process": {"value": one["value"], "cores": 1, "sample": one["sample"]},
               "workers": "processes (fork) over channel blocks"}
    plan, sched, sos, t0, dt_ns, tg = build_plan(n_ch, n, args.fs, args.dt_out, args.patch_size,
                                                 args.edge_buff)
    x = torch.empty((n_ch, n), dtype=torch.float32, device=dev)
    synth_fill(x, args.fs, 1234 + rank)
    y = torch.empty((n_ch, plan.n_grid), dtype=torch.float32, device=dev)
    wsb = plan.alloc_workspace(dev)
    stream = torch.cuda.current_stream(dev)

    def barrier():
        torch.cuda.synchronize(dev)
        if ws > 1:
            torch.distributed.barrier()

    set_timing(True)
    for _ in range(args.warmup):
        plan.execute(x, y, wsb, stream)
    barrier()
    k1_ms = []
    scan_ms = []
    t_a = time.perf_counter()
    for _ in range(args.steps):
        plan.execute(x, y, wsb, stream)
        a, b = plan.last_timing_ms()  # syncs on this step's events
        k1_ms.append(a)
        scan_ms.append(b)
    barrier()
    el = time.perf_counter() - t_a
    set_timing(False)
    k1_kernel = plan.last_kernel()
    if ws > 1:
        tt = torch.tensor([el], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        el = float(tt.item())

    R = int(round(args.fs * args.dt_out))
    samples = n_ch * n * ws
    value = samples * args.steps / el
    k1 = float(np.mean(k1_ms))
    alg_bytes = n_ch * n * (4.0 + 4.0 / R)
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
        # ends with all n_ch * ws channels
        from lfdas.shard import all_gather_channels
        try:
            g_ms = []
            for i in range(4):
                barrier()
                t_g = time.perf_counter()
                full = all_gather_channels(y, n_ch * ws)
                torch.cuda.synchronize(dev)
                if i:
                    g_ms.append((time.perf_counter() - t_g) * 1e3)
            del full
            tt = torch.tensor([float(np.median(g_ms))], device=dev, dtype=torch.float64)
            torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
            secondary["allgather_outputs"] = {
                "ms": float(tt.item()), "bytes_per_rank": int(y.numel() * 4),
                "frac_of_step": float(tt.item()) / (el / args.steps * 1e3),
                "note": "RCCL all_gather of every rank's (n_ch, n_grid) float32 outputs; not in the timed step"}
        except Exception as e:  # the optional gather never voids the bench line
            secondary["allgather_outputs"] = {"error": repr(e)}
    if ws == 1:
        del x, y, wsb
        plan.close()
        torch.cuda.empty_cache()
    if not args.no_rolling and ws == 1:
        from lfdas.plan import rolling_mean_device
        xr = torch.empty((5000, 600_000), dtype=torch.float32, device=dev)
        synth_fill(xr, 1000.0, 99)
        for _ in range(2):
            rolling_mean_device(xr, 1000, 1000)
        torch.cuda.synchronize(dev)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        reps = 10
        for _ in range(reps):
            rolling_mean_device(xr, 1000, 1000)
        e1.record()
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1) / reps
        gbs = 5000 * 600_000 * (4 + 4 / 1000) / (ms * 1e-3) / 1e9
        secondary["rolling_mean_cfg2"] = {
            "value": 5000 * 600_000 / (ms * 1e-3), "unit": "channel-samples/s", "ms": ms,
            "config": "5,000 ch x 10 min @ 1 kHz fp32, W = S = 1000",
            "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": gbs / HBM_PEAK_GBS}}
        del xr
        torch.cuda.empty_cache()
    if not args.no_stream and ws == 1:
        secondary["edge_latency_cfg4"] = bench_edge_cfg4(dev)
        secondary["edge_latency_cfg4_time_major"] = bench_edge_cfg4(dev, time_major=True)
        torch.cuda.empty_cache()
        secondary["out_of_core_cfg5"] = bench_ooc_cfg5(dev)
        torch.cuda.empty_cache()


    if rank == 0:
        out = {
            "metric": "channel-samples/s low-pass+decimate",
            "value": value,
            "unit": "channel-samples/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": el / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (0.5 + sin + N(0,1), generated on device)",
            "config": {"workload": "cfg3: 10,000 ch x 1 h @ 500 Hz fp32 (72 GB) per GPU, 4th-order "
                                   "Butterworth 0.45 Hz zero-phase, decimate to 1 Hz, LFProc P=600 B=7",
                       "channels_per_gpu": n_ch, "samples": n, "fs": args.fs, "dt_out": args.dt_out,
                       "chunks": len(sched), "outputs_per_channel": int(sum(b - a for _, _, a, b in sched)),
                       "parallelism": f"channel-shard x{ws}", "io_dtype": "f32"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": {"mfma_runs": "k_block_runs_mfma", "mfma": "k_block_functionals_mfma"}
                                   .get(k1_kernel, "k_block_functionals_lds"), "kernel_ms": k1,
                         "scan_kernel_ms": float(np.mean(scan_ms))},
            "cpu_baseline": cpu,
            "secondary": secondary,
        }
        print(json.dumps(out))
    if ws > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
