"""In-process A/B of low-pass plan env knobs on ONE input allocation.

K1's speed depends on the physical placement of the big input allocation
(DESIGN §6 "per-process modes": a fresh 72 GB tensor can run 5 % faster or
slower), so variants are compared on the same tensor, alternating.

    python tools/ab_plan.py [--tm] [--fs 500] [--seconds 3600] [--dt 1]
        [--ch 10000] [--off-ns 0] [--reps 4] "SPEC" "SPEC" ...

SPEC = space-separated NAME=VALUE env settings ("" = defaults). Outputs of
every spec are compared bit for bit with the first spec's (y is filled with
NaN before every compared execute, so a variant that writes nothing cannot
pass as identical).  The knobs exist only in the diagnostic build: this tool
loads liblfdas_diag.so (LFDAS_LIB), never the product library."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("LFDAS_LIB", os.path.join(ROOT, "low-freq-real-time_amd", "lfdas", "liblfdas_diag.so"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "low-freq-real-time_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from lfdas.plan import set_timing  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--tm", action="store_true", help="(time, channel) storage")
ap.add_argument("--fs", type=float, default=500.0)
ap.add_argument("--seconds", type=float, default=3600.0)
ap.add_argument("--dt", type=float, default=1.0)
ap.add_argument("--ch", type=int, default=10_000)
ap.add_argument("--P", type=int, default=600)
ap.add_argument("--B", type=int, default=7)
ap.add_argument("--off-ns", type=int, default=0)
ap.add_argument("--reps", type=int, default=4)
ap.add_argument("--steps", type=int, default=4)
ap.add_argument("--replan", action="store_true", help="rebuild the plan per spec (plan-time knobs)")
ap.add_argument("--pad", type=int, default=0, help="channel rows padded by this many samples (row stride)")
ap.add_argument("--alloc-ch", type=int, default=0,
                help="allocate this many channel rows and run the plan on the first --ch of them "
                     "(a narrow shard inside a wide allocation: placement vs width)")
ap.add_argument("--alloc-off", type=int, default=0, help="first channel row of the view (with --alloc-ch)")
ap.add_argument("specs", nargs="*")
a = ap.parse_args()
specs = a.specs or [""]
n = int(a.seconds * a.fs)
plan, *_ = bench.build_plan(a.ch, n, a.fs, a.dt, a.P, a.B, a.off_ns)
dev = torch.device("cuda", 0)
if a.tm:
    xs = torch.empty((n, a.ch), dtype=torch.float32, device=dev)
    bench.synth_fill_time_major(xs, a.fs, 77)
    x = xs.t()
else:
    xp = torch.empty((max(a.ch + a.alloc_off, a.alloc_ch), n + a.pad), dtype=torch.float32, device=dev)
    bench.synth_fill(xp, a.fs, 77)
    x = xp[a.alloc_off:a.alloc_off + a.ch, :n]
y = torch.empty((a.ch, plan.n_grid), dtype=torch.float64, device=dev)
wsb = plan.alloc_workspace(dev)
st = torch.cuda.current_stream(dev)
R = int(round(a.fs * a.dt))
alg = a.ch * n * (4.0 + 8.0 / R)
set_timing(True)
keys = sorted({kv.split("=", 1)[0] for s in specs for kv in s.split()})
ref = None
res = {s: ([], []) for s in specs}
for rep in range(a.reps):
    for s in specs:
        for k in keys:
            os.environ.pop(k, None)
        for kv in s.split():
            k, v = kv.split("=", 1)
            os.environ[k] = v
        if a.replan:
            plan.close()
            plan, *_ = bench.build_plan(a.ch, n, a.fs, a.dt, a.P, a.B, a.off_ns)
            del wsb
            wsb = plan.alloc_workspace(dev)
        y.fill_(float("nan"))
        plan.execute(x, y, wsb, st)
        torch.cuda.synchronize()
        if ref is None:
            ref = y.clone()
        elif rep == 0:
            same = bool(torch.equal(torch.nan_to_num(y, 7.0), torch.nan_to_num(ref, 7.0)))
            m = ~torch.isnan(ref)
            d = (y[m].double() - ref[m].double())
            rel = float(torch.sqrt(torch.sum(d * d) / torch.sum(ref[m].double() ** 2)))
            print(f"[{s}] {plan.last_kernel()} bit-identical to [{specs[0]}]: {same}  relRMS {rel:.2e}", flush=True)
        for _ in range(a.steps):
            plan.execute(x, y, wsb, st)
            k1, sc = plan.last_timing_ms()
            res[s][0].append(k1)
            res[s][1].append(sc)
for s in specs:
    k1, sc = np.array(res[s][0]), np.array(res[s][1])
    print(f"[{s:36s}] K1 median {np.median(k1):.3f} mean {k1.mean():.3f} min {k1.min():.3f} max {k1.max():.3f} ms  "
          f"frac {alg / (k1.mean() * 1e-3) / 8e12:.3f}  scan {sc.mean():.3f} ms", flush=True)
