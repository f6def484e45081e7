"""K1 time by input layout: the cfg3 plan (10,000 ch @ 500 Hz, dt = 1 s) over
a (channel, time) array and over a (time, channel) array viewed as
(channel, time) (DASCore dims ("time", "distance"), s_ch = 1).
    python tools/bench_layout.py [--seconds 720]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "low-freq-real-time_amd"))
import bench  # noqa: E402
from lfdas.plan import set_timing  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--seconds", type=float, default=720.0)
    p.add_argument("--channels", type=int, default=10_000)
    p.add_argument("--reps", type=int, default=5)
    a = p.parse_args()
    fs, n_ch = 500.0, a.channels
    n = int(a.seconds * fs)
    plan, sched, *_ = bench.build_plan(n_ch, n, fs, 1.0, 600, 7)
    dev = torch.device("cuda", 0)
    out = {"channels": n_ch, "samples": n}
    y = torch.empty((n_ch, plan.n_grid), dtype=torch.float32, device=dev)
    ref = None
    for layout in ("channel_major", "time_major"):
        if layout == "channel_major":
            x = torch.empty((n_ch, n), dtype=torch.float32, device=dev)
            bench.synth_fill(x, fs, 7)
            xv = x
        else:
            xc = torch.empty((n_ch, n), dtype=torch.float32, device=dev)
            bench.synth_fill(xc, fs, 7)
            x = xc.t().contiguous()
            del xc
            xv = x.t()
        wsb = plan.alloc_workspace(dev)
        st = torch.cuda.current_stream(dev)
        set_timing(True)
        plan.execute(xv, y, wsb, st)
        k1, sc = [], []
        for _ in range(a.reps):
            plan.execute(xv, y, wsb, st)
            t1, t2 = plan.last_timing_ms()
            k1.append(t1)
            sc.append(t2)
        set_timing(False)
        torch.cuda.synchronize(dev)
        yy = y.clone()
        if ref is None:
            ref = yy
            diff = 0.0
        else:
            diff = float(((yy - ref).norm() / ref.norm()).item())
        gbs = n_ch * n * (4 + 4 / 500) / (np.mean(k1) * 1e-3) / 1e9
        out[layout] = {"kernel": plan.last_kernel(), "k1_ms": float(np.mean(k1)),
                       "scan_ms": float(np.mean(sc)), "GBps": gbs, "rel_diff_vs_channel_major": diff}
        print(layout, out[layout], flush=True)
        del x, xv, wsb
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
