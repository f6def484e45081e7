"""K1 time vs the base address of the cfg3 sample array (diagnostic).

One 72 GB buffer plus slack; x is a (10,000 x 1.8 M) view at several byte
offsets, each timed over a few steps. Prints offset, data_ptr mod 2 MB and the
mean K1 / scan ms. Usage (GPU box): python tools/probe_align.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "low-freq-real-time_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from lfdas.plan import set_timing  # noqa: E402

n_ch, n = 10000, 1_800_000
plan, *_ = bench.build_plan(n_ch, n, 500.0, 1.0, 600, 7)
dev = torch.device("cuda", 0)
slack = 4 << 20
raw = torch.empty(n_ch * n + slack // 4, dtype=torch.float32, device=dev)
y = torch.empty((n_ch, plan.n_grid), dtype=torch.float32, device=dev)
wsb = plan.alloc_workspace(dev)
st = torch.cuda.current_stream(dev)
print("raw ptr mod 2MB:", raw.data_ptr() % (2 << 20), flush=True)
set_timing(True)
for rep in range(2):
    for off in (0, 256, 4096, 65536, 1 << 20, 2 << 20, 3 << 20):
        x = raw[off // 4: off // 4 + n_ch * n].view(n_ch, n)
        if rep == 0:
            bench.synth_fill(x, 500.0, 1234)
        plan.execute(x, y, wsb, st)
        k, s = [], []
        for _ in range(5):
            plan.execute(x, y, wsb, st)
            a, b = plan.last_timing_ms()
            k.append(a)
            s.append(b)
        print(f"rep {rep} off {off:8d} ptr%2MB {x.data_ptr() % (2 << 20):8d} K1 {np.mean(k):.3f} "
              f"(min {np.min(k):.3f} max {np.max(k):.3f}) scan {np.mean(s):.3f}", flush=True)
