"""K1 unit order A/B inside one process (diagnostic).

K1 runs in one of two per-process modes, so orders are compared
within a process: LFD_K1_BAND = 0 (channel-group-major) against bands of 16..128
channel groups, alternating, on the cfg3 array. Usage (GPU box):
python tools/probe_band.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("LFDAS_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "low-freq-real-time_amd", "lfdas", "liblfdas_diag.so"))  # A/B knobs: diagnostic build only
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "low-freq-real-time_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from lfdas.plan import set_timing  # noqa: E402

n_ch, n = 10000, 1_800_000
plan, *_ = bench.build_plan(n_ch, n, 500.0, 1.0, 600, 7)
dev = torch.device("cuda", 0)
x = torch.empty((n_ch, n), dtype=torch.float32, device=dev)
bench.synth_fill(x, 500.0, 1234)
y = torch.empty((n_ch, plan.n_grid), dtype=torch.float32, device=dev)
wsb = plan.alloc_workspace(dev)
st = torch.cuda.current_stream(dev)
set_timing(True)
ref = None
for rep in range(3):
    for band in (0, 8, 32, 128, 0):
        os.environ["LFD_K1_BAND"] = str(band)
        plan.execute(x, y, wsb, st)
        torch.cuda.synchronize()
        if ref is None:
            ref = y.clone()
        same = bool(torch.equal(y, ref))
        k = []
        for _ in range(5):
            plan.execute(x, y, wsb, st)
            k.append(plan.last_timing_ms()[0])
        print(f"rep {rep} band {band:4d} K1 {np.mean(k):.3f} (min {np.min(k):.3f} max {np.max(k):.3f}) "
              f"bit-identical {same}", flush=True)
