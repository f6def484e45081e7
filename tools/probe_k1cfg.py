"""K1 launch configurations compared inside one process (diagnostic).

Env knobs are read per launch, so configurations alternate within a process
and share its memory mode. Usage (GPU box):
python tools/probe_k1cfg.py
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

# (the default registers are capped for 4 waves per SIMD at depth 1; the
# other depths run with the compiler's allocation, LFD_RUN_MINW=0)
CFGS = {
    "base": {},
    "pf2nt512": {"LFD_RUN_PF": "2", "LFD_RUN_NT": "512", "LFD_RUN_MINW": "0"},
    "pf3nt512": {"LFD_RUN_PF": "3", "LFD_RUN_NT": "512", "LFD_RUN_MINW": "0"},
    "pf4nt512": {"LFD_RUN_PF": "4", "LFD_RUN_NT": "512", "LFD_RUN_MINW": "0"},
}
KNOBS = ("LFD_RUN_NT", "LFD_RUN_PF", "LFD_RUN_MINW")

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
    for name, env in CFGS.items():
        for kk in KNOBS:
            os.environ.pop(kk, None)
        os.environ.update(env)
        plan.execute(x, y, wsb, st)
        torch.cuda.synchronize()
        if ref is None:
            ref = y.clone()
        same = bool(torch.equal(y, ref))
        k = []
        for _ in range(5):
            plan.execute(x, y, wsb, st)
            k.append(plan.last_timing_ms()[0])
        print(f"rep {rep} {name:10s} {plan.last_kernel()} K1 {np.mean(k):.3f} "
              f"(min {np.min(k):.3f} max {np.max(k):.3f}) bit-identical {same}", flush=True)
