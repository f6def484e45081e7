"""Scan-kernel phase times (LFD_SCAN_DIAG bits; results invalid when set) for
cfg3-sized plans: aligned, off-sample (1.9 ms), 1 kHz dt = 10 s, and the
1,250-channel shard of cfg3 ("narrow", deferred outputs)."""
import os
import subprocess
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
os.environ.setdefault("LFDAS_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "low-freq-real-time_amd", "lfdas", "liblfdas_diag.so"))  # A/B knobs: diagnostic build only

CHILD = r'''
import os, sys, numpy as np
sys.path.insert(0, %r); sys.path.insert(0, os.path.join(%r, "low-freq-real-time_amd"))
import torch, bench
from lfdas.plan import set_timing
cfg = sys.argv[1]
nc = 1250 if cfg == "narrow" else 10000
if cfg == "narrow":
    plan, *_ = bench.build_plan(nc, 1_800_000, 500.0, 1.0, 600, 7)
    n = 1_800_000
elif cfg == "offsample":
    plan, *_ = bench.build_plan(10000, 1_800_000, 500.0, 1.0, 600, 7, off_ns=1_900_000)
    n = 1_800_000
elif cfg == "dt10":
    plan, *_ = bench.build_plan(10000, 3_600_000, 1000.0, 10.0, 120, 6)
    n = 3_600_000
else:
    plan, *_ = bench.build_plan(10000, 1_800_000, 500.0, 1.0, 600, 7)
    n = 1_800_000
x = torch.empty((nc, n), dtype=torch.float32, device="cuda")
bench.synth_fill(x, 500.0, 1)
y = torch.empty((nc, plan.n_grid), dtype=torch.float32, device="cuda")
ws = plan.alloc_workspace()
set_timing(True)
t = []
for _ in range(4):
    plan.execute(x, y, ws)
    t.append(plan.last_timing_ms()[1])
print(cfg, os.environ.get("LFD_SCAN_DIAG", "0"), "scan ms %%.3f" %% np.median(t[1:]), flush=True)
''' % (ROOT, ROOT)

for cfg in sys.argv[1:] or ["offsample"]:
    for diag in ["0", "1", "2", "4", "8", "15"]:
        env = dict(os.environ, LFD_SCAN_DIAG=diag)
        subprocess.run([sys.executable, "-c", CHILD, cfg], env=env, check=True, timeout=240)
