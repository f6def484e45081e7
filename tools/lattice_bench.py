"""Lattice (composite) plan vs the per-chunk general path on a 3 kHz record
with integer-ns sample times (varying interpolation fraction, spacing 3,000
or 3,001 samples): 2,000 ch x 30 min, dt = 1 s, P = 600, B = 7."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("LFDAS_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "low-freq-real-time_amd", "lfdas", "liblfdas_diag.so"))  # A/B knobs: diagnostic build only
sys.path.insert(0, os.path.join(ROOT, "low-freq-real-time_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from lfdas.design import default_padlen  # noqa: E402
from lfdas.plan import filtfilt_resample_device  # noqa: E402

n_ch, fs, secs = 2000, 3000.0, 1800.0
n = int(secs * fs)
plan, sched, sos, t0, dt_ns, tg = bench.build_plan(n_ch, n, fs, 1.0, 600, 7)
dev = torch.device("cuda", 0)
x = torch.empty((n_ch, n), dtype=torch.float32, device=dev)
bench.synth_fill(x, fs, 5)
y = torch.empty((n_ch, plan.n_grid), dtype=torch.float32, device=dev)
wsb = plan.alloc_workspace(dev)
st = torch.cuda.current_stream(dev)
el, k1, _ = bench.time_plan(plan, x, y, wsb, st, 5, 1)
print(f"lattice plan ({plan.last_kernel()}): {el / 5 * 1e3:.2f} ms per pass, "
      f"{n_ch * n / (el / 5) / 1e9:.1f} G ch-samples/s", flush=True)
from lfdas import schedule as S  # noqa: E402
lo, w = S.grid_positions(t0, dt_ns, tg)
chunks = [(*S.select_range(t0, dt_ns, n, tg[a], tg[b]), oa, ob) for a, b, oa, ob in sched]
padlen = default_padlen(sos)
os.environ["LFD_NO_LATTICE"] = "1"
y2 = torch.empty_like(y)
for rep in range(2):
    torch.cuda.synchronize()
    ta = time.perf_counter()
    for s0, s1, oa, ob in chunks:
        y2[:, oa:ob] = filtfilt_resample_device(x[:, s0:s1 + 1], sos, lo[oa:ob] - s0, w[oa:ob], padlen)
    torch.cuda.synchronize()
    tb = time.perf_counter()
print(f"per-chunk general path (full-rate + interp): {(tb - ta) * 1e3:.2f} ms per pass", flush=True)
g0, g1 = chunks[0][2], chunks[-1][3]
a_, b_ = y[:, g0:g1].double(), y2[:, g0:g1].double()
print(f"relRMS lattice vs general: {float(torch.sqrt(((a_ - b_) ** 2).sum() / (b_ ** 2).sum())):.2e}")
