"""Lattice plan on a 3 kHz record with integer-ns sample times (varying
interpolation fraction, spacing 3,000 or 3,001 samples): 2,000 ch x 30 min,
dt = 1 s, P = 600, B = 7.  The one-pass form (one K1 with every phase's
outputs) against the per-phase sub-plans (option lattice_phases), in one
process on the same input; outputs compared."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "low-freq-real-time_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from lfdas._lib import kernel_options  # noqa: E402

n_ch, fs, secs = 2000, 3000.0, 1800.0
n = int(secs * fs)
dev = torch.device("cuda", 0)
x = torch.empty((n_ch, n), dtype=torch.float32, device=dev)
bench.synth_fill(x, fs, 5)
st = torch.cuda.current_stream(dev)
ys = {}
for phases in (0, 1, 0):
    with kernel_options(lattice_phases=phases):
        plan, sched, sos, t0, dt_ns, tg = bench.build_plan(n_ch, n, fs, 1.0, 600, 7)
        y = torch.full((n_ch, plan.n_grid), float("nan"), dtype=torch.float32, device=dev)
        wsb = plan.alloc_workspace(dev)
        el, k1, sc = bench.time_plan(plan, x, y, wsb, st, 5, 1)
        n_off, onepass, _ = plan.lattice()
    name = "one-pass" if onepass else "per-phase"
    print(f"{name:9s} (offsets {n_off}, {plan.last_kernel()}): {el / 5 * 1e3:.2f} ms per pass, "
          f"K1 {sum(k1) / len(k1):.3f} ms, rest {sum(sc) / len(sc):.3f} ms, "
          f"{n_ch * n / (el / 5) / 1e9:.1f} G ch-samples/s, K1 frac "
          f"{n_ch * n * 4.0 / (sum(k1) / len(k1) * 1e-3) / 8e12:.3f}", flush=True)
    ys[name] = y
    plan.close()
    del wsb
a_, b_ = ys["one-pass"].double(), ys["per-phase"].double()
f = torch.isfinite(b_)
print(f"NaN footprints equal: {bool(torch.equal(torch.isfinite(a_), f))}")
print(f"relRMS one-pass vs per-phase: {float(torch.sqrt(((a_[f] - b_[f]) ** 2).sum() / (b_[f] ** 2).sum())):.2e}")
