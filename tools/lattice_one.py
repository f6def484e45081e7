"""The bench's lattice workload (2,000 ch x 30 min @ 3 kHz on integer-ns
times, dt = 1 s, P = 600, B = 7), a few executes of its one-pass plan
(PMC / rocprofv3 driver)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "low-freq-real-time_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

n_ch, fs = 2000, 3000.0
n = int(1800.0 * fs)
plan, *_ = bench.build_plan(n_ch, n, fs, 1.0, 600, 7)
x = torch.empty((n_ch, n), dtype=torch.float32, device="cuda")
bench.synth_fill(x, fs, 5)
y = torch.empty((n_ch, plan.n_grid), dtype=torch.float32, device="cuda")
ws = plan.alloc_workspace()
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    plan.execute(x, y, ws)
torch.cuda.synchronize()
print("done", plan.lattice()[:2], flush=True)
