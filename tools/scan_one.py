"""The 1,250-channel shard of cfg3 (one rank of 8): a few executes of its
plan (rocprofv3 driver for the scan kernels' durations)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "low-freq-real-time_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

nc = int(sys.argv[1]) if len(sys.argv) > 1 else 1250
plan, *_ = bench.build_plan(nc, 1_800_000, 500.0, 1.0, 600, 7)
x = torch.empty((nc, 1_800_000), dtype=torch.float32, device="cuda")
bench.synth_fill(x, 500.0, 1)
y = torch.empty((nc, plan.n_grid), dtype=torch.float32, device="cuda")
ws = plan.alloc_workspace()
for _ in range(5):
    plan.execute(x, y, ws)
torch.cuda.synchronize()
print("done", flush=True)
