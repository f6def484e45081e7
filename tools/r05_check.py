import sys
sys.path.insert(0, "low-freq-real-time_amd")
sys.path.insert(0, ".")
order = sys.argv[1]
import numpy as np
import bench
if order == "torch_first":
    import torch
    print("torch", torch.cuda.is_available(), flush=True)
plan, *_ = bench.build_plan(64, 500 * 400, 500.0, 1.0, 60, 7)
print("plan ok", flush=True)
import torch
print("torch", torch.cuda.is_available(), flush=True)
