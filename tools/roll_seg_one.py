"""The bench's cfg2 rolling-mean line with W = 1000, S = 250 alone
(k_rolling_seg), for rocprofv3 PMC passes (tools/pmc_kernel.sh)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

print(json.dumps(bench.bench_rolling(torch.device("cuda", 0), 1000, 250, reps=3)), flush=True)
