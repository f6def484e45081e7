"""The bench's two cfg2 rolling-mean lines alone (W = S = 1000 and W = 1000,
S = 1), for rocprofv3 PMC passes on the rolling kernels (tools/profile.sh)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
for W, S_ in ((1000, 1000), (1000, 1)):
    print(json.dumps(bench.bench_rolling(dev, W, S_, reps=3)), flush=True)
