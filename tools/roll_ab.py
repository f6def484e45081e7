"""cfg2 rolling mean (5,000 ch x 10 min @ 1 kHz) A/B of diagnostic-build
knobs on one input allocation, alternating:

    python tools/roll_ab.py W S "SPEC" "SPEC" ...     (SPEC: NAME=VALUE ..., "" = defaults)

e.g. the segment prefix-sum kernel against the running-sum scan
(``1000 250 "" "LFD_ROLL_SEGSUM=0"``, profiles/archive_r01_r03.md (r03_ab_roll_segsum.txt)) or the
scan's LDS ring / DPP steps (``1000 1 "" "LFD_ROLL_RING=0" "LFD_ROLL_DPP=0"``,
profiles/archive_r01_r03.md (r02_ab_roll_ring.txt)).  Loads liblfdas_diag.so (the product library
reads no environment); every variant's output is compared with the first
spec's after a NaN fill."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("LFDAS_LIB", os.path.join(ROOT, "low-freq-real-time_amd", "lfdas", "liblfdas_diag.so"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "low-freq-real-time_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from lfdas.plan import rolling_mean_device  # noqa: E402

W, S_ = int(sys.argv[1]), int(sys.argv[2])
specs = sys.argv[3:] or [""]
keys = sorted({kv.split("=", 1)[0] for s in specs for kv in s.split()})
dev = torch.device("cuda", 0)
x = torch.empty((5000, 600_000), dtype=torch.float32, device=dev)
bench.synth_fill(x, 1000.0, 99)
ref = None
ms = {s: [] for s in specs}
for rep in range(3):
    for s in specs:
        for k in keys:
            os.environ.pop(k, None)
        for kv in s.split():
            k, v = kv.split("=", 1)
            os.environ[k] = v
        y = rolling_mean_device(x, W, S_)
        y.fill_(float("nan"))
        y = rolling_mean_device(x, W, S_)
        torch.cuda.synchronize()
        if ref is None:
            ref = y.clone()
        elif rep == 0:
            same = bool(torch.equal(torch.nan_to_num(y, 7.0), torch.nan_to_num(ref, 7.0)))
            print(f"[{s}] bit-identical to [{specs[0]}]: {same}", flush=True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            rolling_mean_device(x, W, S_)
        e1.record()
        torch.cuda.synchronize()
        ms[s].append(e0.elapsed_time(e1) / 5)
alg = 5000 * 600_000 * (4 + 4 / S_)
for s in specs:
    m = float(np.median(ms[s]))
    print(f"W={W} S={S_} [{s:28s}] {m:.3f} ms  frac {alg / (m * 1e-3) / 8e12:.3f}", flush=True)
