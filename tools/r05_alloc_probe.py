"""Narrow-shard K1 time by the input allocation's size / alignment: the
1,250-channel cfg3 shard (9 GB) run on the first rows of torch allocations
of several sizes (translation misses, profiles/r05_narrow_tlb.txt)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "low-freq-real-time_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from lfdas.plan import set_timing  # noqa: E402

ch, n = int(sys.argv[1]) if len(sys.argv) > 1 else 1250, 1_800_000
plan, *_ = bench.build_plan(ch, n, 500.0, 1.0, 600, 7)
dev = torch.device("cuda", 0)
y = torch.empty((ch, plan.n_grid), dtype=torch.float32, device=dev)
wsb = plan.alloc_workspace(dev)
st = torch.cuda.current_stream(dev)
set_timing(True)
GB = 1 << 30
row = n * 4
for label, extra_gb, align in [("own", 0, 0), ("own", 0, 0), ("+7GB", 7, 0), ("+9GB", 9, 0), ("+15GB", 15, 0),
                               ("+27GB", 27, 0), ("+1GB aligned1G", 1, GB), ("+2GB aligned2M", 1, 2 << 20),
                               ("own", 0, 0), ("+27GB", 27, 0)]:
    nbytes = ch * row + extra_gb * GB
    buf = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
    base = buf.data_ptr()
    off = 0
    if align:
        off = ((base + align - 1) // align * align - base) // 4
    x = buf[off:off + ch * n].view(ch, n)
    bench.synth_fill(x, 500.0, 77)
    ts = []
    for _ in range(6):
        plan.execute(x, y, wsb, st)
        ts.append(plan.last_timing_ms()[0])
    k1 = float(np.median(ts[1:]))
    frac = ch * n * 4.008 / (k1 * 1e-3) / 8e12
    print(f"{label:18s} alloc {nbytes / GB:6.1f} GB base%1G {base % GB:>11d} base%2M {base % (2 << 20):>8d} "
          f"slice%1G {(base + 4 * off) % GB:>11d}  K1 {k1:.3f} ms  frac {frac:.3f}", flush=True)
    del x, buf
    torch.cuda.empty_cache()
