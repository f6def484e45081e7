"""In-process A/B of the rolling-mean scan kernel's env knobs on cfg2
(5,000 ch x 600,000 @ 1 kHz, W = 1000), step S (default 1).

    python tools/ab_roll_env.py [S] "LFD_ROLL_PF=1" "LFD_ROLL_PF=2" ...

Each spec is a space-separated list of NAME=VALUE; the specs are timed in
alternation (3 rounds x 5 calls each) and their outputs compared bit for bit
with the first spec's."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "low-freq-real-time_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from lfdas.plan import rolling_mean_device  # noqa: E402

args = sys.argv[1:]
S = int(args.pop(0)) if args and args[0].isdigit() else 1
specs = args or ["LFD_ROLL_PF=1"]
W = 1000
n_ch, n_t = 5000, 600_000
x = torch.empty((n_ch, n_t), dtype=torch.float32, device="cuda")
bench.synth_fill(x, 1000.0, 99)
alg = n_ch * n_t * (4 + 4 / S)


def apply(spec):
    for kv in spec.split():
        k, v = kv.split("=", 1)
        os.environ[k] = v


ref = None
times = {s: [] for s in specs}
for rnd in range(3):
    for s in specs:
        apply(s)
        y = rolling_mean_device(x, W, S)
        torch.cuda.synchronize()
        if ref is None:
            ref = y.clone()
        elif rnd == 0:
            same = torch.equal(torch.nan_to_num(y, 7.0), torch.nan_to_num(ref, 7.0))
            print(f"{s}: outputs {'identical' if same else 'DIFFER'}", flush=True)
        del y
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            rolling_mean_device(x, W, S)
        e1.record()
        torch.cuda.synchronize()
        times[s].append(e0.elapsed_time(e1) / 5)
for s in specs:
    ms = min(times[s])
    print(f"S={S} {s:40s} " + " ".join(f"{t:.3f}" for t in times[s]) +
          f"  best {ms:.3f} ms  frac {alg / (ms * 1e-3) / 8e12:.3f}", flush=True)
