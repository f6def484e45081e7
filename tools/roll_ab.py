"""cfg2 rolling mean (5,000 ch x 10 min @ 1 kHz): the segment prefix-sum
kernel (k_rolling_seg) against the running-sum scan (LFD_ROLL_SEGSUM=0) at
1 < S < W, same input allocation, alternating."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402

dev = torch.device("cuda", 0)
for rep in range(2):
    for W, S_ in [(1000, 250), (1000, 200), (1000, 500), (1000, 100)]:
        for seg in ("1", "0"):
            os.environ["LFD_ROLL_SEGSUM"] = seg
            r = bench.bench_rolling(dev, W, S_, reps=5)
            print(f"W={W} S={S_} segsum={seg} {r['ms']:.3f} ms frac {r['roofline']['frac']:.3f}", flush=True)
