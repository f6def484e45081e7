"""A/B timings of the time-major K1 variants and the rolling-scan staging
modes (run on the GPU box; knobs read per launch from the environment)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402

dev = torch.device("cuda", 0)
for nt, pf, sw, ntl in [("512", "2", "0", "2"), ("512", "2", "0", "1"), ("512", "2", "0", "2"), ("512", "2", "0", "1")]:
    os.environ["LFD_TM_NT"], os.environ["LFD_TM_PF"], os.environ["LFD_TM_SWAP"] = nt, pf, sw
    os.environ["LFD_TM_NTILE"] = ntl
    r = bench.bench_lowpass_line(dev, 10_000, 500.0, 3600.0, 1.0, 600, 7, time_major=True, label="tm")
    print("TM", nt, pf, sw, ntl, r["k1"], round(r["roofline"]["kernel_ms"], 3), round(r["roofline"]["frac"], 3),
          round(r["ms_per_step"], 3), flush=True)
for st in ():
    os.environ["LFD_ROLL_STAGE"] = st
    for W, S_ in [(1000, 1), (1000, 250)]:
        q = bench.bench_rolling(dev, W, S_, reps=5)
        print("roll stage", st, W, S_, round(q["ms"], 3), round(q["roofline"]["frac"], 3), flush=True)
