"""A/B timings of the time-major K1 variants and the rolling-scan staging
modes (run on the GPU box; knobs read per launch from the environment)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402

dev = torch.device("cuda", 0)
specs = sys.argv[1:] or ["LFD_TM_X2=1", "LFD_TM_X2=0", "LFD_TM_X2=1 LFD_TM_PF=3", "LFD_TM_X2=1 LFD_TM_PF=1"]
for rep in range(2):
    for spec in specs:
        for k in ("LFD_TM_NT", "LFD_TM_PF", "LFD_TM_SWAP", "LFD_TM_NTILE", "LFD_TM_X2"):
            os.environ.pop(k, None)
        for kv in spec.split():
            k, v = kv.split("=", 1)
            os.environ[k] = v
        r = bench.bench_lowpass_line(dev, 10_000, 500.0, 3600.0, 1.0, 600, 7, time_major=True, label="tm")
        print("TM", spec, r["k1"], round(r["roofline"]["kernel_ms"], 3), round(r["roofline"]["frac"], 3),
              round(r["ms_per_step"], 3), flush=True)
for st in ():
    os.environ["LFD_ROLL_STAGE"] = st
    for W, S_ in [(1000, 1), (1000, 250)]:
        q = bench.bench_rolling(dev, W, S_, reps=5)
        print("roll stage", st, W, S_, round(q["ms"], 3), round(q["roofline"]["frac"], 3), flush=True)
