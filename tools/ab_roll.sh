# A/B of the rolling-mean kernel (cfg2: 5,000 ch x 600,000, W = S = 1000) across library variants
set -e -o pipefail
for rep in 1 2 3; do
  for v in "$@"; do
    LFDAS_LIB=$PWD/build/variants/lib_$v.so timeout -k 10 120 python - <<'PY'
import os, sys, torch
sys.path.insert(0, "low-freq-real-time_amd"); sys.path.insert(0, ".")
import bench
from lfdas.plan import rolling_mean_device
x = torch.empty((5000, 600_000), dtype=torch.float32, device="cuda")
bench.synth_fill(x, 1000.0, 99)
for _ in range(3): rolling_mean_device(x, 1000, 1000)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20): rolling_mean_device(x, 1000, 1000)
e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 20
print(os.path.basename(os.environ["LFDAS_LIB"]), round(ms, 3), "ms", round(5000 * 600000 * 4.004 / ms / 1e9 / 8000 * 1e3, 3), "frac")
PY
  done
done
