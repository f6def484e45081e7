"""One FIR decimation case for profiling (rocprofv3 --pmc): 2,000 x 600,000
float32, q from argv (default 10), a few launches."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("LFDAS_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "low-freq-real-time_amd", "lfdas", "liblfdas_diag.so"))  # A/B knobs: diagnostic build only
sys.path.insert(0, os.path.join(ROOT, "low-freq-real-time_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from lfdas.plan import fir_decimate_device  # noqa: E402
from lfdas.proc import fir_decimate_design  # noqa: E402

q = int(sys.argv[1]) if len(sys.argv) > 1 else 10
x = torch.empty((2000, 600_000), dtype=torch.float32, device="cuda")
bench.synth_fill(x, 1000.0, 5)
taps, delay = fir_decimate_design(q)
for _ in range(3):
    fir_decimate_device(x, taps, q, delay)
torch.cuda.synchronize()
