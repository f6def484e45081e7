"""Timing of the device FIR decimation (Patch.decimate(filter_type='fir')
kernel) on a 2,000 x 600,000 float32 record: HIP-event time, HBM rate of the
algorithmic bytes (4 B read + 8/q B written per sample)."""
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
from lfdas._lib import load  # noqa: E402

n_ch, n = 2000, 600_000
x = torch.empty((n_ch, n), dtype=torch.float32, device="cuda")
bench.synth_fill(x, 1000.0, 5)
for q in (2, 5, 10, 50):
    taps, delay = fir_decimate_design(q)
    fir_decimate_device(x, taps, q, delay)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        fir_decimate_device(x, taps, q, delay)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 5
    alg = n_ch * n * (4 + 8 / q)
    kern = "mfma" if load().lfd_fir_decimate_last_kernel() == 1 else "valu"
    print(f"{kern} q={q:3d} taps={taps.size:5d} {ms:.3f} ms  {alg / ms / 1e6:.0f} GB/s  frac {alg / ms / 1e6 / 8000:.3f}  "
          f"{n_ch * n * taps.size / q / ms / 1e9:.1f} TFMA/s", flush=True)
