"""One full-rate band-pass shape, a few calls (PMC / rocprofv3 driver)."""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
os.environ.setdefault("LFDAS_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "low-freq-real-time_amd", "lfdas", "liblfdas_diag.so"))  # A/B knobs: diagnostic build only
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "low-freq-real-time_amd"))
import torch  # noqa: E402

import oracle  # noqa: E402
from lfdas.plan import load, sosfiltfilt_device  # noqa: E402

n_ch, n = 2000, 600_000
sos = oracle.dascore_pass_filter_sos(1000.0, 1.0, 10.0)
x = torch.randn((n_ch, n), device="cuda", dtype=torch.float32)
y = torch.empty((n_ch, n), dtype=torch.float64, device="cuda")
ws = torch.empty(int(load().lfd_sosfiltfilt_workspace_bytes(n_ch, n, -1, 4)), dtype=torch.uint8, device="cuda")
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    sosfiltfilt_device(x, sos, y=y, ws=ws)
torch.cuda.synchronize()
print("done", flush=True)
