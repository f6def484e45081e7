"""Kernel times of the blocked full-rate path over a few shapes (probe)."""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "low-freq-real-time_amd"))
import torch  # noqa: E402

import oracle  # noqa: E402
from lfdas.plan import load, set_timing, sosfiltfilt_device, sosfiltfilt_last_timing_ms  # noqa: E402

sos = oracle.dascore_pass_filter_sos(1000.0, 1.0, 10.0)
for n_ch, n in [(2000, 2049), (2000, 4095), (2000, 292 * 2048 + 1), (2000, 600_000), (8000, 600_000 // 4)]:
    x = torch.randn((n_ch, n), device="cuda", dtype=torch.float32)
    y = torch.empty((n_ch, n), dtype=torch.float64, device="cuda")
    ws = torch.empty(int(load().lfd_sosfiltfilt_workspace_bytes(n_ch, n, -1, 4)), dtype=torch.uint8, device="cuda")
    sosfiltfilt_device(x, sos, y=y, ws=ws)
    set_timing(True)
    t = []
    for _ in range(3):
        sosfiltfilt_device(x, sos, y=y, ws=ws)
        t.append(sosfiltfilt_last_timing_ms())
    set_timing(False)
    print(n_ch, n, "nb", (n - 1) // 2048, "tail", n - (n - 1) // 2048 * 2048, "ms", np.round(np.mean(t, axis=0), 3), flush=True)
