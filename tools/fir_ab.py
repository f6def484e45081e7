"""A/B of diagnostic-build FIR-decimation knobs (k_fir_decimate_mfma) on one
2,000 x 600,000 float32 input, alternating specs in one process:

    python tools/fir_ab.py Q "SPEC" "SPEC" ...     (SPEC: NAME=VALUE ..., "" = defaults)

Each variant's output is compared with the first spec's (bit-identical
expected for scheduling-only variants)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("LFDAS_LIB", os.path.join(ROOT, "low-freq-real-time_amd", "lfdas", "liblfdas_diag.so"))
sys.path.insert(0, os.path.join(ROOT, "low-freq-real-time_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from lfdas.plan import fir_decimate_device  # noqa: E402
from lfdas.proc import fir_decimate_design  # noqa: E402

q = int(sys.argv[1])
specs = sys.argv[2:] or [""]
keys = sorted({kv.split("=", 1)[0] for s in specs for kv in s.split()})
n_ch, n = 2000, 600_000
x = torch.empty((n_ch, n), dtype=torch.float32, device="cuda")
bench.synth_fill(x, 1000.0, 5)
taps, delay = fir_decimate_design(q)
ref = None
ms = {s: [] for s in specs}
for rep in range(3):
    for s in specs:
        for k in keys:
            os.environ.pop(k, None)
        for kv in s.split():
            k, v = kv.split("=", 1)
            os.environ[k] = v
        y = fir_decimate_device(x, taps, q, delay)
        torch.cuda.synchronize()
        if ref is None:
            ref = y.clone()
        elif rep == 0:
            print(f"[{s}] bit-identical to [{specs[0]}]: {bool(torch.equal(y, ref))}", flush=True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            fir_decimate_device(x, taps, q, delay)
        e1.record()
        torch.cuda.synchronize()
        ms[s].append(e0.elapsed_time(e1) / 5)
alg = n_ch * n * (4 + 8 / q)
for s in specs:
    m = float(np.median(ms[s]))
    print(f"q={q} [{s:28s}] {m:.3f} ms  frac {alg / (m * 1e-3) / 8e12:.3f}", flush=True)
