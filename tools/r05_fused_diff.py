"""Every scan / K1 mode of a cfg1-geometry plan with a large DC against the
oracle: where do they differ (by output index)?"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "low-freq-real-time_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
from lfdas import schedule as S  # noqa: E402
from lfdas._lib import kernel_options  # noqa: E402
import test_gpu_lowpass as T  # noqa: E402

fs, dt_out, P, B, n_ch, n = 250.0, 0.2, 40, 6, 37, 6000
x = (np.random.default_rng(7).standard_normal((n_ch, n)) + 300.0).astype(np.float32)
plan, n_grid = T._plan_cfg(fs, dt_out, P, B, n_ch, n)
xd = torch.from_numpy(x).cuda()
ws = plan.alloc_workspace()
dt_ns = int(round(1e9 / fs))
tg = S.time_grid(T.T0, T.T0 + n * dt_ns, dt_out)
sched = S.lfproc_chunks(len(tg), P, B)
ref = oracle.lfproc_process(x, T.T0, dt_ns, tg[0], tg[-1] + 1, dt_out, P, B)
R = np.full((n_ch, n_grid), np.nan)
for (_, r), (_, _, oa, ob) in zip(ref, sched):
    R[:, oa:ob] = r
m = ~np.isnan(R)
modes = {"fused": {"scan_defer": 4}, "deferred": {"scan_defer": 2}, "inchain": {"scan_defer": 1},
         "noruns": {"no_runs": 1}, "rec": {"no_runs": 1, "k1_recurrence": 1}, "recfold": {"k1_recurrence": 1}}
for name, o in modes.items():
    yd = torch.full((n_ch, n_grid), float("nan"), dtype=torch.float32, device="cuda")
    with kernel_options(**o):
        plan.execute(xd, yd, ws)
    torch.cuda.synchronize()
    y = yd.cpu().numpy().astype(np.float64)
    d = np.abs(np.where(m, y - R, 0))
    rel = np.sqrt(np.sum(d ** 2) / np.sum(R[m] ** 2))
    bad = np.where(d.max(axis=0) > 3e-5)[0]
    print(f"{name:9s} {plan.last_kernel():16s} relRMS vs oracle {rel:.3e}  cols |d|>3e-5: {bad.tolist()[:20]}")
print("chunks", sched)
