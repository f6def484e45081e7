"""K1 whole-line loads A/B (diagnostic build): the same cfg3 plan built with
LFD_K1_LINES=0 (16 rows x 64 B per wave instruction) and =1 (8 rows x 128 B +
DPP exchange), executed alternately in one process at full width and at the
8-GPU shard width; K1 HIP-event times and the outputs' agreement.
Usage (GPU box): python tools/k1_lines_ab.py [rounds]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("LFDAS_LIB", os.path.join(ROOT, "low-freq-real-time_amd", "lfdas", "liblfdas_diag.so"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "low-freq-real-time_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from lfdas.plan import set_timing  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev)
set_timing(True)
for n_ch in (10_000, 1_250):
    n = 1_800_000
    plans = {}
    for lines in (0, 1):
        os.environ["LFD_K1_LINES"] = str(lines)
        plans[lines] = bench.build_plan(n_ch, n, 500.0, 1.0, 600, 7)[0]
    os.environ.pop("LFD_K1_LINES")
    x = bench.device_samples((n_ch, n), device=dev)
    bench.synth_fill(x, 500.0, 1234)
    ys = {k: torch.empty((n_ch, p.n_grid), dtype=torch.float64, device=dev) for k, p in plans.items()}
    wsb = plans[0].alloc_workspace(dev)
    ms = {0: [], 1: []}
    for r in range(rounds + 1):
        for k in (0, 1):
            for _ in range(3):
                plans[k].execute(x, ys[k], wsb, st)
                torch.cuda.synchronize(dev)
                if r:
                    ms[k].append(plans[k].last_timing_ms()[0])
    a, b = ys[0].cpu().numpy(), ys[1].cpu().numpy()
    # (outputs outside the chunks' ranges are never written: compare the produced ones)
    _, sched0, *_ = bench.build_plan(n_ch, n, 500.0, 1.0, 600, 7)
    f = np.zeros(a.shape, bool)
    for _, _, oa, ob in sched0:
        f[:, oa:ob] = True
    rel = float(np.sqrt(np.sum((a[f] - b[f]) ** 2) / np.sum(a[f] ** 2)))
    alg = n_ch * n * (4.0 + 8.0 / 500)
    for k in (0, 1):
        m = float(np.median(ms[k]))
        print(f"n_ch {n_ch:6d} lines={k} ({plans[k].last_kernel()}): K1 median {m:.3f} ms "
              f"(min {min(ms[k]):.3f}) = {alg / (m * 1e-3) / 8e12:.3f} of 8 TB/s")
    print(f"n_ch {n_ch:6d} produced outputs lines=1 vs lines=0: relRMS {rel:.2e}, NaN footprint equal "
          f"{bool(np.array_equal(np.isnan(a[f]), np.isnan(b[f])))}")
    # which is right: sampled channels against the oracle
    import oracle
    rows = [0, 1, 7, 8, 9, 15, 16, n_ch - 1]
    plan0, sched, sos, t0, dt_ns, tg = bench.build_plan(n_ch, n, 500.0, 1.0, 600, 7)
    plan0.close()
    ref = oracle.lfproc_process(x[rows].cpu().numpy(), t0, dt_ns, tg[0], tg[-1] + 1, 1.0, 600, 7)
    want = np.concatenate([r for _, r in ref], axis=1)
    for k, yy in ((0, a), (1, b)):
        got = np.concatenate([yy[rows][:, oa:ob] for _, _, oa, ob in sched], axis=1)
        per = [float(np.sqrt(np.sum((got[i] - want[i]) ** 2) / np.sum(want[i] ** 2))) for i in range(len(rows))]
        print(f"  lines={k} vs oracle per row {rows}: " + " ".join(f"{v:.1e}" for v in per))
    d = np.abs(a - b)
    d[~f] = 0
    ch, j = np.unravel_index(np.argmax(d), d.shape)
    print(f"  max |diff| {d.max():.3e} at channel {ch}, output {j}; channels with diff > 1e-9: "
          f"{int(np.sum(d.max(axis=1) > 1e-9))}, outputs: {np.nonzero(d.max(axis=0) > 1e-9)[0][:20]}")
    for p in plans.values():
        p.close()
    del x, ys, wsb
    torch.cuda.empty_cache()
