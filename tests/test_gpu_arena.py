"""lfdas.arena.device_samples: sample buffers of >= 1 GiB live in a >= 32 GiB
allocation (the translation-friendly placement measured in
profiles/r05_alloc_placement.txt); results are those of any other buffer."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_device_samples_pool_view_and_parity():
    import torch
    from lfdas import arena
    from lfdas import schedule as S
    from lfdas.design import lowpass_sos
    from lfdas.plan import LowpassPlan
    small = arena.device_samples((4, 1000))
    assert small.is_contiguous() and small.shape == (4, 1000)
    assert small.untyped_storage().nbytes() < arena.MIN_BYTES
    n_ch, n = 300, 1_000_000  # 1.2 GB: pooled
    x = arena.device_samples((n_ch, n))
    assert x.shape == (n_ch, n) and x.dtype == torch.float32 and x.is_contiguous()
    free, _ = torch.cuda.mem_get_info()
    if free > 2 * arena.POOL_BYTES:
        assert x.untyped_storage().nbytes() >= arena.POOL_BYTES
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    torch.randn(x.shape, generator=g, device="cuda", out=x)
    x += 2.0
    xc = torch.empty_like(x).copy_(x)
    fs, dt_out, P, B = 500.0, 1.0, 600, 7
    t0, dt_ns = 1_505_692_800_000_000_000, 2_000_000
    tg = S.time_grid(t0, t0 + n * dt_ns, dt_out)
    sched = S.lfproc_chunks(len(tg), P, B)
    lo, w = S.grid_positions(t0, dt_ns, tg)
    chunks = [(*S.select_range(t0, dt_ns, n, tg[a], tg[b]), oa, ob) for a, b, oa, ob in sched]
    plan = LowpassPlan(lowpass_sos(fs, 0.45), n_ch, n, lo, w, chunks)
    ws = plan.alloc_workspace()
    ya = torch.full((n_ch, len(tg)), float("nan"), dtype=torch.float64, device="cuda")
    yb = torch.full_like(ya, float("nan"))
    plan.execute(x, ya, ws)
    plan.execute(xc, yb, ws)
    torch.cuda.synchronize()
    assert torch.equal(torch.nan_to_num(ya, 7.0), torch.nan_to_num(yb, 7.0))
    plan.close()
