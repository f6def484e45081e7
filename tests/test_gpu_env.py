"""The product library's results cannot depend on the environment.

Rounds 1-3 kept A/B knobs and "timing only, results invalid" kernel modes
behind LFD_* environment variables inside liblfdas.so.  They now exist only
in liblfdas_diag.so (-DLFD_DIAG, loaded by tools/ through LFDAS_LIB); the
product reads no environment variable.  This test sets every knob a previous
round's library honoured — the five invalidating diagnostics included — and
checks the cfg1 plan (both layouts), the rolling mean, the full-rate filter
and the FIR decimation against the oracle (relRMS gates.MFMA / 1e-6 / 1e-10 / 1e-9)."""
import numpy as np
import pytest

import gates
import oracle
from lfdas import schedule as S

pytestmark = pytest.mark.gpu

KNOBS = {
    # "results invalid" diagnostics of rounds 1-3
    "LFD_TM_MODE": "3", "LFD_MF_MODE": "3", "LFD_RUN_MODE": "1", "LFD_SCAN_DIAG": "15", "LFD_FIR_DIAG": "2",
    # measured-and-rejected variants / tuning knobs
    "LFD_FIR_DB": "1", "LFD_SCAN_DEEP": "1", "LFD_TM_M4": "1", "LFD_K1_BAND": "8", "LFD_RUN_M4": "1",
    "LFD_RUN_PF": "3", "LFD_RUN_NT": "768", "LFD_RUN_MINW": "0", "LFD_RUN_BUF": "1", "LFD_RUN_SEPI": "1",
    "LFD_TM_NT": "768", "LFD_TM_PF": "3", "LFD_TM_SWAP": "1", "LFD_TM_NTILE": "1", "LFD_TM_BUF": "0",
    "LFD_TM_SEPI": "0", "LFD_TM_DIAG_LDS": "1", "LFD_MF_PF": "1", "LFD_MF_THREADS": "1024", "LFD_MF_BPW": "3",
    "LFD_SCAN_THREADS": "64", "LFD_SCAN_DEFER_THREADS": "128", "LFD_FR_STAGE_OLD": "1", "LFD_ROLL_STAGE": "0",
    "LFD_ROLL_PF": "3", "LFD_ROLL_MINW": "4", "LFD_ROLL_DPP": "0", "LFD_ROLL_RING": "0", "LFD_ROLL_SEG": "99",
    "LFD_ROLL_SEGSUM": "0", "LFD_ROLL_DIRECT_MAX": "100", "LFD_FIR_STRIP": "1", "LFD_SUBBLOCK": "1",
    "LFD_RUN_UNIT": "8", "LFD_RUN_TAIL": "9", "LFD_K1_NOLDS": "1", "LFD_K1_CHAN_FAST": "1",
    "LFD_STREAM_DIRECT2D": "1",
    # the old kernel selectors (now lfd_set_option)
    "LFD_NO_RUNS": "1", "LFD_K1_REC": "1", "LFD_TM_X2": "0", "LFD_SCAN_DEFER": "0", "LFD_FULLRATE_SERIAL": "1",
    "LFD_NO_LATTICE": "1", "LFD_NO_HSKIP": "1", "LFD_FIR_VALU": "1",
}


def _relrms(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(np.sum((a - b) ** 2) / np.sum(b ** 2)))


@pytest.mark.parametrize("time_major", [False, True])
def test_env_knobs_do_not_change_results(monkeypatch, time_major):
    import torch
    from lfdas.design import lowpass_sos, pass_filter_sos
    from lfdas.plan import LowpassPlan, fir_decimate_device, rolling_mean_device, sosfiltfilt_device
    from lfdas.proc import fir_decimate_design
    for k, v in KNOBS.items():
        monkeypatch.setenv(k, v)
    # cfg1 geometry: 250 Hz, dt = 0.2 s, P = 40, B = 6
    fs, dt_out, P, B, n_ch, n = 250.0, 0.2, 40, 6, 64, 6000
    x = (np.random.default_rng(11).standard_normal((n_ch, n)) + 1.5).astype(np.float32)
    dt_ns, t0 = 4_000_000, 1_505_692_800_000_000_000
    tg = S.time_grid(t0, t0 + n * dt_ns, dt_out)
    sched = S.lfproc_chunks(len(tg), P, B)
    lo, w = S.grid_positions(t0, dt_ns, tg)
    chunks = [(*S.select_range(t0, dt_ns, n, tg[a], tg[b]), oa, ob) for a, b, oa, ob in sched]
    plan = LowpassPlan(lowpass_sos(fs, 1 / dt_out / 2 * 0.9), n_ch, n, lo, w, chunks)
    xd = torch.from_numpy(np.ascontiguousarray(x.T)).cuda().t() if time_major else torch.from_numpy(x).cuda()
    yd = torch.full((n_ch, len(tg)), float("nan"), dtype=torch.float64, device="cuda")
    plan.execute(xd, yd, plan.alloc_workspace())
    torch.cuda.synchronize()
    assert plan.last_kernel() == ("mfma_runs_tm" if time_major else "mfma_runs")
    y = yd.cpu().numpy()
    ref = oracle.lfproc_process(x, t0, dt_ns, tg[0], tg[-1] + 1, dt_out, P, B)
    for (_, r), (_, _, oa, ob) in zip(ref, sched):
        gates.check(f"env_knobs tm={time_major}", _relrms(y[:, oa:ob], r), gates.MFMA)
    plan.close()
    if time_major:
        return
    # rolling mean: W = S (k_rolling_tc), S < W (segment sums), S = 1 (running sum)
    xr = (np.random.default_rng(12).standard_normal((8, 20_000)) + 0.5).astype(np.float32)
    for W, S_ in ((100, 100), (256, 64), (100, 1)):
        got = rolling_mean_device(torch.from_numpy(xr).cuda(), W, S_).cpu().numpy()
        want = oracle.rolling_mean(xr, W, S_)
        m = ~np.isnan(want)
        assert np.array_equal(np.isnan(got), ~m)
        assert _relrms(got[m], want[m]) < 1e-6, (W, S_)
    # full-rate zero-phase band-pass (blocked path, not the serial kernel)
    xf = (np.random.default_rng(13).standard_normal((6, 30_000))).astype(np.float32)
    sos = pass_filter_sos(1000.0, 1.0, 10.0)
    got = sosfiltfilt_device(torch.from_numpy(xf).cuda(), sos).cpu().numpy()
    # float32 samples to the oracle: SciPy forms the odd extension in the input
    # dtype (_signaltools.py:4684), as the device does
    assert _relrms(got, oracle.sosfiltfilt(sos, xf)) < 1e-10
    # FIR decimation on the matrix cores (q = 10)
    taps, delay = fir_decimate_design(10)
    got = fir_decimate_device(torch.from_numpy(xf).cuda(), taps, 10, delay).cpu().numpy()
    assert _relrms(got, oracle.decimate_fir(xf.astype(np.float64), 10)) < 1e-9
    from lfdas._lib import load
    assert load().lfd_fir_decimate_last_kernel() == 1
