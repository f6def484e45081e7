"""Host logic on CPU: C-ABI exports, schedule/index arithmetic, plan geometry
and the plan's kernel constants (via the NumPy kernel model in emulate.py)."""
import os
import re

import numpy as np
import pytest

import gates
import oracle
import synth
from emulate import emulate
from lfdas import _lib
from lfdas import schedule as S
from lfdas.design import default_padlen, lowpass_sos
from lfdas.plan import LowpassPlan

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(os.path.dirname(__file__), "golden")


def test_library_exports_every_header_symbol():
    hdr = open(os.path.join(ROOT, "include", "lfdas.h")).read()
    names = set(re.findall(r"\b(lfd_[a-z0-9_]+)\s*\(", hdr))
    assert names, "no functions parsed from include/lfdas.h"
    lib = _lib.load()
    for n in sorted(names):
        assert hasattr(lib, n), n
    assert names == set(_lib.EXPORTED)
    assert lib.lfd_version() >= 100


def test_production_library_reads_no_environment():
    """liblfdas.so (the product) holds no getenv call site and no LFD_* knob
    name: its outputs and kernel choices cannot depend on the environment.
    The A/B knobs and the "timing only" diagnostic modes exist only in
    liblfdas_diag.so (-DLFD_DIAG), which tools/ load through LFDAS_LIB."""
    import subprocess
    so = os.path.join(os.path.dirname(_lib.__file__), "liblfdas.so")
    blob = open(so, "rb").read()
    assert [m for m in re.findall(rb"LFD_[A-Z0-9_]{3,}", blob) if not m.startswith(b"LFD_OPT_")] == []
    und = subprocess.run(["nm", "-D", "--undefined-only", so], capture_output=True, text=True).stdout
    assert "getenv" not in und
    diag = os.path.join(os.path.dirname(_lib.__file__), "liblfdas_diag.so")
    assert b"LFD_TM_MODE" in open(diag, "rb").read()
    # the sources: every getenv sits behind LFD_DIAG
    for f in ("lfd_kernels.hip", "lfd_capi.cpp", "lfd_stream.cpp", "lfd_internal.h"):
        src = open(os.path.join(ROOT, "low-freq-real-time_amd", "csrc", f)).read()
        guarded = []  # per open #if: is it the LFD_DIAG branch
        for ln in src.splitlines():
            t = ln.strip()
            if t.startswith("#if"):
                guarded.append(t.startswith("#ifdef LFD_DIAG") or t == "#if defined(LFD_DIAG)")
            elif t.startswith("#el") and guarded:
                guarded[-1] = False
            elif t.startswith("#endif") and guarded:
                guarded.pop()
            if "getenv(" in t and not t.startswith("//"):
                assert any(guarded), (f, ln)
        assert guarded == [], f


def test_kernel_options_roundtrip_and_validation():
    lib = _lib.load()
    import ctypes
    v = ctypes.c_int64(-1)
    for name, oid in _lib.OPTIONS.items():
        assert lib.lfd_get_option(oid, ctypes.byref(v)) == 0 and v.value == 0, name
    with _lib.kernel_options(no_runs=1, scan_defer=2):
        lib.lfd_get_option(_lib.OPTIONS["scan_defer"], ctypes.byref(v))
        assert v.value == 2
    lib.lfd_get_option(_lib.OPTIONS["scan_defer"], ctypes.byref(v))
    assert v.value == 0
    assert lib.lfd_set_option(99, 1) == _lib.LFD_EINVAL
    assert lib.lfd_set_option(_lib.OPTIONS["no_runs"], 3) == _lib.LFD_EINVAL
    assert lib.lfd_set_option(_lib.OPTIONS["scan_defer"], 5) == _lib.LFD_EINVAL


def test_design_matches_oracle():
    for fs, fc in [(250.0, 1.0), (500.0, 0.45), (200.0, 0.045), (2000.0, 0.45)]:
        np.testing.assert_array_equal(lowpass_sos(fs, fc), oracle.butter_sos(4, fc / (fs / 2)))
        assert default_padlen(lowpass_sos(fs, fc)) == 15


def test_time_grid_ms_truncation():
    tg = S.time_grid(0, 10_000_000_000, 0.0015)  # int(1.5) ms step
    assert tg[1] - tg[0] == 1_000_000
    np.testing.assert_array_equal(S.time_grid(0, 5_000_000_000, 1.0), np.arange(5) * 1_000_000_000)


@pytest.mark.parametrize("L,P,B", [(120, 40, 6), (3600, 600, 7), (30, 40, 6), (96, 40, 6), (8640, 2, 0), (7, 3, 1)])
def test_schedule_matches_oracle(L, P, B):
    assert S.lfproc_chunks(L, P, B) == oracle.lfproc_schedule(L, P, B)
    sched, kinds = S.lfproc_chunks(L, P, B, with_kind=True)
    assert kinds[0] == "first" and all(k in ("body", "tail") for k in kinds[1:])
    # outputs contiguous, disjoint
    outs = [(a, b) for _, _, a, b in sched]
    for (a0, b0), (a1, b1) in zip(outs, outs[1:]):
        assert b0 == a1


def test_schedule_property_random():
    """Property check over 300 seeded random (L, P, B) with P > 2B: the Python
    and the native (C-ABI) chunk schedules equal the oracle's restatement of
    lf_das.py:258-290, and the output ranges tile [B, ...) contiguously."""
    from lfdas.stream import lfproc_schedule as native_schedule
    rng = np.random.default_rng(77)
    for _ in range(300):
        B = int(rng.integers(0, 12))
        P = int(rng.integers(2 * B + 1, 2 * B + 80))
        L = int(rng.integers(2, 6 * P + 10))
        try:
            want = oracle.lfproc_schedule(L, P, B)
        except ValueError:  # P clipped to L - 1 <= 2B: the reference never ends; all three refuse
            with pytest.raises(ValueError):
                S.lfproc_chunks(L, P, B)
            with pytest.raises(Exception):
                native_schedule(L, P, B)
            continue
        assert S.lfproc_chunks(L, P, B) == want, (L, P, B)
        got = [tuple(int(v) for v in row) for row in native_schedule(L, P, B)]
        assert got == [tuple(w) for w in want], (L, P, B)
        outs = [(a, b) for _, _, a, b in want]
        for (a0, b0), (a1, b1) in zip(outs, outs[1:]):
            assert b0 == a1


def test_schedule_rejects_non_advancing():
    with pytest.raises(ValueError):
        S.lfproc_chunks(100, 10, 5)


def test_grid_positions_and_select():
    lo, w = S.grid_positions(1000, 4, [1000, 1004, 1006, 1400])
    np.testing.assert_array_equal(lo, [0, 1, 1, 100])
    np.testing.assert_allclose(w, [0, 0, 0.5, 0])
    assert S.select_range(1000, 4, 50, 1001, 1008) == (1, 2)
    assert S.select_range(1000, 4, 50, 0, 10 ** 6) == (0, 49)


def _plan_for(fs, dt_out, P, B, n_ch, n):
    dt_ns = int(round(1e9 / fs))
    t0 = synth.T0_NS
    tg = S.time_grid(t0, t0 + n * dt_ns, dt_out)
    sched = S.lfproc_chunks(len(tg), P, B)
    lo, w = S.grid_positions(t0, dt_ns, tg)
    chunks = [(*S.select_range(t0, dt_ns, n, tg[a], tg[b]), oa, ob) for a, b, oa, ob in sched]
    sos = lowpass_sos(fs, 1 / dt_out / 2 * 0.9)
    return LowpassPlan(sos, n_ch, n, lo, w, chunks), sched, tg


def test_plan_geometry_cfg3():
    plan, sched, tg = _plan_for(500.0, 1.0, 600, 7, 10_000, 1_800_000)
    assert plan.block_len == 500 and plan.n_blocks == 3599
    bc, sc, cg = plan.constants()
    assert len(cg) == 7
    # every output grid point maps to exactly one chunk output
    produced = np.zeros(len(tg), int)
    for G_, (a, b, oa, ob) in zip(cg, sched):
        assert G_["head_end"] == G_["s0"] and G_["tail_begin"] == G_["s1"]  # 1-sample tail
        produced[oa:ob] += 1
        assert G_["kout1"] - G_["kout0"] == ob - oa
    assert produced.sum() == 3585 and produced.max() == 1
    # workspace: F (9 doubles/block/ch) + SF + TP
    assert plan.workspace_bytes >= 9 * 8 * plan.n_blocks * 10_000


def test_plan_rejects_unsupported_grids():
    sos = lowpass_sos(250.0, 1.0)
    # a phase per point: no lattice plan either (the per-chunk general path)
    with pytest.raises(_lib.LFDUnsupported, match="lattice phases for 3 points"):
        LowpassPlan(sos, 2, 1000, [0, 10, 25], [0, 0, 0], [(0, 999, 0, 3)])
    # uniform spacing with one off-sample point: two phases (y[lo], y[lo + 1])
    plan = LowpassPlan(sos, 2, 1000, [0, 10, 20], [0, 0.5, 0], [(0, 999, 0, 3)])
    with pytest.raises(_lib.LFDUnsupported, match="lattice"):
        plan.constants()
    plan.close()
    # a slowly drifting grid (one phase step per 20 points): a lattice plan
    lo = np.arange(60) * 100 + np.arange(60) // 20
    plan = LowpassPlan(sos, 2, 7000, lo, np.full(60, 0.25), [(0, 6999, 0, 60)])
    with pytest.raises(_lib.LFDUnsupported, match="lattice"):
        plan.constants()
    plan.close()
    # more than 32 lattice phases (a jittered grid): the general path
    rng = np.random.default_rng(3)
    lo = np.arange(60) * 100 + rng.integers(-30, 30, 60)
    with pytest.raises(_lib.LFDUnsupported, match="32 lattice phases"):
        LowpassPlan(sos, 2, 7000, np.sort(lo), np.zeros(60), [(0, 6999, 0, 60)])
    with pytest.raises(ValueError, match="padlen"):
        LowpassPlan(sos, 2, 1000, [0, 10, 20], [0, 0, 0], [(0, 12, 0, 1)])


def test_lattice_plan_3khz_grid_host_only():
    """3 kHz on integer-ns times (333,333 ns): the 1 s grid's fraction varies
    and its spacing is 3,000 or 3,001 samples; the plan is a lattice plan
    (a few phases), created without a device."""
    plan, sched, tg = _plan_for(3000.0, 1.0, 120, 7, 8, 3000 * 1300)
    lo, w = S.grid_positions(synth.T0_NS, 333_333, tg)
    assert len(np.unique(np.diff(lo))) == 2 and len(np.unique(w)) > 100
    with pytest.raises(_lib.LFDUnsupported, match="lattice"):
        plan.constants()
    assert plan.block_len == 500  # the sub-plans' sub-blocks (R = 3,000 = 6 x 500)
    plan.close()


def _r_model(sos):
    """Realization R of the cascade (lfd_internal.h RCoef): FIR c (c[0] = 1),
    gain G, all-pole sections (a1, a2)."""
    num = np.array([1.0])
    for s in sos:
        num = np.convolve(num, s[:3])
    return num / num[0], num[0], [(s[4], s[5]) for s in sos]


def _allpole(secs, w):
    v = np.array(w, dtype=np.float64)
    for a1, a2 in secs:
        out = np.zeros_like(v)
        p1 = p2 = 0.0
        for i, u in enumerate(v):
            o = u - a1 * p1 - a2 * p2
            p2, p1 = p1, o
            out[i] = o
        v = out
    return v


def test_lattice_onepass_plan_host_math():
    """The lattice plan's one-pass form (3 kHz on integer-ns times): the
    output rows 8 + d of its block taps are the zero-boundary zero-phase
    output at offset d of a block (forward all-pole from zero state with the
    block's true FIR history, reverse from zero state at the block end),
    every output block starts a run, and each offset's chunk outputs cover
    the points that need that phase."""
    plan, sched, tg = _plan_for(3000.0, 1.0, 120, 7, 8, 3000 * 1300)
    n_off, last, view = plan.lattice()
    assert 2 <= n_off <= 8 and not last and view is not None
    Kx = view.block_taps()
    L, J = view.block_len if hasattr(view, "block_len") else 500, 4
    assert Kx.shape == (8 + n_off, L + J)
    c, G, secs = _r_model(plan.sos)
    rng = np.random.default_rng(11)
    xe = rng.standard_normal(L + J)
    w = np.array([np.dot(c, xe[J + t - np.arange(J + 1)]) for t in range(L)])
    yf = G * _allpole(secs, w)
    ql = _allpole(secs, yf[::-1])[::-1]
    for d in range(n_off):
        ref = G * np.dot(c, ql[d:d + J + 1])
        got = Kx[8 + d] @ xe
        assert abs(got - ref) <= 1e-10 * max(1.0, abs(ref)), (d, got, ref)
    ks, ln, rc = view.runs()
    _, _, cg = view.constants()
    starts = set(ks.tolist())
    for G_ in cg:
        for k in range(G_["kout0"], G_["kout1"], G_["kstep"]):
            assert k in starts
        assert G_["tail_out_j"] < 0 and (G_["kout1"] == G_["kout0"] or G_["kout0"] > G_["kb"])
    # H0 of offset 0 is the plan's own H0; later offsets differ
    np.testing.assert_allclose(rc["H0L"][0], rc["H0"], rtol=1e-13)
    assert not np.allclose(rc["H0L"][1], rc["H0"])
    plan.close()
    with _lib.kernel_options(lattice_phases=1):
        plan2, _, _ = _plan_for(3000.0, 1.0, 120, 7, 8, 3000 * 1300)
        assert plan2.lattice()[0] == 0
        plan2.close()


@pytest.mark.parametrize("name", ["lfproc_cfg1.npz", "lfproc_cfg5_slice.npz"])
def test_plan_constants_reproduce_golden(name):
    """Host-only plan → NumPy model of the kernels → SciPy golden vectors."""
    g = np.load(os.path.join(G, name), allow_pickle=False)
    if "cfg1" in name:
        x = synth.random_das_spool_data().astype(np.float32)[:24]
        ref = g["y"][:24]
    else:
        x = synth.noise_sine(4, 600_000, 200.0, seed=5, dc=1000.0)
        ref = g["y"]
    fs, dt_out, P, B = float(g["fs"]), float(g["dt_out"]), int(g["P"]), int(g["B"])
    plan, sched, tg = _plan_for(fs, dt_out, P, B, x.shape[0], x.shape[1])
    y = emulate(plan, x, 15)
    m = ~np.isnan(ref)
    assert np.array_equal(np.isnan(y), ~m)
    rel = np.sqrt(np.sum((y[m] - ref[m]) ** 2) / np.sum(ref[m] ** 2))
    gates.check(f"emulate_recurrence {name}", rel, gates.EMU_REC)


@pytest.mark.parametrize("name", ["lfproc_cfg1.npz", "lfproc_cfg5_slice.npz"])
def test_block_taps_reproduce_golden(name):
    """The MFMA kernel's formulation (block functionals as taps . samples, the
    taps from the plan) reproduces the SciPy golden vectors, and agrees with
    the recurrence formulation functional by functional."""
    g = np.load(os.path.join(G, name), allow_pickle=False)
    if "cfg1" in name:
        x = synth.random_das_spool_data().astype(np.float32)[:24]
        ref = g["y"][:24]
    else:
        x = synth.noise_sine(4, 600_000, 200.0, seed=5, dc=1000.0)
        ref = g["y"]
    fs, dt_out, P, B = float(g["fs"]), float(g["dt_out"]), int(g["P"]), int(g["B"])
    plan, sched, tg = _plan_for(fs, dt_out, P, B, x.shape[0], x.shape[1])
    Kx = plan.block_taps()
    assert Kx.shape == (4 * plan.n_sec + 1, plan.block_len + 2 * plan.n_sec)
    m = ~np.isnan(ref)
    # cfg5's R = 2000 runs as 4 sub-blocks of 500 (taps + run buffers fit LDS)
    assert plan.runs() is not None and plan.block_len <= 504
    for k1 in ("taps", "runs"):
        y = emulate(plan, x, 15, k1=k1)
        assert np.array_equal(np.isnan(y), ~m)
        rel = np.sqrt(np.sum((y[m] - ref[m]) ** 2) / np.sum(ref[m] ** 2))
        gates.check(f"emulate_{k1} {name}", rel, gates.EMU_TAPS)


def _plan_off(fs, dt_out, P, B, n_ch, n, off_ns, grid_start_s=1.0):
    """Samples at t0 + i dt with t0 = T0 + off_ns; the output grid starts on a
    whole second (the notebooks' bgtime): every grid point falls the same
    fraction w of a sample past a sample."""
    dt_ns = int(round(1e9 / fs))
    t0 = synth.T0_NS + off_ns
    t1 = synth.T0_NS + int(grid_start_s * 1e9)
    t2 = t0 + (n - 1) * dt_ns
    tg = S.time_grid(t1, t2, dt_out)
    sched = S.lfproc_chunks(len(tg), P, B)
    lo, w = S.grid_positions(t0, dt_ns, tg)
    chunks = [(*S.select_range(t0, dt_ns, n, tg[a], tg[b]), oa, ob) for a, b, oa, ob in sched]
    sos = lowpass_sos(fs, 1 / dt_out / 2 * 0.9)
    return LowpassPlan(sos, n_ch, n, lo, w, chunks), sched, tg, t0, t1, t2, dt_ns, w


@pytest.mark.parametrize("cfg", [
    (250.0, 0.2, 40, 6, 6000, 370_000),       # cfg1 geometry, t0 0.37 ms past the grid
    (500.0, 1.0, 60, 7, 90_000, 1_900_000),   # cfg3 parameters, 1.9 ms
    (200.0, 10.0, 40, 6, 200_000, 1_900_000),  # cfg5 parameters: R = 2000 -> 4 sub-blocks of 500
    (1000.0, 10.0, 20, 3, 400_000, 0),        # dt = 10 s at 1 kHz: R = 10,000 -> 20 sub-blocks
])
@pytest.mark.parametrize("k1", ["recurrence", "taps", "runs"])
def test_offsample_and_subblock_plans_match_oracle(cfg, k1):
    """Off-sample uniform grids (constant w) and long grid spacings (sub-blocks)
    stay in the block plan: its host constants, driven through the NumPy
    kernel model, reproduce the oracle's chunked sosfiltfilt + interp1d."""
    fs, dt_out, P, B, n, off = cfg
    x = synth.noise_sine(3, n, fs, seed=21, dc=50.0)
    plan, sched, tg, t0, t1, t2, dt_ns, w = _plan_off(fs, dt_out, P, B, 3, n, off)
    R = int(round(fs * dt_out))
    assert np.all(w == w[0]) and (w[0] > 0) == (off > 0)
    assert plan.block_len * (R // plan.block_len) == R and plan.block_len <= 504
    _, _, cg = plan.constants()
    assert np.all(cg["kstep"] == R // plan.block_len)
    if k1 == "runs":
        assert plan.runs() is not None
    y = emulate(plan, x, 15, k1=k1)
    ref = oracle.lfproc_process(x, t0, dt_ns, t1, t2, dt_out, P, B)
    num = den = 0.0
    produced = np.zeros(len(tg), bool)
    for (tt, r), (a, b, oa, ob) in zip(ref, sched):
        np.testing.assert_array_equal(tt, tg[oa:ob])
        num += float(np.sum((y[:, oa:ob] - r) ** 2))
        den += float(np.sum(r ** 2))
        produced[oa:ob] = True
    gates.check(f"emulate_offgrid {k1}", (num / den) ** 0.5, gates.EMU_REC if k1 == "recurrence" else gates.EMU_TAPS)
    assert np.all(np.isnan(y[:, ~produced]))


def test_offsample_tail_output_blends_two_samples():
    """A single chunk whose last grid point lies in the partial tail block
    (the one-shot Patch.pass_filter().interpolate() shape): the scan's tail
    output interpolates between the two zero-phase samples around it."""
    fs, n = 250.0, 2000
    x = synth.noise_sine(2, n, fs, seed=5)
    lo = np.arange(3, n - 1, 50, dtype=np.int64)
    w = np.full(len(lo), 0.25)
    sos = lowpass_sos(fs, 1.0)
    plan = LowpassPlan(sos, 2, n, lo, w, [(0, n - 1, 0, len(lo))])
    _, _, cg = plan.constants()
    assert cg[0]["tail_out_j"] == len(lo) - 1
    y = emulate(plan, x, 15, k1="runs")
    yf = oracle.sosfiltfilt(oracle.butter_sos(4, 1.0 / 125.0), x)
    ref = yf[:, lo] + 0.25 * (yf[:, lo + 1] - yf[:, lo])
    gates.check("emulate_runs_blended", np.sqrt(np.sum((y - ref) ** 2) / np.sum(ref ** 2)), gates.EMU_TAPS)


def test_host_only_plan_cannot_execute():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    plan, _, _ = _plan_for(250.0, 0.2, 40, 6, 2, 6000)
    with pytest.raises((ValueError, TypeError)):
        plan.execute(torch.zeros(2, 6000), torch.zeros(2, 120), torch.zeros(10, dtype=torch.uint8))


def test_units_and_coordinate_derived_time_step():
    """dascore.units.s windows (rolling notebooks cell 7) and a time_step that
    follows the time coordinate (what chunk(time=None) merges decimated or
    rolled outputs on)."""
    import lfdas.dc as dc
    from lfdas.core import to_timedelta64
    s = dc.units.s
    assert to_timedelta64(10.0 * s) == np.timedelta64(10, "s")
    assert to_timedelta64(250 * dc.units.ms) == np.timedelta64(250, "ms")
    p = dc.get_example_patch()
    assert p.attrs["step_time"] == np.timedelta64(4, "ms") == p.attrs["d_time"]
    q = p.new(coords=p.coords.update(time=p.coords["time"][::50]), data=p.data[:, ::50])
    assert q.attrs["time_step"] == np.timedelta64(200, "ms")
    a = q.update_attrs(d_time=0.2)
    assert a.attrs["d_time"] == 0.2 and a.attrs["time_step"] == np.timedelta64(200, "ms")
    half = [q.select(time=(None, q.coords["time"][19])), q.select(time=(q.coords["time"][20], None))]
    merged = dc.spool(half).chunk(time=None)
    assert len(merged) == 1 and merged[0].shape == q.shape


def test_spool_chunk_windows_and_keep_partial():
    """Spool.chunk(time=T, overlap=O): windows [start, start + T) stepping by
    T - O from the merged patch's first sample; the last window past the
    data is dropped unless keep_partial (then it ends at the last sample).
    T = P dt, O = 2 B dt start exactly where LFProc's chunks start."""
    import lfdas.dc as dc
    sp = dc.get_example_spool()  # 3 x 2000 samples @ 250 Hz, contiguous: 24 s
    P, B, dt = 40, 6, 0.2
    for keep in (False, True):
        ch = sp.chunk(time=P * dt, overlap=2 * B * dt, keep_partial=keep)
        t0 = sp[0].coords["time"][0]
        starts = [(c.coords["time"][0] - t0) / np.timedelta64(1, "ms") for c in ch]
        ends = [(c.coords["time"][-1] - t0) / np.timedelta64(1, "ms") for c in ch]
        assert starts == [0, 5600, 11200, 16800][: len(ch)]
        assert ends[:3] == [7996, 13596, 19196]
        assert len(ch) == (4 if keep else 3)
        if keep:
            assert ends[3] == 23996  # the partial last window ends at the last sample
        for c in ch:
            assert c.shape[0] == 300
            grp, s0, s1 = c._chunk_window
            assert s1 - s0 + 1 == c.shape[1]
    # LFProc's schedule on the same spool starts its chunks at the same samples
    tg = S.time_grid(sp[0].coords["time"][0], sp[-1].coords["time"][-1], dt)
    sched = S.lfproc_chunks(len(tg), P, B)
    np.testing.assert_array_equal([tg[a] for a, _, _, _ in sched],
                                  [c.coords["time"][0].astype(np.int64) for c in
                                   sp.chunk(time=P * dt, overlap=2 * B * dt, keep_partial=True)])
    with pytest.raises(ValueError, match="overlap"):
        sp.chunk(time=1.0, overlap=1.0)
    # a gap splits the merged patches: windows never straddle it
    gapped = dc.get_example_spool(time_gap=2.0).chunk(time=4.0, overlap=1.0)
    assert all((c.coords["time"][-1] - c.coords["time"][0]) < np.timedelta64(4, "s") for c in gapped)
