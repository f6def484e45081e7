"""GPU tests of the drop-in surface (lf_das.LFProc, Patch/Spool ops) against
the SciPy golden vectors and the oracle.  Tolerances: tests/gates.py for the
float64 low-pass+decimate outputs (<= 10x the measured relRMS), <= 1e-6
(rolling mean); identical output times."""
import os

import numpy as np
import pytest

import gates
import oracle
import synth

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(np.sum((a - b) ** 2) / np.sum(b ** 2)))


def _example_spool(dims=("distance", "time"), gap_s=0.0):
    import lfdas.dc as dc
    sp = dc.get_example_spool(time_gap=gap_s)
    if dims == ("time", "distance"):
        sp = dc.spool([p.new(data=np.ascontiguousarray(p.data.T), dims=dims) for p in sp])
    return sp


@pytest.mark.parametrize("dims", [("distance", "time"), ("time", "distance")])
def test_lfproc_cfg1_matches_scipy_golden(tmp_path, capsys, dims):
    import lf_das
    g = np.load(os.path.join(G, "lfproc_cfg1.npz"), allow_pickle=False)
    sp = _example_spool(dims)
    lfp = lf_das.LFProc(sp)
    lfp.update_processing_parameter(output_sample_interval=0.2, process_patch_size=40, edge_buff_size=6)
    lfp.set_output_folder(str(tmp_path / "out"))
    t1 = np.datetime64("2017-09-18T00:00:00")
    t2 = np.datetime64("2017-09-18T00:00:24")
    lfp.process_time_range(t1, t2)
    lines = [l for l in capsys.readouterr().out.splitlines() if "Processing patch" in l]
    assert lines[0] == "Processing patch  1" and lines[-1] == "Processing patch 4 (Last portion of data)"
    assert len(lfp.outputs) == 4
    tg = g["tg"]
    for out, (oa, ob) in zip(lfp.outputs, g["sched"]):
        np.testing.assert_array_equal(out.coords["time"].astype(np.int64), tg[oa:ob])
        d = out.data if dims[0] == "distance" else out.data.T
        assert d.shape == (300, ob - oa)
        assert d.dtype == np.float64  # SciPy's result dtype (sosfiltfilt promotes)
        gates.check(f"lfproc_cfg1_golden {dims} {oa}", _rel(d, g["y"][:, oa:ob]), gates.MFMA)
        assert out.attrs["d_time"] == 0.2
    files = sorted(os.listdir(tmp_path / "out"))
    assert len(files) == 4 and all(f.startswith("LFDAS_2017-09-18T") and f.endswith(".h5") for f in files)
    t_last = lfp.get_last_processed_time()
    assert np.datetime64(t_last, "ns").astype(np.int64) == tg[g["sched"][-1][1] - 1]


def test_lfproc_errors(tmp_path):
    import lf_das
    lfp = lf_das.LFProc(_example_spool())
    with pytest.raises(Exception, match="Please setup output folder first"):
        lfp.process_time_range(np.datetime64("2017-09-18T00:00:00"), np.datetime64("2017-09-18T00:00:20"))
    lfp = lf_das.LFProc(_example_spool(gap_s=2.0), verbose=False)
    lfp.update_processing_parameter(output_sample_interval=0.2, process_patch_size=40, edge_buff_size=6)
    lfp.set_output_folder(str(tmp_path / "o"))
    with pytest.raises(Exception, match="patch merge failed! Gap in data exists"):
        lfp.process_time_range(np.datetime64("2017-09-18T00:00:00"), np.datetime64("2017-09-18T00:00:24"))
    assert len(lfp.outputs) == 1  # chunk 1 (0-8 s) precedes the gap at ~8 s


def test_sharded_driver_world1_matches_lfproc(tmp_path):
    """lfdas.shard.process_time_range_sharded without a process group (one
    rank): the device plan on the whole spool, the same outputs and files as
    LFProc.process_time_range."""
    import lf_das
    from lfdas.shard import process_time_range_sharded
    sp = _example_spool()
    params = {"output_sample_interval": 0.2, "process_patch_size": 40, "edge_buff_size": 6}
    t1, t2 = np.datetime64("2017-09-18T00:00:00"), np.datetime64("2017-09-18T00:00:24")
    outs = process_time_range_sharded(sp, t1, t2, params, output_folder=str(tmp_path / "sh"), verbose=False)
    lfp = lf_das.LFProc(sp, verbose=False)
    lfp.update_processing_parameter(**params)
    lfp.set_output_folder(str(tmp_path / "one"))
    lfp.process_time_range(t1, t2)
    assert len(outs) == len(lfp.outputs) == 4
    for a, b in zip(outs, lfp.outputs):
        np.testing.assert_array_equal(a.coords["time"], b.coords["time"])
        np.testing.assert_array_equal(a.data, b.data)
    assert sorted(os.listdir(tmp_path / "sh")) == sorted(os.listdir(tmp_path / "one"))


def test_realtime_resume_contiguous(tmp_path):
    """low_pass_dascore_edge.ipynb:215-233: second run starts at
    last_out - (ceil(edge/dt)-1)*dt and continues the output grid."""
    import lf_das
    sp = _example_spool()
    dt, B = 0.2, 6
    folder = str(tmp_path / "rt")
    lfp = lf_das.LFProc(sp.select(time=(None, np.datetime64("2017-09-18T00:00:15.996"))), verbose=False)
    lfp.update_processing_parameter(output_sample_interval=dt, process_patch_size=40, edge_buff_size=B)
    lfp.set_output_folder(folder)
    lfp.process_time_range(np.datetime64("2017-09-18T00:00:00"), np.datetime64("2017-09-18T00:00:15.996"))
    t_last = np.datetime64(lfp.get_last_processed_time(), "ns")
    lfp2 = lf_das.LFProc(sp, verbose=False)
    lfp2.update_processing_parameter(output_sample_interval=dt, process_patch_size=40, edge_buff_size=B)
    lfp2.set_output_folder(folder)
    t1 = t_last - np.timedelta64(int((B - 1) * dt * 1e9), "ns")
    lfp2.process_time_range(t1, np.datetime64("2017-09-18T00:00:23.996"))
    first_new = lfp2.outputs[0].coords["time"][0]
    assert first_new == t_last + np.timedelta64(int(dt * 1e9), "ns")


def test_pass_filter_interpolate_fused_and_general():
    import lfdas.dc as dc
    p = dc.get_example_patch()  # 300 x 2000 @ 250 Hz, dims (distance, time)
    t = p.coords["time"]
    x = p.data.astype(np.float32)
    sos = oracle.butter_sos(4, 1.0 / 125.0)
    yfull = oracle.sosfiltfilt(sos, x)
    tt = (t.astype(np.int64) - t[0].astype(np.int64)).astype(np.float64)
    for grid in (np.arange(t[0], t[-1], np.timedelta64(200, "ms")),            # aligned (block path)
                 np.arange(t[0] + np.timedelta64(2, "ms"), t[-1], np.timedelta64(230, "ms"))):  # general
        out = p.pass_filter(time=(None, 1.0)).interpolate(time=grid)
        ref = oracle.interp1d_linear(tt, yfull, (grid.astype(np.int64) - t[0].astype(np.int64)).astype(np.float64))
        np.testing.assert_array_equal(out.coords["time"], grid)
        assert out.data.dtype == np.float64
        gates.check(f"pass_filter_interpolate {grid[1] - grid[0]}", _rel(out.data, ref), gates.MFMA)


def test_pass_filter_full_rate_data():
    import lfdas.dc as dc
    p = dc.get_example_patch()
    y = p.pass_filter(time=(None, 10.0)).data
    ref = oracle.sosfiltfilt(oracle.butter_sos(4, 10.0 / 125.0), p.data.astype(np.float32))
    assert y.dtype == np.float64 and _rel(y, ref) < 1e-9


@pytest.mark.parametrize("dims", [("distance", "time"), ("time", "distance")])
def test_rolling_mean_patch(dims):
    import lfdas.dc as dc
    x = synth.noise_sine(6, 10_000, 1000.0, seed=4)
    t = np.datetime64("2023-03-22T03:00:00", "ns") + np.arange(10_000) * np.timedelta64(1, "ms")
    data = x if dims[0] == "distance" else x.T.copy()
    p = dc.Patch(data=data, coords={"distance": np.arange(6.0), "time": t}, dims=dims)
    r = p.rolling(time=1.0, step=1.0, engine="numpy").mean()
    ref = oracle.rolling_mean(x, 1000, 1000)
    d = r.data if dims[0] == "distance" else r.data.T
    assert d.shape == ref.shape and np.array_equal(np.isnan(d), np.isnan(ref))
    m = ~np.isnan(ref)
    gates.check(f"rolling_patch {dims}", _rel(d[m], ref[m]), gates.ROLL)
    np.testing.assert_array_equal(r.coords["time"], t[::1000])
    dn = r.dropna("time")
    assert dn.shape[dims.index("time")] == 9


def test_get_edge_effect_time_matches_oracle():
    import lf_das
    e = lf_das.get_edge_effect_time(sampling_interval=1 / 250.0, total_T=120.0, tol=1e-3, freq=5)
    e_ref = oracle.get_edge_effect_time(1 / 250.0, 120.0, tol=1e-3, freq=5)
    assert abs(e - e_ref) < 1e-9
    with pytest.raises(ValueError):
        lf_das.get_edge_effect_time(sampling_interval=1 / 200.0, total_T=20.8, tol=1e-3, freq=0.1)


def test_spool_chunk_windows_reproduce_lfproc_in_one_plan():
    """LFProc's schedule is Spool.chunk(time=P dt, overlap=2B dt)
    trimmed by B dt per side.  The windows' pass_filter().interpolate() at the
    trimmed grid reproduce LFProc's outputs and the oracle, and the whole
    list runs as ONE plan execute over the merged samples."""
    import lf_das
    import lfdas.dc as dc
    from lfdas import plan as PL
    from lfdas import schedule as S
    sp = _example_spool()
    P, B, dt = 40, 6, 0.2
    t1, t2 = np.datetime64("2017-09-18T00:00:00", "ns"), np.datetime64("2017-09-18T00:00:24", "ns")
    tg = S.time_grid(t1, t2, dt)
    sched = S.lfproc_chunks(len(tg), P, B)
    windows = sp.chunk(time=P * dt, overlap=2 * B * dt, keep_partial=True)
    assert len(windows) == len(sched) == 4
    fc = 1 / dt / 2 * 0.9
    n0 = PL.launch_count
    outs = [w.pass_filter(time=(None, fc)).interpolate(time=tg[oa:ob].astype("datetime64[ns]"))
            for w, (_, _, oa, ob) in zip(windows, sched)]
    assert PL.launch_count == n0  # nothing computed yet
    datas = [o.data for o in outs]
    assert PL.launch_count == n0 + 1  # one plan execute for every window
    lfp = lf_das.LFProc(sp, verbose=False, write_files=False)
    lfp.update_processing_parameter(output_sample_interval=dt, process_patch_size=P, edge_buff_size=B)
    lfp.process_time_range(t1, t2)
    x = dc.spool(sp).chunk(time=None)[0]
    tx = x.sample_times_ns()
    xd = np.asarray(x.data, np.float32)
    for d, o, w, ref_lp, (_, _, oa, ob) in zip(datas, outs, windows, lfp.outputs, sched):
        np.testing.assert_array_equal(o.coords["time"].astype(np.int64), tg[oa:ob])
        gates.check(f"chunk_windows_vs_lfproc {oa}", _rel(d, ref_lp.data), gates.MFMA)  # the §3.1 equivalence
        # the window's own semantics: sosfiltfilt of exactly its samples, then interp1d
        _, s0, s1 = w._chunk_window
        yf = oracle.sosfiltfilt(oracle.butter_sos(4, fc / 125.0), xd[:, s0:s1 + 1])
        want = oracle.interpolate(yf, -1, tx[s0:s1 + 1], tg[oa:ob])
        gates.check(f"chunk_windows_oracle {oa}", _rel(d, want), gates.MFMA)
    # two short grids far apart (a lattice phase per point): no shared plan,
    # one fused call each
    n1 = PL.launch_count
    outs2 = [windows[0].pass_filter(time=(None, fc)).interpolate(time=windows[0].coords["time"][1500:1510]),
             windows[1].pass_filter(time=(None, fc)).interpolate(time=windows[1].coords["time"][0:10])]
    for o in outs2:
        assert o.data.shape == (300, 10)
    assert PL.launch_count == n1 + 2


def test_chunk_window_output_shared_by_update_attrs_copy():
    """A lazy chunk-window output and its update_attrs copy share one
    request: both read the same data, in either order, any number of times
    (the result used to be popped on the first read)."""
    sp = _example_spool()
    P, B, dt = 40, 6, 0.2
    from lfdas import schedule as S
    t1, t2 = np.datetime64("2017-09-18T00:00:00", "ns"), np.datetime64("2017-09-18T00:00:24", "ns")
    tg = S.time_grid(t1, t2, dt)
    sched = S.lfproc_chunks(len(tg), P, B)
    windows = sp.chunk(time=P * dt, overlap=2 * B * dt, keep_partial=True)
    fc = 1 / dt / 2 * 0.9
    a = [w.pass_filter(time=(None, fc)).interpolate(time=tg[oa:ob].astype("datetime64[ns]"))
         for w, (_, _, oa, ob) in zip(windows, sched)]
    b = [o.update_attrs(d_time=dt) for o in a]
    d_a1 = a[1].data
    d_b1 = b[1].data
    d_b0 = b[0].data
    d_a0 = a[0].data
    np.testing.assert_array_equal(d_a1, d_b1)
    np.testing.assert_array_equal(d_a0, d_b0)
    assert b[0].attrs["d_time"] == dt
    for o in a[2:] + b[2:]:
        assert o.data.shape == (300, o.coords["time"].size)
