"""Archive spools and out-of-core LFProc: a directory
of patch files is indexed from headers only (``dc.spool(path).update()``,
low_pass_dascore.ipynb:78) and ``LFProc.process_time_range`` over a range
larger than the device budget streams the files through the device arena
(``lfd_stream_*`` continuous mode) with the resident path's chunks, outputs,
file names and gap error."""
import os

import numpy as np
import pytest

import gates
import oracle
import synth

T0 = np.datetime64("2017-09-18T00:00:00", "ns")


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(np.sum((a - b) ** 2) / np.sum(b ** 2)))


def _write_archive(folder, n_files=6, n_ch=24, n_t=2000, fs=250.0, dims=("distance", "time"),
                   skip=None, seed=1, jitter=None):
    """jitter = (file i, ns): files >= i start that much later (a boundary gap
    of one sample + jitter before file i)."""
    import lfdas.dc as dc
    os.makedirs(folder, exist_ok=True)
    x = synth.noise_sine(n_ch, n_files * n_t, fs, seed=seed, dc=5.0).astype(np.float64)
    step = np.timedelta64(int(round(1e9 / fs)), "ns")
    for i in range(n_files):
        if skip is not None and i == skip:
            continue
        blk = x[:, i * n_t:(i + 1) * n_t]
        t = T0 + (i * n_t + np.arange(n_t)) * step
        if jitter is not None and i >= jitter[0]:
            t = t + np.timedelta64(int(jitter[1]), "ns")
        data = blk if dims[0] == "distance" else np.ascontiguousarray(blk.T)
        p = dc.Patch(data=data, coords={"distance": np.arange(float(n_ch)), "time": t}, dims=dims,
                     attrs={"time_step": step})
        p.io.write(os.path.join(folder, f"raw_{i:03d}.h5"), "dasdae")
    return x


def test_directory_index_is_header_only(tmp_path):
    import lfdas.dc as dc
    from lfdas import io as lio
    _write_archive(str(tmp_path / "a"), n_files=3)
    sp = dc.spool(str(tmp_path / "a"))
    assert len(sp) == 3
    p = sp[1]
    assert isinstance(p._lazy, lio._FileData) and p._data is None
    assert p.shape == (24, 2000)
    assert p.attrs["time_min"] == T0 + 2000 * np.timedelta64(4, "ms")
    d = p.data  # read on use, not kept
    assert d.shape == (24, 2000) and p._data is None
    sub = p.select(time=(p.coords["time"][10], p.coords["time"][19]))
    assert sub.shape == (24, 10)
    # update() re-uses the header index and picks up new files
    import shutil
    _write_archive(str(tmp_path / "b"), n_files=4)
    shutil.copy(tmp_path / "b" / "raw_003.h5", tmp_path / "a" / "raw_003.h5")
    sp2 = sp.update()
    assert len(sp2) == 4 and sp2[1] is sp[1]


@pytest.mark.gpu
@pytest.mark.parametrize("dims", [("distance", "time"), ("time", "distance")])
def test_out_of_core_lfproc_matches_resident(tmp_path, capsys, dims):
    import lf_das
    import lfdas.dc as dc
    x = _write_archive(str(tmp_path / "raw"), dims=dims)
    t1, t2 = T0, T0 + np.timedelta64(6 * 8, "s") - np.timedelta64(4, "ms")
    res = {}
    for mode, budget in (("resident", None), ("stream", 1)):
        lfp = lf_das.LFProc(dc.spool(str(tmp_path / "raw")), max_resident_bytes=budget)
        lfp.update_processing_parameter(output_sample_interval=0.2, process_patch_size=40, edge_buff_size=6)
        lfp.set_output_folder(str(tmp_path / f"out_{mode}"))
        lfp.process_time_range(t1, t2)
        assert lfp.last_mode == mode
        res[mode] = (lfp.outputs, capsys.readouterr().out, sorted(os.listdir(tmp_path / f"out_{mode}")))
    (o_r, log_r, f_r), (o_s, log_s, f_s) = res["resident"], res["stream"]
    assert f_r == f_s and len(o_r) == len(o_s) > 3
    pl = lambda s: [l for l in s.splitlines() if "Processing patch" in l]  # noqa: E731
    assert pl(log_r) == pl(log_s)
    ref = oracle.lfproc_process(x.astype(np.float32), int(T0.astype(np.int64)), 4_000_000,
                                int(t1.astype(np.int64)), int(t2.astype(np.int64)), 0.2, 40, 6)
    for a, b, (rt, ry) in zip(o_r, o_s, ref):
        np.testing.assert_array_equal(a.coords["time"], b.coords["time"])
        np.testing.assert_array_equal(b.coords["time"].astype(np.int64), rt)
        da = a.data if dims[0] == "distance" else a.data.T
        db = b.data if dims[0] == "distance" else b.data.T
        gates.check(f"archive_stream_vs_resident {dims}", _rel(db, da), gates.PATHS)
        gates.check(f"archive_oracle {dims}", _rel(db, ry), gates.STREAM)


@pytest.mark.gpu
def test_out_of_core_gap_error(tmp_path):
    import lf_das
    import lfdas.dc as dc
    _write_archive(str(tmp_path / "raw"), skip=3)
    lfp = lf_das.LFProc(dc.spool(str(tmp_path / "raw")), max_resident_bytes=1, verbose=False)
    lfp.update_processing_parameter(output_sample_interval=0.2, process_patch_size=40, edge_buff_size=6)
    lfp.set_output_folder(str(tmp_path / "out"))
    with pytest.raises(Exception, match="patch merge failed! Gap in data exists"):
        lfp.process_time_range(T0, T0 + np.timedelta64(47, "s"))
    # the chunks before the gap were written, as the reference does
    assert 0 < len(os.listdir(tmp_path / "out")) == len(lfp.outputs)


@pytest.mark.gpu
@pytest.mark.parametrize("jitter_ns,merges", [(800_000, True), (2_400_000, False)])
def test_jittered_boundary_same_rule_resident_and_stream(tmp_path, jitter_ns, merges):
    """One continuity rule on both paths (chunk(time=None), tolerance 1.5
    samples): a 1.2-sample boundary gap merges onto the first file's sample
    grid whether the range is processed resident or streamed (identical
    outputs, equal to the oracle on the regular-grid series); a 1.6-sample
    gap raises the reference's gap error on both."""
    import lf_das
    import lfdas.dc as dc
    x = _write_archive(str(tmp_path / "raw"), jitter=(3, jitter_ns))
    t1, t2 = T0, T0 + np.timedelta64(6 * 8, "s") - np.timedelta64(4, "ms")
    res = {}
    for mode, budget in (("resident", None), ("stream", 1)):
        lfp = lf_das.LFProc(dc.spool(str(tmp_path / "raw")), max_resident_bytes=budget, verbose=False)
        lfp.update_processing_parameter(output_sample_interval=0.2, process_patch_size=40, edge_buff_size=6)
        lfp.set_output_folder(str(tmp_path / f"out_{mode}"))
        if not merges:
            with pytest.raises(Exception, match="patch merge failed! Gap in data exists"):
                lfp.process_time_range(t1, t2)
            res[mode] = len(lfp.outputs)
            continue
        lfp.process_time_range(t1, t2)
        assert lfp.last_mode == mode
        res[mode] = lfp.outputs
    if not merges:
        assert res["resident"] == res["stream"]
        return
    ref = oracle.lfproc_process(x.astype(np.float32), int(T0.astype(np.int64)), 4_000_000,
                                int(t1.astype(np.int64)), int(t2.astype(np.int64)), 0.2, 40, 6)
    assert len(res["resident"]) == len(res["stream"]) == len(ref)
    for a, b, (rt, ry) in zip(res["resident"], res["stream"], ref):
        np.testing.assert_array_equal(a.coords["time"].astype(np.int64), rt)
        np.testing.assert_array_equal(b.coords["time"].astype(np.int64), rt)
        gates.check("jitter_stream_vs_resident", _rel(b.data, a.data), gates.PATHS)
        gates.check("jitter_oracle", _rel(a.data, ry), gates.MFMA)
