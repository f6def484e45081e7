"""DASDAE-layout HDF5 patch files (liblfdas_h5.so on the image's libhdf5):
the format step of lp_process (lf_das.py:230-232) and of
get_last_processed_time (lf_das.py:214-217).  DASCore/pytables are not
installed, so the layout follows DASCore's public DASDAE writer and
byte-level compatibility with DASCore's reader is unpinned; these tests pin
the round trip, the HDF5 structure (checked with h5dump) and the resume
rule."""
import os
import subprocess

import numpy as np
import pytest

from lfdas import io as lio

H5DUMP = "/opt/conda/bin/h5dump"
pytestmark = pytest.mark.skipif(not lio.h5_available(), reason="liblfdas_h5.so not built")


def _patch(dims=("distance", "time"), n_ch=7, n_t=50, t0="2023-03-22T03:00:00"):
    import lfdas.dc as dc
    t = np.datetime64(t0, "ns") + np.arange(n_t) * np.timedelta64(1, "s")
    data = np.random.default_rng(0).standard_normal((n_ch, n_t))
    if dims[0] == "time":
        data = data.T.copy()
    return dc.Patch(data=data, coords={"distance": np.arange(n_ch) * 1.02 - 115.0, "time": t}, dims=dims,
                    attrs={"station": "S8", "gauge_length": 10.2, "category": "DAS",
                           "time_step": np.timedelta64(1, "s"), "flag": True, "n_id": 42}).update_attrs(d_time=1.0)


@pytest.mark.parametrize("dims", [("distance", "time"), ("time", "distance")])
def test_round_trip_exact(tmp_path, dims):
    p = _patch(dims)
    fn = str(tmp_path / "LFDAS_2023-03-22T03_00_00_2023-03-22T03_00_49.h5")
    p.io.write(fn, "dasdae")
    with open(fn, "rb") as fh:
        assert fh.read(8) == b"\x89HDF\r\n\x1a\n"
    q = lio.read_patch(fn)
    assert q.dims == p.dims and q.shape == p.shape
    np.testing.assert_array_equal(q.data, p.data)
    for k, v in p.coords.coord_map.items():
        np.testing.assert_array_equal(q.coords[k], v)
        assert q.coords[k].dtype == np.asarray(v).dtype
    for k in ("station", "gauge_length", "category", "time_step", "flag", "n_id", "d_time",
              "time_min", "time_max"):
        assert q.attrs[k] == p.attrs[k] and type(q.attrs[k]) is type(p.attrs[k]) or q.attrs[k] == p.attrs[k]
    # header-only index: no samples read until used
    idx = lio.index_patch(fn)
    assert idx._data is None and idx.shape == p.shape
    np.testing.assert_array_equal(idx.data, p.data)


@pytest.mark.skipif(not os.path.exists(H5DUMP), reason="h5dump not in the image")
def test_layout_seen_by_h5dump(tmp_path):
    p = _patch()
    fn = str(tmp_path / "x.h5")
    p.io.write(fn, "dasdae")
    out = subprocess.run([H5DUMP, "-H", fn], capture_output=True, text=True, check=True).stdout
    assert 'GROUP "waveforms"' in out
    assert 'GROUP "DAS__' in out and '__S8__' in out
    for name in ('DATASET "data"', 'DATASET "_coord_time"', 'DATASET "_coord_distance"',
                 'ATTRIBUTE "__format__"', 'ATTRIBUTE "_dims"', 'ATTRIBUTE "_attrs_gauge_length"',
                 'ATTRIBUTE "is_datetime64"'):
        assert name in out, name
    vals = subprocess.run([H5DUMP, "-a", "/__format__", fn], capture_output=True, text=True).stdout
    assert '"DASDAE"' in vals


def test_folder_resume_rule_reads_hdf5(tmp_path):
    """get_last_processed_time (lf_das.py:214-217): the last output file's
    time_max, through the spool's header-only index."""
    import lf_das
    import lfdas.dc as dc
    for i in range(3):
        p = _patch(n_t=30, t0=str(np.datetime64("2023-03-22T03:00:00") + np.timedelta64(30 * i, "s")))
        fn = lf_das._get_filename(p.attrs["time_min"], p.attrs["time_max"])
        p.io.write(str(tmp_path / fn), "dasdae")
    lfp = lf_das.LFProc(dc.spool(str(tmp_path)))
    lfp.set_output_folder(str(tmp_path))
    assert lfp.get_last_processed_time() == np.datetime64("2023-03-22T03:01:29", "ns")


def test_npz_stand_in_still_readable(tmp_path):
    p = _patch()
    fn = str(tmp_path / "y.h5")
    p.io.write(fn, "npz")
    q = lio.read_patch(fn)
    np.testing.assert_array_equal(q.data, p.data)
