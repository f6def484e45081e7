"""The reference's four notebooks run end to end through the drop-in
(``import lfdas.dc as dc``, ``from lf_das import ...``) on a synthetic archive
of DASDAE files, against the oracle's restatement of the same loops.

* low_pass_dascore.ipynb cells 3-7, 11, 13 (batch: spool → select(distance,
  time) → LFProc.process_time_range → dc.spool(out).chunk(time=None)), for the
  resident and the out-of-core (streamed) LFProc paths;
* low_pass_dascore_edge.ipynb cell 11 (real-time: one new file per
  iteration, resume at get_last_processed_time() - (ceil(edge/d_t)-1)*d_t);
* rolling_mean_dascore(_edge).ipynb cell 9 (per-file rolling(time=d_t*s,
  step=d_t*s).mean() * scale_iDAS, written, merged, dropna('time')).

Tolerances: tests/gates.py for the float64 low-pass outputs (<= 10x the
measured relRMS; north_star's bar is 1e-4), <= 1e-6 for rolling means; output times identical.  The archive is (time, distance) like
the reference's raw files; the sleep between real-time runs is replaced by the
arrival of the next file."""
import os

import numpy as np
import pytest

import gates
import oracle

pytestmark = pytest.mark.gpu

T0 = np.datetime64("2023-03-22T06:00:00", "ns")
FS = 100.0
DT_NS = 10_000_000
FILE_S = 30
N_FILES = 6
N_CH = 32
CH_START, CH_END = 4, 28
GAUGE = 10.0


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(np.sum((a - b) ** 2) / np.sum(b ** 2)))


def _raw(seed=11):
    """(time, channel) float32 samples: noise plus slow sines below the new
    Nyquist, so the low-pass output is not just noise."""
    n = int(FILE_S * FS) * N_FILES
    rng = np.random.default_rng(seed)
    t = np.arange(n) / FS
    slow = np.sin(2 * np.pi * 0.07 * t)[:, None] * (1.0 + np.arange(N_CH) / N_CH)
    return (rng.standard_normal((n, N_CH)) + 3.0 * slow).astype(np.float32)


class _Archive:
    """The acquisition side: DASDAE files of FILE_S seconds each, (time,
    distance) layout, written into ``folder`` one at a time."""

    def __init__(self, folder, x):
        import lfdas.dc as dc
        self.dc = dc
        self.folder = folder
        self.x = x
        self.per = int(FILE_S * FS)
        self.dist = np.arange(N_CH) * 2.0 - 10.0
        self.written = 0
        os.makedirs(folder, exist_ok=True)

    def arrive(self):
        """Write the next file; False when the acquisition has ended."""
        i = self.written
        if i >= N_FILES:
            return False
        s = slice(i * self.per, (i + 1) * self.per)
        t = T0 + np.arange(s.start, s.stop) * np.timedelta64(DT_NS, "ns")
        p = self.dc.Patch(data=self.x[s], coords={"time": t, "distance": self.dist},
                          dims=("time", "distance"),
                          attrs={"gauge_length": GAUGE, "category": "DAS", "data_units": "rad/s"})
        p.io.write(os.path.join(self.folder, f"raw_{i:03d}.h5"), "dasdae")
        self.written += 1
        return True

    def sel(self):
        """Samples of the notebooks' sub-spool, (channel, time):
        select(distance=(d_1, d_2)) is inclusive of ch_end."""
        return np.ascontiguousarray(self.x[:, CH_START:CH_END + 1].T)


def _lowpass_params(sub_sp, sp):
    """low_pass_dascore*.ipynb cells 5, 7, 9."""
    import lf_das
    patch_0 = sp[0]
    sampling_interval = patch_0.attrs["step_time"]
    sampling_rate = 1 / (sampling_interval / np.timedelta64(1, "s"))
    num_sec = len(patch_0.coords["time"]) / sampling_rate
    memory_size = 4.61  # MB: a 40 s patch at this width
    patch_length = lf_das.get_patch_time(memory_size=memory_size, sampling_rate=sampling_rate,
                                         num_ch=CH_END - CH_START)
    d_t = 1.0
    tolerance = 1e-3
    edge_buffer = lf_das.get_edge_effect_time(sampling_interval=1 / sampling_rate, total_T=patch_length,
                                              tol=tolerance, freq=1 / d_t)
    assert abs(edge_buffer - oracle.get_edge_effect_time(1 / sampling_rate, patch_length, tol=tolerance,
                                                         freq=1 / d_t)) < 1e-9
    time_step_for_processing = max(125, num_sec)
    if time_step_for_processing < (2 * edge_buffer) * 1.5:
        time_step_for_processing = (2 * edge_buffer) * 1.5
        patch_length = min(patch_length, time_step_for_processing)
    assert sampling_rate == FS and num_sec == FILE_S
    return d_t, int(patch_length / d_t), int(np.ceil(edge_buffer / d_t)), edge_buffer


def _concat(chunks):
    t = np.concatenate([c[0] for c in chunks])
    y = np.concatenate([c[1] for c in chunks], axis=-1)
    return t, y


@pytest.mark.parametrize("mode", ["resident", "stream"])
def test_low_pass_notebook_batch(tmp_path, mode):
    import lfdas.dc as dc
    from lf_das import LFProc
    arch = _Archive(str(tmp_path / "data"), _raw())
    while arch.arrive():
        pass
    out_folder = str(tmp_path / "results")
    sp = dc.spool(arch.folder).sort("time").update()
    assert len(sp) == N_FILES
    patch_0 = sp[0]
    d_1 = patch_0.coords["distance"][CH_START]
    d_2 = patch_0.coords["distance"][CH_END]
    t_1 = T0 + np.timedelta64(5, "s")
    t_2 = T0 + np.timedelta64(170, "s")
    sub_sp = sp.select(distance=(d_1, d_2), time=(t_1, t_2))
    d_t, P, B, _ = _lowpass_params(sub_sp, sp)

    lfp = LFProc(sub_sp, verbose=False, max_resident_bytes=(1 if mode == "stream" else None))
    lfp.update_processing_parameter(output_sample_interval=d_t, process_patch_size=P, edge_buff_size=B)
    lfp.set_output_folder(out_folder, delete_existing=True)
    lfp.process_time_range(t_1, t_2)
    assert lfp.last_mode == mode

    ref = oracle.lfproc_process(arch.sel(), int(T0.astype(np.int64)), DT_NS, int(t_1.astype(np.int64)),
                                int(t_2.astype(np.int64)), d_t, P, B)
    assert len(lfp.outputs) == len(ref) and len(ref) >= 4
    for out, (tr, yr) in zip(lfp.outputs, ref):
        np.testing.assert_array_equal(out.coords["time"].astype(np.int64), tr)
        gates.check(f"notebook_batch {mode}", _rel(out.data.T, yr), gates.STREAM if mode == "stream" else gates.MFMA)

    # cell 13: read the results back and merge them into one patch
    sp_result = dc.spool(out_folder)
    sp_result = sp_result.chunk(time=None)
    assert len(sp_result) == 1
    sub_sp_result = sp_result.select(distance=(d_1, d_2))
    merged = sub_sp_result.chunk(time=None)[0]
    tr, yr = _concat(ref)
    np.testing.assert_array_equal(merged.coords["time"].astype(np.int64), tr)
    assert merged.dims == ("time", "distance") and merged.shape == (len(tr), CH_END - CH_START + 1)
    gates.check(f"notebook_batch_merged {mode}", _rel(merged.data.T, yr),
                gates.STREAM if mode == "stream" else gates.MFMA)
    assert merged.attrs["time_step"] == np.timedelta64(int(d_t * 1e9), "ns")


def test_low_pass_notebook_realtime(tmp_path):
    import lfdas.dc as dc
    from lf_das import LFProc
    arch = _Archive(str(tmp_path / "data"), _raw(seed=5))
    arch.arrive()
    data_path = arch.folder
    output_data_folder = str(tmp_path / "results")
    os.makedirs(output_data_folder)
    sp = dc.spool(data_path).sort("time").update()
    patch_0 = sp[0]
    d_1 = patch_0.coords["distance"][CH_START]
    d_2 = patch_0.coords["distance"][CH_END]
    sub_sp = sp.select(distance=(d_1, d_2))
    d_t, P, B, edge_buffer = _lowpass_params(sub_sp, sp)
    start_processing_time = T0

    # cell 11, with the next file's arrival in place of time.sleep
    runs = []
    initial_run = True
    while True:
        sp = dc.spool(data_path).update()
        sub_sp = sp.select(distance=(d_1, d_2))
        len_updated_sp = len(sub_sp)
        if not initial_run and len_last_sp == len_updated_sp:
            break
        lfp = LFProc(sub_sp, verbose=False)
        lfp.update_processing_parameter(output_sample_interval=d_t, process_patch_size=P, edge_buff_size=B)
        lfp.set_output_folder(output_data_folder, delete_existing=False)
        if initial_run:
            t_1 = start_processing_time
            t_2 = np.datetime64(sub_sp[-1].attrs["time_max"])
            lfp.process_time_range(t_1, t_2)
            initial_run = False
            len_last_sp = len(sub_sp)
        else:
            t_2 = lfp.get_last_processed_time()
            buffer = int((np.ceil(edge_buffer / d_t) - 1) * d_t)
            t_1 = t_2 - np.timedelta64(buffer, "s")
            t_2 = np.datetime64(sub_sp[-1].attrs["time_max"])
            lfp.process_time_range(t_1, t_2)
            len_last_sp = len(sub_sp)
        runs.append([(o.coords["time"].astype(np.int64), o.data.T) for o in lfp.outputs])
        arch.arrive()

    back_ns = int((np.ceil(edge_buffer / d_t) - 1) * d_t) * 1_000_000_000
    ref = oracle.edge_loop(arch.sel(), int(T0.astype(np.int64)), DT_NS, int(FILE_S * FS),
                           int(T0.astype(np.int64)), d_t, P, B, back_ns)
    assert len(runs) == len(ref) == N_FILES
    for got, exp in zip(runs, ref):
        assert len(got) == len(exp) >= 1
        for (tg, yg), (te, ye) in zip(got, exp):
            np.testing.assert_array_equal(tg, te)
            gates.check("notebook_realtime", _rel(yg, ye), gates.MFMA)

    # every run continues the previous one's output grid: one merged patch
    merged = dc.spool(output_data_folder).chunk(time=None)
    assert len(merged) == 1
    te, ye = _concat([c for run in ref for c in run])
    np.testing.assert_array_equal(merged[0].coords["time"].astype(np.int64), te)
    gates.check("notebook_realtime_merged", _rel(merged[0].data.T, ye), gates.MFMA)


@pytest.mark.parametrize("realtime", [False, True])
def test_rolling_mean_notebook(tmp_path, realtime):
    import lfdas.dc as dc
    from lf_das import _get_filename
    s = dc.units.s  # dascore.units.s (rolling notebooks cell 1)
    arch = _Archive(str(tmp_path / "data"), _raw(seed=8))
    if not realtime:
        while arch.arrive():
            pass
    else:
        arch.arrive()
    data_path = arch.folder
    output_data_folder = str(tmp_path / "results")
    os.makedirs(output_data_folder)
    sp = dc.spool(data_path).sort("time").update()
    patch_0 = sp[0]
    gauge_length = patch_0.attrs["gauge_length"]
    sampling_interval = patch_0.attrs["d_time"]
    sampling_rate = 1 / (sampling_interval / np.timedelta64(1, "s"))
    d_1 = patch_0.coords["distance"][CH_START]
    d_2 = patch_0.coords["distance"][CH_END]
    d_t = 10.0
    window = d_t * s
    step = d_t * s
    scale_iDAS = float((116 * sampling_rate / gauge_length) / 1e9)

    def work(patch):
        rolling_mean_patch = patch.rolling(time=window, step=step, engine="numpy").mean()
        new_scaled_patch = rolling_mean_patch.new(data=rolling_mean_patch.data * scale_iDAS)
        filename = _get_filename(new_scaled_patch.attrs["time_min"], new_scaled_patch.attrs["time_max"])
        new_scaled_patch.io.write(output_data_folder + "/" + filename, "dasdae")

    # rolling_mean_dascore_edge.ipynb cell 9 (the batch notebook is its first run)
    initial_run = True
    while True:
        sp = dc.spool(data_path).sort("time").update()
        sub_sp = sp.select(distance=(d_1, d_2))
        len_updated_sp = len(sub_sp)
        if not initial_run and len_last_sp == len_updated_sp:
            break
        if initial_run:
            for patch in sub_sp:
                work(patch)
            initial_run = False
        else:
            for j in range(len_last_sp, len_updated_sp):
                work(sub_sp[j])
        len_last_sp = len(sub_sp)
        arch.arrive()

    # rolling_mean_dascore.ipynb cell 9: merge the results and drop the NaN heads
    sp_result = dc.spool(output_data_folder).chunk(time=None)
    assert len(sp_result) == 1
    merged = sp_result[0].dropna("time")

    W = S = int(d_t * FS)
    x = arch.sel()
    per = arch.per
    ys, ts = [], []
    for i in range(N_FILES):
        seg = x[:, i * per:(i + 1) * per]
        y = oracle.rolling_mean(seg, W, S) * scale_iDAS
        t = oracle.rolling_out_times(int(T0.astype(np.int64)) + i * per * DT_NS, DT_NS, per, S)
        keep = ~np.isnan(y).any(axis=0)
        ys.append(y[:, keep])
        ts.append(t[keep])
    yr = np.concatenate(ys, axis=1)
    tr = np.concatenate(ts)
    np.testing.assert_array_equal(merged.coords["time"].astype(np.int64), tr)
    assert merged.shape == (len(tr), CH_END - CH_START + 1)
    gates.check(f"rolling_notebook realtime={realtime}", _rel(merged.data.T, yr), gates.ROLL)
