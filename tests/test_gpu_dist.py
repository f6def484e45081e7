"""The multi-GPU driver with the DEVICE compute (lfdas.shard.
process_time_range_sharded, default ``lfproc_shard``): world_size-2 gloo
ranks, both on cuda:0 (a 1-GPU box cannot run RCCL with two ranks), each
running LFProc's device plan on its channel block and gathering the float64
device outputs.  Compared with the oracle's process_time_range over the
whole spool (tests/gates.py, identical times, the reference's files).  The
RCCL branch (backend "nccl", HBM-to-HBM gathers) runs at world_size 1 on the
one GPU (test_rccl_world1_*)."""
import os
import queue
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import gates

pytestmark = pytest.mark.gpu

PARAMS = {"output_sample_interval": 0.2, "process_patch_size": 40, "edge_buff_size": 6}
T1, T2 = np.datetime64("2017-09-18T00:00:00"), np.datetime64("2017-09-18T00:00:23.996")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, out_dir, gap, dims, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        import lfdas.dc as dc
        from lfdas import plan as PL
        from lfdas.shard import process_time_range_sharded
        sp = dc.get_example_spool(time_gap=gap)
        if dims == ("time", "distance"):
            sp = dc.spool([p.new(data=np.ascontiguousarray(p.data.T), dims=dims) for p in sp])
        n0 = PL.launch_count
        try:
            outs = process_time_range_sharded(sp, T1, T2, PARAMS, output_folder=out_dir, device="cuda:0",
                                              gather="all", verbose=False)
            q.put((rank, "ok", PL.launch_count - n0,
                   [(o.coords["time"].astype(np.int64), o.data, o.dims) for o in outs]))
        except Exception as e:  # the agreed error, raised on every rank
            q.put((rank, "error", PL.launch_count - n0, str(e)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _run(world, out_dir, gap=0.0, dims=("distance", "time")):
    here = os.path.dirname(os.path.abspath(__file__))
    os.environ["PYTHONPATH"] = os.pathsep.join([here, os.path.dirname(here),
                                                os.path.join(os.path.dirname(here), "low-freq-real-time_amd"),
                                                os.environ.get("PYTHONPATH", "")])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, out_dir, gap, dims, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = []
    try:
        for _ in range(world):
            got.append(q.get(timeout=100))
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    except queue.Empty:
        pytest.fail("a rank did not report within 100 s")
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
    return sorted(got, key=lambda g: g[0])


def _oracle_outputs():
    import lfdas.dc as dc
    import oracle
    from lfdas import schedule as S
    merged = dc.spool(dc.get_example_spool()).chunk(time=None)[0]
    t = merged.sample_times_ns()
    return oracle.lfproc_process(np.asarray(merged.data, np.float32), int(t[0]), int(t[1] - t[0]),
                                 S.to_ns(T1), S.to_ns(T2), 0.2, 40, 6)


@pytest.mark.parametrize("dims", [("distance", "time"), ("time", "distance")])
def test_sharded_device_compute_world2_matches_oracle(tmp_path, dims):
    out_dir = str(tmp_path / "out")
    got = _run(2, out_dir, dims=dims)
    ref = _oracle_outputs()
    for rank, status, launches, outs in got:
        assert status == "ok", outs
        assert launches == 1  # ONE plan execute per rank for all 4 chunks
        assert len(outs) == len(ref) == 4
        for (t, d, odims), (rt, ry) in zip(outs, ref):
            np.testing.assert_array_equal(t, rt)
            d = d if odims[0] == "distance" else d.T
            assert d.shape == ry.shape == (300, len(rt))
            assert d.dtype == np.float64
            rel = float(np.sqrt(np.sum((d - ry) ** 2) / np.sum(ry ** 2)))
            gates.check(f"sharded_world2 {dims} rank{rank}", rel, gates.MFMA)
    # both ranks hold the identical full-width result (gathered float64)
    for (_, d0, _), (_, d1, _) in zip(got[0][3], got[1][3]):
        np.testing.assert_array_equal(d0, d1)
    files = sorted(os.listdir(out_dir))
    assert len(files) == 4 and all(f.startswith("LFDAS_2017-09-18T") for f in files)


def test_sharded_device_compute_world2_gap_raises_on_every_rank(tmp_path):
    got = _run(2, str(tmp_path / "o"), gap=2.0)
    assert [g[1] for g in got] == ["error", "error"]
    assert all("patch merge failed! Gap in data exists" in g[3] for g in got)


# --- the out-of-core form (cfg5 across GPUs: shard_stream + push_rows) ------

S_T0 = 1_679_464_800_000_000_000  # 2023-03-22T06:00:00 (the edge notebook's start)
S_FS, S_DT_NS = 200.0, 5_000_000  # cfg5: 200 Hz, dt = 10 s, P = 120, B = 6
S_NCH, S_PUSH, S_NPUSH = 37, 12_000, 48  # ragged 19 + 18 channels, 60 s pushes, 48 min


def _stream_block(k, time_major):
    """Full-width host block k of the synthetic spool (every rank makes the
    same one; only its own rows are pinned and pushed)."""
    import synth
    b = synth.noise_sine(S_NCH, S_PUSH, S_FS, seed=500 + k, dc=3.0)
    return np.ascontiguousarray(b.T) if time_major else b


def _stream_rank(rank, world, port, time_major, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from lfdas.shard import pin_rows, push_rows, shard_stream
        t_end = S_T0 + (S_PUSH * S_NPUSH - 1) * S_DT_NS
        st, (c0, c1) = shard_stream(S_NCH, S_DT_NS, output_sample_interval=10.0, process_patch_size=120,
                                    edge_buff_size=6, mode="continuous", t_start=S_T0, t_end=t_end,
                                    capacity=int(1300 * S_FS) + 2 * S_PUSH, device="cuda:0")
        st.reserve(S_PUSH)
        ys, ts, counts = [], [], []
        tax = 0 if time_major else 1
        pins = []
        try:
            for k in range(S_NPUSH):
                blk = _stream_block(k, time_major)
                if not time_major:  # this rank's rows page-locked in place: one direct DMA
                    pins.append(pin_rows(blk, (c0, c1)))
                o = push_rows(st, blk, (c0, c1), S_T0 + k * S_PUSH * S_DT_NS, time_axis=tax)
                if o.n_out:
                    ys.append(st.fetch())
                    ts.append(o.times_ns)
                    counts.extend(c for c in o.chunk_counts if c > 0)
                else:
                    st.wait_copy()
                for p in pins:
                    p.release()
                pins.clear()
            o = st.flush()
            if o.n_out:
                ys.append(st.fetch())
                ts.append(o.times_ns)
                counts.extend(c for c in o.chunk_counts if c > 0)
            st.synchronize()
        finally:
            for p in pins:
                p.release()
            st.close()
        q.put((rank, (c0, c1), np.concatenate(ys, axis=1), np.concatenate(ts), counts))
    except Exception as e:  # reported, so the test fails with the rank's error
        q.put((rank, None, repr(e), None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("time_major", [False, True])
def test_shard_stream_world2_device_matches_oracle(time_major):
    """cfg5 geometry (200 Hz, dt = 10 s, P = 120, B = 6) streamed in 60 s
    pushes through ``shard_stream`` + ``push_rows`` on two gloo ranks sharing
    cuda:0: each rank's device outputs for its channel block (19 + 18 of 37)
    equal the oracle's process_time_range over the whole spool (gates.STREAM
    per rank, on every channel incl. each block's first and last),
    with identical output times and chunk (file) boundaries."""
    here = os.path.dirname(os.path.abspath(__file__))
    os.environ["PYTHONPATH"] = os.pathsep.join([here, os.path.dirname(here),
                                                os.path.join(os.path.dirname(here), "low-freq-real-time_amd"),
                                                os.environ.get("PYTHONPATH", "")])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stream_rank, args=(r, 2, port, time_major, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = []
    try:
        for _ in range(2):
            got.append(q.get(timeout=100))
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    except queue.Empty:
        pytest.fail("a rank did not report within 100 s")
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
    got = sorted(got, key=lambda g: g[0])
    for g in got:
        assert g[1] is not None, g[2]
    import oracle
    x = np.concatenate([_stream_block(k, False) for k in range(S_NPUSH)], axis=1)
    ref = oracle.lfproc_process(x, S_T0, S_DT_NS, S_T0, S_T0 + (S_PUSH * S_NPUSH - 1) * S_DT_NS, 10.0, 120, 6)
    want = np.concatenate([r for _, r in ref], axis=1)
    want_t = np.concatenate([t for t, _ in ref])
    assert [g[1] for g in got] == [(0, 19), (19, 37)]
    for _, (c0, c1), y, t, counts in got:
        np.testing.assert_array_equal(t, want_t)
        assert counts == [len(tt) for tt, _ in ref if len(tt)]
        assert y.shape == (c1 - c0, want.shape[1])
        w = want[c0:c1]
        assert y.dtype == np.float64
        rel = float(np.sqrt(np.sum((y - w) ** 2) / np.sum(w ** 2)))
        gates.check(f"shard_stream tm={time_major} {c0}", rel, gates.STREAM)
        for r in (0, c1 - c0 - 1):  # the block's first and last channel alone
            rr = float(np.sqrt(np.sum((y[r] - w[r]) ** 2) / np.sum(w[r] ** 2)))
            gates.check(f"shard_stream tm={time_major} ch{c0 + r}", rr, gates.STREAM)


# --- the RCCL branch on the one GPU (backend "nccl", world_size 1) ----------

def _rccl_rank(port, out_dir, q):
    """One rank on backend "nccl": process_time_range_sharded with the
    all-gather (default) and the gather to rank 0, plus the gather helpers on
    HBM tensors — RCCL's all_gather / gather on device memory, the branch
    that the gloo tests never reach (_comm_device -> cuda)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        import lfdas.dc as dc
        from lfdas.shard import (_comm_device, all_gather_channels, gather_channels_to_root,
                                 process_time_range_sharded)
        assert dist.get_backend() == "nccl" and _comm_device().type == "cuda"
        sp = dc.get_example_spool()
        res = {}
        for mode in (True, "root", "all"):
            outs = process_time_range_sharded(sp, T1, T2, PARAMS, output_folder=out_dir if mode == "root" else None,
                                              device="cuda:0", gather=mode, verbose=False)
            res[str(mode)] = [(o.coords["time"].astype(np.int64), o.data) for o in outs]
        y = torch.arange(21 * 5, dtype=torch.float64, device="cuda").reshape(21, 5)
        a = all_gather_channels(y, 21)
        g = gather_channels_to_root(y, 21)
        ok = bool(a.is_cuda and g.is_cuda and torch.equal(a, y) and torch.equal(g, y))
        q.put(("ok", res, ok))
    except Exception as e:  # reported, so the test fails with the rank's error
        q.put(("error", repr(e), False))
    finally:
        dist.destroy_process_group()


def test_rccl_world1_sharded_driver_matches_oracle(tmp_path):
    """The "nccl" (RCCL) backend of the sharded driver, executed: one rank on
    the box's GPU gathers its device outputs HBM to HBM through RCCL's
    all_gather (gather=True / "all") and gather (gather="root"), and the
    results equal the oracle's process_time_range over the whole spool.  No
    scaling is claimed from it (one rank)."""
    here = os.path.dirname(os.path.abspath(__file__))
    os.environ["PYTHONPATH"] = os.pathsep.join([here, os.path.dirname(here),
                                                os.path.join(os.path.dirname(here), "low-freq-real-time_amd"),
                                                os.environ.get("PYTHONPATH", "")])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    out_dir = str(tmp_path / "rccl")
    p = ctx.Process(target=_rccl_rank, args=(_free_port(), out_dir, q))
    p.start()
    try:
        status, res, ok = q.get(timeout=100)
        p.join(timeout=60)
        assert p.exitcode == 0
    except queue.Empty:
        pytest.fail("the RCCL rank did not report within 100 s")
    finally:
        if p.is_alive():
            p.kill()
            p.join(timeout=10)
    assert status == "ok", res
    assert ok  # all_gather_channels / gather_channels_to_root on HBM tensors
    ref = _oracle_outputs()
    for mode, outs in res.items():
        assert len(outs) == len(ref) == 4, mode
        for (t, d), (rt, ry) in zip(outs, ref):
            np.testing.assert_array_equal(t, rt)
            assert d.shape == ry.shape == (300, len(rt)) and d.dtype == np.float64
            gates.check(f"rccl_world1 gather={mode}", gates.relrms(d, ry), gates.MFMA)
    files = sorted(os.listdir(out_dir))
    assert len(files) == 4 and all(f.startswith("LFDAS_2017-09-18T") for f in files)
