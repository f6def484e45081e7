"""The multi-GPU driver with the DEVICE compute (lfdas.shard.
process_time_range_sharded, default ``lfproc_shard``): world_size-2 gloo
ranks, both on cuda:0 (a 1-GPU box cannot run RCCL with two ranks), each
running LFProc's device plan on its channel block and gathering the float32
device outputs.  Compared with the oracle's process_time_range over the
whole spool (relRMS <= 1e-4, identical times, the reference's files)."""
import os
import queue
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

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
                                              verbose=False)
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
            assert rel < 1e-4, rel
    # both ranks hold the identical full-width result (gathered float32)
    for (_, d0, _), (_, d1, _) in zip(got[0][3], got[1][3]):
        np.testing.assert_array_equal(d0, d1)
    files = sorted(os.listdir(out_dir))
    assert len(files) == 4 and all(f.startswith("LFDAS_2017-09-18T") for f in files)


def test_sharded_device_compute_world2_gap_raises_on_every_rank(tmp_path):
    got = _run(2, str(tmp_path / "o"), gap=2.0)
    assert [g[1] for g in got] == ["error", "error"]
    assert all("patch merge failed! Gap in data exists" in g[3] for g in got)
