"""N>1 path on CPU: world_size-2 gloo processes shard channels, compute their
slice (oracle stands in for the device plan here — CPU test of the sharding
and gather logic only) and all-gather the decimated outputs."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from lfdas.shard import all_gather_channels, channel_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_ch, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle
    import synth
    x = synth.noise_sine(n_ch, 6000, 250.0, seed=9)
    c0, c1 = channel_range(n_ch, world, rank)
    outs = oracle.lfproc_process(x[c0:c1], synth.T0_NS, 4_000_000, synth.T0_NS,
                                 synth.T0_NS + 6000 * 4_000_000, 0.2, 40, 6)
    y_local = torch.from_numpy(np.concatenate([o[1] for o in outs], axis=1))
    y = all_gather_channels(y_local, n_ch)
    if rank == 0:
        out_q.put(y.numpy())
    dist.barrier()
    dist.destroy_process_group()


def _oracle_shard(sub, bgtime, edtime, params):
    """CPU stand-in for the device compute of one rank (the oracle's
    process_time_range on the rank's merged sub-spool), returned as LFProc's
    output patches."""
    import lfdas.dc as dc
    import oracle
    from lfdas import schedule as S
    merged = dc.spool(sub).chunk(time=None)[0]
    t = merged.sample_times_ns()
    dt = params["output_sample_interval"]
    outs = oracle.lfproc_process(np.asarray(merged.data, np.float32), int(t[0]), int(t[1] - t[0]),
                                 S.to_ns(bgtime), S.to_ns(edtime), dt, params["process_patch_size"],
                                 params["edge_buff_size"])
    return [dc.Patch(data=y, coords={"distance": merged.coords["distance"], "time": tt.astype("datetime64[ns]")},
                     dims=merged.dims) for tt, y in outs]


PARAMS = {"output_sample_interval": 0.2, "process_patch_size": 40, "edge_buff_size": 6}
T1, T2 = np.datetime64("2017-09-18T00:00:00"), np.datetime64("2017-09-18T00:00:23.996")


def _sharded_worker(rank, world, port, out_dir, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import lfdas.dc as dc
    from lfdas.shard import process_time_range_sharded, shard_spool
    sp = dc.get_example_spool()  # 3 x (300 ch x 2000) @ 250 Hz
    sub, (c0, c1) = shard_spool(sp, world, rank)
    assert sub[0].shape[0] == c1 - c0
    outs = process_time_range_sharded(sp, T1, T2, PARAMS, output_folder=out_dir, run_shard=_oracle_shard,
                                      verbose=False)
    out_q.put((rank, (c0, c1), [(o.coords["time"].astype(np.int64), o.data) for o in outs]))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world3_sharded_lfproc_driver(tmp_path):
    """process_time_range_sharded over 3 gloo ranks (300 channels: 100 each):
    every rank gets the full-width outputs of every chunk, equal to one
    process over the whole spool; rank 0 wrote the reference's files."""
    here = os.path.dirname(os.path.abspath(__file__))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 3
    os.environ["PYTHONPATH"] = os.pathsep.join([here, os.path.dirname(here),
                                                os.path.join(os.path.dirname(here), "low-freq-real-time_amd"),
                                                os.environ.get("PYTHONPATH", "")])
    out_dir = str(tmp_path / "out")
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, out_dir, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    import lfdas.dc as dc
    sp = dc.get_example_spool()
    ref = _oracle_shard(dc.spool(sp), T1, T2, PARAMS)
    assert sorted(r for r, _, _ in got) == [0, 1, 2]
    assert [c for _, c, _ in sorted(got, key=lambda g: g[0])] == [(0, 100), (100, 200), (200, 300)]
    for _, _, outs in got:
        assert len(outs) == len(ref) == 4
        for (t, d), r in zip(outs, ref):
            np.testing.assert_array_equal(t, r.coords["time"].astype(np.int64))
            assert d.shape == (300, len(t))
            np.testing.assert_allclose(d, r.data, rtol=0, atol=1e-12)
    files = sorted(os.listdir(out_dir))
    assert len(files) == 4 and all(f.startswith("LFDAS_2017-09-18T") for f in files)
    back = dc.spool(out_dir)
    assert back[0].shape == (300, len(ref[0].coords["time"]))


def test_channel_range_covers_all():
    for n, w in [(10, 3), (7, 8), (10000, 8), (1, 2)]:
        got = [channel_range(n, w, r) for r in range(w)]
        assert got[0][0] == 0 and got[-1][1] == n
        for (a0, b0), (a1, b1) in zip(got, got[1:]):
            assert b0 == a1


def test_gloo_world2_shard_and_gather():
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    n_ch = 7  # ragged: 4 + 3
    os.environ["PYTHONPATH"] = os.pathsep.join([here, os.path.dirname(here),
                                                os.path.join(os.path.dirname(here), "low-freq-real-time_amd"),
                                                os.environ.get("PYTHONPATH", "")])
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_ch, q)) for r in range(2)]
    for p in procs:
        p.start()
    y = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    import oracle
    import synth
    x = synth.noise_sine(n_ch, 6000, 250.0, seed=9)
    ref = np.concatenate([o[1] for o in oracle.lfproc_process(
        x, synth.T0_NS, 4_000_000, synth.T0_NS, synth.T0_NS + 6000 * 4_000_000, 0.2, 40, 6)], axis=1)
    np.testing.assert_array_equal(y, ref)
    assert sys.modules  # keep linters quiet
