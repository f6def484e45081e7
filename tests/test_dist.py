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
