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
    # gather="root": gathered to rank 0 only (the writer); the others keep their block
    outs = process_time_range_sharded(sp, T1, T2, PARAMS, output_folder=out_dir, run_shard=_oracle_shard,
                                      gather="root", verbose=False)
    # default (gather=True, all-gather): every rank full width
    outs_all = process_time_range_sharded(sp, T1, T2, PARAMS, run_shard=_oracle_shard, verbose=False)
    out_q.put((rank, (c0, c1), [(o.coords["time"].astype(np.int64), o.data) for o in outs],
               [(o.coords["time"].astype(np.int64), o.data) for o in outs_all]))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world3_sharded_lfproc_driver(tmp_path):
    """process_time_range_sharded over 3 gloo ranks (300 channels: 100 each):
    with gather="root" rank 0 gets the full-width outputs of every chunk (the
    others their own 100-channel block), equal to one process over the whole
    spool, and wrote the reference's files; by default (all-gather) every rank
    gets the full width."""
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
    assert sorted(r for r, _, _, _ in got) == [0, 1, 2]
    assert [c for _, c, _, _ in sorted(got, key=lambda g: g[0])] == [(0, 100), (100, 200), (200, 300)]
    for rank, (c0, c1), outs, outs_all in got:
        assert len(outs) == len(outs_all) == len(ref) == 4
        for (t, d), (ta, da), r in zip(outs, outs_all, ref):
            np.testing.assert_array_equal(t, r.coords["time"].astype(np.int64))
            np.testing.assert_array_equal(ta, t)
            assert da.shape == (300, len(t))
            np.testing.assert_allclose(da, r.data, rtol=0, atol=1e-12)
            want = r.data if rank == 0 else r.data[c0:c1]
            assert d.shape == want.shape
            np.testing.assert_allclose(d, want, rtol=0, atol=1e-12)
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


def _stream_worker(rank, world, port, n_ch, push, n_push, out_q):
    """One rank of the out-of-core cfg5 form (``shard_stream`` + ``push_rows``)
    in dry-run mode: the rank's bookkeeping per push."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from lfdas.shard import push_rows, shard_stream
    st, rng = shard_stream(n_ch, 10_000_000, output_sample_interval=1.0, process_patch_size=40,
                           edge_buff_size=5, mode="continuous", t_start=STREAM_T0,
                           t_end=STREAM_T0 + (push * n_push - 1) * 10_000_000, dry_run=True)
    rec = []
    block = np.zeros((n_ch, push), np.float32)  # full-width host block
    for k in range(n_push):
        o = push_rows(st, block, rng, STREAM_T0 + k * push * 10_000_000)
        rec.append((o.n_out, o.t_first_ns if o.n_out else 0, tuple(o.chunk_counts)))
    o = st.flush()
    rec.append((o.n_out, o.t_first_ns if o.n_out else 0, tuple(o.chunk_counts)))
    # time-major full-width blocks go through the strided view of the rank's columns
    st2, _ = shard_stream(n_ch, 10_000_000, output_sample_interval=1.0, process_patch_size=40,
                          edge_buff_size=5, mode="edge", t_start=STREAM_T0, dry_run=True)
    o2 = push_rows(st2, np.zeros((push, n_ch), np.float32), rng, STREAM_T0, time_axis=0)
    out_q.put((rank, rng, st.n_ch, rec, o2.n_out))
    st.close()
    st2.close()
    dist.barrier()
    dist.destroy_process_group()


STREAM_T0 = 1_679_464_800_000_000_000


def test_gloo_world2_shard_stream_dry_run_matches_single_stream():
    """cfg5 across GPUs (``shard_stream`` / ``push_rows``) on 2 gloo ranks in
    dry-run mode: each rank's stream owns its ragged channel block (4 + 3 of
    7) and produces per push exactly the outputs, times and chunk (file)
    boundaries of ONE stream over all channels."""
    import lfdas.stream as ST
    here = os.path.dirname(os.path.abspath(__file__))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    n_ch, push, n_push = 7, 2_000, 9  # 100 Hz, 20 s pushes, 180 s
    os.environ["PYTHONPATH"] = os.pathsep.join([here, os.path.dirname(here),
                                                os.path.join(os.path.dirname(here), "low-freq-real-time_amd"),
                                                os.environ.get("PYTHONPATH", "")])
    procs = [ctx.Process(target=_stream_worker, args=(r, 2, port, n_ch, push, n_push, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted([q.get(timeout=180) for _ in range(2)], key=lambda g: g[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    one = ST.LowpassStream(n_ch, 10_000_000, 1.0, 40, 5, mode="continuous", t_start=STREAM_T0,
                           t_end=STREAM_T0 + (push * n_push - 1) * 10_000_000, dry_run=True)
    ref = []
    for k in range(n_push):
        o = one.push(np.zeros((n_ch, push), np.float32), STREAM_T0 + k * push * 10_000_000)
        ref.append((o.n_out, o.t_first_ns if o.n_out else 0, tuple(o.chunk_counts)))
    o = one.flush()
    ref.append((o.n_out, o.t_first_ns if o.n_out else 0, tuple(o.chunk_counts)))
    assert [g[1] for g in got] == [(0, 4), (4, 7)]
    assert [g[2] for g in got] == [4, 3]
    assert sum(r[0] for r in ref) > 0
    for _, _, _, rec, n_edge in got:
        assert rec == ref
        assert n_edge > 0


def test_bench_refuses_more_gpus_than_present_and_launcher_mismatch():
    """``bench.py --gpus 2`` on a node without 2 GPUs fails clearly and prints
    no JSON line (never an N = 1 line for an N > 1 request); under a launcher
    a WORLD_SIZE that differs from --gpus is refused."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""  # no device: the refusal needs no GPU
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 2 and "needs 2 GPUs" in r.stderr and "{" not in r.stdout
    env["WORLD_SIZE"] = "4"
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 2 and "WORLD_SIZE=4" in r.stderr and "{" not in r.stdout


def test_sharded_driver_prints_reference_messages(tmp_path, capsys):
    """Rank 0 prints the reference's per-chunk messages, the tail chunk as
    ``Processing patch {i} (Last portion of data)`` (lf_das.py:263,276,290)."""
    import lfdas.dc as dc
    from lfdas.shard import process_time_range_sharded
    process_time_range_sharded(dc.get_example_spool(), T1, T2, PARAMS, output_folder=str(tmp_path / "o"),
                               run_shard=_oracle_shard, verbose=True)
    lines = [ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("Processing patch")]
    assert lines == ["Processing patch  1", "Processing patch  2", "Processing patch  3",
                     "Processing patch 4 (Last portion of data)"]


def _random_world_worker(rank, world, port, n_ch, seed, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import lfdas.dc as dc
    import synth
    from lfdas.shard import process_time_range_sharded, shard_spool
    x = synth.noise_sine(n_ch, 6000, 250.0, seed=seed)
    t = (np.datetime64(synth.T0_NS, "ns") + np.arange(6000) * np.timedelta64(4_000_000, "ns"))
    sp = dc.spool([dc.Patch(data=x, coords={"distance": np.arange(float(n_ch)), "time": t},
                            dims=("distance", "time"))])
    sub, (c0, c1) = shard_spool(sp, world, rank)
    outs = process_time_range_sharded(sp, T1, T2, PARAMS, run_shard=_oracle_shard, verbose=False)
    out_q.put((rank, (c0, c1), sub is None, [np.asarray(o.data) for o in outs]))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_random_worlds_including_empty_shards():
    """Seeded random (world, channel count) pairs, including more ranks than
    channels (ranks with an empty shard): every rank gets the full-width
    outputs of every chunk from the all-gather, equal to one process over
    the whole spool."""
    import lfdas.dc as dc
    import synth
    here = os.path.dirname(os.path.abspath(__file__))
    os.environ["PYTHONPATH"] = os.pathsep.join([here, os.path.dirname(here),
                                                os.path.join(os.path.dirname(here), "low-freq-real-time_amd"),
                                                os.environ.get("PYTHONPATH", "")])
    ctx = mp.get_context("spawn")
    for world, n_ch, seed in [(3, 2, 1), (4, 7, 2), (2, 13, 3)]:
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_random_world_worker, args=(r, world, port, n_ch, seed, q)) for r in range(world)]
        for p in procs:
            p.start()
        got = [q.get(timeout=180) for _ in range(world)]
        for p in procs:
            p.join(timeout=120)
            assert p.exitcode == 0
        x = synth.noise_sine(n_ch, 6000, 250.0, seed=seed)
        t = (np.datetime64(synth.T0_NS, "ns") + np.arange(6000) * np.timedelta64(4_000_000, "ns"))
        sp = dc.spool([dc.Patch(data=x, coords={"distance": np.arange(float(n_ch)), "time": t},
                                dims=("distance", "time"))])
        ref = _oracle_shard(sp, T1, T2, PARAMS)
        empties = sum(1 for _, _, e, _ in got if e)
        assert empties == max(0, world - -(-n_ch // -(-n_ch // world)))
        for rank, (c0, c1), empty, outs in got:
            assert len(outs) == len(ref)
            for d, r in zip(outs, ref):
                assert d.shape == r.data.shape
                np.testing.assert_allclose(d, r.data, rtol=0, atol=1e-12)
