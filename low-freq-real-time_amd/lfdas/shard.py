"""Channel sharding across GPUs (one process per GPU, torch.distributed).

Every op of the path is per channel, so ranks own contiguous channel ranges
and run the whole plan on their shard with no data-path exchange
(SURVEY §8e).  ``all_gather_channels`` assembles the decimated outputs (the
only collective; RCCL over xGMI with backend "nccl", gloo on CPU).

* ``process_time_range_sharded`` — the product's multi-GPU form of
  ``LFProc.process_time_range`` (lf_das.py:219-290, the single-process loop
  it replaces): rank r runs LFProc on ``spool.select(distance=...)`` of its
  channel block, then the per-chunk outputs are all-gathered and rank 0
  writes the reference's full-width files.
* ``shard_stream`` — the out-of-core form (cfg5 across 8 GPUs): every rank
  opens its own ``LowpassStream`` on its channel block and pushes its rows of
  each host block (``push_rows``); the streams never exchange data.
"""
from __future__ import annotations

import os

import numpy as np


def channel_range(n_ch: int, world: int, rank: int):
    """Contiguous ceil(n_ch/world) channel block of ``rank`` (may be empty)."""
    per = -(-int(n_ch) // int(world))
    c0 = min(rank * per, n_ch)
    return c0, min(c0 + per, n_ch)


def _grouped() -> bool:
    """A torch.distributed process group is initialised (any world size)."""
    try:
        import torch.distributed as dist
        return dist.is_available() and dist.is_initialized()
    except ImportError:  # pragma: no cover
        return False


def _world(group=None):
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_world_size(group), dist.get_rank(group)
    except ImportError:  # pragma: no cover
        pass
    return 1, 0


def all_gather_channels(y_local, n_ch: int, group=None):
    """Gather every rank's (n_local, n_out) block into (n_ch, n_out) on all
    ranks.  Blocks are padded to the common ceil(n_ch/world) height so a single
    fixed-size all_gather suffices."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    per = -(-int(n_ch) // world)
    pad = torch.zeros((per,) + tuple(y_local.shape[1:]), dtype=y_local.dtype, device=y_local.device)
    pad[: y_local.shape[0]] = y_local
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    return torch.cat(parts, 0)[:n_ch]


def gather_channels_to_root(y_local, n_ch: int, group=None, root: int = 0):
    """Gather every rank's (n_local, n_out) block into (n_ch, n_out) on rank
    ``root`` only (RCCL gather over xGMI on backend "nccl"); other ranks get
    ``None``.  Padded to ceil(n_ch/world) rows like ``all_gather_channels``."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    per = -(-int(n_ch) // world)
    pad = torch.zeros((per,) + tuple(y_local.shape[1:]), dtype=y_local.dtype, device=y_local.device)
    pad[: y_local.shape[0]] = y_local
    parts = [torch.empty_like(pad) for _ in range(world)] if rank == root else None
    dist.gather(pad, parts, dst=root, group=group)
    return torch.cat(parts, 0)[:n_ch] if rank == root else None


def shard_spool(sp, world: int, rank: int):
    """Rank ``rank``'s contiguous channel block of a spool, as
    ``Spool.select(distance=(d[c0], d[c1 - 1]))`` (inclusive, DASCore);
    returns (sub-spool or None when the block is empty, (c0, c1))."""
    d = np.asarray(sp[0].coords["distance"])
    c0, c1 = channel_range(len(d), world, rank)
    if c1 <= c0:
        return None, (c0, c1)
    return sp.select(distance=(d[c0], d[c1 - 1])), (c0, c1)


def lfproc_shard(sub, bgtime, edtime, params, device=None):
    """Default per-rank compute: LFProc on the rank's sub-spool (device plan,
    no files).  Returns the chunks' outputs as ONE float64 (channel, time)
    device tensor (``LFProc.process_time_range_device``), so the gather runs
    HBM to HBM; a range too large for the device budget streams through
    ``process_time_range`` and returns its output patches instead."""
    from .lf_das import LFProc
    lfp = LFProc(sub, device=device, verbose=False, write_files=False)
    lfp.update_processing_parameter(**params)
    res = lfp.process_time_range_device(bgtime, edtime)
    if res is not None:
        return res[0]
    lfp.process_time_range(bgtime, edtime)
    return lfp.outputs


def _shard_block(outs, counts, n_local, tdim):
    """This rank's outputs as one (n_local, sum(counts)) tensor: a device
    tensor from ``lfproc_shard`` as is (float64), output patches (an
    injected ``run_shard``) side by side in their own dtype.  Raises on a
    wrong chunk count or shape, so the error agreement covers it."""
    import torch
    total = int(sum(counts))
    if isinstance(outs, torch.Tensor):
        if tuple(outs.shape) != (n_local, total):
            raise ValueError(f"shard output {tuple(outs.shape)} != {(n_local, total)}")
        return outs
    if len(outs) != len(counts):
        raise ValueError(f"shard produced {len(outs)} chunks, the schedule has {len(counts)}")
    parts = []
    for out, cnt in zip(outs, counts):
        d = np.asarray(out.data)
        d = d.T if tdim == 0 else d
        if d.shape != (n_local, cnt):
            raise ValueError(f"shard chunk output {d.shape} != {(n_local, cnt)}")
        parts.append(d)
    return torch.from_numpy(np.ascontiguousarray(np.concatenate(parts, axis=1)))


def process_time_range_sharded(sp, bgtime, edtime, params=None, output_folder=None, group=None,
                               device=None, run_shard=None, gather=True, verbose=True):
    """``LFProc(sp).process_time_range(bgtime, edtime)`` over the ranks of the
    default process group: rank r processes channel block r (``shard_spool``)
    with ``run_shard(sub_spool, bgtime, edtime, params)`` (default
    ``lfproc_shard``: the device plan), and rank 0 writes the reference's
    full-width files (``LFDAS_<t0>_<t1>.h5``, lf_das.py:230-232) into
    ``output_folder``.  The decimated float64 outputs (SciPy's result dtype)
    move HBM to HBM over RCCL on backend "nccl" (through host memory on gloo):

    * ``gather=True`` (default) or ``"all"``: all-gathered; every rank
      returns the full-width patches;
    * ``gather="root"``: gathered to rank 0 only, the one rank that writes;
      rank 0 returns the full-width patches (one device→host copy of the
      full block, on rank 0 alone), every other rank its own block's;
    * ``gather=False``: no collective; every rank returns its own block (and
      nothing is written unless the run has one rank).

    A failure on any rank (e.g. the gap exception of lf_das.py:18) is raised
    on every rank, after the agreement collective, so no rank is left
    waiting."""
    import torch

    from . import schedule as S
    from .core import Patch
    from .lf_das import LFProc, _get_filename
    params = dict(params or {})
    world, rank = _world(group)
    para = LFProc(None)._default_process_parameters()
    para.update({k: v for k, v in params.items() if k in para})
    tg = S.time_grid(bgtime, edtime, para["output_sample_interval"])
    sched, kinds = S.lfproc_chunks(len(tg), para["process_patch_size"], para["edge_buff_size"], with_kind=True)
    counts = [ob - oa for _, _, oa, ob in sched]
    sub, (c0, c1) = shard_spool(sp, world, rank)
    run_shard = run_shard or (lambda s, a, b, p: lfproc_shard(s, a, b, p, device))
    p0 = sp[0]
    tdim = p0.dims.index("time")
    n_ch = len(np.asarray(p0.coords["distance"]))
    n_local = c1 - c0
    blk, err = None, None
    try:
        if sub is not None:
            blk = _shard_block(run_shard(sub, bgtime, edtime, params), counts, n_local, tdim)
        else:
            blk = torch.zeros((0, sum(counts)), dtype=torch.float64)
    except Exception as e:  # re-raised below, after every rank agreed
        err = e
    # (inside a process group the agreement and the gathers run at any world
    # size, world 1 included: the same RCCL / gloo calls as at world N)
    grouped = _grouped()
    if grouped:
        import torch.distributed as dist
        # the agreement: did any rank fail (every rank then raises)
        flag = torch.tensor([1 if err is not None else 0], dtype=torch.int64, device=_comm_device(group))
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
        if int(flag[0].item()):
            raise err if err is not None else RuntimeError("process_time_range failed on another rank")
    elif err is not None:
        raise err
    dtype = torch.float64  # DASCore's output dtype (an injected run_shard may return float32 patches)
    if gather not in (True, False, "all", "root"):
        raise ValueError('gather must be True / "all" (all-gather), "root" (to rank 0) or False')
    full = None
    if grouped and gather:
        # HBM to HBM over RCCL (backend "nccl"); host tensors over gloo
        t = blk.to(device=_comm_device(group), dtype=dtype)
        if gather is True or gather == "all":
            full = all_gather_channels(t, n_ch, group=group).cpu().numpy()
        else:
            g = gather_channels_to_root(t, n_ch, group=group)
            full = g.cpu().numpy() if g is not None else None
    full_width = full is not None or world == 1
    if full is None:
        full = blk.cpu().numpy()
    dist_coords = (np.asarray(p0.coords["distance"]) if full_width and world > 1 else
                   np.asarray(sub[0].coords["distance"]) if sub is not None else np.zeros(0))
    res = []
    j = 0
    attrs = p0._attrs_wo_coords()
    for i, ((_, _, oa, ob), cnt) in enumerate(zip(sched, counts), start=1):
        seg = np.asarray(full[:, j:j + cnt], dtype=np.float64)  # DASCore's output dtype
        coords = dict(p0.coords.coord_map)
        coords["distance"] = dist_coords
        coords["time"] = tg[oa:ob].astype("datetime64[ns]")
        out = Patch(data=seg.T.copy() if tdim == 0 else seg, coords=coords, dims=p0.dims,
                    attrs=attrs).update_attrs(d_time=para["output_sample_interval"])
        res.append(out)
        if rank == 0 and output_folder and full_width:
            if verbose:  # the reference's messages (lf_das.py:263,276,290)
                if kinds[i - 1] == "tail":
                    print(f"Processing patch {i} (Last portion of data)")
                else:
                    print("Processing patch ", str(i))
            os.makedirs(output_folder, exist_ok=True)
            out.io.write(os.path.join(output_folder, _get_filename(out.attrs["time_min"], out.attrs["time_max"])),
                         "dasdae")
        j += cnt
    return res


def _comm_device(group=None):
    """Tensors of the group's collectives live here (HBM for RCCL, host for gloo)."""
    import torch
    import torch.distributed as dist
    if dist.is_initialized() and dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def shard_stream(n_ch: int, sampling_interval_ns: int, group=None, **stream_kw):
    """This rank's ``LowpassStream`` over its channel block (out-of-core
    cfg5 across GPUs: one host→HBM stream per GPU, no data exchange).
    Returns (stream, (c0, c1)); push this rank's rows with ``push_rows``."""
    from .stream import LowpassStream
    world, rank = _world(group)
    c0, c1 = channel_range(n_ch, world, rank)
    if c1 <= c0:
        return None, (c0, c1)
    return LowpassStream(c1 - c0, sampling_interval_ns, **stream_kw), (c0, c1)


def pin_rows(block: np.ndarray, c_range):
    """Page-lock rows [c0, c1) of a full-width (channel, time) host block in
    place — this rank's part only, so N ranks that share one block's layout
    pin (and touch) only their own rows — and return the registration
    (``lfdas.stream.HostRegistration``; ``release()`` unpins).  Pushes of
    those rows (``push_rows``) are then one direct DMA each."""
    from .stream import register_host
    c0, c1 = c_range
    rows = block[c0:c1]
    if not rows.flags.c_contiguous:
        raise ValueError("pin_rows needs a C-contiguous (channel, time) block")
    return register_host(rows)


def push_rows(stream, block, c_range, t0, time_axis: int = 1):
    """Push rows [c0, c1) of a full-width host block (channel axis 0 for
    ``time_axis=1``, axis 1 for ``time_axis=0``) — a strided host view, no
    copy of the other ranks' channels."""
    c0, c1 = c_range
    view = block[c0:c1] if time_axis == 1 else block[:, c0:c1]
    return stream.push(view, t0, time_axis=time_axis)
