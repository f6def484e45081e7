"""Channel sharding across GPUs (one process per GPU, torch.distributed).

Every op of the path is per channel, so ranks own contiguous channel ranges
and run the whole plan on their shard with no data-path exchange
(SURVEY §8e).  ``all_gather_channels`` assembles the decimated outputs (the
only collective; RCCL over xGMI with backend "nccl", gloo on CPU)."""
from __future__ import annotations


def channel_range(n_ch: int, world: int, rank: int):
    """Contiguous ceil(n_ch/world) channel block of ``rank`` (may be empty)."""
    per = -(-int(n_ch) // int(world))
    c0 = min(rank * per, n_ch)
    return c0, min(c0 + per, n_ch)


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
