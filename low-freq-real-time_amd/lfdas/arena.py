"""Device sample buffers placed for the sample stream's address translation.

K1 (``k_block_runs_mfma``) reads 16 channel rows per wave instruction, rows
a whole record apart (7.2 MB at cfg3), so each instruction needs 16 page
translations.  On MI355X (ROCm 7.2) how many of those miss depends on the
size of the driver allocation the rows live in, not on the rows: the
1,250-channel cfg3 shard (9 GB, the N = 8 share) measured

* its own 9 GB (or 18 GB) allocation: UTCL1 translation misses 1.86 % of
  requests, K1 1.77-1.84 ms (0.63 of HBM);
* the first (or last) rows of a >= 32 GiB allocation: 0.76 %, K1 1.63-1.66 ms
  (0.68-0.69), in fresh processes, every time
  (``profiles/r05_narrow_tlb.txt``, ``profiles/r05_alloc_placement.txt``);

while the 72 GB headline input is that size already (no difference).
``device_samples`` therefore carves sample buffers of at least
``MIN_BYTES`` out of an allocation of at least ``POOL_BYTES`` (free HBM
permitting; 288 GB per GPU).  The view keeps its allocation alive; freed, the
block stays in torch's caching allocator, so the next buffer of the pool size
reuses the same placement.  Smaller buffers are ordinary ``torch.empty``.

It is OPT-IN (bench.py's sample buffers): the view's storage is the whole
pool, so a caller that holds many such buffers at once, or serialises one,
pays for the pool each time.  The library's own patch uploads
(``proc.to_device_ct``) use right-sized buffers.
"""
from __future__ import annotations

POOL_BYTES = 32 << 30  # allocation size from which the translation misses drop
MIN_BYTES = 1 << 30    # smaller buffers gain nothing measurable


def device_samples(shape, dtype=None, device=None):
    """An uninitialised (n_ch, n_t) device tensor (C-contiguous) for samples,
    placed in an allocation of >= POOL_BYTES when it is >= MIN_BYTES and the
    device has room for the pool."""
    import torch
    dtype = dtype or torch.float32
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    shape = tuple(int(s) for s in shape)
    n = 1
    for s in shape:
        n *= s
    nbytes = n * torch.empty((), dtype=dtype).element_size()
    if nbytes < MIN_BYTES or nbytes >= POOL_BYTES or dev.type != "cuda":
        return torch.empty(shape, dtype=dtype, device=dev)
    free, _ = torch.cuda.mem_get_info(dev)
    if POOL_BYTES > free * 0.9:
        return torch.empty(shape, dtype=dtype, device=dev)
    pool = torch.empty(POOL_BYTES, dtype=torch.uint8, device=dev)
    return pool[:nbytes].view(dtype).view(shape)
