"""Host-side index arithmetic of the low-pass path (no compute).

* ``time_grid``      — lf_das.py:252-256
* ``lfproc_chunks``  — the chunk loop of LFProc.process_time_range,
                       lf_das.py:258-290 (first chunk, body, tail)
* ``grid_positions`` — where each output time falls in the sample array
                       (what interp1d's searchsorted computes,
                       scipy/interpolate/_interpolate.py:457-484)
* ``select_range``   — Spool.select(time=(a, b)) is inclusive on both ends
                       (lf_das.py:236-240, 264-266), mapped to sample indices.
All times are int64 nanoseconds.
"""
from __future__ import annotations

import numpy as np


def to_ns(t) -> int:
    """datetime64 / int ns → int ns."""
    if isinstance(t, (int, np.integer)):
        return int(t)
    return int(np.datetime64(t, "ns").astype(np.int64))


def time_grid(bgtime, edtime, dt_s: float) -> np.ndarray:
    """``np.arange(bg, ed, np.timedelta64(int(dt*1000), 'ms'))`` in ns
    (lf_das.py:252-256; note the millisecond truncation of dt)."""
    step = int(dt_s * 1000) * 1_000_000
    if step <= 0:
        raise ValueError("output_sample_interval must be >= 1 ms")
    return np.arange(to_ns(bgtime), to_ns(edtime), step, dtype=np.int64)


def lfproc_chunks(n_grid: int, patch_size: int, buff_size: int, with_kind: bool = False):
    """Chunk schedule of lf_das.py:258-290: list of
    ``(read_first, read_last, out_begin, out_end)`` grid indices.  Chunk k
    selects ``time_grid[read_first] .. time_grid[read_last]`` (inclusive) and
    writes ``time_grid[out_begin:out_end]``.  (The reference loops forever
    when ``process_patch_size <= 2*edge_buff_size``; this raises instead.)"""
    L = int(n_grid)
    P = int(patch_size)
    B = int(buff_size)
    if L < 2:
        raise ValueError("time range holds fewer than 2 output samples")
    if L <= P:
        P = L - 1
    out = [(0, P, B, P - B)]
    kinds = ["first"]
    data_end = P
    new_data_end = data_end + P - 2 * B
    if new_data_end <= data_end and new_data_end < L:
        raise ValueError("process_patch_size must be larger than 2*edge_buff_size")
    while new_data_end < L:
        out.append((data_end - 2 * B, new_data_end, data_end - B, new_data_end - B))
        kinds.append("body")
        data_end = new_data_end
        new_data_end = data_end + P - 2 * B
    if (L - data_end) > 1:
        new_data_end = L - 1
        out.append((data_end - 2 * B, new_data_end, data_end - B, new_data_end - B))
        kinds.append("tail")
    return (out, kinds) if with_kind else out


def grid_positions(t0_ns: int, dt_ns: int, times_ns) -> tuple[np.ndarray, np.ndarray]:
    """Sample position of each time: ``lo`` (floor index) and ``w`` in
    [0, 1) with exact integer-ns arithmetic relative to the first sample."""
    rel = np.asarray(times_ns, dtype=np.int64) - np.int64(t0_ns)
    lo = rel // np.int64(dt_ns)
    rem = rel - lo * np.int64(dt_ns)
    return lo.astype(np.int64), rem.astype(np.float64) / float(dt_ns)


def select_range(t0_ns: int, dt_ns: int, n: int, a_ns: int, b_ns: int):
    """Inclusive sample index range [s0, s1] of times in [a, b] (clipped)."""
    s0 = -((-(int(a_ns) - int(t0_ns))) // int(dt_ns))  # ceil
    s1 = (int(b_ns) - int(t0_ns)) // int(dt_ns)         # floor
    return max(s0, 0), min(s1, n - 1)
