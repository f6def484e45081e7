"""Streaming low-pass + decimate with device-resident overlap
(``lfd_stream_*`` of include/lfdas.h).

* ``mode="edge"`` is the real-time loop of low_pass_dascore_edge.ipynb cell 11
  (:199-235): every push of new data runs ``LFProc.process_time_range(t_1,
  t_2)`` (lf_das.py:219-290) with ``t_2`` = newest sample time and ``t_1`` =
  ``get_last_processed_time()`` (lf_das.py:214-217) minus the notebook's
  ``buffer = int((ceil(edge_buffer/d_t) - 1) * d_t)`` seconds.  The reference
  re-reads that overlap from disk every run; here it never leaves HBM.
* ``mode="continuous"`` is one ``process_time_range(bgtime, edtime)`` over a
  spool pushed piece by piece (out-of-core: more data than HBM holds); chunks
  run as soon as their selection has arrived, ``flush()`` runs the tail.

Output samples, times and chunk (file) boundaries are those of the reference
loop; ``push_patch`` returns them as DASCore-style patches, one per LFProc
chunk, written to ``output_folder`` under the reference's file names when one
is set (``lp_process``, lf_das.py:221-232).
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import check, load
from .design import default_padlen, lowpass_sos


@dataclass
class StreamOutput:
    """What one push produced (``lfd_stream_last_output``)."""
    n_out: int
    t_first_ns: int
    t_step_ns: int
    chunk_counts: list = field(default_factory=list)
    n_runs: int = 0

    @property
    def times_ns(self) -> np.ndarray:
        return self.t_first_ns + np.arange(self.n_out, dtype=np.int64) * self.t_step_ns


# page-locked host ranges registered through ``register_host`` ([start, end))
_REGISTERED: dict = {}


def _in_registered(ptr: int, nbytes: int) -> bool:
    return any(a <= ptr and ptr + nbytes <= b for a, b in _REGISTERED.values())


def _is_pinned_host(a) -> bool:
    """True for pinned host memory: a pinned torch tensor, a numpy view of
    a ``pinned_empty`` buffer, or an array inside a ``register_host`` range."""
    try:
        import torch
        if isinstance(a, torch.Tensor):
            return bool(a.is_pinned())
    except ImportError:  # pragma: no cover
        pass
    if isinstance(a, np.ndarray) and _REGISTERED and a.size:
        lo = a.ctypes.data + sum(min(0, st * (n - 1)) for st, n in zip(a.strides, a.shape))
        hi = a.ctypes.data + sum(max(0, st * (n - 1)) for st, n in zip(a.strides, a.shape)) + a.itemsize
        if _in_registered(lo, hi - lo):
            return True
    b = a
    while b is not None:
        if getattr(b, "_lfd_owner", None) is not None:
            return True
        b = getattr(b, "base", None)
    return False


def _ns(t) -> int:
    if t is None:
        return 0
    if isinstance(t, (int, np.integer)):
        return int(t)
    return int(np.datetime64(t, "ns").astype(np.int64))


def notebook_resume_back_ns(edge_buffer_s: float, d_t: float) -> int:
    """``int((np.ceil(edge_buffer/d_t) - 1) * d_t)`` s of
    low_pass_dascore_edge.ipynb cell 11, in ns."""
    return int((math.ceil(edge_buffer_s / d_t) - 1) * d_t) * 1_000_000_000


class LowpassStream:
    """Device-resident streaming form of the LFProc low-pass path.

    ``sampling_interval_ns``: input sample spacing; ``output_sample_interval``,
    ``process_patch_size``, ``edge_buff_size``: LFProc's parameters
    (lf_das.py:197-204).  ``resume_back_ns`` defaults to the notebook's
    ``int((B - 1) * dt)`` seconds.  ``dry_run`` keeps only the host
    bookkeeping (no device; used by CPU tests of the schedule)."""

    def __init__(self, n_ch: int, sampling_interval_ns: int, output_sample_interval: float = 1.0,
                 process_patch_size: int = 100, edge_buff_size: int = 10, mode: str = "edge",
                 t_start=None, t_end=None, resume_back_ns: int | None = None, capacity: int = 0,
                 corners: int = 4, dry_run: bool = False, device=None):
        lib = load()
        self._lib = lib
        self.n_ch = int(n_ch)
        self.sample_ns = int(sampling_interval_ns)
        self.dt = float(output_sample_interval)
        fs = 1e9 / self.sample_ns
        self.sos = np.ascontiguousarray(lowpass_sos(fs, 1 / self.dt / 2 * 0.9, corners), dtype=np.float64)
        self.padlen = default_padlen(self.sos)
        if resume_back_ns is None:
            resume_back_ns = int((int(edge_buff_size) - 1) * self.dt) * 1_000_000_000
        if mode not in ("edge", "continuous"):
            raise ValueError("mode must be 'edge' or 'continuous'")
        if mode == "continuous" and (t_start is None or t_end is None):
            raise ValueError("continuous mode needs t_start and t_end (process_time_range bounds)")
        cfg = _lib.lfd_stream_config(
            n_ch=self.n_ch, sample_ns=self.sample_ns, output_sample_interval=self.dt,
            process_patch_size=int(process_patch_size), edge_buff_size=int(edge_buff_size),
            mode=_lib.LFD_STREAM_EDGE if mode == "edge" else _lib.LFD_STREAM_CONTINUOUS,
            flags=_lib.LFD_STREAM_DRY_RUN if dry_run else 0, t_start_ns=_ns(t_start),
            t_end_ns=_ns(t_end), resume_back_ns=int(resume_back_ns), capacity=int(capacity))
        self.mode = mode
        self.dry_run = bool(dry_run)
        self._dev_ctx = None
        if not dry_run:
            import torch
            if not torch.cuda.is_available():
                raise RuntimeError("lfdas needs a HIP device (MI355X); no CPU fallback")
            dev = torch.device(device if device is not None else "cuda")
            if dev.index is None:
                dev = torch.device("cuda", torch.cuda.current_device())
            self._dev_ctx = dev
            torch.cuda.set_device(dev)  # the stream lives on the current device
            torch.cuda.current_stream(dev)  # initialise the HIP context
        h = ctypes.c_void_p()
        check(lib.lfd_stream_open(ctypes.byref(h), ctypes.byref(cfg), self.sos.ctypes.data,
                                  self.sos.shape[0], self.padlen))
        self._h = h
        self._keep = []  # host buffers of pushes whose DMA may still be in flight

    # -- pushing -------------------------------------------------------
    def reserve(self, max_push: int):
        """Allocate the arena and staging for pushes of up to ``max_push``
        samples now (keeps allocation out of the first pushes)."""
        check(self._lib.lfd_stream_reserve(self._h, int(max_push)))

    def push(self, x, t0, time_axis: int = 1) -> StreamOutput:
        """Append host samples ``x`` (2-D, channels x time for ``time_axis=1``,
        time x channels for ``time_axis=0``; float32 numpy array or CPU torch
        tensor, pinned or pageable) starting at time ``t0``."""
        ptr, s_ch, s_t, n_t, keep = self._host_view(x, time_axis)
        check(self._lib.lfd_stream_push(self._h, ptr, n_t, s_ch, s_t, _ns(t0)))
        if _is_pinned_host(keep):
            # pinned pushes are DMA'd asynchronously: hold the buffer until the
            # next fetch / wait_copy / synchronize (pageable ones are staged
            # before push returns)
            self._keep.append(keep)
        return self.last_output()

    def flush(self) -> StreamOutput:
        """Continuous mode: run the schedule's remaining chunks."""
        check(self._lib.lfd_stream_flush(self._h))
        return self.last_output()

    def _host_view(self, x, time_axis):
        try:
            import torch
            is_t = isinstance(x, torch.Tensor)
        except ImportError:  # pragma: no cover
            is_t = False
        if is_t:
            if x.is_cuda:
                raise TypeError("push takes host memory (the stream owns the host->HBM copy)")
            if x.dtype != torch.float32 or x.dim() != 2:
                raise TypeError("push needs a 2-D float32 tensor")
            shape, strides, ptr, keep = tuple(x.shape), tuple(x.stride()), x.data_ptr(), x
        else:
            if self.dry_run and x is None:
                raise TypeError("x must be an array")
            a = np.asarray(x)
            if a.dtype != np.float32:
                a = a.astype(np.float32)
            if a.ndim != 2:
                raise ValueError("push needs a 2-D array")
            if not (a.strides[0 if time_axis == 0 else 1] == 4 or a.strides[1 if time_axis == 0 else 0] == 4):
                a = np.ascontiguousarray(a)
            shape, strides, ptr, keep = a.shape, tuple(s // 4 for s in a.strides), a.ctypes.data, a
        if time_axis == 1:
            n_ch, n_t = shape
            s_ch, s_t = strides
        else:
            n_t, n_ch = shape
            s_t, s_ch = strides
        if n_ch != self.n_ch:
            raise ValueError(f"push has {n_ch} channels, stream has {self.n_ch}")
        return ptr, s_ch, s_t, n_t, keep

    # -- results -------------------------------------------------------
    def last_output(self) -> StreamOutput:
        o = _lib.lfd_stream_output()
        check(self._lib.lfd_stream_last_output(self._h, ctypes.byref(o)))
        n = ctypes.c_int64()
        check(self._lib.lfd_stream_last_chunks(self._h, None, 0, ctypes.byref(n)))
        counts = np.zeros(max(n.value, 1), np.int64)
        check(self._lib.lfd_stream_last_chunks(self._h, counts.ctypes.data, counts.size, None))
        return StreamOutput(int(o.n_out), int(o.t_first_ns), int(o.t_step_ns),
                            [int(c) for c in counts[: n.value]], int(o.n_runs))

    def fetch(self, out: np.ndarray | None = None) -> np.ndarray:
        """Wait for the last push and copy its float64 outputs to host, (n_ch, n_out)."""
        o = self.last_output()
        if out is None:
            out = np.empty((self.n_ch, o.n_out), np.float64)
        if out.shape != (self.n_ch, o.n_out) or out.dtype != np.float64:
            raise ValueError("out must be float64 (n_ch, n_out)")
        check(self._lib.lfd_stream_fetch(self._h, out.ctypes.data, out.strides[0] // 8,
                                         max(out.strides[1] // 8, 1)))
        self._keep.clear()
        return out

    def wait_copy(self):
        """Block until the last push's host buffer has been copied to HBM."""
        check(self._lib.lfd_stream_wait_copy(self._h))
        self._keep.clear()

    def synchronize(self):
        check(self._lib.lfd_stream_synchronize(self._h))
        self._keep.clear()

    def last_timing_ms(self):
        """(host->HBM copy ms, run ms) of the last push (needs set_timing(True))."""
        a = ctypes.c_float()
        b = ctypes.c_float()
        check(self._lib.lfd_stream_last_timing(self._h, ctypes.byref(a), ctypes.byref(b)))
        return float(a.value), float(b.value)

    def info(self):
        """(arena capacity, samples held per channel, time of the first held sample)."""
        c, h, t = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        check(self._lib.lfd_stream_info(self._h, ctypes.byref(c), ctypes.byref(h), ctypes.byref(t)))
        return int(c.value), int(h.value), int(t.value)

    def plan_stats(self):
        """(plans built, plan-cache hits) of this stream (``lfd_debug_stream_plans``)."""
        c, h = ctypes.c_int64(), ctypes.c_int64()
        check(self._lib.lfd_debug_stream_plans(self._h, ctypes.byref(c), ctypes.byref(h)))
        return int(c.value), int(h.value)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.lfd_stream_close(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # -- DASCore surface -----------------------------------------------
    def push_patch(self, patch, output_folder: str | None = None):
        """Push a DASCore-style patch (dims ("distance","time") or
        ("time","distance")); returns the output patches of this push, one per
        LFProc chunk, like the files ``lp_process`` writes (lf_das.py:221-232)."""
        from .core import Patch
        from .lf_das import _get_filename
        t = patch.sample_times_ns()
        tax = patch.dims.index("time")
        data = np.asarray(patch.data, dtype=np.float32)
        o = self.push(data, int(t[0]), time_axis=tax)
        if o.n_out == 0:
            return []
        y = self.fetch()
        outs = []
        j = 0
        times = o.times_ns
        for cnt in o.chunk_counts:
            if cnt <= 0:
                continue
            seg = y[:, j:j + cnt]
            coords = dict(patch.coords.coord_map)
            coords["time"] = times[j:j + cnt].astype("datetime64[ns]")
            out = Patch(data=seg.T.copy() if tax == 0 else seg, coords=coords, dims=patch.dims,
                        attrs=patch._attrs_wo_coords()).update_attrs(d_time=self.dt)
            if output_folder:
                fn = _get_filename(out.attrs["time_min"], out.attrs["time_max"])
                out.io.write(output_folder + "/" + fn, "dasdae")
            outs.append(out)
            j += cnt
        return outs


def pinned_empty(shape, dtype=np.float32):
    """Pinned host numpy array (``lfd_host_alloc``): pushes from it are DMA'd
    directly.  The memory lives as long as the returned array."""
    lib = load()
    n = int(np.prod(shape)) * np.dtype(dtype).itemsize
    p = ctypes.c_void_p()
    check(lib.lfd_host_alloc(ctypes.byref(p), n))
    buf = (ctypes.c_char * n).from_address(p.value)
    arr = np.frombuffer(buf, dtype=dtype).reshape(shape)

    class _Owner:
        def __del__(self_inner):  # pragma: no cover
            lib.lfd_host_free(p)
    arr_owner = _Owner()
    # keep the owner alive with the buffer object
    buf._lfd_owner = arr_owner
    return arr


class HostRegistration:
    """A page-locked host range (``lfd_host_register``); ``release()`` (or
    garbage collection) unregisters it.  Keeps the array alive meanwhile."""

    def __init__(self, arr: np.ndarray):
        if not (isinstance(arr, np.ndarray) and arr.flags.c_contiguous and arr.size):
            raise ValueError("register_host needs a non-empty C-contiguous numpy array")
        self._lib = load()
        self.arr = arr
        self.ptr = int(arr.ctypes.data)
        check(self._lib.lfd_host_register(ctypes.c_void_p(self.ptr), arr.nbytes))
        _REGISTERED[self.ptr] = (self.ptr, self.ptr + arr.nbytes)

    def release(self):
        if _REGISTERED.pop(self.ptr, None) is not None:
            check(self._lib.lfd_host_unregister(ctypes.c_void_p(self.ptr)))
            self.arr = None

    def __del__(self):  # pragma: no cover
        try:
            self.release()
        except Exception:
            pass


def register_host(arr: np.ndarray) -> HostRegistration:
    """Page-lock an existing C-contiguous host array in place (e.g. one
    rank's rows of a full-width block): pushes from it are DMA'd directly,
    as from ``pinned_empty``."""
    return HostRegistration(arr)


def lfproc_schedule(n_grid: int, patch_size: int, buff_size: int):
    """``lfd_lfproc_schedule``: the native chunk schedule (lf_das.py:258-290)."""
    lib = load()
    n = ctypes.c_int64()
    check(lib.lfd_lfproc_schedule(int(n_grid), int(patch_size), int(buff_size), None, 0, ctypes.byref(n)))
    rows = np.zeros((n.value, 4), np.int64)
    check(lib.lfd_lfproc_schedule(int(n_grid), int(patch_size), int(buff_size), rows.ctypes.data,
                                  n.value, None))
    return [tuple(int(v) for v in r) for r in rows]
