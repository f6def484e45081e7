"""Python handles over the C-ABI plans (include/lfdas.h).

Device buffers are torch CUDA tensors (PyTorch is plumbing here: HBM
allocation, streams, torch.distributed); every compute call goes through
liblfdas.so.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import check, load

# device launches of the low-pass path issued through this module (a plan
# execute, a one-shot fused call or a full-rate filter each count 1) — lets
# tests see how many passes a Python-level workflow turned into
launch_count = 0


def _count():
    global launch_count
    launch_count += 1


def _ptr(a) -> int:
    """Device pointer of a torch tensor (or None)."""
    return 0 if a is None else int(a.data_ptr())


def _stream_ptr(stream) -> int:
    if stream is None:
        import torch
        return int(torch.cuda.current_stream().cuda_stream)
    return int(getattr(stream, "cuda_stream", stream))


def _require_cuda(t, name, dtype=None):
    import torch
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TypeError(f"{name} must be a CUDA (HIP) torch tensor")
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if t.dim() != 2:
        raise ValueError(f"{name} must be 2-D (channel, time) addressed by strides")


class LowpassPlan:
    """Chunked zero-phase Butterworth low-pass + resample plan
    (``lfd_lowpass_plan_*``): the device form of
    ``LFProc.process_time_range`` (lf_das.py:219-290).

    ``grid_lo``/``grid_w``: output positions (sample index + fraction) in the
    coordinates of the device array; ``chunks``: ``(s0, s1, g0, g1)`` rows —
    inclusive sample range and output grid range of every chunk.
    Raises ``LFDUnsupported`` when the grid is not a uniform sample-aligned
    decimation grid (the host then uses the general full-rate path).
    """

    def __init__(self, sos, n_ch: int, n_t: int, grid_lo, grid_w, chunks, padlen: int = -1):
        lib = load()
        self._lib = lib
        self.sos = np.ascontiguousarray(sos, dtype=np.float64)
        self.n_sec = int(self.sos.shape[0])
        self.n_ch = int(n_ch)
        self.n_t = int(n_t)
        self.grid_lo = np.ascontiguousarray(grid_lo, dtype=np.int64)
        self.grid_w = np.ascontiguousarray(grid_w, dtype=np.float64)
        ch = np.ascontiguousarray(np.asarray(chunks, dtype=np.int64).reshape(-1, 4))
        self.chunks = ch
        h = ctypes.c_void_p()
        rc = lib.lfd_lowpass_plan_create(
            ctypes.byref(h), self.sos.ctypes.data, self.n_sec, int(padlen), self.n_ch,
            self.n_t, self.grid_lo.ctypes.data, self.grid_w.ctypes.data,
            len(self.grid_lo), ch.ctypes.data, ch.shape[0])
        check(rc)
        self._h = h
        ws = ctypes.c_size_t()
        nb = ctypes.c_int64()
        L = ctypes.c_int64()
        check(lib.lfd_lowpass_plan_info(h, ctypes.byref(ws), ctypes.byref(nb), ctypes.byref(L)))
        self.workspace_bytes = int(ws.value)
        self.n_blocks = int(nb.value)
        self.block_len = int(L.value)
        self.n_grid = len(self.grid_lo)

    def close(self):
        if getattr(self, "_h", None):
            if getattr(self, "_owned", True):
                # views handed out by lattice() die with the plan that owns
                # their C handle
                for v in getattr(self, "_views", ()):
                    v._h = None
                self._lib.lfd_lowpass_plan_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def alloc_workspace(self, device=None):
        import torch
        return torch.empty(max(self.workspace_bytes, 256), dtype=torch.uint8, device=device or "cuda")

    def execute(self, x, y, workspace, stream=None):
        """Run on device: ``x`` (n_ch, n_t) float32, ``y`` (n_ch, n_grid)
        float64 — SciPy's sosfiltfilt result dtype — (any strides),
        ``workspace`` >= workspace_bytes."""
        import torch
        _require_cuda(x, "x", torch.float32)
        _require_cuda(y, "y", torch.float64)
        if tuple(x.shape) != (self.n_ch, self.n_t):
            raise ValueError(f"x shape {tuple(x.shape)} != plan {(self.n_ch, self.n_t)}")
        if tuple(y.shape) != (self.n_ch, self.n_grid):
            raise ValueError(f"y shape {tuple(y.shape)} != {(self.n_ch, self.n_grid)}")
        if workspace.numel() * workspace.element_size() < self.workspace_bytes:
            raise ValueError("workspace too small")
        _count()
        check(self._lib.lfd_lowpass_execute(
            self._h, _ptr(x), x.stride(0), x.stride(1), _ptr(y), y.stride(0), y.stride(1),
            _ptr(workspace), _stream_ptr(stream)))

    def execute_split(self, x, y, workspace, block_stream, scan_stream):
        """``execute`` with the block pass (K1) on ``block_stream`` and the
        chunk scan + outputs on ``scan_stream`` after it
        (``lfd_lowpass_execute_split``): y is complete in scan_stream order,
        and the workspace is free once scan_stream has passed this call."""
        import torch
        _require_cuda(x, "x", torch.float32)
        _require_cuda(y, "y", torch.float64)
        if tuple(x.shape) != (self.n_ch, self.n_t):
            raise ValueError(f"x shape {tuple(x.shape)} != plan {(self.n_ch, self.n_t)}")
        if tuple(y.shape) != (self.n_ch, self.n_grid):
            raise ValueError(f"y shape {tuple(y.shape)} != {(self.n_ch, self.n_grid)}")
        if workspace.numel() * workspace.element_size() < self.workspace_bytes:
            raise ValueError("workspace too small")
        if block_stream is None or scan_stream is None:
            raise ValueError("execute_split needs both streams")
        _count()
        check(self._lib.lfd_lowpass_execute_split(
            self._h, _ptr(x), x.stride(0), x.stride(1), _ptr(y), y.stride(0), y.stride(1),
            _ptr(workspace), _stream_ptr(block_stream), _stream_ptr(scan_stream)))

    def last_timing_ms(self):
        a = ctypes.c_float()
        b = ctypes.c_float()
        check(self._lib.lfd_lowpass_last_timing(self._h, ctypes.byref(a), ctypes.byref(b)))
        return float(a.value), float(b.value)

    def timings_ms(self, n: int):
        """(K1 ms, scan ms) lists of the last ``n`` executes timed with
        ``set_timing(ring=n)`` (no host synchronisation between them)."""
        a = np.zeros(n, np.float32)
        b = np.zeros(n, np.float32)
        check(self._lib.lfd_lowpass_timings(self._h, a.ctypes.data, b.ctypes.data, int(n)))
        return [float(v) for v in a], [float(v) for v in b]

    def last_kernel(self) -> str:
        """Block-functional kernel of the last execute: "mfma_runs" (MFMA +
        run folding), "mfma_runs_tm" (the same for (time, channel) rows),
        "mfma" or "recurrence"; "recurrence_fold" / "mfma_fold" when a separate
        fold kernel turns their per-block functionals into runs (4th-order
        cascades)."""
        k = self._lib.lfd_lowpass_last_kernel(self._h)
        return {1: "recurrence", 2: "mfma", 3: "mfma_runs", 4: "recurrence_fold",
                5: "mfma_fold", 6: "mfma_runs_tm"}.get(k, "none")

    def last_scan(self) -> str:
        """Chunk scan of the last execute (``lfd_lowpass_last_scan``): "blocks"
        (no run folding), "in_chain", "deferred", "segmented" or "fused"."""
        k = self._lib.lfd_lowpass_last_scan(self._h)
        return {0: "blocks", 1: "in_chain", 2: "deferred", 3: "segmented", 4: "fused"}.get(k, "none")

    def runs(self):
        """(run_ks, run_len, RunConst record) or None without run mode — testing hook."""
        n = ctypes.c_int64()
        rc = self._lib.lfd_debug_runs(self._h, None, None, 0, ctypes.byref(n), None, 0)
        if rc == _lib.LFD_EUNSUPPORTED:
            return None
        check(rc)
        ks = np.zeros(n.value, np.int64)
        ln = np.zeros(n.value, np.int32)
        cst = np.zeros(1, _lib.RUN_CONST_DTYPE)
        check(self._lib.lfd_debug_runs(self._h, ks.ctypes.data, ln.ctypes.data, n.value, None,
                                       cst.ctypes.data, cst.nbytes))
        return ks, ln, cst[0]

    def block_taps(self):
        """Kx[n_comp, L + J] (F_c(k) = sum_p Kx[c, p] x[base + k L - J + p]) or
        None when the plan runs the recurrence kernel only — testing hook."""
        nc = ctypes.c_int()
        row = ctypes.c_int64()
        rc = self._lib.lfd_debug_block_taps(self._h, None, 0, ctypes.byref(nc), ctypes.byref(row))
        if rc == _lib.LFD_EUNSUPPORTED:
            return None
        check(rc)
        out = np.zeros((nc.value, row.value), np.float64)
        check(self._lib.lfd_debug_block_taps(self._h, out.ctypes.data, out.size, None, None))
        return out

    def lattice(self):
        """(n_offsets, whether the last execute ran the one-pass form, a view
        of the one-pass inner plan or None) of a lattice plan — testing hook."""
        n = ctypes.c_int64()
        last = ctypes.c_int32()
        inner = ctypes.c_void_p()
        check(self._lib.lfd_debug_lattice(self._h, ctypes.byref(n), ctypes.byref(last), ctypes.byref(inner)))
        view = None
        if inner.value:
            view = LowpassPlan.__new__(LowpassPlan)
            view._lib = self._lib
            view._h = inner
            view._owned = False  # owned by this plan
            view._parent = self  # the parent (owner of the C handle) outlives the view
            self.__dict__.setdefault("_views", []).append(view)
            view.chunks = self.chunks
            view.n_ch, view.n_t = self.n_ch, self.n_t
        return int(n.value), bool(last.value), view

    def constants(self):
        """(BlockConst, ScanConst, ChunkGeom[]) numpy records — testing hook."""
        bc = np.zeros(1, _lib.BLOCK_CONST_DTYPE)
        sc = np.zeros(1, _lib.SCAN_CONST_DTYPE)
        cg = np.zeros(self.chunks.shape[0], _lib.CHUNK_GEOM_DTYPE)
        check(self._lib.lfd_debug_plan_constants(
            self._h, bc.ctypes.data, bc.nbytes, sc.ctypes.data, sc.nbytes, cg.ctypes.data, cg.nbytes))
        return bc[0], sc[0], cg



class LowpassPipeline:
    """Back-to-back executes of one plan over a sequence of same-shape batches
    (consecutive time ranges, many records), overlapped on the device.  Every
    batch's block pass (K1) runs on one block stream, its chunk scan and
    outputs on a scan stream after it (``LowpassPlan.execute_split``), with
    the workspaces alternating: batch i's scan — latency-bound, a few hundred
    workgroups — runs beside batch i + 1's HBM-bound block pass instead of
    after it, and a workspace is handed to a new block pass only after the
    scan that read it (an event).  The block passes stay serialised (their
    HIP-event / rocprof durations are those of ``execute``).  Results are bit
    for bit those of ``plan.execute``.  The caller keeps ``x`` / ``y`` alive
    until ``synchronize()`` (or ``wait(stream)``) — they are used on the
    pipeline's streams."""

    def __init__(self, plan, device=None, depth: int = 2):
        import torch
        if depth < 1:
            raise ValueError("depth must be >= 1")
        self.plan = plan
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.ws = [plan.alloc_workspace(self.device) for _ in range(depth)]
        self.block = torch.cuda.Stream(self.device)
        self.scan = torch.cuda.Stream(self.device)
        self._done = [None] * depth
        self._i = 0

    def submit(self, x, y):
        """Queue one batch: ``y`` <- the plan's outputs of ``x``."""
        import torch
        j = self._i % len(self.ws)
        cur = torch.cuda.current_stream(self.device)
        self.block.wait_stream(cur)  # x written on the caller's stream
        self.scan.wait_stream(cur)   # y (and its earlier readers)
        if self._done[j] is not None:
            self.block.wait_event(self._done[j])  # the scan that last read ws[j]
        self.plan.execute_split(x, y, self.ws[j], self.block, self.scan)
        # the caching allocator must not hand x / y / ws[j] to another stream
        # before the pipeline's streams are past them (an x freed by the caller,
        # or the pipeline itself dropped, with batches in flight)
        for t in (x, y, self.ws[j]):
            t.record_stream(self.block)
            t.record_stream(self.scan)
        ev = torch.cuda.Event()
        ev.record(self.scan)
        self._done[j] = ev
        self._i += 1

    def wait(self, stream=None):
        """``stream`` (default: the current stream) waits for every queued batch."""
        import torch
        s = stream or torch.cuda.current_stream(self.device)
        s.wait_stream(self.block)
        s.wait_stream(self.scan)

    def synchronize(self):
        self.block.synchronize()
        self.scan.synchronize()

    def __del__(self):  # pragma: no cover
        # a dropped pipeline waits for its batches (its workspaces go back to
        # the allocator with it)
        try:
            self.synchronize()
        except Exception:
            pass

def set_timing(enable: bool, ring: int = 1):
    """HIP-event timing of executes; ``ring`` > 1 keeps the last ``ring``
    executes' times per plan (``LowpassPlan.timings_ms``)."""
    check(load().lfd_set_timing(max(1, int(ring)) if enable else 0))


def device_count() -> int:
    n = ctypes.c_int()
    check(load().lfd_device_count(ctypes.byref(n)))
    return int(n.value)


def sosfiltfilt_device(x, sos, padlen: int = -1, stream=None, y=None, ws=None):
    """Full-rate zero-phase filter on device → float64 tensor (n_ch, n_t)
    (``lfd_sosfiltfilt_f32``; DASCore ``pass_filter`` alone).  ``y`` / ``ws``:
    preallocated output and workspace (``lfd_sosfiltfilt_workspace_bytes``)."""
    import torch
    _require_cuda(x, "x", torch.float32)
    lib = load()
    sos = np.ascontiguousarray(sos, dtype=np.float64)
    n_ch, n_t = x.shape
    if ws is None:
        wsb = lib.lfd_sosfiltfilt_workspace_bytes(n_ch, n_t, int(padlen), sos.shape[0])
        ws = torch.empty(max(int(wsb), 256), dtype=torch.uint8, device=x.device)
    if y is None:
        y = torch.empty((n_ch, n_t), dtype=torch.float64, device=x.device)
    _count()
    check(lib.lfd_sosfiltfilt_f32(_ptr(x), n_ch, n_t, x.stride(0), x.stride(1), sos.ctypes.data,
                                  sos.shape[0], int(padlen), _ptr(y), y.stride(0), y.stride(1),
                                  _ptr(ws), _stream_ptr(stream)))
    return y


def sosfiltfilt_last_timing_ms():
    """(functionals, scan, output pass) kernel times of the last blocked
    ``sosfiltfilt_device`` call made with ``set_timing(True)``."""
    a, b, c = ctypes.c_float(), ctypes.c_float(), ctypes.c_float()
    check(load().lfd_sosfiltfilt_last_timing(ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
    return float(a.value), float(b.value), float(c.value)


def interp_device(yfull, lo, w, stream=None):
    """Device gather ``y[:, lo] + w*(y[:, lo+1]-y[:, lo])`` → float64."""
    import torch
    lib = load()
    lo_d = torch.as_tensor(np.ascontiguousarray(lo, dtype=np.int64), device=yfull.device)
    w_d = torch.as_tensor(np.ascontiguousarray(w, dtype=np.float64), device=yfull.device)
    n_ch, n_t = yfull.shape
    out = torch.empty((n_ch, len(lo)), dtype=torch.float64, device=yfull.device)
    check(lib.lfd_interp_linear_f64(_ptr(yfull), n_ch, n_t, yfull.stride(0), yfull.stride(1),
                                    _ptr(lo_d), _ptr(w_d), len(lo), _ptr(out), out.stride(0),
                                    out.stride(1), _stream_ptr(stream)))
    return out


def filtfilt_resample_device(x, sos, lo, w, padlen: int = -1, stream=None):
    """One-shot ``pass_filter(...).interpolate(...)`` of one patch on device
    (``lfd_sos_filtfilt_resample_f32``) → float64 (n_ch, n_out)."""
    import torch
    _require_cuda(x, "x", torch.float32)
    lib = load()
    sos = np.ascontiguousarray(sos, dtype=np.float64)
    lo = np.ascontiguousarray(lo, dtype=np.int64)
    w = np.ascontiguousarray(w, dtype=np.float64)
    n_ch, n_t = x.shape
    y = torch.empty((n_ch, len(lo)), dtype=torch.float64, device=x.device)
    _count()
    check(lib.lfd_sos_filtfilt_resample_f32(
        _ptr(x), n_ch, n_t, x.stride(0), x.stride(1), sos.ctypes.data, sos.shape[0], int(padlen),
        lo.ctypes.data, w.ctypes.data, len(lo), _ptr(y), y.stride(0), y.stride(1),
        _stream_ptr(stream)))
    return y


def fir_decimate_device(x, taps, q: int, delay: int, stream=None):
    """FIR decimation ``y[k] = sum_i taps[i] x[k q + delay - i]`` (zeros
    outside the record) → float64 (n_ch, ceil(n_t/q)) (``lfd_fir_decimate_f32``)."""
    import torch
    _require_cuda(x, "x", torch.float32)
    n_ch, n_t = x.shape
    h = torch.as_tensor(np.ascontiguousarray(taps, dtype=np.float64)).to(x.device)
    y = torch.empty((n_ch, -(-n_t // int(q))), dtype=torch.float64, device=x.device)
    if stream is not None:
        # the taps were copied on torch's current stream and are freed on
        # return: order the copy before the launch, and keep the memory from
        # being reused before the kernel on `stream` has read it
        ts = stream if hasattr(stream, "cuda_stream") else torch.cuda.ExternalStream(int(stream))
        ts.wait_stream(torch.cuda.current_stream(x.device))
        h.record_stream(ts)
        y.record_stream(ts)
    _count()
    check(load().lfd_fir_decimate_f32(_ptr(x), n_ch, n_t, x.stride(0), x.stride(1), _ptr(h), h.numel(),
                                      int(q), int(delay), _ptr(y), y.stride(0), y.stride(1),
                                      _stream_ptr(stream)))
    return y


def rolling_mean_device(x, window: int, step: int, stream=None):
    """Rolling mean at the subsampled output points → float32 (n_ch, ceil(n_t/step))."""
    import torch
    _require_cuda(x, "x", torch.float32)
    n_ch, n_t = x.shape
    n_out = -(-n_t // int(step))
    y = torch.empty((n_ch, n_out), dtype=torch.float32, device=x.device)
    check(load().lfd_rolling_mean_f32(_ptr(x), n_ch, n_t, x.stride(0), x.stride(1), int(window),
                                      int(step), _ptr(y), y.stride(0), y.stride(1),
                                      _stream_ptr(stream)))
    return y
