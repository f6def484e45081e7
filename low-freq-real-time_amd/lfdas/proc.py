"""Patch processing ops of the hot path, DASCore-compatible *(DASCore,
external)*, computed on the GPU by liblfdas.so:

* ``pass_filter(time=(lo, hi), corners=4, zerophase=True)`` — Butterworth SOS
  + ``sosfiltfilt`` semantics (lf_das.py:40, :223).  Lazy: the returned patch
  holds the filter; ``.interpolate`` fuses filter + resample into one device
  pass, touching ``.data`` runs the full-rate device filter.
* ``interpolate(time=array, kind='linear')`` — interp1d semantics
  (lf_das.py:42, :223-225).
* ``decimate(time=q, filter_type=None)`` — stride sub-sampling.
* ``rolling(time=w, step=s, engine='numpy').mean()`` — pandas-compatible
  right-aligned windows (rolling_mean_dascore.ipynb:148).
"""
from __future__ import annotations

import weakref

import numpy as np

from . import schedule as S
from .core import Patch, to_timedelta64
from .design import default_padlen, pass_filter_sos


def _get_torch_device(device=None):
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("lfdas needs a HIP device (MI355X); no CPU fallback")
    return torch.device(device if device is not None else "cuda")


def to_device_ct(patch: Patch, device=None, dtype=None):
    """Patch data as a float32 device tensor viewed as (channel, time) —
    strided view for dims ("time", ...), no host transpose."""
    import torch
    dev = _get_torch_device(device)
    d = patch.device_data()
    if patch.dims.index("time") == 0:
        perm = (1, 0)
    else:
        perm = (0, 1)
    dtype = dtype or torch.float32
    if isinstance(d, torch.Tensor):
        t = d.to(device=dev, dtype=dtype)
    else:
        a = np.asarray(d)
        if a.ndim != 2:
            raise ValueError("lfdas patches are 2-D (distance, time)")
        npdt = np.float32 if dtype == torch.float32 else np.float64
        # (a right-sized buffer: lfdas.arena's pooled placement is opt-in, for
        # callers that own their buffers' lifetime — bench.py's inputs)
        t = torch.empty(a.shape, dtype=dtype, device=dev)
        t.copy_(torch.from_numpy(np.ascontiguousarray(a, dtype=npdt)))
    return t.permute(*perm)


def _from_ct(y_ct, patch_dims):
    """(channel, time) device tensor → host array in the patch's dim order."""
    y = y_ct.detach().cpu().numpy()
    return y.T.copy() if patch_dims.index("time") == 0 else y


def _sampling_rate(patch: Patch) -> float:
    return 1.0 / (patch.sampling_interval_ns() / 1e9)


class _LazyFiltfilt:
    """Pending zero-phase filter of ``src`` (materialised on demand)."""

    def __init__(self, src: Patch, sos, padlen: int):
        self.src = src
        self.sos = np.ascontiguousarray(sos, dtype=np.float64)
        self.padlen = int(padlen)
        self.shape = src.shape

    def materialize(self, patch: Patch):
        from .plan import sosfiltfilt_device
        x = to_device_ct(self.src)
        y = sosfiltfilt_device(x, self.sos, self.padlen)
        return _from_ct(y, patch.dims)


def pass_filter(patch: Patch, corners=4, zerophase=True, **kwargs):
    if len(kwargs) != 1:
        raise ValueError("pass_filter takes exactly one dimension keyword, e.g. time=(None, 1.0)")
    (dim, rng), = kwargs.items()
    if dim != "time":
        raise NotImplementedError("only time-axis filtering is on the device path")
    if not zerophase:
        raise NotImplementedError("zerophase=False (causal sosfilt) is not on the device path")
    lo, hi = rng
    sos = pass_filter_sos(_sampling_rate(patch), lo, hi, corners)
    padlen = default_padlen(sos)
    n_t = patch.shape[patch.dims.index("time")]
    if n_t <= padlen:
        raise ValueError(f"The length of the input vector x must be greater than padlen, which is {padlen}.")
    return Patch(data=None, coords=patch.coords, dims=patch.dims,
                 attrs=patch._attrs_wo_coords(), _lazy=_LazyFiltfilt(patch, sos, padlen))


def _positions(patch: Patch, new_times):
    """(lo, w) of each requested time in the patch's sample grid, exact in
    integer ns; raises like interp1d(bounds_error=True) outside the data."""
    t = patch.sample_times_ns()
    tq = np.asarray(new_times).astype("datetime64[ns]").astype(np.int64)
    if tq.size and (tq.min() < t[0] or tq.max() > t[-1]):
        raise ValueError("A value in x_new is outside the interpolation range.")
    if tq.size > 1 and np.any(np.diff(tq) <= 0):
        raise ValueError("Interpolate requires monotonic increasing samples")
    dt = patch.sampling_interval_ns()
    lo, w = S.grid_positions(int(t[0]), dt, tq)
    # a point on the last sample has w == 0 at lo == n-1
    return lo, w


class ChunkGroup:
    """The windows ``Spool.chunk(time=T, overlap=O)`` cut from one merged
    patch (the reference's overlapping LFProc chunks, lf_das.py:236-240).
    ``window`` returns a window patch that remembers its sample range in the
    parent.  ``pass_filter(...).interpolate(...)`` on such windows registers a
    request here instead of computing at once; reading any of them computes
    every request registered so far together — one ``LowpassPlan`` execute
    over the parent's samples, each window a chunk of the plan (overlapping
    samples read from HBM once) — when their output grids interleave into one
    uniform grid, else one fused call per window."""

    def __init__(self, parent: Patch):
        self.parent = parent
        self.t_ns = parent.sample_times_ns()
        # requests not computed yet, held weakly: a window output thrown
        # away unread neither keeps its request alive nor joins a batch
        self.pending = weakref.WeakSet()

    def window(self, start, stop) -> Patch:
        """Inclusive time window [start, stop] of the parent."""
        p = self.parent.select(time=(start, stop))
        tw = p.sample_times_ns()
        if len(tw):
            s0 = int(np.searchsorted(self.t_ns, tw[0]))
            p._chunk_window = (self, s0, s0 + len(tw) - 1)
        return p

    def request(self, window, sos, padlen, lo, w, dims, shape):
        req = _GroupResample(self, window, sos, padlen, lo, w, dims, shape)
        self.pending.add(req)
        return req

    def _run(self, req):
        """Compute ``req`` with every pending sibling of the same cascade.
        Results are stored on the requests themselves (``_result``), and a
        request leaves ``pending`` only once its result is set, so a failed
        execute leaves the batch pending (the next read retries and raises
        the real error) and a request shared by several patches
        (``update_attrs`` copies) can be read any number of times."""
        batch = [r for r in list(self.pending)
                 if r._result is None and r.padlen == req.padlen and np.array_equal(r.sos, req.sos)]
        if req not in batch:
            batch.append(req)
        done = self._run_batched(batch) if len(batch) > 1 else False
        if not done:
            for r in batch:
                r._result = r.compute_alone()
        for r in batch:
            self.pending.discard(r)

    def _run_batched(self, batch) -> bool:
        """One plan over the parent for every request of ``batch``; False
        when their grids do not form one uniform, non-overlapping grid."""
        from ._lib import LFDUnsupported
        from .plan import LowpassPlan
        # order by the first output's position in the PARENT (r.lo is
        # window-relative: every LFProc window starts its outputs B grid
        # points in, so window-relative keys tie)
        batch = sorted(batch, key=lambda r: (r.s0 + int(r.lo[0]) + float(r.w[0])) if len(r.lo) else np.inf)
        if any(len(r.lo) == 0 for r in batch):
            return False
        lo = np.concatenate([r.lo + r.s0 for r in batch])
        w = np.concatenate([r.w for r in batch])
        pos = lo + w
        if np.any(np.diff(pos) <= 0):
            return False  # overlapping output grids: windows would write one column twice
        chunks, g = [], 0
        for r in batch:
            chunks.append((r.s0, r.s1, g, g + len(r.lo)))
            g += len(r.lo)
        n_t = len(self.t_ns)
        try:
            plan = LowpassPlan(batch[0].sos, _n_channels(self.parent), n_t, lo, w, chunks, batch[0].padlen)
        except (LFDUnsupported, ValueError):
            return False
        import torch
        x = to_device_ct(self.parent)
        y = torch.empty((x.shape[0], len(lo)), dtype=torch.float64, device=x.device)
        plan.execute(x, y, plan.alloc_workspace(x.device))
        plan.close()
        yh = y.cpu().numpy()
        for r, (_, _, g0, g1) in zip(batch, chunks):
            seg = yh[:, g0:g1]
            r._result = seg.T.copy() if r.dims.index("time") == 0 else seg
        return True


def _n_channels(patch: Patch) -> int:
    return int(np.prod([n for d, n in zip(patch.dims, patch.shape) if d != "time"]))


class _GroupResample:
    """A pending ``pass_filter(...).interpolate(...)`` of one chunk window."""

    def __init__(self, group, window, sos, padlen, lo, w, dims, shape):
        self.group = group
        self.window = window
        _, self.s0, self.s1 = window._chunk_window
        self.sos = np.ascontiguousarray(sos, dtype=np.float64)
        self.padlen = int(padlen)
        self.lo = np.asarray(lo, np.int64)
        self.w = np.asarray(w, np.float64)
        self.dims = tuple(dims)
        self.shape = tuple(shape)
        self._result = None

    def compute_alone(self):
        from .plan import filtfilt_resample_device
        x = to_device_ct(self.window)
        y = filtfilt_resample_device(x, self.sos, self.lo, self.w, self.padlen)
        return _from_ct(y, self.dims)

    def materialize(self, patch: Patch):
        if self._result is None:
            self.group._run(self)
        return self._result


def interpolate(patch: Patch, kind="linear", **kwargs):
    if kind != "linear":
        raise NotImplementedError("only linear interpolation is on the device path")
    if len(kwargs) != 1:
        raise ValueError("interpolate takes exactly one dimension keyword, e.g. time=array")
    (dim, new), = kwargs.items()
    if dim != "time":
        raise NotImplementedError("only time-axis interpolation is on the device path")
    new = np.asarray(new).astype("datetime64[ns]")
    lo, w = _positions(patch, new)
    coords = dict(patch.coords.coord_map)
    coords["time"] = new
    lazy = patch._lazy
    cw = getattr(lazy.src, "_chunk_window", None) if isinstance(lazy, _LazyFiltfilt) else None
    if cw is not None:
        # a Spool.chunk window: computed with its siblings on first read
        shape = list(patch.shape)
        shape[patch.dims.index("time")] = len(new)
        req = cw[0].request(lazy.src, lazy.sos, lazy.padlen, lo, w, patch.dims, shape)
        return Patch(data=None, coords=coords, dims=patch.dims, attrs=patch._attrs_wo_coords(), _lazy=req)
    if isinstance(lazy, _LazyFiltfilt):
        from .plan import filtfilt_resample_device
        x = to_device_ct(lazy.src)
        y = filtfilt_resample_device(x, lazy.sos, lo, w, lazy.padlen)
        data = _from_ct(y, patch.dims).astype(np.float64)
    else:
        from .plan import interp_device
        x = to_device_ct(patch, dtype=__import__("torch").float64)
        y = interp_device(x, lo, w)
        data = _from_ct(y, patch.dims).astype(np.float64)
    return Patch(data=data, coords=coords, dims=patch.dims, attrs=patch._attrs_wo_coords())


def decimate(patch: Patch, filter_type=None, **kwargs):
    """``Patch.decimate(time=q, filter_type=None | 'iir')``.  ``None``: every
    q-th sample.  ``'iir'``: restated as ``scipy.signal.decimate(x, q,
    ftype='iir', axis=time, zero_phase=True)`` — 8th-order Chebyshev I at
    0.8/q (designed on the host), zero-phase ``sosfiltfilt`` and the q-th
    sample pick fused in one device pass (``lfd_sos_filtfilt_resample_f32``,
    grid = every q-th sample).  ``'fir'``: ``scipy.signal.decimate(...,
    ftype='fir')`` = ``resample_poly`` with decimate's 20q+1-tap Hamming
    FIR (``_decimate_fir``).  *(DASCore, external: the wrapper is unpinned.)*"""
    if len(kwargs) != 1:
        raise ValueError("decimate takes exactly one dimension keyword, e.g. time=5")
    (dim, q), = kwargs.items()
    q = int(q)
    if q < 1:
        raise ValueError("decimation factor must be >= 1")
    ax = patch.dims.index(dim)
    coords = dict(patch.coords.coord_map)
    coords[dim] = coords[dim][::q]
    if filter_type in (None, False):
        idx = [slice(None)] * len(patch.dims)
        idx[ax] = slice(None, None, q)
        return Patch(data=patch.device_data()[tuple(idx)], coords=coords, dims=patch.dims,
                     attrs=patch._attrs_wo_coords())
    if str(filter_type).lower() not in ("iir", "fir"):
        raise ValueError(f"decimate filter_type={filter_type!r}: expected None, 'iir' or 'fir'")
    if dim != "time":
        raise NotImplementedError("only time-axis decimation is on the device path")
    import scipy.signal as _sig
    if str(filter_type).lower() == "fir":
        return _decimate_fir(patch, q, coords)

    from .plan import filtfilt_resample_device
    sos = np.ascontiguousarray(_sig.cheby1(8, 0.05, 0.8 / q, output="sos"), dtype=np.float64)
    padlen = default_padlen(sos)
    n_t = patch.shape[ax]
    if n_t <= padlen:
        raise ValueError(f"The length of the input vector x must be greater than padlen, which is {padlen}.")
    lo = np.arange(0, n_t, q, dtype=np.int64)
    w = np.zeros(len(lo))
    x = to_device_ct(patch)
    y = filtfilt_resample_device(x, sos, lo, w, padlen)
    data = _from_ct(y, patch.dims).astype(np.float64)
    return Patch(data=data, coords=coords, dims=patch.dims, attrs=patch._attrs_wo_coords())


def fir_decimate_design(q: int):
    """scipy.signal.decimate(ftype='fir')'s filter and resample_poly's
    centring (scipy/signal/_signaltools.py decimate: firwin(20q+1, 1/q,
    window='hamming'); resample_poly: n_pre_pad = q - half_len % q, output k
    = full-convolution index (k + (half_len + n_pre_pad) // q) q)."""
    import scipy.signal as _sig
    h = np.asarray(_sig.firwin(20 * q + 1, 1.0 / q, window="hamming"), dtype=np.float64)
    half = (h.size - 1) // 2
    pre_pad = q - half % q
    # resample_poly convolves with the pre-padded filter, so its leading
    # zeros stay in the taps: a NaN there gives NaN as in SciPy (0 * NaN)
    taps = np.concatenate([np.zeros(pre_pad), h])
    delay = (half + pre_pad) // q * q
    return taps, delay


def _decimate_fir(patch: Patch, q: int, coords) -> Patch:
    """``decimate(time=q, filter_type='fir')``: scipy.signal.decimate(x, q,
    ftype='fir', axis=time, zero_phase=True) = resample_poly(x, 1, q,
    window=firwin(20q+1, 1/q)) on the device (``lfd_fir_decimate_f32``:
    LDS-staged float64 FIR at the kept samples only)."""
    from .plan import fir_decimate_device
    taps, delay = fir_decimate_design(q)
    x = to_device_ct(patch)
    y = fir_decimate_device(x, taps, q, delay)
    return Patch(data=_from_ct(y, patch.dims), coords=coords, dims=patch.dims, attrs=patch._attrs_wo_coords())


def _to_samples(patch: Patch, v) -> int:
    if isinstance(v, (int, np.integer)) and not isinstance(v, bool):
        # DASCore treats plain numbers as coordinate units (seconds for time)
        v = float(v)
    td = to_timedelta64(v)
    dt = patch.sampling_interval_ns()
    n = int(round(int(td.astype(np.int64)) / dt))
    if n < 1:
        raise ValueError("rolling window/step shorter than one sample")
    return n


class _Roller:
    def __init__(self, patch: Patch, W: int, S_: int):
        self.patch = patch
        self.W = W
        self.S = S_

    def mean(self):
        from .plan import rolling_mean_device
        p = self.patch
        x = to_device_ct(p)
        y = rolling_mean_device(x, self.W, self.S)
        data = _from_ct(y, p.dims)
        src = p.device_data()
        if hasattr(src, "dtype") and np.dtype(str(src.dtype).replace("torch.", "")) == np.float64:
            data = data.astype(np.float64)
        coords = dict(p.coords.coord_map)
        coords["time"] = p.coords["time"][:: self.S]
        return Patch(data=data, coords=coords, dims=p.dims, attrs=p._attrs_wo_coords())


def rolling(patch: Patch, step=None, center=False, engine="numpy", **kwargs):
    if center:
        raise NotImplementedError("center=True rolling is not on the device path")
    if len(kwargs) != 1:
        raise ValueError("rolling takes one dimension keyword, e.g. time=10")
    (dim, window), = kwargs.items()
    if dim != "time":
        raise NotImplementedError("only time-axis rolling is on the device path")
    W = _to_samples(patch, window)
    S_ = 1 if step is None else _to_samples(patch, step)
    return _Roller(patch, W, S_)
