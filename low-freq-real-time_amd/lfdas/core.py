"""Minimal DASCore-compatible data model: ``Patch`` and ``Spool``.

Only what the reference's hot path touches *(DASCore, external; v0.0.13
per README.md:8)*:

* ``Patch(data, coords, dims, attrs)`` (lf_das.py:60), ``.data``, ``.dims``,
  ``.coords[...]`` / ``.coords.get_array``, ``.attrs['time_min'|'time_max'|
  'time_step'|'d_time'|...]``, ``.new``, ``.update_attrs`` (lf_das.py:227),
  ``.pipe`` (lf_das.py:61), ``.select``, ``.dropna`` (rolling nb:189),
  ``.pass_filter`` / ``.interpolate`` / ``.decimate`` / ``.rolling`` (lfdas.proc),
  ``.io.write(path, 'dasdae')`` (lf_das.py:232);
* ``spool(...)``, ``Spool.select`` (inclusive), ``.chunk(time=None)`` (merge,
  lf_das.py:239, 265), ``.chunk(time=T, overlap=O)``, ``.sort``, ``.update``,
  ``len``/indexing/iteration, ``.get_contents()``.

Patch data may live on the host (numpy) or in HBM (torch CUDA tensor); the
low-pass path keeps it lazy so ``pass_filter(...).interpolate(...)`` runs as
one fused device pass (lfdas.proc).
"""
from __future__ import annotations

import os
from collections.abc import Mapping

import numpy as np

_TIME_ALIASES = {"d_time": "time_step", "step_time": "time_step"}
_DIST_ALIASES = {"d_distance": "distance_step", "step_distance": "distance_step"}


def to_datetime64(obj):
    """*(DASCore, external)* ``dc.to_datetime64``: float seconds (since the
    epoch) → datetime64[ns]; strings / datetime64 pass through numpy."""
    arr = np.asarray(obj)
    if arr.dtype.kind in "fi":
        ns = np.round(arr.astype(np.float64) * 1e9).astype(np.int64)
        out = ns.astype("datetime64[ns]")
        return out if arr.ndim else out[()]
    if arr.dtype.kind in "US":
        return np.asarray(arr, dtype="datetime64[ns]") if arr.ndim else np.datetime64(str(arr), "ns")
    return arr.astype("datetime64[ns]") if arr.ndim else np.datetime64(arr[()], "ns")


def to_timedelta64(obj):
    if isinstance(obj, np.timedelta64):
        return obj.astype("timedelta64[ns]")
    if hasattr(obj, "to") and hasattr(obj, "magnitude"):  # quantity-like (lfdas.units)
        obj = float(obj.to("s").magnitude)
    return np.timedelta64(int(round(float(obj) * 1e9)), "ns")


class FrozenDict(Mapping):
    """Immutable mapping (dascore.utils.mapping.FrozenDict, lf_das.py:12)."""

    def __init__(self, *a, **kw):
        self._d = dict(*a, **kw)

    def __getitem__(self, k):
        return self._d[k]

    def __iter__(self):
        return iter(self._d)

    def __len__(self):
        return len(self._d)

    def __repr__(self):
        return f"FrozenDict({self._d!r})"


class PatchAttrs(Mapping):
    """Read-only attribute mapping with DASCore's name aliases."""

    def __init__(self, d):
        self._d = dict(d)

    def _key(self, k):
        if k in self._d:
            return k
        for src, dst in list(_TIME_ALIASES.items()) + list(_DIST_ALIASES.items()):
            if k == src and dst in self._d:
                return dst
            if k == dst and src in self._d:
                return src
        return k

    def __getitem__(self, k):
        return self._d[self._key(k)]

    def __getattr__(self, k):
        if k.startswith("_"):
            raise AttributeError(k)
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __iter__(self):
        return iter(self._d)

    def __len__(self):
        return len(self._d)

    def get(self, k, default=None):
        try:
            return self[k]
        except KeyError:
            return default

    def to_dict(self):
        return dict(self._d)

    def __repr__(self):
        return f"PatchAttrs({self._d!r})"


class Coords(Mapping):
    """Coordinate arrays by name (``time`` is datetime64[ns])."""

    def __init__(self, coords, dims):
        self._c = {}
        for k, v in dict(coords).items():
            arr = np.asarray(v)
            if k == "time" and arr.dtype.kind != "M":
                arr = to_datetime64(arr)
            self._c[k] = arr
        self.dims = tuple(dims)

    def __getitem__(self, k):
        return self._c[k]

    def __iter__(self):
        return iter(self._c)

    def __len__(self):
        return len(self._c)

    def get_array(self, k):
        return self._c[k]

    def update(self, **kw):
        c = dict(self._c)
        c.update(kw)
        return Coords(c, self.dims)

    @property
    def coord_map(self):
        return dict(self._c)


def _is_torch(x):
    try:
        import torch
        return isinstance(x, torch.Tensor)
    except ImportError:  # pragma: no cover
        return False


class Patch:
    """DAS data + coordinates (DASCore ``Patch``, external)."""

    def __init__(self, data=None, coords=None, dims=None, attrs=None, _lazy=None):
        self._lazy = _lazy
        self._data = data
        if dims is None:
            raise ValueError("dims are required")
        self.dims = tuple(dims)
        self.coords = coords if isinstance(coords, Coords) else Coords(coords or {}, self.dims)
        a = dict(attrs.to_dict() if isinstance(attrs, PatchAttrs) else (attrs or {}))
        # keep coordinate-derived attributes consistent (DASCore recomputes them)
        if "time" in self.coords:
            t = self.coords["time"]
            if len(t):
                a["time_min"] = t[0]
                a["time_max"] = t[-1]
            if len(t) > 1:
                # DASCore derives the step from the coordinate, so a decimated
                # or rolled patch reports its own spacing (what chunk(time=None)
                # merges on, lf_das.py:239); a user 'd_time' attr is kept as is
                a.pop("step_time", None)
                a["time_step"] = (t[1] - t[0]).astype("timedelta64[ns]")
        if "distance" in self.coords:
            d = self.coords["distance"]
            if len(d):
                a.setdefault("distance_min", d[0])
                a["distance_min"] = d[0]
                a["distance_max"] = d[-1]
            if len(d) > 1 and not any(k in a for k in ("distance_step", "d_distance", "step_distance")):
                a["distance_step"] = d[1] - d[0]
        self.attrs = PatchAttrs(a)

    # -- data -------------------------------------------------------------
    @property
    def data(self):
        """Host (numpy) view of the data; lazy device results materialise here."""
        if self._lazy is not None:
            if getattr(self._lazy, "transient", False):
                # file-backed samples of an archive index: read on use, not kept
                return self._lazy.materialize(self)
            self._data = self._lazy.materialize(self)
            self._lazy = None
        if _is_torch(self._data):
            return self._data.detach().cpu().numpy()
        return self._data

    def device_data(self):
        """The data as it currently lives (torch tensor stays on device)."""
        if self._lazy is not None:
            return self.data
        return self._data

    @property
    def shape(self):
        if self._lazy is not None:
            return self._lazy.shape
        return tuple(self._data.shape)

    @property
    def time_axis(self):
        return self.dims.index("time")

    def sample_times_ns(self):
        return self.coords["time"].astype("datetime64[ns]").astype(np.int64)

    def sampling_interval_ns(self) -> int:
        t = self.sample_times_ns()
        if len(t) < 2:
            step = self.attrs.get("time_step")
            if step is None:
                raise ValueError("cannot infer the sampling interval of a 1-sample patch")
            return int(np.timedelta64(step, "ns").astype(np.int64))
        return int(t[1] - t[0])

    # -- DASCore-style API --------------------------------------------------
    def new(self, data=None, coords=None, dims=None, attrs=None):
        d = self.device_data() if data is None else data
        c = self.coords if coords is None else coords
        dm = self.dims if dims is None else dims
        a = self.attrs if attrs is None else attrs
        return Patch(data=d, coords=c, dims=dm, attrs=a)

    def update_attrs(self, **kw):
        a = self.attrs.to_dict()
        for k, v in kw.items():
            a[k] = v
        p = Patch(data=self._data, coords=self.coords, dims=self.dims, attrs=a, _lazy=self._lazy)
        return p

    def pipe(self, func, *args, **kwargs):
        return func(self, *args, **kwargs)

    def select(self, **kwargs):
        """Inclusive range selection on time and/or distance."""
        idx = [slice(None)] * len(self.dims)
        coords = dict(self.coords.coord_map)
        for dim, rng in kwargs.items():
            if dim not in self.dims:
                raise ValueError(f"{dim} is not a dimension of this patch")
            arr = coords[dim]
            lo, hi = rng if rng is not None else (None, None)
            m = np.ones(len(arr), bool)
            if dim == "time":
                if lo is not None:
                    m &= arr >= to_datetime64(lo)
                if hi is not None:
                    m &= arr <= to_datetime64(hi)
            else:
                if lo is not None:
                    m &= arr >= lo
                if hi is not None:
                    m &= arr <= hi
            nz = np.nonzero(m)[0]
            sl = slice(int(nz[0]), int(nz[-1]) + 1) if len(nz) else slice(0, 0)
            idx[self.dims.index(dim)] = sl
            coords[dim] = arr[sl]
        data = self.device_data()[tuple(idx)]
        return Patch(data=data, coords=coords, dims=self.dims, attrs=self._attrs_wo_coords())

    def _attrs_wo_coords(self):
        a = self.attrs.to_dict()
        for k in ("time_min", "time_max", "distance_min", "distance_max"):
            a.pop(k, None)
        return a

    def dropna(self, dim, how="any"):
        """Drop labels of ``dim`` where any (or all) values are NaN."""
        data = self.data
        ax = self.dims.index(dim)
        other = tuple(i for i in range(data.ndim) if i != ax)
        nan = np.isnan(data)
        bad = nan.any(axis=other) if how == "any" else nan.all(axis=other)
        keep = ~bad
        coords = dict(self.coords.coord_map)
        coords[dim] = coords[dim][keep]
        return Patch(data=np.compress(keep, data, axis=ax), coords=coords, dims=self.dims,
                     attrs=self._attrs_wo_coords())

    # processing (implemented in lfdas.proc)
    def pass_filter(self, corners=4, zerophase=True, **kwargs):
        from .proc import pass_filter
        return pass_filter(self, corners=corners, zerophase=zerophase, **kwargs)

    def interpolate(self, kind="linear", **kwargs):
        from .proc import interpolate
        return interpolate(self, kind=kind, **kwargs)

    def decimate(self, filter_type=None, **kwargs):
        from .proc import decimate
        return decimate(self, filter_type=filter_type, **kwargs)

    def rolling(self, step=None, center=False, engine="numpy", **kwargs):
        from .proc import rolling
        return rolling(self, step=step, center=center, engine=engine, **kwargs)

    @property
    def io(self):
        from .io import PatchIO
        return PatchIO(self)

    def __repr__(self):
        return f"Patch(dims={self.dims}, shape={self.shape}, time=[{self.attrs.get('time_min')}, {self.attrs.get('time_max')}])"


# ---------------------------------------------------------------------------
class Spool:
    """Ordered collection of patches (DASCore ``Spool``, external)."""

    def __init__(self, patches=(), source=None):
        self._patches = list(patches)
        self._source = source

    def __len__(self):
        return len(self._patches)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return Spool(self._patches[i], self._source)
        return self._patches[i]

    def __iter__(self):
        return iter(self._patches)

    def sort(self, key="time"):
        if key != "time":
            raise NotImplementedError("only time sorting is supported")
        return Spool(sorted(self._patches, key=lambda p: p.coords["time"][0]), self._source)

    def update(self):
        if self._source and os.path.isdir(self._source):
            return spool(self._source)
        return self

    def get_contents(self):
        import pandas as pd
        rows = []
        for p in self._patches:
            a = p.attrs
            rows.append({"time_min": a.get("time_min"), "time_max": a.get("time_max"),
                         "time_step": a.get("time_step"), "distance_min": a.get("distance_min"),
                         "distance_max": a.get("distance_max")})
        return pd.DataFrame(rows)

    def select(self, **kwargs):
        out = []
        for p in self._patches:
            keep = True
            for dim, rng in kwargs.items():
                arr = p.coords[dim]
                lo, hi = rng
                if dim == "time":
                    lo = None if lo is None else to_datetime64(lo)
                    hi = None if hi is None else to_datetime64(hi)
                if (lo is not None and arr[-1] < lo) or (hi is not None and arr[0] > hi):
                    keep = False
            if keep:
                sub = p.select(**kwargs)
                if all(s > 0 for s in sub.shape):
                    out.append(sub)
        return Spool(out, self._source)

    def chunk(self, time=None, overlap=None, keep_partial=False, tolerance=1.5):
        """``chunk(time=None)``: merge time-contiguous patches (lf_das.py:239,
        265); ``chunk(time=T, overlap=O)``: windows ``[start, start + T)`` of
        each merged patch, ``start`` stepping by ``T - O`` from its first
        sample; a last window running past the data is dropped unless
        ``keep_partial`` (then it ends at the last sample).  With
        ``T = P dt`` and ``O = 2 B dt`` these are LFProc's chunks
        (lf_das.py:236-240, 264-266) up to the inclusive end
        sample.  The windows of one merged patch share a chunk group:
        ``pass_filter(...).interpolate(...)`` requests made on them are
        computed together, as one device plan over the merged samples, when
        the first of them is read (lfdas.proc)."""
        pats = sorted(self._patches, key=lambda p: p.coords["time"][0])
        merged = []
        for p in pats:
            if merged and _contiguous(merged[-1][-1], p, tolerance):
                merged[-1].append(p)
            else:
                merged.append([p])
        out = [_merge(g) for g in merged]
        if time is None:
            return Spool(out, self._source)
        T = to_timedelta64(time)
        O = to_timedelta64(overlap or 0)
        if O >= T:
            raise ValueError("overlap must be smaller than the chunk length")
        from .proc import ChunkGroup
        res = []
        for p in out:
            t = p.coords["time"]
            group = ChunkGroup(p)
            start = t[0]
            while True:
                stop = start + T
                if stop > t[-1] + p.attrs["time_step"]:
                    if keep_partial and start <= t[-1]:
                        res.append(group.window(start, t[-1]))
                    break
                res.append(group.window(start, stop - np.timedelta64(1, "ns")))
                start = stop - O
        return Spool(res, self._source)


def _contiguous(a: Patch, b: Patch, tol: float) -> bool:
    ta = a.coords["time"]
    tb = b.coords["time"]
    step = a.attrs["time_step"]
    step = np.timedelta64(step, "ns") if not isinstance(step, float) else to_timedelta64(step)
    gap = (tb[0] - ta[-1]).astype("timedelta64[ns]")
    if a.dims != b.dims:
        return False
    if "distance" in a.coords and not np.array_equal(a.coords["distance"], b.coords["distance"]):
        return False
    return np.timedelta64(0, "ns") < gap <= step * tol or gap == np.timedelta64(0, "ns")


def _merge(group):
    if len(group) == 1:
        return group[0]
    ax = group[0].time_axis
    datas = [g.device_data() for g in group]
    ts = [g.coords["time"] for g in group]
    # drop exactly duplicated boundary samples
    keep = [np.ones(len(t), bool) for t in ts]
    for i in range(1, len(ts)):
        keep[i] = ts[i] > ts[i - 1][-1]
    if _is_torch(datas[0]):
        import torch
        parts = [d.index_select(ax, torch.as_tensor(np.nonzero(k)[0], device=d.device))
                 if not k.all() else d for d, k in zip(datas, keep)]
        data = torch.cat(parts, dim=ax)
    else:
        parts = [np.compress(k, np.asarray(d), axis=ax) if not k.all() else np.asarray(d)
                 for d, k in zip(datas, keep)]
        data = np.concatenate(parts, axis=ax)
    coords = dict(group[0].coords.coord_map)
    coords["time"] = np.concatenate([t[k] for t, k in zip(ts, keep)])
    return Patch(data=data, coords=coords, dims=group[0].dims, attrs=group[0]._attrs_wo_coords())


def spool(obj):
    """``dc.spool``: from a Patch, a list of patches, a Spool or a directory of
    files written by ``Patch.io.write`` (lfdas.io)."""
    if isinstance(obj, Spool):
        return Spool(list(obj), obj._source)
    if isinstance(obj, Patch):
        return Spool([obj])
    if isinstance(obj, (str, os.PathLike)):
        from .io import read_directory
        return Spool(read_directory(os.fspath(obj)), os.fspath(obj)).sort("time")
    return Spool(list(obj))


def get_example_patch(name="random_das", time_min="2017-09-18", shape=(300, 2000),
                      time_step=0.004, distance_step=1.0):
    """*(DASCore, external)* ``get_example_patch('random_das')``: dims
    ("distance", "time"), data ``RandomState(42).random(shape)``."""
    if name != "random_das":
        raise NotImplementedError(name)
    data = np.random.RandomState(42).random(shape)
    t0 = np.datetime64(time_min, "ns")
    step = to_timedelta64(time_step)
    time = t0 + np.arange(shape[1]) * step
    dist = np.arange(shape[0]) * distance_step
    return Patch(data=data, coords={"distance": dist, "time": time}, dims=("distance", "time"),
                 attrs={"time_step": step, "distance_step": distance_step, "category": "DAS"})


def get_example_spool(name="random_das", n_patches=3, time_gap=0, **kw):
    """*(DASCore, external)* three contiguous random_das patches."""
    p0 = get_example_patch(**kw)
    step = p0.attrs["time_step"]
    out = [p0]
    for i in range(1, n_patches):
        prev = out[-1]
        t_start = prev.coords["time"][-1] + step + np.timedelta64(int(time_gap * 1e9), "ns")
        out.append(get_example_patch(time_min=t_start, **kw))
    return Spool(out)
