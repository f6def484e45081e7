"""Patch files in the reference's format step: ``lfDAS.io.write(fn,
"dasdae")`` (lf_das.py:230-232) and ``dc.spool(folder).update()`` reading
them back (lf_das.py:214-217).

* ``dasdae`` (default): HDF5 in DASCore's DASDAE v1 layout, written and read
  by ``liblfdas_h5.so`` (include/lfdas_h5.h) on the image's libhdf5 1.10.
  The layout is restated from DASCore's public writer; DASCore/pytables are
  not installed, so byte-level compatibility with DASCore's reader is
  unpinned.
* ``npz``: the NPZ stand-in, written only when asked for by name (a
  ``dasdae`` write without liblfdas_h5.so raises instead of falling back).

Readers sniff the file signature, so a folder may mix both."""
from __future__ import annotations

import ctypes
import json
import os

import numpy as np

from .core import Patch, PatchAttrs

_MAGIC = "lfdas-npz-v1"
_HDF5_SIG = b"\x89HDF\r\n\x1a\n"

# --- DASDAE HDF5 through liblfdas_h5.so --------------------------------------
LFDH5_STR, LFDH5_F64, LFDH5_I64, LFDH5_BOOL, LFDH5_DT64, LFDH5_TD64 = range(6)


class _H5Attr(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("kind", ctypes.c_int), ("s", ctypes.c_char_p),
                ("f", ctypes.c_double), ("i", ctypes.c_int64)]


class _H5Coord(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("kind", ctypes.c_int), ("len", ctypes.c_int64),
                ("data", ctypes.c_void_p)]


_h5lib = None


def h5_available() -> bool:
    return _h5() is not None


def _h5():
    """liblfdas_h5.so, or None (``dasdae`` writes then raise)."""
    global _h5lib
    if _h5lib is None:
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "liblfdas_h5.so")
        try:
            lib = ctypes.CDLL(path)
        except OSError:
            _h5lib = False
            return None
        i64, vp, cp, ci = ctypes.c_int64, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int
        P = ctypes.POINTER
        for name, args, res in [
            ("lfdh5_last_error", [], cp),
            ("lfdh5_write_patch", [cp, cp, vp, i64, i64, cp, vp, ci, vp, ci], ci),
            ("lfdh5_open", [cp, P(vp), P(i64), P(i64), P(ci), P(ci)], ci),
            ("lfdh5_read_data", [vp, vp], ci),
            ("lfdh5_dims", [vp, cp, ci], ci),
            ("lfdh5_coord_info", [vp, ci, cp, ci, P(ci), P(i64)], ci),
            ("lfdh5_coord_read", [vp, ci, vp], ci),
            ("lfdh5_attr_info", [vp, ci, cp, ci, P(ci), cp, ci, P(ctypes.c_double), P(i64)], ci),
            ("lfdh5_close", [vp], None),
        ]:
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = res
        _h5lib = lib
    return _h5lib or None


def _h5check(rc):
    if rc != 0:
        raise OSError(_h5().lfdh5_last_error().decode("utf-8", "replace"))


def _dasdae_group_name(patch: Patch) -> str:
    """``DAS__<network>__<station>__<tag>__<time_min>__<time_max>`` (DASCore's
    patch naming, times with ':' '-' '.' as '_')."""
    a = patch.attrs

    def f(t):
        return str(np.datetime64(t, "ns")).replace(":", "_").replace("-", "_").replace(".", "_")

    parts = ["DAS", str(a.get("network") or ""), str(a.get("station") or ""), str(a.get("tag") or ""),
             f(a["time_min"]), f(a["time_max"])]
    return "__".join(parts)


def _write_h5(patch: Patch, path: str):
    lib = _h5()
    keep = []
    attrs = []
    for k, v in patch.attrs.to_dict().items():
        if v is None:
            continue
        a = _H5Attr(name=k.encode())
        if isinstance(v, np.datetime64):
            a.kind, a.i = LFDH5_DT64, int(np.datetime64(v, "ns").astype(np.int64))
        elif isinstance(v, np.timedelta64):
            a.kind, a.i = LFDH5_TD64, int(np.timedelta64(v, "ns").astype(np.int64))
        elif isinstance(v, (bool, np.bool_)):
            a.kind, a.i = LFDH5_BOOL, int(bool(v))
        elif isinstance(v, (int, np.integer)):
            a.kind, a.i = LFDH5_I64, int(v)
        elif isinstance(v, (float, np.floating)):
            a.kind, a.f = LFDH5_F64, float(v)
        elif isinstance(v, str):
            a.kind, a.s = LFDH5_STR, v.encode()
        else:
            continue
        attrs.append(a)
    coords = []
    for name, arr in patch.coords.coord_map.items():
        x = np.asarray(arr)
        if x.dtype.kind == "M":
            d, kind = np.ascontiguousarray(x.astype("datetime64[ns]").astype(np.int64)), LFDH5_DT64
        elif x.dtype.kind == "m":
            d, kind = np.ascontiguousarray(x.astype("timedelta64[ns]").astype(np.int64)), LFDH5_TD64
        elif x.dtype.kind in "iu":
            d, kind = np.ascontiguousarray(x.astype(np.int64)), LFDH5_I64
        else:
            d, kind = np.ascontiguousarray(x.astype(np.float64)), LFDH5_F64
        keep.append(d)
        coords.append(_H5Coord(name=name.encode(), kind=kind, len=len(d), data=d.ctypes.data))
    data = np.ascontiguousarray(patch.data, dtype=np.float64)
    if data.ndim != 2:
        raise ValueError("DASDAE patches here are 2-D")
    ca = (_H5Coord * max(1, len(coords)))(*coords)
    aa = (_H5Attr * max(1, len(attrs)))(*attrs)
    _h5check(lib.lfdh5_write_patch(os.fspath(path).encode(), _dasdae_group_name(patch).encode(),
                                   data.ctypes.data, data.shape[0], data.shape[1],
                                   ",".join(patch.dims).encode(), ctypes.cast(ca, ctypes.c_void_p),
                                   len(coords), ctypes.cast(aa, ctypes.c_void_p), len(attrs)))


def _read_h5(path: str, with_data: bool = True):
    """(data or None, shape, coords, dims, attrs) of the file's first patch."""
    lib = _h5()
    if lib is None:
        raise OSError("liblfdas_h5.so is not available to read " + path)
    h = ctypes.c_void_p()
    n0, n1 = ctypes.c_int64(), ctypes.c_int64()
    nc, na = ctypes.c_int(), ctypes.c_int()
    _h5check(lib.lfdh5_open(os.fspath(path).encode(), ctypes.byref(h), ctypes.byref(n0), ctypes.byref(n1),
                            ctypes.byref(nc), ctypes.byref(na)))
    try:
        buf = ctypes.create_string_buffer(4096)
        _h5check(lib.lfdh5_dims(h, buf, len(buf)))
        dims = tuple(buf.value.decode().split(","))
        coords = {}
        for i in range(nc.value):
            kind, ln = ctypes.c_int(), ctypes.c_int64()
            _h5check(lib.lfdh5_coord_info(h, i, buf, len(buf), ctypes.byref(kind), ctypes.byref(ln)))
            name = buf.value.decode()
            arr = np.empty(ln.value, np.float64 if kind.value == LFDH5_F64 else np.int64)
            _h5check(lib.lfdh5_coord_read(h, i, arr.ctypes.data))
            if kind.value == LFDH5_DT64:
                arr = arr.astype("datetime64[ns]")
            elif kind.value == LFDH5_TD64:
                arr = arr.astype("timedelta64[ns]")
            coords[name] = arr
        attrs = {}
        sbuf = ctypes.create_string_buffer(1 << 16)
        for i in range(na.value):
            kind, fv, iv = ctypes.c_int(), ctypes.c_double(), ctypes.c_int64()
            _h5check(lib.lfdh5_attr_info(h, i, buf, len(buf), ctypes.byref(kind), sbuf, len(sbuf),
                                         ctypes.byref(fv), ctypes.byref(iv)))
            k = buf.value.decode()
            attrs[k] = {LFDH5_STR: lambda: sbuf.value.decode(), LFDH5_F64: lambda: fv.value,
                        LFDH5_I64: lambda: iv.value, LFDH5_BOOL: lambda: bool(iv.value),
                        LFDH5_DT64: lambda: np.datetime64(iv.value, "ns"),
                        LFDH5_TD64: lambda: np.timedelta64(iv.value, "ns")}[kind.value]()
        data = None
        if with_data:
            data = np.empty((n0.value, n1.value), np.float64)
            _h5check(lib.lfdh5_read_data(h, data.ctypes.data))
        return data, (n0.value, n1.value), coords, dims, attrs
    finally:
        lib.lfdh5_close(h)


def _is_hdf5(path: str) -> bool:
    with open(path, "rb") as fh:
        return fh.read(8) == _HDF5_SIG


def _attrs_to_json(attrs):
    out = {}
    for k, v in (attrs.to_dict() if isinstance(attrs, PatchAttrs) else dict(attrs)).items():
        if isinstance(v, np.datetime64):
            out[k] = {"datetime64": str(np.datetime64(v, "ns"))}
        elif isinstance(v, np.timedelta64):
            out[k] = {"timedelta64_ns": int(np.timedelta64(v, "ns").astype(np.int64))}
        elif isinstance(v, (np.floating, np.integer)):
            out[k] = v.item()
        elif isinstance(v, (str, int, float, bool)) or v is None:
            out[k] = v
    return out


def _attrs_from_json(d):
    out = {}
    for k, v in d.items():
        if isinstance(v, dict) and "datetime64" in v:
            out[k] = np.datetime64(v["datetime64"], "ns")
        elif isinstance(v, dict) and "timedelta64_ns" in v:
            out[k] = np.timedelta64(v["timedelta64_ns"], "ns")
        else:
            out[k] = v
    return out


def write_patch(patch: Patch, path: str, file_format: str = "dasdae"):
    """``dasdae``: HDF5 (DASDAE layout) through liblfdas_h5.so — raises
    ``OSError`` when that library is missing rather than writing other bytes
    under a DASDAE file name; ``npz``: the NPZ stand-in (explicit only)."""
    if str(file_format).lower() == "dasdae":
        if _h5() is None:
            raise OSError("DASDAE output needs liblfdas_h5.so (build it with "
                          "__graft_entry__.build()); write format 'npz' explicitly for the stand-in")
        _write_h5(patch, path)
        return
    coords = patch.coords.coord_map
    arrays = {"magic": np.array(_MAGIC), "data": np.asarray(patch.data),
              "dims": np.array(list(patch.dims)),
              "attrs": np.array(json.dumps(_attrs_to_json(patch.attrs)))}
    for name, arr in coords.items():
        a = np.asarray(arr)
        if a.dtype.kind == "M":
            arrays["coord_ns__" + name] = a.astype("datetime64[ns]").astype(np.int64)
        else:
            arrays["coord__" + name] = a
    with open(path, "wb") as fh:  # exact file name, no ".npz" suffix added
        np.savez(fh, **arrays)


def read_patch(path: str) -> Patch:
    if _is_hdf5(path):
        data, _, coords, dims, attrs = _read_h5(path)
        return Patch(data=data, coords=coords, dims=dims, attrs=attrs)
    with np.load(path, allow_pickle=False) as z:
        if "magic" not in z.files or str(z["magic"]) != _MAGIC:
            raise ValueError(f"{path} is not an lfdas patch file")
        coords = {}
        for f in z.files:
            if f.startswith("coord_ns__"):
                coords[f[len("coord_ns__"):]] = z[f].astype("datetime64[ns]")
            elif f.startswith("coord__"):
                coords[f[len("coord__"):]] = z[f]
        return Patch(data=z["data"], coords=coords, dims=tuple(str(d) for d in z["dims"]),
                     attrs=_attrs_from_json(json.loads(str(z["attrs"]))))


class _FileData:
    """Lazy data of a patch file: the spool index holds coordinates and
    attributes only; the samples are read when the patch's data is used
    (out-of-core archives: one file in host memory at a time)."""

    transient = True  # Patch.data reads the file on every use and keeps nothing

    def __init__(self, path: str, shape):
        self.path = path
        self.shape = tuple(shape)

    def materialize(self, patch: Patch):
        if _is_hdf5(self.path):
            return _read_h5(self.path)[0]
        with np.load(self.path, allow_pickle=False) as z:
            return z["data"]


def _data_shape(z) -> tuple:
    """Shape of the ``data`` member from its .npy header (no sample read)."""
    with z.zip.open("data.npy") as fh:
        version = np.lib.format.read_magic(fh)
        shape, _, _ = np.lib.format._read_array_header(fh, version)
    return tuple(shape)


def index_patch(path: str) -> Patch:
    """Header-only read of a patch file (coordinates, dims, attributes)."""
    if _is_hdf5(path):
        _, shape, coords, dims, attrs = _read_h5(path, with_data=False)
        p = Patch(data=None, coords=coords, dims=dims, attrs=attrs, _lazy=_FileData(path, shape))
        p.source_path = path
        return p
    with np.load(path, allow_pickle=False) as z:
        if "magic" not in z.files or str(z["magic"]) != _MAGIC:
            raise ValueError(f"{path} is not an lfdas patch file")
        coords = {}
        for f in z.files:
            if f.startswith("coord_ns__"):
                coords[f[len("coord_ns__"):]] = z[f].astype("datetime64[ns]")
            elif f.startswith("coord__"):
                coords[f[len("coord__"):]] = z[f]
        shape = _data_shape(z)
        p = Patch(data=None, coords=coords, dims=tuple(str(d) for d in z["dims"]),
                  attrs=_attrs_from_json(json.loads(str(z["attrs"]))), _lazy=_FileData(path, shape))
    p.source_path = path
    return p


# header index of a directory, reused by Spool.update(): path -> (mtime, size, patch)
_INDEX: dict = {}


def read_directory(folder: str, lazy: bool = True):
    """Every patch file of ``folder`` (the ``dc.spool(path).update()`` index).
    ``lazy``: read headers only and load samples on use; files already indexed
    and unchanged (mtime, size) are not re-read."""
    out = []
    for name in sorted(os.listdir(folder)):
        p = os.path.join(folder, name)
        if not os.path.isfile(p):
            continue
        try:
            if not lazy:
                out.append(read_patch(p))
                continue
            st = os.stat(p)
            hit = _INDEX.get(p)
            if hit is not None and hit[0] == st.st_mtime_ns and hit[1] == st.st_size:
                out.append(hit[2])
                continue
            patch = index_patch(p)
            _INDEX[p] = (st.st_mtime_ns, st.st_size, patch)
            out.append(patch)
        except Exception:
            continue
    return out


class PatchIO:
    def __init__(self, patch: Patch):
        self.patch = patch

    def write(self, path, file_format="dasdae", **kwargs):
        fmt = str(file_format).lower()
        if fmt not in ("dasdae", "lfdas", "npz"):
            raise NotImplementedError(f"format {file_format!r}")
        write_patch(self.patch, os.fspath(path), "npz" if fmt in ("lfdas", "npz") else "dasdae")
