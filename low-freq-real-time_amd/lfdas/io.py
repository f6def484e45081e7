"""Patch files.  The reference writes DASDAE HDF5 (``lfDAS.io.write(fn,
"dasdae")``, lf_das.py:232) through pytables, which is not installed here;
this is an NPZ stand-in with the same file NAMES (``_get_filename``) so the
real-time resume rule (``get_last_processed_time``, lf_das.py:214-217) works.
A real DASDAE writer is SURVEY §8(f) item 1."""
from __future__ import annotations

import json
import os

import numpy as np

from .core import Patch, PatchAttrs

_MAGIC = "lfdas-npz-v1"


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


def write_patch(patch: Patch, path: str):
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
        if str(file_format).lower() not in ("dasdae", "lfdas", "npz"):
            raise NotImplementedError(f"format {file_format!r}")
        write_patch(self.patch, os.fspath(path))
