"""Narrow-shard K1 time by how the input is allocated, as the FIRST device
allocation of a fresh process (the situation of each rank of an N-GPU run):
  torch  torch.empty (caching allocator -> hipMalloc)
  contig hipExtMallocWithFlags(hipDeviceMallocContiguous)
  plain  hipMalloc
  big<k>[last] torch.empty of k x the bytes, the shard in the first (last)
         rows (placement probe)
Usage: python tools/r05_alloc_first.py <method> [channels]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "low-freq-real-time_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from lfdas.plan import set_timing  # noqa: E402

method = sys.argv[1]
ch = int(sys.argv[2]) if len(sys.argv) > 2 else 1250
n = 1_800_000
dev = torch.device("cuda", 0)
torch.cuda.init()
nbytes = ch * n * 4


class _Arr:
    def __init__(self, ptr, shape):
        self.__cuda_array_interface__ = {"shape": shape, "typestr": "<f4", "data": (ptr, False), "version": 3,
                                         "strides": None}


if method in ("contig", "plain"):
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    p = ctypes.c_void_p()
    rc = hip.hipExtMallocWithFlags(ctypes.byref(p), nbytes, 0x4) if method == "contig" else \
        hip.hipMalloc(ctypes.byref(p), nbytes)
    assert rc == 0, rc
    x = torch.as_tensor(_Arr(p.value, (ch, n)), device=dev)
elif method.startswith("vmm"):  # vmm<G>: G GiB physical chunks mapped into a G-GiB-aligned VA range; vmmone: one chunk
    c_sz = ctypes.c_size_t
    hip = ctypes.CDLL("libamdhip64.so.7")  # torch's runtime (already loaded)

    class Loc(ctypes.Structure):
        _fields_ = [("type", ctypes.c_int), ("id", ctypes.c_int)]

    class Flg(ctypes.Structure):
        _fields_ = [("ct", ctypes.c_ubyte), ("rdma", ctypes.c_ubyte), ("usage", ctypes.c_ushort)]

    class Prop(ctypes.Structure):
        _fields_ = [("type", ctypes.c_int), ("handle", ctypes.c_int), ("location", Loc), ("win32", ctypes.c_void_p),
                    ("flags", Flg)]

    class Acc(ctypes.Structure):
        _fields_ = [("location", Loc), ("flags", ctypes.c_int)]

    prop = Prop(1, 0, Loc(1, 0), None, Flg(0, 0, 0))
    gran = c_sz()
    assert hip.hipMemGetAllocationGranularity(ctypes.byref(gran), ctypes.byref(prop), 1) == 0
    G = (nbytes + gran.value - 1) // gran.value * gran.value if method == "vmmone" else int(method[3:] or 1) << 30
    size = (nbytes + G - 1) // G * G
    va = ctypes.c_void_p()
    hip.hipMemAddressReserve.argtypes = [ctypes.POINTER(ctypes.c_void_p), c_sz, c_sz, ctypes.c_void_p,
                                         ctypes.c_ulonglong]
    hip.hipMemCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p), c_sz, ctypes.POINTER(Prop), ctypes.c_ulonglong]
    hip.hipMemMap.argtypes = [ctypes.c_void_p, c_sz, c_sz, ctypes.c_void_p, ctypes.c_ulonglong]
    hip.hipMemSetAccess.argtypes = [ctypes.c_void_p, c_sz, ctypes.POINTER(Acc), c_sz]
    align = min(G, 1 << 30)
    assert hip.hipMemAddressReserve(ctypes.byref(va), size, align, None, 0) == 0
    for i in range(size // G):
        h = ctypes.c_void_p()
        rc = hip.hipMemCreate(ctypes.byref(h), G, ctypes.byref(prop), 0)
        assert rc == 0, rc
        assert hip.hipMemMap(va.value + i * G, G, 0, h, 0) == 0
    acc = Acc(Loc(1, 0), 3)
    assert hip.hipMemSetAccess(va, size, ctypes.byref(acc), 1) == 0
    print(f"vmm granularity {gran.value} chunk {G} size {size}", flush=True)
    x = torch.as_tensor(_Arr(va.value, (ch, n)), device=dev)
elif method.startswith("pool"):  # pool[<GiB>]: lfdas.arena.device_samples with that pool size
    from lfdas import arena
    if method[4:]:
        arena.POOL_BYTES = int(method[4:]) << 30
    x = arena.device_samples((ch, n), device=dev)
elif method.startswith("big"):  # big<k>[last]: k x the rows, the shard at the start / end
    k = int(method[3:].replace("last", "") or 4)
    full = torch.empty((k * ch, n), dtype=torch.float32, device=dev)
    x = full[(k - 1) * ch:] if method.endswith("last") else full[:ch]
else:
    x = torch.empty((ch, n), dtype=torch.float32, device=dev)
plan, *_ = bench.build_plan(ch, n, 500.0, 1.0, 600, 7)
y = torch.empty((ch, plan.n_grid), dtype=torch.float32, device=dev)
wsb = plan.alloc_workspace(dev)
st = torch.cuda.current_stream(dev)
bench.synth_fill(x, 500.0, 77)
set_timing(True)
ts = []
for _ in range(8):
    plan.execute(x, y, wsb, st)
    ts.append(plan.last_timing_ms()[0])
k1 = float(np.median(ts[2:]))
print(f"{method:6s} ch {ch} base%1G {x.data_ptr() % (1 << 30):>11d} K1 {k1:.3f} ms frac {ch * n * 4.008 / (k1 * 1e-3) / 8e12:.3f}",
      flush=True)
