"""K1 speed vs how the 72 GB cfg3 input was allocated (diagnostic).

K1 runs in per-allocation "modes" (the same build measures
12.6-13.2 ms on different tensors).  This probe allocates the cfg3 input
several times with each allocator, fills it with the bench's synthetic
samples and times K1 on it (one allocation alive at a time):
  torch   torch.empty (the caching allocator -> hipMalloc)
  contig  hipExtMallocWithFlags(hipDeviceMallocContiguous)
  plain   hipMalloc directly
Usage (GPU box): python tools/probe_alloc.py [reps]
"""
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

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipFree.argtypes = [ctypes.c_void_p]
HIP_CONTIGUOUS = 0x4


class _Arr:
    def __init__(self, ptr, shape):
        self.__cuda_array_interface__ = {"shape": shape, "typestr": "<f4", "data": (ptr, False), "version": 3,
                                         "strides": None}


reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
n_ch, n = 10_000, 1_800_000
plan, *_ = bench.build_plan(n_ch, n, 500.0, 1.0, 600, 7)
dev = torch.device("cuda", 0)
y = torch.empty((n_ch, plan.n_grid), dtype=torch.float32, device=dev)
wsb = plan.alloc_workspace(dev)
st = torch.cuda.current_stream(dev)
set_timing(True)
nbytes = n_ch * n * 4
for rep in range(reps):
    for kind in ("torch", "contig", "plain"):
        raw = None
        if kind == "torch":
            x = torch.empty((n_ch, n), dtype=torch.float32, device=dev)
        else:
            p = ctypes.c_void_p()
            rc = (hip.hipExtMallocWithFlags(ctypes.byref(p), nbytes, HIP_CONTIGUOUS) if kind == "contig"
                  else hip.hipMalloc(ctypes.byref(p), nbytes))
            if rc != 0:
                print(f"{kind}: allocation failed rc={rc}", flush=True)
                continue
            raw = p.value
            x = torch.as_tensor(_Arr(raw, (n_ch, n)), device=dev)
        bench.synth_fill(x, 500.0, 77)
        plan.execute(x, y, wsb, st)
        torch.cuda.synchronize()
        k = []
        for _ in range(6):
            plan.execute(x, y, wsb, st)
            k.append(plan.last_timing_ms()[0])
        print(f"rep {rep} {kind:6s} base 0x{x.data_ptr():x} K1 median {np.median(k):.3f} "
              f"min {np.min(k):.3f} max {np.max(k):.3f} ms", flush=True)
        del x
        torch.cuda.synchronize()
        if raw is not None:
            hip.hipFree(ctypes.c_void_p(raw))
        torch.cuda.empty_cache()
