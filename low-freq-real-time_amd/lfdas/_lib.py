"""ctypes binding of liblfdas.so (include/lfdas.h).

The HIP library is the product: there is no CPU fallback.  If the shared
object is missing or fails to load, every compute entry point raises
``LFDLibraryError`` — build it with ``python -c "import __graft_entry__ as g;
g.build()"`` (or ``make -C low-freq-real-time_amd/csrc``).
"""
from __future__ import annotations

import contextlib
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LFDAS_LIB") or os.path.join(_HERE, "liblfdas.so")

LFD_OK = 0
LFD_EINVAL = -1
LFD_EHIP = -2
LFD_EUNSUPPORTED = -3
LFD_ENOMEM = -4

MAX_SEC = 4
MAX_N = 2 * MAX_SEC

# numpy mirrors of the internal kernel-constant structs (csrc/lfd_internal.h),
# used only by lfd_debug_plan_constants in tests.
MAX_J = 2 * MAX_SEC
_RCOEF = np.dtype([("na1", "f8", MAX_SEC), ("na2", "f8", MAX_SEC), ("nia2", "f8", MAX_SEC),
                   ("nra", "f8", MAX_SEC), ("dcg", "f8", MAX_SEC), ("c64", "f8", MAX_J + 1),
                   ("c32", "f4", MAX_J + 1), ("G", "f8"), ("csum", "f8")], align=True)
BLOCK_CONST_DTYPE = np.dtype([("r", _RCOEF), ("T", "f8", (MAX_N, MAX_N)), ("cp", "f8", MAX_N),
                              ("dp", "f8", MAX_J + 1)], align=True)
SCAN_CONST_DTYPE = np.dtype([("r", _RCOEF), ("PhiF", "f8", (MAX_N, MAX_N)),
                             ("PhiR", "f8", (MAX_N, MAX_N)), ("M", "f8", (MAX_N, MAX_N)),
                             ("G0", "f8", MAX_N), ("H0", "f8", MAX_N),
                             ("Kc", "f8", (2 * MAX_N + 1, MAX_J)), ("ow", "f8")], align=True)
CHUNK_GEOM_DTYPE = np.dtype([(n, "i8") for n in (
    "s0", "s1", "kb", "ke", "head_end", "tail_begin", "kout0", "kout1", "jout0",
    "sf_off", "tail_out_pos", "tail_out_j", "r0", "r1", "sr_off", "kstep", "hskip")])
RUN_R = 8  # lfd::RUN_R
RUN_CONST_DTYPE = np.dtype([("PhiFp", "f8", (RUN_R + 1, 16)), ("PhiRp", "f8", (RUN_R + 1, 16)),
                            ("C", "f8", (RUN_R + 1, 16)), ("A", "f8", (RUN_R + 1, RUN_R, 4)),
                            ("B", "f8", (RUN_R, 4)), ("PhiF", "f8", 16), ("M", "f8", 16),
                            ("PhiR", "f8", 16), ("G0", "f8", 4), ("H0", "f8", 4),
                            ("KfH", "f8", (4, 32)), ("H0L", "f8", (8, 4))])


class LFDLibraryError(RuntimeError):
    """liblfdas.so is missing or could not be loaded."""


class LFDError(RuntimeError):
    """A liblfdas call returned an error code."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"liblfdas error {code}: {msg}")
        self.code = code
        self.msg = msg


class LFDUnsupported(LFDError):
    pass


class lfd_stream_config(ctypes.Structure):
    """include/lfdas.h lfd_stream_config."""
    _fields_ = [("n_ch", ctypes.c_int64), ("sample_ns", ctypes.c_int64),
                ("output_sample_interval", ctypes.c_double),
                ("process_patch_size", ctypes.c_int64), ("edge_buff_size", ctypes.c_int64),
                ("mode", ctypes.c_int), ("flags", ctypes.c_int),
                ("t_start_ns", ctypes.c_int64), ("t_end_ns", ctypes.c_int64),
                ("resume_back_ns", ctypes.c_int64), ("capacity", ctypes.c_int64)]


class lfd_stream_output(ctypes.Structure):
    """include/lfdas.h lfd_stream_output."""
    _fields_ = [("n_out", ctypes.c_int64), ("t_first_ns", ctypes.c_int64),
                ("t_step_ns", ctypes.c_int64), ("n_chunks", ctypes.c_int64),
                ("n_runs", ctypes.c_int64), ("y", ctypes.c_void_p), ("ys_ch", ctypes.c_int64)]


LFD_STREAM_EDGE = 0
LFD_STREAM_CONTINUOUS = 1
LFD_STREAM_DRY_RUN = 1


class lfd_chunk(ctypes.Structure):
    _fields_ = [("s0", ctypes.c_int64), ("s1", ctypes.c_int64),
                ("g0", ctypes.c_int64), ("g1", ctypes.c_int64)]


_lib = None


def load():
    """Load liblfdas.so once; raise LFDLibraryError if it is not there."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise LFDLibraryError(
            f"{LIB_PATH} not found: the HIP extension is not built (run "
            "__graft_entry__.build()); lfdas has no CPU fallback")
    # One HIP runtime per process.  torch ships its own libamdhip64 (SONAME
    # libamdhip64.so.7); loaded first, it also serves this library's NEEDED
    # libamdhip64.so.7, so torch's streams, graphs and allocations are the
    # library's own.  Loaded after this library, torch (whose NEEDED entry is
    # the file name libamdhip64.so) brings a second runtime copy, and whichever
    # initialises second finds no GPU ("No HIP GPUs are available").
    try:
        import torch  # noqa: F401
    except ImportError:  # a torch-free caller: the system runtime alone
        pass
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover
        raise LFDLibraryError(f"cannot load {LIB_PATH}: {e}") from e
    if os.path.basename(LIB_PATH) != "liblfdas.so":
        import sys
        print(f"lfdas: loaded {LIB_PATH} (not the product library: in the diagnostic build LFD_* "
              "environment knobs change kernels, some into timing-only modes)", file=sys.stderr)
    i64, i32, vp, sz = ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t
    P = ctypes.POINTER
    sig = {
        "lfd_last_error": ([], ctypes.c_char_p),
        "lfd_version": ([], i32),
        "lfd_device_count": ([P(i32)], i32),
        "lfd_set_timing": ([i32], i32),
        "lfd_set_option": ([i32, i64], i32),
        "lfd_get_option": ([i32, P(i64)], i32),
        "lfd_lowpass_plan_create": ([P(vp), vp, i32, i32, i64, i64, vp, vp, i64,
                                     vp, i64], i32),
        "lfd_lowpass_plan_info": ([vp, P(sz), P(i64), P(i64)], i32),
        "lfd_lowpass_execute": ([vp, vp, i64, i64, vp, i64, i64, vp, vp], i32),
        "lfd_lowpass_execute_split": ([vp, vp, i64, i64, vp, i64, i64, vp, vp, vp], i32),
        "lfd_lowpass_last_timing": ([vp, P(ctypes.c_float), P(ctypes.c_float)], i32),
        "lfd_lowpass_timings": ([vp, vp, vp, i64], i32),
        "lfd_lowpass_plan_destroy": ([vp], None),
        "lfd_debug_plan_constants": ([vp, vp, sz, vp, sz, vp, sz], i32),
        "lfd_debug_block_taps": ([vp, vp, sz, P(i32), P(i64)], i32),
        "lfd_lowpass_last_kernel": ([vp], i32),
        "lfd_lowpass_last_scan": ([vp], i32),
        "lfd_debug_runs": ([vp, vp, vp, i64, P(i64), vp, sz], i32),
        "lfd_sos_filtfilt_resample_f32": ([vp, i64, i64, i64, i64, vp, i32, i32,
                                           vp, vp, i64, vp, i64, i64, vp], i32),
        "lfd_sosfiltfilt_workspace_bytes": ([i64, i64, i32, i32], sz),
        "lfd_sosfiltfilt_f32": ([vp, i64, i64, i64, i64, vp, i32, i32, vp, i64,
                                 i64, vp, vp], i32),
        "lfd_sosfiltfilt_last_timing": ([P(ctypes.c_float), P(ctypes.c_float), P(ctypes.c_float)], i32),
        "lfd_interp_linear_f64": ([vp, i64, i64, i64, i64, vp, vp, i64, vp, i64,
                                   i64, vp], i32),
        "lfd_rolling_mean_f32": ([vp, i64, i64, i64, i64, i64, i64, vp, i64, i64,
                                  vp], i32),
        "lfd_fir_decimate_f32": ([vp, i64, i64, i64, i64, vp, i64, i64, i64, vp, i64, i64, vp], i32),
        "lfd_fir_decimate_last_kernel": ([], i32),
        "lfd_lfproc_schedule": ([i64, i64, i64, vp, i64, P(i64)], i32),
        "lfd_demean_scale_f64": ([vp, i64, i64, i64, i64, i64, i64, ctypes.c_double, vp, i64, i64, vp], i32),
        "lfd_median_filter_f64": ([vp, i64, i64, i64, i64, i32, i32, vp, i64, i64, vp], i32),
        "lfd_stream_open": ([P(vp), vp, vp, i32, i32], i32),
        "lfd_stream_push": ([vp, vp, i64, i64, i64, i64], i32),
        "lfd_stream_reserve": ([vp, i64], i32),
        "lfd_stream_flush": ([vp], i32),
        "lfd_stream_last_output": ([vp, vp], i32),
        "lfd_stream_last_chunks": ([vp, vp, i64, P(i64)], i32),
        "lfd_stream_fetch": ([vp, vp, i64, i64], i32),
        "lfd_stream_synchronize": ([vp], i32),
        "lfd_stream_wait_copy": ([vp], i32),
        "lfd_stream_last_timing": ([vp, P(ctypes.c_float), P(ctypes.c_float)], i32),
        "lfd_stream_info": ([vp, P(i64), P(i64), P(i64)], i32),
        "lfd_stream_close": ([vp], None),
        "lfd_debug_stream_plans": ([vp, P(i64), P(i64)], i32),
        "lfd_debug_lattice": ([vp, P(i64), P(i32), P(vp)], i32),
        "lfd_host_alloc": ([P(vp), sz], i32),
        "lfd_host_free": ([vp], None),
        "lfd_host_register": ([vp, sz], i32),
        "lfd_host_unregister": ([vp], i32),
    }
    for name, (args, res) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    _lib = lib
    return lib


EXPORTED = (
    "lfd_last_error", "lfd_version", "lfd_device_count", "lfd_set_timing", "lfd_set_option", "lfd_get_option",
    "lfd_lowpass_plan_create", "lfd_lowpass_plan_info", "lfd_lowpass_execute", "lfd_lowpass_execute_split",
    "lfd_lowpass_last_timing", "lfd_lowpass_timings", "lfd_lowpass_plan_destroy",
    "lfd_debug_plan_constants", "lfd_debug_block_taps", "lfd_lowpass_last_kernel", "lfd_lowpass_last_scan", "lfd_debug_runs",
    "lfd_sos_filtfilt_resample_f32",
    "lfd_sosfiltfilt_workspace_bytes", "lfd_sosfiltfilt_f32", "lfd_sosfiltfilt_last_timing",
    "lfd_interp_linear_f64", "lfd_rolling_mean_f32", "lfd_fir_decimate_f32", "lfd_fir_decimate_last_kernel",
    "lfd_lfproc_schedule", "lfd_stream_open", "lfd_stream_reserve", "lfd_stream_push", "lfd_stream_flush",
    "lfd_stream_last_output", "lfd_stream_last_chunks", "lfd_stream_fetch",
    "lfd_stream_synchronize", "lfd_stream_wait_copy", "lfd_stream_last_timing", "lfd_stream_info", "lfd_stream_close",
    "lfd_debug_stream_plans", "lfd_debug_lattice",
    "lfd_host_alloc", "lfd_host_free", "lfd_host_register", "lfd_host_unregister", "lfd_demean_scale_f64", "lfd_median_filter_f64",
)


# include/lfdas.h LFD_OPT_*: result-neutral kernel-selection overrides (the
# library reads no environment variable; tests drive the fallback kernels
# through these)
OPTIONS = {"no_runs": 1, "k1_recurrence": 2, "tm_no_pairs": 3, "scan_defer": 4, "fullrate_serial": 5,
           "no_lattice": 6, "no_head_skip": 7, "fir_valu": 8, "fullrate_bigblock": 9, "lattice_phases": 10}


@contextlib.contextmanager
def kernel_options(**kw):
    """Set LFD_OPT_* overrides (``no_runs=1``, ``scan_defer=2`` ...) for the
    body of a ``with`` block, restoring the previous values afterwards."""
    lib = load()
    old = {}
    try:
        for name, v in kw.items():
            oid = OPTIONS[name]
            cur = ctypes.c_int64()
            check(lib.lfd_get_option(oid, ctypes.byref(cur)))
            old[oid] = cur.value
            check(lib.lfd_set_option(oid, int(v)))
        yield
    finally:
        for oid, v in old.items():
            lib.lfd_set_option(oid, v)


def check(rc: int):
    if rc == LFD_OK:
        return
    msg = load().lfd_last_error().decode("utf-8", "replace")
    if rc == LFD_EUNSUPPORTED:
        raise LFDUnsupported(rc, msg)
    if rc == LFD_EINVAL:
        raise ValueError(msg)
    raise LFDError(rc, msg)
