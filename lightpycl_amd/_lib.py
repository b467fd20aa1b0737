"""ctypes binding of liblpc.so (include/lpc.h).

The library is built in-tree (``lightpycl_amd/liblpc.so``) by
:func:`lightpycl_amd.build.build`.  There is no fallback: if the library is
missing or no HIP device is present, the calls raise.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liblpc.so")

_lib = None
ABI_VERSION = 4         # include/lpc.h LPC_ABI_VERSION


class LpcError(RuntimeError):
    """Error returned by liblpc (carries the library's message)."""


class IterStats(ctypes.Structure):
    _fields_ = [("n_in", ctypes.c_int64), ("n_reflect", ctypes.c_int64),
                ("n_refract", ctypes.c_int64), ("n_measured", ctypes.c_int64),
                ("power_next", ctypes.c_double), ("power_nonneg", ctypes.c_int64)]


class Prof(ctypes.Structure):
    _fields_ = [("intersect_ms", ctypes.c_double), ("shade_ms", ctypes.c_double),
                ("intersect_launches", ctypes.c_int64), ("pairs", ctypes.c_int64),
                ("node_visits", ctypes.c_int64), ("group_tests", ctypes.c_int64),
                ("wave_traversals", ctypes.c_int64), ("exact_tests", ctypes.c_int64),
                ("wave_hist", ctypes.c_int64 * 24), ("heavy_piece", ctypes.c_int64),
                ("heavy_piece_ticks", ctypes.c_int64), ("piece_ticks", ctypes.c_int64),
                ("tail_waves", ctypes.c_int64), ("tail_nodes", ctypes.c_int64),
                ("tail_spread_urad", ctypes.c_int64), ("tail_exact", ctypes.c_int64),
                ("kernel_ms", ctypes.c_double), ("xchg_us", ctypes.c_double), ("xchg_calls", ctypes.c_int64),
                ("walk_cycles", ctypes.c_int64), ("drain_cycles", ctypes.c_int64),
                ("fan_exact", ctypes.c_int64), ("behind_exact", ctypes.c_int64),
                ("hit_exact", ctypes.c_int64)]


_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_F32 = ctypes.c_float
_F64 = ctypes.c_double
_INT = ctypes.c_int

# name -> argtypes (all functions return int status except lpc_last_error)
_PROTOS = {
    "lpc_device_query": [_INT, _P, _INT, _P, _INT, _P],
    "lpc_abi_version": [],
    "lpc_device_count": [_P],
    "lpc_open": [_INT, _P],
    "lpc_close": [_P],
    "lpc_device_info": [_P, _P, _INT, _P],
    "lpc_scene_upload": [_P, _I32, _P, _P, _P, _P, _I32, _P, _P, _P, _P],
    "lpc_bounce_host": [_P, _I64, _P, _P, _P, _P, _P, _F32, _F32, _P, _P, _P, _P, _P, _P, _P,
                        _P, _P, _P, _P, _P],
    "lpc_intersect": [_P, _I64, _P, _P, _F32, _P, _P, _P],
    "lpc_intersect_postproc": [_P, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _F32],
    "lpc_reflect_refract_rays": [_P, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                 _P, _P, _P, _P, _F32],
    "lpc_trace_set_rays": [_P, _I64, _P, _P, _P, _F32, _F32],
    "lpc_trace_reset": [_P],
    "lpc_trace_iterate": [_P, _P, _P, _P, _P, _P, _P],
    "lpc_trace_run": [_P, _I32, _F64, _P, _P, _P, _P, _I32],
    "lpc_trace_run_async": [_P, _I32, _F64, _P, _P, _P, _P, _I32],
    "lpc_trace_rerun_async": [_P, _I32, _F64, _P, _P, _P, _P, _I32],
    "lpc_trace_stage_rays": [_P, _I64, _P, _P, _P, _F32, _F32],
    "lpc_trace_run_staged_async": [_P, _I32, _F64, _P, _P, _P, _P, _I32],
    "lpc_sync": [_P],
    "lpc_trace_iterate_export": [_P, _P, _I32, _P],
    "lpc_trace_population_power": [_P, _P],
    "lpc_host_alloc": [ctypes.c_size_t, _P],
    "lpc_host_free": [_P],
    "lpc_host_seq_sum_f32": [_P, _I64, _P],
    "lpc_trace_population": [_P, _P],
    "lpc_trace_measured": [_P, _P, _P, _I32],
    "lpc_trace_fetch_measured": [_P, _P, _P, _P],
    "lpc_set_chunk": [_P, _I64],
    "lpc_set_walk_grid": [_P, _I64],
    "lpc_project_hist": [_P, _INT, _I64, _P, _P, _P, _P, _P, _INT, _P, _INT, _F64, _P, _P, _P,
                         _P],
    "lpc_prof_enable": [_P, _INT],
    "lpc_prof_read": [_P, _P, _INT],
    "lpc_filter_eval": [_P, _I64, _P, _P, _P, _INT, _P],
    "lpc_set_allreduce": [_P, _P, _P],
    "lpc_trace_global_stats": [_P, _P, _I32, _P],
    "lpc_shm_comm_open": [ctypes.c_char_p, _I32, _I32, _I32, _P],
    "lpc_shm_comm_unlink": [_P],
    "lpc_shm_allreduce": [_P, _P, _I32],
    "lpc_shm_comm_abort": [_P],
    "lpc_shm_comm_close": [_P],
}

# lpc_allreduce_fn (include/lpc.h): int (*)(void *ctx, double *vals, int32_t n)
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_int32)

EXPORTED = tuple(_PROTOS) + ("lpc_last_error",)


def _preload_hip_runtime():
    """Share ONE HIP runtime with PyTorch.  torch links its own copy
    (torch/lib/libamdhip64.so, DT_NEEDED "libamdhip64.so"); liblpc.so links
    "libamdhip64.so.7".  Loading liblpc first would bring in /opt/rocm's runtime
    and torch would later load a second one (two HSA runtimes -> "No HIP GPUs are
    available").  Preloading torch's copy RTLD_GLOBAL makes liblpc's SONAME match
    it.  LPC_HIP_RUNTIME=system keeps /opt/rocm's runtime (no torch in-process)."""
    if os.environ.get("LPC_HIP_RUNTIME", "torch") == "system":
        return None
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        return None
    cand = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    if os.path.exists(cand):
        ctypes.CDLL(cand, mode=ctypes.RTLD_GLOBAL)
        return cand
    return None


def load(path: str = LIB_PATH):
    """Load liblpc.so and declare every entry point of include/lpc.h.
    LPC_LIB_PATH names another in-tree build of the same sources (A/B of
    compile-time variants, tools/ab.py); the default is lightpycl_amd/liblpc.so."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("LPC_LIB_PATH") or path
    _preload_hip_runtime()
    if not os.path.exists(path):
        raise LpcError(f"liblpc.so not built ({path}); run lightpycl_amd.build.build() "
                       "(hipcc --offload-arch=gfx950)")
    L = ctypes.CDLL(path)
    for name, args in _PROTOS.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = ctypes.c_int
    L.lpc_last_error.argtypes = [_P]
    L.lpc_last_error.restype = ctypes.c_char_p
    if L.lpc_abi_version() != ABI_VERSION:
        raise LpcError("liblpc ABI version mismatch")
    _lib = L
    return L


def check(rc: int, handle=None):
    if rc != 0:
        msg = load().lpc_last_error(handle)
        raise LpcError(f"liblpc error {rc}: {msg.decode() if msg else ''}")


def ptr(a):
    """Data pointer of a contiguous numpy array (None -> NULL)."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "array must be C-contiguous"
    return a.ctypes.data_as(ctypes.c_void_p)


def f32(a, shape=None):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float32))
    return a.reshape(shape) if shape is not None else a


def i32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.int32))


def device_count() -> int:
    c = ctypes.c_int(0)
    check(load().lpc_device_count(ctypes.byref(c)))
    return c.value
