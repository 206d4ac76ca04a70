"""ctypes binding of libgmagg.so (the C ABI declared in include/gmagg.h).

The library is built in-tree (``make`` or ``__graft_entry__.build()``) and
loaded from this package directory.  There is no fallback: if the library is
missing or was built for another ABI, ``load()`` raises.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GMAGG_LIB") or os.path.join(HERE, "libgmagg.so")
ABI_VERSION = 4

GM_MODE_IDEAL, GM_MODE_AIRCOMP = 0, 1
GM_NOISE_PHILOX, GM_NOISE_HOST = 0, 1
GM_ALGO_AUTO, GM_ALGO_STREAM, GM_ALGO_TWOPASS, GM_ALGO_GRAM, GM_ALGO_RESIDENT = 0, 1, 2, 3, 4
GM_ALGO_GRAM_F32 = 5
GM_LAYOUT_ROWS, GM_LAYOUT_PANELS = 0, 1
GM_GUARD_NONE, GM_GUARD_ACCEPTED, GM_GUARD_REJECTED, GM_GUARD_ACCEPTED_FLOOR = 0, 1, 2, 3
GM_EXCHANGE_NONE, GM_EXCHANGE_AGENT, GM_EXCHANGE_XCD_LOCAL, GM_EXCHANGE_XCD_HIER = 0, 1, 2, 3
GM_EXCHANGE_XCD_SPLIT = 4

NOISE_CB = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int64, C.POINTER(C.c_float),
                       C.POINTER(C.c_float), C.POINTER(C.c_float))
ALLREDUCE_CB = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p)


class GmOpts(C.Structure):
    _fields_ = [
        ("maxiter", C.c_int64),
        ("tol", C.c_double),
        ("eps", C.c_double),
        ("mode", C.c_int32),
        ("has_noise", C.c_int32),
        ("noise_var", C.c_double),
        ("P_max", C.c_double),
        ("seed", C.c_uint64),
        ("noise_source", C.c_int32),
        ("algo", C.c_int32),
        ("noise_cb", NOISE_CB),
        ("noise_user", C.c_void_p),
        ("check_every", C.c_int32),
        ("layout", C.c_int32),
        ("pre_oma", C.c_int32),
        ("pre_oma_var", C.c_double),
        ("pre_oma_seed", C.c_uint64),
    ]


class GmResult(C.Structure):
    _fields_ = [
        ("iters", C.c_int64),
        ("last_movement", C.c_double),
        ("converged", C.c_int32),
        ("algo_used", C.c_int32),
        ("guard", C.c_int32),
        ("gram_kind", C.c_int32),
        ("exchange", C.c_int32),
    ]


# (name, restype, argtypes) for every symbol the header declares.
_P = C.c_void_p
_I64 = C.c_int64
SIGNATURES = [
    ("gm_ctx_create", C.c_int, [C.c_int, C.POINTER(_P)]),
    ("gm_ctx_destroy", C.c_int, [_P]),
    ("gm_ctx_set_shard", C.c_int, [_P, _I64, _I64]),
    ("gm_ctx_set_allreduce", C.c_int, [_P, ALLREDUCE_CB, _P]),
    ("gm_rccl_get_unique_id", C.c_int, [_P]),
    ("gm_ctx_init_rccl", C.c_int, [_P, _P, C.c_int, C.c_int]),
    ("gm_weiszfeld_f32", C.c_int, [_P, _P, _I64, _I64, _I64, _P, _P, C.POINTER(GmOpts),
                                   C.POINTER(GmResult), _P]),
    ("gm_panel_width", _I64, [_I64]),
    ("gm_weiszfeld_batched_f32", C.c_int, [_P, _P, _I64, _I64, _I64, _I64, _I64, _P, _I64, _P,
                                           _I64, C.POINTER(GmOpts), C.POINTER(GmResult), _P]),
    ("gm_mean_f32", C.c_int, [_P, _P, _I64, _I64, _I64, _P, _P]),
    ("gm_median_f32", C.c_int, [_P, _P, _I64, _I64, _I64, _P, _P]),
    ("gm_trimmed_mean_f32", C.c_int, [_P, _P, _I64, _I64, _I64, _I64, _P, _P]),
    ("gm_krum_f32", C.c_int, [_P, _P, _I64, _I64, _I64, _I64, _P, C.POINTER(_I64), _P]),
    ("gm_mean_panels_f32", C.c_int, [_P, _P, _I64, _I64, _I64, _P, _P]),
    ("gm_median_panels_f32", C.c_int, [_P, _P, _I64, _I64, _I64, _P, _P]),
    ("gm_trimmed_mean_panels_f32", C.c_int, [_P, _P, _I64, _I64, _I64, _I64, _P, _P]),
    ("gm_krum_panels_f32", C.c_int, [_P, _P, _I64, _I64, _I64, _I64, _P, C.POINTER(_I64), _P]),
    ("gm_krum_last_info", C.c_int, [_P, C.POINTER(_I64)]),
    ("gm_oma_philox_f32", C.c_int, [_P, _P, _I64, _I64, _I64, C.c_double, C.c_uint64, _P]),
    ("gm_honest_variance_f32", C.c_int, [_P, _P, _I64, _I64, _I64, _P, _P]),
    ("gm_honest_variance_panels_f32", C.c_int, [_P, _P, _I64, _I64, _I64, _I64, _P, _P]),
    ("gm_oma_philox_batched_f32", C.c_int,
     [_P, _P, _I64, _I64, _I64, _I64, _I64, C.c_double, C.c_uint64, _P]),
    ("gm_oma_philox_panels_f32", C.c_int, [_P, _P, _I64, _I64, _I64, C.c_double, C.c_uint64,
                                            _P]),
    ("gm_oma_philox_batched_panels_f32", C.c_int,
     [_P, _P, _I64, _I64, _I64, _I64, _I64, C.c_double, C.c_uint64, _P]),
    ("gm_rows_to_panels_f32", C.c_int, [_P, _P, _I64, _I64, _I64, _P, _I64, _I64, _P]),
    ("gm_oma_apply_f32", C.c_int, [_P, _P, _I64, _I64, _I64, _P, _P, _P, _P, _P]),
    ("gm_client_chain_f32", C.c_int, [_P, _P, _I64, _P, _I64, _I64, _P, _I64, _I64, _I64,
                                      C.c_int32, C.c_float, C.c_float, _P, _P, _P, _I64,
                                      C.c_int32, _P]),
    ("gm_fill_clients_f32", C.c_int, [_P, _P, _I64, _I64, _I64, _I64, C.c_float, C.c_float,
                                      C.c_float, C.c_float, C.c_uint64, _P]),
    ("gm_fill_normal_f32", C.c_int, [_P, _P, _I64, C.c_float, C.c_float, C.c_uint64, _P]),
    ("gm_ctx_pass_timing", C.c_int, [_P, C.c_int, C.POINTER(C.c_double), C.POINTER(_I64)]),
    ("gm_last_error", C.c_char_p, []),
    ("gm_abi_version", C.c_int, []),
]

_lib = None
_lock = threading.Lock()


class GmError(RuntimeError):
    """A libgmagg call returned a negative status."""


def load():
    """Load libgmagg.so and bind every exported symbol (raises if absent)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"libgmagg.so not found at {LIB_PATH}: build it with `make` (or "
                "__graft_entry__.build()); there is no non-HIP fallback")
        lib = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        if lib.gm_abi_version() != ABI_VERSION:
            raise ImportError(f"libgmagg ABI {lib.gm_abi_version()} != {ABI_VERSION}")
        _lib = lib
        return lib


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = (_lib.gm_last_error() or b"").decode(errors="replace") if _lib else ""
        raise GmError(f"{what} failed ({rc}): {msg}")
    return rc
