"""ctypes binding of libmpcqp.so (the C ABI declared in include/mpcqp.h).

The library is built in-tree by ``__graft_entry__.build()`` (or
``make -C model_predictive_control_amd/csrc``) into
``model_predictive_control_amd/lib/libmpcqp.so``.  There is no fallback: if the
library is missing, or no GPU is present when a kernel is called, the call
raises -- the product path never silently drops to a CPU implementation.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MPCQP_LIB", os.path.join(_HERE, "lib", "libmpcqp.so"))

F64 = 0
F32 = 1
TV = 1
GAM_PACKED = 8  # mpcqp_condense: Gam as its lower block triangle
IPM = 2
STRICT = 4
STATUS_POLISHED = 1 << 24
STATUS_UNREFINED = 1 << 25
SQP_DONE = 1
SQP_EXACT = 2
SQP_FAIL = 4
SQP_PROJ = 8
SQP_HESS = {"gauss-newton": 0, "exact": 1, "exact-raw": 2}  # MPCQP_SQP_HESS_*
MODEL_FE = 0
MODEL_RK4 = 1
PLANT_FE = 0
PLANT_RK4 = 1
PLANT_RK4_SUB = 2

STATUS_OPTIMAL = 0
STATUS_MAXITER = 1
STATUS_NOT_CONVEX = 2
STATUS_INFEASIBLE = 3
STATUS_NONFINITE = 4
STATUS_NAMES = {0: "optimal", 1: "max_iter", 2: "not_convex", 3: "infeasible", 4: "nonfinite"}

# every symbol include/mpcqp.h declares, with (restype, argtypes)
_vp = ctypes.c_void_p
_i = ctypes.c_int
_i64 = ctypes.c_int64
_d = ctypes.c_double
SIGNATURES = {
    "mpcqp_abi_version": (_i, []),
    "mpcqp_last_error": (ctypes.c_char_p, []),
    "mpcqp_max_box_n": (_i, [_i]),
    "mpcqp_condense": (_i, [_i, _i, _i, _i, _i, _i,
                            _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64,
                            _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "mpcqp_solve_box": (_i, [_i, _i, _i, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64,
                             _vp, _vp, _i, _d, _vp]),
    "mpcqp_mpc_box": (_i, [_i, _i, _i, _i, _i, _i,
                           _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64,
                           _vp, _i64, _vp, _i64, _vp, _i64, _vp, _vp, _i, _d, _vp]),
    "mpcqp_solve_poly_workspace": (_i64, [_i, _i, _i, _i, _i]),
    "mpcqp_solve_poly": (_i, [_i, _i, _i, _i, _vp, _vp, _i64, _vp, _vp, _vp, _i64, _vp, _vp,
                              _vp, _vp, _vp, _i, _d, _vp, _i64, _vp]),
    "mpcqp_poly_workspace": (_i64, [_i, _i, _i, _i, _i]),
    "mpcqp_poly_setup": (_i, [_i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _i64, _vp]),
    "mpcqp_poly_solve": (_i, [_i, _i, _i, _i, _i, _i, _vp, _vp, _i64, _vp, _i64, _vp, _vp, _i64,
                              _vp, _vp, _vp, _vp, _vp, _i, _d, _vp]),
    "mpcqp_max_qp_size": (_i, [_i]),
    "mpcqp_solve_qp": (_i, [_i, _i, _i, _i, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _vp, _i64,
                            _vp, _i64, _vp, _i64, _vp, _vp, _vp, _i, _d, _vp]),
    "mpcqp_solve_qp_workspace": (ctypes.c_size_t, [_i, _i, _i, _i]),
    "mpcqp_sweep": (_i, [_i, _i, _i, _i, _vp, _i64, _vp, _i64, _vp, _i, _vp, _vp]),
    "mpcqp_solve_qp_ws": (_i, [_i, _i, _i, _i, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _vp, _i64,
                               _vp, _i64, _vp, _i64, _vp, _vp, _vp, _i, _d, _vp, ctypes.c_size_t,
                               _vp]),
    "mpcqp_solve_box_ws": (_i, [_i, _i, _i, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64,
                                _vp, _vp, _i, _d, _vp, ctypes.c_size_t, _vp]),
    "mpcqp_mpc_qp_workspace": (ctypes.c_size_t, [_i, _i, _i, _i, _i, _i]),
    "mpcqp_mpc_qp": (_i, [_i, _i, _i, _i, _i, _i,
                          _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64,
                          _vp, _i64, _vp, _vp, _i64, _vp, _i64, _vp, _i64,
                          _vp, _vp, _vp, _vp, _i, _d, _vp, ctypes.c_size_t, _vp]),
    "mpcqp_mpc_ipm_workspace": (ctypes.c_size_t, [_i, _i, _i, _i, _i]),
    "mpcqp_mpc_ipm": (_i, [_i, _i, _i, _i, _i, _i,
                           _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64,
                           _vp, _i64, _vp, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64,
                           _vp, _i64, _vp, _i64,
                           _vp, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_int32, _i, _d, _vp,
                           ctypes.c_size_t, _vp]),
    "mpcqp_mpc_box_loop": (_i, [_i] * 6 + [_vp, _i64] * 7 + [_vp] * 3 + [_vp, _i, _d, _vp]),
    "mpcqp_mpc_qp_profile": (_i, [_i]),
    "mpcqp_mpc_qp_stage_ms": (_i, [ctypes.POINTER(ctypes.c_float)]),
    "mpcqp_bicycle_hessian": (_i, [_i, _i, _i, _d, ctypes.POINTER(ctypes.c_double), _i, _vp, _vp,
                                   _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "mpcqp_bicycle_hessian_convex": (_i, [_i, _i, _i, _d, ctypes.POINTER(ctypes.c_double), _i, _vp,
                                          _vp, _vp, _vp, _vp, _vp, _vp, _vp, _d, _vp, _vp, _vp]),
    "mpcqp_bicycle_linearise": (_i, [_i, _i, _i, _d, ctypes.POINTER(ctypes.c_double), _i, _vp,
                                     _i64, _vp, _i64, _vp, _vp, _vp, _vp, _vp]),
    "mpcqp_bicycle_sqp_step": (_i, [_i, _i, _i, _d, ctypes.POINTER(ctypes.c_double), _i, _vp, _i64,
                                    _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _vp,
                                    _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _d, _vp]),
    "mpcqp_bicycle_sqp_solve_workspace": (ctypes.c_size_t, [_i, _i]),
    "mpcqp_bicycle_sqp_solve": (_i, [_i, _i, _i, _d, ctypes.POINTER(ctypes.c_double), _i, _i, _vp,
                                     _i64, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _i64, _vp, _vp,
                                     _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _d, _vp,
                                     ctypes.c_size_t, _vp]),
    "mpcqp_bicycle_mpc_loop": (_i, [_i, _i, _i, _i, _d, ctypes.POINTER(ctypes.c_double), _i, _i,
                                    ctypes.POINTER(ctypes.c_double), _i, _i, _vp, _vp, _vp, _vp,
                                    _vp, _i64, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                    _vp, _vp, _i, _i, _i, _d, _d, _vp, _vp, _vp, _vp, _vp, _vp,
                                    _vp, ctypes.c_size_t, _vp]),
    "mpcqp_bicycle_plant": (_i, [_i, _i, _d, ctypes.POINTER(ctypes.c_double), _i, _i, _vp, _vp,
                                 _i64, _vp, _vp, _vp]),
    "mpcqp_sqp_shift": (_i, [_i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _d, _vp]),
    "mpcqp_riccati": (_i, [_i, _i, _i, _i, _i, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64,
                           _vp, _i64, _vp, _vp, _vp]),
    "mpcqp_bicycle_rti": (_i, [_i, _i, _i, _d, ctypes.POINTER(ctypes.c_double), _vp, _i64, _vp, _i64,
                               _vp, _vp, _vp, _vp, _vp]),
    "mpcqp_gemv": (_i, [_i, _i, _i, _i, _d, _vp, _i64, _vp, _i64, _d, _vp, _i64, _vp]),
    "mpcqp_rollout": (_i, [_i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp]),
}

ABI_VERSION = 1

_lock = threading.Lock()
_lib = None


class MpcqpError(RuntimeError):
    """A libmpcqp entry point returned a negative code."""


def load(path: str | None = None):
    """Load (once) and return the ctypes library; raise if it is missing."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise ImportError(
                f"libmpcqp.so not found at {p}: build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` "
                "(the HIP path has no CPU fallback)")
        lib = ctypes.CDLL(p)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        v = lib.mpcqp_abi_version()
        if v != ABI_VERSION:
            raise ImportError(f"libmpcqp ABI {v} != expected {ABI_VERSION}")
        if path is None:
            _lib = lib
        return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().mpcqp_last_error().decode(errors="replace")
        raise MpcqpError(f"{what} failed ({rc}): {msg}")
