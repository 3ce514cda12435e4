"""ctypes wrapper of oracle/c/mpcqp_oracle.c (TEST INFRASTRUCTURE / CPU BASELINE ONLY)."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-C", HERE, "-s"], check=True)
    return LIB


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = ctypes.CDLL(LIB)
        dp = ctypes.POINTER(ctypes.c_double)
        lib.oracle_mpc_box.restype = ctypes.c_int
        lib.oracle_mpc_box.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       dp, ctypes.c_long, dp, ctypes.c_long, dp, dp, dp, dp, dp,
                                       dp, dp, ctypes.POINTER(ctypes.c_int), ctypes.c_int]
        _lib = lib
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def mpc_box(A, B, Q, R, Qf, N, x0, lb, ub, nthreads=1):
    """Batched condense + box QP on the host.  A, B: (nx,nx)/(nx,nu) shared or
    (batch,nx,nx)/(batch,nx,nu).  Returns (z (batch, N*nu), iters (batch,))."""
    A = np.ascontiguousarray(A, float)
    B = np.ascontiguousarray(B, float)
    x0 = np.ascontiguousarray(x0, float)
    batch = x0.shape[0]
    nx, nu = B.shape[-2], B.shape[-1]
    n = N * nu
    sA = nx * nx if A.ndim == 3 else 0
    sB = nx * nu if B.ndim == 3 else 0
    lb = np.ascontiguousarray(np.broadcast_to(lb, (n,)), float)
    ub = np.ascontiguousarray(np.broadcast_to(ub, (n,)), float)
    Q = np.ascontiguousarray(Q, float)
    R = np.ascontiguousarray(np.broadcast_to(np.asarray(R, float), (nu, nu)))
    Qf = np.ascontiguousarray(Qf, float)
    z = np.empty((batch, n))
    it = np.empty(batch, dtype=np.int32)
    load().oracle_mpc_box(batch, nx, nu, N, _p(A), sA, _p(B), sB, _p(Q), _p(R), _p(Qf), _p(x0),
                          _p(lb), _p(ub), _p(z), it.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                          int(nthreads))
    return z, it
