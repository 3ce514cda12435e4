"""Multi-core CPU baselines (TEST/BENCH INFRASTRUCTURE ONLY -- bench.py's
cpu_baseline leg): the oracle's per-x0 solves spread over the host cores,
as SURVEY.md 8(d) asks ("per-x0 solves are spread across all host cores with
multiprocessing").  Workers are started with the 'spawn' method (fresh
interpreters that never touch the GPU) and each runs its chunk of instances
until a common deadline; the rate is instances done / wall time.
"""
from __future__ import annotations

import multiprocessing as mp
import os
import time

import numpy as np


def host_cores(cap: int = 16) -> int:
    """CPU share of this process (a GPU box shares its host: at most ``cap``)."""
    return max(1, min(cap, len(os.sched_getaffinity(0))))


_BLAS_ENV = ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS")


def _noop(_):
    return os.getpid()


# ----------------------------------------------------------------- workers
def cfg3_chunk(a):
    from oracle import condense as oc
    from oracle import qp as oq

    A, B, c, X0, Q, R, QN, N, xmin, xmax, lb, ub, deadline = a
    done = 0
    for i in range(A.shape[0]):
        if time.time() >= deadline:
            break
        d = oc.condense(A[i], B[i], Q, R, QN, N, x0=X0[i], c=c[i])
        G = np.vstack([d["Gam"], -d["Gam"]])
        h = np.concatenate([np.tile(xmax, N) - d["xbar"], -(np.tile(xmin, N) - d["xbar"])])
        try:
            oq.poly_qp(d["H"], d["f"], G, h, lb, ub)
        except ValueError:
            pass
        done += 1
    return done


def cfg4_chunk(a):
    from oracle import qp as oq

    H, F, G, h, X0, deadline = a
    done = 0
    for i in range(X0.shape[0]):
        if time.time() >= deadline:
            break
        oq.poly_qp(H, F @ X0[i], G, h)
        done += 1
    return done


def cfg5_chunk(a):
    from oracle import condense as oc
    from oracle import qp as oq

    A, B, X0, Q, R, N, lo, hi, deadline = a
    n = N * B.shape[-1]
    done = 0
    for i in range(A.shape[0]):
        if time.time() >= deadline:
            break
        d = oc.condense(A[i], B[i], Q, R, Q, N, x0=X0[i])
        oq.box_qp(d["H"], d["f"], np.full(n, lo), np.full(n, hi))
        done += 1
    return done


def nlp_chunk(a):
    from oracle import nlp

    N, ts, Q, QN, R, xlo, lbu, X0, deadline = a
    ocp = nlp.OCP(N, ts, Q, QN, R, xlo, -xlo, lbu, -lbu)
    done = 0
    for i in range(X0.shape[0]):
        if time.time() >= deadline:
            break
        ocp.solve(X0[i], tol=1e-9)
        done += 1
    return done


def loop_chunk(a):
    """The reference's closed loop on the host (simulate(x0, dynamics, n, policy),
    session_4/main.py:270-271): per sample one converged NLP solve (oracle/nlp.py,
    warm-started from the shifted previous solution, as the device loop is), u_0
    through the forward-Euler plant.  Returns the closed-loop steps done before
    the deadline."""
    from oracle import nlp

    N, ts, Q, QN, R, xlo, lbu, X0, T, deadline = a
    ocp = nlp.OCP(N, ts, Q, QN, R, xlo, -xlo, lbu, -lbu)
    done = 0
    for i in range(X0.shape[0]):
        x, U = np.asarray(X0[i], float), None
        for _ in range(T):
            if time.time() >= deadline:
                return done
            U, _, _ = ocp.solve(x, U0=U, tol=1e-9)
            U = np.asarray(U, float).reshape(N, 2)
            x = nlp.fe(x, U[0], ts)
            U = np.vstack([U[1:], U[-1:]])
            done += 1
    return done


# -------------------------------------------- spot-check solves (bench check)
def cfg3_solve(a):
    """Oracle solutions of config-3 instances (None where infeasible)."""
    from oracle import condense as oc
    from oracle import qp as oq

    A, B, c, X0, Q, R, QN, N, xlo, xhi, lb, ub = a
    out = []
    for i in range(A.shape[0]):
        d = oc.condense(A[i], B[i], Q, R, QN, N, x0=X0[i], c=c[i])
        G = np.vstack([d["Gam"], -d["Gam"]])
        h = np.concatenate([xhi - d["xbar"], -(xlo - d["xbar"])])
        try:
            out.append(oq.poly_qp(d["H"], d["f"], G, h, lb, ub)[0])
        except ValueError:
            out.append(None)
    return out


def cfg4_solve(a):
    from oracle import qp as oq

    H, F, G, h, X0 = a
    return [oq.poly_qp(H, F @ X0[i], G, h)[0] for i in range(X0.shape[0])]


def cfg5_solve(a):
    from oracle import condense as oc
    from oracle import qp as oq

    A, B, X0, Q, R, N, lo, hi = a
    n = N * B.shape[-1]
    out = []
    for i in range(A.shape[0]):
        d = oc.condense(A[i], B[i], Q, R, Q, N, x0=X0[i])
        out.append(oq.box_qp(d["H"], d["f"], np.full(n, lo), np.full(n, hi))[0])
    return out


def solve_map(worker, make_args, total: int, cores: int | None = None) -> list:
    """``worker`` over chunks [lo, hi) of ``total`` instances on ``cores``
    spawned processes (one BLAS thread each); the per-instance results in
    order."""
    if total <= 0:
        return []
    cores = min(cores or host_cores(), max(1, total))
    ctx = mp.get_context("spawn")
    saved = {k: os.environ.get(k) for k in _BLAS_ENV}
    os.environ.update({k: "1" for k in _BLAS_ENV})
    try:
        pool = ctx.Pool(cores)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    per = -(-total // cores)
    try:
        parts = pool.map(worker, [make_args(k * per, min(total, (k + 1) * per))
                                  for k in range(cores) if k * per < total])
    finally:
        _shutdown(pool)
    return [x for part in parts for x in part]


def _shutdown(pool) -> None:
    """Let the workers exit on their own (close + join).  Leaving ``with pool:``
    calls Pool.terminate(), which SIGTERMs every worker -- under rocprofv3 its
    preloaded signal handler reports each one as an abort in the run's log."""
    pool.close()
    pool.join()


def rate(worker, make_args, total: int, seconds: float, cores: int | None = None) -> dict:
    """Run ``worker`` over ``cores`` spawned processes; ``make_args(lo, hi,
    deadline)`` builds the argument of the chunk [lo, hi) of ``total``
    instances.  Returns dict(value=instances/s, done, seconds, cores)."""
    cores = cores or host_cores()
    ctx = mp.get_context("spawn")
    # one BLAS thread per worker (the workers ARE the parallelism); the
    # spawned interpreters read these when they import NumPy
    saved = {k: os.environ.get(k) for k in _BLAS_ENV}
    os.environ.update({k: "1" for k in _BLAS_ENV})
    try:
        pool = ctx.Pool(cores)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    try:
        pool.map(_noop, range(cores))          # every worker up before the clock
        t0 = time.time()
        deadline = t0 + seconds
        per = -(-total // cores)
        args = [make_args(k * per, min(total, (k + 1) * per), deadline) for k in range(cores)
                if k * per < total]
        counts = pool.map(worker, args)
        dt = time.time() - t0
    finally:
        _shutdown(pool)
    done = int(sum(counts))
    return {"value": done / dt, "done": done, "seconds": dt, "cores": cores}
