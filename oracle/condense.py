"""Explicit-matrix condensing oracle (TEST INFRASTRUCTURE ONLY).

The reference builds its optimal-control problem by *single shooting*: the
decision vector is z = vertcat(u_0, ..., u_{N-1}) (stage-major,
session_4/main.py:46,110), the state is eliminated by rolling the model
forward symbolically (main.py:86-88, session4_sol.py:195-199) and the cost is

    sum_{i<N} x_i^T Q x_i + u_i^T R u_i  +  x_N^T Q_N x_N      (main.py:86,106)

with state-box rows on x_1..x_N (main.py:91-93, session4_sol.py:200-202).
For linear(ised) dynamics x_{k+1} = A_k x_k + B_k u_k + c_k this is the
condensed QP written out here with dense matrices:

    X = [x_1; ...; x_N] = Phi x0 + Gamma z + w
    H = Gamma^T Qhat Gamma + Rhat          (N*nu x N*nu)
    F = Gamma^T Qhat Phi                   (N*nu x nx)
    f = Gamma^T Qhat (Phi x0 + w)          (N*nu)      -- linear term
    J(z) = z^T H z + 2 f^T z + const       -> argmin of 1/2 z^T H z + f^T z

Everything is formed the slow, obvious way (explicit Gamma, explicit Qhat)
so that it is an independent check of the device kernel, which uses a
backward cost-to-go recursion instead.
"""
from __future__ import annotations

import numpy as np


def _stage(M, k):
    M = np.asarray(M, dtype=float)
    return M[k] if M.ndim == 3 else M


def condense(A, B, Q, R, Qf, N, x0=None, c=None):
    """Return dict(H, F, f, Gam, Phi, w, xbar) for one instance.

    A: (nx,nx) or (N,nx,nx); B: (nx,nu) or (N,nx,nu); c: None or (N,nx).
    """
    A0 = _stage(A, 0)
    B0 = _stage(B, 0)
    nx, nu = B0.shape
    n = N * nu
    m = N * nx
    Phi = np.zeros((m, nx))
    Gam = np.zeros((m, n))
    w = np.zeros(m)
    P = np.eye(nx)
    wk = np.zeros(nx)
    for k in range(N):                      # x_{k+1} = A_k x_k + B_k u_k + c_k
        Ak, Bk = _stage(A, k), _stage(B, k)
        P = Ak @ P
        Phi[k * nx:(k + 1) * nx] = P
        if k > 0:
            Gam[k * nx:(k + 1) * nx, : k * nu] = Ak @ Gam[(k - 1) * nx:k * nx, : k * nu]
        Gam[k * nx:(k + 1) * nx, k * nu:(k + 1) * nu] = Bk
        wk = Ak @ wk + (0.0 if c is None else np.asarray(c, float)[k])
        w[k * nx:(k + 1) * nx] = wk
    Qhat = np.zeros((m, m))
    for k in range(N):
        Qhat[k * nx:(k + 1) * nx, k * nx:(k + 1) * nx] = Qf if k == N - 1 else Q
    Rhat = np.kron(np.eye(N), np.asarray(R, float).reshape(nu, nu))
    H = Gam.T @ Qhat @ Gam + Rhat
    F = Gam.T @ Qhat @ Phi
    x0v = np.zeros(nx) if x0 is None else np.asarray(x0, float).reshape(nx)
    xbar = Phi @ x0v + w
    f = Gam.T @ Qhat @ xbar
    return dict(H=H, F=F, f=f, Gam=Gam, Phi=Phi, w=w, xbar=xbar)


def rollout_cost(A, B, Q, R, Qf, N, x0, z, c=None):
    """Direct restatement of the cost loop of session_4/main.py:86-106."""
    B0 = _stage(B, 0)
    nx, nu = B0.shape
    x = np.asarray(x0, float).reshape(nx)
    cost = 0.0
    for i in range(N):
        u = z[i * nu:(i + 1) * nu]
        cost += x @ Q @ x + u @ np.asarray(R, float).reshape(nu, nu) @ u
        x = _stage(A, i) @ x + _stage(B, i) @ u + (0.0 if c is None else np.asarray(c, float)[i])
    return cost + x @ Qf @ x


def rollout_states(A, B, N, x0, z, c=None):
    """x_1..x_N (N, nx) for input sequence z (stage-major)."""
    B0 = _stage(B, 0)
    nx, nu = B0.shape
    x = np.asarray(x0, float).reshape(nx)
    out = []
    for i in range(N):
        x = _stage(A, i) @ x + _stage(B, i) @ z[i * nu:(i + 1) * nu] \
            + (0.0 if c is None else np.asarray(c, float)[i])
        out.append(x)
    return np.array(out)


def pack_lower(H):
    """Row-major packed lower triangle: element (i, j<=i) at i(i+1)/2 + j."""
    n = H.shape[0]
    return np.concatenate([H[i, : i + 1] for i in range(n)])


def unpack_lower(p, n):
    H = np.zeros((n, n), dtype=np.asarray(p).dtype)
    k = 0
    for i in range(n):
        H[i, : i + 1] = p[k:k + i + 1]
        k += i + 1
    return H + np.tril(H, -1).T
