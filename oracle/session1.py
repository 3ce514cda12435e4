"""NumPy restatement of the session-1 reference (TEST INFRASTRUCTURE ONLY).

Restates, function by function:

* ``get_dynamics_continuous`` / ``get_dynamics_discrete``  -- FHC.py:32-48
  (identical in session1_sol.py:11-41): double integrator, Euler
  discretisation Ad = I + A*ts, Bd = B*ts.
* ``ricatti_recursion(A,B,Q,R,P_f,N)``  -- FHC.py:51-61 (``inv`` form,
  argument order Q before R, lists reversed so K[0] is the first-stage gain).
* ``riccati_recursion(A,B,R,Q,Pf,N)``   -- session1_sol.py:44-65 (``solve`` form,
  argument order R before Q).
* ``linear_simulate`` / ``linear_prediction`` -- LinearSystem.py:16-35
  (state tensor (nx, batch, T); prediction uses pred_law(x, t) for
  t = 1..horizon-1, i.e. gains[1..N-1] -- the reference quirk is kept).
* ``generic_simulate``  -- session1_sol.py:68-91 (returns (steps+1, nx) and
  the instability flag ||x|| > 100).
* ``fhc_setup``         -- FHC.py:136-142 constants (Ts=0.5, C=[1,-2/3]^T,
  Q = C C^T + 1e-3 I, R = [0.1] with shape (1,), P_f = Q).
"""
from __future__ import annotations

import numpy as np


def get_dynamics_continuous():
    """FHC.py:32-41."""
    A = np.array([[0.0, 1.0], [0.0, 0.0]])
    B = np.array([[0.0], [-1.0]])
    return A, B


def get_dynamics_discrete(ts: float):
    """FHC.py:44-48: forward-Euler discretisation."""
    A, B = get_dynamics_continuous()
    return np.eye(2) + A * ts, B * ts


def fhc_setup():
    """FHC.py:136-142 (main): returns A, B, Q, R, P_f, x0."""
    A, B = get_dynamics_discrete(0.5)
    C = np.array([[1.0], [-2.0 / 3.0]])
    Q = C @ C.T + 1e-3 * np.eye(2)
    R = np.array([0.1])
    x0 = np.array([[10.0], [10.0]])
    return A, B, Q, R, Q, x0


def ricatti_recursion(A, B, Q, R, P_f, N):
    """FHC.py:51-61 -- backward Riccati with ``inv``; R may have shape (1,)."""
    P = [np.asarray(P_f, dtype=float)]
    K = []
    for _ in range(N):
        Pn = P[-1]
        K_k = -np.linalg.inv(R + B.T @ Pn @ B) @ B.T @ Pn @ A
        P_k = Q + A.T @ Pn @ A + A.T @ Pn @ B @ K_k
        K.append(K_k)
        P.append(P_k)
    return P[::-1], K[::-1]


def riccati_recursion(A, B, R, Q, Pf, N):
    """session1_sol.py:44-65 -- same recursion via ``solve``; R before Q."""
    P = [np.asarray(Pf, dtype=float)]
    K = []
    for _ in range(N):
        Pn = P[-1]
        Kk = -np.linalg.solve(R + B.T @ Pn @ B, B.T @ Pn @ A)
        K.append(Kk)
        P.append(Q + A.T @ Pn @ (A + B @ Kk))
    return P[::-1], K[::-1]


def linear_simulate(A, B, x0, control_law, steps):
    """LinearSystem.py:20-26 -- returns the (nx, batch, steps) state tensor."""
    x = np.expand_dims(x0, axis=2)
    for t in range(1, steps):
        u = control_law(x[:, :, -1], t)
        x = np.dstack((x, A @ x[:, :, -1] + B @ u))
    return x


def linear_prediction(A, B, xt, pred_law, horizon):
    """LinearSystem.py:28-35 -- open-loop prediction (gains[1..] quirk kept)."""
    xp = np.expand_dims(xt, axis=2)
    for t in range(1, horizon):
        u = pred_law(xp[:, :, -1], t)
        xp = np.dstack((xp, A @ xp[:, :, -1] + B @ u))
    return xp


def generic_simulate(x0, f, policy, steps):
    """session1_sol.py:68-91 -- returns (np.array(x), instability_flag)."""
    unstable = False
    x = [x0]
    for t in range(steps):
        xn = f(x[-1], policy(x[-1], t))
        x.append(xn)
        if np.linalg.norm(xn) > 100 and not unstable:
            unstable = True
    return np.array(x), unstable
