"""Kinematic bicycle oracle (TEST INFRASTRUCTURE ONLY) -- PARITY UNPINNED.

``rcracers.simulator.dynamics.KinematicBicycle`` (session_4/main.py:250-251)
is not available, so this restates the same ODE the product uses
(x = [p_x, p_y, psi, v], u = [a, delta]) in NumPy, with forward-Euler
(main.py:132-135) Jacobians by central finite differences -- independent of
the analytic device-side Jacobians -- and a real-time-iteration MPC step
built from the explicit-matrix condensing oracle and the exact box QP.
"""
from __future__ import annotations

import numpy as np

from . import condense as oc
from . import qp as oq


def f(x, u, lf=0.047, lr=0.05, acc=2.0, fric=1.0):
    beta = np.arctan(lr / (lf + lr) * np.tan(u[1]))
    return np.array([x[3] * np.cos(x[2] + beta), x[3] * np.sin(x[2] + beta),
                     x[3] / lr * np.sin(beta), acc * u[0] - fric * x[3]])


def fe(x, u, ts):
    return x + ts * f(x, u)


def fe_jac_fd(x, u, ts, eps=1e-7):
    A = np.zeros((4, 4))
    B = np.zeros((4, 2))
    for i in range(4):
        d = np.zeros(4); d[i] = eps
        A[:, i] = (fe(x + d, u, ts) - fe(x - d, u, ts)) / (2 * eps)
    for i in range(2):
        d = np.zeros(2); d[i] = eps
        B[:, i] = (fe(x, u + d, ts) - fe(x, u - d, ts)) / (2 * eps)
    return A, B


def rti_step(x0, U, ts, Q, QN, R, lbu, ubu, N, jac=fe_jac_fd, xmin=None, xmax=None):
    """One SQP-RTI iteration: rollout, linearise, condense, exact QP with the
    input box (main.py:68-69) and, when xmin/xmax are given, the state box on
    x_1..x_N (main.py:58-61) as rows Gam z within [xmin, xmax] - xbar."""
    xs = [np.asarray(x0, float)]
    for k in range(N - 1):
        xs.append(fe(xs[-1], U[k], ts))
    A = np.zeros((N, 4, 4)); B = np.zeros((N, 4, 2)); c = np.zeros((N, 4))
    for k in range(N):
        A[k], B[k] = jac(xs[k], U[k], ts)
        c[k] = fe(xs[k], U[k], ts) - A[k] @ xs[k] - B[k] @ U[k]
    d = oc.condense(A, B, Q, R, QN, N, x0=x0, c=c)
    if xmin is None:
        z, _, _ = oq.box_qp(d["H"], d["f"], np.tile(lbu, N), np.tile(ubu, N))
    else:
        G = np.vstack([d["Gam"], -d["Gam"]])
        h = np.concatenate([np.tile(xmax, N) - d["xbar"], d["xbar"] - np.tile(xmin, N)])
        z, _, _ = oq.poly_qp(d["H"], d["f"], G, h, np.tile(lbu, N), np.tile(ubu, N))
    return z.reshape(N, 2), d
