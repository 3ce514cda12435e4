"""Kinematic bicycle + integrators for the session-4 MPC (session_4/main.py).

``rcracers.simulator.dynamics.KinematicBicycle`` (used at main.py:250-251,260)
is git-ignored in the reference (.gitignore:1) and absent here, so the ODE is
restated from its parameters (parameters.py:7-8,47-48) -- PARITY UNPINNED:

    x = [p_x, p_y, psi, v]   (state order of main.py:58-61, plotting.py:64,93)
    u = [a, delta]           (drive, steer: main.py:68, plotting.py:19-20)
    beta   = atan( l_r / (l_f + l_r) * tan(delta) )
    p_x'   = v cos(psi + beta)
    p_y'   = v sin(psi + beta)
    psi'   = v / l_r * sin(beta)
    v'     = acceleration * a - friction * v

``fwd_euler`` / ``runge_kutta4`` / ``exact_integration`` restate
main.py:132-170.  The batched per-stage Jacobians (A_k = I + ts df/dx,
B_k = ts df/du, c_k) of the re-linearised condensing are the device kernels
mpcqp_bicycle_rti / mpcqp_bicycle_linearise (batched.bicycle_rti).
"""
from __future__ import annotations

from typing import Callable

import numpy as np

from .parameters import VehicleParameters


class KinematicBicycle:
    """Callable  f(x, u) -> x_dot  (numpy, single state)."""

    def __init__(self, params: VehicleParameters | None = None, symbolic: bool = False):
        self.params = params or VehicleParameters()
        self.symbolic = symbolic

    def __call__(self, x, u):
        p = self.params
        x = np.asarray(x, dtype=float).reshape(-1)
        u = np.asarray(u, dtype=float).reshape(-1)
        lf, lr = p.axis_front, p.axis_rear
        beta = np.arctan(lr / (lf + lr) * np.tan(u[1]))
        return np.array([
            x[3] * np.cos(x[2] + beta),
            x[3] * np.sin(x[2] + beta),
            x[3] / lr * np.sin(beta),
            p.acceleration * u[0] - p.friction * x[3],
        ])


def fwd_euler(f: Callable, ts: float) -> Callable:
    """main.py:132-135."""
    def fw_eul(x, u):
        return x + f(x, u) * ts
    return fw_eul


def runge_kutta4(f: Callable, ts: float) -> Callable:
    """main.py:138-147."""
    def rk4_dyn(x, u):
        s1 = f(x, u)
        s2 = f(x + (ts / 2) * s1, u)
        s3 = f(x + (ts / 2) * s2, u)
        s4 = f(x + ts * s3, u)
        return x + (ts / 6) * (s1 + 2 * s2 + 2 * s3 + s4)
    return rk4_dyn


def exact_integration(f: Callable, ts: float) -> Callable:
    """main.py:150-170 (scipy odeint as the ground-truth plant)."""
    from scipy.integrate import odeint

    def dt_dyn(x, u):
        x = np.asarray(x, dtype=float)
        y = odeint(lambda xx, t: np.array(f(xx, u)).reshape([x.size]), x.reshape([x.size]), [0, ts])
        return y[-1].reshape((x.size,))
    return dt_dyn
