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
main.py:132-170.  ``fe_linearize_batched`` gives the per-stage Jacobians of the
forward-Euler model, A_k = I + ts df/dx, B_k = ts df/du and the affine term
c_k, on device (batched torch ops) for the re-linearised condensing of
``mpc.MPCController`` (BASELINE configs 3 and 5).
"""
from __future__ import annotations

from typing import Callable

import numpy as np
import torch

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


# ---------------------------------------------------------------- batched
def _beta(delta, p):
    k = p.axis_rear / (p.axis_front + p.axis_rear)
    return torch.atan(k * torch.tan(delta)), k


def f_batched(x: torch.Tensor, u: torch.Tensor, p: VehicleParameters) -> torch.Tensor:
    """x (..., 4), u (..., 2) -> x_dot (..., 4)."""
    beta, _ = _beta(u[..., 1], p)
    v, psi = x[..., 3], x[..., 2]
    return torch.stack([v * torch.cos(psi + beta), v * torch.sin(psi + beta),
                        v / p.axis_rear * torch.sin(beta),
                        p.acceleration * u[..., 0] - p.friction * v], dim=-1)


def fe_step_batched(x, u, p, ts):
    return x + ts * f_batched(x, u, p)


def fe_linearize_batched(xn: torch.Tensor, un: torch.Tensor, p: VehicleParameters, ts: float):
    """Jacobians of the FE model at (xn, un) (..., 4)/(..., 2).

    Returns A (..., 4, 4), B (..., 4, 2), c (..., 4) with
    x+ ~= A x + B u + c  (c = f_d(xn, un) - A xn - B un).
    """
    beta, k = _beta(un[..., 1], p)
    v, psi, delta = xn[..., 3], xn[..., 2], un[..., 1]
    th = psi + beta
    tdel = torch.tan(delta)
    dbeta = k / torch.cos(delta) ** 2 / (1 + (k * tdel) ** 2)
    z = torch.zeros_like(v)
    o = torch.ones_like(v)
    lr = p.axis_rear
    J = torch.stack([
        torch.stack([z, z, -v * torch.sin(th), torch.cos(th)], -1),
        torch.stack([z, z, v * torch.cos(th), torch.sin(th)], -1),
        torch.stack([z, z, z, torch.sin(beta) / lr], -1),
        torch.stack([z, z, z, -p.friction * o], -1),
    ], -2)
    Ju = torch.stack([
        torch.stack([z, -v * torch.sin(th) * dbeta], -1),
        torch.stack([z, v * torch.cos(th) * dbeta], -1),
        torch.stack([z, v * torch.cos(beta) * dbeta / lr], -1),
        torch.stack([p.acceleration * o, z], -1),
    ], -2)
    eye = torch.eye(4, dtype=xn.dtype, device=xn.device).expand_as(J)
    A = eye + ts * J
    B = ts * Ju
    xnext = fe_step_batched(xn, un, p, ts)
    c = xnext - (A @ xn.unsqueeze(-1)).squeeze(-1) - (B @ un.unsqueeze(-1)).squeeze(-1)
    return A, B, c
