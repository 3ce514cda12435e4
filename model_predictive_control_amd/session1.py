"""session1_sol -- the call surface of session_1/session1_sol.py on the MI355X path.

* ``riccati_recursion(A, B, R, Q, Pf, N)`` (session1_sol.py:44-65): NOTE the
  argument order (R before Q) differs from FHC.ricatti_recursion; same
  reversed-list outputs; computed by the ``mpcqp_riccati`` HIP kernel.
* ``simulate(x0, f, policy, steps)`` (session1_sol.py:68-91): generic host
  loop around user callables, returns (np.array of steps+1 states,
  instability flag ||x|| > 100).
* ``setup()`` (session1_sol.py:136-144) and the dynamics helpers.
"""
from __future__ import annotations

from typing import Callable

import numpy as np

from .fhc import get_dynamics_continuous, get_dynamics_discrete, ricatti_recursion

__all__ = ["get_dynamics_continuous", "get_dynamics_discrete", "riccati_recursion", "simulate",
           "setup"]


def riccati_recursion(A, B, R, Q, Pf, N: int):  # noqa: F811 -- session1_sol argument order
    """session1_sol.py:44-65 (R before Q)."""
    return ricatti_recursion(A, B, Q, R, Pf, N)


def simulate(x0: np.ndarray, f: Callable, policy: Callable, steps: int):
    """session1_sol.py:68-91."""
    unstable = False
    x = [x0]
    for t in range(steps):
        xn = f(x[-1], policy(x[-1], t))
        x.append(xn)
        if np.linalg.norm(xn) > 100 and not unstable:
            unstable = True
    return np.array(x), unstable


def setup():
    """session1_sol.py:136-144."""
    ts = 0.5
    C = np.array([[1, -2. / 3]])
    Q = C.T @ C + 1e-3 * np.eye(2)
    R = np.array([[0.1]])
    A, B = get_dynamics_discrete(ts)
    return A, B, Q, R
