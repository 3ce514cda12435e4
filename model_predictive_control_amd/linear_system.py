"""LinearSystem -- the call surface of session_1/LinearSystem.py, unchanged.

``LinearSystem(A, B)`` keeps ``f``, ``simulate`` and ``prediction`` with the
reference's semantics (LinearSystem.py:7-35):

* x0 must be 2-D (nx, batch): the columns are independent initial states
  and the state tensor ``self.x`` is (nx, batch, steps) (LinearSystem.py:21,26);
* ``simulate`` produces ``steps`` states (t = 1 .. steps-1 are computed);
* ``prediction`` produces ``horizon`` states using ``pred_law(x, t)`` for
  t = 1 .. horizon-1 (the reference quirk of skipping gains[0] is kept).

For an arbitrary Python ``control_law`` the loop runs on the host, exactly as
the reference does (it is plumbing around a user callable).  When the law is
a linear state feedback (``AutoCruising.control_law``, see ``fhc.py``) the
whole closed loop runs on the GPU in one ``mpcqp_rollout`` launch.
"""
from __future__ import annotations

from typing import Callable

import numpy as np


class LinearSystem:
    def __init__(self, A, B) -> None:
        self.A = np.asarray(A)
        self.B = np.asarray(B)

    def set_output_eq(self, C, D) -> None:
        self.C = C
        self.D = D

    def f(self, x, u) -> np.ndarray:
        """LinearSystem.py:16-18."""
        return self.A @ x + self.B @ u

    def simulate(self, x0: np.ndarray, control_law: Callable, steps: int) -> None:
        """LinearSystem.py:20-26 (same output; the history is preallocated
        instead of re-copied by ``np.dstack`` every step)."""
        x0 = np.expand_dims(np.asarray(x0), axis=2)[:, :, 0]  # same AxisError as the reference for 1-D x0
        xs = np.empty(x0.shape + (max(steps, 1),), dtype=np.result_type(x0, self.A, self.B))
        xs[:, :, 0] = x0  # raises like np.expand_dims(x0, 2) for 1-D x0
        for t in range(1, steps):
            u_t = control_law(xs[:, :, t - 1], t)
            xs[:, :, t] = self.f(xs[:, :, t - 1], u_t)
        self.x = xs

    def prediction(self, xt: np.ndarray, pred_law: Callable, horizon: int) -> np.ndarray:
        """LinearSystem.py:28-35."""
        xt = np.expand_dims(np.asarray(xt), axis=2)[:, :, 0]
        xp = np.empty(xt.shape + (max(horizon, 1),), dtype=np.result_type(xt, self.A, self.B))
        xp[:, :, 0] = xt
        for t in range(1, horizon):
            xp[:, :, t] = self.f(xp[:, :, t - 1], pred_law(xp[:, :, t - 1], t))
        return xp

    def plot_traj(self) -> None:  # LinearSystem.py:37-40 (visualisation)
        import matplotlib.pyplot as plt

        plt.plot(self.x[0, 0, :], self.x[1, 0, :], "x", linestyle="--", color="#685BF5",
                 label="Trajectory")
        plt.legend()

    def plot_cost(self, P_N) -> None:
        pass

    def plot_pred(self, horizon: int) -> None:
        pass
