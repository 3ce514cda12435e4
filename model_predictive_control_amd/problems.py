"""Problem data of sessions 2 and 3 and the per-step controller log schema.

* ``Problem``  -- session_2/problem.py:4-33 (Ts=0.3, Q=diag(10,1),
  R=diag(0.01), p in [-150, 1], v in [-20, 25], u in [-20, 10], N=5).
* ``Problem3`` -- session_3/problem.py:8-36 (same with p_min=-120,
  v_min=-50).
* ``ControllerLog`` -- session_2/log.py:8-12 / session_3/log.py:8-12:
  per-step ``solver_success``, ``state_prediction``, ``input_prediction``
  (the ``rcracers`` BaseControllerLog parent is absent; this is a plain
  dataclass with the same fields).
* ``state_box_rows`` -- the condensed form of the state box of these
  problems (x_1..x_N within [x_min, x_max]) as rows ``G z`` with
  per-instance bounds, for ``batched.solve_poly``.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np


@dataclass
class Problem:
    Ts: float = 0.3
    Q: np.ndarray = field(default_factory=lambda: np.diag([10, 1]))
    R: np.ndarray = field(default_factory=lambda: np.diag([0.01]))
    p_min: float = -150
    p_max: float = 1.0
    v_min: float = -20
    v_max: float = 25.0
    u_min: float = -20.0
    u_max: float = 10.0
    N: int = 5
    A: np.ndarray = None
    B: np.ndarray = None

    def __post_init__(self):
        self.A = np.array([[1.0, self.Ts], [0, 1.0]])
        self.B = np.array([[0], [self.Ts]])

    @property
    def n_state(self):
        return self.A.shape[0]

    @property
    def n_input(self):
        return self.B.shape[1]

    @property
    def x_min(self):
        return np.array([self.p_min, self.v_min], dtype=float)

    @property
    def x_max(self):
        return np.array([self.p_max, self.v_max], dtype=float)


@dataclass
class Problem3(Problem):
    p_min: float = -120
    v_min: float = -50


@dataclass
class ControllerLog:
    solver_success: list = field(default_factory=list)
    state_prediction: list = field(default_factory=list)
    input_prediction: list = field(default_factory=list)
