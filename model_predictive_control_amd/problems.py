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


def state_box_rows(problem: Problem, x0, N: int | None = None):
    """The state box x_min <= x_k <= x_max on x_1..x_N of a session-2/3
    ``Problem`` in condensed form, as the rows of ``batched.solve_poly`` /
    ``batched.solve_qp``:

        x_k = A^k x0 + sum_{j<k} A^{k-1-j} B u_j     (stage-major z = [u_0..u_{N-1}])
        hl = x_min - Phi x0  <=  Gam z  <=  x_max - Phi x0 = hu

    x0 is (nx,) or (batch, nx).  Returns (G (N*nx, N*nu), hl, hu) with hl/hu
    (N*nx,) or (batch, N*nx).  Host-side problem setup (numpy), like the
    reference's own problem data (session_2/problem.py:4-33)."""
    N = problem.N if N is None else int(N)
    A = np.asarray(problem.A, float)
    B = np.asarray(problem.B, float)
    nx, nu = B.shape
    x0 = np.asarray(x0, float)
    single = x0.ndim == 1
    X0 = x0.reshape(-1, nx)
    G = np.zeros((N * nx, N * nu))
    Phi = np.zeros((N * nx, nx))
    Ak = np.eye(nx)
    AkB = [B]
    for k in range(N):
        Ak = A @ Ak
        Phi[k * nx:(k + 1) * nx] = Ak
        if k:
            AkB.append(A @ AkB[-1])
        for j in range(k + 1):
            G[k * nx:(k + 1) * nx, j * nu:(j + 1) * nu] = AkB[k - j]
    free = X0 @ Phi.T
    hl = np.tile(problem.x_min, N)[None, :] - free
    hu = np.tile(problem.x_max, N)[None, :] - free
    return (G, hl[0], hu[0]) if single else (G, hl, hu)
