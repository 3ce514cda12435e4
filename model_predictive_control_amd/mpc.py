"""MPCController -- the per-step OCP of session_4 on the MI355X path.

Reference: ``MPCController`` in session_4/main.py:29-129 (and the box-only
variant session4_sol.py:113-230).  The reference builds a single-shooting
NLP in CasADi (z = [u_0..u_{N-1}], main.py:46; cost main.py:86-106) and calls
IPOPT every closed-loop step (``solve`` main.py:115-116, ``__call__``
main.py:121-129).  Here each ``solve`` is a real-time-iteration SQP step on
device:

  1.+2. nominal rollout of the forward-Euler model from x0 with the warm-
     started input sequence (previous solution shifted one stage) and the
     per-stage linearisation (A_k, B_k, c_k)    (libmpcqp ``mpcqp_bicycle_rti``),
  3.+4. time-varying condensing and the QP, with the predicted states, in
     one call                                (libmpcqp ``mpcqp_mpc_qp``),

repeated ``sqp_iters`` times.  Any number of initial states is solved in one
batch (``solve`` accepts x of shape (nx,) or (batch, nx)).

With ``state_box=True`` (default) the state box of main.py:58-61 on x_1..x_N
is enforced as well (rows  x_min - xbar <= Gam z <= x_max - xbar  of the
condensed QP; needs N*(nx+nu) <= 192, i.e. N <= 32); without it the QP has
the input box only.  The
collision rows of main.py:95-104 are non-convex and out of scope.
"""
from __future__ import annotations

import inspect
import warnings

import numpy as np
import torch

from . import batched
from .bicycle import KinematicBicycle
from .parameters import VehicleParameters


class MPCController:
    def __init__(self, N: int, ts: float, params: VehicleParameters | None = None, model=None,
                 x_obs=None, *, Q=None, QN=None, R=None, sqp_iters: int = 3,
                 state_box: bool = True, dtype=torch.float64, device=None) -> None:
        self.N = N
        self.ts = ts
        # The prediction model is linearised on device (mpcqp_bicycle_rti),
        # which reads the kinematic parameters; a model passed in (main.py:
        # 250-251 passes KinematicBicycle(params)) therefore supplies them.
        mparams = getattr(model, "params", None) if model is not None else None
        if params is None:
            params = mparams or VehicleParameters()
        elif mparams is not None and _kinematic(mparams) != _kinematic(params):
            raise ValueError("MPCController: model.params and params disagree on the "
                             "kinematic fields (axis_front, axis_rear, acceleration, friction); "
                             "the device linearisation can use only one set")
        self.params = params
        self.model = model or KinematicBicycle(self.params)
        self.x_obs = x_obs
        if x_obs is not None:
            warnings.warn("MPCController: x_obs is ignored -- the collision rows of "
                          "main.py:95-104 are non-convex and not part of the QP path",
                          stacklevel=2)
        self.nx, self.nu = 4, 2
        # weights of main.py:72-74
        Q = np.diag([1., 6., 0.2, 0.05]) if Q is None else np.asarray(Q, float)
        QN = 100 * Q if QN is None else np.asarray(QN, float)
        R = np.diag([1, 0.01]) if R is None else np.asarray(R, float)
        self.dtype = dtype
        self.device = device or torch.device("cuda")
        if not torch.cuda.is_available():
            raise RuntimeError("MPCController needs a ROCm GPU (no CPU fallback)")
        t = lambda a: torch.as_tensor(a, dtype=dtype, device=self.device)  # noqa: E731
        self.Q, self.QN, self.R = t(Q), t(QN), t(R)
        p = self.params
        # input box of main.py:68-69 (drive, steer), repeated over the horizon
        self.lb_inputs, self.ub_inputs = p.input_box()
        self.lbz = t(np.tile(self.lb_inputs, N))
        self.ubz = t(np.tile(self.ub_inputs, N))
        # state box of main.py:58-61 on x_1..x_N (the g rows of main.py:99-100)
        self.lb_states, self.ub_states = p.state_box()
        self.state_box = state_box
        if state_box and N * (self.nx + self.nu) > batched.max_qp_size(dtype):
            raise ValueError(f"state box needs N*(nx+nu) <= {batched.max_qp_size(dtype)} (N={N})")
        self.xmin = t(np.tile(self.lb_states, N))
        self.xmax = t(np.tile(self.ub_states, N))
        self.bounds = dict(lbx=np.tile(self.lb_inputs, N), ubx=np.tile(self.ub_inputs, N),
                           lbg=np.tile(self.lb_states, N), ubg=np.tile(self.ub_states, N))
        self.sqp_iters = sqp_iters
        self._warm = None
        self.last_status = None

    # ------------------------------------------------------------- solve
    def solve_batch(self, X0: torch.Tensor):
        """X0 (batch, 4) device tensor -> (z (batch, N*nu), status (batch,))."""
        N, nu = self.N, self.nu
        X0 = X0.to(self.dtype).contiguous()
        b = X0.shape[0]
        if self._warm is not None and self._warm.shape[0] == b:
            U = self._warm
        else:
            U = torch.zeros((b, N, nu), dtype=self.dtype, device=self.device)
        z = status = X = None
        for _ in range(self.sqp_iters):
            # FE rollout from x0 under U + per-stage (A_k, B_k, c_k): one launch
            A, B, c = batched.bicycle_rti(X0, U, self.params, self.ts)
            # condense + QP (+ predicted states) in one libmpcqp call
            box = dict(xlo=self.xmin, xhi=self.xmax) if self.state_box else {}
            z, lam, status, X = batched.mpc_qp(A, B, self.Q, self.R, self.QN, N, X0, c=c,
                                               lb=self.lbz, ub=self.ubz, tv=True, states=True,
                                               **box)
            self.last_lam_g = lam
            U = z.view(b, N, nu)
        # predicted states x_1..x_N of the last linearisation (IPOPT's "g" rows)
        self.last_prediction = X
        self._warm = torch.cat([U[:, 1:], U[:, -1:]], 1).contiguous()
        self.last_status = status
        return z, status

    def solve(self, x) -> dict:
        """main.py:115-116: returns {"x": (N*nu, 1)} (or (batch, N*nu))."""
        xa = np.asarray(x, dtype=float)
        single = xa.ndim == 1
        X0 = torch.as_tensor(xa.reshape(-1, self.nx), dtype=self.dtype, device=self.device)
        z, status = self.solve_batch(X0)
        zn = z.cpu().numpy()
        st = batched.status_code(status).cpu().numpy()
        g = self.last_prediction.reshape(X0.shape[0], -1).cpu().numpy()
        return {"x": zn.reshape(-1, 1) if single else zn,
                "g": g.reshape(-1, 1) if single else g,
                "status": st[0] if single else st,
                "success": bool(st[0] == 0) if single else st == 0}

    def log_step(self, log, sol, x0) -> None:
        """Append one step to a session_2/log.py:8-12 ControllerLog:
        solver_success, state_prediction (N+1, nx) = [x0; g], input_prediction (N, nu)."""
        log.solver_success.append(bool(sol["success"]))
        log.state_prediction.append(np.vstack([np.asarray(x0, float).reshape(1, -1),
                                               np.asarray(sol["g"]).reshape(-1, self.nx)]))
        log.input_prediction.append(self.reshape_input(sol))

    def reshape_input(self, sol):
        """main.py:118-119."""
        return np.reshape(sol["x"], (-1, 2))

    def __call__(self, y):
        """main.py:121-129: solve for measured state y, return u[0]."""
        return self.reshape_input(self.solve(y))[0]


def _kinematic(p) -> tuple:
    """The parameter fields the device bicycle model reads (bicycle.hip)."""
    return (float(p.axis_front), float(p.axis_rear), float(p.acceleration), float(p.friction))


def simulate(x0, dynamics, n_steps: int, policy):
    """Restatement of ``rcracers.simulator.simulate`` as used at main.py:270-271
    (source unavailable): returns the (n_steps+1, nx) state sequence; the
    policy is called as policy(x, t) when it accepts two arguments, else
    policy(x) (MPCController.__call__, main.py:121)."""
    try:
        two = len(inspect.signature(policy).parameters) >= 2
    except (TypeError, ValueError):
        two = False
    xs = [np.asarray(x0, dtype=float)]
    for t in range(n_steps):
        u = policy(xs[-1], t) if two else policy(xs[-1])
        xs.append(np.asarray(dynamics(xs[-1], u), dtype=float))
    return np.array(xs)
