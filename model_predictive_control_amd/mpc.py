"""MPCController -- the per-step OCP of session_4 on the MI355X path.

Reference: ``MPCController`` in session_4/main.py:29-129 (and the box-only
variant session4_sol.py:113-230).  The reference builds a single-shooting
NLP in CasADi (z = [u_0..u_{N-1}], main.py:46; cost main.py:86-106; input box
main.py:68-69; state box on x_1..x_N main.py:58-61) and returns IPOPT's
optimum every closed-loop step (``solve`` main.py:115-116, ``__call__``
main.py:121-129).  Here ``solve`` returns the optimum of the same NLP, found
on device by SQP (``mode="sqp"``, the default):

  1. linearise the forward-Euler bicycle at the current inputs U
     (libmpcqp ``mpcqp_bicycle_rti``);
  2. once the optimality residual is small, the curvature of the dynamics
     weighted by the costates -- the exact Hessian of the Lagrangian
     (``mpcqp_bicycle_hessian``); before that, Gauss-Newton;
  3. the QP on the stage-wise interior point (``mpcqp_mpc_ipm``, any
     horizon: the reference's own N = 50 controllers of session4_sol.py
     included);
  4. an L1-merit line search, the update, and the first-order optimality
     (KKT) residual of the NLP at the new point (``mpcqp_bicycle_sqp_step``)
     -- iterations stop when it is below ``tol`` (status OPTIMAL), or at
     ``max_iter`` (status MAXITER).

``mode="rti"`` keeps the real-time-iteration scheme: exactly ``sqp_iters``
linearise + QP steps (``mpcqp_mpc_qp``) from the shifted previous solution,
no convergence test -- the fixed-cost step of the batched benchmark.

Any number of initial states is solved in one batch (``solve`` accepts x of
shape (nx,) or (batch, nx)).  The collision rows of main.py:95-104 are
non-convex and out of scope.
"""
from __future__ import annotations

import inspect
import os
import warnings

import numpy as np
import torch

from . import _native as nat
from . import batched
from ._native import SQP_DONE, SQP_FAIL, STATUS_MAXITER, STATUS_OPTIMAL
from .bicycle import KinematicBicycle
from .parameters import VehicleParameters

# the weights of the two reference controllers
WEIGHTS_MAIN = dict(Q=np.diag([1., 6., 0.2, 0.05]), QN_scale=100.0, R=np.diag([1., 0.01]))  # main.py:72-74
WEIGHTS_SOL = dict(Q=np.diag([1., 3., 0.1, 0.01]), QN_scale=10.0, R=np.diag([1., 1e-2]))    # session4_sol.py:166-169


class MPCController:
    def __init__(self, N: int, ts: float, params: VehicleParameters | None = None, model=None,
                 x_obs=None, *, Q=None, QN=None, R=None, mode: str = "sqp",
                 max_iter: int = 200, tol: float = 1e-9, hessian: str = "exact",
                 integrator: str = "fe",
                 sqp_iters: int = 3, state_box: bool = True, dtype=torch.float64,
                 device=None, fused: bool = True) -> None:
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
        if mode not in ("sqp", "rti"):
            raise ValueError(f"mode must be 'sqp' or 'rti', got {mode!r}")
        if hessian not in ("exact", "exact-raw", "gauss-newton"):
            raise ValueError(f"hessian must be 'exact', 'exact-raw' or 'gauss-newton', got {hessian!r}")
        if integrator not in ("fe", "rk4"):
            raise ValueError(f"integrator must be 'fe' or 'rk4', got {integrator!r}")
        # the prediction model: fwd_euler (main.py:132-135, the model of
        # main.py:76 and session4_sol.py:192) or runge_kutta4 (main.py:138-147,
        # template.py:141); the exact Hessian follows the model (RK4: the
        # second-order adjoint through its four stages)
        self.integrator = integrator
        self.mode, self.hessian = mode, hessian
        self.max_iter, self.tol = int(max_iter), float(tol)
        self.nx, self.nu = 4, 2
        Q = WEIGHTS_MAIN["Q"] if Q is None else np.asarray(Q, float)
        QN = WEIGHTS_MAIN["QN_scale"] * Q if QN is None else np.asarray(QN, float)
        R = WEIGHTS_MAIN["R"] if R is None else np.asarray(R, float)
        self.dtype = dtype if mode == "rti" else torch.float64  # the SQP runs in fp64
        self.device = device or torch.device("cuda")
        if not torch.cuda.is_available():
            raise RuntimeError("MPCController needs a ROCm GPU (no CPU fallback)")
        t = lambda a: torch.as_tensor(a, dtype=self.dtype, device=self.device)  # noqa: E731
        self.Q, self.QN, self.R = t(Q), t(QN), t(R)
        p = self.params
        # input box of main.py:68-69 (drive, steer), repeated over the horizon
        self.lb_inputs, self.ub_inputs = p.input_box()
        self.lbz = t(np.tile(self.lb_inputs, N))
        self.ubz = t(np.tile(self.ub_inputs, N))
        # state box of main.py:58-61 on x_1..x_N (the g rows of main.py:99-100)
        self.lb_states, self.ub_states = p.state_box()
        self.state_box = state_box
        self.xmin = t(np.tile(self.lb_states, N))
        self.xmax = t(np.tile(self.ub_states, N))
        self.bounds = dict(lbx=np.tile(self.lb_inputs, N), ubx=np.tile(self.ub_inputs, N),
                           lbg=np.tile(self.lb_states, N), ubg=np.tile(self.ub_states, N))
        self.sqp_iters = sqp_iters
        # SQP mode: the whole solve in one launch (SqpSolver.solve) or one
        # launch sequence per iteration over the batch (SqpSolver.iterate)
        self.fused = fused
        self._warm = None
        self._last = None
        self.last_status = None
        self.last_kkt = None
        self.last_iters = None

    @classmethod
    def from_session4_sol(cls, N: int, ts: float, *, params: VehicleParameters | None = None,
                          **kw) -> "MPCController":
        """The controller of session4_sol.py:113-230 (``MPCController(N, ts, *,
        params)``): its weights Q = diag(1, 3, .1, .01), Q_N = 10 Q,
        R = diag(1, 1e-2) (session4_sol.py:166-169), input and state box."""
        Q = WEIGHTS_SOL["Q"]
        return cls(N, ts, params, Q=Q, QN=WEIGHTS_SOL["QN_scale"] * Q, R=WEIGHTS_SOL["R"], **kw)

    # ------------------------------------------------------------- solve
    def solve_batch(self, X0: torch.Tensor):
        """X0 (batch, 4) device tensor -> (z (batch, N*nu), status (batch,))."""
        X0 = X0.to(self.dtype).contiguous()
        if self.mode == "rti":
            return self._solve_rti(X0)
        return self._solve_sqp(X0)

    def _warm_start(self, b: int):
        if self._warm is not None and self._warm.shape[0] == b:
            return self._warm.clone()
        return torch.zeros((b, self.N, self.nu), dtype=self.dtype, device=self.device)

    def _linearise(self, X0, U):
        """(A_k, B_k, c_k) along the rollout of U (the RTI linearisation)."""
        if self.integrator == "rk4":
            A, B, c, _ = batched.bicycle_linearise(X0.double(), U.double(), self.params, self.ts,
                                                   nat.MODEL_RK4)
            return A.to(self.dtype), B.to(self.dtype), c.to(self.dtype)
        return batched.bicycle_rti(X0, U, self.params, self.ts)

    def _box(self):
        return dict(xlo=self.xmin, xhi=self.xmax) if self.state_box else {}

    def _solve_rti(self, X0):
        N, nu = self.N, self.nu
        b = X0.shape[0]
        U = self._warm_start(b)
        z = status = X = None
        for _ in range(self.sqp_iters):
            # FE rollout from x0 under U + per-stage (A_k, B_k, c_k): one launch
            A, B, c = self._linearise(X0, U)
            # condense + QP (+ predicted states) in one libmpcqp call
            z, lam, status, X = batched.mpc_qp(A, B, self.Q, self.R, self.QN, N, X0, c=c,
                                               lb=self.lbz, ub=self.ubz, tv=True, states=True,
                                               **self._box())
            self.last_lam_g = lam
            U = z.view(b, N, nu)
        # IPOPT's "g", "f", "lam_x" and "lam_p" are computed by solve() only
        # (_nlp_terms): a raw batched call pays for the RTI steps alone
        self._last = dict(X0=X0, U=U, y=self.last_lam_g, X=None)
        self._warm = torch.cat([U[:, 1:], U[:, -1:]], 1).contiguous()
        self.last_status = status
        return z, status

    def _nlp_terms(self):
        """IPOPT's result terms of the last solve_batch, on demand: "g" and
        "f" are those of the NLP at the returned inputs -- the states of the
        prediction model's own rollout (RTI: not the last linearisation's),
        and the objective along it; lam_p (and lam_x in RTI mode) follow
        from the adjoint along that rollout."""
        t = self._last
        X0, U, y = t["X0"], t["U"], t["y"]
        Xn, lam_u, lam_0 = self._adjoint(X0, U, y)
        X = Xn if t["X"] is None else t["X"]
        self.last_prediction = X[:, 1:].to(self.dtype)
        if self.mode == "rti":
            self.last_lam_u = lam_u
        self.last_lam_p = lam_0
        self.last_cost = self._cost(X0, X[:, 1:], U)

    def _adjoint(self, X0, U, y):
        """The NLP's adjoint at inputs U (fp64, prediction model's rollout):
        lambda_N = Q_N x_N + y_N, lambda_k = Q x_k + y_k + A_k' lambda_{k+1},
        with y the state-row multipliers of the halved objective (> 0 at
        xhi; None = 0).  Returns the rollout X (b, N+1, 4), the input gradient
        of J/2 + y'g, R u_k + B_k' lambda_{k+1} (b, N, 2), and
        lambda_0 = Q x0 + A_0' lambda_1 (b, 4) -- the halved Lagrangian's
        derivative in x0 (oracle/nlp.py grad / lam_p)."""
        b, N = X0.shape[0], self.N
        X0d, Ud = X0.double().contiguous(), U.double().reshape(b, N, self.nu).contiguous()
        if self.integrator == "rk4":
            A, B, _, X = batched.bicycle_linearise(X0d, Ud, self.params, self.ts, nat.MODEL_RK4)
        else:
            A, B, _, X = batched.bicycle_rti(X0d, Ud, self.params, self.ts, states=True)
        Q, QN, R = self.Q.double(), self.QN.double(), self.R.double()
        Y = torch.zeros((b, N, 4), dtype=torch.float64, device=X.device) if y is None \
            else y.double().reshape(b, N, 4)
        g = torch.empty((b, N, self.nu), dtype=torch.float64, device=X.device)
        lam = X[:, N] @ QN.T + Y[:, N - 1]
        for k in range(N - 1, -1, -1):
            g[:, k] = Ud[:, k] @ R.T + torch.einsum("bij,bi->bj", B[:, k], lam)
            q = Y[:, k - 1] if k > 0 else 0.0
            lam = X[:, k] @ Q.T + q + torch.einsum("bij,bi->bj", A[:, k], lam)
        return X, g, lam

    def _solve_sqp(self, X0):
        """SQP to a first-order point of the NLP (module docstring)."""
        N, nu = self.N, self.nu
        b = X0.shape[0]
        sqp = SqpSolver(self, b)
        sqp.reset(self._warm_start(b))
        if self.fused:
            sqp.solve(X0, self.max_iter)
        else:
            for _ in range(self.max_iter):
                sqp.iterate(X0)
                if bool((sqp.flags & SQP_DONE).all()):
                    break
        status = sqp.status()
        self.last_lam_g = sqp.y
        self.last_lam_u = sqp.qp["lam_u"] if sqp.qp is not None else None
        self._last = dict(X0=X0, U=sqp.U, y=sqp.y, X=sqp.X)
        self.last_costates = sqp.pi
        self.last_kkt = sqp.kkt
        self.last_iters = sqp.iters()
        U = sqp.U
        self._warm = torch.cat([U[:, 1:], U[:, -1:]], 1).contiguous()
        self.last_status = status
        return U.reshape(b, N * nu), status

    def _cost(self, X0, X, U):
        """The reference's objective, NOT halved (main.py:86,106): sum over
        k < N of x_k'Q x_k + u_k'R u_k, plus x_N'Q_N x_N; X = x_1..x_N."""
        b = X0.shape[0]
        Xs = torch.cat([X0.reshape(b, 1, self.nx), X.reshape(b, self.N, self.nx)], 1).to(self.Q.dtype)
        Us = U.reshape(b, self.N, self.nu).to(self.Q.dtype)
        J = torch.einsum("bki,ij,bkj->b", Xs[:, :-1], self.Q, Xs[:, :-1])
        J = J + torch.einsum("bki,ij,bkj->b", Us, self.R, Us)
        return J + torch.einsum("bi,ij,bj->b", Xs[:, -1], self.QN, Xs[:, -1])

    def solve(self, x) -> dict:
        """main.py:115-116 (IPOPT through CasADi's nlpsol): returns
          "x"      (N*nu, 1) stage-major inputs (or (batch, N*nu)),
          "f"      the objective at x -- the reference's cost, not halved
                   (main.py:86,106),
          "g"      the constraint rows: the predicted states x_1..x_N,
          "lam_g"  their multipliers in IPOPT's convention for that cost
                   (> 0 at the upper bound xhi),
          "lam_x"  the input-bound multipliers (> 0 at ubx): the QP's in SQP
                   mode; in RTI mode -2 x the input gradient of the
                   Lagrangian by the adjoint along the rollout,
          "lam_p"  the multipliers of the parameter p = x0 (CasADi's
                   convention, lam_p = -d(f + lam_g'g)/dp = -2 lambda_0:
                   dJ*/dx0 = -lam_p at the optimum),
        plus "status", "success" and, in SQP mode, "kkt" (the NLP optimality
        residual) and "iterations".  The device solvers work with the halved
        cost J/2, so their multipliers are doubled here.  In RTI mode "g" and
        "f" are the prediction model's rollout of x and the objective along it
        (IPOPT's values at that x), not the last linearisation's."""
        xa = np.asarray(x, dtype=float)
        single = xa.ndim == 1
        X0 = torch.as_tensor(xa.reshape(-1, self.nx), dtype=self.dtype, device=self.device)
        z, status = self.solve_batch(X0)
        self._nlp_terms()
        zn = z.cpu().numpy()
        st = batched.status_code(status).cpu().numpy()
        b = X0.shape[0]
        g = self.last_prediction.reshape(b, -1).cpu().numpy()
        lam = (2.0 * self.last_lam_g.reshape(b, -1).double()).cpu().numpy() \
            if self.last_lam_g is not None else None
        if self.mode == "rti":  # -2 x the Lagrangian's input gradient (zero where free at a KKT point)
            lam_u = (-2.0 * self.last_lam_u.reshape(b, -1)).cpu().numpy()
        else:
            lam_u = (2.0 * self.last_lam_u.reshape(b, -1).double()).cpu().numpy() \
                if self.last_lam_u is not None else None
        lam_p = (-2.0 * self.last_lam_p).cpu().numpy()
        f = self.last_cost.double().cpu().numpy()
        one = (lambda a: a[0].reshape(-1, 1)) if single else (lambda a: a)  # noqa: E731
        out = {"x": one(zn), "f": float(f[0]) if single else f, "g": one(g),
               "status": st[0] if single else st,
               "success": bool(st[0] == 0) if single else st == 0}
        if lam is not None:
            out["lam_g"] = one(lam)
        if lam_u is not None:
            out["lam_x"] = one(lam_u)
        out["lam_p"] = one(lam_p)
        if self.mode == "sqp":
            kkt = self.last_kkt.cpu().numpy()
            it = self.last_iters.cpu().numpy()
            out["kkt"] = float(kkt[0]) if single else kkt
            out["iterations"] = int(it[0]) if single else it
        return out

    def log_step(self, log, sol, x0) -> None:
        """Append one step to a session_2/log.py:8-12 ControllerLog:
        solver_success, state_prediction (N+1, nx) = [x0; g], input_prediction
        (N, nu).  ``sol`` may be a batch (solve() of (batch, nx)): each field
        then gets the batch's arrays -- (batch,), (batch, N+1, nx),
        (batch, N, nu)."""
        x0 = np.asarray(x0, float)
        if x0.ndim == 1:
            log.solver_success.append(bool(sol["success"]))
            log.state_prediction.append(np.vstack([x0.reshape(1, -1),
                                                   np.asarray(sol["g"]).reshape(-1, self.nx)]))
            log.input_prediction.append(self.reshape_input(sol))
            return
        b = x0.shape[0]
        g = np.asarray(sol["g"]).reshape(b, -1, self.nx)
        log.solver_success.append(np.asarray(sol["success"], bool).reshape(b))
        log.state_prediction.append(np.concatenate([x0.reshape(b, 1, self.nx), g], 1))
        log.input_prediction.append(np.asarray(sol["x"]).reshape(b, -1, self.nu))

    def reshape_input(self, sol):
        """main.py:118-119."""
        return np.reshape(sol["x"], (-1, 2))

    def __call__(self, y):
        """main.py:121-129: solve for measured state y, return u[0]."""
        return self.reshape_input(self.solve(y))[0]


class SqpSolver:
    """Device state of the batched SQP of ``MPCController`` (mode "sqp") for
    a batch of b initial states, preallocated so that ``iterate`` -- one SQP
    iteration, four libmpcqp launches, no host synchronisation -- can be
    repeated or captured in a HIP graph:

      mpcqp_bicycle_rti -> mpcqp_bicycle_hessian -> mpcqp_mpc_ipm
      -> mpcqp_bicycle_sqp_step

    Instances that reach the KKT tolerance are frozen by the step kernel
    (flag SQP_DONE): the interior point skips them and the others keep
    iterating."""

    MU0 = 1e-3  # initial Levenberg-Marquardt damping of the exact-Hessian QPs
    # interior-point budget of one QP: a convex one takes 6-10 iterations; one
    # that stalls is abandoned and the step kernel switches to the projected
    # curvature or raises the damping instead.  Every launch lasts as long as
    # its slowest QP, so the cap is also the batch's per-iteration time: 25
    # against 40 is +18 % converged NLP solves/s at 0.992 instead of 0.994
    # converged in 60 iterations (MPCQP_SQP_QP_MAX_ITER overrides)
    QP_MAX_ITER = int(os.environ.get("MPCQP_SQP_QP_MAX_ITER", "25"))
    # the QP takes as many inertia corrections as it needs (not strict): the
    # exact-Hessian QP is often non-convex away from its active face while
    # the barrier terms of the active bounds are still small; the inputs the
    # step kernel holds at their bounds (fix) remove the directions along
    # which it is non-convex at the solution
    STRICT = False

    def __init__(self, ctl: "MPCController", b: int):
        self.ctl, self.b = ctl, b
        N, dev = ctl.N, ctl.device
        f64 = dict(dtype=torch.float64, device=dev)
        self.U = torch.zeros((b, N, 2), **f64)
        self.y = torch.zeros((b, N * 4), **f64)
        self.pi = torch.zeros((b, N, 4), **f64)
        self.X = torch.zeros((b, N + 1, 4), **f64)
        self.rho = torch.zeros(b, **f64)
        self.kkt = torch.full((b,), float("inf"), **f64)
        self.mu = torch.full((b,), self.MU0, **f64)
        self.flags = torch.zeros(b, dtype=torch.int32, device=dev)
        self.fix = torch.zeros((b, N), dtype=torch.int32, device=dev)
        self.qp = None
        self.box = ctl._box()
        self.ws = None  # workspace of the one-launch solve

    def state(self) -> dict:
        # held inputs exist only for exact-Hessian QPs (the proximal term of
        # bicycle_hessian); a Gauss-Newton controller never builds H2
        fix = None if self.ctl.hessian == "gauss-newton" else self.fix
        return dict(rho=self.rho, kkt=self.kkt, mu=self.mu, flags=self.flags, fix=fix)

    def reset(self, U0=None):
        """Cold (U0 None: zeros) or warm start; multipliers and state cleared."""
        if U0 is None:
            self.U.zero_()
        else:
            self.U.copy_(U0)
        self.y.zero_()
        self.pi.zero_()
        self.rho.zero_()
        self.kkt.fill_(float("inf"))
        self.mu.fill_(self.MU0)
        self.flags.zero_()
        self.fix.zero_()

    def iterate(self, X0):
        ctl, N, box = self.ctl, self.ctl.N, self.box
        if ctl.integrator == "rk4":
            A, B, c, Xr = batched.bicycle_linearise(X0, self.U, ctl.params, ctl.ts, nat.MODEL_RK4)
        else:
            A, B, c, Xr = batched.bicycle_rti(X0, self.U, ctl.params, ctl.ts, states=True)
        H2 = q2 = None
        if ctl.hessian != "gauss-newton":
            # "exact": the Lagrangian curvature; after a QP that it made
            # non-convex, projected per stage for a few steps (flag SQP_PROJ,
            # set by the step kernel); "exact-raw": never projected, the
            # damping mu handles indefiniteness
            cw = dict(Q=ctl.Q, R=ctl.R) if ctl.hessian == "exact" else {}
            H2, q2 = batched.bicycle_hessian(Xr, self.U, self.pi, ctl.params, ctl.ts,
                                             flags=self.flags, mu=self.mu, fix=self.fix,
                                             integrator=nat.MODEL_RK4 if ctl.integrator == "rk4"
                                             else nat.MODEL_FE, **cw)
        self.qp = batched.mpc_ipm(A, B, ctl.Q, ctl.R, ctl.QN, N, X0, lb=ctl.lbz, ub=ctl.ubz,
                                  c=c, tv=True, H2=H2, q2=q2, strict=self.STRICT, skip=self.flags,
                                  skip_mask=SQP_DONE, max_iter=self.QP_MAX_ITER, out=self.qp,
                                  **box)
        batched.bicycle_sqp_step(X0, self.U, self.qp["z"], self.qp["y"], self.qp["pi"], self.y,
                                 self.pi, self.X, self.state(), ctl.params, ctl.ts, ctl.Q, ctl.R,
                                 ctl.QN, xlo=box.get("xlo"), xhi=box.get("xhi"), lb=ctl.lbz,
                                 ub=ctl.ubz, tol=ctl.tol, qp_status=self.qp["status"],
                                 integrator=nat.MODEL_RK4 if ctl.integrator == "rk4" else nat.MODEL_FE)

    def solve(self, X0, max_iter: int):
        """Up to ``max_iter`` more iterations per instance in ONE launch
        (mpcqp_bicycle_sqp_solve): each instance iterates until its own KKT
        residual is below tol, in its own workgroup -- the same iterations as
        ``iterate`` repeated (linearisation of mpcqp_bicycle_linearise), but
        the launch lasts as long as the slowest instance's solve instead of
        the sum over iterations of each iteration's slowest QP.  Continues
        from the current state (reset() first for a fresh solve)."""
        ctl = self.ctl
        if self.qp is None or "ws_solve" not in self.qp:
            b, N, dev = self.b, ctl.N, ctl.device
            self.qp = {"lam_u": torch.zeros((b, N * 2), dtype=torch.float64, device=dev),
                       "status": torch.zeros(b, dtype=torch.int32, device=dev), "ws_solve": True}
        self.ws = batched.bicycle_sqp_solve(
            X0, self.U, self.y, self.pi, self.X, self.state(), ctl.params, ctl.ts, ctl.Q, ctl.R,
            ctl.QN, hessian=ctl.hessian, xlo=self.box.get("xlo"), xhi=self.box.get("xhi"),
            lb=ctl.lbz, ub=ctl.ubz, tol=ctl.tol, max_iter=max_iter, qp_max_iter=self.QP_MAX_ITER,
            integrator=nat.MODEL_RK4 if ctl.integrator == "rk4" else nat.MODEL_FE,
            lam_u=self.qp["lam_u"], qp_status=self.qp["status"], ws=self.ws)

    def done(self):
        """Converged instances (KKT <= tol)."""
        return ((self.flags & SQP_DONE) != 0) & ((self.flags & SQP_FAIL) == 0)

    def iters(self):
        return (self.flags >> 8) & 0xFFFF

    def status(self):
        """MPCQP status words: OPTIMAL (KKT <= tol), MAXITER, or the status
        of the QP that stopped the instance (a Gauss-Newton QP failing
        repeatedly); iterations in bits 8..23."""
        failed = (self.flags & SQP_FAIL) != 0
        code = torch.where(self.done(), STATUS_OPTIMAL, STATUS_MAXITER).to(torch.int32)
        code = torch.where(failed, (self.flags >> 28) & 0x7, code).to(torch.int32)
        return code | (self.iters() << 8)


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
