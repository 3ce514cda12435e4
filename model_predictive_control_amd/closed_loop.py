"""The receding-horizon loop on device.

Reference: ``simulate(x0, dynamics, n_steps, policy=controller)`` of the
course package (rcracers, main.py:270-271; session4_sol.py:458,465): every
step calls ``MPCController.__call__`` (main.py:121-129) -- a full NLP solve --
and advances the plant (``exact_integration``/``fwd_euler``, main.py:132-170)
with the first input.  ``mpc.simulate`` restates that host loop; here the
whole loop stays on the GPU for a batch of initial states:

  per step t:  MPC solve (SQP iterations or RTI steps, no host sync)
               -> plant x_{t+1} = F(x_t, u_t)   (libmpcqp ``mpcqp_bicycle_plant``)
               -> warm start: shift U, y, pi    (``mpcqp_sqp_shift``)

and the T steps are captured once in a HIP graph and replayed.  The plant
may use its own parameters (the friction mismatch of session4_sol.py:
461-462) and integrator (FE, RK4, or RK4 with sub-steps as the stand-in for
odeint).  The per-step ``ControllerLog`` fields (session_2/log.py:8-12) are
recorded batched: solver_success (T, b), state_prediction (T, b, N+1, 4),
input_prediction (T, b, N, 2).
"""
from __future__ import annotations

import torch

from . import _native as nat
from . import batched
from .mpc import MPCController, SqpSolver
from .parameters import VehicleParameters

PLANTS = {"fe": nat.PLANT_FE, "rk4": nat.PLANT_RK4, "exact": nat.PLANT_RK4_SUB}


class ClosedLoop:
    """Batched closed loop of ``controller`` on a kinematic-bicycle plant.

    ``controller.mode == "sqp"``: each step runs up to ``iters_per_step`` SQP
    iterations from the shifted previous solution (with ``controller.fused``
    in one launch, ``mpcqp_bicycle_sqp_solve``, each instance stopping at its
    own convergence; otherwise one launch sequence per iteration, converged
    instances frozen by the step kernel), the first step --
    a cold start from U = 0 -- ``iters_first`` (default: the controller's
    ``max_iter``, at most 60); ``"rti"``: each step runs the controller's
    ``sqp_iters`` linearise + QP steps.
    """

    def __init__(self, controller: MPCController, plant: str = "fe",
                 plant_params: VehicleParameters | None = None, substeps: int = 20,
                 iters_per_step: int = 10, graph: bool = True, iters_first: int | None = None):
        if plant not in PLANTS:
            raise ValueError(f"plant must be one of {sorted(PLANTS)}, got {plant!r}")
        self.ctl = controller
        self.plant = PLANTS[plant]
        self.plant_params = plant_params or controller.params
        self.substeps = int(substeps)
        self.iters = int(iters_per_step)
        # the cold first step: the controller's own budget when the SQP runs
        # in one launch (a cap: each instance stops at its own convergence),
        # else at most 60 batch-wide iterations
        self.iters_first = int(iters_first) if iters_first is not None else \
            max(self.iters, controller.max_iter if controller.fused else min(controller.max_iter, 60))
        self.graph = graph
        self._graphs: dict = {}

    # ----------------------------------------------------------- buffers
    def _alloc(self, b: int, T: int):
        ctl, N, dev = self.ctl, self.ctl.N, self.ctl.device
        f64 = dict(dtype=torch.float64, device=dev)
        s = dict(
            xs=torch.zeros((T + 1, b, 4), **f64), us=torch.zeros((T, b, 2), **f64),
            success=torch.zeros((T, b), dtype=torch.bool, device=dev),
            iters=torch.zeros((T, b), dtype=torch.int32, device=dev),
            state_prediction=torch.zeros((T, b, N + 1, 4), **f64),
            input_prediction=torch.zeros((T, b, N, 2), **f64))
        s["sqp"] = SqpSolver(ctl, b)
        return s

    # ------------------------------------------------------------ one step
    def _mpc(self, s, t):
        ctl, N, sqp = self.ctl, self.ctl.N, s["sqp"]
        x0 = s["xs"][t]
        if ctl.mode == "rti":
            for _ in range(ctl.sqp_iters):
                A, B, c = ctl._linearise(x0, sqp.U)
                z, _, st, X = batched.mpc_qp(A, B, ctl.Q, ctl.R, ctl.QN, N, x0, c=c, lb=ctl.lbz,
                                             ub=ctl.ubz, tv=True, states=True, **ctl._box())
                sqp.U.copy_(z.view_as(sqp.U))
            sqp.X[:, 0].copy_(x0)
            sqp.X[:, 1:].copy_(X)
            s["success"][t].copy_(batched.status_code(st) == 0)
            return
        n = self.iters_first if t == 0 else self.iters
        if ctl.fused:  # every instance iterates to its own convergence, one launch
            sqp.solve(x0, n)
        else:
            for _ in range(n):
                sqp.iterate(x0)
        s["success"][t].copy_(sqp.done())
        s["iters"][t].copy_(sqp.iters())

    def _step(self, s, t):
        self._mpc(s, t)
        self._step_tail(s, t)

    def _step_tail(self, s, t):
        """The ControllerLog record, the plant and the warm-start shift of step t."""
        ctl = self.ctl
        b = s["sqp"].b
        sqp = s["sqp"]
        # ControllerLog of the step: [x_t; predicted states], the input plan
        s["state_prediction"][t].copy_(sqp.X)
        s["input_prediction"][t].copy_(sqp.U)
        p = self.plant_params
        prm = batched._bike_params(p)
        lib = nat.load()
        rc = lib.mpcqp_bicycle_plant(nat.F64, b, float(ctl.ts), prm, self.plant, self.substeps,
                                     s["xs"][t].data_ptr(), sqp.U.data_ptr(), 2 * ctl.N,
                                     s["xs"][t + 1].data_ptr(), s["us"][t].data_ptr(),
                                     batched._stream())
        nat.check(rc, "mpcqp_bicycle_plant")
        rc = lib.mpcqp_sqp_shift(nat.F64, b, ctl.N, sqp.U.data_ptr(), sqp.y.data_ptr(),
                                 sqp.pi.data_ptr(), sqp.flags.data_ptr(), sqp.rho.data_ptr(),
                                 sqp.mu.data_ptr(), sqp.kkt.data_ptr(), sqp.MU0,
                                 batched._stream())
        nat.check(rc, "mpcqp_sqp_shift")

    def _episode(self, s, T: int):
        """All T steps from s["xs"][0]: one launch (mpcqp_bicycle_mpc_loop,
        every instance its own episode) when the controller runs the fused
        SQP, else T calls of _step."""
        ctl = self.ctl
        if ctl.mode == "sqp" and ctl.fused and ctl.N <= 64:
            sqp = s["sqp"]
            sqp.reset()
            sqp.ws = batched.bicycle_mpc_loop(
                s["xs"], s["us"], s["success"], s["iters"], s["state_prediction"],
                s["input_prediction"], sqp.U, sqp.y, sqp.pi, sqp.X, sqp.state(), ctl.params,
                ctl.ts, ctl.Q, ctl.R, ctl.QN, plant_params=self.plant_params, plant=self.plant,
                substeps=self.substeps, hessian=ctl.hessian, xlo=sqp.box.get("xlo"),
                xhi=sqp.box.get("xhi"), lb=ctl.lbz, ub=ctl.ubz, tol=ctl.tol,
                iters_first=self.iters_first, iters_per_step=self.iters,
                qp_max_iter=sqp.QP_MAX_ITER,
                integrator=nat.MODEL_RK4 if ctl.integrator == "rk4" else nat.MODEL_FE,
                mu0=sqp.MU0, ws=sqp.ws)
            return
        self._reset(s)
        for t in range(T):
            self._step(s, t)

    # ---------------------------------------------------------------- run
    def run(self, X0, steps: int) -> dict:
        """X0 (b, 4) -> dict of device tensors: xs (T+1, b, 4), us (T, b, 2),
        success (T, b), iters (T, b) (SQP iterations per step; 0 in RTI mode),
        state_prediction (T, b, N+1, 4), input_prediction (T, b, N, 2)."""
        X0 = torch.as_tensor(X0, dtype=torch.float64, device=self.ctl.device).reshape(-1, 4)
        b, T = X0.shape[0], int(steps)
        key = (b, T)
        if self.graph:
            g = self._graphs.get(key)
            if g is None:
                s = self._alloc(b, T)
                s["xs"][0].copy_(X0)
                # warm up (allocations, workspaces, kernel loading) off the graph
                side = torch.cuda.Stream()
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    self._step(s, 0)
                torch.cuda.current_stream().wait_stream(side)
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    self._episode(s, T)
                g = self._graphs[key] = (graph, s)
            graph, s = g
            s["xs"][0].copy_(X0)
            graph.replay()
        else:
            s = self._alloc(b, T)
            s["xs"][0].copy_(X0)
            self._episode(s, T)
        keys = ("xs", "us", "success", "iters", "state_prediction", "input_prediction")
        # graph mode replays into buffers cached per (b, T): hand out copies, so a
        # later run() of the same shape cannot overwrite results the caller holds
        return {k: s[k].clone() if self.graph else s[k] for k in keys}

    def _reset(self, s):
        s["sqp"].reset()


def lti_box_mpc_loop(A, B, Q, R, Qf, N: int, X0, lb, ub, steps: int) -> dict:
    """The receding-horizon loop of the input-box MPC on a linear plant
    (LinearSystem.simulate, session_1/LinearSystem.py:20-26, with the
    box-constrained MPC step as the policy; simulate(...) main.py:270-271),
    all ``steps`` in one launch (``batched.mpc_box_loop``; each step
    warm-started from the shifted previous active set).  X0 (b, nx) ->
    xs (T+1, b, nx), us (T, b, nu), success (T, b), iters (T, b), and the
    ControllerLog input_prediction (T, b, N, nu)."""
    dev = torch.device("cuda")
    t = lambda a: torch.as_tensor(a, dtype=torch.float64, device=dev)  # noqa: E731
    A, B, X0 = t(A), t(B), t(X0).reshape(-1, t(A).shape[-1])
    r = batched.mpc_box_loop(A, B, t(Q), t(R), t(Qf), N, X0, lb, ub, steps, plans=True)
    nu = B.shape[-1]
    return {"xs": r["xs"], "us": r["us"], "success": batched.status_code(r["status"]) == 0,
            "iters": batched.status_iters(r["status"]),
            "input_prediction": r["zs"].reshape(steps, X0.shape[0], N, nu)}
