"""GPU parity: the CONVERGED MPCController.solve (SQP on device: bicycle_rti
-> bicycle_hessian -> mpc_ipm -> bicycle_sqp_step) against the NLP-optimal
fixtures of tests/golden/nlp_s4.npz -- the optimum of the NLP IPOPT solves in
the reference's MPCController.solve (session_4/main.py:115-116 on the OCP of
main.py:41-113 without the non-convex collision rows; session4_sol.py:132-217
exactly), from oracle/nlp.py (SQP + Newton polish, KKT < 1e-11) and agreeing
with SciPy SLSQP.  The bicycle ODE itself is the build's restatement
(rcracers is absent): parity of the model is unpinned, parity of the
optimiser on that model is what these tests pin."""
import numpy as np
import pytest
import torch

from model_predictive_control_amd import batched
from model_predictive_control_amd.mpc import MPCController
from model_predictive_control_amd.parameters import VehicleParameters
from oracle import nlp

pytestmark = pytest.mark.gpu

TOL_U = 1e-7      # the fixtures are KKT points to 1e-11; the bar is 1e-5
TOL_U_STRAG = 5e-7  # nlp_maxiter.npz's ill-conditioned stragglers (see the test)
TOL_KKT = 1e-8


def _ocp(g, tag):
    xlo, lbu = g["xlo"], g["lbu"]
    return nlp.OCP(int(g[f"{tag}_N"]), float(g[f"{tag}_ts"]), g[f"{tag}_Q"], g[f"{tag}_QN"],
                   g[f"{tag}_R"], xlo, -xlo, lbu, -lbu)


def _controller(g, tag):
    N, ts = int(g[f"{tag}_N"]), float(g[f"{tag}_ts"])
    if tag == "sol":  # session4_sol.py:342,455: MPCController(N=50, ts=0.05, params=...)
        return MPCController.from_session4_sol(N, ts, params=VehicleParameters())
    return MPCController(N, ts, VehicleParameters())  # main.py:242-251 weights and box


@pytest.mark.parametrize("tag", ["main", "sol"])
def test_solve_matches_nlp_fixtures(golden, tag):
    """One solve per fixture x0 (the reference's single-x0 call surface):
    u within 1e-7 of the NLP optimum, status optimal, NLP KKT residual (the
    device's and the oracle's evaluation of it) below 1e-8."""
    g = golden("nlp_s4.npz")
    ocp = _ocp(g, tag)
    X0, Ustar = g[f"{tag}_x0"], g[f"{tag}_U"]
    for i, x0 in enumerate(X0):
        ctl = _controller(g, tag)
        sol = ctl.solve(x0)
        U = np.asarray(sol["x"]).reshape(-1)
        assert sol["success"], (i, sol["status"], sol["kkt"], sol["iterations"])
        assert sol["kkt"] < TOL_KKT, (i, sol["kkt"])
        err = np.abs(U - Ustar[i]).max()
        assert err < TOL_U, (i, err)
        # the oracle's own evaluation of first-order optimality at (U, lam_g)
        # (IPOPT's multipliers for the unhalved cost: the oracle's halved y x 2)
        assert ocp.kkt(x0, U, np.asarray(sol["lam_g"]).reshape(-1) / 2) < 10 * TOL_KKT
        # g: the predicted states x_1..x_N along the solution
        assert np.abs(np.asarray(sol["g"]).reshape(-1, 4) - g[f"{tag}_X"][i][1:]).max() < 1e-6
        # __call__ (main.py:121-129) returns u_0 of a fresh solve
        u0 = _controller(g, tag)(x0)
        assert np.abs(u0 - Ustar[i][:2]).max() < TOL_U


@pytest.mark.parametrize("tag", ["main", "sol"])
def test_solve_returns_ipopt_result_mapping(golden, tag):
    """main.py:115-116 returns CasADi's nlpsol dict: "f" is the reference's
    objective (not halved, main.py:86,106), "lam_g" the state-row and "lam_x"
    the input-bound multipliers in IPOPT's convention for that objective
    (> 0 at the upper bound).  Against the oracle at the fixture optimum: f =
    cost(U*), lam_g = 2 y*, lam_x = -2 grad(J/2 + y*'g)(U*) (zero on free
    inputs, the bound's multiplier on active ones)."""
    g = golden("nlp_s4.npz")
    ocp = _ocp(g, tag)
    X0, Ustar, Ystar = g[f"{tag}_x0"], g[f"{tag}_U"], g[f"{tag}_y"]
    sol = _controller(g, tag).solve(X0)
    assert np.asarray(sol["success"]).all()
    for i, x0 in enumerate(X0):
        J = ocp.cost(x0, Ustar[i])
        assert abs(J - g[f"{tag}_J"][i]) < 1e-9 * (1 + abs(J))
        assert abs(sol["f"][i] - J) < 1e-8 * (1 + abs(J)), (i, sol["f"][i], J)
        lam_g = 2 * Ystar[i]
        assert np.abs(sol["lam_g"][i] - lam_g).max() < 1e-6 * (1 + np.abs(lam_g).max())
        grad, _ = ocp.grad(x0, Ustar[i], Ystar[i])
        lam_x = -2 * grad
        assert np.abs(sol["lam_x"][i] - lam_x).max() < 1e-6 * (1 + np.abs(lam_x).max()), i
    one = _controller(g, tag).solve(X0[0])
    assert isinstance(one["f"], float) and one["lam_x"].shape == (Ustar.shape[1], 1)


@pytest.mark.parametrize("tag", ["main", "sol"])
def test_batched_solve_equals_single(golden, tag):
    """All fixture x0 in one batched call: the same optimum per instance."""
    g = golden("nlp_s4.npz")
    X0, Ustar = g[f"{tag}_x0"], g[f"{tag}_U"]
    sol = _controller(g, tag).solve(X0)
    assert np.asarray(sol["success"]).all(), (sol["status"], sol["kkt"])
    assert np.abs(np.asarray(sol["x"]) - Ustar).max() < TOL_U
    assert (np.asarray(sol["kkt"]) < TOL_KKT).all()


def test_n50_state_box_controller_runs(golden):
    """session4_sol.py:342 exercise3 exactly: N = 50, ts = 0.05, x0 =
    [0.6, -0.25, 0, 0] with the state box (n + m = 300: the case the dense
    kernels' 192 cap refused)."""
    g = golden("nlp_s4.npz")
    ctl = MPCController.from_session4_sol(50, 0.05, params=VehicleParameters())
    sol = ctl.solve(np.array([0.6, -0.25, 0.0, 0.0]))
    assert sol["success"] and sol["kkt"] < TOL_KKT
    assert np.abs(ctl.reshape_input(sol) - g["sol_U"][0].reshape(-1, 2)).max() < TOL_U


def test_saturated_tail_fixtures(golden):
    """The saturated tail of the nlp bench's x0 distribution
    (tests/golden/nlp_tail.npz: 24-27 of the 60 inputs at a bound at the
    optimum, oracle KKT < 1e-11): every instance converges within the
    controller's default iteration budget, in one batched solve, to the
    oracle's optimum (u to 1e-7, KKT < 1e-8)."""
    g = golden("nlp_tail.npz")
    ctl = MPCController(int(g["N"]), float(g["ts"]), VehicleParameters())
    sol = ctl.solve(g["x0"])
    its = np.asarray(sol["iterations"])
    assert np.asarray(sol["success"]).all(), (sol["status"], sol["kkt"], its)
    assert (np.asarray(sol["kkt"]) < TOL_KKT).all(), sol["kkt"]
    err = np.abs(np.asarray(sol["x"]) - g["U"]).max(1)
    assert err.max() < TOL_U, (err, its)
    assert its.max() <= 60, its


def test_hessian_convex_projection(dev):
    """mpcqp_bicycle_hessian_convex: per stage, blkdiag(Q, R) + H2 is
    positive definite (eigenvalues >= eps up to rounding); stages where the
    exact one already is keep the exact curvature; q2 = -H2 w."""
    p = VehicleParameters()
    rng = np.random.default_rng(23)
    b, N, ts = 4, 6, 0.08
    X = rng.normal(size=(b, N + 1, 4)) * [1, 1, 1, 0.3]
    U = rng.uniform(-0.35, 0.35, (b, N, 2))
    pi = rng.normal(size=(b, N, 4)) * np.array([30, 30, 3, 3])  # large costates: indefinite
    Q, R = np.diag([1., 6., .2, .05]), np.diag([1., .01])
    t = lambda a: torch.as_tensor(a, dtype=torch.float64, device=dev)  # noqa: E731
    H_ex, _ = batched.bicycle_hessian(t(X), t(U), t(pi), p, ts)
    H_cv, q_cv = batched.bicycle_hessian(t(X), t(U), t(pi), p, ts, Q=t(Q), R=t(R), eps=1e-6)
    torch.cuda.synchronize()
    H_ex, H_cv, q_cv = H_ex.cpu().numpy(), H_cv.cpu().numpy(), q_cv.cpu().numpy()
    Wb = np.zeros((6, 6)); Wb[:4, :4] = Q; Wb[4:, 4:] = R
    projected = 0
    for i in range(b):
        for k in range(N):
            ev_ex = np.linalg.eigvalsh(Wb + H_ex[i, k])
            ev_cv = np.linalg.eigvalsh(Wb + H_cv[i, k])
            assert ev_cv.min() > 1e-6 - 1e-9, ev_cv
            if ev_ex.min() > 1e-6:
                assert np.abs(H_cv[i, k] - H_ex[i, k]).max() < 1e-15
            else:
                projected += 1
                # the projection only lifts eigenvalues: W' - W is PSD
                assert np.linalg.eigvalsh(H_cv[i, k] - H_ex[i, k]).min() > -1e-9
            w = np.concatenate([X[i, k], U[i, k]])
            assert np.abs(q_cv[i, k] + H_cv[i, k] @ w).max() < 1e-12 * (1 + np.abs(q_cv[i, k]).max())
    assert projected > 0


@pytest.mark.parametrize("integ", ["fe", "rk4"])
def test_hessian_kernel_vs_oracle(dev, integ):
    """mpcqp_bicycle_hessian (FE: analytic second derivatives; RK4: the
    second-order adjoint through the four stages, bike.hpp) against the
    oracle's complex-step + central-difference curvature of fwd_euler /
    runge_kutta4 (main.py:132-147)."""
    from model_predictive_control_amd import _native as nat

    p = VehicleParameters()
    rng = np.random.default_rng(21)
    b, N, ts = 3, 5, 0.08
    X = rng.normal(size=(b, N + 1, 4)) * [1, 1, 1, 0.3]
    U = rng.uniform(-0.35, 0.35, (b, N, 2))
    pi = rng.normal(size=(b, N, 4)) * 10
    t = lambda a: torch.as_tensor(a, dtype=torch.float64, device=dev)  # noqa: E731
    H2, q2 = batched.bicycle_hessian(t(X), t(U), t(pi), p, ts,
                                     integrator=nat.MODEL_RK4 if integ == "rk4" else nat.MODEL_FE)
    torch.cuda.synchronize()
    H2, q2 = H2.cpu().numpy(), q2.cpu().numpy()
    for i in range(b):
        for k in range(N):
            w = np.concatenate([X[i, k], U[i, k]])
            L = nlp._stage_curvature(w, pi[i, k], ts, nlp.PARAMS, step=nlp.STEPS[integ])
            assert np.abs(H2[i, k] - L).max() < 1e-6 * (1 + np.abs(L).max())
            assert np.abs(q2[i, k] + H2[i, k] @ w).max() < 1e-12 * (1 + np.abs(q2[i, k]).max())


def test_gauss_newton_mode_and_rti_mode(golden):
    """hessian='gauss-newton' converges to the same optimum (more
    iterations); mode='rti' keeps the fixed-iteration scheme (no KKT)."""
    g = golden("nlp_s4.npz")
    x0, Ustar = g["main_x0"][0], g["main_U"][0]
    gn = MPCController(30, 0.08, VehicleParameters(), hessian="gauss-newton", max_iter=400,
                       tol=1e-8)
    s1 = gn.solve(x0)
    ex = MPCController(30, 0.08, VehicleParameters())
    s2 = ex.solve(x0)
    assert s1["success"] and s2["success"]
    assert s2["iterations"] < s1["iterations"]
    assert np.abs(np.asarray(s1["x"]).reshape(-1) - Ustar).max() < 1e-5
    rti = MPCController(30, 0.08, VehicleParameters(), mode="rti", sqp_iters=3)
    s3 = rti.solve(x0)
    assert "kkt" not in s3 and np.asarray(s3["x"]).shape == (60, 1)


def test_receding_horizon_warm_start(golden):
    """Consecutive solves along the closed loop (main.py:270-271) start from
    the shifted previous solution and need fewer iterations than a cold
    start; every step converges."""
    g = golden("nlp_s4.npz")
    ctl = MPCController(30, 0.08, VehicleParameters())
    x = g["main_x0"][0].copy()
    its = []
    for _ in range(5):
        sol = ctl.solve(x)
        assert sol["success"] and sol["kkt"] < TOL_KKT
        its.append(sol["iterations"])
        x = nlp.fe(x, ctl.reshape_input(sol)[0], 0.08)
    assert max(its[1:]) < its[0], its


@pytest.mark.parametrize("integ", ["fe", "rk4"])
def test_linearise_kernel_vs_complex_step(dev, integ):
    """mpcqp_bicycle_linearise (FE: analytic; RK4: forward sensitivities
    through the four stages) against the oracle's complex-step Jacobians of
    fwd_euler / runge_kutta4 (main.py:132-147) along the same rollout."""
    from model_predictive_control_amd import _native as nat

    p = VehicleParameters()
    rng = np.random.default_rng(5)
    b, N, ts = 4, 12, 0.08
    X0 = rng.normal(size=(b, 4)) * [0.5, 0.5, 0.5, 0.2]
    U = rng.uniform(-0.38, 0.38, (b, N, 2))
    t = lambda a: torch.as_tensor(a, dtype=torch.float64, device=dev)  # noqa: E731
    A, B, c, X = batched.bicycle_linearise(t(X0), t(U), p, ts,
                                           nat.MODEL_RK4 if integ == "rk4" else nat.MODEL_FE)
    torch.cuda.synchronize()
    A, B, c, X = (v.cpu().numpy() for v in (A, B, c, X))
    step = nlp.STEPS[integ]
    for i in range(b):
        x = X0[i]
        for k in range(N):
            assert np.abs(X[i, k] - x).max() < 1e-13
            Ar, Br = nlp.fe_jac(x, U[i, k], ts, step=step)
            xn = step(x, U[i, k], ts)
            assert np.abs(A[i, k] - Ar).max() < 1e-12
            assert np.abs(B[i, k] - Br).max() < 1e-12
            assert np.abs(A[i, k] @ x + B[i, k] @ U[i, k] + c[i, k] - xn).max() < 1e-13
            x = xn


def test_rk4_controller_matches_rk4_oracle():
    """template.py:141 builds the OCP on runge_kutta4: MPCController with
    integrator='rk4' (exact RK4 Hessian) reaches the optimum of that NLP
    (oracle/nlp.py with the RK4 model), KKT below 1e-8, within the default
    iteration budget and in about as many iterations as the FE controller."""
    x0 = np.array([0.3, -0.1, 0.0, 0.0])
    ctl = MPCController(30, 0.08, VehicleParameters(), integrator="rk4")
    sol = ctl.solve(x0)
    assert sol["success"] and sol["kkt"] < TOL_KKT, (sol["status"], sol["kkt"])
    fe = MPCController(30, 0.08, VehicleParameters()).solve(x0)
    assert sol["iterations"] <= fe["iterations"] + 5, (sol["iterations"], fe["iterations"])
    Q = np.diag([1., 6., .2, .05])
    xlo, lbu = np.array([-3, -2, -2 * np.pi, -0.5]), np.array([-1, -0.384])
    ocp = nlp.OCP(30, 0.08, Q, 100 * Q, np.diag([1., .01]), xlo, -xlo, lbu, -lbu, model="rk4")
    U, y, k = ocp.solve(x0)
    assert k < 1e-10
    assert np.abs(np.asarray(sol["x"]).reshape(-1) - U).max() < 1e-6


def test_controller_log_batched(golden):
    """session_2/log.py:8-12 ControllerLog fields from a batched solve:
    solver_success (b,), state_prediction (b, N+1, nx) = [x0; g],
    input_prediction (b, N, nu)."""
    from model_predictive_control_amd.problems import ControllerLog

    g = golden("nlp_s4.npz")
    X0 = g["main_x0"]
    ctl = _controller(g, "main")
    log = ControllerLog()
    sol = ctl.solve(X0)
    ctl.log_step(log, sol, X0)
    b = X0.shape[0]
    assert log.solver_success[0].shape == (b,) and log.solver_success[0].all()
    assert log.state_prediction[0].shape == (b, 31, 4)
    assert np.array_equal(log.state_prediction[0][:, 0], X0)
    assert np.abs(log.state_prediction[0][:, 1:] - g["main_X"][:, 1:]).max() < 1e-6
    assert log.input_prediction[0].shape == (b, 30, 2)
    assert np.abs(log.input_prediction[0].reshape(b, -1) - g["main_U"]).max() < TOL_U


def test_held_inputs_sit_on_their_bounds(golden):
    """mpcqp_bicycle_sqp_step's held-input bits (SqpSolver.fix): an input is
    held only where it sits exactly on a bound; on the saturated-tail
    fixtures some are held once the exact Hessian is in use, and the converged
    solution keeps them on their bounds."""
    from model_predictive_control_amd.mpc import SqpSolver

    g = golden("nlp_tail.npz")
    ctl = MPCController(int(g["N"]), float(g["ts"]), VehicleParameters())
    X0 = torch.as_tensor(g["x0"], dtype=torch.float64, device=ctl.device)
    sqp = SqpSolver(ctl, X0.shape[0])
    sqp.reset()
    held_seen = 0
    for _ in range(ctl.max_iter):
        sqp.iterate(X0)
        fix = sqp.fix.cpu().numpy()
        U = sqp.U.cpu().numpy()
        lo, hi = ctl.lb_inputs, ctl.ub_inputs
        for q in range(2):
            held = (fix >> q) & 1 == 1
            u = U[..., q][held]
            assert np.all((u == lo[q]) | (u == hi[q])), u
            held_seen += int(held.sum())
        if bool(sqp.done().all()):
            break
    assert bool(sqp.done().all())
    assert held_seen > 0


def test_gauss_newton_on_saturated_tail(golden):
    """A Gauss-Newton controller never builds the held-input proximal term, so
    its step kernel gets no held inputs (fix stays clear) and moves every input
    along the QP's own direction: on the saturated-tail fixtures
    (tests/golden/nlp_tail.npz) it reaches the oracle's optimum."""
    from model_predictive_control_amd.mpc import SqpSolver

    g = golden("nlp_tail.npz")
    ctl = MPCController(int(g["N"]), float(g["ts"]), VehicleParameters(),
                        hessian="gauss-newton", max_iter=400, tol=1e-8)
    X0 = torch.as_tensor(g["x0"], dtype=torch.float64, device=ctl.device)
    sqp = SqpSolver(ctl, X0.shape[0])
    sqp.reset()
    for _ in range(ctl.max_iter):
        sqp.iterate(X0)
        if bool(sqp.done().all()):
            break
    assert int(sqp.fix.abs().sum()) == 0
    assert bool(sqp.done().all()), sqp.kkt.cpu().numpy()
    U = sqp.U.reshape(X0.shape[0], -1).cpu().numpy()
    assert np.abs(U - g["U"]).max() < 1e-5


@pytest.mark.parametrize("tag", ["main", "sol"])
def test_solve_returns_lam_p(golden, tag):
    """CasADi's nlpsol dict (main.py:115-116) also carries lam_p, the multiplier of
    the parameter p = x0: -d(f + lam_g'g)/dx0 along the rollout, i.e. -2 lambda_0 of
    the device adjoint at the returned optimum.  Against oracle/nlp.py lam_p at the
    fixture optimum (which test_oracle pins to the optimal value's sensitivity)."""
    g = golden("nlp_s4.npz")
    ocp = _ocp(g, tag)
    X0, Ustar, Ystar = g[f"{tag}_x0"], g[f"{tag}_U"], g[f"{tag}_y"]
    sol = _controller(g, tag).solve(X0)
    assert np.asarray(sol["success"]).all()
    for i, x0 in enumerate(X0):
        lp = ocp.lam_p(x0, Ustar[i], Ystar[i])
        assert np.abs(sol["lam_p"][i] - lp).max() < 1e-6 * (1 + np.abs(lp).max()), (i, sol["lam_p"][i], lp)
    one = _controller(g, tag).solve(X0[0])
    assert one["lam_p"].shape == (4, 1)


def test_rti_mode_result_mapping(golden):
    """mode='rti' (fixed RTI steps on mpcqp_mpc_qp) reports IPOPT's keys at the inputs
    it returns: "g" and "f" on the prediction model's own rollout of x (not the last
    linearisation's states); lam_x and lam_p from the adjoint along that rollout with
    the returned lam_g -- each against oracle/nlp.py evaluated at the same point."""
    g = golden("nlp_s4.npz")
    ocp = _ocp(g, "main")
    x0 = g["main_x0"][0]
    rti = MPCController(30, 0.08, VehicleParameters(), mode="rti", sqp_iters=3)
    sol = rti.solve(x0)
    U = np.asarray(sol["x"]).reshape(-1)
    y = np.asarray(sol["lam_g"]).reshape(-1) / 2.0
    X, _, _, _ = ocp.linearise(x0, U)
    assert np.abs(np.asarray(sol["g"]).reshape(-1) - X[1:].reshape(-1)).max() < 1e-12
    assert abs(sol["f"] - ocp.cost(x0, U)) < 1e-10 * (1 + abs(sol["f"]))
    grad, _ = ocp.grad(x0, U, y)
    lam_x = np.asarray(sol["lam_x"]).reshape(-1)
    assert np.abs(lam_x + 2 * grad).max() < 1e-9 * (1 + np.abs(grad).max())
    lp = ocp.lam_p(x0, U, y)
    assert np.abs(np.asarray(sol["lam_p"]).reshape(-1) - lp).max() < 1e-9 * (1 + np.abs(lp).max())


def _bench_like_x0(n, seed=20261015 + 6):
    rng = np.random.default_rng(seed)
    return np.stack([rng.uniform(-.8, .8, n), rng.uniform(-.4, .4, n), rng.uniform(-.5, .5, n),
                     rng.uniform(-.2, .2, n)], -1)


@pytest.mark.parametrize("hessian,integrator", [("exact", "fe"), ("gauss-newton", "fe"),
                                                ("exact-raw", "fe"), ("exact", "rk4")])
def test_one_launch_solve_equals_iteration(hessian, integrator):
    """mpcqp_bicycle_sqp_solve (SqpSolver.solve: the whole SQP per instance in
    one launch) runs the iterations of SqpSolver.iterate repeated: the same
    converged set and optimum per instance (the one-launch QPs stop their
    polish at the first step that passes its final test and warm-polish near
    convergence, so iteration counts may differ by a few).  Every Hessian
    mode and both prediction models."""
    from model_predictive_control_amd.mpc import SqpSolver

    iters = 40 if hessian != "gauss-newton" else 25
    ctl = MPCController(30, 0.08, VehicleParameters(), tol=1e-9, hessian=hessian,
                        integrator=integrator)
    X0 = torch.as_tensor(_bench_like_x0(192), dtype=torch.float64, device="cuda")
    out = {}
    for mode in ("iterate", "solve"):
        sqp = SqpSolver(ctl, X0.shape[0])
        sqp.reset()
        if mode == "solve":
            sqp.solve(X0, iters)
        else:
            for _ in range(iters):
                sqp.iterate(X0)
        out[mode] = (sqp.U.reshape(X0.shape[0], -1).cpu().numpy(), sqp.done().cpu().numpy(),
                     sqp.iters().cpu().numpy(), sqp.kkt.cpu().numpy())
    Ui, di, ii, ki = out["iterate"]
    Us, ds, is_, ks = out["solve"]
    assert (ks[ds] <= 1e-9).all()
    if hessian == "gauss-newton":
        # linear convergence: few reach 1e-9 in 25 iterations, and one that
        # reaches it in the last iteration may take one more on the other path
        assert (di != ds).sum() <= 3, ((di != ds).sum(), di.sum(), ds.sum())
        assert np.abs(Ui - Us).max() < 1e-5, np.abs(Ui - Us).max()
        return
    assert di.sum() >= 0.8 * di.size, di.sum()
    assert (di == ds).mean() >= 0.97, (di != ds).sum()
    both = di & ds
    # the one-launch QPs end their polish early (MPCQP_POLISH_EARLY) and are
    # warm-polished near convergence: a few iterations more or less
    assert (np.abs(ii[both] - is_[both]) <= 3).mean() >= 0.9
    assert np.abs(Ui[both] - Us[both]).max() < TOL_U  # two KKT <= 1e-9 points of one optimum


def test_one_launch_solve_continues_from_its_state():
    """Two launches of 6 + 34 iterations end where one of 40 does (the state
    U, y, pi, X, rho, kkt, mu, flags, fix carries over; converged instances
    stay frozen).  Only the QP's warm polish (the previous QP's active set,
    kept in LDS within a launch) starts cold in the second launch, so the
    iterates agree to the QP's rounding, not bit for bit."""
    from model_predictive_control_amd.mpc import SqpSolver

    ctl = MPCController(30, 0.08, VehicleParameters(), tol=1e-9)
    X0 = torch.as_tensor(_bench_like_x0(64, seed=5), dtype=torch.float64, device="cuda")
    a, b = SqpSolver(ctl, 64), SqpSolver(ctl, 64)
    a.reset()
    b.reset()
    a.solve(X0, 40)
    b.solve(X0, 6)
    b.solve(X0, 34)
    da, db = a.done(), b.done()
    assert int(da.sum()) >= 56 and torch.equal(da, db)
    assert float((a.U - b.U).abs().max()) < 1e-9
    assert int((a.iters() - b.iters()).abs().max()) <= 1


def test_one_launch_solve_checks_arguments():
    from model_predictive_control_amd import _native as nat
    from model_predictive_control_amd.mpc import SqpSolver

    ctl = MPCController(30, 0.08, VehicleParameters(), tol=1e-9)
    sqp = SqpSolver(ctl, 4)
    sqp.reset()
    with pytest.raises(ValueError):
        sqp.solve(torch.zeros((4, 3), dtype=torch.float64, device="cuda"), 5)
    with pytest.raises((ValueError, nat.MpcqpError)):
        batched.bicycle_sqp_solve(torch.zeros((4, 4), dtype=torch.float64, device="cuda"), sqp.U,
                                  sqp.y, sqp.pi, sqp.X, sqp.state(), ctl.params, ctl.ts, ctl.Q,
                                  ctl.R, ctl.QN, max_iter=5,
                                  ws=torch.empty(16, dtype=torch.uint8, device="cuda"))


def test_maxiter_stragglers_converge(golden):
    """tests/golden/nlp_maxiter.npz: the 64 bench x0 the round-5 SQP left at
    MAXITER after 60 iterations (tools/sqp_straggler.py; 56 of them cycling
    between the exact and the projected curvature after 15 Gauss-Newton
    iterations above KKT 0.3).  In one batched solve with the nlp bench's
    per-instance cap (150) every one converges (KKT < 1e-8), 55 to the
    oracle's optimum, the other 9 to the lower-cost local minimum the device
    SQP finds (the round-5 device point).  The solve stops at KKT <= 1e-9
    (tol); on these ill-conditioned stragglers that leaves u up to ~1.5e-7
    from the KKT-1e-12 points (the summation order of the QP's reductions
    moves the stopping iterate), so the bar here is TOL_U_STRAG = 5e-7."""
    from model_predictive_control_amd.mpc import SqpSolver

    g = golden("nlp_maxiter.npz")
    ctl = MPCController(int(g["N"]), float(g["ts"]), VehicleParameters(), tol=1e-9)
    X0 = torch.as_tensor(g["x0"], dtype=torch.float64, device="cuda")
    sqp = SqpSolver(ctl, X0.shape[0])
    sqp.reset()
    sqp.solve(X0, 150)
    done = sqp.done().cpu().numpy()
    assert done.all(), np.nonzero(~done)[0]
    assert float(sqp.kkt.max()) < TOL_KKT
    U = sqp.U.reshape(X0.shape[0], -1).cpu().numpy()
    same = g["minimum"] == 0
    err_o = np.abs(U - g["U"]).max(1)
    err_d = np.abs(U - g["U_device"]).max(1)
    assert (err_o[same] < TOL_U_STRAG).all(), (np.nonzero(same & (err_o >= TOL_U_STRAG))[0],
                                                err_o[same].max())
    assert (err_d[~same] < TOL_U_STRAG).all(), err_d[~same].max()
    assert int(sqp.iters().max()) <= 150
