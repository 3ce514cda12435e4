"""CPU: pin the oracle against the reference's own outputs (golden vectors)."""
import numpy as np
import pytest

from oracle import bicycle as ob
from oracle import cbaseline as cb
from oracle import condense as oc
from oracle import qp as oq
from oracle import session1 as s1


def test_fhc_riccati_matches_reference(golden):
    g = golden("session1.npz")
    A, B, Q, R, Pf, x0 = s1.fhc_setup()
    assert np.array_equal(A, g["fhc_A"]) and np.array_equal(B, g["fhc_B"])
    assert np.allclose(Q, g["fhc_Q"], rtol=0, atol=0) and np.array_equal(R, g["fhc_R"])
    for N in list(range(1, 11)) + [20]:
        P, K = s1.ricatti_recursion(A, B, Q, R, Pf, N)
        assert np.abs(np.array(P) - g[f"fhc_P_N{N}"]).max() < 1e-12
        assert np.abs(np.array(K) - g[f"fhc_K_N{N}"]).max() < 1e-12


def test_session1_sol_riccati_and_sim(golden):
    g = golden("session1.npz")
    A, B, Q, R = g["s1_A"], g["s1_B"], g["s1_Q"], g["s1_R"]
    for N in (4, 6, 10, 20):
        P, K = s1.riccati_recursion(A, B, R, Q, Q, N)
        assert np.abs(np.array(P) - g[f"s1_P_N{N}"]).max() < 1e-12
        assert np.abs(np.array(K) - g[f"s1_K_N{N}"]).max() < 1e-12
        x, flag = s1.generic_simulate(10 * np.ones(2), lambda x, u: A @ x + B @ u,
                                      lambda x, t: K[0] @ x, 30)
        assert np.abs(x - g[f"s1_sim_N{N}"]).max() < 1e-11
        assert bool(flag) == bool(g[f"s1_flag_N{N}"])
    assert bool(g["s1_flag_bad"])


def test_linear_system_sim_and_prediction(golden):
    g = golden("session1.npz")
    A, B, Q, R, Pf, x0 = s1.fhc_setup()
    for N in (4, 6, 10):
        _, K = s1.ricatti_recursion(A, B, Q, R, Pf, N)
        x = s1.linear_simulate(A, B, x0, lambda x, t: K[0] @ x, 30)
        assert np.abs(x - g[f"fhc_sim_N{N}"]).max() < 1e-11
        xb = s1.linear_simulate(A, B, g["fhc_xbatch"], lambda x, t: K[0] @ x, 30)
        assert np.abs(xb - g[f"fhc_simbatch_N{N}"]).max() < 1e-11
        for t in (0, 7, 29):
            xp = s1.linear_prediction(A, B, x[:, :, t], lambda x, tt: K[tt] @ x, N)
            assert np.abs(xp - g[f"fhc_pred_N{N}"][t]).max() < 1e-11


def test_condensed_equals_riccati_known_answer():
    """-H^-1 F x0 equals the Riccati rollout (9.1e-14)."""
    A, B, Q, R, Pf, x0 = s1.fhc_setup()
    for N in (1, 5, 10, 20):
        d = oc.condense(A, B, Q, R.reshape(1, 1), Pf, N, x0=x0)
        z = -np.linalg.solve(d["H"], d["f"])
        _, K = s1.ricatti_recursion(A, B, Q, R, Pf, N)
        x = x0.ravel()
        for k in range(N):
            u = K[k] @ x
            assert abs(u[0] - z[k]) < 1e-10
            x = A @ x + B @ u
        assert np.abs(d["F"] @ x0.ravel() - d["f"]).max() < 1e-10


def test_condense_cost_identity_tv_drift():
    rng = np.random.default_rng(3)
    nx, nu, N = 3, 2, 6
    A = rng.normal(size=(N, nx, nx)) * 0.6
    B = rng.normal(size=(N, nx, nu))
    c = rng.normal(size=(N, nx))
    M = rng.normal(size=(nx, nx)); Q = M @ M.T + np.eye(nx)
    R = np.diag([0.5, 2.0]); Qf = 3 * Q
    x0 = rng.normal(size=nx)
    d = oc.condense(A, B, Q, R, Qf, N, x0=x0, c=c)
    J0 = oc.rollout_cost(A, B, Q, R, Qf, N, x0, np.zeros(N * nu), c=c)
    for _ in range(5):
        z = rng.normal(size=N * nu)
        J = oc.rollout_cost(A, B, Q, R, Qf, N, x0, z, c=c)
        assert abs(J - (z @ d["H"] @ z + 2 * d["f"] @ z + J0)) < 1e-8 * max(1, abs(J))
        X = oc.rollout_states(A, B, N, x0, z, c=c).ravel()
        assert np.abs(X - (d["xbar"] + d["Gam"] @ z)).max() < 1e-10


def test_box_fixture_pinned(golden):
    g = golden("boxqp_cfg2.npz")
    N = int(g["N"])
    for i in range(0, g["x0"].shape[0], 7):
        z, _, _ = oq.box_qp(g["H"][i], g["f"][i], -np.ones(N), np.ones(N))
        assert np.abs(z - g["z"][i]).max() < 1e-9
        zb = oq.box_qp_bvls(g["H"][i], g["f"][i], -1.0, 1.0)
        assert np.abs(zb - g["z"][i]).max() < 1e-7


def test_poly_fixture_pinned(golden):
    pr = golden("problems.npz")
    gp = golden("polyqp_s2.npz")
    for tag in ("session_2", "session_3"):
        A, B, Q, R, N = pr[f"{tag}_A"], pr[f"{tag}_B"], pr[f"{tag}_Q"], pr[f"{tag}_R"], int(pr[f"{tag}_N"])
        xmin = np.array([pr[f"{tag}_p_min"], pr[f"{tag}_v_min"]], float)
        xmax = np.array([pr[f"{tag}_p_max"], pr[f"{tag}_v_max"]], float)
        for x0, z_ref, ok in list(zip(gp[f"{tag}_x0"], gp[f"{tag}_z"], gp[f"{tag}_feasible"]))[:8]:
            d = oc.condense(A, B, Q, R, Q, N, x0=x0)
            G = np.vstack([d["Gam"], -d["Gam"]])
            h = np.concatenate([np.tile(xmax, N) - d["xbar"], -np.tile(xmin, N) + d["xbar"]])
            if ok:
                z, lam, _ = oq.poly_qp(d["H"], d["f"], G, h, lb=np.full(N, float(pr[f"{tag}_u_min"])),
                                       ub=np.full(N, float(pr[f"{tag}_u_max"])))
                assert np.abs(z - z_ref).max() < 1e-8
            else:
                with pytest.raises(ValueError):
                    oq.poly_qp(d["H"], d["f"], G, h, lb=np.full(N, float(pr[f"{tag}_u_min"])),
                               ub=np.full(N, float(pr[f"{tag}_u_max"])))


def test_c_oracle_matches_golden(golden):
    g = golden("boxqp_cfg2.npz")
    A, B, Q, R, Pf = g["A"], g["B"], g["Q"], g["R"], g["Pf"]
    z, it = cb.mpc_box(A, B, Q, R, Pf, int(g["N"]), g["x0"], -1.0, 1.0, nthreads=2)
    assert (it >= 0).all()
    assert np.abs(z - g["z"]).max() < 1e-9


def test_poly_oracle_random_vs_box():
    rng = np.random.default_rng(11)
    for _ in range(20):
        n = int(rng.integers(2, 15))
        M = rng.normal(size=(n, n)); H = M @ M.T + 0.1 * np.eye(n)
        f = rng.normal(size=n) * 4
        z1, _, _ = oq.box_qp(H, f, -np.ones(n), np.ones(n))
        z2, lam, _ = oq.poly_qp(H, f, np.zeros((0, n)), np.zeros(0), lb=-np.ones(n), ub=np.ones(n))
        assert np.abs(z1 - z2).max() < 1e-8


def test_bicycle_oracle_jacobian():
    x = np.array([0.3, -0.1, 0.4, 0.2]); u = np.array([0.5, 0.2])
    A, B = ob.fe_jac_fd(x, u, 0.08)
    assert A.shape == (4, 4) and B.shape == (4, 2)
    assert abs(A[3, 3] - (1 - 0.08)) < 1e-7 and abs(B[3, 0] - 0.16) < 1e-7


def test_oracle_lam_p_is_value_sensitivity(golden):
    """oracle/nlp.py lam_p (CasADi's multiplier of the parameter x0): by the envelope
    theorem the optimal value's derivative dJ*/dx0 equals -lam_p.  Checked by central
    differences of the oracle's own optimum (warm-started re-solves) on a fixture of
    tests/golden/nlp_s4.npz (session_4/main.py weights)."""
    from oracle import nlp

    g = golden("nlp_s4.npz")
    xlo, lbu = g["xlo"], g["lbu"]
    ocp = nlp.OCP(int(g["main_N"]), float(g["main_ts"]), g["main_Q"], g["main_QN"],
                  g["main_R"], xlo, -xlo, lbu, -lbu)
    x0, U, y = g["main_x0"][0], g["main_U"][0], g["main_y"][0]
    lp = ocp.lam_p(x0, U, y)
    h = 1e-5
    fd = np.zeros(4)
    for i in range(4):
        J = []
        for sgn in (1.0, -1.0):
            xp = x0.copy()
            xp[i] += sgn * h
            Up, _, k = ocp.solve(xp, U0=U)
            assert k < 1e-10
            J.append(ocp.cost(xp, Up))
        fd[i] = (J[0] - J[1]) / (2 * h)
    assert np.abs(fd + lp).max() < 1e-5 * (1 + np.abs(lp).max()), (fd, -lp)


def test_nlp_maxiter_fixture_certified(golden):
    """tests/golden/nlp_maxiter.npz (the 64 bench x0 the round-5 device SQP
    left at MAXITER after 60 iterations): every oracle optimum is a KKT point
    to 1e-11 on the oracle's own evaluation, and where the device converged
    to another local minimum (minimum == 1) that point is a KKT point too,
    with a lower cost (none is higher: minimum == 2 never occurs)."""
    from oracle import nlp

    g = golden("nlp_maxiter.npz")
    ocp = nlp.OCP(int(g["N"]), float(g["ts"]), g["Q"], g["QN"], g["R"], g["xlo"], -g["xlo"],
                  g["lbu"], -g["lbu"])
    assert g["x0"].shape == (64, 4) and (g["minimum"] != 2).all()
    for i in range(0, 64, 4):  # every fourth: the KKT evaluation is complex-step heavy
        x0 = g["x0"][i]
        assert ocp.kkt(x0, g["U"][i], g["y"][i]) < 1e-11, i
        assert abs(ocp.cost(x0, g["U"][i]) - g["J"][i]) < 1e-9 * (1 + abs(g["J"][i]))
    other = np.nonzero(g["minimum"] == 1)[0]
    assert (g["J_device"][other] < g["J"][other]).all()
