"""Generate the golden fixtures in tests/golden/ (run in the build container).

session1.npz  -- outputs of the *reference's own code*, imported from
                 /root/reference/session_1 (FHC.py, LinearSystem.py,
                 session1_sol.py).  FHC.py imports ``casadi`` (FHC.py:1) and
                 ``rcracers`` (FHC.py:5) without using them; both are absent
                 here, so empty placeholder modules are registered before the
                 import.  Nothing else is stubbed.
problems.npz  -- the session 2/3 ``Problem`` dataclass values, imported from
                 /root/reference/session_2/problem.py and session_3/problem.py.
boxqp_cfg2.npz -- config 2 (double integrator of FHC.py:136-142, N=20,
                 |u|<=1, 64 seeded x0 ~ U(-10,10)^2): condensed (H, f) from
                 the explicit-matrix oracle and the minimiser from SciPy BVLS,
                 cross-checked against the oracle active-set solver and
                 certified by KKT residuals (the reference's own solver,
                 CasADi/IPOPT, is not installed: parity vs IPOPT unpinned).
vehicle.npz   -- every field of session_4's ``VehicleParameters`` dataclass,
                 read statically (ast) from /root/reference/session_4/parameters.py.
nlp_s4.npz    -- NLP-optimal inputs of the session-4 MPC step (main.py and
                 session4_sol.py controllers) from the oracle SQP + Newton
                 polish (KKT < 1e-11), agreeing with SciPy SLSQP to 1e-5.
polyqp_s2.npz -- session-2/3 problem data with input box and state box
                 (x_1..x_N), solved by the Goldfarb-Idnani oracle, KKT
                 certified.

The reference's source never travels: only these .npz data files are
committed.  Re-run with:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)


def _import_session1():
    import matplotlib

    matplotlib.use("Agg")
    for name in ("casadi", "rcracers"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.path.insert(0, os.path.join(REF, "session_1"))
    import FHC  # noqa: E402
    import LinearSystem  # noqa: E402
    import session1_sol  # noqa: E402
    return FHC, LinearSystem, session1_sol


def make_session1():
    FHC, LinearSystem, s1 = _import_session1()
    from scipy import linalg

    out = {}
    # --- FHC.main data (FHC.py:136-144)
    A, B = FHC.get_dynamics_discrete(0.5)
    C = np.array([[1], [-2 / 3]])
    Q = np.matmul(C, C.T) + 1e-3 * np.eye(2, 2)
    R = np.array([0.1])
    P_f = Q
    x0 = np.array([[10.], [10.]])
    out.update(fhc_A=A, fhc_B=B, fhc_Q=Q, fhc_R=R, fhc_Pf=P_f, fhc_x0=x0)
    Ac, Bc = FHC.get_dynamics_continuous()
    out.update(fhc_Ac=Ac, fhc_Bc=Bc)
    # --- ricatti_recursion (FHC.py:51-61)
    for N in list(range(1, 11)) + [20]:
        P, K = FHC.ricatti_recursion(A, B, Q, R, P_f, N)
        out[f"fhc_P_N{N}"] = np.array(P)
        out[f"fhc_K_N{N}"] = np.array(K)
    # --- compare_term_cost values (FHC.py:117-127)
    VN = []
    for N in range(1, 10):
        P_n, _ = FHC.ricatti_recursion(A, B, Q, R, P_f, N)
        VN.append(np.squeeze(x0.T @ P_n[0] @ x0))
    P_inf = linalg.solve_discrete_are(A, B, Q, R)
    out["fhc_VN"] = np.array(VN)
    out["fhc_Vinf"] = np.squeeze(x0.T @ P_inf @ x0)
    out["fhc_Pinf"] = P_inf
    # --- AutoCruising closed loop + predictions (FHC.py:64-101)
    rng = np.random.default_rng(20261015)
    xb = rng.uniform(-10, 10, size=(2, 8))
    out["fhc_xbatch"] = xb
    for N in (4, 6, 10):
        _, gains = FHC.ricatti_recursion(A, B, Q, R, P_f, N)
        sys_ = FHC.AutoCruising(A, B)
        sys_.set_opti_gain(gains)
        sys_.simulate(x0, sys_.control_law, 30)
        out[f"fhc_sim_N{N}"] = sys_.x.copy()
        preds = np.stack([sys_.prediction(sys_.x[:, :, t], sys_.pred, N) for t in range(30)])
        out[f"fhc_pred_N{N}"] = preds
        sys_.simulate(xb, sys_.control_law, 30)
        out[f"fhc_simbatch_N{N}"] = sys_.x.copy()
    K_inf = -np.linalg.inv(R + B.T @ P_inf @ B) @ B.T @ P_inf @ A
    sys_ = FHC.AutoCruising(A, B)
    sys_.set_opti_gain([K_inf] * 10)
    sys_.simulate(x0, sys_.control_law, 30)
    out["fhc_Kinf"] = K_inf
    out["fhc_sim_inf"] = sys_.x.copy()
    # --- session1_sol (session1_sol.py:44-91, 136-170)
    A2, B2, Q2, R2 = s1.setup()
    out.update(s1_A=A2, s1_B=B2, s1_Q=Q2, s1_R=R2)
    x0s = 10 * np.ones(2)
    for N in (4, 6, 10, 20):
        P, K = s1.riccati_recursion(A2, B2, R2, Q2, Q2, N)
        out[f"s1_P_N{N}"] = np.array(P)
        out[f"s1_K_N{N}"] = np.array(K)

        def f(x, u, A2=A2, B2=B2):
            return A2 @ x + B2 @ u

        def kappa(x, t, K=K):
            return K[0] @ x

        def kappa_pred(x, t, K=K):
            return K[t] @ x

        xcl, flag = s1.simulate(x0s, f, kappa, 30)
        out[f"s1_sim_N{N}"] = xcl
        out[f"s1_flag_N{N}"] = np.array(flag)
        out[f"s1_pred_N{N}"] = np.stack([s1.simulate(xt, f, kappa_pred, N)[0] for xt in xcl])
    # an unstable closed loop to exercise the instability flag (session1_sol.py:86-89)
    _, Kbad = s1.riccati_recursion(A2, B2, R2, Q2, Q2, 1)
    xbad, flag_bad = s1.simulate(x0s, lambda x, u: A2 @ x + B2 @ u, lambda x, t: -Kbad[0] @ x, 30)
    out["s1_sim_bad"] = xbad
    out["s1_flag_bad"] = np.array(flag_bad)
    # --- LinearSystem.f on a batch (LinearSystem.py:16-18)
    ls = LinearSystem.LinearSystem(A, B)
    ub = rng.uniform(-1, 1, size=(1, 8))
    out["ls_f_x"] = xb
    out["ls_f_u"] = ub
    out["ls_f_out"] = ls.f(xb, ub)
    np.savez_compressed(os.path.join(HERE, "session1.npz"), **out)
    return out


def make_problems():
    out = {}
    for tag in ("session_2", "session_3"):
        sys.path.insert(0, os.path.join(REF, tag))
        import importlib

        mod = importlib.import_module("problem")
        p = mod.Problem()
        for k in ("Ts", "p_min", "p_max", "v_min", "v_max", "u_min", "u_max", "N"):
            out[f"{tag}_{k}"] = np.array(getattr(p, k))
        for k in ("Q", "R", "A", "B"):
            out[f"{tag}_{k}"] = np.asarray(getattr(p, k), dtype=float)
        out[f"{tag}_n_state"] = np.array(p.n_state)
        out[f"{tag}_n_input"] = np.array(p.n_input)
        del sys.modules["problem"]
        sys.path.pop(0)
    np.savez_compressed(os.path.join(HERE, "problems.npz"), **out)
    return out


def make_vehicle():
    """Field names and defaults of ``VehicleParameters`` read STATICALLY from
    session_4/parameters.py (ast; nothing of the file is executed): each
    annotated assignment of the dataclass body, its default evaluated with
    literal_eval, or as ``2*np.pi`` / ``-2*np.pi`` (the only non-literal
    defaults)."""
    import ast
    import math

    src = open(os.path.join(REF, "session_4", "parameters.py")).read()
    cls = next(n for n in ast.parse(src).body
               if isinstance(n, ast.ClassDef) and n.name == "VehicleParameters")
    out, order = {}, []

    def value(node):
        seg = ast.get_source_segment(src, node).replace(" ", "")
        if seg in ("2*np.pi", "-2*np.pi"):
            return (-1.0 if seg.startswith("-") else 1.0) * 2.0 * math.pi
        return float(ast.literal_eval(node))

    for st in cls.body:
        if isinstance(st, ast.AnnAssign) and isinstance(st.target, ast.Name):
            out[st.target.id] = np.array(value(st.value))
            order.append(st.target.id)
    out["_field_order"] = np.array(order)
    np.savez_compressed(os.path.join(HERE, "vehicle.npz"), **out)
    return out


def make_nlp():
    """NLP-optimal inputs of the session-4 MPC step (the NLP IPOPT solves in
    MPCController.solve, main.py:115-116, without the non-convex collision
    rows; session4_sol.py:132-217 exactly) for the two reference
    controllers, from oracle/nlp.py (SQP + Newton polish, KKT-certified) and
    cross-checked against SciPy SLSQP on the same NLP: only initial states
    where the two agree to 1e-5 (the same local optimum) are kept.
      main: N = 30, ts = 0.08, weights main.py:72-74, x0 of main.py:248 + 4 seeded
      sol:  N = 50, ts = 0.05, weights session4_sol.py:166-169, x0 of
            session4_sol.py:344 + 2 seeded"""
    from oracle import nlp

    xlo = np.array([-3.0, -2.0, -2 * np.pi, -0.5])
    lbu = np.array([-1.0, -0.384])
    Qm, Qs = np.diag([1., 6., .2, .05]), np.diag([1., 3., .1, .01])
    cases = {"main": (30, 0.08, Qm, 100 * Qm, np.diag([1., .01]), [0.3, -0.1, 0.0, 0.0], 4),
             "sol": (50, 0.05, Qs, 10 * Qs, np.diag([1., 1e-2]), [0.6, -0.25, 0.0, 0.0], 2)}
    out = {}
    rng = np.random.default_rng(20261015 + 40)
    for tag, (N, ts, Q, QN, R, xref, nrand) in cases.items():
        ocp = nlp.OCP(N, ts, Q, QN, R, xlo, -xlo, lbu, -lbu)
        cand = [np.array(xref)] + [np.array([rng.uniform(-.8, .8), rng.uniform(-.4, .4),
                                             rng.uniform(-.5, .5), rng.uniform(-.2, .2)])
                                   for _ in range(2 * nrand)]
        X0, Us, Ys, Xs, K, J, Usl = [], [], [], [], [], [], []
        for x0 in cand:
            U, y, k = ocp.solve(x0)
            Usq, _ = ocp.solve_slsqp(x0)
            if k > 1e-11 or np.abs(U - Usq).max() > 1e-5:
                continue
            X0.append(x0); Us.append(U); Ys.append(y); Xs.append(ocp.rollout(x0, U)); K.append(k)
            J.append(ocp.cost(x0, U)); Usl.append(Usq)
            if len(X0) == nrand + 1:
                break
        assert len(X0) == nrand + 1, (tag, len(X0))
        out.update({f"{tag}_N": np.array(N), f"{tag}_ts": np.array(ts), f"{tag}_Q": Q,
                    f"{tag}_QN": QN, f"{tag}_R": R, f"{tag}_x0": np.array(X0),
                    f"{tag}_U": np.array(Us), f"{tag}_y": np.array(Ys), f"{tag}_X": np.array(Xs),
                    f"{tag}_kkt": np.array(K), f"{tag}_J": np.array(J),
                    f"{tag}_U_slsqp": np.array(Usl)})
    out["xlo"], out["lbu"] = xlo, lbu
    np.savez_compressed(os.path.join(HERE, "nlp_s4.npz"), **out)
    return out


def make_boxqp_cfg2(s1):
    from oracle import condense as oc
    from oracle import qp as oq

    A, B, Q, R, Pf = s1["fhc_A"], s1["fhc_B"], s1["fhc_Q"], s1["fhc_R"].reshape(1, 1), s1["fhc_Pf"]
    N, nb = 20, 64
    rng = np.random.default_rng(20261015 + 2)
    X0 = rng.uniform(-10, 10, size=(nb, 2))
    Hs, fs, Zs = [], [], []
    for x0 in X0:
        d = oc.condense(A, B, Q, R, Pf, N, x0=x0)
        z_b = oq.box_qp_bvls(d["H"], d["f"], -1.0, 1.0)
        z_a, _, _ = oq.box_qp(d["H"], d["f"], -np.ones(N), np.ones(N))
        assert np.abs(z_a - z_b).max() < 1e-8, np.abs(z_a - z_b).max()
        assert oq.kkt_box(d["H"], d["f"], -1.0, 1.0, z_a) < 1e-9
        Hs.append(d["H"]); fs.append(d["f"]); Zs.append(z_a)
    np.savez_compressed(os.path.join(HERE, "boxqp_cfg2.npz"), A=A, B=B, Q=Q, R=R, Pf=Pf, N=N,
                        x0=X0, H=np.array(Hs), f=np.array(fs), z=np.array(Zs))


def make_polyqp_s2(pr):
    from oracle import condense as oc
    from oracle import qp as oq

    out = {}
    for tag in ("session_2", "session_3"):
        A, B = pr[f"{tag}_A"], pr[f"{tag}_B"]
        Q, R, N = pr[f"{tag}_Q"], pr[f"{tag}_R"], int(pr[f"{tag}_N"])
        xmin = np.array([pr[f"{tag}_p_min"], pr[f"{tag}_v_min"]], float)
        xmax = np.array([pr[f"{tag}_p_max"], pr[f"{tag}_v_max"]], float)
        umin, umax = float(pr[f"{tag}_u_min"]), float(pr[f"{tag}_u_max"])
        rng = np.random.default_rng(20261015 + (22 if tag == "session_2" else 33))
        X0 = np.column_stack([rng.uniform(-100, 0, 32), rng.uniform(-15, 20, 32)])
        Zs, ok = [], []
        for x0 in X0:
            d = oc.condense(A, B, Q, R, Q, N, x0=x0)
            G = np.vstack([d["Gam"], -d["Gam"]])
            h = np.concatenate([np.tile(xmax, N) - d["xbar"], -np.tile(xmin, N) + d["xbar"]])
            try:
                z, lam, _ = oq.poly_qp(d["H"], d["f"], G, h, lb=np.full(N, umin), ub=np.full(N, umax))
                C = np.vstack([G, np.eye(N), -np.eye(N)])
                dd = np.concatenate([h, np.full(N, umax), -np.full(N, umin)])
                assert oq.kkt_poly(d["H"], d["f"], C, dd, z, lam) < 1e-7
                Zs.append(z); ok.append(True)
            except ValueError:
                Zs.append(np.full(N, np.nan)); ok.append(False)
        out[f"{tag}_x0"] = X0
        out[f"{tag}_z"] = np.array(Zs)
        out[f"{tag}_feasible"] = np.array(ok)
    np.savez_compressed(os.path.join(HERE, "polyqp_s2.npz"), **out)


def make_nlp_tail(count=10, min_active=24):
    """The saturated tail of the nlp bench's x0 distribution: initial states
    of the main.py controller (N = 30, ts = 0.08, weights main.py:72-74,
    input + state box) whose NLP optimum has at least ``min_active`` of its 60
    inputs at a bound -- the instances the device SQP needed most iterations
    on.  Kept whenever the oracle (oracle/nlp.py SQP + Newton polish) reaches
    KKT < 1e-11, whether or not SciPy SLSQP finds the same point (on these it
    often stops early); the oracle's point is a certified first-order
    optimum, the one IPOPT would return from the same start."""
    from oracle import nlp

    xlo = np.array([-3.0, -2.0, -2 * np.pi, -0.5])
    lbu = np.array([-1.0, -0.384])
    Q = np.diag([1., 6., .2, .05])
    ocp = nlp.OCP(30, 0.08, Q, 100 * Q, np.diag([1., .01]), xlo, -xlo, lbu, -lbu)
    lb, ub = np.tile(lbu, 30), -np.tile(lbu, 30)
    rng = np.random.default_rng(20261015 + 41)
    X0, Us, Ys, K, J, NA = [], [], [], [], [], []
    for _ in range(400):
        x0 = np.array([rng.uniform(-.8, .8), rng.uniform(-.4, .4), rng.uniform(-.5, .5),
                       rng.uniform(-.2, .2)])
        U, y, k = ocp.solve(x0)
        na = int(((np.abs(U - lb) < 1e-9) | (np.abs(U - ub) < 1e-9)).sum())
        if k > 1e-11 or na < min_active:
            continue
        X0.append(x0); Us.append(U); Ys.append(y); K.append(k); J.append(ocp.cost(x0, U))
        NA.append(na)
        if len(X0) == count:
            break
    assert len(X0) == count, len(X0)
    np.savez_compressed(os.path.join(HERE, "nlp_tail.npz"), x0=np.array(X0), U=np.array(Us),
                        y=np.array(Ys), kkt=np.array(K), J=np.array(J), n_active=np.array(NA),
                        N=np.array(30), ts=np.array(0.08), Q=Q, QN=100 * Q, R=np.diag([1., .01]),
                        xlo=xlo, lbu=lbu)


def _oracle_solve_one(args):
    from oracle import nlp
    x0, Q, QN, R, xlo, lbu = args
    ocp = nlp.OCP(30, 0.08, Q, QN, R, xlo, -xlo, lbu, -lbu)
    U, y, k = ocp.solve(x0)
    if k >= 1e-9:  # the polish did not contract from the 1e-7 point: Gauss-Newton on to 1e-10
        U, y, k, _ = ocp.solve_sqp(x0, U0=U, tol=1e-10, hessian="gauss-newton", max_iter=8000)
        U2, y2, k2 = ocp.newton_polish(x0, U, y, tol=1e-13)
        if k2 < k:
            U, y, k = U2, y2, k2
    return U, y, k, ocp.cost(x0, U)


def make_nlp_maxiter(dump=os.path.join(REPO, "gpurun_out", "sqp_straggler.npz")):
    """The 64 x0 of the nlp bench (seed 20261015 + 6, both slots) that the
    round-5 device SQP left at MAXITER after 60 iterations, from
    tools/sqp_straggler.py's dump (per-iteration KKT, flags, mu and QP status of
    each, run on to convergence): the oracle's optimum of each (oracle/nlp.py:
    Gauss-Newton SQP to 1e-7, Newton polish to KKT < 1e-12), the device's
    converged inputs, and a classification --
      minimum: 0 = the oracle's (|U_dev - U*| < 1e-7), 1 = another local
               minimum with a lower cost, 2 = another with a higher cost;
      cause:   0 = slow convergence (at most two switches to the projected
               curvature), 1 = cycling between the exact and the projected
               curvature (three or more), with the Gauss-Newton stall before
               the switch (15 iterations still above KKT 0.3) in gn_stall."""
    from multiprocessing import Pool

    d = np.load(dump)
    xlo = np.array([-3.0, -2.0, -2 * np.pi, -0.5])
    lbu = np.array([-1.0, -0.384])
    Q = np.diag([1., 6., .2, .05])
    QN, R = 100 * Q, np.diag([1., .01])
    X0 = d["x0"]
    with Pool(8) as pool:
        res = pool.map(_oracle_solve_one, [(x0, Q, QN, R, xlo, lbu) for x0 in X0])
    from oracle import nlp
    ocp = nlp.OCP(30, 0.08, Q, QN, R, xlo, -xlo, lbu, -lbu)
    U = np.array([r[0] for r in res]); Y = np.array([r[1] for r in res])
    K = np.array([r[2] for r in res]); J = np.array([r[3] for r in res])
    Ud = d["U_end"].reshape(len(X0), -1)
    Jd = np.array([ocp.cost(x0, u) for x0, u in zip(X0, Ud)])
    dev = np.abs(Ud - U).max(1)
    minimum = np.where(dev < 1e-7, 0, np.where(Jd < J, 1, 2))
    fl = d["flags"]
    # projected-curvature episodes: entries into PROJ mode (flag 8 rising)
    proj = ((fl[1:] & 8) != 0) & ((fl[:-1] & 8) == 0)
    n_proj = proj.sum(0) + ((fl[0] & 8) != 0)
    exact_from = np.argmax((fl & 2) != 0, 0) + 1
    kk = d["kkt"]
    gn_stall = np.array([exact_from[j] >= 15 and kk[13, j] > 0.3 for j in range(len(X0))])
    cause = (n_proj >= 3).astype(int)
    conv = d["conv_it"][d["idx"]]
    assert (K < 1e-9).all(), K
    np.savez_compressed(os.path.join(HERE, "nlp_maxiter.npz"), x0=X0, bench_index=d["idx"],
                        U=U, y=Y, kkt=K, J=J, U_device=Ud, J_device=Jd, conv_it_r05=conv,
                        minimum=minimum, cause=cause, gn_stall=gn_stall, n_proj=n_proj,
                        qp_fail=((d["qp_status"] & 0xFF) != 0).sum(0), N=np.array(30),
                        ts=np.array(0.08), Q=Q, QN=QN, R=R, xlo=xlo, lbu=lbu)
    print("minimum", np.bincount(minimum, minlength=3), "cause", np.bincount(cause, minlength=2),
          "gn_stall", int(gn_stall.sum()), "oracle kkt max", float(K.max()))


def make_cfg3_tail(dump=os.path.join(REPO, "tools", "cfg3_tail_inputs.npz")):
    """The config-3 parity tail: the instances of the full B = 65,536 config-3
    batch (seed 20261015 + 3, bicycle linearised about the zero-input rollout;
    bench.py Config3) on which round 3's fp32 path ended >= 1e-6 from the fp64
    solution, with their fp32-valued inputs as the GPU produced them
    (tools/tail_dump.py dump -> tools/cfg3_tail_inputs.npz).  Each gets the
    fp64 oracle solution of the QP those inputs define (oracle/condense.py +
    oracle/qp.py poly_qp, Goldfarb-Idnani), KKT-certified here (< 1e-9): the
    reference's IPOPT would return the same unique minimiser."""
    from oracle import condense as oc
    from oracle import qp as oq
    from model_predictive_control_amd.parameters import VehicleParameters

    d = np.load(dump)
    N, p = 30, VehicleParameters()
    r = lambda a: np.asarray(a, np.float32).astype(np.float64)  # noqa: E731
    Q, R = r(np.diag([1., 6., .2, .05])), r(np.diag([1., .01]))
    xlo = r(np.tile([p.min_pos_x, p.min_pos_y, p.min_heading, p.min_vel], N))
    xhi = r(np.tile([p.max_pos_x, p.max_pos_y, p.max_heading, p.max_vel], N))
    lb = r(np.tile([p.min_drive, -p.max_steer], N))
    ub = r(np.tile([p.max_drive, p.max_steer], N))
    Z, K = [], []
    for j in range(len(d["index"])):
        A, B, c, x0 = (d[k][j].astype(np.float64) for k in ("A", "B", "c", "x0"))
        dd = oc.condense(A, B, Q, R, 100 * Q, N, x0=x0, c=c)
        G = np.vstack([dd["Gam"], -dd["Gam"]])
        h = np.concatenate([xhi - dd["xbar"], -(xlo - dd["xbar"])])
        z, lam, _ = oq.poly_qp(dd["H"], dd["f"], G, h, lb, ub)
        C = np.vstack([G, np.eye(60), -np.eye(60)])
        rhs = np.concatenate([h, ub, -lb])
        k = oq.kkt_poly(dd["H"], dd["f"], C, rhs, z, lam)
        assert k < 1e-9, (j, k)
        Z.append(z); K.append(k)
    np.savez_compressed(os.path.join(HERE, "cfg3_tail.npz"), index=d["index"], A=d["A"], B=d["B"],
                        c=d["c"], x0=d["x0"], z=np.array(Z), kkt=np.array(K),
                        err_round3=d["err"])


if __name__ == "__main__":
    only = sys.argv[1:]
    if not only or "session1" in only:
        s1 = make_session1()
    if not only or "problems" in only:
        pr = make_problems()
    if not only or "vehicle" in only:
        make_vehicle()
    if not only:
        make_boxqp_cfg2(s1)
        make_polyqp_s2(pr)
    if not only or "nlp" in only:
        make_nlp()
    if not only or "cfg3_tail" in only:
        make_cfg3_tail()
    if not only or "nlp_tail" in only:
        make_nlp_tail()
    if "nlp_maxiter" in only:  # needs tools/sqp_straggler.py's GPU dump
        make_nlp_maxiter()
    print("wrote", sorted(f for f in os.listdir(HERE) if f.endswith(".npz")))
