"""GPU parity: mpcqp_mpc_ipm -- the MPC step (input box + state box) on the
stage-wise interior point, which has no horizon limit.  It carries the
reference's own N = 50 controllers (session4_sol.py:342,391,445: state box
session4_sol.py:176-181, input box :180-181; n + m = 100 + 200, beyond the
dense condensed kernels) and is checked against the fp64 oracle (explicit
condensing oracle/condense.py + Goldfarb-Idnani oracle/qp.py) on the same
inputs: the polish step makes it the exact active-set vertex, so the fp64
tolerance is the one of the active-set kernels (1e-9)."""
import numpy as np
import pytest
import torch

from model_predictive_control_amd import batched
from model_predictive_control_amd._native import STATUS_POLISHED
from model_predictive_control_amd.parameters import VehicleParameters
from oracle import condense as oc
from oracle import qp as oq

pytestmark = pytest.mark.gpu

TOL_F64 = 1e-9


def _bicycle(dev, b, N, ts, seed, warm=0.3):
    """FE bicycle linearised about a random input sequence (mpcqp_bicycle_rti)."""
    p = VehicleParameters()
    rng = np.random.default_rng(20261015 + seed)
    X0 = np.stack([rng.uniform(-1, 1, b), rng.uniform(-.5, .5, b),
                   rng.uniform(-np.pi / 4, np.pi / 4, b), rng.uniform(-.3, .3, b)], -1)
    U = rng.uniform(-warm, warm, (b, N, 2))
    x = torch.as_tensor(X0, dtype=torch.float64, device=dev)
    A, B, c = batched.bicycle_rti(x, torch.as_tensor(U, dtype=torch.float64, device=dev), p, ts)
    return dict(A=A, B=B, c=c, x0=x, N=N, p=p,
                xlo=np.array([p.min_pos_x, p.min_pos_y, p.min_heading, p.min_vel]),
                xhi=np.array([p.max_pos_x, p.max_pos_y, p.max_heading, p.max_vel]),
                lb=np.tile([p.min_drive, -p.max_steer], N),
                ub=np.tile([p.max_drive, p.max_steer], N))


def _oracle(A, B, c, x0, Q, R, QN, N, xlo, xhi, lb, ub):
    d = oc.condense(A, B, Q, R, QN, N, x0=x0, c=c)
    G = np.vstack([d["Gam"], -d["Gam"]])
    h = np.concatenate([np.tile(xhi, N) - d["xbar"], -(np.tile(xlo, N) - d["xbar"])])
    z, lam, _ = oq.poly_qp(d["H"], d["f"], G, h, lb, ub)
    m = N * A.shape[-1]
    return z, lam[:m] - lam[m:2 * m], d


def _t(a, dev, dt=torch.float64):
    return torch.as_tensor(np.asarray(a, float), dtype=dt, device=dev)


# weights: main.py:72-74 (N = 30, ts = 0.08) and session4_sol.py:166-169
# (N = 50, ts = 0.05)
_MAIN = (np.diag([1., 6., .2, .05]), 100.0, np.diag([1., .01]))
_SOL = (np.diag([1., 3., .1, .01]), 10.0, np.diag([1., 1e-2]))


@pytest.mark.parametrize("N,ts,w,seed", [(30, 0.08, _MAIN, 1), (50, 0.05, _SOL, 2),
                                          (50, 0.05, _MAIN, 3)])
def test_ipm_vs_oracle(dev, N, ts, w, seed):
    """z and the state multipliers against the oracle; every instance
    optimal and polished to the vertex."""
    Q, qn, R = w
    pb = _bicycle(dev, 12, N, ts, seed)
    r = batched.mpc_ipm(pb["A"], pb["B"], _t(Q, dev), _t(R, dev), _t(qn * Q, dev), N, pb["x0"],
                        xlo=_t(pb["xlo"], dev), xhi=_t(pb["xhi"], dev), lb=_t(pb["lb"], dev),
                        ub=_t(pb["ub"], dev), c=pb["c"], tv=True)
    torch.cuda.synchronize()
    st = r["status"].cpu().numpy()
    assert ((st & 0xFF) == 0).all(), st & 0xFF
    assert ((st & STATUS_POLISHED) != 0).all()
    A, B, c, X0 = (pb[k].cpu().numpy() for k in ("A", "B", "c", "x0"))
    Z, Y, X = r["z"].cpu().numpy(), r["y"].cpu().numpy(), r["X"].cpu().numpy()
    ez = ey = ex = 0.0
    for i in range(Z.shape[0]):
        zr, yr, d = _oracle(A[i], B[i], c[i], X0[i], Q, R, qn * Q, N, pb["xlo"], pb["xhi"],
                            pb["lb"], pb["ub"])
        ez = max(ez, float(np.abs(Z[i] - zr).max()))
        ey = max(ey, float(np.abs(Y[i] - yr).max()) / (1.0 + float(np.abs(yr).max())))
        ex = max(ex, float(np.abs(X[i].reshape(-1) - (d["xbar"] + d["Gam"] @ zr)).max()))
    assert ez < TOL_F64, ez
    assert ex < TOL_F64, ex
    assert ey < 1e-7, ey


def test_mpc_qp_routes_n50_to_ipm_and_n30_agrees(dev):
    """mpcqp_mpc_qp: N = 50 with the state box (n + m = 300 > 192) now solves
    (stage-wise interior point); at N = 30 the interior point (MPCQP_IPM) and
    the dense workgroup active set give the same z."""
    Q, qn, R = _SOL
    pb = _bicycle(dev, 8, 50, 0.05, 4)
    args = (pb["A"], pb["B"], _t(Q, dev), _t(R, dev), _t(qn * Q, dev), 50, pb["x0"])
    kw = dict(xlo=_t(pb["xlo"], dev), xhi=_t(pb["xhi"], dev), lb=_t(pb["lb"], dev),
              ub=_t(pb["ub"], dev), c=pb["c"], tv=True)
    z, y, st = batched.mpc_qp(*args, **kw)
    r = batched.mpc_ipm(*args, **kw)
    torch.cuda.synchronize()
    assert (batched.status_code(st) == 0).all()
    assert float((z - r["z"]).abs().max()) == 0.0  # the same kernel
    Q, qn, R = _MAIN
    pb = _bicycle(dev, 24, 30, 0.08, 5)
    args = (pb["A"], pb["B"], _t(Q, dev), _t(R, dev), _t(qn * Q, dev), 30, pb["x0"])
    kw = dict(xlo=_t(pb["xlo"], dev), xhi=_t(pb["xhi"], dev), lb=_t(pb["lb"], dev),
              ub=_t(pb["ub"], dev), c=pb["c"], tv=True)
    z1, y1, st1 = batched.mpc_qp(*args, **kw)
    z2, y2, st2 = batched.mpc_qp(*args, **kw, ipm=True)
    torch.cuda.synchronize()
    assert (batched.status_code(st1) == 0).all() and (batched.status_code(st2) == 0).all()
    assert float((z1 - z2).abs().max()) < TOL_F64
    assert float((y1 - y2).abs().max()) < 1e-7 * (1 + float(y1.abs().max()))


def test_ipm_cfg2_golden(dev, golden):
    """Config 2 (double integrator, |u| <= 1, N = 20, shared plant): the 64
    golden BVLS minimisers."""
    g = golden("boxqp_cfg2.npz")
    N = int(g["N"])
    t = lambda a: _t(a, dev)  # noqa: E731
    r = batched.mpc_ipm(t(g["A"]), t(g["B"]), t(g["Q"]), t(g["R"]), t(g["Pf"]), N, t(g["x0"]),
                        lb=-1.0, ub=1.0)
    torch.cuda.synchronize()
    assert (batched.status_code(r["status"]) == 0).all()
    err = float(np.abs(r["z"].cpu().numpy() - g["z"]).max())
    assert err < TOL_F64, err


def test_ipm_unconstrained_is_riccati(dev, golden):
    """No bounds at all: one Newton step is the LQR solution; it must equal
    the rollout of the reference's Riccati gains (FHC.py:51-61)."""
    s1 = golden("session1.npz")
    A, B, Q, R, Pf = s1["fhc_A"], s1["fhc_B"], s1["fhc_Q"], s1["fhc_R"].reshape(1, 1), s1["fhc_Pf"]
    N = 10
    K = s1[f"fhc_K_N{N}"]
    rng = np.random.default_rng(9)
    X0 = rng.uniform(-10, 10, (5, 2))
    t = lambda a: _t(a, dev)  # noqa: E731
    r = batched.mpc_ipm(t(A), t(B), t(Q), t(R), t(Pf), N, t(X0))
    torch.cuda.synchronize()
    assert (batched.status_code(r["status"]) == 0).all()
    Z = r["z"].cpu().numpy()
    for i in range(5):
        x = X0[i].copy()
        for k in range(N):
            u = K[k] @ x
            assert abs(Z[i, k] - u[0]) < 1e-10
            x = A @ x + B @ u


def test_ipm_f32_inputs(dev):
    """fp32 storage, fp64 arithmetic: against the fp64 oracle on the
    fp32-rounded inputs, far below the north-star 1e-5."""
    Q, qn, R = _MAIN
    N, dt = 30, torch.float32
    pb = _bicycle(dev, 8, N, 0.08, 6)
    A, B, c, x0 = (pb[k].to(dt).contiguous() for k in ("A", "B", "c", "x0"))
    t = lambda a: _t(a, dev, dt)  # noqa: E731
    r = batched.mpc_ipm(A, B, t(Q), t(R), t(qn * Q), N, x0, xlo=t(pb["xlo"]), xhi=t(pb["xhi"]),
                        lb=t(pb["lb"]), ub=t(pb["ub"]), c=c, tv=True)
    torch.cuda.synchronize()
    assert (batched.status_code(r["status"]) == 0).all()
    rd = lambda a: torch.as_tensor(np.asarray(a, float), dtype=dt).double().numpy()  # noqa: E731
    An, Bn, cn, Xn = (v.double().cpu().numpy() for v in (A, B, c, x0))
    err = 0.0
    for i in range(8):
        zr, _, _ = _oracle(An[i], Bn[i], cn[i], Xn[i], rd(Q), rd(R), rd(qn * Q), N, rd(pb["xlo"]),
                           rd(pb["xhi"]), rd(pb["lb"]), rd(pb["ub"]))
        err = max(err, float(np.abs(r["z"][i].double().cpu().numpy() - zr).max()))
    assert err < 1e-6, err


def test_ipm_one_sided_and_per_instance_bounds(dev):
    """Per-instance state bounds, upper side only, shared plant (session-2
    style double integrator, N = 40): against the oracle; instances the
    oracle finds infeasible are skipped (the interior point reports them as
    not converged)."""
    rng = np.random.default_rng(12)
    nx, N, b = 2, 40, 10
    A = np.array([[1.0, 0.5], [0.0, 1.0]])
    B = np.array([[0.0], [-0.5]])
    Q, R = np.diag([1.0, 0.1]), np.array([[0.1]])
    X0 = np.stack([rng.uniform(-4, 6, b), rng.uniform(-2, 3, b)], -1)
    xhi = np.tile([8.0, 6.0], (b, N)) + rng.uniform(0, 1, (b, N * nx))
    t = lambda a: _t(a, dev)  # noqa: E731
    r = batched.mpc_ipm(t(A), t(B), t(Q), t(R), t(Q), N, t(X0), xhi=t(xhi), lb=-1.0, ub=1.0)
    torch.cuda.synchronize()
    code = batched.status_code(r["status"]).cpu().numpy()
    Z = r["z"].cpu().numpy()
    solved = 0
    for i in range(b):
        d = oc.condense(A, B, Q, R, Q, N, x0=X0[i])
        try:
            zr = oq.poly_qp(d["H"], d["f"], d["Gam"], xhi[i] - d["xbar"], -np.ones(N),
                            np.ones(N))[0]
        except ValueError:
            assert code[i] != 0
            continue
        solved += 1
        assert code[i] == 0, code[i]
        assert np.abs(Z[i] - zr).max() < TOL_F64
    assert solved > 0


def test_ipm_large_batch_kkt(dev):
    """A full batch (4096, N = 50, session4_sol weights): every instance
    optimal and polished, and the KKT conditions of the condensed QP hold for
    a sample (size-independent certificate)."""
    Q, qn, R = _SOL
    N, b = 50, 4096
    pb = _bicycle(dev, b, N, 0.05, 7)
    r = batched.mpc_ipm(pb["A"], pb["B"], _t(Q, dev), _t(R, dev), _t(qn * Q, dev), N, pb["x0"],
                        xlo=_t(pb["xlo"], dev), xhi=_t(pb["xhi"], dev), lb=_t(pb["lb"], dev),
                        ub=_t(pb["ub"], dev), c=pb["c"], tv=True)
    torch.cuda.synchronize()
    st = r["status"].cpu().numpy()
    assert ((st & 0xFF) == 0).all(), np.unique(st & 0xFF, return_counts=True)
    assert ((st & STATUS_POLISHED) != 0).all()
    A, B, c, X0 = (pb[k].cpu().numpy() for k in ("A", "B", "c", "x0"))
    Z, Y, LU = r["z"].cpu().numpy(), r["y"].cpu().numpy(), r["lam_u"].cpu().numpy()
    for i in np.linspace(0, b - 1, 12).astype(int):
        d = oc.condense(A[i], B[i], Q, R, qn * Q, N, x0=X0[i], c=c[i])
        xs = d["xbar"] + d["Gam"] @ Z[i]
        xlo, xhi = np.tile(pb["xlo"], N), np.tile(pb["xhi"], N)
        assert (xs <= xhi + 1e-9).all() and (xs >= xlo - 1e-9).all()
        assert (Z[i] <= pb["ub"] + 1e-12).all() and (Z[i] >= pb["lb"] - 1e-12).all()
        g = d["H"] @ Z[i] + d["f"] + d["Gam"].T @ Y[i] + LU[i]
        assert np.abs(g).max() < 1e-8 * (1 + np.abs(d["f"]).max())
        assert (Y[i][xs < xhi - 1e-7] <= 1e-9).all() and (Y[i][xs > xlo + 1e-7] >= -1e-9).all()
        assert (LU[i][Z[i] < pb["ub"] - 1e-7] <= 1e-9).all()
        assert (LU[i][Z[i] > pb["lb"] + 1e-7] >= -1e-9).all()


@pytest.mark.parametrize("N,ts,w,seed", [(30, 0.08, _MAIN, 5), (50, 0.05, _SOL, 6)])
def test_ipm_wave_vs_quad_kernel(dev, monkeypatch, N, ts, w, seed):
    """The whole-wave kernel (ipm_wave_kernel: per-stage work on 16 quads,
    the Riccati and forward recursions on the fp64 matrix cores) against the
    quad kernel it replaced (MPCQP_IPM_WAVE=0, read at every launch): the same
    polished vertices to 1e-9, status and iteration counts alike for almost
    every instance (the reductions' summation order differs)."""
    Q, qn, R = w
    pb = _bicycle(dev, 48, N, ts, seed)

    def run():
        r = batched.mpc_ipm(pb["A"], pb["B"], _t(Q, dev), _t(R, dev), _t(qn * Q, dev), N, pb["x0"],
                            xlo=_t(pb["xlo"], dev), xhi=_t(pb["xhi"], dev), lb=_t(pb["lb"], dev),
                            ub=_t(pb["ub"], dev), c=pb["c"], tv=True)
        torch.cuda.synchronize()
        return r["z"].cpu().numpy(), r["status"].cpu().numpy()

    zw, sw = run()
    monkeypatch.setenv("MPCQP_IPM_WAVE", "0")
    zq, sq = run()
    assert ((sw & 0xFF) == 0).all() and ((sq & 0xFF) == 0).all()
    assert ((sw & STATUS_POLISHED) != 0).all() and ((sq & STATUS_POLISHED) != 0).all()
    assert np.abs(zw - zq).max() < TOL_F64
    its_w, its_q = (sw >> 8) & 0xFFFF, (sq >> 8) & 0xFFFF
    assert (np.abs(its_w - its_q) <= 1).mean() >= 0.9, (its_w, its_q)
