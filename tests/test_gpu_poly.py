"""GPU parity: mpcqp_solve_poly vs the Goldfarb-Idnani oracle and the committed
session-2/3 golden minimisers (state box on x_1..x_N + input box, the OCP of
session_4/main.py:58-69 restricted to the linear session-2/3 plants)."""
import numpy as np
import pytest
import torch

from model_predictive_control_amd import batched, problems
from oracle import condense as oc
from oracle import qp as oq

pytestmark = pytest.mark.gpu


def _t(a, dev, dt=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)


@pytest.mark.parametrize("tag,cls", [("session_2", problems.Problem), ("session_3", problems.Problem3)])
def test_poly_session_golden(dev, golden, tag, cls):
    gp = golden("polyqp_s2.npz")
    p = cls()
    N = p.N
    X0 = gp[f"{tag}_x0"]
    b = X0.shape[0]
    d = batched.condense(_t(p.A, dev), _t(p.B, dev), _t(p.Q, dev), _t(p.R, dev), _t(p.Q, dev), N,
                         x0=_t(X0, dev), outputs=("H", "f", "Gam", "xbar"))
    G = d["Gam"][0]
    hl = _t(np.tile(p.x_min, N), dev) - d["xbar"]
    hu = _t(np.tile(p.x_max, N), dev) - d["xbar"]
    z, y, st = batched.solve_poly(d["H"][0], d["f"], G, hl, hu, lbz=p.u_min, ubz=p.u_max)
    code = batched.status_code(st).cpu().numpy()
    z = z.cpu().numpy()
    feas = gp[f"{tag}_feasible"]
    assert (code[feas] == 0).all(), code
    assert (code[~feas] == 3).all(), code
    assert np.abs(z[feas] - gp[f"{tag}_z"][feas]).max() < 1e-8


@pytest.mark.parametrize("n,m", [(5, 3), (20, 20), (40, 24), (64, 40), (200, 40)])
def test_poly_random_polytope(dev, n, m):
    """Config-4 shape family: shared H, G (m rows, h > 0 so z = 0 is feasible)."""
    rng = np.random.default_rng(n * 131 + m)
    M = rng.normal(size=(n, n))
    H = M @ M.T / n + 0.5 * np.eye(n)
    G = rng.normal(size=(m, n))
    batch = 16 if n < 200 else 6
    f = rng.normal(size=(batch, n)) * 4
    h = rng.uniform(0.2, 1.0, size=(batch, m))
    z, y, st = batched.solve_poly(_t(oc.pack_lower(H), dev), _t(f, dev), _t(G, dev), None, _t(h, dev))
    z = z.cpu().numpy()
    y = y.cpu().numpy()
    assert (batched.status_code(st) == 0).all()
    for b in range(batch):
        zr, lam, _ = oq.poly_qp(H, f[b], G, h[b])
        assert np.abs(z[b] - zr).max() < 1e-8 * max(1, np.abs(zr).max()), np.abs(z[b] - zr).max()
        assert np.abs(np.maximum(y[b], 0) - lam).max() < 1e-6 * max(1, np.abs(lam).max())
        assert (G @ z[b] - h[b]).max() < 1e-9


def test_poly_two_sided_with_box(dev):
    rng = np.random.default_rng(3)
    n, m, batch = 12, 10, 20
    M = rng.normal(size=(n, n)); H = M @ M.T + np.eye(n)
    G = rng.normal(size=(m, n))
    f = rng.normal(size=(batch, n)) * 5
    hl = -rng.uniform(0.5, 1.0, (batch, m)); hu = rng.uniform(0.5, 1.0, (batch, m))
    z, y, st = batched.solve_poly(_t(oc.pack_lower(H), dev), _t(f, dev), _t(G, dev), _t(hl, dev),
                                  _t(hu, dev), lbz=-0.7, ubz=0.7)
    z = z.cpu().numpy()
    assert (batched.status_code(st) == 0).all()
    for b in range(batch):
        Gs = np.vstack([G, -G])
        hs = np.concatenate([hu[b], -hl[b]])
        zr, _, _ = oq.poly_qp(H, f[b], Gs, hs, lb=np.full(n, -0.7), ub=np.full(n, 0.7))
        assert np.abs(z[b] - zr).max() < 1e-8


@pytest.mark.parametrize("nx,nu,N,m,box", [(12, 4, 50, 40, False), (4, 2, 10, 12, True), (2, 1, 20, 6, True)])
def test_poly_parametric_x0(dev, nx, nu, N, m, box):
    """PolyQP: shared factors once (poly_setup), per-instance x0 -> z with the
    fused s0 / z epilogue; BASELINE config-4 shape first.  Checked against the
    Goldfarb-Idnani oracle on the explicitly condensed QP."""
    rng = np.random.default_rng(nx * 100 + N)
    U, _ = np.linalg.qr(rng.normal(size=(nx, nx)))
    A = (U * rng.uniform(0.5, 0.98, nx)) @ U.T
    B = rng.normal(size=(nx, nu)) / np.sqrt(nx)
    Q, R = np.eye(nx), 0.1 * np.eye(nu)
    n = N * nu
    d = oc.condense(A, B, Q, R, Q, N)
    G = rng.normal(size=(m, n))
    h = rng.uniform(0.5, 1.5, size=m)
    b = 24
    X0 = rng.normal(size=(b, nx)) * 3
    f1 = rng.normal(size=(b, n)) * 0.1
    lbz, ubz = (-0.4, 0.4) if box else (None, None)
    qp = batched.PolyQP(_t(oc.pack_lower(d["H"]), dev), _t(G, dev), _t(d["F"], dev), lbz, ubz)
    z, y, st = qp.solve(_t(X0, dev), _t(f1, dev), hu=_t(h, dev))
    assert (batched.status_code(st) == 0).all(), batched.status_code(st)
    z = z.cpu().numpy()
    for i in range(b):
        fi = d["F"] @ X0[i] + f1[i]
        zr = oq.poly_qp(d["H"], fi, G, h, None if lbz is None else np.full(n, lbz),
                        None if ubz is None else np.full(n, ubz))[0]
        assert np.abs(z[i] - zr).max() < 1e-8 * max(1.0, np.abs(zr).max()), np.abs(z[i] - zr).max()
    # same factors, gradient-only form (x0 = None) gives the same answer
    z2, _, st2 = qp.solve(None, _t(X0 @ d["F"].T + f1, dev), hu=_t(h, dev))
    assert (batched.status_code(st2) == 0).all()
    assert np.abs(z2.cpu().numpy() - z).max() < 1e-9
