"""GPU parity: mpcqp_solve_qp (one QP per workgroup, mixed primal/dual active
set on [[H, G'], [G, 0]]) against the CPU oracles -- the per-step QP of
session_4/main.py:115-116 with input box (main.py:68-69) and state box
(main.py:58-61) rows, per-instance data (BASELINE configs 3 and 5)."""
import numpy as np
import pytest
import torch

from model_predictive_control_amd import batched, problems
from oracle import condense as oc
from oracle import qp as oq

pytestmark = pytest.mark.gpu


def _t(a, dev, dt=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)


def _spd(rng, n, cond=50.0):
    Qm, _ = np.linalg.qr(rng.normal(size=(n, n)))
    ev = np.geomspace(1.0, cond, n)
    return (Qm * ev) @ Qm.T


def _oracle_two_sided(H, f, G, hl, hu, lb, ub):
    """poly_qp wants C z <= d: stack [G; -G] with the finite sides."""
    rows, rhs = [], []
    for r in range(G.shape[0]):
        if np.isfinite(hu[r]):
            rows.append(G[r]); rhs.append(hu[r])
        if np.isfinite(hl[r]):
            rows.append(-G[r]); rhs.append(-hl[r])
    C = np.array(rows).reshape(-1, f.size)
    d = np.array(rhs)
    z, lam, _ = oq.poly_qp(H, f, C, d, lb, ub)
    return z


def _kkt_two_sided(H, f, G, hl, hu, lb, ub, z, y, tol):
    """Stationarity with row multipliers y (>0 at hu) and box multipliers
    read off the residual; sign, complementarity and feasibility."""
    r = H @ z + f + (G.T @ y if G is not None else 0.0)
    scale = max(1.0, np.abs(f).max())
    at_l = np.isclose(z, lb, atol=tol * scale, rtol=0) if lb is not None else np.zeros_like(z, bool)
    at_u = np.isclose(z, ub, atol=tol * scale, rtol=0) if ub is not None else np.zeros_like(z, bool)
    free = ~(at_l | at_u)
    assert np.abs(r[free]).max(initial=0) < tol * scale, np.abs(r[free]).max(initial=0)
    assert (r[at_l & ~at_u] > -tol * scale).all()
    assert (r[at_u & ~at_l] < tol * scale).all()
    if G is not None:
        gz = G @ z
        assert (gz - hu).max(initial=-1) < tol * scale
        assert (hl - gz).max(initial=-1) < tol * scale
        ya = np.abs(y) > tol * scale
        up = y > tol * scale
        lo = y < -tol * scale
        assert np.abs(gz[up] - hu[up]).max(initial=0) < tol * scale
        assert np.abs(gz[lo] - hl[lo]).max(initial=0) < tol * scale
        assert ya.sum() <= z.size


def test_qp_box_cfg2_golden_block_kernel(dev, golden, monkeypatch):
    """Config-2 box QPs through the workgroup kernel (MPCQP_KERNEL=block)."""
    g = golden("boxqp_cfg2.npz")
    monkeypatch.setenv("MPCQP_KERNEL", "block")
    z, st = batched.solve_box(batched.pack_lower(_t(g["H"], dev)), _t(g["f"], dev), -1.0, 1.0)
    assert (batched.status_code(st) == 0).all()
    assert np.abs(z.cpu().numpy() - g["z"]).max() < 1e-9


@pytest.mark.parametrize("n", [48, 100, 160, 192])
def test_qp_box_large(dev, n):
    """Input-box QPs beyond the wavefront kernels (config 5: n = N*nu = 160)."""
    rng = np.random.default_rng(1000 + n)
    b = 6
    Hs = [_spd(rng, n) for _ in range(b)]
    f = rng.normal(size=(b, n)) * 20
    lb = -rng.uniform(0.5, 2.0, size=(b, n))
    ub = rng.uniform(0.5, 2.0, size=(b, n))
    Hp = np.stack([oc.pack_lower(H) for H in Hs])
    z, st = batched.solve_box(_t(Hp, dev), _t(f, dev), _t(lb, dev), _t(ub, dev))
    assert (batched.status_code(st) == 0).all(), st
    z = z.cpu().numpy()
    for i in range(b):
        zr = oq.box_qp(Hs[i], f[i], lb[i], ub[i])[0]
        assert np.abs(z[i] - zr).max() < 1e-8 * max(1.0, np.abs(zr).max())


@pytest.mark.parametrize("n,m", [(6, 4), (20, 40), (40, 24), (60, 120), (100, 28)])
def test_qp_rows_random(dev, n, m):
    """Per-instance H, G, two-sided rows and a box: oracle GI + KKT."""
    rng = np.random.default_rng(7 * n + m)
    b = 5
    Hs = [_spd(rng, n) for _ in range(b)]
    Gs = rng.normal(size=(b, m, n))
    f = rng.normal(size=(b, n)) * 10
    hl = -rng.uniform(0.2, 1.5, size=(b, m))
    hu = rng.uniform(0.2, 1.5, size=(b, m))
    hl[:, ::5] = -np.inf  # one-sided rows
    lb = -np.full(n, 1.5)
    ub = np.full(n, 1.5)
    Hp = np.stack([oc.pack_lower(H) for H in Hs])
    z, y, st = batched.solve_qp(_t(Hp, dev), _t(f, dev), _t(Gs, dev), _t(hl, dev), _t(hu, dev),
                                _t(lb, dev), _t(ub, dev))
    assert (batched.status_code(st) == 0).all(), batched.status_code(st)
    z, y = z.cpu().numpy(), y.cpu().numpy()
    for i in range(b):
        zr = _oracle_two_sided(Hs[i], f[i], Gs[i], hl[i], hu[i], lb, ub)
        assert np.abs(z[i] - zr).max() < 1e-7 * max(1.0, np.abs(zr).max()), np.abs(z[i] - zr).max()
        _kkt_two_sided(Hs[i], f[i], Gs[i], hl[i], hu[i], lb, ub, z[i], y[i], 1e-7)


def test_qp_dependent_rows(dev):
    """Duplicated rows and rows parallel to box directions (dependent on the
    active set) must not stall or break the active set."""
    rng = np.random.default_rng(5)
    n, b = 12, 8
    H = _spd(rng, n)
    G0 = rng.normal(size=(4, n))
    G = np.vstack([G0, G0, np.eye(n)[:3], 2 * G0[:2]])  # 4 + 4 + 3 + 2 rows
    m = G.shape[0]
    hu = np.concatenate([np.full(4, 0.3), np.full(4, 0.3), np.full(3, 0.2), np.full(2, 0.6)])
    hl = -hu
    f = rng.normal(size=(b, n)) * 30
    z, y, st = batched.solve_qp(_t(oc.pack_lower(H), dev), _t(f, dev), _t(G, dev), _t(hl, dev),
                                _t(hu, dev), -1.0, 1.0)
    assert (batched.status_code(st) == 0).all(), batched.status_code(st)
    z = z.cpu().numpy()
    for i in range(b):
        zr = _oracle_two_sided(H, f[i], G, hl, hu, -np.ones(n), np.ones(n))
        assert np.abs(z[i] - zr).max() < 1e-7, np.abs(z[i] - zr).max()


def test_qp_infeasible_and_nonconvex(dev):
    n = 4
    H = np.eye(n)
    G = np.vstack([np.ones(n), np.ones(n)])
    hl = np.array([1.0, -np.inf])
    hu = np.array([np.inf, -1.0])  # sum z >= 1 and sum z <= -1
    f = np.zeros((2, n))
    z, y, st = batched.solve_qp(_t(oc.pack_lower(H), dev), _t(f, dev), _t(G, dev), _t(hl, dev),
                                _t(hu, dev))
    assert (batched.status_code(st) == 3).all()
    Hn = np.diag([1.0, -1.0, 1.0, 1.0])
    z, y, st = batched.solve_qp(_t(oc.pack_lower(Hn), dev), _t(f, dev), _t(G, dev), None,
                                _t(np.ones(2), dev))
    assert (batched.status_code(st) == 2).all()


@pytest.mark.parametrize("tag,cls", [("session_2", problems.Problem), ("session_3", problems.Problem3)])
def test_qp_session_golden(dev, golden, tag, cls):
    """Session-2/3 state-box OCPs (golden minimisers) with per-instance rows."""
    gp = golden("polyqp_s2.npz")
    p = cls()
    N = p.N
    X0 = gp[f"{tag}_x0"]
    d = batched.condense(_t(p.A, dev), _t(p.B, dev), _t(p.Q, dev), _t(p.R, dev), _t(p.Q, dev), N,
                         x0=_t(X0, dev), outputs=("H", "f", "Gam", "xbar"))
    hl = _t(np.tile(p.x_min, N), dev) - d["xbar"]
    hu = _t(np.tile(p.x_max, N), dev) - d["xbar"]
    z, y, st = batched.solve_qp(d["H"][0], d["f"], d["Gam"][0], hl, hu, p.u_min, p.u_max)
    code = batched.status_code(st).cpu().numpy()
    feas = gp[f"{tag}_feasible"]
    assert (code[feas] == 0).all(), code
    assert (code[~feas] == 3).all(), code
    assert np.abs(z.cpu().numpy()[feas] - gp[f"{tag}_z"][feas]).max() < 1e-8


def test_qp_fp32_matches_fp64(dev):
    """Config-5 shape (n = 160 input box) in fp32 against the fp64 solve."""
    rng = np.random.default_rng(55)
    n, b = 160, 8
    Hs = [_spd(rng, n, cond=20.0) for _ in range(b)]
    Hp = np.stack([oc.pack_lower(H) for H in Hs])
    f = rng.normal(size=(b, n)) * 10
    z64, st64 = batched.solve_box(_t(Hp, dev), _t(f, dev), -1.0, 1.0)
    z32, st32 = batched.solve_box(_t(Hp, dev, torch.float32), _t(f, dev, torch.float32), -1.0, 1.0)
    assert (batched.status_code(st64) == 0).all() and (batched.status_code(st32) == 0).all()
    assert (z32.double() - z64).abs().max().item() < 2e-3
