"""GPU parity: mpcqp_solve_box vs the committed golden minimisers (SciPy BVLS,
cross-checked by the oracle active set) and vs the oracle on random problems.

Bar (BASELINE.json north star): max|u - u_ref| < 1e-5; in fp64 the kernel is
held to 1e-9 (relative to max(1, |u|)).  fp32 problems: 1e-3 relative to the
problem's condition-scaled accuracy (documented per test).
"""
import numpy as np
import pytest
import torch

from model_predictive_control_amd import batched
from oracle import condense as oc
from oracle import qp as oq
from oracle import session1 as s1

pytestmark = pytest.mark.gpu


def _t(a, dev, dt=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)


def _pack(H):
    return np.stack([oc.pack_lower(h) for h in H])


def test_box_golden_cfg2(dev, golden):
    g = golden("boxqp_cfg2.npz")
    N = int(g["N"])
    z, st = batched.solve_box(_t(_pack(g["H"]), dev), _t(g["f"], dev), -1.0, 1.0)
    z = z.cpu().numpy()
    assert (batched.status_code(st) == 0).all()
    assert np.abs(z - g["z"]).max() < 1e-9


def test_box_end_to_end_cfg2_from_plant(dev, golden):
    """Per-instance condense -> solve (the bench pipeline) vs the golden minimisers."""
    g = golden("boxqp_cfg2.npz")
    N = int(g["N"])
    b = g["x0"].shape[0]
    d = batched.condense(_t(np.broadcast_to(g["A"], (b, 2, 2)), dev),
                         _t(np.broadcast_to(g["B"], (b, 2, 1)), dev), _t(g["Q"], dev),
                         _t(g["R"], dev), _t(g["Pf"], dev), N, x0=_t(g["x0"], dev))
    z, st = batched.solve_box(d["H"], d["f"], -1.0, 1.0)
    assert (batched.status_code(st) == 0).all()
    assert np.abs(z.cpu().numpy() - g["z"]).max() < 1e-9


def _random_box_problems(rng, n, batch, cond=1e3):
    Hs, fs, lbs, ubs = [], [], [], []
    for _ in range(batch):
        U, _ = np.linalg.qr(rng.normal(size=(n, n)))
        ev = np.logspace(0, np.log10(cond), n)
        H = (U * ev) @ U.T
        H = 0.5 * (H + H.T)
        f = rng.normal(size=n) * 3 * np.sqrt(cond)
        lb = -rng.uniform(0.1, 2, n)
        ub = rng.uniform(0.1, 2, n)
        lb[rng.random(n) < 0.15] = -np.inf
        ub[rng.random(n) < 0.15] = np.inf
        fx = rng.random(n) < 0.05
        lb[fx] = ub[fx] = np.where(np.isfinite(lb[fx]), lb[fx], 0.3)
        Hs.append(H); fs.append(f); lbs.append(lb); ubs.append(ub)
    return np.array(Hs), np.array(fs), np.array(lbs), np.array(ubs)


@pytest.mark.parametrize("n", [1, 2, 7, 8, 9, 16, 20, 24, 31, 40, 48, 60, 64])
def test_box_random_fp64(dev, n):
    rng = np.random.default_rng(1000 + n)
    H, f, lb, ub = _random_box_problems(rng, n, 24)
    z, st = batched.solve_box(_t(_pack(H), dev), _t(f, dev), _t(lb, dev), _t(ub, dev))
    z = z.cpu().numpy()
    code = batched.status_code(st).cpu().numpy()
    assert (code == 0).all(), code
    for b in range(H.shape[0]):
        zr, _, _ = oq.box_qp(H[b], f[b], lb[b], ub[b])
        assert np.abs(z[b] - zr).max() < 1e-9 * max(1.0, np.abs(zr).max()), (b, np.abs(z[b] - zr).max())
        assert oq.kkt_box(H[b], f[b], lb[b], ub[b], z[b]) < 1e-7 * max(1, np.abs(f[b]).max())


def test_box_shared_H_and_bounds(dev):
    A, B, Q, R, Pf, _ = s1.fhc_setup()
    N = 20
    ref = oc.condense(A, B, Q, R.reshape(1, 1), Pf, N)
    rng = np.random.default_rng(9)
    X0 = rng.uniform(-10, 10, (300, 2))
    f = X0 @ ref["F"].T
    z, st = batched.solve_box(_t(oc.pack_lower(ref["H"]), dev), _t(f, dev), -1.0, 1.0)
    z = z.cpu().numpy()
    assert (batched.status_code(st) == 0).all()
    for b in range(0, 300, 13):
        zr, _, _ = oq.box_qp(ref["H"], f[b], -np.ones(N), np.ones(N))
        assert np.abs(z[b] - zr).max() < 1e-9


def test_box_statuses(dev):
    n = 4
    H = np.eye(n)
    Hbad = np.diag([1.0, -1.0, 1.0, 1.0])
    f = np.ones((3, n))
    P = np.stack([oc.pack_lower(H), oc.pack_lower(Hbad), oc.pack_lower(H)])
    f[2, 1] = np.nan
    z, st = batched.solve_box(_t(P, dev), _t(f, dev), -1.0, 1.0)
    code = batched.status_code(st).cpu().numpy()
    assert code.tolist() == [0, 2, 4]
    assert np.allclose(z[0].cpu().numpy(), -1.0)
    lb = np.zeros((1, n)); ub = np.zeros((1, n)); lb[0, 2] = 1.0
    z, st = batched.solve_box(_t(oc.pack_lower(H), dev), _t(f[:1], dev), _t(lb, dev), _t(ub, dev))
    assert int(batched.status_code(st)[0]) == 3


def test_box_unconstrained_is_linear_solve(dev):
    rng = np.random.default_rng(4)
    H, f, _, _ = _random_box_problems(rng, 20, 16, cond=1e2)
    z, st = batched.solve_box(_t(_pack(H), dev), _t(f, dev))
    z = z.cpu().numpy()
    for b in range(16):
        assert np.abs(z[b] + np.linalg.solve(H[b], f[b])).max() < 1e-10 * max(1, np.abs(z[b]).max())


def test_box_fp32(dev):
    """fp32: cond(H) ~ 1e2, tolerance 2e-4 relative (fp32 eps * cond * n)."""
    rng = np.random.default_rng(77)
    H, f, lb, ub = _random_box_problems(rng, 20, 32, cond=1e2)
    z, st = batched.solve_box(_t(_pack(H), dev, torch.float32), _t(f, dev, torch.float32),
                              _t(lb, dev, torch.float32), _t(ub, dev, torch.float32))
    z = z.double().cpu().numpy()
    assert (batched.status_code(st) == 0).all()
    for b in range(32):
        zr, _, _ = oq.box_qp(H[b], f[b], lb[b], ub[b])
        assert np.abs(z[b] - zr).max() < 2e-4 * max(1, np.abs(zr).max())


def test_box_cfg2_full_batch_kkt(dev):
    """BASELINE config 2 at full size (B = 4096): every instance optimal, every
    KKT residual certified on device, oracle spot-checks."""
    A, B, Q, R, Pf, _ = s1.fhc_setup()
    R = R.reshape(1, 1)
    N, batch = 20, 4096
    rng = np.random.default_rng(20261015 + 2)
    X0 = rng.uniform(-10, 10, (batch, 2))
    d = batched.condense(_t(np.broadcast_to(A, (batch, 2, 2)), dev),
                         _t(np.broadcast_to(B, (batch, 2, 1)), dev), _t(Q, dev), _t(R, dev),
                         _t(Pf, dev), N, x0=_t(X0, dev))
    z, st = batched.solve_box(d["H"], d["f"], -1.0, 1.0)
    assert (batched.status_code(st) == 0).all()
    Hf = batched.unpack_lower(d["H"], N)
    g = torch.einsum("bij,bj->bi", Hf, z) + d["f"]
    at_l = z <= -1 + 1e-12
    at_u = z >= 1 - 1e-12
    free = ~(at_l | at_u)
    assert float(g[free].abs().max()) < 1e-9
    assert float((-g[at_l]).clamp(min=0).max()) < 1e-9
    assert float(g[at_u].clamp(min=0).max()) < 1e-9
    assert float(z.abs().max()) <= 1.0
    zc = z.cpu().numpy()
    for b in (0, 1, 2047, 4095):
        ref = oc.condense(A, B, Q, R, Pf, N, x0=X0[b])
        zr, _, _ = oq.box_qp(ref["H"], ref["f"], -np.ones(N), np.ones(N))
        assert np.abs(zc[b] - zr).max() < 1e-9
    it = batched.status_iters(st)
    assert int(it.max()) <= 3 * N + 30


# ------------------------------------------------ fused condense + box solve
@pytest.mark.parametrize("nx,nu,N,tv", [(2, 1, 20, False), (1, 1, 7, False), (2, 2, 16, True),
                                        (3, 1, 12, True), (4, 2, 16, True), (4, 1, 32, False),
                                        (2, 1, 1, False)])
def test_mpc_box_fused_vs_oracle(dev, nx, nu, N, tv):
    rng = np.random.default_rng(31 * nx + 7 * nu + N)
    batch = 12
    shA = (batch, N, nx, nx) if tv else (batch, nx, nx)
    shB = (batch, N, nx, nu) if tv else (batch, nx, nu)
    A = rng.normal(size=shA) * (0.8 / np.sqrt(nx)) + 0.4 * np.eye(nx)
    # keep the plants (marginally) stable so cond(H) stays moderate over N=32
    rho = np.abs(np.linalg.eigvals(A.reshape(-1, nx, nx))).max(axis=-1).reshape(A.shape[:-2])
    A = A / np.maximum(1.0, rho / 1.02)[..., None, None]
    B = rng.normal(size=shB)
    M = rng.normal(size=(nx, nx)); Q = M @ M.T / nx + 0.2 * np.eye(nx)
    R = np.diag(rng.uniform(0.1, 1.0, nu)); Qf = 3 * Q
    x0 = rng.normal(size=(batch, nx)) * 3
    c = rng.normal(size=(batch, N, nx)) * 0.3 if tv else None
    n = N * nu
    lb = -rng.uniform(0.2, 1.0, (batch, n)); ub = rng.uniform(0.2, 1.0, (batch, n))
    z, st = batched.mpc_box(_t(A, dev), _t(B, dev), _t(Q, dev), _t(R, dev), _t(Qf, dev), N,
                            _t(x0, dev), _t(lb, dev), _t(ub, dev),
                            c=None if c is None else _t(c, dev), tv=tv)
    z = z.cpu().numpy()
    assert (batched.status_code(st) == 0).all(), st
    for b in range(batch):
        ref = oc.condense(A[b], B[b], Q, R, Qf, N, x0=x0[b], c=None if c is None else c[b])
        zr, _, _ = oq.box_qp(ref["H"], ref["f"], lb[b], ub[b])
        assert np.abs(z[b] - zr).max() < 1e-9 * max(1, np.abs(zr).max()), (b, np.abs(z[b] - zr).max())


def test_mpc_box_cfg2_golden_and_full_batch(dev, golden):
    g = golden("boxqp_cfg2.npz")
    N = int(g["N"])
    z, st = batched.mpc_box(_t(g["A"], dev), _t(g["B"], dev), _t(g["Q"], dev), _t(g["R"], dev),
                            _t(g["Pf"], dev), N, _t(g["x0"], dev), -1.0, 1.0)
    assert (batched.status_code(st) == 0).all()
    assert np.abs(z.cpu().numpy() - g["z"]).max() < 1e-9
    # full config-2 batch: fused == split pipeline
    A, B, Q, R, Pf, _ = s1.fhc_setup()
    R = R.reshape(1, 1)
    batch = 4096
    X0 = np.random.default_rng(5).uniform(-10, 10, (batch, 2))
    Ab = _t(np.broadcast_to(A, (batch, 2, 2)), dev)
    Bb = _t(np.broadcast_to(B, (batch, 2, 1)), dev)
    zf, stf = batched.mpc_box(Ab, Bb, _t(Q, dev), _t(R, dev), _t(Pf, dev), N, _t(X0, dev), -1.0, 1.0)
    d = batched.condense(Ab, Bb, _t(Q, dev), _t(R, dev), _t(Pf, dev), N, x0=_t(X0, dev))
    zs, sts = batched.solve_box(d["H"], d["f"], -1.0, 1.0)
    assert (batched.status_code(stf) == 0).all() and (batched.status_code(sts) == 0).all()
    assert float((zf - zs).abs().max()) < 1e-9


def test_mpc_box_fp32(dev):
    A, B, Q, R, Pf, _ = s1.fhc_setup()
    R = R.reshape(1, 1)
    N, batch = 20, 64
    X0 = np.random.default_rng(8).uniform(-3, 3, (batch, 2))
    f32 = torch.float32
    z, st = batched.mpc_box(_t(A, dev, f32), _t(B, dev, f32), _t(Q, dev, f32), _t(R, dev, f32),
                            _t(Pf, dev, f32), N, _t(X0, dev, f32), -1.0, 1.0)
    z = z.double().cpu().numpy()
    assert (batched.status_code(st) == 0).all()
    for b in range(0, batch, 5):
        ref = oc.condense(A, B, Q, R, Pf, N, x0=X0[b])
        zr, _, _ = oq.box_qp(ref["H"], ref["f"], -np.ones(N), np.ones(N))
        # fp32 with cond(H) ~ 6e3: 2e-3 absolute on |u| <= 1
        assert np.abs(z[b] - zr).max() < 2e-3


@pytest.mark.parametrize("n", [3, 13, 20, 32])
def test_quad_and_wave_kernels_agree(dev, n, monkeypatch):
    """The 4-QPs-per-wavefront kernels (n <= 32) and the one-QP-per-wavefront
    kernels solve the same problems to the same minimisers (odd batch sizes
    exercise the empty groups of the last wavefront)."""
    rng = np.random.default_rng(500 + n)
    H, f, lb, ub = _random_box_problems(rng, n, 37)
    args = (_t(_pack(H), dev), _t(f, dev), _t(lb, dev), _t(ub, dev))
    monkeypatch.setenv("MPCQP_KERNEL", "wave")
    zw, sw = batched.solve_box(*args)
    monkeypatch.delenv("MPCQP_KERNEL")
    zq, sq = batched.solve_box(*args)
    assert (batched.status_code(sw) == 0).all() and (batched.status_code(sq) == 0).all()
    assert float((zw - zq).abs().max()) < 1e-9 * max(1.0, float(zw.abs().max()))
    zq = zq.cpu().numpy()
    for b in range(0, 37, 6):
        zr, _, _ = oq.box_qp(H[b], f[b], lb[b], ub[b])
        assert np.abs(zq[b] - zr).max() < 1e-9 * max(1.0, np.abs(zr).max())
