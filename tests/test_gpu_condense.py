"""GPU parity: mpcqp_condense vs the explicit-matrix oracle (oracle/condense.py).

Tolerances: fp64 1e-10 relative to the matrix scale; fp32 2e-5 relative.
"""
import numpy as np
import pytest
import torch

from model_predictive_control_amd import batched
from oracle import condense as oc
from oracle import session1 as s1

pytestmark = pytest.mark.gpu


def _t(a, dev, dt=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)


def _rand_plant(rng, nx, nu, N, tv, batch):
    shapeA = (batch, N, nx, nx) if tv else (batch, nx, nx)
    shapeB = (batch, N, nx, nu) if tv else (batch, nx, nu)
    A = rng.normal(size=shapeA) * (0.9 / np.sqrt(nx)) + (np.eye(nx) * 0.3)
    B = rng.normal(size=shapeB)
    M = rng.normal(size=(nx, nx)); Q = M @ M.T / nx + 0.1 * np.eye(nx)
    Mr = rng.normal(size=(nu, nu)); R = Mr @ Mr.T / nu + 0.5 * np.eye(nu)
    Qf = 2.0 * Q
    return A, B, Q, R, Qf


# output sets of the parity tests: (outputs, gam_packed)
OUTPUT_SETS = {"all": (("H", "F", "f", "Gam", "Phi", "xbar"), False),
               "noGam": (("H", "F", "f", "Phi", "xbar"), False),
               "packed": (("H", "f", "Gam"), True)}


def _condense_set(dev, dt, A, B, Q, R, Qf, N, x0, c, tv, outs):
    """mpcqp_condense with the output set `outs` (OUTPUT_SETS); a packed
    Gamma comes back unpacked, every output in fp64."""
    names, packed = OUTPUT_SETS[outs]
    out = batched.condense(_t(A, dev, dt), _t(B, dev, dt), _t(Q, dev, dt), _t(R, dev, dt),
                           _t(Qf, dev, dt), N, x0=_t(x0, dev, dt),
                           c=None if c is None else _t(c, dev, dt), tv=tv, outputs=names,
                           gam_packed=packed)
    torch.cuda.synchronize()
    if packed:
        out["Gam"] = batched.unpack_gam(out["Gam"], N, A.shape[-2], B.shape[-1])
    return {k: v.double() for k, v in out.items()}


def _check(out, ref, n, rtol):
    H = batched.unpack_lower(out["H"], n).cpu().numpy()
    for b, r in enumerate(ref):
        s = max(1.0, np.abs(r["H"]).max())
        assert np.abs(H[b] - r["H"]).max() <= rtol * s, ("H", b, np.abs(H[b] - r["H"]).max())
        for k in ("F", "f", "Gam", "Phi", "xbar"):
            if k in out:
                got = out[k][b].cpu().numpy().reshape(r[k].shape)
                sk = max(1.0, np.abs(r[k]).max())
                assert np.abs(got - r[k]).max() <= rtol * sk, (k, b, np.abs(got - r[k]).max())


@pytest.mark.parametrize("nx,nu,N", [(1, 1, 1), (2, 1, 20), (3, 2, 7), (4, 2, 30), (5, 3, 6),
                                     (8, 2, 10), (12, 4, 12), (16, 1, 5)])
@pytest.mark.parametrize("tv", [False, True])
@pytest.mark.parametrize("outs", list(OUTPUT_SETS))
def test_condense_fp64_random(dev, nx, nu, N, tv, outs):
    """Every output set routes to its own kernel: with a dense Gamma to
    condense_kernel, without one (nx <= 8) to condense_stream_kernel (F, Phi,
    xbar with padding nx < NX, drift), packed Gamma to either."""
    rng = np.random.default_rng(100 * nx + 10 * nu + N + tv)
    batch = 5
    A, B, Q, R, Qf = _rand_plant(rng, nx, nu, N, tv, batch)
    x0 = rng.normal(size=(batch, nx))
    c = rng.normal(size=(batch, N, nx)) if tv else None
    out = _condense_set(dev, torch.float64, A, B, Q, R, Qf, N, x0, c, tv, outs)
    ref = [oc.condense(A[b], B[b], Q, R, Qf, N, x0=x0[b], c=None if c is None else c[b])
           for b in range(batch)]
    _check(out, ref, N * nu, 1e-10)


def test_condense_shared_plant_per_instance_x0(dev):
    A, B, Q, R, Pf, _ = s1.fhc_setup()
    R = R.reshape(1, 1)
    N, batch = 20, 33
    rng = np.random.default_rng(5)
    X0 = rng.uniform(-10, 10, (batch, 2))
    out = batched.condense(_t(A, dev), _t(B, dev), _t(Q, dev), _t(R, dev), _t(Pf, dev), N,
                           x0=_t(X0, dev), outputs=("H", "F", "f", "xbar"))
    torch.cuda.synchronize()
    ref = [oc.condense(A, B, Q, R, Pf, N, x0=X0[b]) for b in range(batch)]
    _check(out, ref, N, 1e-11)


def test_condense_r_shape_1_like_fhc(dev):
    """FHC.py:141 passes R = np.array([0.1]) (shape (1,))."""
    A, B, Q, R, Pf, x0 = s1.fhc_setup()
    out = batched.condense(_t(A, dev), _t(B, dev), _t(Q, dev), _t(R, dev), _t(Pf, dev), 10,
                           x0=_t(x0.ravel(), dev), outputs=("H", "f"))
    ref = oc.condense(A, B, Q, R.reshape(1, 1), Pf, 10, x0=x0)
    H = batched.unpack_lower(out["H"], 10)[0].cpu().numpy()
    assert np.abs(H - ref["H"]).max() < 1e-11


def test_condense_known_answer_riccati(dev, golden):
    """-H^-1 f from the device condense equals the reference's Riccati rollout."""
    g = golden("session1.npz")
    A, B, Q, R, Pf, x0 = g["fhc_A"], g["fhc_B"], g["fhc_Q"], g["fhc_R"], g["fhc_Pf"], g["fhc_x0"]
    N = 10
    out = batched.condense(_t(A, dev), _t(B, dev), _t(Q, dev), _t(R.reshape(1, 1), dev),
                           _t(Pf, dev), N, x0=_t(x0.ravel(), dev), outputs=("H", "f"))
    H = batched.unpack_lower(out["H"], N)[0].cpu().numpy()
    z = -np.linalg.solve(H, out["f"][0].cpu().numpy())
    K = g["fhc_K_N10"]
    x = x0.ravel()
    for k in range(N):
        u = K[k] @ x
        assert abs(u[0] - z[k]) < 1e-10
        x = A @ x + B @ u


@pytest.mark.parametrize("nx,nu,N", [(2, 1, 20), (4, 2, 30), (12, 4, 40), (1, 1, 9), (3, 2, 12),
                                     (8, 4, 8), (4, 1, 25)])
@pytest.mark.parametrize("outs", list(OUTPUT_SETS))
@pytest.mark.parametrize("drift", [False, True])
def test_condense_fp32(dev, nx, nu, N, outs, drift):
    rng = np.random.default_rng(7 + nx)
    batch = 4
    A, B, Q, R, Qf = _rand_plant(rng, nx, nu, N, True, batch)
    A *= 0.8
    x0 = rng.normal(size=(batch, nx))
    c = rng.normal(size=(batch, N, nx)) * 0.3 if drift else None
    out = _condense_set(dev, torch.float32, A, B, Q, R, Qf, N, x0, c, True, outs)
    A32, B32 = A.astype(np.float32).astype(np.float64), B.astype(np.float32).astype(np.float64)
    ref = [oc.condense(A32[b], B32[b], Q, R, Qf, N, x0=x0[b], c=None if c is None else c[b])
           for b in range(batch)]
    _check(out, ref, N * nu, 2e-5)


@pytest.mark.parametrize("tv", [True, False])
def test_condense_fh_operand_at_allocation_end(dev, tv):
    """condense_mfma_fh_kernel's X3 path (nx % 3 == 0, config 5's nx = 12) loads
    rows of A as 12-byte vectors: with A ending exactly at the end of its
    allocation (and shared, stride 0, when not tv) the last instance's last
    row must read no further than A's last element."""
    rng = np.random.default_rng(91 + tv)
    nx, nu, N, batch = 12, 4, 8, 3
    A, B, Q, R, Qf = _rand_plant(rng, nx, nu, N, True, batch)
    A = A * 0.8 if tv else A[0, 0] * 0.8
    x0 = rng.normal(size=(batch, nx))
    f32 = torch.float32
    numel = A.size
    # a block of whole 512-byte allocator units whose last element is A's last
    total = -(-numel * 4 // 512) * 512 // 4
    buf = torch.zeros(total, dtype=f32, device=dev)
    At = buf[total - numel:].view(A.shape)
    At.copy_(torch.as_tensor(A, dtype=f32))
    Bt = _t(B if tv else B[0, 0], dev, f32)
    out = batched.condense(At, Bt, _t(Q, dev, f32), _t(R, dev, f32), _t(Qf, dev, f32), N,
                           x0=_t(x0, dev, f32), tv=tv, outputs=("H", "f"))
    torch.cuda.synchronize()
    A32 = A.astype(np.float32).astype(np.float64)
    B32 = B.astype(np.float32).astype(np.float64)
    ref = [oc.condense(A32[b] if tv else A32, B32[b] if tv else B32[0, 0], Q, R, Qf, N, x0=x0[b])
           for b in range(batch)]
    _check({k: v.double() for k, v in out.items()}, ref, N * nu, 2e-5)


def test_condense_large_batch_pointwise(dev):
    """Config-2 shape at the bench batch: spot-check instances against the oracle."""
    A, B, Q, R, Pf, _ = s1.fhc_setup()
    R = R.reshape(1, 1)
    N, batch = 20, 4096
    rng = np.random.default_rng(20261017)
    X0 = rng.uniform(-10, 10, (batch, 2))
    Ab = np.broadcast_to(A, (batch, 2, 2))
    Bb = np.broadcast_to(B, (batch, 2, 1))
    out = batched.condense(_t(Ab, dev), _t(Bb, dev), _t(Q, dev), _t(R, dev), _t(Pf, dev), N,
                           x0=_t(X0, dev), outputs=("H", "f"))
    H0 = out["H"][0]
    # identical plants -> identical H for every instance (bitwise)
    assert torch.equal(out["H"], H0.expand_as(out["H"]))
    for b in (0, 1, 777, 4095):
        ref = oc.condense(A, B, Q, R, Pf, N, x0=X0[b])
        assert np.abs(out["f"][b].cpu().numpy() - ref["f"]).max() < 1e-10 * max(1, np.abs(ref["f"]).max())


@pytest.mark.parametrize("nx,nu,N,tv", [(5, 3, 6, True), (8, 2, 10, True), (12, 4, 40, True),
                                        (15, 1, 9, True), (12, 6, 20, True), (6, 12, 10, True),
                                        (12, 4, 40, False), (7, 16, 16, True), (12, 4, 7, True),
                                        (9, 1, 33, True)])
@pytest.mark.parametrize("drift", [True, False])
@pytest.mark.parametrize("outs", [("H", "F", "f", "Gam", "Phi", "xbar"), ("H", "f", "Gam", "xbar"),
                                  ("H", "f")])
def test_condense_fp32_mfma_all_outputs(dev, nx, nu, N, tv, drift, outs):
    """fp32 with 5 <= nx <= 15 runs condense_mfma_kernel (augmented-state
    MFMA recursion; per-stage drift c_k; the x0 columns F, Phi) or, without
    drift, F and Phi for nx <= 12 and nu <= 4, condense_mfma_fh_kernel (H rows
    from the forward MFMA's free state slots, f and xbar from a VALU mat-vec):
    every requested output vs the fp64 oracle."""
    rng = np.random.default_rng(31 + 7 * nx + nu + N)
    batch = 3
    A, B, Q, R, Qf = _rand_plant(rng, nx, nu, N, tv, batch)
    A *= 0.8
    x0 = rng.normal(size=(batch, nx))
    c = rng.normal(size=(batch, N, nx)) * 0.3 if (tv and drift) else None
    f32 = torch.float32
    out = batched.condense(_t(A, dev, f32), _t(B, dev, f32), _t(Q, dev, f32), _t(R, dev, f32),
                           _t(Qf, dev, f32), N, x0=_t(x0, dev, f32),
                           c=None if c is None else _t(c, dev, f32), tv=tv,
                           outputs=outs)
    torch.cuda.synchronize()
    A32, B32 = A.astype(np.float32).astype(np.float64), B.astype(np.float32).astype(np.float64)
    ref = [oc.condense(A32[b], B32[b], Q, R, Qf, N, x0=x0[b], c=None if c is None else c[b])
           for b in range(batch)]
    out = {k: v.double() for k, v in out.items()}
    _check(out, ref, N * nu, 2e-5)


@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
@pytest.mark.parametrize("off", [1, 2, 3])
def test_condense_streamed_outputs_misaligned(dev, dt, off):
    """The streamed sweep (n <= 64) writes H and Gamma as 16-byte vectors from an LDS ring,
    with the stream start aligned down; outputs placed `off` elements past a 16-byte boundary
    must come out identical to aligned ones, and nothing outside them may be written."""
    rng = np.random.default_rng(31 + off)
    nx, nu, N, batch = 4, 2, 30, 7
    A, B, Q, R, Qf = _rand_plant(rng, nx, nu, N, True, batch)
    x0 = rng.normal(size=(batch, nx))
    c = rng.normal(size=(batch, N, nx))
    args = (_t(A, dev, dt), _t(B, dev, dt), _t(Q, dev, dt), _t(R, dev, dt), _t(Qf, dev, dt), N)
    kw = dict(x0=_t(x0, dev, dt), c=_t(c, dev, dt), tv=True, outputs=("H", "f", "Gam", "xbar"))
    ref = batched.condense(*args, **kw)
    n = N * nu
    shapes = {"H": (batch, n * (n + 1) // 2), "f": (batch, n), "Gam": (batch, N * nx, n),
              "xbar": (batch, N, nx)}
    bufs, out = {}, {}
    for k, shp in shapes.items():
        numel = int(np.prod(shp))
        bufs[k] = torch.full((numel + off + 8,), 7.0, dtype=dt, device=dev)
        out[k] = bufs[k][off:off + numel].view(shp)
    got = batched.condense(*args, **kw, out=out)
    torch.cuda.synchronize()
    for k in shapes:
        assert torch.equal(got[k].reshape(-1), ref[k].reshape(-1)), k
        assert bool((bufs[k][:off] == 7.0).all()) and bool((bufs[k][off + got[k].numel():] == 7.0).all()), k
    o = oc.condense(A[0], B[0], Q, R, Qf, N, x0=x0[0], c=c[0])
    Hd = batched.unpack_lower(got["H"].double(), n).cpu().numpy()[0]
    tol = 1e-10 if dt == torch.float64 else 2e-5
    assert np.abs(Hd - o["H"]).max() <= tol * max(1.0, np.abs(o["H"]).max())


@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
@pytest.mark.parametrize("nx,nu,N,off", [(4, 2, 30, 0), (4, 2, 30, 3), (2, 1, 20, 1), (3, 2, 7, 2),
                                         (6, 2, 10, 0), (4, 3, 40, 1)])
def test_condense_gam_packed(dev, dt, nx, nu, N, off):
    """MPCQP_GAM_PACKED: Gamma's lower block triangle only (SURVEY 8(d)'s output list).
    Streamed (n <= 64) and direct sweeps, misaligned starts, an nx that would take the
    MFMA kernel in fp32 (it runs on the wavefront kernel): the packed stream equals the
    dense call's lower block triangle bit for bit, matches the explicit oracle, and
    nothing outside it is written."""
    rng = np.random.default_rng(700 + 10 * nx + N + off)
    batch = 5
    A, B, Q, R, Qf = _rand_plant(rng, nx, nu, N, True, batch)
    x0 = rng.normal(size=(batch, nx))
    c = rng.normal(size=(batch, N, nx))
    args = (_t(A, dev, dt), _t(B, dev, dt), _t(Q, dev, dt), _t(R, dev, dt), _t(Qf, dev, dt), N)
    kw = dict(x0=_t(x0, dev, dt), c=_t(c, dev, dt), tv=True, outputs=("H", "f", "Gam"))
    dense = batched.condense(*args, **kw)
    numel = batch * nx * nu * N * (N + 1) // 2
    buf = torch.full((numel + off + 8,), 7.0, dtype=dt, device=dev)
    pk = buf[off:off + numel].view(batch, -1)
    got = batched.condense(*args, **kw, out={"Gam": pk}, gam_packed=True)
    torch.cuda.synchronize()
    assert bool((buf[:off] == 7.0).all()) and bool((buf[off + numel:] == 7.0).all())
    G = batched.unpack_gam(got["Gam"], N, nx, nu)
    tol = 1e-10 if dt == torch.float64 else 2e-5
    if dt == torch.float32 and 5 <= nx <= 15:
        # the dense fp32 call ran on the MFMA kernel: same values up to rounding
        for k, v in (("H", got["H"]), ("f", got["f"]), ("Gam", G)):
            s = max(1.0, float(dense[k].abs().max()))
            assert float((v - dense[k]).abs().max()) <= tol * s, k
    else:
        # same recursion for H and Gamma; f comes from the affine lane (y = W xbar + eta)
        # here and from the adjoint chain on the dense call's kernel: equal up to rounding
        assert torch.equal(got["H"], dense["H"])
        assert torch.equal(G, dense["Gam"])  # the upper block triangle of the dense call is 0
        s = max(1.0, float(dense["f"].abs().max()))
        assert float((got["f"] - dense["f"]).abs().max()) <= tol * s
    for b in range(batch):
        o = oc.condense(A[b], B[b], Q, R, Qf, N, x0=x0[b], c=c[b])
        g = G[b].double().cpu().numpy()
        assert np.abs(g - o["Gam"]).max() <= tol * max(1.0, np.abs(o["Gam"]).max())
        f = got["f"][b].double().cpu().numpy()
        assert np.abs(f - o["f"]).max() <= tol * max(1.0, np.abs(o["f"]).max())
