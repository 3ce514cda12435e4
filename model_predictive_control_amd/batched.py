"""Batched device API over libmpcqp (torch tensors on the GPU).

This is the layer the reference-shaped surfaces (``fhc``, ``linear_system``,
``session1``, ``mpc``) and ``bench.py`` call.  Every function enqueues HIP
kernels on torch's current stream through the C ABI of include/mpcqp.h; no
computation happens on the host.

Shape conventions (batch-outermost, row-major):

* a per-instance input carries a leading batch dimension, a shared input
  does not (it is passed with stride 0);
* ``z`` is stage-major  [u_0; ...; u_{N-1}]  (session_4/main.py:46,110);
* symmetric matrices (H) are packed lower, n(n+1)/2 per instance
  (``pack_lower`` / ``unpack_lower`` convert).
"""
from __future__ import annotations

import ctypes

import math

import torch

from . import _native as nat

__all__ = [
    "condense", "solve_box", "mpc_box", "mpc_box_loop", "mpc_qp", "mpc_ipm", "solve_poly", "solve_qp", "sweep", "riccati", "gemv",
    "rollout", "bicycle_rti", "bicycle_linearise", "bicycle_hessian", "bicycle_sqp_step",
    "pack_lower", "unpack_lower", "status_code", "status_iters", "workspace_bytes",
]


def _lib():
    return nat.load()


def _code(dtype: torch.dtype) -> int:
    if dtype == torch.float64:
        return nat.F64
    if dtype == torch.float32:
        return nat.F32
    raise TypeError(f"libmpcqp supports float64/float32, got {dtype}")


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t):
    return None if t is None else t.data_ptr()


_WS: dict = {}


def _workspace(nbytes: int, dev, ws: torch.Tensor | None = None) -> torch.Tensor | None:
    """Device scratch of the two-kernel QP path (swept matrix, s0, hand-off
    counter and list).

    * ``ws`` given: the caller's buffer is used as is (checked for size).
    * inside a HIP-graph capture: a fresh buffer, which the graph's private
      pool keeps for the graph's lifetime; never a cached one, so a later
      resize of the cache cannot pull memory out from under a captured graph.
    * otherwise: one grow-only buffer per (device, stream).  Kernels on one
      stream run in order, so solves on the same stream may share it; solves
      on different streams get different buffers.  Growing drops the smaller
      buffer (the caching allocator reuses it stream-ordered on that stream).
    """
    if nbytes <= 0:
        return None
    if ws is not None:
        if ws.device.type != "cuda" or ws.numel() * ws.element_size() < nbytes:
            raise ValueError(f"workspace must be a device buffer of >= {nbytes} bytes")
        return ws
    if torch.cuda.is_current_stream_capturing():
        return torch.empty((int(nbytes),), dtype=torch.uint8, device=dev)
    key = (str(dev), torch.cuda.current_stream(dev).cuda_stream)
    buf = _WS.get(key)
    if buf is None or buf.numel() < nbytes:
        _WS.pop(key, None)
        buf = _WS[key] = torch.empty((int(nbytes),), dtype=torch.uint8, device=dev)
    return buf


def workspace_bytes(dtype: torch.dtype, batch: int, n: int, m: int = 0) -> int:
    """Bytes of the ``ws=`` buffer solve_box (m = 0) / solve_qp need."""
    return int(_lib().mpcqp_solve_qp_workspace(_code(dtype), batch, n, m))


def _dev(x, dtype, device):
    if x is None:
        return None
    t = torch.as_tensor(x, dtype=dtype, device=device)
    if t.device.type != "cuda":
        raise ValueError("libmpcqp needs CUDA(HIP) tensors")
    return t.contiguous()


def _inst(t, base_ndim: int, name: str):
    """(stride, batch) of an input that is shared (ndim == base) or batched."""
    if t is None:
        return 0, None
    if t.ndim == base_ndim:
        return 0, None
    if t.ndim == base_ndim + 1:
        return int(t[0].numel()), int(t.shape[0])
    raise ValueError(f"{name}: expected {base_ndim} or {base_ndim + 1} dims, got {tuple(t.shape)}")


def _batch_of(*pairs):
    bs = {b for _, b in pairs if b is not None}
    if len(bs) > 1:
        raise ValueError(f"inconsistent batch sizes {sorted(bs)}")
    return bs.pop() if bs else 1


def status_code(status: torch.Tensor) -> torch.Tensor:
    return status & 0xFF


def status_iters(status: torch.Tensor) -> torch.Tensor:
    return (status >> 8) & 0xFFFF


# ----------------------------------------------------------------- packing
def _tril_index(n: int, device) -> tuple[torch.Tensor, torch.Tensor]:
    r, c = torch.tril_indices(n, n, device=device)
    return r, c


def pack_lower(H: torch.Tensor) -> torch.Tensor:
    """(..., n, n) symmetric -> (..., n(n+1)/2) row-major packed lower."""
    n = H.shape[-1]
    r, c = _tril_index(n, H.device)
    return H[..., r, c].contiguous()


def unpack_lower(P: torch.Tensor, n: int) -> torch.Tensor:
    """(..., n(n+1)/2) packed lower -> (..., n, n) symmetric."""
    r, c = _tril_index(n, P.device)
    out = P.new_zeros(P.shape[:-1] + (n, n))
    out[..., r, c] = P
    out[..., c, r] = P
    return out


# ---------------------------------------------------------------- condense
def condense(A, B, Q, R, Qf, N: int, x0=None, c=None, *, tv: bool = False,
             outputs=("H", "f"), out: dict | None = None, gam_packed: bool = False) -> dict:
    """Batched condensing (include/mpcqp.h ``mpcqp_condense``).

    A: (nx,nx) | (b,nx,nx) | with ``tv``: (N,nx,nx) | (b,N,nx,nx); B likewise
    with nu columns; Q/Qf (nx,nx) | (b,nx,nx); R (nu,nu) | (b,nu,nu);
    x0 (nx,) | (b,nx); c (N,nx) | (b,N,nx).  Returns a dict with the requested
    ``outputs`` among H (packed), F, f, Gam, Phi, xbar.  ``gam_packed``: Gam
    as its lower block triangle, (b, nx*nu*N*(N+1)/2) (``MPCQP_GAM_PACKED``;
    ``unpack_gam`` restores the dense (b, N*nx, N*nu) form).
    """
    dt = A.dtype if isinstance(A, torch.Tensor) else torch.float64
    dev = A.device if isinstance(A, torch.Tensor) else torch.device("cuda")
    A, B, Q, R, Qf = (_dev(v, dt, dev) for v in (A, B, Q, R, Qf))
    x0, c = _dev(x0, dt, dev), _dev(c, dt, dev)
    nx, nu = int(B.shape[-2]), int(B.shape[-1])
    R = _weight_r(R, nu)
    base = 3 if tv else 2
    sA, bA = _inst(A, base, "A")
    sB, bB = _inst(B, base, "B")
    sQ, bQ = _inst(Q, 2, "Q")
    sR, bR = _inst(R, 2, "R")
    sQf, bQf = _inst(Qf, 2, "Qf")
    sC, bC = _inst(c, 2, "c")
    sX, bX = _inst(x0, 1, "x0")
    batch = _batch_of((sA, bA), (sB, bB), (sQ, bQ), (sR, bR), (sQf, bQf), (sC, bC), (sX, bX))
    n = N * nu
    want = set(outputs) | {"H"}
    out = dict(out or {})
    shapes = {"H": (batch, n * (n + 1) // 2), "F": (batch, n, nx), "f": (batch, n),
              "Gam": (batch, nx * nu * N * (N + 1) // 2) if gam_packed else (batch, N * nx, n), "Phi": (batch, N * nx, nx), "xbar": (batch, N * nx)}
    for k in want:
        if k not in out:
            out[k] = torch.empty(shapes[k], dtype=dt, device=dev)
    rc = _lib().mpcqp_condense(
        _code(dt), batch, nx, nu, N, (nat.TV if tv else 0) | (nat.GAM_PACKED if gam_packed else 0),
        _ptr(A), sA, _ptr(B), sB, _ptr(Q), sQ, _ptr(R), sR, _ptr(Qf), sQf, _ptr(c), sC,
        _ptr(x0), sX, _ptr(out.get("H")), _ptr(out.get("F")), _ptr(out.get("f")),
        _ptr(out.get("Gam")), _ptr(out.get("Phi")), _ptr(out.get("xbar")), _stream())
    nat.check(rc, "mpcqp_condense")
    return {k: out[k] for k in want}


def unpack_gam(P, N: int, nx: int, nu: int):
    """Dense (..., N*nx, N*nu) Gamma from its packed lower block triangle
    (``condense(..., gam_packed=True)``): block row k holds its (k+1)*nu
    leading columns from offset nx*nu*k*(k+1)/2, column by column (entry
    (k*nx + q, col) at nx*nu*k*(k+1)/2 + col*nx + q)."""
    out = P.new_zeros(P.shape[:-1] + (N * nx, N * nu))
    for k in range(N):
        o, w = nx * nu * k * (k + 1) // 2, (k + 1) * nu
        out[..., k * nx:(k + 1) * nx, :w] = P[..., o:o + nx * w].reshape(P.shape[:-1] + (w, nx)).transpose(-1, -2)
    return out


# ---------------------------------------------------- fused condense + box
def mpc_box(A, B, Q, R, Qf, N: int, x0, lb=None, ub=None, c=None, *, tv: bool = False,
            max_iter: int = 0, tol: float = 0.0, out: tuple | None = None):
    """Fused per-instance condense + input-box QP (include/mpcqp.h
    ``mpcqp_mpc_box``).  Same plant conventions as ``condense``; lb/ub are
    scalars, (N*nu,) shared or (b, N*nu).  Returns (z (b, N*nu), status)."""
    dt = A.dtype if isinstance(A, torch.Tensor) else torch.float64
    dev = A.device if isinstance(A, torch.Tensor) else torch.device("cuda")
    A, B, Q, R, Qf = (_dev(v, dt, dev) for v in (A, B, Q, R, Qf))
    x0, c = _dev(x0, dt, dev), _dev(c, dt, dev)
    nx, nu = int(B.shape[-2]), int(B.shape[-1])
    R = _weight_r(R, nu)
    n = N * nu
    base = 3 if tv else 2
    sA, bA = _inst(A, base, "A")
    sB, bB = _inst(B, base, "B")
    sQ, bQ = _inst(Q, 2, "Q")
    sR, bR = _inst(R, 2, "R")
    sQf, bQf = _inst(Qf, 2, "Qf")
    sC, bC = _inst(c, 2, "c")
    sX, bX = _inst(x0, 1, "x0")
    lbt, slb = _bound(lb, n, dt, dev)
    ubt, sub = _bound(ub, n, dt, dev)
    batch = _batch_of((sA, bA), (sB, bB), (sQ, bQ), (sR, bR), (sQf, bQf), (sC, bC), (sX, bX),
                      (slb, lbt.shape[0] if lbt is not None and lbt.ndim == 2 else None),
                      (sub, ubt.shape[0] if ubt is not None and ubt.ndim == 2 else None))
    if out is None:
        z = torch.empty((batch, n), dtype=dt, device=dev)
        status = torch.empty((batch,), dtype=torch.int32, device=dev)
    else:
        z, status = out
    rc = _lib().mpcqp_mpc_box(
        _code(dt), batch, nx, nu, N, nat.TV if tv else 0,
        _ptr(A), sA, _ptr(B), sB, _ptr(Q), sQ, _ptr(R), sR, _ptr(Qf), sQf, _ptr(c), sC,
        _ptr(x0), sX, _ptr(lbt), slb, _ptr(ubt), sub, _ptr(z), _ptr(status), int(max_iter),
        float(tol), _stream())
    nat.check(rc, "mpcqp_mpc_box")
    return z, status


# --------------------------------------- fused condense + state/input box
def mpc_qp_workspace_bytes(dtype: torch.dtype, batch: int, nx: int, nu: int, N: int,
                           state_box: bool = True) -> int:
    """Bytes of the ``ws=`` buffer ``mpc_qp`` needs."""
    return int(_lib().mpcqp_mpc_qp_workspace(_code(dtype), batch, nx, nu, N, int(bool(state_box))))


def _mpc_step_args(A, B, Q, R, Qf, N, x0, xlo, xhi, lb, ub, c, tv):
    """Normalise the arguments shared by mpc_qp / mpc_ipm (plant conventions
    of ``condense``; state bounds (nx,) repeated over the horizon, (N*nx,)
    shared or (b, N*nx); input bounds as ``mpc_box``)."""
    dt = A.dtype if isinstance(A, torch.Tensor) else torch.float64
    dev = A.device if isinstance(A, torch.Tensor) else torch.device("cuda")
    A, B, Q, R, Qf = (_dev(v, dt, dev) for v in (A, B, Q, R, Qf))
    x0, c = _dev(x0, dt, dev), _dev(c, dt, dev)
    nx, nu = int(B.shape[-2]), int(B.shape[-1])
    R = _weight_r(R, nu)
    n, m = N * nu, N * nx
    base = 3 if tv else 2
    sA, bA = _inst(A, base, "A")
    sB, bB = _inst(B, base, "B")
    sQ, bQ = _inst(Q, 2, "Q")
    sR, bR = _inst(R, 2, "R")
    sQf, bQf = _inst(Qf, 2, "Qf")
    sC, bC = _inst(c, 2, "c")
    sX, bX = _inst(x0, 1, "x0")

    def sbound(v):
        if v is None:
            return None, 0, None
        t = _dev(v, dt, dev)
        if t.ndim == 1 and t.shape[0] == nx and nx != m:
            t = t.repeat(N)
        s, bb = _inst(t, 1, "state bound")
        if t.shape[-1] != m:
            raise ValueError(f"state bounds need {m} (= N*nx) entries, got {tuple(t.shape)}")
        return t, s, bb

    xlo_t, sxl, bxl = sbound(xlo)
    xhi_t, sxh, bxh = sbound(xhi)
    if xlo_t is not None and xhi_t is not None and sxl != sxh:
        raise ValueError("xlo and xhi must both be shared or both per instance")
    sXb = max(sxl, sxh)
    lbt, slb = _bound(lb, n, dt, dev)
    ubt, sub = _bound(ub, n, dt, dev)
    batch = _batch_of((sA, bA), (sB, bB), (sQ, bQ), (sR, bR), (sQf, bQf), (sC, bC), (sX, bX),
                      (sxl, bxl), (sxh, bxh),
                      (slb, lbt.shape[0] if lbt is not None and lbt.ndim == 2 else None),
                      (sub, ubt.shape[0] if ubt is not None and ubt.ndim == 2 else None))
    return dict(dt=dt, dev=dev, nx=nx, nu=nu, n=n, m=m, batch=batch,
                head=(_ptr(A), sA, _ptr(B), sB, _ptr(Q), sQ, _ptr(R), sR, _ptr(Qf), sQf,
                      _ptr(c), sC, _ptr(x0), sX, _ptr(xlo_t), _ptr(xhi_t), sXb,
                      _ptr(lbt), slb, _ptr(ubt), sub),
                keep=(A, B, Q, R, Qf, c, x0, xlo_t, xhi_t, lbt, ubt),
                sbox=xlo_t is not None or xhi_t is not None)


def mpc_qp(A, B, Q, R, Qf, N: int, x0, xlo=None, xhi=None, lb=None, ub=None, c=None, *,
           tv: bool = False, states: bool = False, max_iter: int = 0, tol: float = 0.0,
           out: tuple | None = None, ws: torch.Tensor | None = None, ipm: bool = False):
    """One MPC step with input box and state box, end to end (include/mpcqp.h
    ``mpcqp_mpc_qp``): condense + QP, fp32 refined against the dynamics.
    Steps beyond the dense kernels' size (and every step with ``ipm=True``)
    run on the stage-wise interior point (``mpc_ipm``).

    Plant conventions as ``condense``; xlo/xhi: state bounds on x_1..x_N,
    (nx,) repeated over the horizon, (N*nx,) shared or (b, N*nx); lb/ub as
    ``mpc_box``.  Returns (z (b, N*nu), y (b, N*nx) or None, status[, X
    (b, N, nx) when ``states``]); y are the state-row multipliers (> 0 at xhi).
    """
    g = _mpc_step_args(A, B, Q, R, Qf, N, x0, xlo, xhi, lb, ub, c, tv)
    dt, dev, batch, n, m, nx = g["dt"], g["dev"], g["batch"], g["n"], g["m"], g["nx"]
    sbox = g["sbox"]
    if out is None:
        z = torch.empty((batch, n), dtype=dt, device=dev)
        y = torch.empty((batch, m), dtype=dt, device=dev) if sbox else None
        status = torch.empty((batch,), dtype=torch.int32, device=dev)
        X = torch.empty((batch, N, nx), dtype=dt, device=dev) if states else None
    else:
        z, y, status = out[:3]
        X = out[3] if len(out) > 3 else None
    lib = _lib()
    wsb = int(lib.mpcqp_mpc_qp_workspace(_code(dt), batch, nx, g["nu"], N, int(sbox)))
    ws = _workspace(wsb, dev, ws)
    flags = (nat.TV if tv else 0) | (nat.IPM if ipm else 0)
    rc = lib.mpcqp_mpc_qp(_code(dt), batch, nx, g["nu"], N, flags, *g["head"],
                          _ptr(z), _ptr(y), _ptr(X), _ptr(status), int(max_iter), float(tol),
                          _ptr(ws), wsb, _stream())
    nat.check(rc, "mpcqp_mpc_qp")
    return (z, y, status, X) if states else (z, y, status)


def mpc_ipm(A, B, Q, R, Qf, N: int, x0, xlo=None, xhi=None, lb=None, ub=None, c=None, *,
            tv: bool = False, U0=None, H2=None, q2=None, max_iter: int = 0, tol: float = 0.0,
            strict: bool = False, skip=None, skip_mask: int = 0, out: dict | None = None,
            ws: torch.Tensor | None = None):
    """The MPC step of ``mpc_qp`` on the stage-wise interior point, any horizon
    (include/mpcqp.h ``mpcqp_mpc_ipm``; nx <= 4, nu <= 2).  U0: optional
    starting inputs (b, N, nu) or (b, N*nu).  H2 (b, N, nx+nu, nx+nu), q2
    (b, N, nx+nu): optional extra stage cost 1/2 w'H2 w + q2'w over
    w = [x_k; u_k] (may be indefinite).  Returns a dict with z (b, N*nu),
    X (b, N, nx) = x_1..x_N, y (b, N*nx) state-bound and lam_u (b, N*nu)
    input-bound multipliers (> 0 at the upper bound), pi (b, N, nx) costates
    of the dynamics, status (b,).  ``strict``: a non-positive pivot ends an
    instance with STATUS_NOT_CONVEX instead of regularising.  ``skip`` (b,)
    int32 with ``skip_mask``: instances with skip & skip_mask != 0 are left
    untouched.  ``out``: a dict of preallocated outputs."""
    g = _mpc_step_args(A, B, Q, R, Qf, N, x0, xlo, xhi, lb, ub, c, tv)
    dt, dev, batch, n, m, nx = g["dt"], g["dev"], g["batch"], g["n"], g["m"], g["nx"]
    U0t = None if U0 is None else _dev(U0, dt, dev).reshape(batch, n)
    n2 = nx + g["nu"]
    H2t = None if H2 is None else _dev(H2, dt, dev).reshape(batch, N * n2 * n2)
    q2t = None if q2 is None else _dev(q2, dt, dev).reshape(batch, N * n2)
    o = dict(out or {})
    shapes = dict(z=((batch, n), dt), y=((batch, m), dt), lam_u=((batch, n), dt),
                  X=((batch, N, nx), dt), pi=((batch, N, nx), dt), status=((batch,), torch.int32))
    for k, (shp, kd) in shapes.items():
        if k not in o:
            o[k] = torch.empty(shp, dtype=kd, device=dev)
    lib = _lib()
    wsb = int(lib.mpcqp_mpc_ipm_workspace(_code(dt), batch, nx, g["nu"], N))
    ws = _workspace(wsb, dev, ws)
    if skip is not None and (skip.dtype != torch.int32 or skip.shape != (batch,)
                             or skip.device != dev):
        raise ValueError("skip must be an int32 device tensor of shape (batch,)")
    flags = (nat.TV if tv else 0) | (nat.STRICT if strict else 0)
    rc = lib.mpcqp_mpc_ipm(_code(dt), batch, nx, g["nu"], N, flags, *g["head"],
                           _ptr(U0t), 0 if U0t is None else n, _ptr(H2t),
                           0 if H2t is None else N * n2 * n2, _ptr(q2t),
                           0 if q2t is None else N * n2, _ptr(o["z"]), _ptr(o["y"]), _ptr(o["X"]),
                           _ptr(o["lam_u"]), _ptr(o["pi"]), _ptr(o["status"]), _ptr(skip),
                           int(skip_mask) if skip is not None else 0, int(max_iter),
                           float(tol), _ptr(ws), wsb, _stream())
    nat.check(rc, "mpcqp_mpc_ipm")
    return o


def mpc_box_loop(A, B, Q, R, Qf, N: int, x0, lb=None, ub=None, steps: int = 1, *,
                 plans: bool = False, max_iter: int = 0, tol: float = 0.0,
                 condensed: dict | None = None, out: dict | None = None) -> dict:
    """The receding-horizon loop of the input-box MPC on a linear plant, on
    the device (include/mpcqp.h ``mpcqp_mpc_box_loop``): for t < steps,
    z_t = argmin 1/2 z'Hz + (F x_t)'z over lb <= z <= ub, x_{t+1} = A x_t + B
    u_0(z_t) -- LinearSystem.simulate (LinearSystem.py:20-26) under the MPC
    policy of MPCController.solve (main.py:115-116).  A (nx,nx) | (b,nx,nx), B
    likewise; x0 (b, nx).  H and F come from ``condense`` of the same plant
    (once; pass ``condensed`` to reuse them).  Returns xs (steps+1, b, nx), us
    (steps, b, nu), status (steps, b), and with ``plans`` zs (steps, b, N*nu)."""
    dt = A.dtype if isinstance(A, torch.Tensor) else torch.float64
    dev = A.device if isinstance(A, torch.Tensor) else torch.device("cuda")
    A, B = _dev(A, dt, dev), _dev(B, dt, dev)
    x0 = _dev(x0, dt, dev)
    nx, nu = int(B.shape[-2]), int(B.shape[-1])
    if x0.ndim != 2 or x0.shape[1] != nx:
        raise ValueError(f"x0 must be (batch, {nx}), got {tuple(x0.shape)}")
    batch, n, T = int(x0.shape[0]), N * nu, int(steps)
    cd = condensed or condense(A, B, Q, R, Qf, N, outputs=("H", "F"))
    H, F = cd["H"], cd["F"]
    sH, _ = _inst(H, 1, "H")
    sF, _ = _inst(F, 2, "F")
    if H.ndim == 2 and H.shape[0] == 1:   # a shared plant condenses to one instance
        sH = 0
    if F.ndim == 3 and F.shape[0] == 1:
        sF = 0
    sA, _ = _inst(A, 2, "A")
    sB, _ = _inst(B, 2, "B")
    lbt, slb = _bound(lb, n, dt, dev)
    ubt, sub = _bound(ub, n, dt, dev)
    o = dict(out or {})
    shapes = dict(xs=((T + 1, batch, nx), dt), us=((T, batch, nu), dt),
                  status=((T, batch), torch.int32))
    if plans:
        shapes["zs"] = ((T, batch, n), dt)
    for k, (shp, kd) in shapes.items():
        if k not in o:
            o[k] = torch.empty(shp, dtype=kd, device=dev)
    rc = _lib().mpcqp_mpc_box_loop(_code(dt), batch, nx, nu, N, T, _ptr(H), sH, _ptr(F), sF,
                                   _ptr(A), sA, _ptr(B), sB, _ptr(x0), nx, _ptr(lbt), slb,
                                   _ptr(ubt), sub, _ptr(o["xs"]), _ptr(o["us"]), _ptr(o.get("zs")),
                                   _ptr(o["status"]), int(max_iter), float(tol), _stream())
    nat.check(rc, "mpcqp_mpc_box_loop")
    return o


def _weight_r(R, nu: int):
    """R as (nu, nu) (or batched).  FHC.py:141 passes R with shape (1,), which
    NumPy broadcasts; a 1-D R is accepted only for nu == 1 (shape (1,)) -- a
    vector of diagonal weights must be given as a matrix (torch.diag)."""
    if R.ndim == 1:
        if R.shape[0] != 1 or nu != 1:
            raise ValueError(f"R of shape {tuple(R.shape)} with nu={nu}: pass an (nu, nu) matrix")
        return R.reshape(1, 1).contiguous()
    return R


# ----------------------------------------------------------------- box QP
def _bound(v, n, dt, dev):
    if v is None:
        return None, 0
    if not isinstance(v, torch.Tensor) and (isinstance(v, (int, float))):
        return torch.full((n,), float(v), dtype=dt, device=dev), 0
    t = _dev(v, dt, dev)
    if t.ndim == 0:
        return t.expand(n).contiguous(), 0
    s, _ = _inst(t, 1, "bound")
    return t, s


def solve_box(H, f, lb=None, ub=None, *, max_iter: int = 0, tol: float = 0.0,
              out: tuple | None = None, presweep: bool = True, ws: torch.Tensor | None = None):
    """Batched  min 1/2 z'Hz + f'z  s.t.  lb <= z <= ub.  Returns (z, status).
    ``ws``: optional caller-owned scratch (``workspace_bytes(dtype, batch, n)``).

    fp32 with n > 64: the -H^-1 sweep runs first as its own MFMA kernel
    (``mpcqp_solve_box_ws``) unless ``presweep=False``."""
    dt, dev = f.dtype, f.device
    f = _dev(f, dt, dev)
    H = _dev(H, dt, dev)
    n = int(f.shape[-1])
    if H.shape[-1] != n * (n + 1) // 2:
        raise ValueError(f"H must be packed lower with {n * (n + 1) // 2} entries, got {tuple(H.shape)}")
    sH, bH = _inst(H, 1, "H")
    sf, bf = _inst(f, 1, "f")
    lbt, slb = _bound(lb, n, dt, dev)
    ubt, sub = _bound(ub, n, dt, dev)
    batch = _batch_of((sH, bH), (sf, bf),
                      (slb, lbt.shape[0] if lbt is not None and lbt.ndim == 2 else None),
                      (sub, ubt.shape[0] if ubt is not None and ubt.ndim == 2 else None))
    if out is None:
        z = torch.empty((batch, n), dtype=dt, device=dev)
        status = torch.empty((batch,), dtype=torch.int32, device=dev)
    else:
        z, status = out
    lib = _lib()
    wsb = int(lib.mpcqp_solve_qp_workspace(_code(dt), batch, n, 0)) if presweep else 0
    ws = _workspace(wsb, dev, ws)
    rc = lib.mpcqp_solve_box_ws(_code(dt), batch, n, _ptr(H), sH, _ptr(f), sf, _ptr(lbt), slb,
                                _ptr(ubt), sub, _ptr(z), _ptr(status), int(max_iter), float(tol),
                                _ptr(ws), wsb, _stream())
    nat.check(rc, "mpcqp_solve_box_ws")
    return z, status


# ------------------------------------------------------------- polytope QP
def solve_poly(H, f, G=None, hl=None, hu=None, lbz=None, ubz=None, *, max_iter: int = 0,
               tol: float = 0.0):
    """Batched  min 1/2 z'Hz + f'z  s.t.  hl <= G z <= hu,  lbz <= z <= ubz.

    H (packed, shared) and G (m, n) shared; f, hl, hu per instance or shared.
    Returns (z, y, status); y are the multipliers of the rows [G; I].
    """
    dt, dev = f.dtype, f.device
    f = _dev(f, dt, dev)
    H = _dev(H, dt, dev)
    n = int(f.shape[-1])
    if H.ndim != 1:
        raise ValueError("solve_poly: H must be shared (packed, 1-D)")
    m = 0 if G is None else int(G.shape[0])
    G = _dev(G, dt, dev)
    sf, bf = _inst(f, 1, "f")
    hl = _dev(hl, dt, dev)
    hu = _dev(hu, dt, dev)
    sh, bh = 0, None
    for h in (hl, hu):
        if h is not None:
            s, b = _inst(h, 1, "h")
            sh, bh = max(sh, s), b if b is not None else bh
    if hl is not None and hu is not None and hl.shape != hu.shape:
        raise ValueError("hl and hu must have the same shape")
    lbz_t, _ = _bound(lbz, n, dt, dev)
    ubz_t, _ = _bound(ubz, n, dt, dev)
    nbox = 1 if (lbz_t is not None or ubz_t is not None) else 0
    mt = m + (n if nbox else 0)
    batch = _batch_of((sf, bf), (sh, bh))
    lib = _lib()
    wsb = int(lib.mpcqp_solve_poly_workspace(_code(dt), batch, n, m, nbox))
    ws = torch.empty((wsb,), dtype=torch.uint8, device=dev)
    z = torch.empty((batch, n), dtype=dt, device=dev)
    y = torch.empty((batch, mt), dtype=dt, device=dev)
    status = torch.empty((batch,), dtype=torch.int32, device=dev)
    rc = lib.mpcqp_solve_poly(_code(dt), batch, n, m, _ptr(H), _ptr(f), sf, _ptr(G), _ptr(hl),
                              _ptr(hu), sh, _ptr(lbz_t), _ptr(ubz_t), _ptr(z), _ptr(y),
                              _ptr(status), int(max_iter), float(tol), _ptr(ws), wsb, _stream())
    nat.check(rc, "mpcqp_solve_poly")
    return z, y, status


class PolyQP:
    """Shared-structure polytope QP for the receding-horizon loop
    (include/mpcqp.h ``mpcqp_poly_setup`` / ``mpcqp_poly_solve``):

        min 1/2 z'Hz + (F x0 + f)'z   s.t.  hl <= G z <= hu,  lbz <= z <= ubz

    H (packed, n(n+1)/2), G (m, n) and F (n, nx) are fixed at construction
    (the factors are formed once on device); ``solve`` takes a batch of x0
    and/or extra gradients f and per-instance or shared row bounds.
    """

    def __init__(self, H, G=None, F=None, lbz=None, ubz=None, *, dtype=None, device=None):
        dt = dtype or H.dtype
        dev = device or H.device
        self.dtype, self.device = dt, dev
        self.H = _dev(H, dt, dev)
        self.n = n = isqrt_packed(int(self.H.shape[-1]))
        self.G = _dev(G, dt, dev)
        self.m = 0 if G is None else int(self.G.shape[0])
        self.F = _dev(F, dt, dev)
        self.nx = 0 if F is None else int(self.F.shape[-1])
        self.lbz, _ = _bound(lbz, n, dt, dev)
        self.ubz, _ = _bound(ubz, n, dt, dev)
        self.nbox = 1 if (self.lbz is not None or self.ubz is not None) else 0
        self.mt = self.m + (n if self.nbox else 0)
        lib = _lib()
        wsb = int(lib.mpcqp_poly_workspace(_code(dt), n, self.m, self.nbox, self.nx))
        self.ws = torch.empty((wsb,), dtype=torch.uint8, device=dev)
        rc = lib.mpcqp_poly_setup(_code(dt), n, self.m, self.nbox, self.nx, _ptr(self.H),
                                  _ptr(self.G), _ptr(self.F), _ptr(self.ws), wsb, _stream())
        nat.check(rc, "mpcqp_poly_setup")

    def solve(self, x0=None, f=None, hl=None, hu=None, *, max_iter: int = 0, tol: float = 0.0,
              out: tuple | None = None):
        """Returns (z (b, n), y (b, m_total), status (b,))."""
        dt, dev, n = self.dtype, self.device, self.n
        x0, f = _dev(x0, dt, dev), _dev(f, dt, dev)
        hl, hu = _dev(hl, dt, dev), _dev(hu, dt, dev)
        sX, bX = _inst(x0, 1, "x0")
        sf, bf = _inst(f, 1, "f")
        sh, bh = 0, None
        for h in (hl, hu):
            if h is not None:
                sh, bh = _inst(h, 1, "h")
        batch = _batch_of((sX, bX), (sf, bf), (sh, bh))
        if out is None:
            z = torch.empty((batch, n), dtype=dt, device=dev)
            y = torch.empty((batch, self.mt), dtype=dt, device=dev)
            status = torch.empty((batch,), dtype=torch.int32, device=dev)
        else:
            z, y, status = out
        rc = _lib().mpcqp_poly_solve(_code(dt), batch, n, self.m, self.nbox, self.nx,
                                     _ptr(self.ws), _ptr(x0), sX, _ptr(f), sf, _ptr(hl), _ptr(hu),
                                     sh, _ptr(self.lbz), _ptr(self.ubz), _ptr(z), _ptr(y),
                                     _ptr(status), int(max_iter), float(tol), _stream())
        nat.check(rc, "mpcqp_poly_solve")
        return z, y, status


# ------------------------------------------ general QP, per-instance rows
def solve_qp(H, f, G=None, hl=None, hu=None, lb=None, ub=None, *, max_iter: int = 0,
             tol: float = 0.0, out: tuple | None = None, presweep: bool = True,
             ws: torch.Tensor | None = None):
    """Batched  min 1/2 z'Hz + f'z  s.t.  lb <= z <= ub,  hl <= G z <= hu.

    Every operand may be per instance (leading batch dim) or shared: H packed
    lower (n(n+1)/2), G (m, n), hl/hu (m), lb/ub (n).  n + m <= 192.
    One instance per workgroup (libmpcqp ``mpcqp_solve_qp``); fp32 with
    64 < n + m runs the z sweep first as its own MFMA kernel
    (``mpcqp_solve_qp_ws``) unless ``presweep=False``.
    Returns (z, y, status); y (batch, m) are the row multipliers
    (y > 0 at the upper bound, y < 0 at the lower bound).
    ``ws``: optional caller-owned scratch (``workspace_bytes(dtype, batch, n, m)``).
    """
    dt, dev = f.dtype, f.device
    f = _dev(f, dt, dev)
    H = _dev(H, dt, dev)
    n = int(f.shape[-1])
    if H.shape[-1] != n * (n + 1) // 2:
        raise ValueError(f"H must be packed lower with {n * (n + 1) // 2} entries, got {tuple(H.shape)}")
    sH, bH = _inst(H, 1, "H")
    sf, bf = _inst(f, 1, "f")
    m = 0 if G is None else int(G.shape[-2])
    G = _dev(G, dt, dev)
    sG, bG = (0, None) if G is None else _inst(G, 2, "G")
    hl = _dev(hl, dt, dev)
    hu = _dev(hu, dt, dev)
    if hl is not None and hu is not None and hl.shape != hu.shape:
        raise ValueError("hl and hu must have the same shape")
    sh, bh = 0, None
    for h in (hl, hu):
        if h is not None:
            sh, bh = _inst(h, 1, "h")
    lbt, slb = _bound(lb, n, dt, dev)
    ubt, sub = _bound(ub, n, dt, dev)
    batch = _batch_of((sH, bH), (sf, bf), (sG, bG), (sh, bh),
                      (slb, lbt.shape[0] if lbt is not None and lbt.ndim == 2 else None),
                      (sub, ubt.shape[0] if ubt is not None and ubt.ndim == 2 else None))
    if out is None:
        z = torch.empty((batch, n), dtype=dt, device=dev)
        y = torch.empty((batch, m), dtype=dt, device=dev) if m else None
        status = torch.empty((batch,), dtype=torch.int32, device=dev)
    else:
        z, y, status = out
    lib = _lib()
    wsb = int(lib.mpcqp_solve_qp_workspace(_code(dt), batch, n, m)) if presweep else 0
    ws = _workspace(wsb, dev, ws)
    rc = lib.mpcqp_solve_qp_ws(_code(dt), batch, n, m, _ptr(H), sH, _ptr(f), sf, _ptr(G), sG,
                               _ptr(hl), _ptr(hu), sh, _ptr(lbt), slb, _ptr(ubt), sub, _ptr(z),
                               _ptr(y), _ptr(status), int(max_iter), float(tol), _ptr(ws), wsb,
                               _stream())
    nat.check(rc, "mpcqp_solve_qp_ws")
    return z, y, status


def sweep(H, G=None, *, full: bool = False):
    """Batched M = SWEEP_z([[H, G'], [G, 0]]) (libmpcqp ``mpcqp_sweep``, fp32,
    MFMA): returns (M, status) with M = [[-H^-1, H^-1 G'], [G H^-1, -G H^-1 G']]
    over n + m per instance, packed lower, or dense (n+m, n+m) if ``full``."""
    dt, dev = H.dtype, H.device
    H = _dev(H, dt, dev)
    nH = int(H.shape[-1])
    n = isqrt_packed(nH)
    sH, bH = _inst(H, 1, "H")
    m = 0 if G is None else int(G.shape[-2])
    G = _dev(G, dt, dev)
    sG, bG = (0, None) if G is None else _inst(G, 2, "G")
    batch = _batch_of((sH, bH), (sG, bG))
    nt = n + m
    shape = (batch, nt, nt) if full else (batch, nt * (nt + 1) // 2)
    M = torch.empty(shape, dtype=dt, device=dev)
    status = torch.empty((batch,), dtype=torch.int32, device=dev)
    rc = _lib().mpcqp_sweep(_code(dt), batch, n, m, _ptr(H), sH, _ptr(G), sG, _ptr(M),
                            int(bool(full)), _ptr(status), _stream())
    nat.check(rc, "mpcqp_sweep")
    return M, status


# ---------------------------------------------------------------- Riccati
def riccati(A, B, Q, R, Pf, N: int):
    """Batched FHC.ricatti_recursion: returns P (b,N+1,nx,nx), K (b,N,nu,nx)."""
    dt = A.dtype
    dev = A.device
    A, B, Q, R, Pf = (_dev(v, dt, dev) for v in (A, B, Q, R, Pf))
    nx, nu = int(B.shape[-2]), int(B.shape[-1])
    R = _weight_r(R, nu)
    sA, bA = _inst(A, 2, "A")
    sB, bB = _inst(B, 2, "B")
    sQ, bQ = _inst(Q, 2, "Q")
    sR, bR = _inst(R, 2, "R")
    sP, bP = _inst(Pf, 2, "Pf")
    batch = _batch_of((sA, bA), (sB, bB), (sQ, bQ), (sR, bR), (sP, bP))
    P = torch.empty((batch, N + 1, nx, nx), dtype=dt, device=dev)
    K = torch.empty((batch, N, nu, nx), dtype=dt, device=dev)
    rc = _lib().mpcqp_riccati(_code(dt), batch, nx, nu, N, _ptr(A), sA, _ptr(B), sB, _ptr(Q), sQ,
                              _ptr(R), sR, _ptr(Pf), sP, _ptr(P), _ptr(K), _stream())
    nat.check(rc, "mpcqp_riccati")
    return P, K


# ------------------------------------------------------------------ gemv
def gemv(M, x, alpha: float = 1.0, beta: float = 0.0, y=None):
    """Batched y = alpha M x + beta y; M (r,c) shared or (b,r,c); x (c,) or (b,c)."""
    dt, dev = x.dtype, x.device
    M, x = _dev(M, dt, dev), _dev(x, dt, dev)
    rows, cols = int(M.shape[-2]), int(M.shape[-1])
    sM, bM = _inst(M, 2, "M")
    sX, bX = _inst(x, 1, "x")
    batch = _batch_of((sM, bM), (sX, bX))
    if y is None:
        y = torch.zeros((batch, rows), dtype=dt, device=dev)
    rc = _lib().mpcqp_gemv(_code(dt), batch, rows, cols, float(alpha), _ptr(M), sM, _ptr(x), sX,
                           float(beta), _ptr(y), rows, _stream())
    nat.check(rc, "mpcqp_gemv")
    return y


# ------------------------------------------------- bicycle re-linearisation
def bicycle_rti(x0, U, params, ts: float, *, states: bool = False):
    """Batched FE rollout + per-stage linearisation of the kinematic bicycle
    (include/mpcqp.h ``mpcqp_bicycle_rti``).  x0 (b, 4), U (b, N, 2) device
    tensors; params a VehicleParameters.  Returns A (b,N,4,4), B (b,N,4,2),
    c (b,N,4) [, X (b,N+1,4) when states]."""
    dt, dev = x0.dtype, x0.device
    x0 = x0.contiguous()
    U = U.contiguous()
    b, N = int(U.shape[0]), int(U.shape[1])
    A = torch.empty((b, N, 4, 4), dtype=dt, device=dev)
    B = torch.empty((b, N, 4, 2), dtype=dt, device=dev)
    c = torch.empty((b, N, 4), dtype=dt, device=dev)
    X = torch.empty((b, N + 1, 4), dtype=dt, device=dev) if states else None
    prm = _bike_params(params)
    rc = _lib().mpcqp_bicycle_rti(_code(dt), b, N, float(ts), prm, _ptr(x0), 4, _ptr(U), 2 * N,
                                  _ptr(X), _ptr(A), _ptr(B), _ptr(c), _stream())
    nat.check(rc, "mpcqp_bicycle_rti")
    return (A, B, c, X) if states else (A, B, c)


def _bike_params(params):
    return (ctypes.c_double * 4)(params.axis_front, params.axis_rear, params.acceleration,
                                 params.friction)


def bicycle_hessian(X, U, pi, params, ts: float, flags=None, mu=None,
                    out: tuple | None = None, Q=None, R=None, eps: float = 1e-6, fix=None,
                    integrator: int = 0):
    """Per stage, the curvature of the dynamics weighted by the costates plus
    a proximal mu I (include/mpcqp.h ``mpcqp_bicycle_hessian``): X (b, N+1,
    4), U (b, N, 2), pi (b, N, 4) fp64, mu (b,) or None -> H2 (b, N, 6, 6),
    q2 (b, N, 6); zeros where flags (b,) lacks SQP_EXACT.  With the stage
    weights Q (4, 4) and R (2, 2): ``mpcqp_bicycle_hessian_convex``, the
    curvature projected so that blkdiag(Q, R) + H2 >= eps I per stage.
    fix (b, N) int32 or None: inputs held at their bound (bits written by
    bicycle_sqp_step) get a proximal term on their diagonal.  integrator:
    the prediction model (0 forward Euler, 1 RK4)."""
    b, N = int(U.shape[0]), int(U.shape[1])
    if out is None:
        H2 = torch.empty((b, N, 6, 6), dtype=torch.float64, device=U.device)
        q2 = torch.empty((b, N, 6), dtype=torch.float64, device=U.device)
    else:
        H2, q2 = out
    if Q is not None:
        Qc = Q.to(torch.float64).contiguous()
        Rc = R.to(torch.float64).contiguous()
        rc = _lib().mpcqp_bicycle_hessian_convex(nat.F64, b, N, float(ts), _bike_params(params),
                                                 int(integrator), _ptr(X), _ptr(U), _ptr(pi), _ptr(flags), _ptr(mu),
                                                 _ptr(fix), _ptr(Qc), _ptr(Rc), float(eps), _ptr(H2),
                                                 _ptr(q2), _stream())
        nat.check(rc, "mpcqp_bicycle_hessian_convex")
        return H2, q2
    rc = _lib().mpcqp_bicycle_hessian(nat.F64, b, N, float(ts), _bike_params(params),
                                      int(integrator), _ptr(X),
                                      _ptr(U), _ptr(pi), _ptr(flags), _ptr(mu), _ptr(fix), _ptr(H2),
                                      _ptr(q2), _stream())
    nat.check(rc, "mpcqp_bicycle_hessian")
    return H2, q2


def _bound_pair(lo, hi, b: int, width: int, what: str):
    """A lower/upper bound pair that the C call reads with ONE instance stride:
    each side None, (width,) shared or (b, width).  A shared side next to a
    per-instance one is broadcast to (b, width), so the shared stride is never
    applied to a per-instance buffer or the reverse (which would read past
    the shared side's end).  Returns (lo, hi, stride)."""
    sides = [v for v in (lo, hi) if v is not None]
    for v in sides:
        if tuple(v.shape) not in ((width,), (b, width)):
            raise ValueError(f"{what}: shape {tuple(v.shape)} is neither ({width},) nor ({b}, {width})")
    if not any(v.ndim == 2 for v in sides):
        return lo, hi, 0
    ex = lambda v: None if v is None else v.expand(b, width).contiguous()  # noqa: E731
    return ex(lo), ex(hi), width


def bicycle_sqp_step(x0, U, Z, yq, piq, y, pi, X, state: dict, params, ts: float, Q, R, Qf,
                     xlo=None, xhi=None, lb=None, ub=None, tol: float = 1e-9, qp_status=None,
                     integrator: int = 0):
    """Line search + update + NLP optimality residual (include/mpcqp.h
    ``mpcqp_bicycle_sqp_step``), in place on U, y, pi, X and ``state``
    (rho, kkt, mu float64 (b,), flags int32 (b,), optional fix int32 (b, N):
    the inputs to hold at their bound in the next exact-Hessian QP).  Bounds: xlo/xhi (N*4,)
    shared or (b, N*4); lb/ub (N*2,) shared or (b, N*2)."""
    b, N = int(U.shape[0]), int(U.shape[1])
    xlo, xhi, sxb = _bound_pair(xlo, xhi, b, 4 * N, "xlo/xhi")
    lb, ub, slb = _bound_pair(lb, ub, b, 2 * N, "lb/ub")
    rc = _lib().mpcqp_bicycle_sqp_step(
        nat.F64, b, N, float(ts), _bike_params(params), int(integrator), _ptr(x0), 4, _ptr(Q),
        _ptr(R), _ptr(Qf),
        _ptr(xlo), _ptr(xhi), sxb, _ptr(lb), _ptr(ub), slb, _ptr(U), _ptr(Z), _ptr(yq), _ptr(piq),
        _ptr(qp_status), _ptr(y), _ptr(pi), _ptr(X), _ptr(state["rho"]), _ptr(state["kkt"]), _ptr(state["mu"]),
        _ptr(state["flags"]), _ptr(state.get("fix")), float(tol), _stream())
    nat.check(rc, "mpcqp_bicycle_sqp_step")


def bicycle_sqp_solve(x0, U, y, pi, X, state: dict, params, ts: float, Q, R, Qf, *,
                      hessian: str = "exact", xlo=None, xhi=None, lb=None, ub=None,
                      tol: float = 1e-9, max_iter: int = 60, qp_max_iter: int = 25,
                      integrator: int = 0, lam_u=None, qp_status=None,
                      ws: torch.Tensor | None = None) -> torch.Tensor:
    """The whole device SQP, up to max_iter iterations per instance, in one
    launch (include/mpcqp.h ``mpcqp_bicycle_sqp_solve``), in place on the SQP
    state U (b, N, 2), y (b, N*4), pi (b, N, 4), X (b, N+1, 4) and ``state``
    (rho, kkt, mu float64 (b,), flags int32 (b,), fix int32 (b, N)) -- the
    state of ``bicycle_sqp_step``, so a solve continues from it.  hessian:
    "exact", "exact-raw" or "gauss-newton".  lam_u (b, N*2) and qp_status
    (b,): optional outputs of the last QP.  Returns the workspace (pass it
    back as ``ws`` to reuse it)."""
    b, N = int(U.shape[0]), int(U.shape[1])
    xlo, xhi, sxb = _bound_pair(xlo, xhi, b, 4 * N, "xlo/xhi")
    lb, ub, slb = _bound_pair(lb, ub, b, 2 * N, "lb/ub")
    for name, t, shp, dt in (("U", U, (b, N, 2), torch.float64), ("y", y, (b, N * 4), torch.float64),
                             ("pi", pi, (b, N, 4), torch.float64),
                             ("X", X, (b, N + 1, 4), torch.float64),
                             ("x0", x0, (b, 4), torch.float64)):
        if tuple(t.shape) != shp or t.dtype != dt or not t.is_contiguous() or t.device != U.device:
            raise ValueError(f"bicycle_sqp_solve: {name} must be a contiguous {dt} device tensor "
                             f"of shape {shp}")
    lib = _lib()
    wsb = int(lib.mpcqp_bicycle_sqp_solve_workspace(b, N))
    ws = _workspace(wsb, U.device, ws)
    rc = lib.mpcqp_bicycle_sqp_solve(
        nat.F64, b, N, float(ts), _bike_params(params), int(integrator), nat.SQP_HESS[hessian],
        _ptr(x0), 4, _ptr(Q), _ptr(R), _ptr(Qf), _ptr(xlo), _ptr(xhi), sxb, _ptr(lb), _ptr(ub), slb,
        _ptr(U), _ptr(y), _ptr(pi), _ptr(X), _ptr(state["rho"]), _ptr(state["kkt"]),
        _ptr(state["mu"]), _ptr(state["flags"]), _ptr(state.get("fix")), _ptr(lam_u),
        _ptr(qp_status), int(max_iter), int(qp_max_iter), float(tol), _ptr(ws), wsb, _stream())
    nat.check(rc, "mpcqp_bicycle_sqp_solve")
    return ws


def bicycle_mpc_loop(xs, us, success, iters, state_prediction, input_prediction, U, y, pi, X,
                     state: dict, params, ts: float, Q, R, Qf, *, plant_params, plant: int = 0,
                     substeps: int = 20, hessian: str = "exact", xlo=None, xhi=None, lb=None,
                     ub=None, tol: float = 1e-9, iters_first: int = 60, iters_per_step: int = 10,
                     qp_max_iter: int = 25, integrator: int = 0, mu0: float = 1e-3,
                     ws: torch.Tensor | None = None) -> torch.Tensor:
    """The receding-horizon loop, every sample in one launch (include/mpcqp.h
    ``mpcqp_bicycle_mpc_loop``): xs (T+1, b, 4) with xs[0] given, us (T, b, 2),
    success (T, b) bool, iters (T, b) int32, state_prediction (T, b, N+1, 4),
    input_prediction (T, b, N, 2); the SQP state as ``bicycle_sqp_solve``'s
    (reset before).  Returns the workspace."""
    T, b = int(us.shape[0]), int(U.shape[0])
    N = int(U.shape[1])
    xlo, xhi, sxb = _bound_pair(xlo, xhi, b, 4 * N, "xlo/xhi")
    lb, ub, slb = _bound_pair(lb, ub, b, 2 * N, "lb/ub")
    for name, t, shp, dt in (("xs", xs, (T + 1, b, 4), torch.float64), ("us", us, (T, b, 2), torch.float64),
                             ("success", success, (T, b), torch.bool),
                             ("iters", iters, (T, b), torch.int32),
                             ("state_prediction", state_prediction, (T, b, N + 1, 4), torch.float64),
                             ("input_prediction", input_prediction, (T, b, N, 2), torch.float64)):
        if tuple(t.shape) != shp or t.dtype != dt or not t.is_contiguous() or t.device != U.device:
            raise ValueError(f"bicycle_mpc_loop: {name} must be a contiguous {dt} device tensor "
                             f"of shape {shp}")
    lib = _lib()
    wsb = int(lib.mpcqp_bicycle_sqp_solve_workspace(b, N))
    ws = _workspace(wsb, U.device, ws)
    rc = lib.mpcqp_bicycle_mpc_loop(
        nat.F64, b, N, T, float(ts), _bike_params(params), int(integrator), nat.SQP_HESS[hessian],
        _bike_params(plant_params), int(plant), int(substeps), _ptr(Q), _ptr(R), _ptr(Qf),
        _ptr(xlo), _ptr(xhi), sxb, _ptr(lb), _ptr(ub), slb, _ptr(U), _ptr(y), _ptr(pi), _ptr(X),
        _ptr(state["rho"]), _ptr(state["kkt"]), _ptr(state["mu"]), _ptr(state["flags"]),
        _ptr(state.get("fix")), int(iters_first), int(iters_per_step), int(qp_max_iter), float(tol),
        float(mu0), _ptr(xs), _ptr(us), _ptr(success), _ptr(iters), _ptr(state_prediction),
        _ptr(input_prediction), _ptr(ws), wsb, _stream())
    nat.check(rc, "mpcqp_bicycle_mpc_loop")
    return ws


def bicycle_linearise(x0, U, params, ts: float, integrator: int = 0, out: tuple | None = None):
    """Rollout + linearisation of the prediction model (include/mpcqp.h
    ``mpcqp_bicycle_linearise``; integrator 0 = forward Euler, 1 = RK4):
    x0 (b, 4), U (b, N, 2) fp64 -> A (b,N,4,4), B (b,N,4,2), c (b,N,4),
    X (b,N+1,4)."""
    b, N = int(U.shape[0]), int(U.shape[1])
    dev = U.device
    x0, U = x0.contiguous(), U.contiguous()
    if out is None:
        f64 = dict(dtype=torch.float64, device=dev)
        A = torch.empty((b, N, 4, 4), **f64)
        B = torch.empty((b, N, 4, 2), **f64)
        c = torch.empty((b, N, 4), **f64)
        X = torch.empty((b, N + 1, 4), **f64)
    else:
        A, B, c, X = out
    rc = _lib().mpcqp_bicycle_linearise(nat.F64, b, N, float(ts), _bike_params(params),
                                        int(integrator), _ptr(x0), 4, _ptr(U), 2 * N, _ptr(X),
                                        _ptr(A), _ptr(B), _ptr(c), _stream())
    nat.check(rc, "mpcqp_bicycle_linearise")
    return A, B, c, X


# --------------------------------------------------------------- rollout
def rollout(A, B, K, x0, steps: int):
    """Closed loop x_{t+1} = (A + B K) x_t for a batch of x0 (b,nx).

    Returns xs (steps, b, nx) time-major; ``xs.permute(2, 1, 0)`` is the
    reference's (nx, batch, steps) state tensor (LinearSystem.py:21,26).
    """
    dt, dev = x0.dtype, x0.device
    A, B, K, x0 = (_dev(v, dt, dev) for v in (A, B, K, x0))
    nx, nu = int(B.shape[-2]), int(B.shape[-1])
    batch = int(x0.shape[0])
    xs = torch.empty((steps, batch, nx), dtype=dt, device=dev)
    rc = _lib().mpcqp_rollout(_code(dt), batch, nx, nu, steps, _ptr(A), _ptr(B), _ptr(K), _ptr(x0),
                              _ptr(xs), _stream())
    nat.check(rc, "mpcqp_rollout")
    return xs


def max_qp_size(dtype=torch.float64) -> int:
    """Largest n + m accepted by solve_qp (and n by solve_box) for dtype."""
    return int(_lib().mpcqp_max_qp_size(_code(dtype)))


def n_packed(n: int) -> int:
    return n * (n + 1) // 2


def isqrt_packed(p: int) -> int:
    n = int((math.isqrt(8 * p + 1) - 1) // 2)
    assert n * (n + 1) // 2 == p
    return n
