"""Exact fp64 QP oracles with KKT certificates (TEST INFRASTRUCTURE ONLY).

The reference hands its per-step OCP to CasADi/IPOPT
(``session_4/main.py:38-39`` builds ``cs.nlpsol("solver","ipopt",...)``,
``main.py:115-116`` calls it with ``lbx/ubx`` = input box and ``lbg/ubg`` =
state box).  Neither CasADi nor IPOPT is installed in this container, so the
substitute oracles below are used; because the condensed QP is strictly
convex (H positive definite) its minimiser is unique, and each solution is
*certified* by its KKT residuals -- parity with IPOPT itself is unpinned.

* ``box_qp``      -- primal active-set method (Nocedal & Wright Alg. 16.3)
                     for  min 1/2 z'Hz + f'z  s.t.  lb <= z <= ub.
* ``box_qp_bvls`` -- independent cross-check via SciPy's bounded-variable
                     least squares on (L^T, -L^-1 f) with H = L L^T.
* ``poly_qp``     -- Goldfarb-Idnani dual active-set method for
                     min 1/2 z'Hz + f'z  s.t.  G z <= h  (box rows optional),
                     with the (J, R) factors recomputed by QR at every change
                     of the active set (slow, simple, exact).
* ``kkt_box`` / ``kkt_poly`` -- KKT residual certificates.
"""
from __future__ import annotations

import numpy as np


# ----------------------------------------------------------------------------
# box-constrained QP
# ----------------------------------------------------------------------------
def box_qp(H, f, lb, ub, max_iter=1000, tol=1e-12):
    """Primal active set; returns (z, mult, iters). mult>0 at lower, <0 at upper."""
    H = np.asarray(H, float)
    f = np.asarray(f, float)
    n = f.size
    lb = np.full(n, -np.inf) if lb is None else np.broadcast_to(np.asarray(lb, float), (n,)).copy()
    ub = np.full(n, np.inf) if ub is None else np.broadcast_to(np.asarray(ub, float), (n,)).copy()
    if np.any(lb > ub):
        raise ValueError("infeasible bounds")
    z = np.clip(np.zeros(n), lb, ub)
    W = np.zeros(n, dtype=int)          # 0 free, -1 at lower, +1 at upper
    W[z == lb] = -1
    W[(z == ub) & (W == 0)] = 1
    scale = max(1.0, np.abs(f).max(initial=0.0))
    for it in range(max_iter):
        F = W == 0
        zs = z.copy()
        if F.any():
            rhs = -(f[F] + H[np.ix_(F, ~F)] @ z[~F])
            zs[F] = np.linalg.solve(H[np.ix_(F, F)], rhs)
        p = zs - z
        alpha, block = 1.0, -1
        for i in np.nonzero(F)[0]:
            if p[i] < 0 and np.isfinite(lb[i]):
                a = (lb[i] - z[i]) / p[i]
            elif p[i] > 0 and np.isfinite(ub[i]):
                a = (ub[i] - z[i]) / p[i]
            else:
                continue
            if a < alpha:
                alpha, block = a, i
        if block >= 0:
            z = z + alpha * p
            z[block] = lb[block] if p[block] < 0 else ub[block]
            W[block] = -1 if p[block] < 0 else 1
            continue
        z = zs
        g = H @ z + f
        mu = np.where(W == -1, g, np.where(W == 1, -g, np.inf))
        mu[lb == ub] = np.inf
        j = int(np.argmin(mu))
        if mu[j] >= -tol * scale:
            return z, np.where(W != 0, g, 0.0), it + 1
        W[j] = 0
    raise RuntimeError("box_qp: max_iter reached")


def box_qp_bvls(H, f, lb, ub):
    """SciPy BVLS cross-check: min ||L^T z + L^{-1} f||^2 over the box."""
    from scipy.optimize import lsq_linear

    L = np.linalg.cholesky(np.asarray(H, float))
    b = -np.linalg.solve(L, np.asarray(f, float))
    n = b.size
    lb = np.full(n, -np.inf) if lb is None else np.broadcast_to(lb, (n,))
    ub = np.full(n, np.inf) if ub is None else np.broadcast_to(ub, (n,))
    res = lsq_linear(L.T, b, bounds=(lb, ub), method="bvls", tol=1e-14, max_iter=10 * n + 100)
    return res.x


def kkt_box(H, f, lb, ub, z):
    """Max KKT residual (stationarity on the free set, sign of multipliers, bounds)."""
    n = f.size
    lb = np.full(n, -np.inf) if lb is None else np.broadcast_to(lb, (n,))
    ub = np.full(n, np.inf) if ub is None else np.broadcast_to(ub, (n,))
    g = H @ z + f
    span = np.maximum(1.0, np.abs(z))
    at_l = np.abs(z - lb) <= 1e-9 * span
    at_u = np.abs(z - ub) <= 1e-9 * span
    free = ~(at_l | at_u)
    r_stat = np.abs(g[free]).max(initial=0.0)
    r_sign = max(np.maximum(-g[at_l & ~at_u], 0).max(initial=0.0),
                 np.maximum(g[at_u & ~at_l], 0).max(initial=0.0))
    r_feas = max(np.maximum(lb - z, 0).max(initial=0.0), np.maximum(z - ub, 0).max(initial=0.0))
    return max(r_stat, r_sign, r_feas)


# ----------------------------------------------------------------------------
# polytope QP: Goldfarb-Idnani dual active set
# ----------------------------------------------------------------------------
def poly_qp(H, f, G, h, lb=None, ub=None, max_iter=5000, tol=1e-11):
    """min 1/2 z'Hz + f'z  s.t.  G z <= h  [and lb <= z <= ub].

    Returns (z, lam, iters) where lam are the multipliers of the rows of
    ``[G; I; -I]`` (box rows appended only when lb/ub are given).
    """
    H = np.asarray(H, float)
    f = np.asarray(f, float)
    n = f.size
    rows = [np.asarray(G, float).reshape(-1, n)]
    rhs = [np.asarray(h, float).reshape(-1)]
    if ub is not None:
        ubv = np.broadcast_to(np.asarray(ub, float), (n,))
        k = np.isfinite(ubv)
        rows.append(np.eye(n)[k]); rhs.append(ubv[k])
    if lb is not None:
        lbv = np.broadcast_to(np.asarray(lb, float), (n,))
        k = np.isfinite(lbv)
        rows.append(-np.eye(n)[k]); rhs.append(-lbv[k])
    C = np.vstack(rows)                 # C z <= d
    d = np.concatenate(rhs)
    m = C.shape[0]
    L = np.linalg.cholesky(H)
    Linv = np.linalg.inv(L)
    x = -np.linalg.solve(H, f)
    act: list[int] = []
    u = np.zeros(0)
    scale = max(1.0, np.abs(d).max(initial=0.0), np.abs(f).max(initial=0.0))

    def factors():
        q = len(act)
        if q == 0:
            return Linv.T, np.zeros((0, 0))
        Nt = Linv @ (-C[act].T)          # normals of  s_i = d_i - C_i z >= 0 are -C_i
        Qm, Rm = np.linalg.qr(Nt, mode="complete")
        return Linv.T @ Qm, Rm[:q, :q]

    it = 0
    while True:
        s = d - C @ x
        s[act] = np.inf
        p = int(np.argmin(s))
        if s[p] >= -tol * scale:
            lam = np.zeros(m)
            lam[act] = u
            return x, lam, it
        npl = -C[p]
        up = 0.0
        while True:
            it += 1
            if it > max_iter:
                raise RuntimeError("poly_qp: max_iter reached")
            J, Rm = factors()
            q = len(act)
            dv = J.T @ npl
            zdir = J[:, q:] @ dv[q:]
            r = np.linalg.solve(Rm, dv[:q]) if q else np.zeros(0)
            t1, k = np.inf, -1
            for j in range(q):
                if r[j] > 0 and u[j] / r[j] < t1:
                    t1, k = u[j] / r[j], j
            zn = zdir @ npl
            t2 = np.inf if np.linalg.norm(zdir) <= 1e-14 * max(1.0, np.linalg.norm(npl)) else -(d[p] - C[p] @ x) / zn
            t = min(t1, t2)
            if not np.isfinite(t):
                raise ValueError("poly_qp: infeasible")
            if not np.isfinite(t2):
                u = u - t * r
                up += t
                del act[k]
                u = np.delete(u, k)
                continue
            x = x + t * zdir
            u = u - t * r
            up += t
            if t == t2:
                act.append(p)
                u = np.append(u, up)
                break
            del act[k]
            u = np.delete(u, k)


def kkt_poly(H, f, C, d, z, lam):
    """Max KKT residual for C z <= d with multipliers lam >= 0."""
    g = H @ z + f + C.T @ lam
    s = d - C @ z
    return max(np.abs(g).max(initial=0.0),
               np.maximum(-s, 0).max(initial=0.0),
               np.maximum(-lam, 0).max(initial=0.0),
               np.abs(lam * s).max(initial=0.0))
