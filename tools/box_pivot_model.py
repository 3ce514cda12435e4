"""CPU model of block-pivoting box-QP solvers on the config-2 distribution
(the headline fused kernel's problem: FHC double integrator, N = 20,
|u| <= 1, x0 ~ U(-10, 10)^2), counting iterations per QP.

Each iteration solves the LQ problem with the current set of inputs fixed at
a bound by one Riccati pass (backward factorisation + forward rollout, the
gradient g_k = R u_k + B' (P_{k+1} x_{k+1} + p_{k+1}) of every fixed input),
i.e. the serial per-QP work a one-lane-per-QP kernel would do per iteration.

    python tools/box_pivot_model.py [M]     # M instances (default 2000)

Rules:
  pdas   primal-dual active set (Hintermueller-Ito-Kunisch), set update
         mu + c (u - bound), for several c;
  bpp    safeguarded block principal pivoting (Judice-Pires: full exchange
         while the infeasibility count falls, p chances, then Murty's
         single least-index exchange -- finite for this P-matrix LCP).
Starts: 'free' (unconstrained) or 'clip' (the saturated LQR rollout).
Every converged solution is checked against oracle/qp.py on the condensed QP.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import condense as oc  # noqa: E402
from oracle import qp as oq  # noqa: E402

TS = 0.5
A = np.array([[1, TS], [0, 1.]])
B = np.array([[0], [-TS]])
_C = np.array([[1], [-2 / 3]])
Q = _C @ _C.T + 1e-3 * np.eye(2)
R = np.array([[0.1]])
QN = Q.copy()
N = 20
LB, UB = -1., 1.
b = B[:, 0]


def solve_fixed(x0, fix):
    """u and the gradient g of the LQ problem with u_k = bound where fix[k] != 0."""
    P, p = QN.copy(), np.zeros(2)
    Ks, kf = [None] * N, np.zeros(N)
    Ps, ps = [None] * (N + 1), [None] * (N + 1)
    Ps[N], ps[N] = P, p
    for k in range(N - 1, -1, -1):
        if fix[k] == 0:
            s = R[0, 0] + b @ P @ b
            K, kff = -(b @ P @ A) / s, -(b @ p) / s
            Ks[k], kf[k] = K, kff
            P, p = Q + A.T @ P @ A + np.outer(A.T @ P @ b, K), A.T @ p + A.T @ P @ b * kff
        else:
            ubar = UB if fix[k] > 0 else LB
            P, p = Q + A.T @ P @ A, A.T @ (P @ b * ubar + p)
        Ps[k], ps[k] = P, p
    x, u, g = x0.copy(), np.zeros(N), np.zeros(N)
    for k in range(N):
        u[k] = Ks[k] @ x + kf[k] if fix[k] == 0 else (UB if fix[k] > 0 else LB)
        xn = A @ x + b * u[k]
        g[k] = R[0, 0] * u[k] + b @ (Ps[k + 1] @ xn + ps[k + 1])
        x = xn
    return u, g


def clip_start(x0):
    P, Ks = QN.copy(), [None] * N
    for k in range(N - 1, -1, -1):
        s = R[0, 0] + b @ P @ b
        Ks[k] = -(b @ P @ A) / s
        P = Q + A.T @ P @ A + np.outer(A.T @ P @ b, Ks[k])
    fix, x = np.zeros(N, int), x0.copy()
    for k in range(N):
        u = Ks[k] @ x
        fix[k] = 1 if u > UB else (-1 if u < LB else 0)
        x = A @ x + b * np.clip(u, LB, UB)
    return fix


def pdas(x0, start, c, maxit=60):
    fix = clip_start(x0) if start == "clip" else np.zeros(N, int)
    for it in range(1, maxit + 1):
        u, g = solve_fixed(x0, fix)
        mu = np.where(fix != 0, -g, 0.0)
        nf = np.zeros(N, int)
        nf[mu + c * (u - UB) > 0] = 1
        nf[mu + c * (u - LB) < 0] = -1
        if (nf == fix).all():
            return u, it
        fix = nf
    return u, -1


def bpp(x0, start, pmax, tol=1e-12, maxit=200):
    fix = clip_start(x0) if start == "clip" else np.zeros(N, int)
    best, p = N + 1, pmax
    for it in range(1, maxit + 1):
        u, g = solve_fixed(x0, fix)
        up, lo = (fix == 0) & (u > UB + tol), (fix == 0) & (u < LB - tol)
        dual = ((fix > 0) & (g > tol)) | ((fix < 0) & (g < -tol))
        bad = up | lo | dual
        nb = int(bad.sum())
        if nb == 0:
            return u, it
        if nb < best:
            best, p, sel = nb, pmax, bad
        elif p > 0:
            p, sel = p - 1, bad
        else:
            sel = np.zeros(N, bool)
            sel[np.flatnonzero(bad)[0]] = True
        fix = fix.copy()
        fix[sel & up], fix[sel & lo], fix[sel & dual] = 1, -1, 0
    return u, -1


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    X0 = np.random.default_rng(20261015 + 2).uniform(-10, 10, size=(M, 2))
    ref = {}
    runs = [("pdas", s, c) for s in ("free", "clip") for c in (1e-3, 1.0, 1e3)]
    runs += [("bpp", s, pm) for s in ("free", "clip") for pm in (1, 3, 8)]
    for kind, start, par in runs:
        its, err = [], 0.0
        for i, x0 in enumerate(X0):
            u, it = (pdas if kind == "pdas" else bpp)(x0, start, par)
            its.append(it)
            if it > 0 and i < 64:
                if i not in ref:
                    d = oc.condense(A, B, Q, R, QN, N, x0=x0)
                    ref[i] = oq.box_qp(d["H"], d["f"], np.full(N, LB), np.full(N, UB))[0]
                err = max(err, float(np.abs(ref[i] - u).max()))
        its = np.array(its)
        ok = its[its > 0]
        print(f"{kind:4s} start={start:4s} par={par:<6g} cycled {int((its < 0).sum()):4d}/{M}"
              f"  mean {ok.mean():5.2f}  p95 {np.percentile(ok, 95):4.0f}  max {ok.max():3d}"
              f"  max|u-u_oracle| {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
