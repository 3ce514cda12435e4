"""Single-shooting NLP oracle of the session-4 MPC step (TEST INFRASTRUCTURE
ONLY -- imported by tests/, tests/golden/make_golden.py and bench.py's
checker, never by the product path).

The reference's ``MPCController.solve`` (session_4/main.py:115-116,
session4_sol.py:129-130) hands IPOPT the NLP that ``build_ocp`` writes
(main.py:41-113 without the non-convex collision rows; session4_sol.py:
132-217 exactly):

    min_U  sum_{k<N} x_k'Q x_k + u_k'R u_k + x_N'Q_N x_N          (main.py:86-88,106)
    s.t.   x_{k+1} = fwd_euler(bicycle)(x_k, u_k),  x_0 = x       (main.py:88, 132-135)
           lbx <= u_k <= ubx                                      (main.py:68-69, 89-90)
           lbg <= x_{k+1} <= ubg                                  (main.py:58-61, 91-93)

CasADi/IPOPT are not installed, so the optimum is pinned two independent
ways here: SciPy SLSQP on this NLP (``solve_slsqp``) and a Gauss-Newton SQP
on the oracle's own condensing + active-set QP (``solve_sqp``), certified by
the first-order KKT residual (``kkt``).  The bicycle ODE is the restatement
of oracle/bicycle.py (rcracers is absent: parity of the model unpinned);
every derivative here is by the complex step, independent of the analytic
Jacobians the device uses.
"""
from __future__ import annotations

import numpy as np

from . import condense as oc
from . import qp as oq

# kinematic parameters of parameters.py:7-8,47-48 (l_f, l_r, acceleration, friction)
PARAMS = (0.047, 0.05, 2.0, 1.0)


def f_ode(x, u, prm=PARAMS):
    lf, lr, acc, fric = prm
    beta = np.arctan(lr / (lf + lr) * np.tan(u[1]))
    return np.array([x[3] * np.cos(x[2] + beta), x[3] * np.sin(x[2] + beta),
                     x[3] / lr * np.sin(beta), acc * u[0] - fric * x[3]])


def fe(x, u, ts, prm=PARAMS):
    """main.py:132-135."""
    return x + ts * f_ode(x, u, prm)


def rk4(x, u, ts, prm=PARAMS):
    """main.py:138-147 (the model template.py:141 builds its OCP on)."""
    s1 = f_ode(x, u, prm)
    s2 = f_ode(x + ts / 2 * s1, u, prm)
    s3 = f_ode(x + ts / 2 * s2, u, prm)
    s4 = f_ode(x + ts * s3, u, prm)
    return x + ts / 6 * (s1 + 2 * s2 + 2 * s3 + s4)


STEPS = {"fe": fe, "rk4": rk4}


def fe_jac(x, u, ts, prm=PARAMS, h=1e-30, step=fe):
    """A = d step / dx, B = d step / du by the complex step (exact to
    rounding); step = fe (default) or rk4."""
    x = np.asarray(x, complex)
    u = np.asarray(u, complex)
    A = np.zeros((4, 4))
    B = np.zeros((4, 2))
    for i in range(4):
        d = np.zeros(4, complex); d[i] = 1j * h
        A[:, i] = step(x + d, u, ts, prm).imag / h
    for i in range(2):
        d = np.zeros(2, complex); d[i] = 1j * h
        B[:, i] = step(x, u + d, ts, prm).imag / h
    return A, B


def _stage_curvature(w, lam, ts, prm, step=fe, e=1e-6):
    """sum_i lam_i d2 fe_i / dw2 at w = [x; u] (6 x 6): central differences of
    the complex-step gradient of lam' fe."""
    def grad(wv):
        out = np.zeros(6)
        for j in range(6):
            d = np.zeros(6, complex)
            d[j] = 1e-30j
            ww = wv + d
            out[j] = (lam @ step(ww[:4], ww[4:], ts, prm)).imag / 1e-30
        return out
    H = np.zeros((6, 6))
    for j in range(6):
        d = np.zeros(6)
        d[j] = e
        H[:, j] = (grad(w + d) - grad(w - d)) / (2 * e)
    return 0.5 * (H + H.T)


class OCP:
    """The NLP of one MPC step; the cost is the reference's (not halved)."""

    def __init__(self, N, ts, Q, QN, R, xlo, xhi, lbu, ubu, prm=PARAMS, model="fe"):
        self.N, self.ts = N, ts
        self.step = STEPS[model]
        self.Q, self.QN, self.R = (np.asarray(v, float) for v in (Q, QN, R))
        self.xlo, self.xhi = np.asarray(xlo, float), np.asarray(xhi, float)
        self.lbu, self.ubu = np.asarray(lbu, float), np.asarray(ubu, float)
        self.prm = prm

    def rollout(self, x0, U):
        U = np.asarray(U).reshape(self.N, 2)
        xs = [np.asarray(x0, U.dtype if np.iscomplexobj(U) else float)]
        for k in range(self.N):
            xs.append(self.step(xs[-1], U[k], self.ts, self.prm))
        return np.array(xs)

    def cost(self, x0, U):
        U = np.asarray(U).reshape(self.N, 2)
        X = self.rollout(x0, U)
        J = sum(X[k] @ self.Q @ X[k] + U[k] @ self.R @ U[k] for k in range(self.N))
        return J + X[-1] @ self.QN @ X[-1]

    def linearise(self, x0, U):
        U = np.asarray(U, float).reshape(self.N, 2)
        X = self.rollout(x0, U)
        A = np.zeros((self.N, 4, 4)); B = np.zeros((self.N, 4, 2)); c = np.zeros((self.N, 4))
        for k in range(self.N):
            A[k], B[k] = fe_jac(X[k], U[k], self.ts, self.prm, step=self.step)
            c[k] = X[k + 1] - A[k] @ X[k] - B[k] @ U[k]
        return X, A, B, c

    def grad(self, x0, U, y=None):
        """Gradient of J/2 + y'[x_1; ..; x_N] w.r.t. U by the adjoint (y: state
        multipliers, N*4, > 0 at the upper bound; None = 0)."""
        X, A, B, _ = self.linearise(x0, U)
        U = np.asarray(U, float).reshape(self.N, 2)
        y = np.zeros((self.N, 4)) if y is None else np.asarray(y, float).reshape(self.N, 4)
        lam = self.QN @ X[self.N] + y[self.N - 1]
        g = np.zeros((self.N, 2))
        for k in range(self.N - 1, -1, -1):
            g[k] = self.R @ U[k] + B[k].T @ lam
            if k > 0:
                lam = self.Q @ X[k] + y[k - 1] + A[k].T @ lam
        return g.reshape(-1), X

    def lam_p(self, x0, U, y=None):
        """CasADi's lam_p for p = x0 in IPOPT's convention for the unhalved
        objective: lam_p = -d/dx0 (J + lam_g'g) along the single-shooting
        rollout = -2 lambda_0, lambda_0 = Q x0 + A_0' lambda_1 (the adjoint
        of grad() carried one stage further).  By the envelope theorem
        dJ*/dx0 = -lam_p at a KKT point."""
        X, A, _, _ = self.linearise(x0, U)
        y = np.zeros((self.N, 4)) if y is None else np.asarray(y, float).reshape(self.N, 4)
        lam = self.QN @ X[self.N] + y[self.N - 1]
        for k in range(self.N - 1, 0, -1):
            lam = self.Q @ X[k] + y[k - 1] + A[k].T @ lam
        return -2.0 * (self.Q @ X[0] + A[0].T @ lam)

    def kkt(self, x0, U, y):
        """First-order optimality residual of (U, y): projected gradient of the
        Lagrangian on the input box, state-box violation, wrong-sign and
        non-complementary state multipliers (max over all)."""
        U = np.asarray(U, float).reshape(-1)
        g, X = self.grad(x0, U, y)
        lb, ub = np.tile(self.lbu, self.N), np.tile(self.ubu, self.N)
        r_stat = np.abs(U - np.clip(U - g, lb, ub)).max()
        Xs = X[1:].reshape(-1)
        xlo, xhi = np.tile(self.xlo, self.N), np.tile(self.xhi, self.N)
        r_feas = max(np.maximum(Xs - xhi, 0).max(), np.maximum(xlo - Xs, 0).max())
        y = np.asarray(y, float).reshape(-1)
        r_comp = max(np.minimum(np.maximum(y, 0), xhi - Xs).max(initial=0),
                     np.minimum(np.maximum(-y, 0), Xs - xlo).max(initial=0))
        return max(r_stat, r_feas, r_comp)

    # ----------------------------------------------------------- solvers
    def qp_step(self, x0, U, HL=None):
        """QP at U (the oracle condensing and active set), Gauss-Newton
        Hessian plus HL (the curvature term, at U) when given: the minimiser
        Z and the state multipliers y (> 0 at xhi); (None, None) when the
        Hessian is not positive definite."""
        _, A, B, c = self.linearise(x0, U)
        N = self.N
        d = oc.condense(A, B, self.Q, self.R, self.QN, N, x0=x0, c=c)
        H, f = d["H"], d["f"]
        if HL is not None:
            Uv = np.asarray(U, float).reshape(-1)
            H, f = H + HL, f - HL @ Uv
            try:
                np.linalg.cholesky(H)
            except np.linalg.LinAlgError:
                return None, None
        G = np.vstack([d["Gam"], -d["Gam"]])
        h = np.concatenate([np.tile(self.xhi, N) - d["xbar"], d["xbar"] - np.tile(self.xlo, N)])
        Z, lam, _ = oq.poly_qp(H, f, G, h, np.tile(self.lbu, N), np.tile(self.ubu, N))
        m = N * 4
        return Z, lam[:m] - lam[m:2 * m]

    def merit(self, x0, U, rho):
        X = self.rollout(x0, U)[1:].reshape(-1)
        viol = np.maximum(X - np.tile(self.xhi, self.N), 0).sum() + \
            np.maximum(np.tile(self.xlo, self.N) - X, 0).sum()
        return 0.5 * self.cost(x0, U) + rho * viol, viol

    def lag_hessian(self, x0, U, y):
        """Condensed Hessian of sum_k pi_{k+1}' fe(x_k, u_k) w.r.t. U, the
        costates pi from the adjoint recursion with state multipliers y: the
        part of the exact Hessian of the Lagrangian that Gauss-Newton drops.
        Stage curvatures by central differences of complex-step gradients."""
        N = self.N
        X, A, B, c = self.linearise(x0, U)
        Ur = np.asarray(U, float).reshape(N, 2)
        yr = np.asarray(y, float).reshape(N, 4)
        lam = [None] * (N + 1)
        lam[N] = self.QN @ X[N] + yr[N - 1]
        for k in range(N - 1, 0, -1):
            lam[k] = self.Q @ X[k] + yr[k - 1] + A[k].T @ lam[k + 1]
        d = oc.condense(A, B, self.Q, self.R, self.QN, N, x0=x0, c=c)
        HL = np.zeros((2 * N, 2 * N))
        for k in range(N):
            w = np.concatenate([X[k], Ur[k]])
            L = _stage_curvature(w, lam[k + 1], self.ts, self.prm, self.step)
            M = np.zeros((6, 2 * N))
            if k > 0:
                M[:4] = d["Gam"][(k - 1) * 4:k * 4]
            M[4:, 2 * k:2 * k + 2] = np.eye(2)
            HL += M.T @ L @ M
        return HL

    def solve_sqp(self, x0, U0=None, tol=1e-12, max_iter=400, hessian="exact", switch=1e-2):
        """SQP with an L1-merit line search (quadratic-interpolation
        backtracking, Armijo).  Gauss-Newton QPs until the KKT residual is
        below ``switch``, then the exact Hessian of the Lagrangian (if it
        makes the QP strictly convex; a step that needs backtracking lowers
        the switch level).  Returns (U, y, kkt, iterations)."""
        N = self.N
        U = np.zeros(2 * N) if U0 is None else np.asarray(U0, float).reshape(-1).copy()
        y = np.zeros(4 * N)
        rho, k = 1.0, np.inf
        for it in range(1, max_iter + 1):
            HL = None
            if hessian == "exact" and k < switch:
                HL = self.lag_hessian(x0, U, y)
            Z, yq = self.qp_step(x0, U, HL)
            exact = HL is not None and Z is not None
            if Z is None:  # exact-Hessian QP not convex: Gauss-Newton this time
                switch = min(switch, 0.1 * k)
                Z, yq = self.qp_step(x0, U)
            d = Z - U
            rho = max(rho, 2.0 * np.abs(yq).max(initial=0.0))
            phi0, viol0 = self.merit(x0, U, rho)
            g, _ = self.grad(x0, U)
            D = g @ d - rho * viol0
            a = 1.0
            while a > 1e-10 and np.abs(d).max() > 1e-15:
                pa = self.merit(x0, U + a * d, rho)[0]
                if pa <= phi0 + 1e-4 * a * D:
                    break
                den = 2.0 * (pa - phi0 - a * D)
                at = -D * a * a / den if den > 0 else 0.5 * a
                a = min(0.5 * a, max(0.1 * a, at))
            U = U + a * d
            y = y + a * (yq - y)
            k = self.kkt(x0, U, y)
            if exact and a < 1.0:
                switch = min(switch, 0.1 * k)
            if k < tol:
                break
        return U, y, k, it

    def newton_polish(self, x0, U, y, iters=8, tol=1e-13):
        """Newton's method on the first-order conditions with the active set
        of (U, y) held fixed (inputs at a bound stay there, state rows with a
        multiplier are equalities): the exact Hessian of the Lagrangian need
        only be positive definite on the null space of the active rows, and
        convergence is quadratic.  Returns (U, y, kkt) -- the input point if
        no Newton step improves it."""
        N = self.N
        U = np.asarray(U, float).reshape(-1).copy()
        y = np.asarray(y, float).reshape(-1).copy()
        lb, ub = np.tile(self.lbu, N), np.tile(self.ubu, N)
        xlo, xhi = np.tile(self.xlo, N), np.tile(self.xhi, N)
        best = (U.copy(), y.copy(), self.kkt(x0, U, y))
        for _ in range(iters):
            g0, X = self.grad(x0, U)                     # gradient of J/2
            _, A, B, c = self.linearise(x0, U)
            d = oc.condense(A, B, self.Q, self.R, self.QN, N, x0=x0, c=c)
            H = d["H"] + self.lag_hessian(x0, U, y)
            Gam = d["Gam"]
            Xs = X[1:].reshape(-1)
            rows = np.nonzero(y != 0.0)[0]
            bnd = np.where(y[rows] > 0, xhi[rows], xlo[rows])
            fixed = (np.abs(U - lb) < 1e-12) | (np.abs(U - ub) < 1e-12)
            F = np.nonzero(~fixed)[0]
            C = Gam[np.ix_(rows, F)]
            nF, nA = F.size, rows.size
            K = np.zeros((nF + nA, nF + nA))
            K[:nF, :nF] = H[np.ix_(F, F)]
            K[:nF, nF:] = C.T
            K[nF:, :nF] = C
            rhs = np.concatenate([-(g0[F]), -(Xs[rows] - bnd)])
            try:
                sol = np.linalg.solve(K, rhs)
            except np.linalg.LinAlgError:
                break
            U[F] += sol[:nF]
            U = np.clip(U, lb, ub)
            y = np.zeros_like(y)
            y[rows] = sol[nF:]
            k = self.kkt(x0, U, y)
            if k < best[2]:
                best = (U.copy(), y.copy(), k)
            if k < tol:
                break
        return best

    def solve(self, x0, U0=None, tol=1e-12):
        """The oracle's optimum: the SQP (Gauss-Newton to a 1e-7 residual)
        then ``newton_polish``.  Returns (U, y, kkt)."""
        U, y, k, _ = self.solve_sqp(x0, U0, tol=1e-7, hessian="gauss-newton", max_iter=2000)
        if k >= tol:
            U, y, k = self.newton_polish(x0, U, y, tol=tol)
        return U, y, k

    def solve_slsqp(self, x0, U0=None):
        """SciPy SLSQP on the NLP itself (cost and constraint gradients by the
        adjoint / complex step).  Returns U."""
        from scipy.optimize import minimize

        N = self.N
        U0 = np.zeros(2 * N) if U0 is None else np.asarray(U0, float).reshape(-1)
        xlo, xhi = np.tile(self.xlo, N), np.tile(self.xhi, N)

        def fun(U):
            g, _ = self.grad(x0, U)
            return 0.5 * self.cost(x0, U), g

        def states(U):
            return self.rollout(x0, U)[1:].reshape(-1)

        def states_jac(U):
            _, A, B, _ = self.linearise(x0, U)
            d = oc.condense(A, B, self.Q, self.R, self.QN, N, x0=x0)
            return d["Gam"]

        cons = [dict(type="ineq", fun=lambda U: xhi - states(U), jac=lambda U: -states_jac(U)),
                dict(type="ineq", fun=lambda U: states(U) - xlo, jac=states_jac)]
        bounds = list(zip(np.tile(self.lbu, N), np.tile(self.ubu, N)))
        r = minimize(fun, U0, jac=True, method="SLSQP", bounds=bounds, constraints=cons,
                     options=dict(ftol=1e-16, maxiter=2000))
        return r.x, r
