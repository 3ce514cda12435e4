"""NumPy model of qp_pf_kernel (solve_pf.hip) for one instance -- a line-by-line
transcription used to debug the product-form active set on the CPU.

    python tools/pf_model.py [cfg3|cfg5|box]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def swept(H, G):
    Hi = np.linalg.inv(H)
    if G is None or G.shape[0] == 0:
        return -Hi
    return np.block([[-Hi, Hi @ G.T], [G @ Hi, -G @ Hi @ G.T]])


def pf_solve(H, f, G, lo, hi, tol=1e-6, max_iter=None, dt=np.float32, refine=2, verbose=False):
    n = H.shape[0]
    m = 0 if G is None else G.shape[0]
    nt = n + m
    M0 = swept(H.astype(np.float64), None if G is None else G.astype(np.float64)).astype(dt)
    max_iter = max_iter or 3 * nt + 30
    lo = lo.astype(dt)
    hi = hi.astype(dt)
    fz = np.zeros(nt, dt)
    fz[:n] = f
    sl = np.where(np.isfinite(lo), 1 / (1 + np.abs(lo)), np.nan).astype(dt)
    su = np.where(np.isfinite(hi), 1 / (1 + np.abs(hi)), np.nan).astype(dt)
    scl = np.abs(np.diag(M0))
    st = np.zeros(nt, int)
    slot = -np.ones(nt, int)
    val = np.zeros(nt, dt)
    mu = np.zeros(nt, dt)
    S = np.zeros((64, 64), dt)
    aidx = -np.ones(64, int)
    sbnd = np.zeros(64, dt)
    sisz = np.zeros(64, bool)
    used = np.zeros(64, bool)
    isz = np.arange(nt) < n
    s0 = (M0[:, :n] @ fz[:n]).astype(dt)

    def act():
        return (st == 1) | (st == 2)

    def gather(x):
        return np.where(used, x[np.maximum(aidx, 0)], 0).astype(dt)

    def pcols(q, out, sign):
        for j in np.nonzero(used)[0]:
            out += sign * q[j] * M0[aidx[j]]

    def refresh():
        yv = s0.copy()
        for j in np.nonzero(used)[0]:
            if aidx[j] < n:
                yv -= fz[aidx[j]] * M0[aidx[j]]
        ys = gather(yv)
        t = np.where(used, ys - np.where(sisz, sbnd, -sbnd), 0).astype(dt)
        q = S @ t
        pcols(q, yv, 1)
        a = act()
        qi = q[np.maximum(slot, 0)]
        msw = np.where(a, -qi, yv)
        s = np.where(a & isz, -msw, msw)
        bnd = np.where(st == 1, lo, hi)
        mval = np.where(isz, fz - s, s)
        sside = np.where(st == 1, 1, -1) * np.where(isz, 1, -1)
        val[:] = np.where(a, bnd, np.where(isz, s, -s))
        mu[:] = np.where(a, sside * mval, 0)

    def scan():
        with np.errstate(invalid="ignore"):
            vl = (lo - val) * sl
            vu = (val - hi) * su
            v = np.where(st == 0, np.fmax(vl, vu), -np.inf)
        v = np.where(v == v, v, -np.inf)
        p = int(np.argmax(v))
        return v[p], p

    iters = 0
    code = 0
    refresh()
    active = True
    for pas in range(3):
        if not active:
            break
        while True:
            viol, p = scan()
            if not viol > tol:
                break
            valp = val[p]
            lop, hip = lo[p], hi[p]
            side = 1 if valp < lop else 2
            tgt = lop if side == 1 else hip
            pz = p < n
            epsp = -1.0 if pz else 1.0
            sidesign = (1.0 if side == 1 else -1.0) * (1.0 if pz else -1.0)
            sgn = 1.0 if tgt > valp else -1.0
            scp = scl[p]
            tau = 0.0
            added = False
            while not added:
                iters += 1
                if iters > max_iter:
                    return val, 1, iters
                col = M0[p].copy()
                u = gather(col)
                v = (S @ u).astype(dt)
                pcols(v, col, 1)
                a = act()
                vs = v[np.maximum(slot, 0)]
                col = np.where(a, np.where(isz, vs, -vs), col).astype(dt)
                mpp = col[p]
                dep = not (-mpp > 2e-5 * scp)
                dtds = sidesign if dep else sgn * epsp / mpp
                t2 = np.inf if dep else abs(tgt - valp)
                dq = col * dtds
                dmu = np.where(a, np.where(st == 1, dq, -dq), 0)
                with np.errstate(divide="ignore", invalid="ignore"):
                    t = np.where(a & (dmu < 0), -mu / dmu, np.inf)
                t = np.where(t == t, t, np.inf)
                k = int(np.argmin(t))
                ti = t[k]
                if not ti < np.inf and not t2 < np.inf:
                    return val, 3, iters
                partial = ti < t2
                s_eff = ti if partial else t2
                dval = np.where(st == 0, np.where(isz, -dq, dq), 0)
                val[:] = val + s_eff * dval
                mu[:] = mu + s_eff * dmu
                tau += s_eff * dtds
                if verbose:
                    print(f"it {iters} p {p} k {k} partial {partial} dep {dep} mpp {mpp:.3e} "
                          f"s {s_eff:.3e} nact {used.sum()}")
                if partial:
                    if not dep:
                        valp = valp + sgn * s_eff
                    q = slot[k]
                    d = S[q, q]
                    if not d > 0:
                        return val, 2, iters
                    r = S[:, q].copy()
                    S[:] = S - np.outer(r, r) / d
                    S[q, :] = 0
                    S[:, q] = 0
                    used[q] = False
                    aidx[q] = -1
                    st[k] = 0
                    mu[k] = 0
                    slot[k] = -1
                else:
                    if not mpp < 0:
                        return val, 2, iters
                    snew = int(np.argmin(used))
                    w = v.copy()
                    w[snew] = 1
                    S[:] = S + np.outer(w, w) / (-mpp)
                    used[snew] = True
                    aidx[snew] = p
                    sbnd[snew] = tgt
                    sisz[snew] = pz
                    st[p] = side
                    mu[p] = sidesign * tau
                    val[p] = tgt
                    slot[p] = snew
                added = not partial
        refresh()
        viol, p = scan()
        active = viol > tol
    if active:
        code = 1
    K = np.zeros((nt, nt))
    K[:n, :n] = H
    if m:
        K[n:, :n] = G
        K[:n, n:] = G.T
    for _ in range(refine):
        a = act()
        sside = np.where(st == 1, 1, -1) * np.where(isz, 1, -1)
        x = np.where(isz, val, np.where(a, sside * mu, 0)).astype(np.float64)
        yk = K @ x
        bnd = np.where(st == 1, lo, hi).astype(np.float64)
        inS = np.where(isz, st == 0, a)
        e = np.where(isz, yk + fz, yk - bnd)
        w = np.where(inS, e, 0).astype(dt)
        y2 = (M0[:n].T @ w[:n]).astype(dt)
        ys = gather(y2)
        wsl = gather(w)
        q = S @ np.where(used, ys - wsl, 0).astype(dt)
        pcols(q, y2, 1)
        qi = q[np.maximum(slot, 0)]
        sv = np.where(a, -qi, y2)
        val[:] = np.where(isz & (st == 0), val + sv, val)
        mu[:] = np.where(~isz & a, mu + sside * sv, mu)
    z = np.clip(val[:n], lo[:n], hi[:n])
    return z, code, iters


def _spd(rng, n, cond=30.0):
    Qm, _ = np.linalg.qr(rng.normal(size=(n, n)))
    return (Qm * np.geomspace(1.0, cond, n)) @ Qm.T


if __name__ == "__main__":
    from oracle import condense as oc
    from oracle import qp as oq
    which = sys.argv[1] if len(sys.argv) > 1 else "box"
    rng = np.random.default_rng(1)
    if which == "box":
        n = 100
        H = _spd(rng, n)
        f = rng.normal(size=n) * 10
        z, code, it = pf_solve(H, f, None, -np.ones(n), np.ones(n), verbose=False)
        zr = oq.box_qp(H, f, -np.ones(n), np.ones(n))[0]
        print(which, code, it, np.abs(z - zr).max())
    elif which == "cfg5":
        import bench  # noqa: F401
        nx, nu, N = 12, 4, 40
        A, B = bench._stable_plant(np.random.default_rng(20261015 + 4), nx, nu)
        for trial in range(4):
            Ak = A + 0.01 * rng.normal(size=(N, nx, nx))
            Bk = B + 0.01 * rng.normal(size=(N, nx, nu))
            x0 = 3 * rng.normal(size=nx)
            d = oc.condense(Ak, Bk, np.eye(nx), 0.1 * np.eye(nu), np.eye(nx), N, x0=x0)
            n = N * nu
            z, code, it = pf_solve(d["H"], d["f"], None, -0.5 * np.ones(n), 0.5 * np.ones(n))
            zr = oq.box_qp(d["H"], d["f"], -0.5 * np.ones(n), 0.5 * np.ones(n))[0]
            print(which, code, it, np.abs(z - zr).max(), np.linalg.cond(d["H"]))
    elif which == "rows":
        n, m = 60, 120
        H = _spd(rng, n)
        G = rng.normal(size=(m, n))
        f = rng.normal(size=n) * 10
        hl = -rng.uniform(0.5, 3.0, size=m)
        hu = rng.uniform(0.5, 3.0, size=m)
        lo = np.concatenate([-1.5 * np.ones(n), hl])
        hi = np.concatenate([1.5 * np.ones(n), hu])
        z, code, it = pf_solve(H, f, G, lo, hi, verbose="-v" in sys.argv)
        print(which, code, it)
