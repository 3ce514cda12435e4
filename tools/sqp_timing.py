"""Development probe: device time of the batched SQP (MPCController's
SqpSolver) for a few batch sizes and horizons -- the launches of one
iteration timed separately, then whole solves from U = 0 with the fraction
converged after each block of iterations -- printed as it goes.
Usage: python tools/sqp_timing.py [N ...]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from model_predictive_control_amd import batched  # noqa: E402
from model_predictive_control_amd.mpc import MPCController, SqpSolver  # noqa: E402
from model_predictive_control_amd.parameters import VehicleParameters  # noqa: E402


def ms(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


Ns = [int(a) for a in sys.argv[1:]] or [30, 50]
for N in Ns:
    for b in (1, 64, 1024, 4096):
        ctl = MPCController(N, 0.08, VehicleParameters())
        sqp = SqpSolver(ctl, b)
        rng = np.random.default_rng(1)
        X0 = torch.as_tensor(np.stack([rng.uniform(-.8, .8, b), rng.uniform(-.4, .4, b),
                                       rng.uniform(-.5, .5, b), rng.uniform(-.2, .2, b)], -1),
                             dtype=torch.float64, device=ctl.device)
        # whole solves: iterations until every instance is done (cap 80)
        sqp.reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        trace = []
        for it in range(1, 81):
            sqp.iterate(X0)
            if it % 5 == 0:
                nd = int(sqp.done().sum())
                trace.append(f"{it}:{nd}")
                if nd == b:
                    break
        torch.cuda.synchronize()
        t_solve = (time.perf_counter() - t0) * 1e3
        # launches of one iteration at the final state
        A, B, c, Xr = batched.bicycle_rti(X0, sqp.U, ctl.params, ctl.ts, states=True)
        H2, q2 = batched.bicycle_hessian(Xr, sqp.U, sqp.pi, ctl.params, ctl.ts, mu=sqp.mu)
        box = ctl._box()
        kw = dict(lb=ctl.lbz, ub=ctl.ubz, c=c, tv=True, H2=H2, q2=q2, strict=True,
                  max_iter=SqpSolver.QP_MAX_ITER, **box)
        t_rti = ms(lambda: batched.bicycle_rti(X0, sqp.U, ctl.params, ctl.ts, states=True))
        t_ipm = ms(lambda: batched.mpc_ipm(A, B, ctl.Q, ctl.R, ctl.QN, N, X0, **kw))
        r = batched.mpc_ipm(A, B, ctl.Q, ctl.R, ctl.QN, N, X0, **kw)
        it_q = ((r["status"] >> 8) & 0xFFFF).double()
        print(f"N={N} b={b}: solve {t_solve:.1f} ms ({it} iters, {t_solve / it:.2f} ms/iter; "
              f"done {' '.join(trace)}; kkt max {sqp.kkt.max().item():.1e}) | final-state rti "
              f"{t_rti:.3f} ms, ipm {t_ipm:.3f} ms (qp iters mean {it_q.mean().item():.1f} "
              f"max {it_q.max().item():.0f})", flush=True)
