"""Development probe: device time of one SQP iteration's launches
(bicycle_rti, bicycle_hessian, mpc_ipm, bicycle_sqp_step) for a few batch
sizes and horizons, printed as it goes.  Usage: python tools/sqp_timing.py"""
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


for N in (30, 50):
    for b in (1, 64, 1024, 4096):
        ctl = MPCController(N, 0.08, VehicleParameters())
        sqp = SqpSolver(ctl, b)
        rng = np.random.default_rng(1)
        X0 = torch.as_tensor(np.stack([rng.uniform(-.8, .8, b), rng.uniform(-.4, .4, b),
                                       rng.uniform(-.5, .5, b), rng.uniform(-.2, .2, b)], -1),
                             dtype=torch.float64, device=ctl.device)
        sqp.reset()
        for _ in range(3):
            sqp.iterate(X0)
        torch.cuda.synchronize()
        A, B, c, Xr = batched.bicycle_rti(X0, sqp.U, ctl.params, ctl.ts, states=True)
        H2, q2 = batched.bicycle_hessian(Xr, sqp.U, sqp.pi, ctl.params, ctl.ts, mu=sqp.mu)
        box = ctl._box()
        t_rti = ms(lambda: batched.bicycle_rti(X0, sqp.U, ctl.params, ctl.ts, states=True))
        t_h = ms(lambda: batched.bicycle_hessian(Xr, sqp.U, sqp.pi, ctl.params, ctl.ts, mu=sqp.mu))
        t_ipm = ms(lambda: batched.mpc_ipm(A, B, ctl.Q, ctl.R, ctl.QN, N, X0, lb=ctl.lbz, ub=ctl.ubz,
                                           c=c, tv=True, H2=H2, q2=q2, **box))
        t_it = ms(lambda: sqp.iterate(X0))
        r = batched.mpc_ipm(A, B, ctl.Q, ctl.R, ctl.QN, N, X0, lb=ctl.lbz, ub=ctl.ubz, c=c, tv=True,
                            H2=H2, q2=q2, **box)
        it = ((r["status"] >> 8) & 0xFFFF).double()
        print(f"N={N} b={b}: rti {t_rti:.3f} ms, hess {t_h:.3f} ms, ipm {t_ipm:.3f} ms "
              f"(iters mean {it.mean().item():.1f} max {it.max().item():.0f}), "
              f"sqp iteration {t_it:.3f} ms", flush=True)
