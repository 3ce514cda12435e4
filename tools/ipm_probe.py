"""Development probe for counter runs: 8 SQP iterations of MPCController on
a batch, then 5 launches of the interior point on the QP of the final state
(strict, as SqpSolver runs it).  Usage: python tools/ipm_probe.py [b] [N]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from model_predictive_control_amd import batched  # noqa: E402
from model_predictive_control_amd.mpc import MPCController, SqpSolver  # noqa: E402
from model_predictive_control_amd.parameters import VehicleParameters  # noqa: E402

b = int(sys.argv[1]) if len(sys.argv) > 1 else 64
N = int(sys.argv[2]) if len(sys.argv) > 2 else 30
ctl = MPCController(N, 0.08, VehicleParameters())
sqp = SqpSolver(ctl, b)
rng = np.random.default_rng(1)
X0 = torch.as_tensor(np.stack([rng.uniform(-.8, .8, b), rng.uniform(-.4, .4, b),
                               rng.uniform(-.5, .5, b), rng.uniform(-.2, .2, b)], -1),
                     dtype=torch.float64, device=ctl.device)
sqp.reset()
for _ in range(8):
    sqp.iterate(X0)
A, B, c, Xr = batched.bicycle_rti(X0, sqp.U, ctl.params, ctl.ts, states=True)
H2, q2 = batched.bicycle_hessian(Xr, sqp.U, sqp.pi, ctl.params, ctl.ts, mu=sqp.mu)
kw = dict(lb=ctl.lbz, ub=ctl.ubz, c=c, tv=True, H2=H2, q2=q2, strict=True,
          max_iter=SqpSolver.QP_MAX_ITER, **ctl._box())
for _ in range(5):
    r = batched.mpc_ipm(A, B, ctl.Q, ctl.R, ctl.QN, N, X0, **kw)
torch.cuda.synchronize()
it = ((r["status"] >> 8) & 0xFFFF).double()
print(f"b={b} N={N}: qp iters mean {it.mean().item():.2f} max {it.max().item():.0f}", flush=True)
