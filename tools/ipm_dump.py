"""Development probe: run the batched SQP of MPCController on the GPU and
save the QP data of every SQP iteration (A, B, c, H2, q2, U, flags) with the
interior point's status words to gpurun_out/ipm_dump.npz, for replay on the
host (tools/ipm_host.cpp).  Usage: python tools/ipm_dump.py [b] [N] [iters]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from model_predictive_control_amd import batched  # noqa: E402
from model_predictive_control_amd.mpc import MPCController, SqpSolver  # noqa: E402
from model_predictive_control_amd.parameters import VehicleParameters  # noqa: E402

b = int(sys.argv[1]) if len(sys.argv) > 1 else 256
N = int(sys.argv[2]) if len(sys.argv) > 2 else 30
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 8
ctl = MPCController(N, 0.08, VehicleParameters())
sqp = SqpSolver(ctl, b)
rng = np.random.default_rng(1)
X0 = torch.as_tensor(np.stack([rng.uniform(-.8, .8, b), rng.uniform(-.4, .4, b),
                               rng.uniform(-.5, .5, b), rng.uniform(-.2, .2, b)], -1),
                     dtype=torch.float64, device=ctl.device)
sqp.reset()
out = dict(X0=X0.cpu().numpy(), Q=ctl.Q.cpu().numpy(), R=ctl.R.cpu().numpy(),
           QN=ctl.QN.cpu().numpy(), lbz=ctl.lbz.cpu().numpy(), ubz=ctl.ubz.cpu().numpy())
box = ctl._box()
for k, v in box.items():
    out[k] = v.cpu().numpy()
for it in range(iters):
    A, B, c, Xr = batched.bicycle_rti(X0, sqp.U, ctl.params, ctl.ts, states=True)
    H2, q2 = batched.bicycle_hessian(Xr, sqp.U, sqp.pi, ctl.params, ctl.ts, flags=sqp.flags,
                                     mu=sqp.mu)
    if it < 12 or it % 10 == 0:
        for name, v in dict(A=A, B=B, c=c, H2=H2, q2=q2, U=sqp.U, flags=sqp.flags,
                            mu=sqp.mu).items():
            out[f"{name}_{it}"] = v.cpu().numpy()
    out[f"Ucur_{it}"] = sqp.U.cpu().numpy()
    sqp.iterate(X0)
    out[f"kkt_{it}"] = sqp.kkt.cpu().numpy()
    out[f"mu_after_{it}"] = sqp.mu.cpu().numpy()
    st = sqp.qp["status"].cpu().numpy()
    out[f"status_{it}"] = st
    its = (st >> 8) & 0xFFFF
    print(f"sqp it {it}: qp iters mean {its.mean():.1f} max {its.max()} "
          f"codes {np.bincount(st & 0xFF, minlength=5)} done {int(sqp.done().sum())}", flush=True)
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed("gpurun_out/ipm_dump.npz", **out)
