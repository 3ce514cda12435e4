"""Save the converged inputs of the nlp bench batch (one knob setting per
process, from the environment) to compare which local minimum each instance
ends in across settings: python tools/sqp_minima.py OUT.npz"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from model_predictive_control_amd.mpc import MPCController, SqpSolver  # noqa: E402
from model_predictive_control_amd.parameters import VehicleParameters  # noqa: E402
from tools.sqp_straggler import bench_x0  # noqa: E402

ctl = MPCController(30, 0.08, VehicleParameters(), tol=1e-9)
X0 = bench_x0(4096, 1)
x0 = torch.as_tensor(X0, dtype=torch.float64, device="cuda")
sqp = SqpSolver(ctl, X0.shape[0])
sqp.reset()
sqp.solve(x0, 150)
torch.cuda.synchronize()
np.savez(sys.argv[1], U=sqp.U.reshape(X0.shape[0], -1).cpu().numpy(), done=sqp.done().cpu().numpy(),
         J=np.zeros(1))
print("saved", sys.argv[1], flush=True)
