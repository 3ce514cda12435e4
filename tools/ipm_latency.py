"""Latency of the fp64 stage-wise interior point (mpcqp_mpc_ipm) on
config-3 instances against the batch size: the cost model of the config-3
fallback (a few hundred instances per step).  GPU tool."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from model_predictive_control_amd import batched  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--sizes", default="1,16,64,256,675,4096")
a = ap.parse_args()
dev = torch.device("cuda")
args = argparse.Namespace(batch=4096, slots=1, horizon=30, reps=5, check=0)
C = bench.Config3(args, dev, 0)
for b in [int(v) for v in a.sizes.split(",")]:
    kw = dict(xlo=C.xmin_t, xhi=C.xmax_t, lb=C.lbz, ub=C.ubz, c=C.c[0][:b], tv=True)
    run = lambda: batched.mpc_ipm(C.A[0][:b], C.B[0][:b], C.Q_t, C.R_t, C.QN_t, C.N,  # noqa: E731
                                  C.X0_t[0][:b], **kw)
    o = run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        o = run()
    e1.record()
    e1.synchronize()
    its = ((o["status"] >> 8) & 0xFFFF).double()
    pol = ((o["status"] >> 24) & 1).double()
    print(f"b {b:5d} ms {e0.elapsed_time(e1) / 5:.3f} iters mean {float(its.mean()):.1f} "
          f"max {int(its.max())} polished {float(pol.mean()):.2f} "
          f"codes {np.unique(batched.status_code(o['status']).cpu().numpy())}", flush=True)
