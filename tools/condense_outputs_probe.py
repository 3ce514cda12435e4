"""Config-3 condensing (condense_kernel<float,4>, B = 65,536) timed per output set.

    python tools/condense_outputs_probe.py          # time H+f+Gam+xbar, H+f+xbar, H, H+Gam
    python tools/condense_outputs_probe.py pmc     # 5 launches of the mpc_qp output set (for rocprofv3 --pmc)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from model_predictive_control_amd import batched  # noqa: E402


class A:
    pass


a = A(); a.batch = 65536; a.slots = 1; a.horizon = 0; a.reps = 20; a.check = 0
w = bench.Config3(a, torch.device("cuda"), 0)
sets = [("H", "f", "Gam", "xbar"), ("H", "f", "xbar"), ("H",), ("H", "Gam")]
pmc = len(sys.argv) > 1 and sys.argv[1] == "pmc"
for outs in sets[:1] if pmc else sets:
    out = {}
    fn = lambda: batched.condense(w.A[0], w.B[0], w.Q_t, w.R_t, w.QN_t, w.N, x0=w.X0_t[0],  # noqa: E731
                                  c=w.c[0], tv=True, outputs=outs, out=out)
    fn()
    out.update(fn())
    if pmc:
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        continue
    t = bench.time_kernel(fn, 20, torch.device("cuda"))
    print(outs, round(t * 1e3, 1), "us")
