"""Config-5 condensing alone (condense_mfma_fh_kernel, B = 32,768, outputs H
and f as in mpcqp_mpc_qp): time it, or run 5 launches for a rocprofv3 --pmc
pass.  With MPCQP_LIB pointing at an A/B build (tools/ab_build.sh; the
MPCQP_FH_* timing-probe macros of condense.hip) it times that build.

    python tools/condense5_probe.py [pmc]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from model_predictive_control_amd import batched  # noqa: E402


class _A:
    pass


a = _A()
a.batch, a.slots, a.horizon, a.reps, a.check = 32768, 1, 0, 20, 0
dev = torch.device("cuda")
w = bench.Config5(a, dev, 0)
out = {}
fn = lambda: batched.condense(w.A[0], w.B[0], w.Q_t, w.R_t, w.Q_t, w.N, x0=w.X0_t[0],  # noqa: E731
                              tv=True, outputs=("H", "f"), out=out)
out.update(fn())
if len(sys.argv) > 1 and sys.argv[1] == "pmc":
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
else:
    ms = bench.time_kernel(fn, 20, dev)
    nb = bench.condense_bytes_survey(12, 4, 40, 4, False) * a.batch
    print(f"condense cfg5 {ms * 1e3:.1f} us  {nb / ms / 1e6:.1f} GB/s (8(d) bytes) "
          f"= {nb / ms / 1e6 / 8000:.3f} of HBM")
