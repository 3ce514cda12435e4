"""Time mpcqp_sweep on config-3 shaped data (n = 60, m = 120, full M, B = 65,536).

    python tools/sweep_probe.py [cfg]      # cfg 3 (default) or 5
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from model_predictive_control_amd import batched  # noqa: E402


class A:
    pass


cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
dev = torch.device("cuda")
a = A(); a.batch = 65536 if cfg == 3 else 32768; a.slots = 1; a.horizon = 0; a.reps = 1; a.check = 0
w = bench.CONFIGS[cfg](a, dev, 0)
if cfg == 3:
    d = batched.condense(w.A[0], w.B[0], w.Q_t, w.R_t, w.QN_t, w.N, x0=w.X0_t[0], c=w.c[0], tv=True,
                         outputs=("H", "Gam"))
    H, G = d["H"], d["Gam"]
else:
    d = batched.condense(w.A[0], w.B[0], w.Q_t, w.R_t, w.Q_t, w.N, x0=w.X0_t[0], tv=True, outputs=("H",))
    H, G = d["H"], None
fn = lambda: batched.sweep(H, G, full=True)  # noqa: E731
t = bench.time_kernel(fn, 10, dev)
print(f"cfg{cfg} sweep dbg={os.environ.get('MPCQP_SWEEP_DBG', '0')}: {t * 1e3:.1f} us")
