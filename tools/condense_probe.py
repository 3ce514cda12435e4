"""Config-3 condense: device time vs output set (is it write-bandwidth bound?)."""
import sys, os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
from model_predictive_control_amd import batched

class A: pass
a = A(); a.batch = int(sys.argv[1]) if len(sys.argv) > 1 else 65536; a.slots = 1; a.horizon = 0; a.reps = 10
w = bench.Config3(a, torch.device("cuda"), 0)
for outs in (("H",), ("H", "f"), ("H", "f", "xbar"), ("H", "f", "Gam", "xbar")):
    o = {k: w.out[k] for k in outs}
    fn = lambda: batched.condense(w.A[0], w.B[0], w.Q_t, w.R_t, w.QN_t, w.N, x0=w.X0_t[0], c=w.c[0],
                                  tv=True, outputs=outs, out=o)
    ms = bench.time_kernel(fn, 10, torch.device("cuda"))
    nb = bench.condense_bytes_per_instance(4, 2, 30, 4, tv=True, gam="Gam" in outs, xbar="xbar" in outs,
                                           f="f" in outs) * a.batch
    print(f"{'+'.join(outs):18s} {ms*1e3:9.1f} us  {nb/1e6:8.1f} MB  {nb/ms/1e6:7.1f} GB/s")
