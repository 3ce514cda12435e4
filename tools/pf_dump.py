"""GPU debug: config-3 instances where the product-form path disagrees with
the workgroup path; dumps the worst instance's data and swept matrix."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from model_predictive_control_amd import batched
import bench


class A:
    pass


a = A(); a.batch = 512; a.slots = 1; a.horizon = 0; a.reps = 1
w = bench.CONFIGS[3](a, torch.device("cuda"), 0)
d = batched.condense(w.A[0], w.B[0], w.Q_t, w.R_t, w.QN_t, w.N, x0=w.X0_t[0], c=w.c[0], tv=True,
                     outputs=("H", "f", "Gam", "xbar"))
hl = w.xmin_t - d["xbar"]
hu = w.xmax_t - d["xbar"]
args = (d["H"], d["f"], d["Gam"], hl, hu, w.lbz, w.ubz)
z1, y1, s1 = batched.solve_qp(*args)
z2, y2, s2 = batched.solve_qp(*args, presweep=False)
d64 = {k: v.double() for k, v in d.items()}
z3, y3, s3 = batched.solve_qp(d64["H"], d64["f"], d64["Gam"], hl.double(), hu.double(), w.lbz.double(), w.ubz.double())
M, sst = batched.sweep(d["H"], d["Gam"], full=True)
torch.cuda.synchronize()
e1 = (z1.double() - z3).abs().max(1).values
e2 = (z2.double() - z3).abs().max(1).values
print("pf  : max", e1.max().item(), "n>1e-3", int((e1 > 1e-3).sum()))
print("wg  : max", e2.max().item(), "n>1e-3", int((e2 > 1e-3).sum()))
print("iters pf", (s1 >> 8).float().mean().item(), "wg", (s2 >> 8).float().mean().item())
bad = torch.nonzero(e1 > 1e-3).flatten().tolist()
print("bad", bad[:20], "codes", (s1[bad] & 0xff).tolist()[:20], "iters", (s1[bad] >> 8).tolist()[:20], (s2[bad] >> 8).tolist()[:20])
if bad:
    i = max(bad, key=lambda j: e1[j].item())
    np.savez("gpurun_out/pf_bad.npz", H=d["H"][i].cpu().numpy(), f=d["f"][i].cpu().numpy(),
             G=d["Gam"][i].cpu().numpy(), hl=hl[i].cpu().numpy(), hu=hu[i].cpu().numpy(),
             lb=w.lbz.cpu().numpy(), ub=w.ubz.cpu().numpy(), M=M[i].cpu().numpy(),
             z_pf=z1[i].cpu().numpy(), z_wg=z2[i].cpu().numpy(), z64=z3[i].cpu().numpy(),
             st_pf=s1[i].item(), st_wg=s2[i].item())
    print("dumped", i, e1[i].item())
