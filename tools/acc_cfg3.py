"""Accuracy diagnosis of the config-3 MPC step (mpcqp_mpc_qp, fp32) against
the fp64 oracle on the same fp32-valued inputs: error distribution over the
first K instances and, for the worst ones, how the active sets differ.

GPU box:  python tools/acc_cfg3.py [K [BATCH]]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from model_predictive_control_amd import batched  # noqa: E402
from oracle import condense as oc  # noqa: E402
from oracle import qp as oq  # noqa: E402


class A:
    pass


K = int(sys.argv[1]) if len(sys.argv) > 1 else 256
BATCH = int(sys.argv[2]) if len(sys.argv) > 2 else 65536  # the bench's x0 draws depend on it
a = A(); a.batch = max(K, BATCH); a.slots = 1; a.horizon = 0; a.reps = 1; a.check = 0
w = bench.Config3(a, torch.device("cuda"), 0)
w.step(0)
torch.cuda.synchronize()
r = lambda t: t.double().cpu().numpy()  # noqa: E731
Av, Bv, cv, X0 = r(w.A[0]), r(w.B[0]), r(w.c[0]), r(w.X0_t[0])
Q, QN, Rm = r(w.Q_t), r(w.QN_t), r(w.R_t)
xlo, xhi, lb, ub = r(w.xmin_t), r(w.xmax_t), r(w.lbz), r(w.ubz)
Z, Y = r(w.Z[0]), r(w.Y)
N = w.N
errs = []
info = []
for i in range(K):
    d = oc.condense(Av[i], Bv[i], Q, Rm, QN, N, x0=X0[i], c=cv[i])
    G = np.vstack([d["Gam"], -d["Gam"]])
    h = np.concatenate([xhi - d["xbar"], -(xlo - d["xbar"])])
    zr, lam, _ = oq.poly_qp(d["H"], d["f"], G, h, lb, ub)
    e = np.abs(Z[i] - zr).max()
    errs.append(e)
    xs_gpu = d["xbar"] + d["Gam"] @ Z[i]
    xs_ref = d["xbar"] + d["Gam"] @ zr
    viol = max((xs_gpu - xhi).max(), (xlo - xs_gpu).max(), (Z[i] - ub).max(), (lb - Z[i]).max())
    act_ref = set(np.nonzero(np.abs(lam) > 1e-9)[0].tolist())
    info.append((e, i, viol, len(act_ref), int((np.abs(Y[i]) > 0).sum()),
                 float(np.abs(xs_gpu - xs_ref).max())))
errs = np.array(errs)
print(f"K={K} max {errs.max():.3e} p99 {np.quantile(errs, .99):.3e} median {np.median(errs):.3e}")
for e, i, viol, na, ng, dx in sorted(info, reverse=True)[:8]:
    print(f"  inst {i:4d} err {e:.3e}  gpu max viol {viol:.3e}  |act oracle| {na}  "
          f"gpu rows with y!=0 {ng}  max|dx| {dx:.3e}")

# the worst instance in detail: where z differs, the bound status on both
# sides and the gradient of the GPU point (H z + f + Gam'y; y from the GPU)
e, i = max((x[0], x[1]) for x in info)
d = oc.condense(Av[i], Bv[i], Q, Rm, QN, N, x0=X0[i], c=cv[i])
G = np.vstack([d["Gam"], -d["Gam"]])
h = np.concatenate([xhi - d["xbar"], -(xlo - d["xbar"])])
zr, lam, _ = oq.poly_qp(d["H"], d["f"], G, h, lb, ub)
g = d["H"] @ Z[i] + d["f"] + d["Gam"].T @ Y[i]
gr = d["H"] @ zr + d["f"]
m2 = G.shape[0]
lam_rows = lam[:m2]
lam_ub = lam[m2:m2 + len(zr)]
lam_lb = lam[m2 + len(zr):]
print(f"worst inst {i}: oracle active rows {np.nonzero(lam_rows > 1e-12)[0].tolist()}")
print(f"  oracle row multipliers {lam_rows[lam_rows > 1e-12]}")
print(f"  gpu y nonzero {np.nonzero(Y[i])[0].tolist()} values {Y[i][Y[i] != 0]}")
for j in np.argsort(-np.abs(Z[i] - zr))[:8]:
    print(f"  z[{j:2d}] gpu {Z[i][j]: .9f} ref {zr[j]: .9f}  lb {lb[j]: .4f} ub {ub[j]: .4f}  "
          f"g_gpu {g[j]: .3e}  lam_ub {lam_ub[j]:.3e} lam_lb {lam_lb[j]:.3e}")
