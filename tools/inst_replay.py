"""Debug probe: replay one config-3 full-batch instance (index argv[1]) at
b = 1 through mpc_qp fp32 (env knobs apply) and the generic fp32 path, and
print the error against the fp64 oracle."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from model_predictive_control_amd import batched  # noqa: E402
from model_predictive_control_amd.parameters import VehicleParameters  # noqa: E402
from oracle import condense as oc, qp as oq  # noqa: E402

dev = torch.device("cuda")
i = int(sys.argv[1])
b, N, ts = 65536, 30, 0.08
p = VehicleParameters()
rng = np.random.default_rng(20261015 + 3)
X0 = np.stack([rng.uniform(-1, 1, b), rng.uniform(-.5, .5, b),
               rng.uniform(-np.pi / 4, np.pi / 4, b), rng.uniform(-.3, .3, b)], -1)[i:i + 1]
x = torch.as_tensor(X0, dtype=torch.float64, device=dev)
A, B, c = batched.bicycle_rti(x, torch.zeros((1, N, 2), dtype=torch.float64, device=dev), p, ts)
Q = np.diag([1., 6., .2, .05]); R = np.diag([1., .01])
xlo = np.tile([p.min_pos_x, p.min_pos_y, p.min_heading, p.min_vel], N)
xhi = np.tile([p.max_pos_x, p.max_pos_y, p.max_heading, p.max_vel], N)
lb, ub = np.tile([p.min_drive, -p.max_steer], N), np.tile([p.max_drive, p.max_steer], N)
A, B, c, x = (t.to(torch.float32).contiguous() for t in (A, B, c, x))
t = lambda a: torch.as_tensor(np.asarray(a, float), dtype=torch.float32, device=dev)
r = lambda a: torch.as_tensor(np.asarray(a, float), dtype=torch.float32).double().numpy()
dd = oc.condense(A[0].double().cpu().numpy(), B[0].double().cpu().numpy(), r(Q), r(R), r(100 * Q), N,
                 x0=x[0].double().cpu().numpy(), c=c[0].double().cpu().numpy())
G = np.vstack([dd["Gam"], -dd["Gam"]])
h = np.concatenate([r(xhi) - dd["xbar"], -(r(xlo) - dd["xbar"])])
zr = oq.poly_qp(dd["H"], dd["f"], G, h, r(lb), r(ub))[0]
z, y, st = batched.mpc_qp(A, B, t(Q), t(R), t(100 * Q), N, x, xlo=t(xlo), xhi=t(xhi), lb=t(lb),
                          ub=t(ub), c=c, tv=True)
d = batched.condense(A, B, t(Q), t(R), t(100 * Q), N, x0=x, c=c, tv=True,
                     outputs=("H", "f", "Gam", "xbar"))
z2, _, st2 = batched.solve_qp(d["H"], d["f"], d["Gam"], t(xlo) - d["xbar"], t(xhi) - d["xbar"],
                              t(lb), t(ub))
z3, _, st3 = batched.solve_qp(d["H"], d["f"], d["Gam"], t(xlo) - d["xbar"], t(xhi) - d["xbar"],
                              t(lb), t(ub), presweep=False)
torch.cuda.synchronize()
env = {k: v for k, v in os.environ.items() if k.startswith("MPCQP_")}
print(i, env, "mpc_qp err", np.abs(z[0].double().cpu().numpy() - zr).max(), "st", int(st[0]),
      "| solve_qp(two-kernel) err", np.abs(z2[0].double().cpu().numpy() - zr).max(), "st", int(st2[0]),
      "| solve_qp(wg) err", np.abs(z3[0].double().cpu().numpy() - zr).max(), "st", int(st3[0]))
zz = z[0].double().cpu().numpy()
print("   z==lb:", int((zz == r(lb)).sum()), " z==ub:", int((zz == r(ub)).sum()), " y finite:",
      bool(torch.isfinite(y).all()), " y absmax", float(y.abs().max()))
M, sst = batched.sweep(d["H"], d["Gam"], full=True)
torch.cuda.synchronize()
Mn = M[0].double().cpu().numpy()
bad = np.argwhere(~np.isfinite(Mn))
print("   sweep status", int(sst[0]), "nonfinite M0 entries", len(bad), bad[:8].tolist())
Hd = oc.unpack_lower(d["H"][0].double().cpu().numpy(), 60)
Gd = d["Gam"][0].double().cpu().numpy()
K = np.block([[Hd, Gd.T], [Gd, np.zeros((120, 120))]])
Hi = np.linalg.inv(Hd)
Mref = np.block([[-Hi, Hi @ Gd.T], [Gd @ Hi, -Gd @ Hi @ Gd.T]])
fin = np.isfinite(Mn)
print("   max |M0 - ref| (finite)", float(np.abs(np.where(fin, Mn - Mref, 0)).max()), " cond(H)", np.linalg.cond(Hd))
# active sets: oracle vs the mpc_qp result
zf = z[0].double().cpu().numpy()
so = dd["xbar"] + dd["Gam"] @ zr
sf = dd["xbar"] + dd["Gam"] @ zf
def act(zv, sv, tz, ts_):
    az = set(np.where((zv <= r(lb) + tz) | (zv >= r(ub) - tz))[0].tolist())
    ar = set((np.where((sv <= r(xlo) + ts_) | (sv >= r(xhi) - ts_))[0] + 60).tolist())
    return az | ar
Ao, Af = act(zr, so, 1e-9, 1e-9), act(zf, sf, 1e-6, 1e-5)
print("   active oracle", sorted(Ao))
print("   active f32   ", sorted(Af), " only-oracle", sorted(Ao - Af), " only-f32", sorted(Af - Ao))
yy = y[0].double().cpu().numpy()
print("   f32 row multipliers (nonzero):", {int(j) + 60: round(float(yy[j]), 6) for j in np.nonzero(yy)[0]})
