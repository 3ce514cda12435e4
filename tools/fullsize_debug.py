"""Debug probe: config-3 full batch, fp32 product path vs fp64 path; the
worst instances against the fp64 oracle (which path is off)."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from model_predictive_control_amd import batched  # noqa: E402
from model_predictive_control_amd.parameters import VehicleParameters  # noqa: E402
from oracle import condense as oc, qp as oq  # noqa: E402

dev = torch.device("cuda")
b = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
N, ts = 30, 0.08
p = VehicleParameters()
rng = np.random.default_rng(20261015 + 3)
X0 = np.stack([rng.uniform(-1, 1, b), rng.uniform(-.5, .5, b),
               rng.uniform(-np.pi / 4, np.pi / 4, b), rng.uniform(-.3, .3, b)], -1)
x = torch.as_tensor(X0, dtype=torch.float64, device=dev)
A, B, c = batched.bicycle_rti(x, torch.zeros((b, N, 2), dtype=torch.float64, device=dev), p, ts)
Q = np.diag([1., 6., .2, .05]); R = np.diag([1., .01])
xlo = np.tile([p.min_pos_x, p.min_pos_y, p.min_heading, p.min_vel], N)
xhi = np.tile([p.max_pos_x, p.max_pos_y, p.max_heading, p.max_vel], N)
lb, ub = np.tile([p.min_drive, -p.max_steer], N), np.tile([p.max_drive, p.max_steer], N)
f32 = [t.to(torch.float32).contiguous() for t in (A, B, c, x)]
f64 = [t.double().contiguous() for t in f32]
def run(dt, A_, B_, c_, x_):
    t = lambda a: torch.as_tensor(np.asarray(a, float), dtype=torch.float32, device=dev).to(dt)
    return batched.mpc_qp(A_, B_, t(Q), t(R), t(100 * Q), N, x_, xlo=t(xlo), xhi=t(xhi),
                          lb=t(lb), ub=t(ub), c=c_, tv=True)
z32, _, st32 = run(torch.float32, *f32)
z64, _, st64 = run(torch.float64, *f64)
torch.cuda.synchronize()
d = (z32.double() - z64).abs().amax(1)
print("bad instances (>1e-5):", int((d > 1e-5).sum()), "of", b, " max", float(d.max()))
idx = torch.argsort(d, descending=True)[:6].cpu().numpy()
r = lambda a: torch.as_tensor(np.asarray(a, float), dtype=torch.float32).double().numpy()
Ah, Bh, ch, xh = (t.cpu().numpy() for t in f64)
for i in idx:
    dd = oc.condense(Ah[i], Bh[i], r(Q), r(R), r(100 * Q), N, x0=xh[i], c=ch[i])
    G = np.vstack([dd["Gam"], -dd["Gam"]])
    h = np.concatenate([r(xhi) - dd["xbar"], -(r(xlo) - dd["xbar"])])
    try:
        zr = oq.poly_qp(dd["H"], dd["f"], G, h, r(lb), r(ub))[0]
        e32 = np.abs(z32[i].double().cpu().numpy() - zr).max()
        e64 = np.abs(z64[i].cpu().numpy() - zr).max()
    except ValueError as e:
        e32 = e64 = str(e)
    print(i, "diff", float(d[i]), "st32", int(st32[i]), "st64", int(st64[i]), "err32", e32, "err64", e64)

# single-instance replays of the worst ones
for i in idx[:2]:
    sl = slice(int(i), int(i) + 1)
    zz, yy, ss = run(torch.float32, *(t[sl].contiguous() for t in f32))
    torch.cuda.synchronize()
    print("replay b=1", i, "diff vs f64", float((zz.double() - z64[sl]).abs().max()), "st", int(ss[0]))
    # 16 copies of it (same wave count pattern) and it placed at another index
    rep = [t[sl].repeat(*([64] + [1] * (t.dim() - 1))).contiguous() for t in f32]
    zz, yy, ss = run(torch.float32, *rep)
    torch.cuda.synchronize()
    print("replay b=64 copies: max diff", float((zz.double() - z64[sl]).abs().max()))
    dd = oc.condense(Ah[i], Bh[i], r(Q), r(R), r(100 * Q), N, x0=xh[i], c=ch[i])
    zf = z32[i].double().cpu().numpy(); z6 = z64[i].cpu().numpy()
    s = dd["xbar"] + dd["Gam"] @ zf; s6 = dd["xbar"] + dd["Gam"] @ z6
    print("  f32: z at bounds", int(((zf <= r(lb) + 1e-6) | (zf >= r(ub) - 1e-6)).sum()),
          "rows active", int(((s <= r(xlo) + 1e-5) | (s >= r(xhi) - 1e-5)).sum()),
          "max viol z", float(max((r(lb) - zf).max(), (zf - r(ub)).max())),
          "max viol rows", float(max((r(xlo) - s).max(), (s - r(xhi)).max())))
    print("  f64: z at bounds", int(((z6 <= r(lb) + 1e-9) | (z6 >= r(ub) - 1e-9)).sum()),
          "rows active", int(((s6 <= r(xlo) + 1e-8) | (s6 >= r(xhi) - 1e-8)).sum()))
    obj = lambda z: 0.5 * z @ dd["H"] @ z + dd["f"] @ z
    print("  objective f32", obj(zf), "f64", obj(z6))
