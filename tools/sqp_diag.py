"""SQP convergence diagnostics on the nlp bench's x0 distribution (GPU).

Runs mpc.SqpSolver for --iters iterations per Hessian mode on a batch of the
bench's initial states and prints, per iteration, how many instances are
done / failed / in exact mode / projected, how many QPs failed and how many
steps raised the damping (a shortened step or a failed QP).  Writes the
per-instance convergence iteration and the x0 of the slow ones to
gpurun_out/sqp_diag_<mode>.npz.

    python tools/sqp_diag.py --modes exact,exact-raw,gauss-newton --iters 120
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from model_predictive_control_amd import batched  # noqa: E402
from model_predictive_control_amd._native import SQP_DONE, SQP_FAIL  # noqa: E402
from model_predictive_control_amd.mpc import MPCController, SqpSolver  # noqa: E402
from model_predictive_control_amd.parameters import VehicleParameters  # noqa: E402


def x0_batch(bsz, seed=20261015 + 6):
    rng = np.random.default_rng(seed)
    S = 1
    return np.stack([rng.uniform(-.8, .8, (S, bsz)), rng.uniform(-.4, .4, (S, bsz)),
                     rng.uniform(-.5, .5, (S, bsz)), rng.uniform(-.2, .2, (S, bsz))], -1)[0]


def run(mode, X0, iters, N, out_dir, trace=0):
    ctl = MPCController(N, 0.08, VehicleParameters(), tol=1e-9, hessian=mode)
    b = X0.shape[0]
    x0 = torch.as_tensor(X0, dtype=torch.float64, device="cuda")
    sqp = SqpSolver(ctl, b)
    if os.environ.get("DIAG_MU0"):
        sqp.MU0 = float(os.environ["DIAG_MU0"])
    sqp.reset()
    conv_it = torch.full((b,), -1, dtype=torch.int32, device="cuda")
    rows = []
    for it in range(1, iters + 1):
        mu_prev = sqp.mu.clone()
        fl_prev = sqp.flags.clone()
        sqp.iterate(x0)
        fl = sqp.flags
        active = (fl_prev & SQP_DONE) == 0
        done = ((fl & SQP_DONE) != 0) & ((fl & SQP_FAIL) == 0)
        conv_it = torch.where(done & (conv_it < 0), torch.full_like(conv_it, it), conv_it)
        qpst = batched.status_code(sqp.qp["status"])
        row = dict(it=it, done=int(done.sum()), fail=int(((fl & SQP_FAIL) != 0).sum()),
                   exact=int((active & ((fl & 2) != 0)).sum()),
                   proj=int((active & ((fl & 8) != 0)).sum()),
                   qp_fail=int((active & (qpst != 0)).sum()),
                   mu_up=int((active & (sqp.mu > mu_prev)).sum()))
        act = ~done & ((fl & SQP_FAIL) == 0)
        if act.any():
            k = sqp.kkt[act]
            row["kkt_q"] = [float(v) for v in torch.quantile(k.clamp(max=1e30), torch.tensor(
                [0.1, 0.5, 0.9], dtype=torch.float64, device="cuda"))]
        rows.append(row)
        if trace:
            al = torch.where(sqp.mu < mu_prev, 1.0, -1.0)
            for i in range(trace):
                print(f"T{i} it {it:3d} kkt {float(sqp.kkt[i]):.3e} fl {int(fl[i]) & 0xFF:2d} "
                      f"pc {(int(fl[i]) >> 24) & 0xF} qp {int(qpst[i])} qpit {(int(sqp.qp['status'][i]) >> 8) & 0xFFFF:3d} "
                      f"pol {(int(sqp.qp['status'][i]) >> 24) & 1} mu {float(sqp.mu[i]):.2e} full {int(al[i])} rho {float(sqp.rho[i]):.2e} "
                      f"u0 {float(sqp.U[i,0,0]):+.3f} {float(sqp.U[i,0,1]):+.3f}", flush=True)
        if it <= 40 or it % 10 == 0:
            print(mode, json.dumps(row), flush=True)
    ci = conv_it.cpu().numpy()
    ok = ci > 0
    summ = dict(mode=mode, converged=int(ok.sum()), batch=b,
                pct=[int(np.percentile(ci[ok], q)) for q in (50, 90, 95, 99)] if ok.any() else None,
                within30=int((ok & (ci <= 30)).sum()), within60=int((ok & (ci <= 60)).sum()))
    print("SUMMARY", json.dumps(summ), flush=True)
    np.savez(os.path.join(out_dir, f"sqp_diag_{mode}.npz"), conv_it=ci, x0=X0,
             U=sqp.U.cpu().numpy(), kkt=sqp.kkt.cpu().numpy(), flags=sqp.flags.cpu().numpy())
    return summ


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="exact,exact-raw,gauss-newton")
    ap.add_argument("--iters", type=int, default=120)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--horizon", type=int, default=30)
    ap.add_argument("--out", default="gpurun_out")
    ap.add_argument("--slow-from", default=None, help="npz of an earlier run: rerun its slow instances")
    ap.add_argument("--trace", type=int, default=0)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    X0 = x0_batch(a.batch)
    if a.slow_from:
        d = np.load(a.slow_from)
        ci = d["conv_it"]
        X0 = d["x0"][(ci < 0) | (ci > 60)]
    for m in a.modes.split(","):
        run(m, X0, a.iters, a.horizon, a.out, a.trace)


if __name__ == "__main__":
    main()
