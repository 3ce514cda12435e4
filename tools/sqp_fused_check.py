"""The one-launch SQP (SqpSolver.solve, mpcqp_bicycle_sqp_solve) against the
batched iteration (SqpSolver.iterate) on the nlp bench's initial states:
convergence counts, input agreement, wall time of each (GPU).

    python tools/sqp_fused_check.py [--iters 60] [--batch 4096]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from model_predictive_control_amd._native import SQP_DONE  # noqa: E402
from model_predictive_control_amd.mpc import MPCController, SqpSolver  # noqa: E402
from model_predictive_control_amd.parameters import VehicleParameters  # noqa: E402
from tools.sqp_straggler import bench_x0  # noqa: E402

GOLD = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


def timed(fn):
    torch.cuda.synchronize()
    t = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return time.perf_counter() - t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=60)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--hessian", default="exact")
    a = ap.parse_args()
    ctl = MPCController(30, 0.08, VehicleParameters(), tol=1e-9, hessian=a.hessian)
    X0 = bench_x0(a.batch, 1)
    x0 = torch.as_tensor(X0, dtype=torch.float64, device="cuda")
    b = X0.shape[0]
    res = {}
    for mode in ("iterate", "fused", "fused"):
        sqp = SqpSolver(ctl, b)
        sqp.reset()
        if mode == "fused":
            dt = timed(lambda: sqp.solve(x0, a.iters))
        else:
            def run():
                for _ in range(a.iters):
                    sqp.iterate(x0)
            dt = timed(run)
        ok = sqp.done().cpu().numpy()
        it = sqp.iters().cpu().numpy()
        res[mode] = (sqp.U.reshape(b, -1).cpu().numpy(), ok, it, sqp.kkt.cpu().numpy())
        print(json.dumps(dict(mode=mode, secs=round(dt, 4), converged=int(ok.sum()),
                              rate=round(float(ok.sum()) / dt, 1), iters_mean=round(float(it.mean()), 2),
                              iters_max=int(it.max()), kkt_max=float(res[mode][3].max()))), flush=True)
    Ui, oki, iti, _ = res["iterate"]
    Uf, okf, itf, _ = res["fused"]
    both = oki & okf
    d = np.abs(Ui - Uf).max(1)
    print(json.dumps(dict(both=int(both.sum()), only_iter=int((oki & ~okf).sum()),
                          only_fused=int((okf & ~oki).sum()),
                          dU_max_both=float(d[both].max()) if both.any() else None,
                          dU_p99_both=float(np.percentile(d[both], 99)) if both.any() else None,
                          n_dU_gt_1e7=int((d[both] > 1e-7).sum()),
                          same_iters=int((iti[both] == itf[both]).sum()))), flush=True)
    # the NLP fixtures
    for f, kx, ku in (("nlp_tail.npz", "x0", "U"), ("nlp_s4.npz", "main_x0", "main_U")):
        g = np.load(os.path.join(GOLD, f))
        xf = torch.as_tensor(g[kx], dtype=torch.float64, device="cuda")
        sqp = SqpSolver(ctl, xf.shape[0])
        sqp.reset()
        sqp.solve(xf, 200)
        dev = np.abs(sqp.U.reshape(xf.shape[0], -1).cpu().numpy() - g[ku]).max(1)
        print(json.dumps(dict(fixture=f, dev_max=float(dev.max()), bad=int((dev > 1e-7).sum()),
                              iters=[int(v) for v in sqp.iters().cpu().numpy()],
                              done=int(sqp.done().sum()))), flush=True)


if __name__ == "__main__":
    main()
