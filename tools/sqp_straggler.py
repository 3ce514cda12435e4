"""The SQP straggler tail of the nlp bench line (GPU diagnostics).

Runs mpc.SqpSolver on the nlp bench's own initial states (bench.py ConfigNLP:
seed 20261015 + 6, both slots) for --iters iterations, records per iteration
and instance the KKT residual, the flags word, the damping mu and the QP's
status word, and saves, for every instance that is not OPTIMAL after --budget
iterations (the bench's 60), its x0, its full trace and its inputs at the
budget and at the end, to gpurun_out/sqp_straggler.npz; prints the per-
iteration counts and a one-line classification per straggler.

    python tools/sqp_straggler.py --iters 300
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


def bench_x0(bsz=4096, slots=2, rank=0):
    """bench.py ConfigNLP.__init__: the x0 of every slot, (slots * bsz, 4)."""
    rng = np.random.default_rng(20261015 + 6 + 1000 * rank)
    S = slots
    X0 = np.stack([rng.uniform(-.8, .8, (S, bsz)), rng.uniform(-.4, .4, (S, bsz)),
                   rng.uniform(-.5, .5, (S, bsz)), rng.uniform(-.2, .2, (S, bsz))], -1)
    return X0.reshape(S * bsz, 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--budget", type=int, default=60)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--slots", type=int, default=2)
    ap.add_argument("--horizon", type=int, default=30)
    ap.add_argument("--out", default="gpurun_out/sqp_straggler.npz")
    a = ap.parse_args()
    X0 = bench_x0(a.batch, a.slots)
    b = X0.shape[0]
    ctl = MPCController(a.horizon, 0.08, VehicleParameters(), tol=1e-9)
    x0 = torch.as_tensor(X0, dtype=torch.float64, device="cuda")
    sqp = SqpSolver(ctl, b)
    sqp.reset()
    T = a.iters
    kk = torch.empty((T, b), dtype=torch.float64, device="cuda")
    fl = torch.empty((T, b), dtype=torch.int32, device="cuda")
    mu = torch.empty((T, b), dtype=torch.float64, device="cuda")
    qs = torch.empty((T, b), dtype=torch.int32, device="cuda")
    U_budget = None
    for it in range(T):
        sqp.iterate(x0)
        kk[it], fl[it], mu[it] = sqp.kkt, sqp.flags, sqp.mu
        qs[it] = sqp.qp["status"]
        if it + 1 == a.budget:
            U_budget = sqp.U.clone()
        if (it + 1) % 20 == 0:
            done = sqp.done()
            print(json.dumps(dict(it=it + 1, done=int(done.sum()),
                                  fail=int(((sqp.flags & SQP_FAIL) != 0).sum()),
                                  active=int(((sqp.flags & SQP_DONE) == 0).sum()))), flush=True)
        if bool((sqp.flags & SQP_DONE).all()):
            kk, fl, mu, qs = kk[:it + 1], fl[:it + 1], mu[:it + 1], qs[:it + 1]
            break
    torch.cuda.synchronize()
    flc = fl.cpu().numpy()
    ok = ((flc & SQP_DONE) != 0) & ((flc & SQP_FAIL) == 0)
    conv_it = np.where(ok.any(0), ok.argmax(0) + 1, -1)
    slow = np.nonzero((conv_it < 0) | (conv_it > a.budget))[0]
    print("SUMMARY", json.dumps(dict(batch=b, converged_budget=int(((conv_it > 0) & (conv_it <= a.budget)).sum()),
                                     converged_end=int((conv_it > 0).sum()), stragglers=int(slow.size),
                                     pct=[int(np.percentile(conv_it[conv_it > 0], q)) for q in (50, 90, 99, 99.9)])),
          flush=True)
    kkc, muc, qsc = kk.cpu().numpy(), mu.cpu().numpy(), qs.cpu().numpy()
    for i in slow:
        tr = flc[:, i]
        exact_from = int(np.argmax((tr & 2) != 0)) + 1 if ((tr & 2) != 0).any() else -1
        proj_its = int(((tr & 8) != 0).sum())
        qp_fail = int(((qsc[:, i] & 0xFF) != 0).sum())
        print(f"S {i:5d} conv {conv_it[i]:4d} kkt@{a.budget} {kkc[a.budget - 1, i]:.2e} "
              f"kkt_end {kkc[-1, i]:.2e} exact_from {exact_from:3d} proj_its {proj_its:3d} "
              f"qp_fail {qp_fail:3d} mu_end {muc[-1, i]:.1e} x0 {np.array2string(X0[i], precision=4)}",
              flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    np.savez(a.out, x0=X0[slow], idx=slow, conv_it=conv_it, kkt=kkc[:, slow], flags=flc[:, slow],
             mu=muc[:, slow], qp_status=qsc[:, slow], U_budget=U_budget.cpu().numpy()[slow],
             U_end=sqp.U.cpu().numpy()[slow], y_end=sqp.y.cpu().numpy()[slow])


if __name__ == "__main__":
    main()
