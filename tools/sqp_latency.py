"""Per-instance timing of the one-launch SQP (mpcqp_bicycle_sqp_solve) on the
nlp bench's initial states (GPU tool): the kernel records, per instance,
s_memrealtime ticks in all and in the QPs, interior-point iterations and SQP
iterations (the workspace's stats region).  Prints the launch time, the
distribution of per-instance solve times, the time per interior-point
iteration and the slowest instances.

    python tools/sqp_latency.py [--iters 60] [--batch 4096]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from model_predictive_control_amd.mpc import MPCController, SqpSolver  # noqa: E402
from model_predictive_control_amd.parameters import VehicleParameters  # noqa: E402
from tools.sqp_straggler import bench_x0  # noqa: E402

TICK_US = 0.01  # s_memrealtime runs at 100 MHz


def stats_of(sqp, b, N):
    """The kernel's per-instance stats (int64 x 4) from the solve workspace:
    after N*90 + 4 doubles per instance of stage data and outputs."""
    off = b * N * 90 + b * 4
    return sqp.ws.view(torch.float64)[off:off + 4 * b].view(torch.int64).view(b, 4).cpu().numpy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=60)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--hessian", default="exact")
    a = ap.parse_args()
    N = 30
    ctl = MPCController(N, 0.08, VehicleParameters(), tol=1e-9, hessian=a.hessian)
    X0 = bench_x0(a.batch, 1)
    x0 = torch.as_tensor(X0, dtype=torch.float64, device="cuda")
    b = X0.shape[0]
    sqp = SqpSolver(ctl, b)
    for rep in range(2):
        sqp.reset()
        torch.cuda.synchronize()
        t = time.perf_counter()
        sqp.solve(x0, a.iters)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
    st = stats_of(sqp, b, N)
    tot, tqp, ipm = (st[:, i].astype(float) for i in range(3))
    its, hits = (st[:, 3] & 0xFFFFFFFF).astype(float), (st[:, 3] >> 32).astype(float)
    ok = sqp.done().cpu().numpy()
    per_ipm = tqp / np.maximum(ipm, 1) * TICK_US
    per_sqp_other = (tot - tqp) / np.maximum(its, 1) * TICK_US
    q = lambda v: [round(float(np.percentile(v, p)), 1) for p in (50, 90, 99, 100)]  # noqa: E731
    print(json.dumps(dict(launch_ms=round(dt * 1e3, 2), converged=int(ok.sum()),
                          inst_us_p50_90_99_max=q(tot * TICK_US),
                          ipm_iter_us_p50_90_99_max=q(per_ipm),
                          sqp_overhead_us_per_iter=q(per_sqp_other),
                          ipm_iters_per_sqp_iter_mean=round(float(ipm.sum() / its.sum()), 2),
                          sqp_iters_mean=round(float(its.mean()), 2),
                          warm_qp_frac=round(float(hits.sum() / its.sum()), 3),
                          sum_inst_ms=round(float(tot.sum()) * TICK_US / 1e3, 1))), flush=True)
    if os.environ.get("MPCQP_LIB", "").endswith("passclk.so"):
        # the timing build's per-pass clocks: in the workspace after the stage data
        off = b * N * 70
        pc = sqp.ws.view(torch.float64)[off:off + 22 * b].view(torch.int64).view(b, 22).cpu().numpy()
        names = ["pass1_reductions", "pass2_fwd_predictor", "pass3_bwd_corrector_rhs",
                 "pass4_fwd_corrector", "polish", "failed_factorisation", "start", "warm_polish",
                 "pass1a_neighbours", "pass1b_stage_terms", "pass1c_factorisation",
                 "sqp_linearise", "sqp_hessian_and_stage_in", "sqp_step", "sqp_loop_head",
                 "step_merit_at_u", "step_dir_derivative", "step_line_search", "step_update",
                 "step_merit_lin_new_point", "step_adjoint", "step_kkt_flags"]
        totq = pc[:, :11].sum()
        print("PASSCLK", json.dumps({n: round(float(pc[:, i].sum() / totq), 3) for i, n in enumerate(names[:11])}),
              flush=True)
        # absolute: microseconds per interior-point iteration (all instances)
        print("PASSCLK_US_PER_IPM_ITER", json.dumps({n: round(float(pc[:, i].sum()) * TICK_US / max(1.0, ipm.sum()), 2)
                                                     for i, n in enumerate(names[:11])}), flush=True)
        print("SQPCLK_US_PER_SQP_ITER", json.dumps({n: round(float(pc[:, i].sum()) * TICK_US / max(1.0, its.sum()), 2)
                                                    for i, n in list(enumerate(names))[11:]}), flush=True)
    for i in np.argsort(-tot)[:8]:
        print(json.dumps(dict(inst=int(i), us=round(tot[i] * TICK_US, 1), qp_us=round(tqp[i] * TICK_US, 1),
                              ipm_iters=int(ipm[i]), sqp_iters=int(its[i]), ok=bool(ok[i]))), flush=True)


if __name__ == "__main__" and not os.environ.get("SQP_LAT_IPM"):
    main()


def ipm_alone(ctl, X0):
    """The stand-alone interior point (mpcqp_mpc_ipm, the quad kernel) on the
    Gauss-Newton QP at U = 0: launch time at batch 1 and at the full batch
    against the iteration counts -- the per-iteration latency without the
    one-launch kernel's register pressure."""
    from model_predictive_control_amd import batched

    out = []
    for b in (1, 64, X0.shape[0]):
        x0 = X0[:b]
        U = torch.zeros((b, ctl.N, 2), dtype=torch.float64, device="cuda")
        A, B, c = batched.bicycle_rti(x0, U, ctl.params, ctl.ts)
        box = ctl._box()
        run = lambda: batched.mpc_ipm(A, B, ctl.Q, ctl.R, ctl.QN, ctl.N, x0, lb=ctl.lbz,  # noqa: E731
                                      ub=ctl.ubz, c=c, tv=True, max_iter=25, **box)
        o = run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            o = run()
        e1.record()
        e1.synchronize()
        its = ((o["status"] >> 8) & 0xFFFF).cpu().numpy()
        ms = e0.elapsed_time(e1) / 5
        out.append(dict(b=b, ms=round(ms, 3), iters_max=int(its.max()), iters_mean=round(float(its.mean()), 2),
                        us_per_iter_of_max=round(ms * 1e3 / max(1, its.max()), 1)))
    print("IPM_ALONE", json.dumps(out), flush=True)


if __name__ == "__main__" and os.environ.get("SQP_LAT_IPM"):
    ctl = MPCController(30, 0.08, VehicleParameters(), tol=1e-9)
    ipm_alone(ctl, torch.as_tensor(bench_x0(4096, 1), dtype=torch.float64, device="cuda"))
