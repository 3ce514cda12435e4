"""Benchmark: QP solves/sec of the batched condensed-QP MPC step on MI355X.

Workload (BASELINE.json configs[1], the config the metric is quoted on):
double integrator of session_1/FHC.py:136-142 (Ts=0.5, Q=CC'+1e-3I, R=0.1,
P_f=Q), horizon N=20, input box |u|<=1, batch 4096 random x0 ~ U(-10,10)^2
per GPU, fp64.  One step = one pass of the hot path over one batch:

  --mode fused (default)
    mpcqp_mpc_box    per-instance (A, B, x0) -> z, status          [HIP, 1 launch]
  --mode split
    mpcqp_condense   per-instance (A, B, x0) -> H (packed), f     [HIP]
    mpcqp_solve_box  -> z, status                                 [HIP]

A and B are stored per instance (copies of the config-2 plant) so the
condensing really runs per instance, as the north star's "synthetic
(A,B,Q,R,x0)" asks; Q, R, Qf are shared.  Inputs are resident in HBM before
the timed region; steps cycle over 8 distinct x0 batches.  The step is
captured once per batch slot into a HIP graph (torch.cuda.CUDAGraph) and
replayed -- the kernels recompute everything on every replay.

Multi-GPU (torchrun): each rank owns its own batch (weak scaling), no
collective on the solve path; barrier + synchronize around the timed region,
max over ranks.

Prints ONE JSON line on rank 0 (see DESIGN.md "Measurement").
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from model_predictive_control_amd import batched  # noqa: E402
from model_predictive_control_amd import distributed as mdist  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FP64_PEAK_TFS = 78.6       # FP64 vector/matrix peak


def config2_plant():
    ts = 0.5
    A = np.array([[1.0, ts], [0.0, 1.0]])
    B = np.array([[0.0], [-ts]])
    C = np.array([[1.0], [-2.0 / 3.0]])
    Q = C @ C.T + 1e-3 * np.eye(2)
    R = np.array([[0.1]])
    return A, B, Q, R, Q.copy()


def condense_bytes_per_instance(nx, nu, N, es=8):
    """Algorithmic HBM bytes of mpcqp_condense per instance: in A, B, x0;
    out H (packed lower), f  (SURVEY.md 8d formula with F replaced by f)."""
    n = N * nu
    return (nx * nx + nx * nu + nx + n * (n + 1) // 2 + n) * es


def condense_flops_per_instance(nx, nu, N):
    """SURVEY.md 8d algorithmic flop formula (Gamma recursion + Gam'QGam + F + Phi)."""
    n, m = N * nu, N * nx
    return N * (N + 1) // 2 * 2 * nx * nx * nu + m * n + m * n * n + 2 * n * m * nx + 2 * N * nx ** 3


def solve_bytes_per_instance(n, es=8):
    return (n * (n + 1) // 2 + n + n) * es + 4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=4096, help="instances per GPU per step")
    ap.add_argument("--horizon", type=int, default=20)
    ap.add_argument("--slots", type=int, default=8, help="distinct x0 batches cycled over")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=50)
    ap.add_argument("--mode", choices=("fused", "split"), default="fused")
    ap.add_argument("--traffic", default=None,
                    help="JSON with PMC-measured HBM bytes per launch {kernel: bytes} "
                         "(tools/prof_counters.sh); fills roofline.traffic")
    args = ap.parse_args()

    rank, world, local = mdist.env_rank_world()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=dev)

    A, B, Q, R, Qf = config2_plant()
    nx, nu, N = 2, 1, args.horizon
    n = N * nu
    bsz, S = args.batch, args.slots
    dt = torch.float64
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)  # noqa: E731
    rng = np.random.default_rng(20261015 + 2 + 1000 * rank)
    X0 = rng.uniform(-10.0, 10.0, size=(S, bsz, nx))
    A_b = t(np.broadcast_to(A, (bsz, nx, nx)))
    B_b = t(np.broadcast_to(B, (bsz, nx, nu)))
    Q_t, R_t, Qf_t = t(Q), t(R), t(Qf)
    X0_t = t(X0)
    lb = torch.full((n,), -1.0, dtype=dt, device=dev)
    ub = torch.full((n,), 1.0, dtype=dt, device=dev)
    H = torch.empty((S, bsz, n * (n + 1) // 2), dtype=dt, device=dev)
    f = torch.empty((S, bsz, n), dtype=dt, device=dev)
    Z = torch.empty((S, bsz, n), dtype=dt, device=dev)
    ST = torch.empty((S, bsz), dtype=torch.int32, device=dev)

    def step_split(s):
        batched.condense(A_b, B_b, Q_t, R_t, Qf_t, N, x0=X0_t[s], outputs=("H", "f"),
                         out={"H": H[s], "f": f[s]})
        batched.solve_box(H[s], f[s], lb, ub, out=(Z[s], ST[s]))

    def step_fused(s):
        batched.mpc_box(A_b, B_b, Q_t, R_t, Qf_t, N, X0_t[s], lb, ub, out=(Z[s], ST[s]))

    step = step_fused if args.mode == "fused" else step_split

    # warm the JIT-free path once per slot, then capture
    for s in range(S):
        step(s)
    torch.cuda.synchronize()
    graphs = None
    if not args.no_graph:
        try:
            graphs = []
            cap = torch.cuda.Stream(device=dev)
            for s in range(S):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=cap):
                    step(s)
                graphs.append(g)
            torch.cuda.synchronize()
        except Exception as e:  # pragma: no cover - reported in the JSON
            print(f"graph capture failed ({e}); eager launches", file=sys.stderr)
            graphs = None

    def run(k):
        if graphs is not None:
            graphs[k % S].replay()
        else:
            step(k % S)

    for k in range(args.warmup):
        run(k)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        run(k)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = mdist.max_over_ranks(elapsed, dev)
    value = world * bsz * args.steps / elapsed

    # ---- correctness of what was timed: statuses + oracle spot check (rank 0)
    code = batched.status_code(ST)
    opt_frac = float((code == 0).double().mean())
    iters = batched.status_iters(ST).double()

    # ---- per-kernel durations with HIP events on the launch stream (eager)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    tc = ts_ = tf = 0.0
    P = args.profile_steps
    Zc = torch.empty_like(Z[0])
    STc = torch.empty_like(ST[0])
    for k in range(P):
        s = k % S
        ev[0].record()
        batched.condense(A_b, B_b, Q_t, R_t, Qf_t, N, x0=X0_t[s], outputs=("H", "f"),
                         out={"H": H[s], "f": f[s]})
        ev[1].record()
        batched.solve_box(H[s], f[s], lb, ub, out=(Zc, STc))
        ev[2].record()
        batched.mpc_box(A_b, B_b, Q_t, R_t, Qf_t, N, X0_t[s], lb, ub, out=(Z[s], ST[s]))
        ev[3].record()
        ev[3].synchronize()
        tc += ev[0].elapsed_time(ev[1])
        ts_ += ev[1].elapsed_time(ev[2])
        tf += ev[2].elapsed_time(ev[3])
    cond_ms, solve_ms, fused_ms = tc / P, ts_ / P, tf / P
    split_vs_fused = float((Zc - Z[(P - 1) % S]).abs().max())

    out = None
    if rank == 0:
        traffic = {}
        if args.traffic:
            with open(args.traffic) as fh:
                traffic = json.load(fh)
        cb_bytes = condense_bytes_per_instance(nx, nu, N) * bsz
        sv_bytes = solve_bytes_per_instance(n) * bsz
        cond_gbs = cb_bytes / (cond_ms * 1e-3) / 1e9
        solve_gbs = sv_bytes / (solve_ms * 1e-3) / 1e9
        roof_cond = {"kernel": "condense_kernel<double,2>", "bound": "hbm", "achieved": round(cond_gbs, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(cond_gbs / HBM_PEAK_GBS, 4),
                     "traffic": traffic.get("condense"), "bytes_per_launch": cb_bytes,
                     "avg_launch_us": round(cond_ms * 1e3, 2)}
        roof_solve = {"kernel": "box_gi_kernel<double,3>", "bound": "hbm", "achieved": round(solve_gbs, 1),
                      "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(solve_gbs / HBM_PEAK_GBS, 4),
                      "traffic": traffic.get("solve_box"), "bytes_per_launch": sv_bytes,
                      "avg_launch_us": round(solve_ms * 1e3, 2)}
        # fused kernel: SURVEY.md 8(d) per-instance figure (22.0 kflop condense,
        # config 2) against the fp64 peak; it moves only A, B, x0 in and z out.
        fl = condense_flops_per_instance(nx, nu, N) * bsz
        fused_tfs = fl / (fused_ms * 1e-3) / 1e12
        roof_fused = {"kernel": "mpc_box_kernel<double,2,1,3>", "bound": "mfma", "achieved": round(fused_tfs, 3),
                      "peak": FP64_PEAK_TFS, "unit": "TFLOP/s", "frac": round(fused_tfs / FP64_PEAK_TFS, 4),
                      "traffic": traffic.get("mpc_box"), "flops_per_launch": fl,
                      "hbm_bytes_per_launch": (nx * nx + nx * nu + nx + n) * 8 * bsz + 4 * bsz,
                      "avg_launch_us": round(fused_ms * 1e3, 2)}
        if args.mode == "fused":
            roofline = roof_fused
        else:
            roofline = roof_solve if solve_ms >= cond_ms else roof_cond
        # oracle spot check of the timed outputs (first 256 instances of slot 0)
        from oracle import cbaseline as cbl

        nchk = min(256, bsz)
        zr, _ = cbl.mpc_box(A, B, Q, R, Qf, N, X0[0, :nchk], -1.0, 1.0, nthreads=1)
        err = float(np.abs(Z[0, :nchk].cpu().numpy() - zr).max())
        cpu = None
        if not args.no_cpu and world == 1:
            cores = min(16, len(os.sched_getaffinity(0)))
            Xc = X0.reshape(-1, nx)
            done = 0
            tc0 = time.perf_counter()
            while time.perf_counter() - tc0 < args.cpu_seconds:
                cbl.mpc_box(A, np.broadcast_to(B, (bsz, nx, nu)), Q, R, Qf, N, Xc[:bsz], -1.0, 1.0,
                            nthreads=cores)
                done += bsz
            cdt = time.perf_counter() - tc0
            cpu = {"value": round(done / cdt, 1), "unit": "solves/s", "cores": cores, "kind": "port",
                   "sample": f"{done} config-2 solves (per-instance condense + GI box QP, C/OpenMP "
                             f"oracle/c/mpcqp_oracle.c) in {cdt:.1f} s on {cores} host threads"}
        out = {
            "metric": "QP solves/sec (batch, horizon N=20) at 1/2/4/8 MI355X; max|u-u_ref|",
            "value": round(value, 1),
            "unit": "solves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": "cfg2: per-instance condense + box QP, FHC.py double integrator "
                                   "(ts=0.5), N=20, |u|<=1, x0~U(-10,10)^2",
                       "batch_per_gpu": bsz, "horizon": N, "nx": nx, "nu": nu,
                       "parallelism": f"dp{world}", "graph": graphs is not None,
                       "mode": args.mode},
            "max_abs_u_err_vs_oracle": err,
            "optimal_frac": opt_frac,
            "iters_mean": round(float(iters.mean()), 2),
            "iters_max": int(iters.max()),
            "kernel_us": {"mpc_box": round(fused_ms * 1e3, 2), "condense": round(cond_ms * 1e3, 2),
                          "solve_box": round(solve_ms * 1e3, 2)},
            "split_vs_fused_max_abs": split_vs_fused,
            "roofline": roofline,
            "roofline_condense": roof_cond,
            "roofline_solve_box": roof_solve,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
