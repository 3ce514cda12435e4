"""Benchmark: QP solves/sec of the batched condensed-QP MPC step on MI355X.

Default workload: BASELINE.json configs[1], the config the metric is quoted on.
It is the double integrator of session_1/FHC.py:136-142 (Ts=0.5, Q=CC'+1e-3I,
R=0.1, P_f=Q), horizon N=20, input box |u|<=1, batch 4096 random
x0 ~ U(-10,10)^2 per GPU, fp64.  One step = one pass of the hot path over one
batch:

  --mode fused (default)
    mpcqp_mpc_box    per-instance (A, B, x0) -> z, status          [HIP, 1 launch]
  --mode split
    mpcqp_condense   per-instance (A, B, x0) -> H (packed), f     [HIP]
    mpcqp_solve_box  -> z, status                                 [HIP]

A and B are stored per instance (copies of the config-2 plant), so the
condensing really runs per instance, as the north star's "synthetic
(A,B,Q,R,x0)" asks.  Q, R and Qf are shared.

--config 3|4|5 runs the other BASELINE configs with the same
contract; they are parity/roofline cases and not the headline line:
  3  FE-linearised bicycle (parameters.py), N=30, ts=0.08, state box (x_1..x_N)
     + input box, per-instance per-stage (A_k, B_k, c_k), fp32, B=65,536:
     mpcqp_mpc_qp (condense(TV) + rows + MFMA sweep + product-form active set
     refined against the dynamics in fp64)
  4  random stable LTI nx=12, nu=4, N=50, 40 random polytope rows (h>0),
     shared condense, fp64, B=131,072 per GPU: f = F x0 + mpcqp_solve_poly
  5  config-4 plant perturbed per instance and stage, N=40, input box, fp32,
     B=32,768 per GPU: mpcqp_mpc_qp without state box (condense(TV, MFMA) +
     sweep + product-form active set, n = 160)

In every config the inputs are resident in HBM before the timed region, and
steps cycle over distinct x0 batches ("slots").  A round of S steps (slots
0..S-1 in order) is captured once into a HIP graph (torch.cuda.CUDAGraph) and
replayed K // S times, the remainder from one-step graphs (--no-chain: one
graph launch per step); the kernels recompute everything on every replay.

Per-kernel device times: HIP events around a graph of R back-to-back launches
of that kernel alone, on the stream the graph runs on.

Multi-GPU (torchrun): each rank owns its own batch (weak scaling), with no
collective on the solve path.  There is a barrier and a synchronize around
the timed region, and the time is the max over ranks.

Prints ONE JSON line on rank 0 ("Measurement").
"""
from __future__ import annotations

import argparse
import ctypes
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
FP32_PEAK_TFS = 157.3      # FP32 vector/matrix peak
METRIC = "QP solves/sec (batch, horizon N=20) at 1/2/4/8 MI355X; max|u-u_ref|"


# ------------------------------------------------------------- algorithmic counts
def condense_bytes_survey(nx, nu, N, es, state_box):
    """SURVEY.md 8(d) algorithmic bytes of condensing one instance, the count
    roofline.achieved uses: in A_k, B_k per stage + x0; out the packed upper
    triangle of H, F (n x nx), and -- only with state constraints -- Gamma's
    lower block triangle (nx nu N(N+1)/2) and Phi (N nx x nx).  Config 3:
    6,994 elements = 27,976 B; config 5: 22,492 = 89,968 B."""
    n, m = N * nu, N * nx
    inp = N * (nx * nx + nx * nu) + nx
    out = n * (n + 1) // 2 + n * nx
    if state_box:
        out += nx * nu * N * (N + 1) // 2 + m * nx
    return (inp + out) * es


def condense_bytes_per_instance(nx, nu, N, es=8, tv=False, gam=False, xbar=False,
                                F=False, f=True, drift=False):
    """HBM bytes mpcqp_condense actually moves per instance (reported beside
    the 8(d) count): inputs A, B (per stage when TV), c (drift), x0; outputs
    packed H, f and whatever else the workload asks for -- Gam as its lower
    block triangle (MPCQP_GAM_PACKED), xbar, F."""
    n, m = N * nu, N * nx
    S = N if tv else 1
    inp = S * (nx * nx + nx * nu) + nx + (N * nx if drift else 0)
    out = n * (n + 1) // 2 + (n if f else 0) + (nx * nu * N * (N + 1) // 2 if gam else 0) \
        + (m if xbar else 0) + (n * nx if F else 0)
    return (inp + out) * es


def condense_flops_per_instance(nx, nu, N):
    """SURVEY.md 8(d) algorithmic flop formula (Gamma recursion + Gam'QGam + F + Phi)."""
    n, m = N * nu, N * nx
    return N * (N + 1) // 2 * 2 * nx * nx * nu + m * n + m * n * n + 2 * n * m * nx + 2 * N * nx ** 3


def solve_bytes_per_instance(n, es=8, m=0, G=False):
    """QP solve: packed H, f, bounds in (shared bounds not counted), z +
    status out; per-instance G rows and row bounds when G."""
    return (n * (n + 1) // 2 + n + n) * es + 4 + ((m * n + 2 * m) * es if G else 0)


def sweep_flops_per_instance(n, m=0):
    """Dense symmetric inversion of H (Cholesky-based, n^3) plus G H^-1
    (2 m n^2) and the symmetric half of G H^-1 G' (m^2 n): the algorithmic
    flops of mpcqp_sweep's M = [[-H^-1, H^-1 G'], [G H^-1, -G H^-1 G']]."""
    return n ** 3 + 2 * m * n * n + m * m * n


STAGES = ("condense", "sweep", "solve", "fallback", "states")


def mpc_qp_stage_ms(fn, reps: int) -> dict:
    """Per-stage device time (ms) of one mpcqp_mpc_qp call, averaged over
    `reps` calls of fn(): HIP events the library records on the call's own
    stream around each stage (mpcqp_mpc_qp_profile / mpcqp_mpc_qp_stage_ms).
    Stages the call did not run are absent."""
    from model_predictive_control_amd import _native as nat
    lib = nat.load()
    nat.check(lib.mpcqp_mpc_qp_profile(1), "mpcqp_mpc_qp_profile")
    acc, cnt = np.zeros(len(STAGES)), np.zeros(len(STAGES))
    ms = (ctypes.c_float * len(STAGES))()
    try:
        fn()
        for _ in range(reps):
            fn()
            nat.check(lib.mpcqp_mpc_qp_stage_ms(ms), "mpcqp_mpc_qp_stage_ms")
            v = np.frombuffer(ms, dtype=np.float32).astype(float)
            acc += np.where(v >= 0, v, 0.0)
            cnt += v >= 0
    finally:
        nat.check(lib.mpcqp_mpc_qp_profile(0), "mpcqp_mpc_qp_profile")
    return {k: acc[i] / cnt[i] for i, k in enumerate(STAGES) if cnt[i] > 0}


def roof(kernel, bound, amount, ms, es_peak, unit, traffic=None, extra=None):
    achieved = amount / (ms * 1e-3) / (1e9 if unit == "GB/s" else 1e12)
    d = {"kernel": kernel, "bound": bound, "achieved": round(achieved, 3), "peak": es_peak,
         "unit": unit, "frac": round(achieved / es_peak, 5), "traffic": traffic,
         "avg_launch_us": round(ms * 1e3, 2)}
    d.update(extra or {})
    return d


def time_kernel(fn, reps: int, dev) -> float:
    """Average device time (ms) of fn() from HIP events around a graph of
    `reps` back-to-back launches replayed on its own stream."""
    st = torch.cuda.Stream(device=dev)
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        for _ in range(reps):
            fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    with torch.cuda.stream(st):
        for _ in range(3):
            e0.record(st)
            g.replay()
            e1.record(st)
            e1.synchronize()
            best = min(best, e0.elapsed_time(e1) / reps)
    return best


# ---------------------------------------------------------------- workloads
class Config2:
    """BASELINE configs[1]: FHC double integrator, N=20, |u|<=1, fp64."""

    dtype = torch.float64
    dname = "f64"
    default_batch = 4096
    default_slots = 8

    def __init__(self, args, dev, rank):
        self.args, self.dev = args, dev
        ts = 0.5
        A = np.array([[1.0, ts], [0.0, 1.0]])
        B = np.array([[0.0], [-ts]])
        C = np.array([[1.0], [-2.0 / 3.0]])
        Q = C @ C.T + 1e-3 * np.eye(2)
        self.A, self.B, self.Q, self.R, self.Qf = A, B, Q, np.array([[0.1]]), Q.copy()
        self.nx, self.nu, self.N = 2, 1, args.horizon or 20
        n = self.n = self.N
        bsz, S = args.batch, args.slots
        dt = self.dtype
        t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)  # noqa: E731
        rng = np.random.default_rng(20261015 + 2 + 1000 * rank)
        self.X0 = rng.uniform(-10.0, 10.0, size=(S, bsz, 2))
        self.A_b = t(np.broadcast_to(A, (bsz, 2, 2)))
        self.B_b = t(np.broadcast_to(B, (bsz, 2, 1)))
        self.Q_t, self.R_t, self.Qf_t = t(Q), t(self.R), t(Q)
        self.X0_t = t(self.X0)
        self.lb = torch.full((n,), -1.0, dtype=dt, device=dev)
        self.ub = torch.full((n,), 1.0, dtype=dt, device=dev)
        self.H = torch.empty((bsz, n * (n + 1) // 2), dtype=dt, device=dev)
        self.f = torch.empty((bsz, n), dtype=dt, device=dev)
        self.Z = torch.empty((S, bsz, n), dtype=dt, device=dev)
        self.ST = torch.empty((S, bsz), dtype=torch.int32, device=dev)
        self.Zs = torch.empty((bsz, n), dtype=dt, device=dev)
        self.STs = torch.empty((bsz,), dtype=torch.int32, device=dev)

    def workload(self):
        return {"workload": "cfg2: per-instance condense + box QP, FHC.py double integrator "
                            "(ts=0.5), N=20, |u|<=1, x0~U(-10,10)^2",
                "horizon": self.N, "nx": self.nx, "nu": self.nu, "mode": self.args.mode}

    def _condense(self, s):
        batched.condense(self.A_b, self.B_b, self.Q_t, self.R_t, self.Qf_t, self.N,
                         x0=self.X0_t[s], outputs=("H", "f"), out={"H": self.H, "f": self.f})

    def _solve(self, s, out):
        batched.solve_box(self.H, self.f, self.lb, self.ub, out=out)

    def _fused(self, s):
        batched.mpc_box(self.A_b, self.B_b, self.Q_t, self.R_t, self.Qf_t, self.N, self.X0_t[s],
                        self.lb, self.ub, out=(self.Z[s], self.ST[s]))

    def step(self, s):
        if self.args.mode == "fused":
            self._fused(s)
        else:
            self._condense(s)
            self._solve(s, (self.Z[s], self.ST[s]))

    def status(self):
        return self.ST

    def kernels(self, traffic):
        """Per-kernel device times and rooflines; returns (dominant, others)."""
        R = self.args.reps
        bsz, nx, nu, N, n = self.args.batch, self.nx, self.nu, self.N, self.n
        self._condense(0)
        t_c = time_kernel(lambda: self._condense(0), R, self.dev)
        t_s = time_kernel(lambda: self._solve(0, (self.Zs, self.STs)), R, self.dev)
        t_f = time_kernel(lambda: self._fused(0), R, self.dev)
        cb = condense_bytes_per_instance(nx, nu, N) * bsz
        sb = solve_bytes_per_instance(n) * bsz
        fl = condense_flops_per_instance(nx, nu, N) * bsz
        r_c = roof("condense_kernel<double,2>", "hbm", cb, t_c, HBM_PEAK_GBS, "GB/s",
                   traffic.get("condense"), {"bytes_per_launch": cb})
        r_s = roof("box_quad_kernel<double,5>", "hbm", sb, t_s, HBM_PEAK_GBS, "GB/s",
                   traffic.get("solve_box"), {"bytes_per_launch": sb})
        # fused kernel: SURVEY.md 8(d) per-instance figure (22.0 kflop condense,
        # config 2) against the fp64 vector peak; it moves only A, B, x0 in and
        # z out, and issues no MFMA: its roof is fp64 VALU issue
        r_f = roof("mpc_group_kernel<double,2,1,QSym<double,5>,16,2>", "valu-fp64", fl, t_f,
                   FP64_PEAK_TFS, "TFLOP/s",
                   traffic.get("mpc_box"), {"flops_per_launch": fl,
                                            "hbm_bytes_per_launch": (nx * nx + nx * nu + nx + n) * 8 * bsz + 4 * bsz})
        # split vs fused agreement on the same slot
        self._fused(0)
        self._condense(0)
        self._solve(0, (self.Zs, self.STs))
        torch.cuda.synchronize()
        extra = {"kernel_us": {"mpc_box": round(t_f * 1e3, 2), "condense": round(t_c * 1e3, 2),
                               "solve_box": round(t_s * 1e3, 2)},
                 "split_vs_fused_max_abs": float((self.Zs - self.Z[0]).abs().max())}
        if self.args.mode == "fused":
            return r_f, {"roofline_condense": r_c, "roofline_solve_box": r_s}, extra
        dom = r_s if t_s >= t_c else r_c
        return dom, {"roofline_condense": r_c, "roofline_solve_box": r_s}, extra

    def check(self):
        from oracle import cbaseline as cbl

        nchk = min(256, self.args.batch)
        zr, _ = cbl.mpc_box(self.A, self.B, self.Q, self.R, self.Qf, self.N, self.X0[0, :nchk],
                            -1.0, 1.0, nthreads=1)
        return float(np.abs(self.Z[0, :nchk].cpu().numpy() - zr).max())

    def cpu_baseline(self, seconds):
        from oracle import cbaseline as cbl

        bsz = self.args.batch
        cores = min(16, len(os.sched_getaffinity(0)))
        Xc = self.X0.reshape(-1, 2)
        done = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            cbl.mpc_box(self.A, np.broadcast_to(self.B, (bsz, 2, 1)), self.Q, self.R, self.Qf,
                        self.N, Xc[:bsz], -1.0, 1.0, nthreads=cores)
            done += bsz
        dt = time.perf_counter() - t0
        return {"value": round(done / dt, 1), "unit": "solves/s", "cores": cores, "kind": "port",
                "sample": f"{done} config-2 solves (per-instance condense + GI box QP, C/OpenMP "
                          f"oracle/c/mpcqp_oracle.c) in {dt:.1f} s on {cores} host threads"}


class Config2Loop:
    """Config 2's plant and MPC (FHC double integrator, N=20, |u|<=1, fp64) in
    a receding-horizon loop on the device: one bench step = one episode of
    --loop-steps closed-loop steps for the batch (mpcqp_condense once, then
    mpcqp_mpc_box_loop: every step warm-started from the shifted previous
    active set).  Unit: closed-loop MPC steps (instance x step) per second,
    the per-step counterpart of the config-2 solves/s."""

    dtype = torch.float64
    dname = "f64"
    default_batch = 4096
    default_slots = 4
    default_steps = (50, 5)
    default_loop_steps = 50

    def __init__(self, args, dev, rank):
        self.base = Config2(args, dev, rank)
        self.args, self.dev = args, dev
        self.T = args.loop_steps
        self.units_per_step = self.T
        b, c = self.base, self.base
        bsz, S, n = args.batch, args.slots, c.n
        t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64, device=dev)  # noqa: E731
        self.A_t, self.B_t = t(b.A), t(b.B)
        self.cd = {"H": torch.empty((bsz, n * (n + 1) // 2), dtype=torch.float64, device=dev),
                   "F": torch.empty((bsz, n, 2), dtype=torch.float64, device=dev)}
        self.outs = [{"xs": torch.empty((self.T + 1, bsz, 2), dtype=torch.float64, device=dev),
                      "us": torch.empty((self.T, bsz, 1), dtype=torch.float64, device=dev),
                      "status": torch.empty((self.T, bsz), dtype=torch.int32, device=dev)}
                     for _ in range(S)]
        self.ST = torch.empty((S, bsz), dtype=torch.int32, device=dev)

    def workload(self):
        return {"workload": f"cfg2-loop: config-2 plant and MPC (FHC.py double integrator, ts=0.5, "
                            f"N=20, |u|<=1, per-instance (A,B)) in a {self.T}-step receding-horizon "
                            f"loop on the device, x0~U(-10,10)^2; per episode: mpcqp_condense once + "
                            f"mpcqp_mpc_box_loop (warm-started active sets)",
                "horizon": self.base.N, "nx": 2, "nu": 1, "samples": self.T}

    def _episode(self, s):
        b = self.base
        batched.condense(b.A_b, b.B_b, b.Q_t, b.R_t, b.Qf_t, b.N, outputs=("H", "F"), out=self.cd)
        batched.mpc_box_loop(b.A_b, b.B_b, b.Q_t, b.R_t, b.Qf_t, b.N, b.X0_t[s], b.lb, b.ub, self.T,
                             condensed=self.cd, out=self.outs[s])

    def step(self, s):
        self._episode(s)
        # an episode is optimal when every one of its steps is
        st = self.outs[s]["status"]
        self.ST[s].copy_((st & 0xFF).amax(0))

    def status(self):
        return self.ST

    def kernels(self, traffic):
        R = self.args.reps
        b, bsz, n, T = self.base, self.args.batch, self.base.n, self.T
        t_e = time_kernel(lambda: self._episode(0), max(2, R // 10), self.dev)
        t_c = time_kernel(lambda: batched.condense(b.A_b, b.B_b, b.Q_t, b.R_t, b.Qf_t, b.N,
                                                   outputs=("H", "F"), out=self.cd), R, self.dev)
        t_l = t_e - t_c
        torch.cuda.synchronize()
        its = ((self.outs[0]["status"] >> 8) & 0xFFFF).double()
        # per step and instance: each sweep / active-set iteration one rank-1
        # update of the n x n matrix (2 n^2 flops) plus the mat-vec refresh
        flops = float(its.sum()) * 2 * n * n + T * bsz * (2 * n * n + 2 * n * 2)
        r = roof("box_loop_kernel<double,2,1,5>", "valu-fp64", flops, t_l, FP64_PEAK_TFS, "TFLOP/s",
                 traffic.get("box_loop"),
                 {"flops_per_launch": flops, "note": "T closed-loop steps in one launch; flops = "
                  "(sweeps + active-set iterations + 1 refresh) x 2n^2 per step and instance"})
        extra = {"kernel_us": {"episode": round(t_e * 1e3, 2), "condense_once": round(t_c * 1e3, 2),
                               "box_loop": round(t_l * 1e3, 2)},
                 "us_per_closed_loop_step": round(t_e * 1e3 / T, 3),
                 "loop_kernel_us_per_step": round(t_l * 1e3 / T, 3),
                 "sweeps_iters_first_step_mean": round(float(its[0].mean()), 2),
                 "sweeps_iters_later_steps_mean": round(float(its[1:].mean()), 2) if T > 1 else None}
        return r, {}, extra

    def check(self):
        """Max |x - x_ref| over the episode of 16 instances of slot 0 against
        the host loop: the C/OpenMP oracle's config-2 MPC step (per-instance
        condense + GI box QP) and x+ = A x + B u_0 on the host."""
        from oracle import cbaseline as cbl

        b = self.base
        nchk = min(16, self.args.batch)
        x = b.X0[0, :nchk].copy()
        xs = self.outs[0]["xs"][:, :nchk].cpu().numpy()
        err = 0.0
        for k in range(self.T):
            err = max(err, float(np.abs(xs[k] - x).max()))
            zr, _ = cbl.mpc_box(b.A, b.B, b.Q, b.R, b.Qf, b.N, x, -1.0, 1.0, nthreads=1)
            x = x @ b.A.T + zr[:, :1] @ b.B.T
        return err

    def cpu_baseline(self, seconds):
        r = self.base.cpu_baseline(seconds)
        r["unit"] = "closed-loop MPC steps/s"
        r["sample"] += " (one closed-loop step on the host = one such solve + x+ = Ax + Bu)"
        return r


def _stable_plant(rng, nx, nu, rho=0.98):
    U, _ = np.linalg.qr(rng.normal(size=(nx, nx)))
    sig = rng.uniform(0.5, rho, size=nx)
    A = (U * sig) @ U.T
    B = rng.normal(size=(nx, nu)) / np.sqrt(nx)
    return A, B


class Config3:
    """FE-linearised bicycle, N=30, state + input box, per-instance TV, fp32."""

    dtype = torch.float32
    dname = "f32"
    default_batch = 65536
    default_slots = 2

    def __init__(self, args, dev, rank):
        from model_predictive_control_amd.parameters import VehicleParameters

        self.args, self.dev = args, dev
        p = self.p = VehicleParameters()
        self.nx, self.nu, self.N, self.ts = 4, 2, args.horizon or 30, 0.08
        N, nx, nu = self.N, self.nx, self.nu
        n, m = N * nu, N * nx
        self.n, self.m = n, m
        bsz, S = args.batch, args.slots
        dt = self.dtype
        rng = np.random.default_rng(20261015 + 3 + 1000 * rank)
        X0 = np.stack([rng.uniform(-1, 1, (S, bsz)), rng.uniform(-.5, .5, (S, bsz)),
                       rng.uniform(-np.pi / 4, np.pi / 4, (S, bsz)), rng.uniform(-.3, .3, (S, bsz))], -1)
        self.X0 = X0
        Q = np.diag([1., 6., .2, .05])
        t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)  # noqa: E731
        self.Qn, self.QNn, self.Rn = Q, 100 * Q, np.diag([1., .01])
        self.Q_t, self.QN_t, self.R_t = t(Q), t(100 * Q), t(self.Rn)
        # per-slot linearisation about the zero-input rollout (RTI first
        # iterate), fp64 on device (mpcqp_bicycle_rti), stored in the bench dtype
        self.A, self.B, self.c, self.X0_t = [], [], [], []
        for s in range(S):
            x = torch.as_tensor(X0[s], dtype=torch.float64, device=dev)
            u = torch.zeros((bsz, N, nu), dtype=torch.float64, device=dev)
            Ak, Bk, ck = batched.bicycle_rti(x, u, p, self.ts)
            self.A.append(Ak.to(dt).contiguous())
            self.B.append(Bk.to(dt).contiguous())
            self.c.append(ck.to(dt).contiguous())
            self.X0_t.append(t(X0[s]))
        xmin = np.array([p.min_pos_x, p.min_pos_y, p.min_heading, p.min_vel])
        xmax = np.array([p.max_pos_x, p.max_pos_y, p.max_heading, p.max_vel])
        self.xmin_t, self.xmax_t = t(np.tile(xmin, N)), t(np.tile(xmax, N))
        self.xmin, self.xmax = xmin, xmax
        self.lbz = t(np.tile([p.min_drive, -p.max_steer], N))
        self.ubz = t(np.tile([p.max_drive, p.max_steer], N))
        self.Z = torch.empty((S, bsz, n), dtype=dt, device=dev)
        self.Y = torch.empty((bsz, m), dtype=dt, device=dev)
        self.ST = torch.empty((S, bsz), dtype=torch.int32, device=dev)
        self.ws = torch.empty((batched.mpc_qp_workspace_bytes(dt, bsz, nx, self.nu, N),),
                              dtype=torch.uint8, device=dev)

    def workload(self):
        return {"workload": "cfg3: FE-linearised bicycle (parameters.py), ts=0.08, N=30, "
                            "Q=diag(1,6,.2,.05), QN=100Q, R=diag(1,.01), state box x_1..x_N + "
                            "input box, per-instance per-stage (A_k,B_k,c_k) about the zero-input "
                            "rollout; one mpcqp_mpc_qp call: condense(TV) + rows + sweep + pf "
                            "(refined against the dynamics in fp64)",
                "horizon": self.N, "nx": self.nx, "nu": self.nu, "rows": self.m}

    def step(self, s):
        batched.mpc_qp(self.A[s], self.B[s], self.Q_t, self.R_t, self.QN_t, self.N, self.X0_t[s],
                       xlo=self.xmin_t, xhi=self.xmax_t, lb=self.lbz, ub=self.ubz, c=self.c[s],
                       tv=True, out=(self.Z[s], self.Y, self.ST[s]), ws=self.ws)

    def status(self):
        return self.ST

    def kernels(self, traffic):
        """Per-kernel rooflines of the z-space path, every stage timed by the
        library's HIP events on the call's stream (mpc_qp_stage_ms)."""
        R = self.args.reps
        bsz, nx, nu, N, n, m = self.args.batch, self.nx, self.nu, self.N, self.n, self.m
        t_s = time_kernel(lambda: self.step(0), R, self.dev)
        st = mpc_qp_stage_ms(lambda: self.step(0), R)
        t_c, t_w, t_z = st["condense"], st["sweep"], st["solve"]
        # achieved: SURVEY 8(d)'s bytes (H upper, F, Gamma's lower block
        # triangle, Phi; A_k, B_k, x0 in).  The kernel itself reads c_k too and
        # writes packed H, f and the packed Gamma (the row normals; no F, Phi)
        cb = condense_bytes_survey(nx, nu, N, 4, True) * bsz
        cm = condense_bytes_per_instance(nx, nu, N, 4, tv=True, gam=True, drift=True) * bsz
        wf = sweep_flops_per_instance(n, 0) * bsz
        # the z-space kernel reads H^-1 (n x n), s0, f, Gamma packed (its
        # lower block triangle, nx nu N(N+1)/2: the row normals), the dynamics
        # (A_k, B_k, c_k, x0) of the refinement, the shared bounds once;
        # writes z, y, status
        gp = nx * nu * N * (N + 1) // 2
        zb = (n * n + 2 * n + gp + N * (nx * nx + nx * nu + nx) + nx + n + m + 1) * 4 * bsz
        r_c = roof("condense_stream_kernel<float,4,2>", "hbm", cb, t_c, HBM_PEAK_GBS, "GB/s",
                   traffic.get("condense"), {"bytes_per_launch": cb, "bytes_moved_per_launch": cm,
                                             "bytes": "SURVEY 8(d)"})
        r_w = roof("sweep_mfma_kernel<4> (H^-1)", "mfma", wf, t_w, FP32_PEAK_TFS, "TFLOP/s",
                   traffic.get("sweep"), {"flops_per_launch": wf})
        r_z = roof("qp_zf_kernel<4> (DYN refinement)", "hbm", zb, t_z, HBM_PEAK_GBS, "GB/s",
                   traffic.get("solve_zf"), {"bytes_per_launch": zb})
        extra = {"kernel_us": {k: round(v * 1e3, 2) for k, v in st.items()},
                 "mpc_qp_us": round(t_s * 1e3, 2)}
        rs = sorted([(t_c, r_c), (t_w, r_w), (t_z, r_z)], key=lambda x: -x[0])
        return rs[0][1], {"roofline_other": [r for _, r in rs[1:]]}, extra

    def check(self):
        """fp64 oracle (explicit condensing + Goldfarb-Idnani) on a few
        instances of slot 0, from the same fp32-valued (A_k, B_k, c_k, x0,
        weights, bounds) the device saw."""
        from oracle import parallel

        N = self.N
        r = lambda t: t.double().cpu().numpy()  # noqa: E731
        errs = []
        A, B, c, X0 = r(self.A[0]), r(self.B[0]), r(self.c[0]), r(self.X0_t[0])
        Q, QN, Rm = r(self.Q_t), r(self.QN_t), r(self.R_t)
        xlo, xhi, lb, ub = r(self.xmin_t), r(self.xmax_t), r(self.lbz), r(self.ubz)
        Z = self.Z[0].double().cpu().numpy()
        code = batched.status_code(self.ST[0]).cpu().numpy()
        nchk = min(self.args.check, self.args.batch)
        sols = parallel.solve_map(parallel.cfg3_solve, lambda lo, hi: (
            A[lo:hi], B[lo:hi], c[lo:hi], X0[lo:hi], Q, Rm, QN, N, xlo, xhi, lb, ub), nchk)
        for i, zr in enumerate(sols):
            if zr is None:
                assert code[i] == 3
                continue
            errs.append(np.abs(Z[i] - zr).max())
        return float(max(errs)) if errs else None

    def cpu_baseline(self, seconds):
        from oracle import parallel

        N = self.N
        A, B, c = self.A[0].double().cpu().numpy(), self.B[0].double().cpu().numpy(), \
            self.c[0].double().cpu().numpy()
        lb = np.tile([self.p.min_drive, -self.p.max_steer], N)
        ub = np.tile([self.p.max_drive, self.p.max_steer], N)
        cores = parallel.host_cores()
        total = min(self.args.batch, 2000 * cores)
        r = parallel.rate(parallel.cfg3_chunk, lambda lo, hi, dl: (
            A[lo:hi], B[lo:hi], c[lo:hi], self.X0[0, lo:hi], self.Qn, self.Rn, self.QNn, N,
            self.xmin, self.xmax, lb, ub, dl), total, seconds, cores)
        return {"value": round(r["value"], 2), "unit": "solves/s", "cores": r["cores"],
                "kind": "port",
                "sample": f"{r['done']} config-3 instances: NumPy explicit condensing "
                          f"(oracle/condense.py) + Goldfarb-Idnani (oracle/qp.py), per-x0 solves "
                          f"over {r['cores']} spawned processes (oracle/parallel.py) in "
                          f"{r['seconds']:.1f} s"}


class Config4:
    """Random stable LTI nx=12, nu=4, N=50, 40 polytope rows; shared condense; fp64."""

    dtype = torch.float64
    dname = "f64"
    default_batch = 131072
    default_slots = 2

    def __init__(self, args, dev, rank):
        self.args, self.dev = args, dev
        self.nx, self.nu, self.N, self.m = 12, 4, args.horizon or 50, 40
        nx, nu, N, m = self.nx, self.nu, self.N, self.m
        n = self.n = N * nu
        bsz, S = args.batch, args.slots
        dt = self.dtype
        rng = np.random.default_rng(20261015 + 4)          # plant shared by all ranks
        A, B = _stable_plant(rng, nx, nu)
        self.A, self.B = A, B
        self.Qn, self.Rn = np.eye(nx), 0.1 * np.eye(nu)
        self.G = rng.normal(size=(m, n))
        self.h = rng.uniform(0.5, 1.5, size=m)
        t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)  # noqa: E731
        d = batched.condense(t(A), t(B), t(self.Qn), t(self.Rn), t(self.Qn), N, outputs=("H", "F"))
        self.Hs, self.F = d["H"][0].contiguous(), d["F"][0].contiguous()
        self.G_t, self.h_t = t(self.G), t(self.h)
        # shared factors once (the plant and the polytope do not change)
        self.qp = batched.PolyQP(self.Hs, self.G_t, self.F)
        xr = np.random.default_rng(20261015 + 4 + 1000 * (rank + 1))
        self.X0 = xr.normal(size=(S, bsz, nx)) * 3.0
        self.X0_t = t(self.X0)
        self.Z = torch.empty((S, bsz, n), dtype=dt, device=dev)
        self.Y = torch.empty((bsz, m), dtype=dt, device=dev)
        self.ST = torch.empty((S, bsz), dtype=torch.int32, device=dev)

    def workload(self):
        return {"workload": "cfg4: random stable LTI nx=12 nu=4 (rho<=0.98), Q=I, R=0.1I, N=50, "
                            "40 random polytope rows G z <= h (h>0), shared condense + shared "
                            "factors (poly_setup, once); per step poly_solve(x0)",
                "horizon": self.N, "nx": self.nx, "nu": self.nu, "rows": self.m}

    def _solve(self, s):
        self.qp.solve(self.X0_t[s], hu=self.h_t, out=(self.Z[s], self.Y, self.ST[s]))

    def step(self, s):
        self._solve(s)

    def status(self):
        return self.ST

    def kernels(self, traffic):
        R = self.args.reps
        bsz, n, m, nx = self.args.batch, self.n, self.m, self.nx
        t_s = time_kernel(lambda: self._solve(0), R, self.dev)
        sb = (nx + n + m) * 8 * bsz + 4 * bsz      # x0 in; z, y, status out
        # SURVEY.md 8(d), config 4 per instance: f = F x0 4.8 kflop, h(x0) ~1
        # kflop, the dual active set on the shared 40 x 40 M and the primal
        # recovery ~21 kflop.  96 B in / 1.6 KB out per instance is far below
        # the HBM roof: the kernel is fp64 VALU issue/latency bound
        fl = 26_800 * bsz
        r_s = roof("dual_range_kernel<double,5> (fused s0 / z epilogue)", "valu-fp64", fl, t_s,
                   FP64_PEAK_TFS, "TFLOP/s", traffic.get("poly_solve"),
                   {"flops_per_launch": fl, "hbm_bytes_per_launch": sb})
        extra = {"kernel_us": {"poly_solve": round(t_s * 1e3, 2)}}
        return r_s, {}, extra

    def check(self):
        from oracle import condense as oc
        from oracle import parallel

        d = oc.condense(self.A, self.B, self.Qn, self.Rn, self.Qn, self.N)
        Z = self.Z[0].cpu().numpy()
        nchk = min(self.args.check, self.args.batch)
        sols = parallel.solve_map(parallel.cfg4_solve, lambda lo, hi: (
            d["H"], d["F"], self.G, self.h, self.X0[0, lo:hi]), nchk)
        return float(max(np.abs(Z[i] - zr).max() for i, zr in enumerate(sols))) if sols else None

    def cpu_baseline(self, seconds):
        from oracle import condense as oc
        from oracle import parallel

        d = oc.condense(self.A, self.B, self.Qn, self.Rn, self.Qn, self.N)
        cores = parallel.host_cores()
        total = min(self.args.batch, 4000 * cores)
        r = parallel.rate(parallel.cfg4_chunk, lambda lo, hi, dl: (
            d["H"], d["F"], self.G, self.h, self.X0[0, lo:hi], dl), total, seconds, cores)
        return {"value": round(r["value"], 2), "unit": "solves/s", "cores": r["cores"],
                "kind": "port",
                "sample": f"{r['done']} config-4 instances: NumPy Goldfarb-Idnani (oracle/qp.py) "
                          f"on the shared condensed QP, per-x0 solves over {r['cores']} spawned "
                          f"processes in {r['seconds']:.1f} s"}


class Config5:
    """Config-4 plant perturbed per instance/stage, N=40, input box, fp32."""

    dtype = torch.float32
    dname = "f32"
    default_batch = 32768
    default_slots = 2

    def __init__(self, args, dev, rank):
        self.args, self.dev = args, dev
        self.nx, self.nu, self.N = 12, 4, args.horizon or 40
        nx, nu, N = self.nx, self.nu, self.N
        n = self.n = N * nu
        bsz, S = args.batch, args.slots
        dt = self.dtype
        rng = np.random.default_rng(20261015 + 4)
        A, B = _stable_plant(rng, nx, nu)
        self.Qn, self.Rn = np.eye(nx), 0.1 * np.eye(nu)
        t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)  # noqa: E731
        g = torch.Generator(device=dev)
        g.manual_seed(20261015 + 5 + 1000 * rank)
        eps = 0.01
        self.A, self.B, self.X0_t = [], [], []
        for s in range(S):
            self.A.append((t(A) + eps * torch.randn((bsz, N, nx, nx), generator=g, device=dev,
                                                    dtype=dt)).contiguous())
            self.B.append((t(B) + eps * torch.randn((bsz, N, nx, nu), generator=g, device=dev,
                                                    dtype=dt)).contiguous())
            self.X0_t.append((3.0 * torch.randn((bsz, nx), generator=g, device=dev, dtype=dt)).contiguous())
        self.Q_t, self.R_t = t(self.Qn), t(self.Rn)
        self.lb, self.ub = -0.5, 0.5
        self.Z = torch.empty((S, bsz, n), dtype=dt, device=dev)
        self.ST = torch.empty((S, bsz), dtype=torch.int32, device=dev)
        self.lb_t = torch.full((n,), self.lb, dtype=dt, device=dev)
        self.ub_t = torch.full((n,), self.ub, dtype=dt, device=dev)
        self.ws = torch.empty((batched.mpc_qp_workspace_bytes(dt, bsz, nx, nu, N, False),),
                              dtype=torch.uint8, device=dev)

    def workload(self):
        return {"workload": "cfg5: config-4 plant (nx=12, nu=4) with per-instance per-stage "
                            "perturbation A_k=A+0.01*D_k, B_k=B+0.01*E_k, N=40, |u|<=0.5, "
                            "re-condensed every step; one mpcqp_mpc_qp call: condense(TV, MFMA) + "
                            "sweep (n=160) + pf (refined against the dynamics in fp64)",
                "horizon": self.N, "nx": self.nx, "nu": self.nu}

    def step(self, s):
        batched.mpc_qp(self.A[s], self.B[s], self.Q_t, self.R_t, self.Q_t, self.N, self.X0_t[s],
                       lb=self.lb_t, ub=self.ub_t, tv=True, out=(self.Z[s], None, self.ST[s]),
                       ws=self.ws)

    def status(self):
        return self.ST

    def kernels(self, traffic):
        R = self.args.reps
        bsz, nx, nu, N, n = self.args.batch, self.nx, self.nu, self.N, self.n
        t_s = time_kernel(lambda: self.step(0), R, self.dev)
        st = mpc_qp_stage_ms(lambda: self.step(0), R)
        t_c, t_w, t_p = st["condense"], st["sweep"], st["solve"]
        # achieved: SURVEY 8(d)'s bytes (A_k, B_k, x0 in; H upper + F out);
        # the kernel writes f instead of F.  (8(d)'s flop formula counts the
        # explicit Gam'QGam product, which the recursion never forms: it is
        # not a rate of this kernel and is not reported as one)
        cb = condense_bytes_survey(nx, nu, N, 4, False) * bsz
        cm = condense_bytes_per_instance(nx, nu, N, 4, tv=True) * bsz
        r_c = roof("condense_mfma_fh_kernel<10> (fused-H)", "hbm", cb, t_c, HBM_PEAK_GBS, "GB/s",
                   traffic.get("condense"), {"bytes_per_launch": cb, "bytes_moved_per_launch": cm,
                                             "bytes": "SURVEY 8(d)"})
        wf = sweep_flops_per_instance(n) * bsz
        r_w = roof("sweep_mfma_kernel<10>", "mfma", wf, t_w, FP32_PEAK_TFS, "TFLOP/s",
                   traffic.get("sweep"), {"flops_per_launch": wf})
        # pf reads M0, s0 and the dynamics (A_k, B_k, x0) for the refinement
        pb = (n * n + n + N * (nx * nx + nx * nu) + nx + n) * 4 * bsz
        r_p = roof("qp_pf_kernel<3,12> (DYN refinement)", "hbm", pb, t_p, HBM_PEAK_GBS, "GB/s",
                   traffic.get("solve_pf"), {"bytes_per_launch": pb})
        extra = {"kernel_us": {k: round(v * 1e3, 2) for k, v in st.items()},
                 "mpc_qp_us": round(t_s * 1e3, 2)}
        rs = sorted([(t_c, r_c), (t_w, r_w), (t_p, r_p)], key=lambda x: -x[0])
        return rs[0][1], {"roofline_other": [r for _, r in rs[1:]]}, extra

    def check(self):
        from oracle import parallel

        N = self.N
        A, B = self.A[0].double().cpu().numpy(), self.B[0].double().cpu().numpy()
        X0 = self.X0_t[0].double().cpu().numpy()
        Q, Rm = self.Q_t.double().cpu().numpy(), self.R_t.double().cpu().numpy()
        Z = self.Z[0].double().cpu().numpy()
        nchk = min(self.args.check, self.args.batch)
        sols = parallel.solve_map(parallel.cfg5_solve, lambda lo, hi: (
            A[lo:hi], B[lo:hi], X0[lo:hi], Q, Rm, N, self.lb, self.ub), nchk)
        return float(max(np.abs(Z[i] - zr).max() for i, zr in enumerate(sols))) if sols else None

    def cpu_baseline(self, seconds):
        from oracle import parallel

        N = self.N
        cores = parallel.host_cores()
        total = min(self.args.batch, 500 * cores)
        A = self.A[0][:total].double().cpu().numpy()
        B = self.B[0][:total].double().cpu().numpy()
        X0 = self.X0_t[0][:total].double().cpu().numpy()
        r = parallel.rate(parallel.cfg5_chunk, lambda lo, hi, dl: (
            A[lo:hi], B[lo:hi], X0[lo:hi], self.Qn, self.Rn, N, self.lb, self.ub, dl),
            total, seconds, cores)
        return {"value": round(r["value"], 2), "unit": "solves/s", "cores": r["cores"],
                "kind": "port",
                "sample": f"{r['done']} config-5 instances: NumPy explicit condensing + primal "
                          f"active set (oracle/), per-x0 solves over {r['cores']} spawned "
                          f"processes in {r['seconds']:.1f} s"}


class ConfigNLP:
    """Converged NLP solves of the session-4 MPC step (the controller of
    main.py:241-251: N=30, ts=0.08, weights main.py:72-74, input + state box;
    collision rows out of scope): MPCController's SQP (mpc.SqpSolver), a
    fixed budget of --sqp-iters iterations per solve from a cold start
    (U = 0), over a batch of x0.  One step = one batch of NLP solves."""

    dtype = torch.float64
    dname = "f64"
    default_batch = 4096
    default_slots = 2
    default_sqp_iters = 150  # a cap per instance: each stops at its own convergence
    default_steps = (5, 1)  # (steps, warmup) when not given: one step is ~30 SQP iterations

    def __init__(self, args, dev, rank):
        from model_predictive_control_amd.mpc import MPCController, SqpSolver
        from model_predictive_control_amd.parameters import VehicleParameters

        self.args, self.dev = args, dev
        self.N, self.ts = args.horizon or 30, 0.08
        self.iters = args.sqp_iters
        bsz, S = args.batch, args.slots
        self.ctl = MPCController(self.N, self.ts, VehicleParameters(), tol=1e-9,
                                 fused=not args.sqp_iterate)
        self.sqp = SqpSolver(self.ctl, bsz)
        rng = np.random.default_rng(20261015 + 6 + 1000 * rank)
        self.X0 = np.stack([rng.uniform(-.8, .8, (S, bsz)), rng.uniform(-.4, .4, (S, bsz)),
                            rng.uniform(-.5, .5, (S, bsz)), rng.uniform(-.2, .2, (S, bsz))], -1)
        self.X0_t = torch.as_tensor(self.X0, dtype=torch.float64, device=dev)
        self.Z = torch.empty((S, bsz, 2 * self.N), dtype=torch.float64, device=dev)
        self.ST = torch.empty((S, bsz), dtype=torch.int32, device=dev)
        self.KKT = torch.empty((S, bsz), dtype=torch.float64, device=dev)

    def workload(self):
        return {"workload": f"nlp: converged MPCController.solve (main.py controller, N={self.N}, "
                            f"ts=0.08, input + state box) by SQP on device, at most {self.iters} "
                            f"iterations per solve from U=0 (Gauss-Newton, then the exact "
                            f"Hessian, projected per stage after a non-convex QP), x0 ~ U(+-.8, +-.4, +-.5, +-.2); "
                            f"value counts only solves that reached KKT <= 1e-9",
                "horizon": self.N, "nx": 4, "nu": 2, "sqp_iters": self.iters}

    def step(self, s):
        sqp = self.sqp
        sqp.reset()
        if self.ctl.fused:  # one launch: every instance iterates to its own convergence
            sqp.solve(self.X0_t[s], self.iters)
        else:
            for _ in range(self.iters):
                sqp.iterate(self.X0_t[s])
        self.Z[s].copy_(sqp.U.view(self.args.batch, -1))
        self.ST[s].copy_(sqp.status())
        self.KKT[s].copy_(sqp.kkt)

    def status(self):
        return self.ST

    def counted_units(self, steps):
        """NLP solves that reached the KKT tolerance (status OPTIMAL) in the
        timed steps; an instance at MAXITER is not a solve."""
        ok = (batched.status_code(self.ST) == 0).sum(1).cpu().numpy()
        S = self.args.slots
        return int(sum(ok[k % S] for k in range(steps)))

    def kernels(self, traffic):
        """The one-launch solve (sqp_solve_kernel, mpcqp_bicycle_sqp_solve)
        timed on its stream by HIP events over R launches of slot 0, and the
        kernel's own per-instance clocks (s_memrealtime: solve time, time in
        the QPs, interior-point iterations, SQP iterations, warm-polished QPs)
        for the roofline's flop count and the latency profile.  With
        --sqp-iterate: one iteration's four launches timed separately."""
        from model_predictive_control_amd.mpc import SqpSolver

        R = self.args.reps
        sqp, ctl, N, bsz = self.sqp, self.ctl, self.N, self.args.batch
        x0 = self.X0_t[0]
        kkt_final, done_final = float(self.KKT[0].max()), self.ST[0].clone()
        extra = {"kkt_max": kkt_final,
                 "converged_frac": float((batched.status_code(done_final) == 0).double().mean())}
        if not ctl.fused:
            return self._kernels_iterate(traffic, extra)
        t_s = time_kernel(lambda: self.step(0), max(2, R // 4), self.dev)
        st = sqp.ws.view(torch.float64)[bsz * N * 90 + bsz * 4:][:4 * bsz].view(torch.int64) \
            .view(bsz, 4).cpu().numpy().astype(np.float64)
        tot, tqp, ipm = st[:, 0] * 0.01, st[:, 1] * 0.01, st[:, 2]  # us (100 MHz ticks)
        its = (st[:, 3].astype(np.int64) & 0xFFFFFFFF).astype(np.float64)
        hits = (st[:, 3].astype(np.int64) >> 32).astype(np.float64)
        # algorithmic fp64 flops of one interior-point iteration per stage
        # (nx = 4, nu = 2): Riccati factorisation ~270 FMA, residuals and
        # gradients ~90, predictor / corrector sweeps ~180 -> ~540 FMA
        flops = 2 * 540 * N * float(ipm.sum())
        pct = lambda v: [round(float(np.percentile(v, q)), 1) for q in (50, 90, 99, 100)]  # noqa: E731
        r_i = roof("sqp_solve_kernel (whole SQP per instance)", "valu-fp64", flops, t_s,
                   FP64_PEAK_TFS, "TFLOP/s", traffic.get("sqp_solve"),
                   {"flops_per_launch": flops, "avg_launch_us": round(t_s * 1e3, 2),
                    "note": "one single-wave workgroup per instance runs its SQP to convergence "
                            "(QP: interior point on the whole wave, per-stage work on 16 quads and the Riccati chains on one, horizon in LDS; linearisation, "
                            "Hessian and line search one lane per stage); flops = 1080 per stage "
                            "per interior-point iteration summed over the instances' own counts "
                            "(warm polishes, Hessians and line searches not counted): latency-bound"})
        extra.update({
            "kernel_us": {"sqp_solve": round(t_s * 1e3, 2)},
            "instance_us_p50_p90_p99_max": pct(tot),
            "qp_time_share": round(float(tqp.sum() / tot.sum()), 3),
            "ipm_iters_per_sqp_iter": round(float(ipm.sum() / max(1.0, its.sum())), 2),
            "warm_polished_qp_frac": round(float(hits.sum() / max(1.0, its.sum())), 3),
            "sqp_iters_mean": round(float(its.mean()), 2), "sqp_iters_max": int(its.max()),
            "sum_instance_ms": round(float(tot.sum()) / 1e3, 1)})
        return r_i, {}, extra

    def _kernels_iterate(self, traffic, extra):
        """One SQP iteration's launches timed separately, on the state of slot
        0 after 3 iterations from U = 0 (every instance still iterating): the
        interior point as SqpSolver runs it (STRICT, QP_MAX_ITER), no skip."""
        from model_predictive_control_amd.mpc import SqpSolver

        R = self.args.reps
        sqp, ctl, N, bsz = self.sqp, self.ctl, self.N, self.args.batch
        x0 = self.X0_t[0]
        sqp.reset()
        for _ in range(3):
            sqp.iterate(x0)
        A, B, c, Xr = batched.bicycle_rti(x0, sqp.U, ctl.params, ctl.ts, states=True)
        t_r = time_kernel(lambda: batched.bicycle_rti(x0, sqp.U, ctl.params, ctl.ts, states=True), R,
                          self.dev)
        cw = dict(Q=ctl.Q, R=ctl.R) if ctl.hessian == "exact" else {}
        t_h = time_kernel(lambda: batched.bicycle_hessian(Xr, sqp.U, sqp.pi, ctl.params, ctl.ts,
                                                          flags=sqp.flags, mu=sqp.mu, fix=sqp.fix,
                                                          **cw), R,
                          self.dev)
        H2, q2 = batched.bicycle_hessian(Xr, sqp.U, sqp.pi, ctl.params, ctl.ts, flags=sqp.flags,
                                         mu=sqp.mu, fix=sqp.fix, **cw)
        box = ctl._box()
        qp = {}

        def ipm():  # the outputs allocated once, then written in place
            qp.update(batched.mpc_ipm(A, B, ctl.Q, ctl.R, ctl.QN, N, x0, lb=ctl.lbz, ub=ctl.ubz,
                                      c=c, tv=True, H2=H2, q2=q2, strict=SqpSolver.STRICT,
                                      max_iter=SqpSolver.QP_MAX_ITER, out=qp or None, **box))
        t_i = time_kernel(ipm, R, self.dev)
        torch.cuda.synchronize()
        its = ((qp["status"] >> 8) & 0xFFFF).double()
        flops = 2 * 540 * N * float(its.sum())
        r_i = roof("ipm_quad_kernel<double,1>", "valu-fp64", flops, t_i,
                   FP64_PEAK_TFS, "TFLOP/s", traffic.get("ipm"),
                   {"flops_per_launch": flops, "ipm_iters_mean": round(float(its.mean()), 2),
                    "ipm_iters_max": int(its.max()),
                    "note": "four lanes per instance, serial over the stages, the horizon in "
                            "LDS (four per CU, one single-wave workgroup each): latency/LDS-"
                            "bound; flops = 1080 per stage per IPM iteration "
                            "summed over the instances' own iteration counts, polish not counted"})
        extra["kernel_us"] = {"bicycle_rti": round(t_r * 1e3, 2),
                              "bicycle_hessian": round(t_h * 1e3, 2),
                              "mpc_ipm": round(t_i * 1e3, 2)}
        return r_i, {}, extra

    def check(self):
        """max |u - u*| against the NLP oracle (oracle/nlp.py: SQP + Newton
        polish, KKT-certified) on a few instances of slot 0."""
        from oracle import nlp

        g = self.ctl
        xlo, lbu = g.lb_states, g.lb_inputs
        ocp = nlp.OCP(self.N, self.ts, g.Q.cpu().numpy(), g.QN.cpu().numpy(), g.R.cpu().numpy(),
                      xlo, -xlo, lbu, -lbu)
        Z = self.Z[0].cpu().numpy()
        errs = []
        for i in range(min(self.args.check, 4, self.args.batch)):
            U, _, k = ocp.solve(self.X0[0, i])
            if k < 1e-10:
                errs.append(np.abs(Z[i] - U).max())
        return float(max(errs)) if errs else None

    def cpu_baseline(self, seconds):
        from oracle import parallel

        g = self.ctl
        cores = parallel.host_cores()
        total = min(self.args.batch, 64 * cores)
        Q, QN, R = (v.cpu().numpy() for v in (g.Q, g.QN, g.R))
        r = parallel.rate(parallel.nlp_chunk, lambda lo, hi, dl: (
            self.N, self.ts, Q, QN, R, g.lb_states, g.lb_inputs, self.X0[0, lo:hi], dl),
            total, seconds, cores)
        return {"value": round(r["value"], 3), "unit": "solves/s", "cores": r["cores"],
                "kind": "port",
                "sample": f"{r['done']} NLP solves (oracle/nlp.py: Gauss-Newton SQP on the "
                          f"NumPy condensing + Goldfarb-Idnani QP, Newton polish to KKT 1e-9), "
                          f"per-x0 over {r['cores']} spawned processes in {r['seconds']:.1f} s"}


class ConfigLoop:
    """The receding-horizon loop on device (closed_loop.ClosedLoop): the
    main.py controller (converged SQP, --sqp-iters iterations per sample,
    warm-started) on a forward-Euler bicycle plant for --loop-steps samples
    (main.py:270-271 runs 100), batch of x0.  One bench step = one closed-loop
    episode of the batch; value = closed-loop MPC steps (instance x sample)
    per second."""

    dtype = torch.float64
    dname = "f64"
    default_batch = 1024
    default_slots = 2
    default_sqp_iters = 100  # per sample (a cap: each instance stops at its own convergence)
    default_steps = (3, 1)  # one step is a whole episode

    def __init__(self, args, dev, rank):
        from model_predictive_control_amd.closed_loop import ClosedLoop
        from model_predictive_control_amd.mpc import MPCController
        from model_predictive_control_amd.parameters import VehicleParameters

        self.args, self.dev = args, dev
        self.N, self.T = args.horizon or 30, args.loop_steps
        self.units_per_step = self.T
        bsz, S = args.batch, args.slots
        self.ctl = MPCController(self.N, 0.08, VehicleParameters(), tol=1e-9,
                                 fused=not args.sqp_iterate)
        # the cold first sample gets the nlp line's cap (a cap: each instance stops at its own
        # convergence)
        self.loop = ClosedLoop(self.ctl, plant="fe", iters_per_step=args.sqp_iters, graph=False,
                               iters_first=max(args.sqp_iters, ConfigNLP.default_sqp_iters))
        rng = np.random.default_rng(20261015 + 7 + 1000 * rank)
        self.X0 = np.stack([rng.uniform(-.8, .8, (S, bsz)), rng.uniform(-.4, .4, (S, bsz)),
                            rng.uniform(-.5, .5, (S, bsz)), rng.uniform(-.2, .2, (S, bsz))], -1)
        self.X0_t = torch.as_tensor(self.X0, dtype=torch.float64, device=dev)
        self.bufs = [self.loop._alloc(bsz, self.T) for _ in range(S)]
        self.ST = torch.empty((S, bsz), dtype=torch.int32, device=dev)

    def workload(self):
        return {"workload": f"loop: on-device receding-horizon loop, main.py controller (N={self.N}, "
                            f"ts=0.08, input + state box, SQP warm-started from the shifted "
                            f"solution, at most {self.args.sqp_iters} iterations per sample, "
                            f"{self.loop.iters_first} for the cold first one) on a "
                            f"forward-Euler plant, {self.T} samples per episode; value counts "
                            f"only the samples whose controller call converged (KKT <= 1e-9)",
                "horizon": self.N, "nx": 4, "nu": 2, "samples": self.T,
                "sqp_iters_per_sample": self.args.sqp_iters,
                "sqp_iters_first_sample": self.loop.iters_first}

    def step(self, s):
        b = self.bufs[s]
        b["xs"][0].copy_(self.X0_t[s])
        self.loop._episode(b, self.T)
        self.ST[s].copy_(b["success"].all(0).logical_not().to(torch.int32))

    def status(self):
        return self.ST

    def optimal_frac(self):
        """Fraction of the controller calls (instance x sample, all slots)
        that converged."""
        return float(sum(float(b["success"].double().mean()) for b in self.bufs) / len(self.bufs))

    def counted_units(self, steps):
        """Closed-loop samples whose controller call converged, over the
        timed episodes."""
        S = self.args.slots
        ok = [int(self.bufs[s]["success"].sum()) for s in range(S)]
        return int(sum(ok[k % S] for k in range(steps)))

    def kernels(self, traffic):
        """Per-kernel time of one warm-started sample (the second of slot 0's
        episode, replayed from a snapshot of the state before it) on HIP
        events: the controller's SQP (sqp_solve_kernel; with --sqp-iterate the
        four launches per iteration), the plant and the shift; the roofline
        of the SQP kernel from its own interior-point iteration counts."""
        b = self.bufs[0]
        extra = {"success_frac_per_sample": float(b["success"].double().mean()),
                 "episodes_all_converged_frac": float(b["success"].all(0).double().mean()),
                 "iters_per_sample_mean": float(b["iters"].double().mean()),
                 "iters_per_sample_max": int(b["iters"].max())}
        if self.T < 2:
            return None, {}, extra
        R, N, bsz, loop = self.args.reps, self.N, self.args.batch, self.loop
        b["xs"][0].copy_(self.X0_t[0])
        loop._reset(b)
        loop._step(b, 0)
        sqp = b["sqp"]
        keys = ("U", "y", "pi", "X", "rho", "kkt", "mu", "flags", "fix")
        snap = {k: getattr(sqp, k).clone() for k in keys}
        xs1 = b["xs"][1].clone()

        def restore():
            for k in keys:
                getattr(sqp, k).copy_(snap[k])
            b["xs"][1].copy_(xs1)

        def sample_mpc():
            restore()
            loop._mpc(b, 1)

        def plant_shift():
            restore()
            loop._step_tail(b, 1)

        t_m = time_kernel(sample_mpc, R, self.dev)
        t_r = time_kernel(restore, R, self.dev)
        t_p = time_kernel(plant_shift, R, self.dev) - t_r
        extra["kernel_us"] = {"sample_mpc_solve": round((t_m - t_r) * 1e3, 2),
                              "sample_plant_and_shift": round(t_p * 1e3, 2),
                              "state_restore (timing harness)": round(t_r * 1e3, 2)}
        if not (self.ctl.fused and N <= 64):
            return None, {}, extra
        # the bench step itself: one launch of the whole episode (sqp_loop_kernel)
        t_e = time_kernel(lambda: self.step(0), max(2, R // 4), self.dev)
        st = sqp.ws.view(torch.float64)[bsz * N * 90 + bsz * 4:][:4 * bsz].view(torch.int64) \
            .view(bsz, 4).cpu().numpy().astype(np.float64)
        tot, tqp, ipm = st[:, 0] * 0.01, st[:, 1] * 0.01, st[:, 2]
        its = (st[:, 3].astype(np.int64) & 0xFFFFFFFF).astype(np.float64)
        flops = 2 * 540 * N * float(ipm.sum())
        r = roof("sqp_loop_kernel (whole episode per instance)", "valu-fp64", flops, t_e,
                 FP64_PEAK_TFS, "TFLOP/s", traffic.get("sqp_loop"),
                 {"flops_per_launch": flops, "avg_launch_us": round(t_e * 1e3, 2),
                  "note": "one single-wave workgroup per instance runs its whole episode (per "
                          "sample: SQP to convergence, plant, shift); flops = 1080 per stage per "
                          "interior-point iteration summed over the instances: latency-bound"})
        extra["kernel_us"]["episode"] = round(t_e * 1e3, 2)
        extra.update({"episode_instance_us_p50_p99_max": [round(float(np.percentile(tot, q)), 1)
                                                          for q in (50, 99, 100)],
                      "qp_time_share": round(float(tqp.sum() / tot.sum()), 3),
                      "sqp_iters_per_episode_mean": round(float(its.mean()), 2),
                      "ipm_iters_per_sqp_iter": round(float(ipm.sum() / max(1.0, its.sum())), 2)})
        return r, {}, extra

    def check(self):
        """Device episode of 2 instances against the host loop mpc.simulate
        with the same converged controller (max state deviation)."""
        from model_predictive_control_amd import bicycle, mpc
        from model_predictive_control_amd.parameters import VehicleParameters

        xs = self.bufs[0]["xs"].cpu().numpy()
        fe = bicycle.fwd_euler(bicycle.KinematicBicycle(VehicleParameters()), 0.08)
        err = 0.0
        for i in range(2):
            ctl = mpc.MPCController(self.N, 0.08, VehicleParameters(), tol=1e-9)
            ref = mpc.simulate(self.X0[0, i], fe, min(self.T, 10), ctl)
            err = max(err, float(np.abs(xs[:ref.shape[0], i] - ref).max()))
        return err

    def cpu_baseline(self, seconds):
        """The host closed loop (oracle/parallel.py loop_chunk: per sample the
        oracle's converged NLP solve warm-started from the shifted solution,
        then the FE plant) over the host cores -- the reference's
        simulate(..., policy=controller) of main.py:270-271 restated."""
        from oracle import parallel

        g = self.ctl
        cores = parallel.host_cores()
        total = min(self.args.batch, 8 * cores)
        Q, QN, R = (v.cpu().numpy() for v in (g.Q, g.QN, g.R))
        r = parallel.rate(parallel.loop_chunk, lambda lo, hi, dl: (
            self.N, 0.08, Q, QN, R, g.lb_states, g.lb_inputs, self.X0[0, lo:hi], self.T, dl),
            total, seconds, cores)
        return {"value": round(r["value"], 3), "unit": "closed-loop MPC steps/s", "cores": r["cores"],
                "kind": "port",
                "sample": f"{r['done']} closed-loop steps of {self.T}-sample episodes "
                          f"(oracle/nlp.py converged solve to KKT 1e-9 per sample, warm-started "
                          f"from the shifted solution, FE plant), per-x0 episodes over "
                          f"{r['cores']} spawned processes in {r['seconds']:.1f} s"}


CONFIGS = {"2": Config2, "2loop": Config2Loop, "3": Config3, "4": Config4, "5": Config5,
           "nlp": ConfigNLP, "loop": ConfigLoop}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=0, help="timed steps (0 = config default: 200)")
    ap.add_argument("--warmup", type=int, default=-1, help="untimed steps (-1 = config default: 20)")
    ap.add_argument("--config", default="2", choices=sorted(CONFIGS),
                    help="BASELINE configs 2-5 (2 = the headline), nlp (converged "
                         "MPCController.solve), loop (on-device receding-horizon loop)")
    ap.add_argument("--sqp-iters", type=int, default=0,
                    help="nlp: SQP iterations per solve (default 60); loop: per sample (12)")
    ap.add_argument("--sqp-iterate", action="store_true",
                    help="nlp / loop: one launch sequence per SQP iteration over the batch "
                         "(SqpSolver.iterate) instead of the one-launch solve")
    ap.add_argument("--loop-steps", type=int, default=0,
                    help="loop / 2loop: closed-loop steps per episode (default 20 / 50)")
    ap.add_argument("--gather", action="store_true",
                    help="N>1: time the final all-gather of z (RCCL) after the timed loop")
    ap.add_argument("--batch", type=int, default=0, help="instances per GPU per step (0 = config default)")
    ap.add_argument("--horizon", type=int, default=0, help="N (0 = config default)")
    ap.add_argument("--slots", type=int, default=0, help="distinct x0 batches cycled over")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-chain", action="store_true",
                    help="replay one graph per step instead of one per round of slots")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--reps", type=int, default=20, help="launches per kernel-timing graph")
    ap.add_argument("--check", type=int, default=64, help="instances checked against the oracle")
    ap.add_argument("--mode", choices=("fused", "split"), default="fused", help="config 2 only")
    ap.add_argument("--traffic", default=None,
                    help="JSON with PMC-measured HBM bytes per launch {kernel: bytes} "
                         "(tools/prof_counters.sh); fills roofline.traffic")
    args = ap.parse_args()
    C = CONFIGS[args.config]
    args.batch = args.batch or C.default_batch
    args.slots = args.slots or C.default_slots
    args.sqp_iters = args.sqp_iters or getattr(C, "default_sqp_iters", 0)
    args.loop_steps = args.loop_steps or getattr(C, "default_loop_steps", 20)
    dsteps, dwarm = getattr(C, "default_steps", (200, 20))
    args.steps = args.steps or dsteps
    args.warmup = dwarm if args.warmup < 0 else args.warmup

    rank, world, local = mdist.env_rank_world()
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} rank processes")
    # N > 1: the final all-gather of z (the path's only collective) is timed by default
    args.gather = args.gather or world > 1
    # rehearsal knobs (one-GPU box): MPCQP_BENCH_DEVICE pins every rank to one
    # device, MPCQP_DIST_BACKEND=gloo replaces RCCL (which needs one GPU per rank)
    local = int(os.environ.get("MPCQP_BENCH_DEVICE", local))
    backend = os.environ.get("MPCQP_DIST_BACKEND", "nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist

        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    wl = C(args, dev, rank)
    S = args.slots
    for s in range(S):
        wl.step(s)
    torch.cuda.synchronize()
    graphs = None
    chain = None
    tail = None
    if not args.no_graph:
        try:
            graphs = []
            cap = torch.cuda.Stream(device=dev)
            for s in range(S):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=cap):
                    wl.step(s)
                graphs.append(g)
            # one graph holding a whole round of S steps (slots 0..S-1 in
            # order): the timed loop replays it K // S times, so consecutive
            # steps are not separated by a graph launch each
            if S > 1 and not args.no_chain:
                chain = torch.cuda.CUDAGraph()
                with torch.cuda.graph(chain, stream=cap):
                    for s in range(S):
                        wl.step(s)
                # the timed loop's last K % S steps (slots 0..K%S-1) as one graph too
                if args.steps % S > 1:
                    tail = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(tail, stream=cap):
                        for s in range(args.steps % S):
                            wl.step(s)
            torch.cuda.synchronize()
        except Exception as e:  # pragma: no cover - reported in the JSON
            print(f"graph capture failed ({e}); eager launches", file=sys.stderr)
            graphs = None
            chain = None
            tail = None

    def run(k):
        if graphs is not None:
            graphs[k % S].replay()
        else:
            wl.step(k % S)

    def run_steps(k0, count):
        """Steps k0 .. k0+count-1 (slot k % S each), whole rounds through the chain graph."""
        k = k0
        end = k0 + count
        while k < end:
            if chain is not None and k % S == 0 and end - k >= S:
                chain.replay()
                k += S
            elif tail is not None and k % S == 0 and end - k == args.steps % S:
                tail.replay()
                k = end
            else:
                run(k)
                k += 1

    run_steps(0, args.warmup)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_steps(0, args.steps)
    torch.cuda.synchronize()
    # each rank's clock stops when its own K steps are done (the starts are
    # aligned by the barrier above); the max over ranks below is the time until
    # the last rank finished, without the closing barrier's own latency
    elapsed = time.perf_counter() - t0
    if world > 1:
        torch.distributed.barrier()
    elapsed = mdist.max_over_ranks(elapsed, dev if backend == "nccl" else torch.device("cpu"))
    units = getattr(wl, "units_per_step", 1)
    if hasattr(wl, "counted_units"):
        # workloads whose unit can fail to converge (nlp, loop) count only the
        # converged ones: the timed steps' slots replay deterministic inputs,
        # so each slot's recorded statuses are those of every replay
        value = mdist.sum_over_ranks(float(wl.counted_units(args.steps)),
                                     dev if backend == "nccl" else torch.device("cpu")) / elapsed
    else:
        value = world * args.batch * units * args.steps / elapsed
    gather = None
    if args.gather and world > 1 and hasattr(wl, "Z"):
        gather = time_gather(wl, args, world, dev, backend)

    # ---- correctness of what was timed: statuses + oracle spot check (rank 0)
    st = wl.status()
    code = batched.status_code(st)
    opt_frac = float((code == 0).double().mean())
    if hasattr(wl, "optimal_frac"):  # the loop: per controller call, not per episode
        opt_frac = wl.optimal_frac()
    iters = batched.status_iters(st).double()

    out = None
    if rank == 0:
        # PMC-measured HBM bytes per launch (tools/traffic.sh), committed under
        # profiles/ per config; --traffic overrides
        traffic = {}
        tpath = args.traffic or os.path.join(ROOT, "profiles", f"traffic_cfg{args.config}.json")
        if os.path.exists(tpath) and (args.traffic or args.batch == C.default_batch):
            with open(tpath) as fh:
                traffic = json.load(fh)  # measured at the config's default batch
        err = wl.check()
        e2e = host_roundtrip(wl, graphs, args)
        dom, others, extra = wl.kernels(traffic)
        cpu = None
        if not args.no_cpu and world == 1:
            cpu = wl.cpu_baseline(args.cpu_seconds)
        cfg = wl.workload()
        cfg.update({"batch_per_gpu": args.batch, "parallelism": f"dp{world}",
                    "graph": graphs is not None, "graph_steps": S if chain is not None else 1,
                    "config": args.config})
        if dom is None:
            dom = {"note": "no single dominant kernel: see the nlp config for the per-kernel "
                           "rooflines of one SQP iteration"}
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "solves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": wl.dname,
            "data": "synthetic",
            "config": cfg,
            "max_abs_u_err_vs_oracle": err,
            "optimal_frac": opt_frac,
            "status_hist": {int(k): int(v) for k, v in zip(*np.unique(code.cpu().numpy(), return_counts=True))},
            "iters_mean": round(float(iters.mean()), 2),
            "iters_max": int(iters.max()),
            "roofline": dom,
            "cpu_baseline": cpu,
        }
        if e2e is not None:
            out["host_roundtrip"] = e2e
        if gather is not None:
            out["gather"] = gather
        if units != 1:
            out["unit"] = "closed-loop MPC steps/s"
        out.update(others)
        out.update(extra)
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()
    return out


def time_gather(wl, args, world, dev, backend="nccl"):
    """The only collective of the multi-GPU path: all-gather
    of every rank's solutions z (slot 0) into the whole batch on every rank,
    timed with HIP events around the collective, outside the timed loop.
    (gloo, the one-GPU rehearsal backend: host copies, host clock.)"""
    z = wl.Z[0]
    total = world * z.shape[0]
    torch.distributed.barrier()
    if backend != "nccl":
        zc = z.cpu()
        mdist.gather_shards(zc, total)
        t0 = time.perf_counter()
        full = mdist.gather_shards(zc, total)
        ms = mdist.max_over_ranks((time.perf_counter() - t0) * 1e3, torch.device("cpu"))
        note = "all-gather of z over ranks (gloo over host copies: one-GPU rehearsal)"
    else:
        mdist.gather_shards(z, total)          # warm-up (communicator setup)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        full = mdist.gather_shards(z, total)
        e1.record()
        e1.synchronize()
        ms = mdist.max_over_ranks(e0.elapsed_time(e1), dev)
        note = "all-gather of z over ranks (RCCL), after the timed loop"
    nbytes = full.numel() * full.element_size()
    return {"ms": round(ms, 4), "bytes": int(nbytes), "GBps": round(nbytes / (ms * 1e-3) / 1e9, 2),
            "note": note}


def host_roundtrip(wl, graphs, args, reps=50):
    """End-to-end rate of the receding-horizon loop with host buffers (SURVEY.md
    8(d): reported beside, never as, `value`): per step, x0 from pinned host
    memory to the device, the step (its graph), z back to pinned host memory,
    and a stream synchronize -- the host needs u before the next step.  Only
    for workloads whose step reads X0_t[s] and writes Z[s]."""
    if not (hasattr(wl, "X0_t") and hasattr(wl, "Z")):
        return None
    S = args.slots
    x0h = [wl.X0_t[s].cpu().pin_memory() for s in range(S)]
    zh = torch.empty(wl.Z[0].shape, dtype=wl.Z.dtype).pin_memory()
    st = torch.cuda.current_stream()

    def one(k):
        s = k % S
        wl.X0_t[s].copy_(x0h[s], non_blocking=True)
        if graphs is not None:
            graphs[s].replay()
        else:
            wl.step(s)
        zh.copy_(wl.Z[s], non_blocking=True)
        st.synchronize()

    for k in range(5):
        one(k)
    t0 = time.perf_counter()
    for k in range(reps):
        one(k)
    dt = (time.perf_counter() - t0) / reps
    return {"value": round(args.batch / dt, 1), "unit": "solves/s", "ms_per_step": round(dt * 1e3, 4),
            "h2d_bytes": int(x0h[0].numel() * x0h[0].element_size()),
            "d2h_bytes": int(zh.numel() * zh.element_size()),
            "note": "pinned host x0 -> device, one step, z -> pinned host, synchronize; per step"}


def spawn_ranks(n):
    """``--gpus N`` (N > 1) started without a launcher's environment: start N
    rank processes, one per GPU (RANK = LOCAL_RANK = r, WORLD_SIZE = N, a free
    127.0.0.1 rendezvous port), and wait for them.  This process never touches
    the GPU; it only starts children.  If a rank fails the others are stopped
    (they would wait at the first barrier), and the worst exit code is
    returned.  Under torchrun (WORLD_SIZE set) main() runs directly."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rcs = [None] * n
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
        if any(rc not in (None, 0) for rc in rcs):
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    p.terminate()
                    try:
                        rcs[i] = p.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        rcs[i] = p.wait()
            break
        time.sleep(0.2)
    bad = [rc for rc in rcs if rc != 0]
    return (abs(bad[0]) or 1) if bad else 0


def _gpus_arg(argv):
    for i, a in enumerate(argv):
        if a == "--gpus" and i + 1 < len(argv):
            return int(argv[i + 1])
        if a.startswith("--gpus="):
            return int(a.split("=", 1)[1])
    return 1


if __name__ == "__main__":
    ngpu = _gpus_arg(sys.argv[1:])
    if ngpu > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(ngpu))
    main()
