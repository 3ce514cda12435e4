"""Per-phase cycle counts of the fused config-2 kernel (mpc_quad_kernel).

Build (in the container):  python tools/phase_timing.py --build
Run (GPU box):             python tools/phase_timing.py
The debug library (-DMPCQP_PHASE_TIMING) is separate from the product one;
lane 0 of each wave adds s_memtime deltas per phase into a device array.
"""
import ctypes, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CS = os.environ.get("PT_CS", os.path.join(ROOT, "model_predictive_control_amd", "csrc"))
LIB = os.path.join(ROOT, "model_predictive_control_amd", "lib", "libmpcqp_timing.so")
SRCS = ["api.cpp", "condense.hip", "solve_box.hip", "solve_poly.hip", "mpc_box.hip", "quad_box.hip",
        "solve_qp.hip", "sweep.hip", "solve_pf.hip", "solve_zf.hip", "fallback64.hip", "mpc_qp.hip", "bicycle.hip", "misc.hip",
        "ipm.hip", "sqp.hip", "loop_box.hip"]
PHASES = ["stage-in", "Riccati", "xbar/adjoint", "-H^-1 columns", "GI: refresh/recheck", "GI: scan+argmax", "GI: pivot col+ratio", "GI: sweep"]

DYN = "--dyn" in sys.argv or (len(sys.argv) > 1 and sys.argv[1].startswith("dyn"))
if DYN:  # a separate library whose pf kernel clock times the DYN refinement
    LIB = LIB.replace("_timing.so", "_timing_dyn.so")
LIB = os.environ.get("PT_LIB", LIB)  # A/B: build and time two variants side by side

if "--build" in sys.argv:
    from concurrent.futures import ThreadPoolExecutor

    def compile_one(s):
        o = f"/tmp/timing_{os.path.basename(LIB)}_{s}.o"
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
                        "-DMPCQP_PHASE_TIMING"] + (["-DMPCQP_PHASE_DYN"] if DYN else []) + [
                        "-I", os.path.join(ROOT, "include"), "-c"]
                       + (["-mllvm", "-pragma-unroll-threshold=1000000"] if s == "sweep.hip" else []) + [
                        os.path.join(CS, s), "-o", o], check=True)
        return o

    with ThreadPoolExecutor(6) as ex:
        objs = list(ex.map(compile_one, SRCS))
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "--offload-arch=gfx950", "-o", LIB] + objs, check=True)
    print("built", LIB)
    sys.exit(0)

os.environ["MPCQP_LIB"] = LIB
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from model_predictive_control_amd import _native, batched  # noqa: E402

lib = _native.load()
arg = sys.argv[1] if len(sys.argv) > 1 else "2"
zf = arg.startswith("zf")
pf = arg.startswith("pf") or arg.startswith("dyn")
cfg = int(arg[2:]) if zf else int(arg[3:] if arg.startswith("dyn") else (arg[2:] if pf else arg))
reader = lib.mpcqp_debug_phase_cycles if cfg == 2 else lib.mpcqp_debug_phase_cycles_qp
reader.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_ulonglong * 8)()


class A:
    pass


R = 10
if cfg == 2:
    a = A(); a.batch = 4096; a.slots = 1; a.horizon = 0; a.reps = 1; a.mode = "fused"
    w = bench.Config2(a, torch.device("cuda"), 0)
    run = lambda: w._fused(0)  # noqa: E731
    waves = (a.batch + 3) // 4 * R
elif cfg == 55:
    # condense_mfma_kernel of config 5 (phase 0 backward W~/What, 1 forward Gamma~/E)
    reader = lib.mpcqp_debug_phase_cycles_condense
    reader.argtypes = [ctypes.c_void_p, ctypes.c_int]
    PHASES = ["backward W/What", "fw: loads+What", "fw: MFMA tiles", "fw: Gam/H epilogue", "fw: E tile", "", "", ""]
    if os.environ.get("MPCQP_CONDENSE_FH", "1") != "0":  # condense_mfma_fh_kernel's phases
        PHASES = ["backward", "fw: LDS What A, blend", "fw: MFMA tiles + xbar/f", "fw: H stores",
                  "fw: next loads", "", "", ""]
    a = A(); a.batch = 32768; a.slots = 1; a.horizon = 0; a.reps = 1
    w = bench.CONFIGS["5"](a, torch.device("cuda"), 0)
    run = lambda: batched.condense(w.A[0], w.B[0], w.Q_t, w.R_t, w.Q_t, w.N, x0=w.X0_t[0],  # noqa: E731
                                   tv=True, outputs=("H", "f"))
    waves = a.batch * R
elif cfg in (35, 36):
    # sweep_rows_kernel of config 3 (35: one mpc_qp step; the sweep's clock only)
    reader = lib.mpcqp_debug_phase_cycles_sweep
    reader.argtypes = [ctypes.c_void_p, ctypes.c_int]
    PHASES = ["loads", "chol_inv16", "W + zz update", "row tiles", "M_kz, M_kk", "out: zz + s0",
              "out: rows + M_GG", ""]
    a = A(); a.batch = int(os.environ.get("PT_BATCH", 65536)); a.slots = 1; a.horizon = 0; a.reps = 1
    a.check = 0
    w = bench.CONFIGS["3"](a, torch.device("cuda"), 0)
    run = lambda: w.step(0)  # noqa: E731
    waves = a.batch * R
elif cfg == 33:
    # condense_kernel<float, 4> of config 3 (all four outputs of mpc_qp)
    reader = lib.mpcqp_debug_phase_cycles_condense
    reader.argtypes = [ctypes.c_void_p, ctypes.c_int]
    PHASES = ["stage-in", "W + xbar recursion", "adjoint y", "f, xbar out", "What + column sweep", "", "", ""]
    a = A(); a.batch = 65536; a.slots = 1; a.horizon = 0; a.reps = 1; a.check = 0
    w = bench.Config3(a, torch.device("cuda"), 0)
    run = lambda: batched.condense(w.A[0], w.B[0], w.Q_t, w.R_t, w.QN_t, w.N, x0=w.X0_t[0],  # noqa: E731
                                   c=w.c[0], tv=True, outputs=("H", "f", "Gam", "xbar"))
    waves = a.batch * R
elif zf:
    # qp_zf_kernel of config 3 (one mpc_qp step; the zf kernel's clock only)
    reader = lib.mpcqp_debug_phase_cycles_zf
    reader.argtypes = [ctypes.c_void_p, ctypes.c_int]
    PHASES = ["setup: loads, H rows", "H^-1 sweep", "z0 + first rollout", "GI: scan, rows, a",
              "GI: iteration body", "refine: residual", "refine: cert + correction", "output"]
    a = A(); a.batch = int(os.environ.get("PT_BATCH", 65536)); a.slots = 1; a.horizon = 0
    a.reps = 1; a.check = 0
    w = bench.CONFIGS["3"](a, torch.device("cuda"), 0)
    run = lambda: w.step(0)  # noqa: E731
    waves = a.batch * R
elif pf:
    # qp_pf_kernel of config 3 / 5 (one wave per instance)
    reader = lib.mpcqp_debug_phase_cycles_pf
    reader.argtypes = [ctypes.c_void_p, ctypes.c_int]
    # (mpcqp_mpc_qp: the DYN kernel; its refinement residual is charged to
    # phase 0 and the M0 correction to phase 7)
    PHASES = ["setup + s0 (+DYN residual)", "refresh", "scan + col load", "gather + S^-1 u",
              "M0[:,P] v", "ratio + update", "S^-1 update", "refinement (correction)"]
    if DYN:
        PHASES = ["active set (all)", "DYN: stage loads", "DYN: forward", "DYN: backward",
                  "DYN: residual tail", "correction (M0)", "re-scan", "output"]
    a = A(); a.batch = int(os.environ.get("PT_BATCH", 4096)); a.slots = 1; a.horizon = 0; a.reps = 1
    a.check = 0
    w = bench.CONFIGS[str(cfg)](a, torch.device("cuda"), 0)
    run = lambda: w.step(0)  # noqa: E731
    waves = a.batch * R
else:
    # qp_wg_kernel of config 3 / 5 (phases 0..3: K load, z sweep-in, GI, refinement)
    PHASES = ["load K", "sweep-in z", "active set", "refinement", "", "", "", ""]
    a = A(); a.batch = 4096; a.slots = 1; a.horizon = 0; a.reps = 1
    a.check = 0
    w = bench.CONFIGS[str(cfg)](a, torch.device("cuda"), 0)
    if cfg == 3:
        d = batched.condense(w.A[0], w.B[0], w.Q_t, w.R_t, w.QN_t, w.N, x0=w.X0_t[0], c=w.c[0],
                             tv=True, outputs=("H", "f", "Gam", "xbar"))
        run = lambda: batched.solve_qp(d["H"], d["f"], d["Gam"], w.xmin_t - d["xbar"],  # noqa: E731
                                       w.xmax_t - d["xbar"], w.lbz, w.ubz, presweep=False)
    else:
        d = batched.condense(w.A[0], w.B[0], w.Q_t, w.R_t, w.Q_t, w.N, x0=w.X0_t[0], tv=True)
        run = lambda: batched.solve_box(d["H"], d["f"], w.lb_t, w.ub_t, presweep=False)  # noqa: E731
    waves = a.batch * 8 * R  # 512-thread workgroups
run()
torch.cuda.synchronize()
reader(buf, 1)
for _ in range(R):
    run()
torch.cuda.synchronize()
reader(buf, 1)
tot = sum(buf[i] for i in range(8))
for i, name in enumerate(PHASES):
    if not name:
        continue
    print(f"{name:16s} {buf[i] / waves:10.0f} cycles/wave  {100 * buf[i] / tot:5.1f} %")
