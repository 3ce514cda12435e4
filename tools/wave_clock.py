"""Per-wave end-time histogram of the headline kernel (config 2, the fused
mpc_group_kernel at B = 4096: 1,024 waves of four QPs, one wave per SIMD).

Build (container):  bash tools/ab_build.sh wclk "-DMPCQP_WAVE_CLOCK" quad_box.hip
Run (GPU box):      python tools/wave_clock.py [--out profiles/r04/wave_clock_cfg2.json]
Each wave records s_memrealtime (100 MHz) at entry and exit and the largest GI
iteration count of its four QPs; the kernel lasts as long as its slowest wave,
so the tail of this distribution is what the kernel time is made of."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("MPCQP_LIB", os.path.join(ROOT, "model_predictive_control_amd", "lib",
                                                "variants", "libmpcqp_wclk.so"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from model_predictive_control_amd import _native, batched  # noqa: E402

lib = _native.load()
lib.mpcqp_debug_wave_clock.argtypes = [ctypes.c_void_p, ctypes.c_int]
dev = torch.device("cuda")
B, N = 4096, 20
ts = 0.5
A = np.array([[1.0, ts], [0.0, 1.0]]); Bm = np.array([[0.0], [-ts]])
C = np.array([[1.0], [-2.0 / 3.0]]); Q = C @ C.T + 1e-3 * np.eye(2)
t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64, device=dev)  # noqa: E731
rng = np.random.default_rng(20261015 + 2)
X0 = t(rng.uniform(-10.0, 10.0, size=(B, 2)))
Ab, Bb = t(np.broadcast_to(A, (B, 2, 2))), t(np.broadcast_to(Bm, (B, 2, 1)))
lb = torch.full((N,), -1.0, dtype=torch.float64, device=dev)
ub = torch.full((N,), 1.0, dtype=torch.float64, device=dev)
runs = []
for rep in range(6):
    z, st = batched.mpc_box(Ab, Bb, t(Q), t([[0.1]]), t(Q), N, X0, lb, ub)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (3 * 1024))()
    assert lib.mpcqp_debug_wave_clock(buf, 1024) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 3).astype(np.int64)
    if rep >= 1:
        runs.append(a)
res = []
for a in runs:
    t0 = a[:, 0].min()
    start = (a[:, 0] - t0) * 10e-3   # us (100 MHz)
    end = (a[:, 1] - t0) * 10e-3
    dur = end - start
    it = a[:, 2]
    res.append(dict(kernel_us=float(end.max()), start_max_us=float(start.max()),
                    dur_p50=float(np.percentile(dur, 50)), dur_p90=float(np.percentile(dur, 90)),
                    dur_p99=float(np.percentile(dur, 99)), dur_max=float(dur.max()),
                    end_p50=float(np.percentile(end, 50)), end_p90=float(np.percentile(end, 90)),
                    iters_max_mean=float(it.mean()), iters_max_max=int(it.max()),
                    corr_dur_iters=float(np.corrcoef(dur, it)[0, 1])))
a = runs[-1]
t0 = a[:, 0].min()
dur = (a[:, 1] - a[:, 0]) * 10e-3
it = a[:, 2]
hist, edges = np.histogram(dur, bins=12)
by_iter = {int(k): round(float(dur[it == k].mean()), 2) for k in np.unique(it)}
out = {"kernel": "mpc_group_kernel<double,2,1,QSym<double,5>,16,2> (config 2, B = 4096, 1024 waves)",
       "runs": res, "hist_dur_us": {"edges": [round(float(e), 2) for e in edges],
                                     "counts": hist.tolist()},
       "mean_dur_us_by_wave_max_iters": by_iter,
       "waves_by_max_iters": {int(k): int((it == k).sum()) for k in np.unique(it)}}
print(json.dumps(out, indent=1))
if "--out" in sys.argv:
    with open(sys.argv[sys.argv.index("--out") + 1], "w") as fh:
        json.dump(out, fh, indent=1)
