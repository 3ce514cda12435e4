"""Config-3 condensing (condense_kernel<float,4>, B = 65,536): device time per
output set, and the WRITE_SIZE / FETCH_SIZE calibration on known byte counts.

    python tools/condense_probe.py                # time each output set
    python tools/condense_probe.py pmc SET        # 5 launches of SET (for one rocprofv3 --pmc pass)

SETs: H (packed H only: n(n+1)/2 floats per instance, the known byte count of
the ring's 16-byte non-temporal stores), Hf, HfG (the mpcqp_mpc_qp set: H, f,
packed Gamma), HfGd (H, f, dense Gamma).  tools/calib_condense.sh runs the
passes and tools/calib_reduce.py compares the counters with these counts.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from model_predictive_control_amd import batched  # noqa: E402

SETS = {"H": (("H",), False), "Hf": (("H", "f"), False), "HfG": (("H", "f", "Gam"), True),
        "HfGd": (("H", "f", "Gam"), False)}


def known_bytes(name, batch, nx=4, nu=2, N=30):
    """Exact bytes written / read by one launch of SET (4-byte elements)."""
    outs, packed = SETS[name]
    n = N * nu
    w = n * (n + 1) // 2
    if "f" in outs:
        w += n
    if "Gam" in outs:
        w += nx * nu * N * (N + 1) // 2 if packed else N * nx * n
    r = N * (nx * nx + nx * nu + nx) + nx + nx * nx * 2 + nu * nu  # A, B, c, x0, Q, Qf, R
    return {"write": 4 * w * batch, "read": 4 * r * batch}


class _A:
    pass


def main():
    a = _A()
    a.batch, a.slots, a.horizon, a.reps, a.check = 65536, 1, 0, 20, 0
    dev = torch.device("cuda")
    w = bench.Config3(a, dev, 0)
    pmc = len(sys.argv) > 2 and sys.argv[1] == "pmc"
    names = [sys.argv[2]] if pmc else list(SETS)
    for name in names:
        outs, packed = SETS[name]
        out = {}
        fn = lambda: batched.condense(w.A[0], w.B[0], w.Q_t, w.R_t, w.QN_t, w.N,  # noqa: E731
                                      x0=w.X0_t[0], c=w.c[0], tv=True, outputs=outs, out=out,
                                      gam_packed=packed)
        out.update(fn())
        if pmc:
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            continue
        ms = bench.time_kernel(fn, 20, dev)
        kb = known_bytes(name, a.batch)
        tot = kb["write"] + kb["read"]
        print(f"{name:5s} {ms * 1e3:8.1f} us  moved {tot / 1e6:8.1f} MB  {tot / ms / 1e6:7.1f} GB/s")


if __name__ == "__main__":
    main()
