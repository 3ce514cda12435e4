"""Time one mpcqp_mpc_qp step of a bench config with several builds of
libmpcqp.so in one process (bisecting a regression across commits):

    python tools/ab_libs.py CONFIG LIB [LIB ...]

The inputs come from the product library (bench.ConfigN); every other
library is loaded beside it with ctypes (RTLD_LOCAL) and only its
mpcqp_mpc_qp / mpcqp_mpc_qp_workspace are used, with a workspace sized by
that library.  Each library is timed twice, alternating, on HIP events
around a graph of R steps.
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from model_predictive_control_amd import _native as nat  # noqa: E402
from model_predictive_control_amd import batched  # noqa: E402


class _A:
    pass


class _Proxy:
    """The product library, with mpcqp_mpc_qp / _workspace from another build."""

    def __init__(self, base, other):
        self._base, self._other = base, other

    def __getattr__(self, k):
        if k in ("mpcqp_mpc_qp", "mpcqp_mpc_qp_workspace"):
            return getattr(self._other, k)
        return getattr(self._base, k)


def main():
    cfg, libs = int(sys.argv[1]), sys.argv[2:]
    C = {3: bench.Config3, 5: bench.Config5}[cfg]
    a = _A()
    a.batch, a.slots, a.horizon, a.reps, a.check = C.default_batch, 1, 0, 10, 0
    dev = torch.device("cuda")
    w = C(a, dev, 0)
    base = nat.load()
    loaded = {}
    for p in libs:
        lib = ctypes.CDLL(p)
        for name in ("mpcqp_mpc_qp", "mpcqp_mpc_qp_workspace"):
            res, args = nat.SIGNATURES[name]
            getattr(lib, name).restype = res
            getattr(lib, name).argtypes = args
        loaded[p] = lib
    dt = torch.float32
    ws_base = w.ws
    for rep in range(2):
        for p, lib in loaded.items():
            nb = lib.mpcqp_mpc_qp_workspace(1, a.batch, w.nx, w.nu, w.N, 1 if cfg == 3 else 0)
            w.ws = torch.empty((nb,), dtype=torch.uint8, device=dev)
            batched._lib = lambda lib=lib: _Proxy(base, lib)  # noqa: E731
            ms = bench.time_kernel(lambda: w.step(0), 10, dev)
            torch.cuda.synchronize()
            ok = float((batched.status_code(w.ST[0]) == 0).double().mean())
            print(f"{rep} {os.path.basename(p)}"
                  f" {ms * 1e3:9.1f} us  optimal {ok:.4f}", flush=True)
    batched._lib = nat.load
    w.ws = ws_base
    del dt


if __name__ == "__main__":
    main()
