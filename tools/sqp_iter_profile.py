"""Per-iteration device time of the nlp bench line's SQP (B = 4096, N = 30,
from U = 0): HIP events around each of the 60 iterations, with the number of
instances still iterating before it.  Shows where a converged-solve budget
goes: the early full-batch iterations or the latency-bound tail.

    python tools/sqp_iter_profile.py [batch] [iters]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


class _A:
    pass


a = _A()
a.batch = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
a.sqp_iters = int(sys.argv[2]) if len(sys.argv) > 2 else 60
a.slots, a.horizon, a.reps, a.check = 1, 0, 3, 0
dev = torch.device("cuda")
w = bench.ConfigNLP(a, dev, 0)
sqp, x0 = w.sqp, w.X0_t[0]
for rep in range(2):
    sqp.reset()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.sqp_iters + 1)]
    act = []
    ev[0].record()
    for k in range(a.sqp_iters):
        act.append(a.batch - int(sqp.done().sum()) if rep == 1 else -1)
        if rep == 1:
            ev[k].record()
        sqp.iterate(x0)
        ev[k + 1].record()
    torch.cuda.synchronize()
    if rep == 0:
        continue
    ts = [ev[k].elapsed_time(ev[k + 1]) for k in range(a.sqp_iters)]
    tot = sum(ts)
    print(f"total {tot:.1f} ms over {a.sqp_iters} iterations")
    cum = 0.0
    for k, (t, n) in enumerate(zip(ts, act)):
        cum += t
        print(f"it {k:2d} active {n:5d}  {t:7.2f} ms  cum {cum:7.1f} ms ({100 * cum / tot:4.1f} %)")
