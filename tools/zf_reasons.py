"""Why the config-3 fp32 z-space kernel hands instances to the fp64 path:
runs the bench's config-3 batch with MPCQP_MPC_FALLBACK=none and counts the
hand-off reasons (status bits 24..27, solve_zf.hip): 1 row buffers full,
2 working set full, 3 undecided, 4 refinement rounds spent, 5 release
failed, 6 non-finite.  GPU tool."""
import argparse
import os
import sys

import numpy as np
import torch

os.environ["MPCQP_MPC_FALLBACK"] = "none"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda")
args = argparse.Namespace(batch=65536, slots=1, horizon=30, reps=3, check=0)
C = bench.Config3(args, dev, 0)
C.step(0)
torch.cuda.synchronize()
st = C.ST[0].cpu().numpy()
code = st & 0xFF
ret = code == 0x7F
print("hand-offs", int(ret.sum()), "of", st.size)
why = (st[ret] >> 24) & 0xF
print("reasons", dict(zip(*[v.tolist() for v in np.unique(why, return_counts=True)])))
its = (st >> 8) & 0xFFFF
print("iters of hand-offs: mean", float(its[ret].mean()) if ret.any() else 0, "others", float(its[~ret].mean()))
np.save("gpurun_out/zf_retry_idx.npy", np.nonzero(ret)[0])
