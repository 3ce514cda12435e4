"""Worker of tests/test_gpu_multi.py (one process per rank; launched with
RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in the environment).

Every rank solves its contiguous shard of one config-2 batch (per-instance
condense + input-box QP, mpcqp_mpc_box) on the GPU, the shards are gathered
with distributed.gather_shards (the only collective of the path, SURVEY.md
8(e)), and rank 0 compares the gathered trajectories bit for bit with the
unsharded solve of the whole batch.  Backend: gloo (both ranks share the one
GPU of the test box; RCCL needs a GPU per rank), gathering host copies.
"""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from model_predictive_control_amd import batched, distributed  # noqa: E402


def main():
    out_path, total = sys.argv[1], int(sys.argv[2])
    rank, world, _ = distributed.env_rank_world()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    ts = 0.5
    A = np.array([[1.0, ts], [0.0, 1.0]])
    B = np.array([[0.0], [-ts]])
    C = np.array([[1.0], [-2.0 / 3.0]])
    Q = C @ C.T + 1e-3 * np.eye(2)
    N = 20
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64, device=dev)  # noqa: E731
    X0 = np.random.default_rng(20261015 + 77).uniform(-10, 10, (total, 2))
    lo, hi = distributed.shard_bounds(total, rank, world)
    z, st = batched.mpc_box(t(np.broadcast_to(A, (hi - lo, 2, 2))), t(np.broadcast_to(B, (hi - lo, 2, 1))),
                            t(Q), t([[0.1]]), t(Q), N, t(X0[lo:hi]), -1.0, 1.0)
    torch.cuda.synchronize()
    zall = distributed.gather_shards(z.cpu(), total)
    sall = distributed.gather_shards(st.cpu(), total)
    if rank == 0:
        zr, sr = batched.mpc_box(t(np.broadcast_to(A, (total, 2, 2))), t(np.broadcast_to(B, (total, 2, 1))),
                                 t(Q), t([[0.1]]), t(Q), N, t(X0), -1.0, 1.0)
        torch.cuda.synchronize()
        res = {"bitexact": bool(torch.equal(zall, zr.cpu())), "status_equal": bool(torch.equal(sall, sr.cpu())),
               "optimal": bool((batched.status_code(sall) == 0).all()), "shape": list(zall.shape)}
        with open(out_path, "w") as fh:
            json.dump(res, fh)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
