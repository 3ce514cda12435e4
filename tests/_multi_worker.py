"""Worker of tests/test_gpu_multi.py (one process per rank; launched with
RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in the environment).

Every rank solves its contiguous shard of one config-2 batch (per-instance
condense + input-box QP, mpcqp_mpc_box) -- or, with argument "4", of one
config-4 batch (the shared condense and polytope factors recomputed on every
rank, poly_solve of the rank's x0) -- on the GPU, the shards are gathered
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


def _config4(total, rank, world, dev):
    """bench.py Config4's data: random stable LTI nx=12 nu=4 (rho <= 0.98), N=50,
    40 polytope rows G z <= h; every rank builds the shared H, F and the
    poly_setup factors itself (cheaper than a broadcast)."""
    nx, nu, N, m = 12, 4, 50, 40
    rng = np.random.default_rng(20261015 + 4)
    U, _ = np.linalg.qr(rng.normal(size=(nx, nx)))
    A = (U * rng.uniform(0.5, 0.98, size=nx)) @ U.T
    B = rng.normal(size=(nx, nu)) / np.sqrt(nx)
    G = rng.normal(size=(m, N * nu))
    h = rng.uniform(0.5, 1.5, size=m)
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64, device=dev)  # noqa: E731
    d = batched.condense(t(A), t(B), t(np.eye(nx)), t(0.1 * np.eye(nu)), t(np.eye(nx)), N,
                         outputs=("H", "F"))
    qp = batched.PolyQP(d["H"][0].contiguous(), t(G), d["F"][0].contiguous())
    X0 = np.random.default_rng(20261015 + 99).normal(size=(total, nx)) * 3.0
    lo, hi = distributed.shard_bounds(total, rank, world)
    z, _, st = qp.solve(t(X0[lo:hi]), hu=t(h))
    torch.cuda.synchronize()
    ref = (lambda: qp.solve(t(X0), hu=t(h))) if rank == 0 else None
    return z, st, ref


def main():
    out_path, total = sys.argv[1], int(sys.argv[2])
    cfg = sys.argv[3] if len(sys.argv) > 3 else "2"
    rank, world, _ = distributed.env_rank_world()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    if cfg == "4":
        z, st, ref = _config4(total, rank, world, dev)
        zall = distributed.gather_shards(z.cpu(), total)
        sall = distributed.gather_shards(st.cpu(), total)
        if rank == 0:
            zr, _, sr = ref()
            torch.cuda.synchronize()
            res = {"bitexact": bool(torch.equal(zall, zr.cpu())), "status_equal": bool(torch.equal(sall, sr.cpu())),
                   "optimal": bool((batched.status_code(sall) == 0).all()), "shape": list(zall.shape)}
            with open(out_path, "w") as fh:
                json.dump(res, fh)
        dist.barrier()
        dist.destroy_process_group()
        return
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
