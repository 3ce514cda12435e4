"""GPU: the multi-GPU path with the real solver -- two rank
processes each solve a contiguous shard of one config-2 batch on the GPU
(mpcqp_mpc_box), gather_shards reassembles it, and the result must equal the
unsharded solve bit for bit (instances are independent; nothing on the solve
path communicates).  Both ranks share the box's one GPU, so the collective
runs on gloo over host copies; RCCL over xGMI is the same call on an 8-GPU
node (bench.py --gpus N --gather)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("cfg,total,n", [("2", 4096, 20), ("2", 1001, 20), ("4", 3000, 200)])
def test_two_ranks_shard_solve_gather_bitexact(tmp_path, cfg, total, n):
    """Config 2 (per-instance condense + box QP) and config 4 (the shared
    polytope factors poly_setup recomputed on every rank, then poly_solve of
    the rank's x0 shard): the gathered batch equals the unsharded solve bit
    for bit."""
    out = str(tmp_path / "res.json")
    port = 29600 + (os.getpid() % 1000) + (total % 7) + 11 * int(cfg)
    procs = []
    for rank in range(2):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "_multi_worker.py"),
                                       out, str(total), cfg], env=env))
    rcs = [p.wait(timeout=240) for p in procs]
    assert rcs == [0, 0], rcs
    with open(out) as fh:
        res = json.load(fh)
    assert res["shape"] == [total, n]
    assert res["bitexact"] and res["status_equal"] and res["optimal"], res


@pytest.mark.parametrize("cfg,batch,n,es,tol", [(None, None, 20, 8, 1e-9), ("4", 2048, 200, 8, 1e-9),
                                                ("5", 1024, 160, 4, 1e-5)])
def test_bench_gpus2_spawns_two_ranks(cfg, batch, n, es, tol):
    """`python bench.py --gpus 2` without a launcher starts its two rank
    processes itself (the driver's N-GPU invocation).  On the
    one-GPU test box both ranks are pinned to device 0 and gather over gloo.
    Also the two configurations BASELINE names as 8-GPU runs (4: shared
    polytope factors recomputed per rank; 5: per-instance re-condensing) at a
    reduced batch: both ranks solve their shard, every instance optimal, the
    rank-0 oracle check, the gathered bytes."""
    env = dict(os.environ, MPCQP_BENCH_DEVICE="0", MPCQP_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    extra = ["--config", cfg, "--batch", str(batch)] if cfg else []
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "8",
                        "--warmup", "2", "--no-cpu", "--check", "16"] + extra,
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2
    assert res["config"]["parallelism"] == "dp2"
    assert res["optimal_frac"] == 1.0
    assert res["max_abs_u_err_vs_oracle"] < tol
    assert res["gather"]["bytes"] == 2 * res["config"]["batch_per_gpu"] * n * es
