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


@pytest.mark.parametrize("total", [4096, 1001])
def test_two_ranks_shard_solve_gather_bitexact(tmp_path, total):
    out = str(tmp_path / "res.json")
    port = 29600 + (os.getpid() % 1000) + (total % 7)
    procs = []
    for rank in range(2):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "_multi_worker.py"),
                                       out, str(total)], env=env))
    rcs = [p.wait(timeout=240) for p in procs]
    assert rcs == [0, 0], rcs
    with open(out) as fh:
        res = json.load(fh)
    assert res["shape"] == [total, 20]
    assert res["bitexact"] and res["status_equal"] and res["optimal"], res
