set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_closed_loop.py > gpurun_out/t3.log 2>&1 || { tail -30 gpurun_out/t3.log; exit 1; }
tail -2 gpurun_out/t3.log
for it in 12 30 60; do timeout -k 10 300 python -u bench.py --config loop --no-cpu --sqp-iters $it > gpurun_out/b_loop_$it.json 2> gpurun_out/b_loop_$it.err || exit 1; done
