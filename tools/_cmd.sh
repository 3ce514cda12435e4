set -o pipefail
timeout -k 10 200 python -u tools/sqp_latency.py --iters 150 > gpurun_out/lat6.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/sqp_latency.py --batch 64 --iters 150 >> gpurun_out/lat6.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_nlp.py tests/test_gpu_closed_loop.py > gpurun_out/t4.log 2>&1 || { tail -30 gpurun_out/t4.log; exit 1; }
tail -2 gpurun_out/t4.log
timeout -k 10 300 python -u bench.py --config nlp --no-cpu > gpurun_out/b_nlp.json 2> gpurun_out/b_nlp.err || exit 1
timeout -k 10 300 python -u bench.py --config loop --no-cpu > gpurun_out/b_loop.json 2> gpurun_out/b_loop.err || exit 1
