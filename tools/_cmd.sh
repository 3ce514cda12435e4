set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_nlp.py tests/test_gpu_closed_loop.py tests/test_gpu_ipm.py > gpurun_out/t7.log 2>&1 || { tail -30 gpurun_out/t7.log; exit 1; }
tail -1 gpurun_out/t7.log
timeout -k 10 300 python -u bench.py --config nlp --no-cpu > gpurun_out/b_nlp.json 2> gpurun_out/b_nlp.err || exit 1
timeout -k 10 300 python -u bench.py --config loop --no-cpu > gpurun_out/b_loop.json 2> gpurun_out/b_loop.err || exit 1
