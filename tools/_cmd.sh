timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ipm.py > gpurun_out/ipmt.log 2>&1 || exit 1
