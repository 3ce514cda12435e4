rm -f gpurun_out/mf.log
timeout -k 10 200 python -u tools/sqp_knobs.py --tag pipe 2>&1 | grep KNOB >> gpurun_out/mf.log || exit 1
SQP_LAT_IPM=1 timeout -k 10 200 python -u tools/sqp_latency.py >> gpurun_out/mf.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ipm.py tests/test_gpu_nlp.py tests/test_gpu_closed_loop.py tests/test_gpu_mpc_qp.py >> gpurun_out/mf.log 2>&1 || exit 1
