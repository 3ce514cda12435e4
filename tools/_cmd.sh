rm -f gpurun_out/pr.log
timeout -k 10 200 python -u tools/sqp_knobs.py --tag reuse 2>&1 | grep KNOB >> gpurun_out/pr.log || exit 1
for w in 0 1; do
  MPCQP_SQP_WARM=$w timeout -k 10 200 python -u tools/sqp_knobs.py --tag warm$w 2>&1 | grep KNOB >> gpurun_out/pr.log || exit 1
done
SQP_LAT_IPM=1 timeout -k 10 200 python -u tools/sqp_latency.py >> gpurun_out/pr.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ipm.py tests/test_gpu_nlp.py tests/test_gpu_closed_loop.py tests/test_gpu_mpc_qp.py >> gpurun_out/pr.log 2>&1 || exit 1
