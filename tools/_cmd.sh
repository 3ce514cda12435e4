rm -f gpurun_out/ipmw.log
for w in 0 1; do
  echo "== MPCQP_IPM_WAVE=$w" >> gpurun_out/ipmw.log
  MPCQP_IPM_WAVE=$w SQP_LAT_IPM=1 timeout -k 10 200 python -u tools/sqp_latency.py >> gpurun_out/ipmw.log 2>&1 || exit 1
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ipm.py tests/test_gpu_nlp.py tests/test_gpu_closed_loop.py tests/test_gpu_mpc_qp.py >> gpurun_out/ipmw.log 2>&1 || exit 1
