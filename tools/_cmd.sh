L=model_predictive_control_amd/lib/variants/libmpcqp_pe0.so
rm -f gpurun_out/pe0.log
MPCQP_LIB=$L timeout -k 10 200 python -u tools/sqp_knobs.py --tag pe0 2>&1 | grep KNOB >> gpurun_out/pe0.log || exit 1
MPCQP_LIB=$L timeout -k 10 300 python3 bench.py --config loop --no-cpu > gpurun_out/pe0_loop.json 2>/dev/null || exit 1
MPCQP_LIB=$L timeout -k 10 200 python -u tools/sqp_minima.py gpurun_out/min_pe0.npz > /dev/null 2>&1 || exit 1
timeout -k 10 200 python -u tools/sqp_minima.py gpurun_out/min_base.npz > /dev/null 2>&1 || exit 1
MPCQP_LIB=$L timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_nlp.py tests/test_gpu_closed_loop.py tests/test_gpu_ipm.py >> gpurun_out/pe0.log 2>&1 || exit 1
