rm -f gpurun_out/st.log
timeout -k 10 200 python -u tools/sqp_knobs.py --tag hoist 2>&1 | grep KNOB >> gpurun_out/st.log || exit 1
MPCQP_LIB=model_predictive_control_amd/lib/variants/libmpcqp_passclk.so timeout -k 10 200 python -u tools/sqp_latency.py >> gpurun_out/st.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_nlp.py tests/test_gpu_closed_loop.py >> gpurun_out/st.log 2>&1 || exit 1
