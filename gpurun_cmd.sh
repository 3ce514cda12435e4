mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/s9_tests.log 2>&1
echo "tests rc=$?"; tail -12 gpurun_out/s9_tests.log | cut -c1-400
