timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full_gpu5.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke5.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/default5.json 2> gpurun_out/default5.err || exit 1
