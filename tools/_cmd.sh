timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full_gpu2.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke2.log 2>&1 || exit 1
timeout -k 10 600 bash tools/bench_round.sh r06c 2 nlp loop > gpurun_out/r06c_round.log 2>&1 || exit 1
