timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full_gpu4.log 2>&1 || exit 1
timeout -k 10 600 bash tools/bench_round.sh r06e nlp loop > gpurun_out/r06e_round.log 2>&1 || exit 1
