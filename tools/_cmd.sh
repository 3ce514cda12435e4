set -o pipefail
for it in 60 100; do timeout -k 10 300 python -u bench.py --config loop --no-cpu --sqp-iters $it > gpurun_out/b_loop_$it.json 2> gpurun_out/b_loop_$it.err || exit 1; done
