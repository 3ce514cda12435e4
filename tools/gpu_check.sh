#!/bin/bash
# GPU-box check used during development: pytest -m gpu, smoke, bench, rocprof.
# Usage (from the repo root on the GPU box): bash tools/gpu_check.sh TAG [bench args...]
TAG=${1:-r1}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $OUT/${TAG}_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 $OUT/${TAG}_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.log 2>&1 || { echo smoke failed; cat $OUT/${TAG}_smoke.log; exit 3; }
cat $OUT/${TAG}_smoke.log
timeout -k 10 600 python bench.py "$@" > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err || { echo bench failed; tail -20 $OUT/${TAG}_bench.err; exit 4; }
cat $OUT/${TAG}_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_prof -o run --output-format csv -- python $ROOT/bench.py --no-cpu --steps 100 "$@" > $OUT/${TAG}_prof.log 2>&1 || { echo rocprof failed; tail -20 $OUT/${TAG}_prof.log; exit 5; }
for f in $(find $OUT/${TAG}_prof -name "*kernel_stats.csv"); do cat $f | cut -c1-250; done
