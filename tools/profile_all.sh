#!/bin/bash
# Per config: PMC HBM traffic (tools/traffic.sh) and a rocprofv3 kernel-trace
# --stats summary of a short bench run.  Results under gpurun_out/.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}; shift
for c in ${CONFIGS:-2 3 4 5}; do
  bash $ROOT/tools/traffic.sh $c || exit 1
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/${TAG}_prof_cfg$c -o run --output-format csv -- python $ROOT/bench.py --config $c --no-cpu --steps ${STEPS:-20} --warmup 2 > $ROOT/gpurun_out/${TAG}_prof_cfg$c.log 2>&1) || { echo "rocprof cfg$c failed"; tail -5 $ROOT/gpurun_out/${TAG}_prof_cfg$c.log; exit 1; }
  echo "== cfg$c"; cut -c1-200 $(find $ROOT/gpurun_out/${TAG}_prof_cfg$c -name "*kernel_stats.csv") | head -6
done
