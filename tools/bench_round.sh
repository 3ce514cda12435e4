#!/bin/bash
# Round record on the GPU box: the default bench line (config 2, as the driver
# runs it) under rocprofv3 --kernel-trace --stats, then every other workload
# (configs 3-5, nlp, loop) with its CPU baseline.  -> gpurun_out/TAG_*.json,
# gpurun_out/TAG_prof_default/ (kernel stats).
# Usage: bash tools/bench_round.sh TAG [configs...]
TAG=${1:-r03}; shift
CFGS=${@:-2 3 4 5 nlp loop}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_prof_default -o run --output-format csv \
    -- python3 $ROOT/bench.py > $OUT/${TAG}_default.json 2> $OUT/${TAG}_default.err \
    || { echo "default bench failed"; tail -5 $OUT/${TAG}_default.err; exit 1; }
echo "default:"; cut -c1-600 $OUT/${TAG}_default.json
cd $ROOT
for c in $CFGS; do
  [ "$c" = "2" ] && continue
  timeout -k 10 500 python3 bench.py --config $c > $OUT/${TAG}_cfg$c.json 2> $OUT/${TAG}_cfg$c.err
  rc=$?
  echo "cfg$c rc=$rc"; cut -c1-900 $OUT/${TAG}_cfg$c.json; tail -2 $OUT/${TAG}_cfg$c.err
  if [ $rc -ne 0 ]; then exit $rc; fi
done
