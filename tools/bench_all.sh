#!/bin/bash
# Every BASELINE config through bench.py (short runs) -> gpurun_out/TAG_cfgN.json
TAG=${1:-all}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
for c in 2 3 4 5; do
  timeout -k 10 400 python bench.py --config $c --steps ${STEPS:-20} --warmup 3 --cpu-seconds ${CPUS:-5} "$@" \
      > $OUT/${TAG}_cfg$c.json 2> $OUT/${TAG}_cfg$c.err
  rc=$?
  echo "cfg$c rc=$rc"; cat $OUT/${TAG}_cfg$c.json | cut -c1-1500; tail -3 $OUT/${TAG}_cfg$c.err
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
