#!/bin/bash
# WRITE_SIZE / FETCH_SIZE calibration of the config-3 condensing kernel on
# known byte counts (MI355X_MICROARCH.md "HBM": other access widths are
# uncalibrated).  One rocprofv3 --pmc pass per counter and output set.
# On the GPU box: bash tools/calib_condense.sh  ->  gpurun_out/calib_condense.json
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/calib
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for s in H HfG HfGd; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/${s}_$c -o run \
      -- python3 $ROOT/tools/condense_probe.py pmc $s > $OUT/${s}_$c.log 2>&1 \
      || { echo "pass $s $c failed"; tail -5 $OUT/${s}_$c.log; exit 1; }
  done
done
python3 $ROOT/tools/calib_reduce.py $OUT > $ROOT/gpurun_out/calib_condense.json && cat $ROOT/gpurun_out/calib_condense.json
