#!/bin/bash
# HBM traffic per launch from PMC counters, as MI355X_MICROARCH.md "HBM" prescribes:
# FETCH_SIZE and WRITE_SIZE in separate --pmc passes (they do not fit one pass),
# FETCH_SIZE doubled on gfx950 (wide streaming reads are tallied at half), KB -> B.
# Usage on the GPU box: bash tools/traffic.sh CONFIG  ->  gpurun_out/traffic_cfgCONFIG.json
C=${1:-2}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/traffic$C
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BENCH="python $ROOT/bench.py --config $C --no-cpu --no-graph --check 0 --steps 5 --warmup 1 --reps 2 $@"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/f -o run -- $BENCH > $OUT/f.log 2>&1 || { echo "FETCH pass failed"; tail -5 $OUT/f.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/w -o run -- $BENCH > $OUT/w.log 2>&1 || { echo "WRITE pass failed"; tail -5 $OUT/w.log; exit 1; }
python3 $ROOT/tools/traffic_json.py $C $(find $OUT/f -name "*counter_collection.csv") $(find $OUT/w -name "*counter_collection.csv") > $ROOT/gpurun_out/traffic_cfg$C.json
cat $ROOT/gpurun_out/traffic_cfg$C.json
