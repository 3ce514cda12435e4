#!/bin/bash
# MFMA-utilisation counters (one --pmc pass) over a short eager bench run of a
# config, summarised per kernel (tools/mfma_summary.py).
# Usage on the GPU box: bash tools/mfma_counters.sh CONFIG TAG
C=${1:-3}; TAG=${2:-mfma}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG}_cfg$C
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BENCH="python $ROOT/bench.py --config $C --no-cpu --no-graph --steps 5 --warmup 1 --reps 2"
PMC="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -k 10 300 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d $OUT/p -o run -- $BENCH > $OUT/p.log 2>&1 || { echo "pmc pass failed"; tail -5 $OUT/p.log; exit 1; }
python3 $ROOT/tools/mfma_summary.py $(find $OUT/p -name "*counter_collection.csv") $(find $OUT/p -name "*kernel_trace.csv") | tee $OUT/summary.txt
