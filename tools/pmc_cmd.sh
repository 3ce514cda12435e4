#!/bin/bash
# PMC passes (one counter group per pass, each its own rocprofv3 run) over an
# arbitrary python command, then the per-dispatch averages of the kernels
# whose name contains PATTERN.
# Usage on the GPU box: bash tools/pmc_cmd.sh TAG PATTERN script.py [args]
TAG=$1; PAT=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG}
mkdir -p $OUT
SCRIPT=$ROOT/$1; shift
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
           "GRBM_GUI_ACTIVE SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64" \
           ${EXTRA_PMC:-}; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 $SCRIPT "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed: $grp"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 $ROOT/tools/pmc_summary.py $OUT "$PAT" | tee $OUT/summary.txt
