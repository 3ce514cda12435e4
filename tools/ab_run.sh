#!/bin/bash
# On the GPU box: bench one config with the product library and each variant
# (tools/ab_build.sh), alternating twice.  Usage: bash tools/ab_run.sh CFG TAG... [-- bench args]
CFG=$1; shift
TAGS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do TAGS+=("$1"); shift; done
[ "$1" = "--" ] && shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out; mkdir -p $OUT
cd $ROOT
for rep in 1 2; do
  for t in base "${TAGS[@]}"; do
    lib=$ROOT/model_predictive_control_amd/lib/libmpcqp.so
    [ "$t" != base ] && lib=$ROOT/model_predictive_control_amd/lib/variants/libmpcqp_$t.so
    MPCQP_LIB=$lib timeout -k 10 300 python bench.py --config $CFG --no-cpu "$@" > $OUT/ab_${CFG}_${t}_$rep.json 2> $OUT/ab_${CFG}_${t}_$rep.err \
      || { echo "FAIL $t"; tail -5 $OUT/ab_${CFG}_${t}_$rep.err; exit 1; }
    python3 -c "
import json,sys
d=json.load(open('$OUT/ab_${CFG}_${t}_$rep.json'))
print('$t', d['value'], d.get('kernel_us'), 'err', d.get('max_abs_u_err_vs_oracle'), 'it', d.get('iters_mean'), d.get('iters_max'))"
  done
done
