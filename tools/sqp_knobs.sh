#!/bin/bash
# Sweep of SQP knobs (tools/sqp_knobs.py), one process per configuration:
#   bash tools/sqp_knobs.sh > gpurun_out/knobs.log
# Each line of CONFIGS: tag, then VAR=value assignments.
CONFIGS=${CONFIGS:-"base
fix0 MPCQP_SQP_FIX=0
sw1 MPCQP_SQP_SWITCH=1.0
sw01 MPCQP_SQP_SWITCH=0.1
gn8 MPCQP_SQP_GN_MAX=8
gn30 MPCQP_SQP_GN_MAX=30
wd0 MPCQP_SQP_WATCHDOG=0
wd3 MPCQP_SQP_WATCHDOG=3
pj0 MPCQP_SQP_PROJ_STEPS=0
pj8 MPCQP_SQP_PROJ_STEPS=8
mud05 MPCQP_SQP_MU_DEC=0.5
qp40 MPCQP_SQP_QP_MAX_ITER=40
rho10 MPCQP_SQP_FIX_RHO=10
rho1e4 MPCQP_SQP_FIX_RHO=1e4"}
while read -r tag rest; do
  [ -z "$tag" ] && continue
  env $rest timeout -k 5 120 python -u tools/sqp_knobs.py --tag "$tag" 2>&1 | grep "KNOB" || echo "KNOB {\"tag\": \"$tag\", \"failed\": true}"
done <<< "$CONFIGS"
