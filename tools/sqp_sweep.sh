#!/bin/bash
# Development sweep: SQP convergence (tools/sqp_timing.py) under settings of
# the damping schedule.  Usage on the GPU box: bash tools/sqp_sweep.sh N
N=${1:-30}
run() { echo "== $*"; env "$@" timeout -k 10 100 python -u tools/sqp_timing.py $N || exit 1; }
run MPCQP_SQP_MU0=0.1
run MPCQP_SQP_MU0=1e-3 MPCQP_SQP_MUFLOOR=1e-4
run MPCQP_SQP_MU0=1e-4 MPCQP_SQP_MUFLOOR=1e-5 MPCQP_SQP_MUDEC=0.1
run MPCQP_SQP_MU0=1e-3 MPCQP_SQP_MUFLOOR=1e-4 MPCQP_SQP_SWITCH=1
run MPCQP_SQP_MU0=1e-2 MPCQP_SQP_MUFLOOR=1e-3 MPCQP_SQP_SWITCH=10
