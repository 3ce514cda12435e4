#!/bin/bash
# GPU box: full-size parity tests + mpc_qp tests, then config 3 / 5 bench lines.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd $ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_mpc_qp.py tests/test_gpu_workspace.py \
  -q --timeout 200 --timeout-method thread > gpurun_out/check_pf.log 2>&1
rc=$?; tail -4 gpurun_out/check_pf.log; [ $rc -eq 0 ] || exit $rc
for c in 3 5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu --steps 40 > gpurun_out/fix_cfg$c.json 2> gpurun_out/fix_cfg$c.err || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/fix_cfg$c.json'))
print('$c', d['value'], d.get('kernel_us'), d.get('max_abs_u_err_vs_oracle'), d.get('status_hist'))"
done
