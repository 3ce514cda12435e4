#!/bin/bash
# pf-kernel iteration check on the GPU box: qp/sweep/surface GPU tests, phase
# timing of qp_pf_kernel (configs 3, 5), bench configs 3 and 5.
set -e
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_qp.py tests/test_gpu_sweep.py tests/test_gpu_surfaces.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/ab_pytest.log 2>&1 || { tail -30 $O/ab_pytest.log; exit 1; }
tail -1 $O/ab_pytest.log
for c in 3 5; do timeout -k 10 120 python tools/phase_timing.py pf$c 2>/dev/null | tail -8 | sed "s/^/pf$c /"; done
for c in 3 5; do
  timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 3 --no-cpu > $O/ab_cfg$c.json 2>$O/ab_cfg$c.err
  python -c "import json; d=json.load(open('$O/ab_cfg$c.json')); print($c, d['value'], d['max_abs_u_err_vs_oracle'], d['status_hist'], d.get('kernel_us'))"
done
