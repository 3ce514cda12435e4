set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_mpc_qp.py > gpurun_out/g3_mpcqp.log 2>&1; rc=$?
tail -30 gpurun_out/g3_mpcqp.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 240 python -u tools/tail_dump.py dump gpurun_out/tail3.npz 1e-6 > gpurun_out/g3_dump.log 2>&1 || { tail -20 gpurun_out/g3_dump.log; exit 2; }
grep -v amdgpu.ids gpurun_out/g3_dump.log | head -20
for v in "X=1" "MPCQP_MPC_ZF=0"; do env $v timeout -k 10 200 python bench.py --config 3 --no-cpu --steps 10 --warmup 3 > gpurun_out/g3_b3.json 2>gpurun_out/g3_b3.err || { tail gpurun_out/g3_b3.err; exit 3; }; python -c "import json;d=json.load(open('gpurun_out/g3_b3.json'));print('cfg3 [$v]',d['value'],d.get('kernel_us'),d.get('max_abs_u_err_vs_oracle'),d['status_hist'],d.get('iters_mean'))"; done
timeout -k 10 200 python bench.py --config 5 --no-cpu --steps 10 --warmup 3 > gpurun_out/g3_b5.json 2>gpurun_out/g3_b5.err || { tail gpurun_out/g3_b5.err; exit 3; }; python -c "import json;d=json.load(open('gpurun_out/g3_b5.json'));print('cfg5',d['value'],d.get('kernel_us'),d.get('max_abs_u_err_vs_oracle'),d['status_hist'])"
