set -o pipefail
L=$PWD/model_predictive_control_amd/lib/variants/libmpcqp_pfdbg.so
MPCQP_LIB=$L timeout -k 10 120 python -u tools/tail_dump.py replay tools/cfg3_tail_inputs.npz > gpurun_out/g2_replay.log 2>&1 || { tail -20 gpurun_out/g2_replay.log; exit 1; }
grep -v amdgpu.ids gpurun_out/g2_replay.log | grep -v "it=" | head -60
timeout -k 10 120 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gpu_condense.py > gpurun_out/g2_condense.log 2>&1 || { tail -30 gpurun_out/g2_condense.log; exit 5; }
tail -2 gpurun_out/g2_condense.log
timeout -k 10 240 python -u tools/tail_dump.py dump gpurun_out/tail2.npz 1e-6 > gpurun_out/g2_dump.log 2>&1 || { tail -20 gpurun_out/g2_dump.log; exit 2; }
grep -v amdgpu.ids gpurun_out/g2_dump.log | head -30
for c in 3 5; do timeout -k 10 200 python bench.py --config $c --no-cpu --steps 10 --warmup 3 > gpurun_out/g2_b$c.json 2>gpurun_out/g2_b$c.err || { tail gpurun_out/g2_b$c.err; exit 3; }; python -c "import json;d=json.load(open('gpurun_out/g2_b$c.json'));print('cfg$c',d['value'],d.get('kernel_us'),d.get('max_abs_u_err_vs_oracle'),d['status_hist'])"; done
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_mpc_qp.py tests/test_gpu_nlp.py tests/test_gpu_multi.py > gpurun_out/g2_pytest.log 2>&1 || { tail -40 gpurun_out/g2_pytest.log; exit 4; }
tail -3 gpurun_out/g2_pytest.log
timeout -k 10 120 python -u tools/wave_clock.py --out gpurun_out/wave_clock_cfg2.json > gpurun_out/g2_wclk.log 2>&1 || { tail -20 gpurun_out/g2_wclk.log; exit 6; }
grep -v amdgpu.ids gpurun_out/g2_wclk.log | head -40
