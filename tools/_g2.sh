set -o pipefail
L=$PWD/model_predictive_control_amd/lib/variants/libmpcqp_pfdbg.so
MPCQP_LIB=$L timeout -k 10 120 python -u tools/tail_dump.py replay tools/cfg3_tail_inputs.npz > gpurun_out/g2_replay.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/g2_replay.log | grep -v "it=" | head -80
timeout -k 10 240 python -u tools/tail_dump.py dump gpurun_out/tail2.npz 1e-6 > gpurun_out/g2_dump.log 2>&1 || exit 2
cat gpurun_out/g2_dump.log | grep -v amdgpu.ids | head -30
for c in 3 5; do timeout -k 10 200 python bench.py --config $c --no-cpu --steps 10 --warmup 3 > gpurun_out/g2_b$c.json 2>gpurun_out/g2_b$c.err || exit 3; python -c "import json;d=json.load(open('gpurun_out/g2_b$c.json'));print('cfg$c',d['value'],d.get('kernel_us'),d.get('max_abs_u_err_vs_oracle'),d['status_hist'])"; done
