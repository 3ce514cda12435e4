rm -f gpurun_out/mp.log
for m in 1e-6 1e-5 1e-4; do
  MPCQP_SQP_MU_POLISH=$m timeout -k 10 200 python -u tools/sqp_knobs.py --tag mp$m 2>&1 | grep KNOB >> gpurun_out/mp.log || exit 1
  MPCQP_SQP_MU_POLISH=$m timeout -k 10 300 python3 bench.py --config loop --no-cpu > gpurun_out/mp_loop_$m.json 2>/dev/null || exit 1
  MPCQP_SQP_MU_POLISH=$m timeout -k 10 200 python -u tools/sqp_minima.py gpurun_out/min_mp$m.npz > /dev/null 2>&1 || exit 1
done
