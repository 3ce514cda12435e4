rm -f gpurun_out/dpp.log
for c in 2 5 3 4; do
  echo "== cfg $c" >> gpurun_out/dpp.log
  timeout -k 10 600 bash tools/ab_run.sh $c dppold -- --steps 200 >> gpurun_out/dpp.log 2>&1 || exit 1
done
for v in base dppold; do
  if [ $v = base ]; then L=model_predictive_control_amd/lib/libmpcqp.so; else L=model_predictive_control_amd/lib/variants/libmpcqp_$v.so; fi
  MPCQP_LIB=$L timeout -k 10 200 python -u tools/sqp_knobs.py --tag $v 2>&1 | grep KNOB >> gpurun_out/dpp.log || exit 1
done
