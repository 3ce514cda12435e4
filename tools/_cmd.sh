for wk in 1e-3 1e-2 1e-1; do
  MPCQP_SQP_WARM_KKT=$wk timeout -k 10 200 python -u tools/sqp_minima.py gpurun_out/min_$wk.npz > gpurun_out/min_$wk.log 2>&1 || exit 1
done
