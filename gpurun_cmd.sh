timeout -k 10 400 bash tools/traffic.sh 5 > gpurun_out/t5.log 2>&1; echo "traffic rc=$?"; tail -1 gpurun_out/t5.log | cut -c1-800
timeout -k 10 300 bash tools/mfma_counters.sh 5 r05 > /dev/null 2>&1; echo "mfma5 rc=$?"; cat gpurun_out/r05_cfg5/summary.txt
timeout -k 10 300 bash tools/mfma_counters.sh 3 r05 > /dev/null 2>&1; echo "mfma3 rc=$?"; cat gpurun_out/r05_cfg3/summary.txt
