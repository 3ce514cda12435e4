set -e
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_poly.py tests/test_gpu_box.py tests/test_gpu_surfaces.py tests/test_gpu_mpc_qp.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/c4_pytest.log 2>&1 || { tail -30 $O/c4_pytest.log; exit 1; }
tail -1 $O/c4_pytest.log
timeout -k 10 200 python bench.py --config 4 --steps 20 --warmup 3 --no-cpu > $O/c4.json 2>$O/c4.err
python -c "import json; d=json.load(open('$O/c4.json')); print(d['value'], d['max_abs_u_err_vs_oracle'], d['status_hist'], d.get('kernel_us'), d.get('iters_mean'))"
timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu > $O/c2.json 2>$O/c2.err
python -c "import json; d=json.load(open('$O/c2.json')); print(d['value'], d['max_abs_u_err_vs_oracle'], d.get('kernel_us'))"
