for c in nlp loop; do
  timeout -k 10 500 python3 bench.py --config $c > gpurun_out/w_$c.json 2> gpurun_out/w_$c.err || exit 1
done
