set -o pipefail
mkdir -p gpurun_out
for e in "PENROZ_GRAPH_DECODE=0" "PENROZ_GRAPH_DECODE=1"; do
  env $e timeout -k 10 200 python bench/bench_decode.py > gpurun_out/dec.log 2>&1 || { tail -20 gpurun_out/dec.log; exit 1; }
  echo "$e $(grep metric gpurun_out/dec.log)"
  env $e timeout -k 10 200 python bench/bench_decode.py --turbo > gpurun_out/dec.log 2>&1 || { tail -20 gpurun_out/dec.log; exit 1; }
  echo "$e $(grep metric gpurun_out/dec.log)"
done
env PENROZ_GRAPH_DECODE=1 timeout -k 10 200 python bench/bench_decode.py --batch 1 > gpurun_out/dec.log 2>&1 && echo "B1 $(grep metric gpurun_out/dec.log)"
