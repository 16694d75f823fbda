# Same-box A/B of a baseline build (build_ab) vs the working build: headline bench, then GPT-2
# graph decode at B = 1 / 64, two interleaved passes each.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for e in PENROZ_EXT_DIR=build_ab PENROZ_EXT_DIR=build_ext; do
    env $e timeout -k 10 200 python bench.py --steps 20 --warmup 5 --ref-steps 0 > gpurun_out/ab.log 2>&1 \
      || { tail -20 gpurun_out/ab.log; exit 1; }
    echo "gpt2 [$e] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.log)"
  done
done
for i in 1 2; do
 for e in PENROZ_EXT_DIR=build_ab PENROZ_EXT_DIR=build_ext; do
  for b in 1 64; do
    env $e PENROZ_GRAPH_DECODE=1 timeout -k 10 240 python bench/bench_decode.py --model gpt2 --batch $b > gpurun_out/dec.log 2>&1 \
      || { tail -20 gpurun_out/dec.log; exit 1; }
    echo "decode [$e] B$b $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dec.log)"
  done
 done
done
