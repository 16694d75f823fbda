# Same-box A/B of env settings on the graph decode bench: MODEL (default gemma3-1b), batches 64 and 1,
# two interleaved passes: bash bench/gpu_decode_env_ab.sh "A=0" "A=1"
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for e in "$@"; do
    for b in 64 1; do
      env $e PENROZ_GRAPH_DECODE=1 timeout -k 10 240 python bench/bench_decode.py --model ${MODEL:-gemma3-1b} --batch $b \
        > gpurun_out/dec.log 2>&1 || { tail -20 gpurun_out/dec.log; exit 1; }
      echo "${MODEL:-gemma3-1b} [$e] B$b $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dec.log)"
    done
  done
done
