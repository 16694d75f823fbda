# Decode A/B: native skinny GEMM vs hipBLASLt inside the graph-replayed decode programs.
set -o pipefail
mkdir -p gpurun_out
for m in gpt2 gemma3-1b; do
  for b in 1 8; do
    for e in "PENROZ_SKINNY_GEMM=1" "PENROZ_SKINNY_GEMM=0"; do
      env $e timeout -k 10 240 python bench/bench_decode.py --model $m --batch $b > gpurun_out/dec.log 2>&1 \
        || { tail -20 gpurun_out/dec.log; exit 1; }
      echo "$m B$b $e $(grep metric gpurun_out/dec.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms/step", round(d["value"]), "tok/s")')"
    done
  done
done
