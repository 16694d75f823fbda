# Gemma-path decode on one MI355X: decode-attention D=256, fused norm / gated kernels and
# graph-decode tests, then the Gemma-3 1B shaped decode bench (eager, module graph, program graph).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "decode or rms_residual or gated_act_packed" tests/test_graph_decode_gpu.py > gpurun_out/gemma_tests.log 2>&1 \
  || { tail -40 gpurun_out/gemma_tests.log; exit 1; }
tail -3 gpurun_out/gemma_tests.log
for e in "PENROZ_GRAPH_DECODE=0" "PENROZ_DECODE_PROGRAM=0" "PENROZ_DECODE_PROGRAM=1"; do
  for b in 64 1; do
    env $e timeout -k 10 240 python bench/bench_decode.py --model gemma3-1b --batch $b > gpurun_out/dec.log 2>&1 \
      || { tail -20 gpurun_out/dec.log; exit 1; }
    echo "$e B$b $(grep metric gpurun_out/dec.log)"
  done
done
