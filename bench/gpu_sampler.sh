# sampler tests + Gemma-3 1B shaped decode bench and profile (two-stage sampler for V = 262k)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "sampl" tests/test_graph_decode_gpu.py > gpurun_out/sampler_tests.log 2>&1 \
  || { tail -40 gpurun_out/sampler_tests.log; exit 1; }
tail -3 gpurun_out/sampler_tests.log
for b in 64 1; do
  timeout -k 10 240 python bench/bench_decode.py --model gemma3-1b --batch $b > gpurun_out/dec.log 2>&1 \
    || { tail -20 gpurun_out/dec.log; exit 1; }
  echo "B$b $(grep metric gpurun_out/dec.log)"
done
bash bench/gpu_prof_decode_gemma.sh
