# RMSNorm backward rewrite: RMSNorm / generic / Gemma GPU tests, Gemma-3 1B shaped training
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_runtime_gpu.py tests/test_graph_decode_gpu.py -k "rms or gemma or generic or runtime" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_rms.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_rms.log; exit 1; }
tail -2 gpurun_out/pytest_rms.log
for B in 8 16; do
  timeout -k 10 400 python bench.py --model gemma3-1b --batch $B --steps 5 --warmup 2 --ref-steps 0 > gpurun_out/gemma_train_b$B.log 2>&1 || { tail -30 gpurun_out/gemma_train_b$B.log; exit 1; }
  echo "gemma3-1b B=$B: $(grep '^{' gpurun_out/gemma_train_b$B.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"], 1), round(d["mfu_bf16_dense"], 3))')"
done
