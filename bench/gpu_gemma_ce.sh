# fused cross-entropy on the generic engine: CE + model/runtime GPU tests, Gemma-3 1B shaped
# training B = 8 / 16, HF-layout generic engine bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_runtime_gpu.py -k "cross or ce_ or runtime or generic or gemma or rms or adam" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ce.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_ce.log; exit 1; }
tail -2 gpurun_out/pytest_ce.log
for B in 8 16; do
  timeout -k 10 400 python bench.py --model gemma3-1b --batch $B --steps 5 --warmup 2 --ref-steps 0 > gpurun_out/gemma_train_b$B.log 2>&1 || { tail -30 gpurun_out/gemma_train_b$B.log; exit 1; }
  echo "gemma3-1b B=$B: $(grep '^{' gpurun_out/gemma_train_b$B.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"], 1), round(d["mfu_bf16_dense"], 3), round(d["final_loss"], 3))')"
done
timeout -k 10 400 python bench.py --model gpt2-hf --engine generic --steps 10 --warmup 3 --ref-steps 0 > gpurun_out/hf_generic.log 2>&1 || { tail -30 gpurun_out/hf_generic.log; exit 1; }
echo "gpt2-hf generic: $(grep '^{' gpurun_out/hf_generic.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"], 1))')"
