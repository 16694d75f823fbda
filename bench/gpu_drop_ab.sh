# dropout attention: flash tests (mask-revealing reference, variant agreement), attention bench
# at p = 0.1, HF-layout bench (dropout 0.1)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "flash" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_drop.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_drop.log; exit 1; }
tail -2 gpurun_out/pytest_drop.log
for v in 3 4; do
  timeout -k 10 180 python bench/attn_bench.py --p 0.1 --bwd-variants $v --iters 20 > gpurun_out/attn_drop$v.log 2>&1 || { tail -20 gpurun_out/attn_drop$v.log; exit 1; }
  grep '^{' gpurun_out/attn_drop$v.log
done
for v in 3 4 3; do
  timeout -k 10 300 env PENROZ_FLASH_BWD_VARIANT=$v python bench.py --model gpt2-hf --steps 10 --warmup 3 --ref-steps 0 > gpurun_out/bench_hf$v.log 2>&1 || { tail -20 gpurun_out/bench_hf$v.log; exit 1; }
  echo "gpt2-hf bwd variant $v: $(grep '^{' gpurun_out/bench_hf$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"], 2))')"
done
