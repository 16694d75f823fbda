# dropout attention backward: dK/dV variant 2 (default dropout path) vs the unrolled ring (probe
# variant 5): tests, attention bench at p = 0.1, HF-layout bench (dropout 0.1) per variant
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "flash" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_drop.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_drop.log; exit 1; }
tail -2 gpurun_out/pytest_drop.log
timeout -k 10 180 python bench/attn_bench.py --which bwd --p 0.1 --bwd-variants 3,5,3,5 --iters 20 > gpurun_out/attn_drop.log 2>&1 || { tail -20 gpurun_out/attn_drop.log; exit 1; }
grep '^{' gpurun_out/attn_drop.log
for v in 3 5 3 5; do
  timeout -k 10 300 env PENROZ_FLASH_BWD_VARIANT=$v python bench.py --model gpt2-hf --steps 10 --warmup 3 --ref-steps 0 > gpurun_out/bench_hf$v.log 2>&1 || { tail -20 gpurun_out/bench_hf$v.log; exit 1; }
  echo "gpt2-hf bwd variant $v: $(grep '^{' gpurun_out/bench_hf$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"], 2))')"
done
