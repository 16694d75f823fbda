# GQA dK/dV query-head split (D = 256 Gemma shapes): generic-D flash tests, attention bench, Gemma-3
# 1B shaped training B = 8 / 16
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gen or gqa or gemma or rope or rms" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gen.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_gen.log; exit 1; }
tail -2 gpurun_out/pytest_gen.log
for cfg in "--B 8 --T 1024 --H 4 --Hkv 1 --D 256" "--B 16 --T 1024 --H 4 --Hkv 1 --D 256" "--B 16 --T 2048 --H 16 --Hkv 8 --D 128"; do
  timeout -k 10 120 python bench/attn_bench.py $cfg --iters 10 --sdpa 2>&1 | grep '^{' || exit 1
done
for B in 8 16; do
  timeout -k 10 400 python bench.py --model gemma3-1b --batch $B --steps 5 --warmup 2 --ref-steps 0 > gpurun_out/gemma_train_b$B.log 2>&1 || { tail -30 gpurun_out/gemma_train_b$B.log; exit 1; }
  echo "gemma3-1b B=$B: $(grep '^{' gpurun_out/gemma_train_b$B.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"], 1), round(d["mfu_bf16_dense"], 3))')"
done
