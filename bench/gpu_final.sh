# full GPU suite + smoke + headline bench, then the Gemma-3 1B shaped training bench
set -o pipefail
bash bench/gpu_check.sh || exit 1
for B in 8 16; do
  timeout -k 10 400 python bench.py --model gemma3-1b --batch $B --steps 5 --warmup 2 --ref-steps 0 > gpurun_out/gemma_train_b$B.log 2>&1 || { tail -30 gpurun_out/gemma_train_b$B.log; exit 1; }
  echo "gemma3-1b B=$B: $(grep '^{' gpurun_out/gemma_train_b$B.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"], 1), round(d["mfu_bf16_dense"], 3))')"
done
