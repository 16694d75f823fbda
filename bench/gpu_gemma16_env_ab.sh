# Same-box A/B of env settings on Gemma-3 1B (GB = batch, default 16), two interleaved passes: bash bench/gpu_gemma16_env_ab.sh "A=1" "A=2"
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for e in "$@"; do
    env $e timeout -k 10 300 python bench.py --model gemma3-1b --batch ${GB:-16} --steps 8 --warmup 3 --ref-steps 0 \
      > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    echo "gemma3-1b B${GB:-16} [$e] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.log)"
  done
done
