# A/B of the headline bench under two env settings: bash bench/gpu_ab.sh "VAR=a" "VAR=b"
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for e in "$@"; do
    env $e timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    echo "$e $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.log)"
  done
done
