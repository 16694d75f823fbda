# Same-box A/B of the Gemma combine kernels' non-temporal rows (PENROZ_GM_NT) and grid cap
# (PENROZ_GM_GRID), Gemma-3 1B B=8, two interleaved passes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for e in "PENROZ_GM_NT=0 PENROZ_GM_GRID=1024" "PENROZ_GM_NT=1 PENROZ_GM_GRID=1024" "PENROZ_GM_NT=1 PENROZ_GM_GRID=2048" "PENROZ_GM_NT=0 PENROZ_GM_GRID=2048"; do
    env $e timeout -k 10 300 python bench.py --model gemma3-1b --batch 8 --steps 10 --warmup 3 --ref-steps 0 \
      > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    echo "gemma3-1b B8 [$e] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.log)"
  done
done
