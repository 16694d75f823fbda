# Same-box A/B of TunableOp table variants on the Gemma-3 1B B=8 bench (PENROZ_TUNED_GEMM_FILE):
# the current table, then the table without one Gemma entry at a time. Run via gpurun.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${VARIANTS:-cur gdrop0 gdrop1 gdrop2 gdrop3 gdrop4 gdrop5 gdrop6 gdrop7 gdrop8 gdrop9 gdrop10 gdrop11 cur}; do
  PENROZ_TUNED_GEMM_FILE=bench/tuned_ab/$v.csv timeout -k 10 300 python bench.py --model gemma3-1b --batch 8 --steps 10 \
    --warmup 3 --ref-steps 0 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
  echo "gemma3-1b B8 [$v] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.log)"
done
