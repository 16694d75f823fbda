# Same-box A/B of TunableOp table variants (bench/tuned_ab/*.csv through PENROZ_TUNED_GEMM_FILE)
# on the headline bench, two interleaved passes. Run via gpurun.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for v in ${VARIANTS:-full no_gpt2 no_bias no_lmhead no_mid}; do
    PENROZ_TUNED_GEMM_FILE=bench/tuned_ab/$v.csv timeout -k 10 200 python bench.py --steps 20 --warmup 5 --ref-steps 0 \
      > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    echo "gpt2 [$v] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.log)"
  done
done
