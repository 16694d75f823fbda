# TunableOp solution search for the Gemma decode program's library GEMMs at 33-64 rows (Gemma-3 1B
# shapes, batch 64: the QKV / O / gate|up / down projections keep hipBLASLt there), then an A/B of
# the decode bench with the shipped table vs shipped + these results (PENROZ_TUNED_GEMM_FILE).
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/tune_gd
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=60 \
PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=20 PENROZ_TUNED_GEMMS=0 \
PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune_gd/tunableop_gdec.csv \
  timeout -k 10 600 python -u bench/bench_decode.py --model gemma3-1b --batch 64 --new 8 > gpurun_out/tune_gd/tune.log 2>&1 || { tail -20 gpurun_out/tune_gd/tune.log; exit 1; }
F=$(ls gpurun_out/tune_gd/tunableop_gdec*.csv | head -n1)
{ cat penr-oz-neural-network-v3-torch-ddp_amd/ops/tuned/tunableop_gfx950.csv; grep -v '^Validator' "$F" | grep '_64_'; } > gpurun_out/tune_gd/merged.csv
for pass in 1 2; do
  timeout -k 10 300 python -u bench/bench_decode.py --model gemma3-1b --batch 64 2>&1 | grep '^{' | sed "s/^/pass=$pass shipped /" >> gpurun_out/tune_gd/ab.log
  PENROZ_TUNED_GEMM_FILE=gpurun_out/tune_gd/merged.csv timeout -k 10 300 python -u bench/bench_decode.py --model gemma3-1b --batch 64 2>&1 | grep '^{' | sed "s/^/pass=$pass merged /" >> gpurun_out/tune_gd/ab.log
done
