# TunableOp solution search for the decode-shaped library GEMMs (GPT-2 124M /generate at batch 64:
# M = 64 rows per step; prompt prefill M = 64 x 64), then an A/B of the decode bench with the
# shipped file vs shipped + decode results (PENROZ_TUNED_GEMM_FILE).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/tune
timeout -k 10 300 python -u bench/bench_decode.py --batch 64 --new 128 > gpurun_out/tune/dec_base.log 2>&1 && tail -1 gpurun_out/tune/dec_base.log
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=60 \
PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=20 PENROZ_TUNED_GEMMS=0 \
PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune/tunableop_decode.csv \
  timeout -k 10 600 python -u bench/bench_decode.py --batch 64 --new 8 > gpurun_out/tune/dec_tune.log 2>&1 || { tail -20 gpurun_out/tune/dec_tune.log; exit 1; }
ls gpurun_out/tune/
F=$(ls gpurun_out/tune/tunableop_decode*.csv | head -n1)
{ cat penr-oz-neural-network-v3-torch-ddp_amd/ops/tuned/tunableop_gfx950.csv; grep -v '^Validator' "$F"; } > gpurun_out/tune/merged.csv
PENROZ_TUNED_GEMM_FILE=gpurun_out/tune/merged.csv timeout -k 10 300 python -u bench/bench_decode.py --batch 64 --new 128 > gpurun_out/tune/dec_tuned.log 2>&1 && tail -1 gpurun_out/tune/dec_tuned.log
