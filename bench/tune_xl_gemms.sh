# GPT-2 XL (1.56 B) on one MI355X at B = 64 (the 288 GB sizing point): kernel profile, TunableOp
# search over its library GEMM shapes (C = 1600, F = 6400: not in the shipped table), and an A/B of
# the XL bench with shipped vs shipped + XL results (PENROZ_TUNED_GEMM_FILE).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/tune_xl
XLB=${XLB:-64}
timeout -k 10 400 python -u bench.py --model gpt2-xl --batch $XLB --steps 4 --warmup 2 --ref-steps 0 > gpurun_out/tune_xl/base.log 2>&1 || { tail -20 gpurun_out/tune_xl/base.log; exit 1; }
tail -1 gpurun_out/tune_xl/base.log | cut -c1-330
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/tune_xl/prof -o run -- python3 bench.py --model gpt2-xl --batch $XLB --steps 2 --warmup 1 --ref-steps 0 > gpurun_out/tune_xl/prof_bench.log 2>&1 || { tail -20 gpurun_out/tune_xl/prof_bench.log; exit 1; }
DB=$(find gpurun_out/tune_xl/prof -name 'run_results.db' | head -n1)
python3 bench/prof_summary.py $DB --steps 3 > gpurun_out/tune_xl/prof_summary.txt && head -n 30 gpurun_out/tune_xl/prof_summary.txt
rm -rf gpurun_out/tune_xl/prof
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=60 \
PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=10 PENROZ_TUNED_GEMMS=0 \
PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune_xl/tunableop_xl.csv \
  timeout -k 10 900 python -u bench.py --model gpt2-xl --batch $XLB --steps 1 --warmup 1 --ref-steps 0 > gpurun_out/tune_xl/tune.log 2>&1 || { tail -20 gpurun_out/tune_xl/tune.log; exit 1; }
F=$(ls gpurun_out/tune_xl/tunableop_xl*.csv | head -n1)
{ cat penr-oz-neural-network-v3-torch-ddp_amd/ops/tuned/tunableop_gfx950.csv; grep -v '^Validator' "$F"; } > gpurun_out/tune_xl/merged.csv
PENROZ_TUNED_GEMM_FILE=gpurun_out/tune_xl/merged.csv timeout -k 10 400 python -u bench.py --model gpt2-xl --batch $XLB --steps 4 --warmup 2 --ref-steps 0 > gpurun_out/tune_xl/tuned.log 2>&1 || { tail -20 gpurun_out/tune_xl/tuned.log; exit 1; }
tail -1 gpurun_out/tune_xl/tuned.log | cut -c1-330
