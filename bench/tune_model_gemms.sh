# TunableOp solution search (hipBLASLt + rocBLAS) for the library GEMM shapes one bench.py model
# issues that the shipped table lacks, then a same-box A/B of that model's bench with the shipped
# table vs shipped + new results (PENROZ_TUNED_GEMM_FILE). The merged table lands in
# gpurun_out/tune_<model>/merged.csv; ship it as penr-oz-neural-network-v3-torch-ddp_amd/ops/tuned/
# tunableop_gfx950.csv when the A/B says so.
#
#   bash bench/tune_model_gemms.sh gemma3-1b 8 16      (model, then the batch sizes to cover)
#   bash bench/tune_model_gemms.sh gpt2-xl 64
set -o pipefail
export TMPDIR=/tmp
MODEL=$1; shift
OUT=gpurun_out/tune_$MODEL
mkdir -p $OUT
SHIPPED=penr-oz-neural-network-v3-torch-ddp_amd/ops/tuned/tunableop_gfx950.csv
cp $SHIPPED $OUT/merged.csv
for B in "$@"; do
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=60 \
  PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=10 PENROZ_TUNED_GEMMS=0 PYTORCH_TUNABLEOP_FILENAME=$OUT/tune_b$B.csv \
    timeout -k 10 900 python -u bench.py --model $MODEL --batch $B --steps 1 --warmup 1 --ref-steps 0 \
    > $OUT/tune_b$B.log 2>&1 || { tail -20 $OUT/tune_b$B.log; exit 1; }
  F=$(ls $OUT/tune_b$B*.csv | head -n1)
  grep -v '^Validator' "$F" >> $OUT/merged.csv
done
for B in "$@"; do
  for f in $SHIPPED $OUT/merged.csv; do
    PENROZ_TUNED_GEMM_FILE=$f timeout -k 10 400 python -u bench.py --model $MODEL --batch $B --steps 5 --warmup 2 \
      --ref-steps 0 > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
    echo "B=$B $(basename $f): $(grep '^{' $OUT/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"], 2), round(d["mfu_bf16_dense"], 4))')"
  done
done
