# Record PyTorch TunableOp (hipBLASLt + rocBLAS solution search) results for every library GEMM the
# fused executor issues at the headline shapes (GPT-2 124M, B=64, T=1024; forward addmm, dgrad mm on
# the transposed weight copies, lm_head into the padded logits rows), plus the HF-import layout
# (V = 50257). Results are written at process exit; the repo ships them in
# penr-oz-neural-network-v3-torch-ddp_amd/ops/tuned/ and ops/gemm.py loads them read-only.
set -o pipefail
mkdir -p gpurun_out/tune
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=0
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=60 PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=20
export PENROZ_TUNED_GEMMS=0
PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune/tunableop_124m.csv timeout -k 10 900 python -u bench.py --steps 1 --warmup 1 --ref-steps 0 > gpurun_out/tune/tune_124m.log 2>&1 && tail -1 gpurun_out/tune/tune_124m.log | cut -c1-200 && \
PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune/tunableop_hf.csv timeout -k 10 900 python -u bench.py --model gpt2-hf --steps 1 --warmup 1 --ref-steps 0 > gpurun_out/tune/tune_hf.log 2>&1 && tail -1 gpurun_out/tune/tune_hf.log | cut -c1-200
ls -la gpurun_out/tune/
