# HF-import GPT-2 layout (V=50257, dropout 0.1, tanh GELU, bf16 params): fused vs generic engine.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --model gpt2-hf --steps 10 --warmup 3 --ref-steps 0 > gpurun_out/bench_hf_fused.log 2>&1 && tail -1 gpurun_out/bench_hf_fused.log && \
timeout -k 10 300 python bench.py --model gpt2-hf --engine generic --batch 16 --steps 5 --warmup 2 --ref-steps 0 > gpurun_out/bench_hf_generic.log 2>&1 && tail -1 gpurun_out/bench_hf_generic.log
