# Re-measure the secondary configs after the round-4 streaming / attention-balance changes:
# GPT-2 XL B=64, the HF GPT-2 layout, Gemma-3 1B B=8 / 16. Run via gpurun.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/configs_r4.log
: > $L
for m in gpt2-xl gpt2-hf; do
  timeout -k 10 400 python bench.py --model $m --steps 10 --warmup 3 --ref-steps 0 > gpurun_out/cfg.log 2>&1 \
    || { tail -20 gpurun_out/cfg.log; exit 1; }
  grep '^{' gpurun_out/cfg.log >> $L
done
for B in 8 16; do
  timeout -k 10 400 python bench.py --model gemma3-1b --batch $B --steps 10 --warmup 3 --ref-steps 0 > gpurun_out/cfg.log 2>&1 \
    || { tail -20 gpurun_out/cfg.log; exit 1; }
  grep '^{' gpurun_out/cfg.log >> $L
done
cut -c1-330 $L
