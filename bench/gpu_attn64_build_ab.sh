# Same-box A/B of a baseline build (build_ab) vs the working build: GPT-2 attention microbench
# (B=64, T=1024, H=12, D=64) then the headline bench, two interleaved passes each. Run via gpurun.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for e in PENROZ_EXT_DIR=build_ab PENROZ_EXT_DIR=build_ext; do
    env $e timeout -k 10 120 python bench/attn_bench.py --B 64 --T 1024 --H 12 --D 64 --iters 20 \
      > gpurun_out/attn_ab.log 2>&1 || { tail -20 gpurun_out/attn_ab.log; exit 1; }
    echo "[$e] $(grep '^{' gpurun_out/attn_ab.log | cut -c1-300)"
  done
done
for i in 1 2; do
  for e in PENROZ_EXT_DIR=build_ab PENROZ_EXT_DIR=build_ext; do
    env $e timeout -k 10 200 python bench.py --steps 20 --warmup 5 --ref-steps 0 > gpurun_out/ab.log 2>&1 \
      || { tail -20 gpurun_out/ab.log; exit 1; }
    echo "gpt2 [$e] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.log)"
  done
done
