# Causal work-list split of the head_dim >= 128 attention kernels (flash_attn_gen.hip): GPU tests,
# attention microbench at the Gemma-3 1B in-step shape with PENROZ_ATTN_KV_SPLIT 0 / 1, then the
# Gemma-3 1B training bench (B = 8, 16) with 0 / 1 on the same box. Run via gpurun.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/split_r4.log
: > $L
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "flash_gen" >> $L 2>&1 || { tail -30 $L; exit 1; }
tail -2 $L
for B in 8 16; do
  for m in 0 1; do
    echo "== attn B=$B split=$m" >> $L
    PENROZ_ATTN_KV_SPLIT=$m timeout -k 10 120 python bench/attn_bench.py --B $B --T 1024 --H 4 --Hkv 1 --D 256 \
      --iters 30 >> $L 2>&1 || { tail -20 $L; exit 1; }
  done
done
for B in 8 16; do
  for m in 0 1 0 1; do
    echo "== gemma B=$B split=$m" >> $L
    PENROZ_ATTN_KV_SPLIT=$m timeout -k 10 300 python bench.py --model gemma3-1b --batch $B --steps 10 --warmup 3 \
      --ref-steps 0 > gpurun_out/split_gemma.log 2>&1 || { tail -20 gpurun_out/split_gemma.log; exit 1; }
    grep '^{' gpurun_out/split_gemma.log | cut -c1-260 >> $L
  done
done
grep -E "^==|_us|value" $L | cut -c1-260
