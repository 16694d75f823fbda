# Gemma decode at 17-64 rows: decode_gemm (default) vs hipBLASLt (PENROZ_DECODE_GEMM=0), two passes
set -e
export PYTHONUNBUFFERED=1
o=gpurun_out/decode_gemm_ab.log; : > $o
for pass in 1 2; do for arm in 1 0; do for b in 64 32 17; do
  echo "pass=$pass DECODE_GEMM=$arm batch=$b" >> $o
  PENROZ_DECODE_GEMM=$arm timeout -k 10 200 python bench/bench_decode.py --model gemma3-1b --batch $b 2>&1 | grep '^{' >> $o
done; done; done
