set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/skab
for pass in 1 2; do for r in 16 64; do
  PENROZ_SKINNY_MAX_ROWS=$r timeout -k 10 300 python -u bench/bench_decode.py --model gemma3-1b --batch 64 > gpurun_out/skab/o.log 2>&1 || { tail -20 gpurun_out/skab/o.log; exit 1; }
  grep '^{' gpurun_out/skab/o.log | cut -c1-160 | sed "s/^/pass=$pass skinny_max=$r /" >> gpurun_out/skab/ab.log
done; done
