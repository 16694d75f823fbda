# GPT-2 graph decode: MHA head_dim-64 attention through the small one-workgroup-per-(batch, head)
# kernel (PENROZ_DECODE_SMALL_ANY=1, PENROZ_DECODE_SMALL_ITEMS=1024) vs the default split kernel;
# batch 16 / 64, same box, 2 passes.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/smallab
for pass in 1 2; do for b in 16 64; do for arm in default small; do
  if [ $arm = small ]; then export PENROZ_DECODE_SMALL_ANY=1 PENROZ_DECODE_SMALL_ITEMS=1024; else unset PENROZ_DECODE_SMALL_ANY PENROZ_DECODE_SMALL_ITEMS; fi
  timeout -k 10 300 python -u bench/bench_decode.py --model gpt2 --batch $b > gpurun_out/smallab/o.log 2>&1 || { tail -20 gpurun_out/smallab/o.log; exit 1; }
  grep '^{' gpurun_out/smallab/o.log | cut -c1-170 | sed "s/^/pass=$pass arm=$arm /" >> gpurun_out/smallab/ab.log
done; done; done
