# Decode at long contexts (the unsplit small kernel / the 1024-key split rule were only
# measured at prompt 64): default rules vs PENROZ_DECODE_MERGE=0 (no in-launch merge: the combine
# launch and the 1024-key split rule), two passes. Writes gpurun_out/longctx.log.
set -e
export PYTHONUNBUFFERED=1
o=gpurun_out/longctx.log; : > $o
for pass in 1 2; do
for cfg in "--model gpt2 --batch 1 --prompt 64 --new 128" "--model gpt2 --batch 1 --prompt 832 --new 128" \
           "--model gpt2 --batch 64 --prompt 64 --new 128" "--model gemma3-1b --batch 1 --prompt 64 --new 128" \
           "--model gemma3-1b --batch 1 --prompt 3968 --new 128 --block 4096" \
           "--model gemma3-1b --batch 1 --prompt 16256 --new 128 --block 16384"; do
for arm in merge nomerge; do
  if [ $arm = merge ]; then unset PENROZ_DECODE_MERGE; else export PENROZ_DECODE_MERGE=0; fi
  echo "pass=$pass arm=$arm cfg=$cfg" >> $o
  timeout -k 10 200 python bench/bench_decode.py $cfg 2>&1 | grep '^{' >> $o
done; done; done
