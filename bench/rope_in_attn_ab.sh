# RoPE applied inside the decode attention kernel (opt-in, PENROZ_DECODE_ROPE_IN_ATTN=1) vs the separate RoPE pass
# (the default): tests, then Gemma-3 1B graph decode at batch 32 / 64, same box.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/ropeab
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_decode_gpu.py -k "decode or gemma or rope" -x -q --timeout 120 --timeout-method thread > gpurun_out/ropeab/test.log 2>&1 || { tail -40 gpurun_out/ropeab/test.log; exit 1; }
tail -1 gpurun_out/ropeab/test.log
for pass in 1 2; do for b in 32 64; do for p in 0 1; do
  PENROZ_DECODE_ROPE_IN_ATTN=$p timeout -k 10 300 python -u bench/bench_decode.py --model gemma3-1b --batch $b > gpurun_out/ropeab/o.log 2>&1 || { tail -20 gpurun_out/ropeab/o.log; exit 1; }
  grep '^{' gpurun_out/ropeab/o.log | cut -c1-170 | sed "s/^/pass=$pass rope_in_attn=$p /" >> gpurun_out/ropeab/ab.log
done; done; done
