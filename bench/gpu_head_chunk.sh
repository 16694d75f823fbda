# lm_head/CE token-chunk sweep: executor tests, then the headline bench per PENROZ_HEAD_CHUNK.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_executor_gpu.py tests/test_executor_parity_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/exec_tests.log 2>&1; rc=$?
tail -3 gpurun_out/exec_tests.log
[ $rc -eq 0 ] || exit $rc
for c in ${CHUNKS:-0 16384 8192 4096 2048}; do
  PENROZ_HEAD_CHUNK=$c timeout -k 10 200 python bench.py --steps 20 --warmup 5 --ref-steps 0 > gpurun_out/bench_chunk_$c.log 2>&1 || exit $?
  echo "chunk=$c $(tail -1 gpurun_out/bench_chunk_$c.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"],2))')"
done
