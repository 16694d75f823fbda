# fused qkv-bias epilogue (static transpose-reduce) + stream unroll A/B: tests, kernel bench, headline
# benches alternating, serial profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_executor_gpu.py tests/test_executor_parity_gpu.py -k "flash or executor or parity or gelu or colsum" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_bias.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_bias.log; exit 1; }
tail -2 gpurun_out/pytest_bias.log
timeout -k 10 120 python -u bench/kernel_bench.py stream attn 2>&1 | grep "^{" | tee gpurun_out/stream_bench.log
for cfg in "1 4" "0 4" "1 1" "1 4" "0 4" "1 1"; do
  set -- $cfg
  timeout -k 10 300 env PENROZ_FUSED_QKV_BIAS=$1 PENROZ_STREAM_UNROLL=$2 python bench.py --steps 20 --warmup 5 --ref-steps 0 > gpurun_out/bench_ab.log 2>&1 || { tail -20 gpurun_out/bench_ab.log; exit 1; }
  echo "fused_bias=$1 unroll=$2: $(tail -1 gpurun_out/bench_ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"], 2))')"
done
PENROZ_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_serial -o run -- python3 bench.py --steps 5 --warmup 3 --ref-steps 0 > gpurun_out/prof_serial_bench.log 2>&1 || exit $?
DB=$(find gpurun_out/prof_serial -name 'run_results.db' | head -n1)
python3 bench/prof_summary.py $DB --steps 8 > gpurun_out/prof_serial_summary.txt
head -n 16 gpurun_out/prof_serial_summary.txt | cut -c1-130
