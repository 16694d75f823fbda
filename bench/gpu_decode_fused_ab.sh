# Fused decode kernel (add+LN+GEMM(+GELU)): numerics tests, decode-program tests, then the decode
# bench at batch 64 and batch 1 with PENROZ_DECODE_FUSED=0/1; plus the executor regression tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_decode_gpu.py tests/test_distributed_gpu.py tests/test_executor_gpu.py tests/test_executor_parity_gpu.py -m gpu -q --timeout 200 --timeout-method thread -k "decode_ln_linear or graph_decode or decode_program or gemma or executor or distributed or seeded or greedy or stop_token or sampling or rope" > gpurun_out/dfa_tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/dfa_tests.log | head -20; tail -5 gpurun_out/dfa_tests.log; exit 1; }
tail -2 gpurun_out/dfa_tests.log
for b in 64 1; do for f in 0 1; do
  PENROZ_DECODE_FUSED=$f timeout -k 10 300 python -u bench/bench_decode.py --batch $b --new 128 > gpurun_out/dfa_b${b}_f$f.log 2>&1 || { tail -5 gpurun_out/dfa_b${b}_f$f.log; exit 1; }
  echo "batch=$b fused=$f $(tail -1 gpurun_out/dfa_b${b}_f$f.log | cut -c1-160)"
done; done
