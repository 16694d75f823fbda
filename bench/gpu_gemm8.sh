set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemm8_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/g8_test.log 2>&1; rc=$?
tail -15 gpurun_out/g8_test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench/gemm8_bench.py > gpurun_out/g8_bench.log 2>&1; rc=$?
cat gpurun_out/g8_bench.log
exit $rc
