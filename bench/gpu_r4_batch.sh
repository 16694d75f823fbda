# Round-4 GPU batch: deferred-epilogue GEMM tests + bench, then the Gemma-4 / head_dim-512 tests.
# A step that ends in anything but pass / test failures (timeout, abort, fault) ends the script.
set -o pipefail
mkdir -p gpurun_out
ok_or_stop() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ] || { echo "stopping: exit $1"; exit "$1"; }; }
timeout -k 10 300 python -u -m pytest tests/test_gemm_epi_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gemm_epi.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gemm_epi.log; ok_or_stop $rc
if [ $rc -eq 0 ]; then
  timeout -k 10 300 python bench/gemm_epi_bench.py > gpurun_out/gemm_epi_bench.log 2>&1; rc=$?
  tail -8 gpurun_out/gemm_epi_bench.log; ok_or_stop $rc
  bash bench/gpu.sh ab PENROZ_EPI_GEMM=0 PENROZ_EPI_GEMM=1 > gpurun_out/ab_epi_gemm.log 2>&1; rc=$?
  cat gpurun_out/ab_epi_gemm.log; ok_or_stop $rc
fi
timeout -k 10 700 python -u -m pytest tests/test_gemma_executor_gpu.py tests/test_kernels_gpu.py \
  -k "gen or padded or gemma or match or combine" -v --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_r4_gemma4.log 2>&1; rc=$?
grep -E "FAILED|ERROR" gpurun_out/pytest_r4_gemma4.log | head -20; tail -3 gpurun_out/pytest_r4_gemma4.log
exit $rc
