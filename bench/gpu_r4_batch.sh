# Round-4 GPU batch: deferred-epilogue GEMM tests + bench + the headline A/B of the fused fc+GELU,
# then the 2-rank Gemma-executor rehearsal. A step that ends in anything but pass / test failures
# (timeout, abort, fault) ends the script.
set -o pipefail
mkdir -p gpurun_out
ok_or_stop() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ] || { echo "stopping: exit $1"; exit "$1"; }; }
timeout -k 10 300 python -u -m pytest tests/test_gemm_epi_gpu.py -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gemm_epi.log 2>&1; rc=$?
grep -E "FAILED|ERROR" gpurun_out/pytest_gemm_epi.log | head -20; tail -2 gpurun_out/pytest_gemm_epi.log; ok_or_stop $rc
timeout -k 10 300 python bench/gemm_epi_bench.py > gpurun_out/gemm_epi_bench.log 2>&1; rc=$?
cat gpurun_out/gemm_epi_bench.log | grep '^{'; ok_or_stop $rc
if [ "${EPI_AB:-1}" = 1 ]; then
  bash bench/gpu.sh ab PENROZ_EPI_GEMM=0 PENROZ_EPI_GEMM=1 > gpurun_out/ab_epi_gemm.log 2>&1; rc=$?
  cat gpurun_out/ab_epi_gemm.log; ok_or_stop $rc
fi
timeout -k 10 400 python -u -m pytest tests/test_distributed_gemma_gpu.py -v --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_ddp_gemma.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_ddp_gemma.log | head; tail -2 gpurun_out/pytest_ddp_gemma.log
exit $rc
