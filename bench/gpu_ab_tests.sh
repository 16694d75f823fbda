set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_executor_gpu.py tests/test_distributed_gpu.py tests/test_runtime_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/exec_tests.log 2>&1 || { tail -30 gpurun_out/exec_tests.log; exit 1; }
tail -2 gpurun_out/exec_tests.log
bash bench/gpu_ab.sh "$@"
