set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u bench/gemm8_probe.py 2>&1 | tee gpurun_out/g8_probe.log
