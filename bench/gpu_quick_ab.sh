# Quick A/B for memory-bound kernel changes: their GPU tests, kernel micro-benchmarks (new vs
# PENROZ_* legacy switch), then the headline bench. Args: pytest -k expression, kernel_bench
# sections, legacy env assignment (e.g. PENROZ_CE_KERNEL=1024).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
K=${1:-cross_entropy}
SECT=${2:-ce}
LEGACY=${3:-PENROZ_CE_KERNEL=1024}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
timeout -k 10 200 python -u bench/kernel_bench.py $SECT > gpurun_out/ab_kernels.log 2>&1 || { tail -20 gpurun_out/ab_kernels.log; exit 1; }
timeout -k 10 200 env $LEGACY python -u bench/kernel_bench.py $SECT >> gpurun_out/ab_kernels.log 2>&1 || { tail -20 gpurun_out/ab_kernels.log; exit 1; }
cat gpurun_out/ab_kernels.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --ref-steps 0 > gpurun_out/ab_bench.log 2>&1 || { tail -20 gpurun_out/ab_bench.log; exit 1; }
tail -1 gpurun_out/ab_bench.log
