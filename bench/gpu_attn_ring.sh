# flash-attention backward: ring-depth A/B (variants 2 / 3 / 4), the flash kernel tests (incl. the
# fused qkv-bias gradient), and the headline bench with variant 3 vs 4
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "flash" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_flash.log 2>&1 || { echo "flash tests failed"; tail -30 gpurun_out/pytest_flash.log; exit 1; }
tail -2 gpurun_out/pytest_flash.log
timeout -k 10 180 python bench/attn_bench.py --which bwd --iters 20 > gpurun_out/attn_ring.log 2>&1 || { tail -20 gpurun_out/attn_ring.log; exit 1; }
grep '^{' gpurun_out/attn_ring.log
for v in 3 4; do
  timeout -k 10 300 env PENROZ_FLASH_BWD_VARIANT=$v python bench.py --steps 20 --warmup 5 --ref-steps 0 > gpurun_out/bench_v$v.log 2>&1 || { tail -20 gpurun_out/bench_v$v.log; exit 1; }
  echo "variant $v: $(tail -1 gpurun_out/bench_v$v.log | cut -c1-200)"
done
