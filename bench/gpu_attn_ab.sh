# attention kernels: several in-tree builds (PENROZ_EXT_DIR per arm), interleaved, after the
# attention GPU tests of the current build
#   ARMS="build_ab build_ext" bash bench/gpu_attn_ab.sh [attn_bench.py config ...]
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -k "flash" --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_attn.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_attn.log; [ $rc -eq 0 ] || exit 1
[ $# -gt 0 ] || set -- "--B 64 --T 1024 --H 12 --Hkv 12 --D 64"
ARMS=${ARMS:-build_ab build_ext}
for pass in 1 2 3; do
  for cfg in "$@"; do
    for arm in $ARMS; do
      PENROZ_EXT_DIR=$PWD/$arm timeout -k 10 120 python bench/attn_bench.py $cfg --iters 10 > gpurun_out/attn.log 2>&1 \
        || { tail -20 gpurun_out/attn.log; exit 1; }
      echo "$arm $(grep '^{' gpurun_out/attn.log)"
    done
  done
done
