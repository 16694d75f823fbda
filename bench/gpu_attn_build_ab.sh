# Same-box attention microbench of a baseline build (build_ab) vs the working build at the Gemma-3 1B
# in-step shape (D = 256, H = 4, Hkv = 1, T = 1024), B = 8 and 16, two passes. Run via gpurun.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for e in PENROZ_EXT_DIR=build_ab PENROZ_EXT_DIR=build_ext; do
    for B in 8 16; do
      env $e timeout -k 10 120 python bench/attn_bench.py --B $B --T 1024 --H 4 --Hkv 1 --D 256 --iters 30 \
        > gpurun_out/attn_ab.log 2>&1 || { tail -20 gpurun_out/attn_ab.log; exit 1; }
      echo "[$e] B$B $(grep '^{' gpurun_out/attn_ab.log)"
    done
  done
done
