# head_dim 128 / 256 flash attention vs torch SDPA (Gemma-3 1B: H=4, Hkv=1, D=256)
set -o pipefail
mkdir -p gpurun_out
for cfg in "--B 16 --T 2048 --H 4 --Hkv 1 --D 256" "--B 8 --T 4096 --H 4 --Hkv 1 --D 256" "--B 16 --T 2048 --H 16 --Hkv 8 --D 128" "--B 64 --T 1024 --H 12 --Hkv 12 --D 64"; do
  timeout -k 10 120 python bench/attn_bench.py $cfg --iters 10 --sdpa 2>&1 | grep '^{' || exit 1
done
