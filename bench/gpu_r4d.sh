# Round-4 GPU batch: attention D=64 (GPT-2 shape) and D=256 (Gemma in-step shape), new kernels vs
# the previous build (build_ab/, PENROZ_EXT_DIR) interleaved; attention GPU tests; fresh PMC for
# the D=64 kernels; then the secondary BASELINE configs (GPT-2 XL B=64, HF GPT-2 layout).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -k "flash" --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_attn.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_attn.log; [ $rc -eq 0 ] || exit 1
for pass in 1 2; do
  for cfg in "--B 64 --T 1024 --H 12 --Hkv 12 --D 64" "--B 8 --T 1024 --H 4 --Hkv 1 --D 256"; do
    for arm in old new; do
      if [ $arm = old ]; then export PENROZ_EXT_DIR=$PWD/build_ab; else unset PENROZ_EXT_DIR; fi
      timeout -k 10 120 python bench/attn_bench.py $cfg --iters 10 > gpurun_out/attn.log 2>&1 || { tail -20 gpurun_out/attn.log; exit 1; }
      echo "$arm $(grep '^{' gpurun_out/attn.log)"
    done
  done
done
unset PENROZ_EXT_DIR
bash bench/gpu.sh pmc attn64 fa_ -- python bench/attn_bench.py --B 64 --T 1024 --H 12 --Hkv 12 --D 64 --iters 2 || exit 1
for m in gpt2-xl gpt2-hf; do
  timeout -k 10 400 python bench.py --model $m --steps 10 --warmup 3 --ref-steps 0 > gpurun_out/bench_$m.log 2>&1 || { tail -20 gpurun_out/bench_$m.log; exit 1; }
  grep '^{' gpurun_out/bench_$m.log | cut -c1-900
done
