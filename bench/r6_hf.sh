set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for arm in "gpt2-124m:" "gpt2-hf:" "gpt2-hf:PENROZ_BENCH_HF_PDROP=0"; do
  m=${arm%%:*}; e=${arm#*:}
  env $e timeout -k 10 300 python bench.py --model $m --steps 10 --warmup 3 --ref-steps 0 --no-gemm-table-guard > gpurun_out/hf_arm.log 2>&1 || { tail -20 gpurun_out/hf_arm.log; exit 1; }
  echo "$m $e $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/hf_arm.log)"
done
export AMD_SERIALIZE_KERNEL=3
PROF_STEPS=8 PROF_TOP=40 bash bench/gpu.sh prof rocprof_r6_gpt2_hf_serial -- python3 bench.py --model gpt2-hf --steps 5 --warmup 3 --ref-steps 0 --no-gemm-table-guard > /dev/null || exit 1
head -45 gpurun_out/rocprof_r6_gpt2_hf_serial_summary.txt | cut -c1-150
unset AMD_SERIALIZE_KERNEL
timeout -k 10 300 python bench.py --model gemma3-1b --batch 8 --steps 2 --warmup 2 --ref-steps 0 --no-gemm-table-guard --profile gpurun_out/gemma_prof > gpurun_out/gemma_prof.log 2>&1 || { tail -20 gpurun_out/gemma_prof.log; exit 1; }
grep -E "aten::|Name" gpurun_out/gemma_prof/rank0/kernels.txt | head -40 | cut -c1-200
