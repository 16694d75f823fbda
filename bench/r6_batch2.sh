set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "dropout or flash" > gpurun_out/drop_tests.log 2>&1; tail -3 gpurun_out/drop_tests.log
timeout -k 10 300 python -u -m pytest tests/test_executor_gpu.py -x -q --timeout 200 --timeout-method thread -k "dropout or hf" > gpurun_out/drop_exec.log 2>&1; tail -2 gpurun_out/drop_exec.log
timeout -k 10 200 python bench/attn_bench.py --B 64 --T 1024 --H 12 --Hkv 12 --D 64 --p 0.1 --iters 10 > gpurun_out/attn_drop.log 2>&1; grep "{" gpurun_out/attn_drop.log | cut -c1-300
timeout -k 10 300 python bench.py --model gpt2-hf --steps 10 --warmup 3 --ref-steps 0 --no-gemm-table-guard > gpurun_out/hf_arm.log 2>&1 && echo "gpt2-hf $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/hf_arm.log)"
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/gemma_kt -o run -- python3 bench.py --model gemma3-1b --batch 8 --steps 3 --warmup 2 --ref-steps 0 --no-gemm-table-guard > gpurun_out/gemma_kt.log 2>&1 || { tail -5 gpurun_out/gemma_kt.log; exit 1; }
DB=$(find gpurun_out/gemma_kt -name 'run_results.db' | head -n1)
python3 bench/prof_summary.py $DB --steps 5 --top 40 > gpurun_out/rocprof_r6_gemma3_b8_summary.txt; rm -rf gpurun_out/gemma_kt
head -36 gpurun_out/rocprof_r6_gemma3_b8_summary.txt | cut -c1-150
