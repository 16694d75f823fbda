set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_runtime_gpu.py tests/test_graph_decode_gpu.py -k "rope or gemma or generic or runtime" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_rope.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_rope.log; exit 1; }
tail -2 gpurun_out/pytest_rope.log
for B in 8 16; do
  timeout -k 10 400 python bench.py --model gemma3-1b --batch $B --steps 5 --warmup 2 --ref-steps 0 > gpurun_out/gemma_train_b$B.log 2>&1 || { tail -30 gpurun_out/gemma_train_b$B.log; exit 1; }
  echo "gemma3-1b B=$B: $(grep '^{' gpurun_out/gemma_train_b$B.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"], 1), round(d["mfu_bf16_dense"], 3))')"
done
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_gemma3 -o run -- python3 bench.py --model gemma3-1b --batch 8 --steps 3 --warmup 1 --ref-steps 0 > gpurun_out/prof_gemma_bench.log 2>&1 || { tail -20 gpurun_out/prof_gemma_bench.log; exit 1; }
DB=$(find gpurun_out/prof_gemma3 -name 'run_results.db' | head -n1)
python3 bench/prof_summary.py $DB --steps 4 > gpurun_out/prof_gemma_summary.txt
grep -E "rope|ms/step" gpurun_out/prof_gemma_summary.txt | cut -c1-140
