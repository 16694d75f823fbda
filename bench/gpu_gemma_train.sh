# Gemma-3 1B shaped training (generic engine over the HIP layers), B = 8 / 16 x T = 1024, and a
# kernel-trace profile of the B = 8 step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for B in 8 16; do
  timeout -k 10 400 python bench.py --model gemma3-1b --batch $B --steps 5 --warmup 2 --ref-steps 0 > gpurun_out/gemma_train_b$B.log 2>&1 || { tail -30 gpurun_out/gemma_train_b$B.log; exit 1; }
  grep '^{' gpurun_out/gemma_train_b$B.log | cut -c1-400
done
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_gemma -o run -- python3 bench.py --model gemma3-1b --batch 8 --steps 3 --warmup 1 --ref-steps 0 > gpurun_out/prof_gemma_bench.log 2>&1 || { tail -20 gpurun_out/prof_gemma_bench.log; exit 1; }
DB=$(find gpurun_out/prof_gemma -name 'run_results.db' | head -n1)
python3 bench/prof_summary.py $DB --steps 4 > gpurun_out/prof_gemma_summary.txt
head -n 25 gpurun_out/prof_gemma_summary.txt | cut -c1-140
