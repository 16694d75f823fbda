# decode kernel traces (graph replay), GPT-2 124M, batch 64 and 1
set -o pipefail
mkdir -p gpurun_out
for b in 64 1; do
  PROF_STEPS=128 bash bench/gpu.sh prof dec_b$b -- python3 bench/bench_decode.py --model gpt2 --batch $b > gpurun_out/dec_prof_b$b.txt 2>&1 || { tail -5 gpurun_out/dec_prof_b$b.txt; exit 1; }
  head -32 gpurun_out/dec_b${b}_summary.txt | cut -c1-150
done
