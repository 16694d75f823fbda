# kernel-trace profile of the Gemma-3 1B shaped training step (B = 8) + the HF GPT-2 layout on the
# generic engine
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_gemma2 -o run -- python3 bench.py --model gemma3-1b --batch 8 --steps 3 --warmup 1 --ref-steps 0 > gpurun_out/prof_gemma_bench.log 2>&1 || { tail -20 gpurun_out/prof_gemma_bench.log; exit 1; }
DB=$(find gpurun_out/prof_gemma2 -name 'run_results.db' | head -n1)
python3 bench/prof_summary.py $DB --steps 4 > gpurun_out/prof_gemma_summary.txt
head -n 20 gpurun_out/prof_gemma_summary.txt | cut -c1-140
timeout -k 10 400 python bench.py --model gpt2-hf --engine generic --steps 10 --warmup 3 --ref-steps 0 > gpurun_out/hf_generic.log 2>&1 || { tail -30 gpurun_out/hf_generic.log; exit 1; }
echo "gpt2-hf generic: $(grep '^{' gpurun_out/hf_generic.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"], 1))')"
