# Serial-stream kernel profile of the HF-import GPT-2 layout (dropout 0.1, V=50257, bf16 params)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/prof_hf
PENROZ_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT -o run -- python3 bench.py --model gpt2-hf --steps 3 --warmup 2 --ref-steps 0 > gpurun_out/prof_hf_bench.log 2>&1
DB=$(find $OUT -name 'run_results.db' | head -n1)
python3 bench/prof_summary.py $DB --steps 5 > gpurun_out/prof_hf_summary.txt
head -n 30 gpurun_out/prof_hf_summary.txt
