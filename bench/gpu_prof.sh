# rocprofv3 kernel trace of the headline bench (3 warmup + 5 timed = 8 steps)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=${1:-gpurun_out/prof}
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT -o run -- python3 bench.py --steps 5 --warmup 3 --ref-steps 0 > gpurun_out/prof_bench.log 2>&1
DB=$(find $OUT -name 'run_results.db' | head -n1)
python3 bench/prof_summary.py $DB --steps 8 > gpurun_out/prof_summary.txt
cat gpurun_out/prof_summary.txt | head -n 45
