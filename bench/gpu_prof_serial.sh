# Serial-stream kernel profile of the headline step (no side-stream overlap: per-kernel times are
# not inflated by concurrent kernels) + attention PMC counters.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=${1:-gpurun_out/prof_serial}
PENROZ_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT -o run -- python3 bench.py --steps 5 --warmup 3 --ref-steps 0 > gpurun_out/prof_serial_bench.log 2>&1
DB=$(find $OUT -name 'run_results.db' | head -n1)
python3 bench/prof_summary.py $DB --steps 8 > gpurun_out/prof_serial_summary.txt
head -n 40 gpurun_out/prof_serial_summary.txt
tail -1 gpurun_out/prof_serial_bench.log
bash bench/gpu_pmc_attn.sh
