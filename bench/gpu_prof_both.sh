# Kernel-trace profiles of the headline step: serial stream (per-kernel cost without overlap)
# then the default side-stream configuration.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
PENROZ_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_serial -o run -- python3 bench.py --steps 5 --warmup 3 --ref-steps 0 > gpurun_out/prof_serial_bench.log 2>&1 || exit $?
DB=$(find gpurun_out/prof_serial -name 'run_results.db' | head -n1)
python3 bench/prof_summary.py $DB --steps 8 > gpurun_out/prof_serial_summary.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 3 --ref-steps 0 > gpurun_out/prof_bench.log 2>&1 || exit $?
DB=$(find gpurun_out/prof -name 'run_results.db' | head -n1)
python3 bench/prof_summary.py $DB --steps 8 > gpurun_out/prof_summary.txt
head -n 30 gpurun_out/prof_serial_summary.txt | cut -c1-130
head -n 30 gpurun_out/prof_summary.txt | cut -c1-130
