set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/profdec -o run -- python3 bench/bench_decode.py --new 64 > gpurun_out/profdec.log 2>&1
DB=$(find gpurun_out/profdec -name 'run_results.db' | head -n1)
python3 bench/prof_summary.py $DB --steps 67 --top 25 > gpurun_out/profdec_summary.txt
head -n 30 gpurun_out/profdec_summary.txt
