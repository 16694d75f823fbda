# rocprofv3 kernel trace of the Gemma-3 1B shaped graph decode (batch 1 and 64)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in 1 64; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/profgem$b -o run -- python3 bench/bench_decode.py --model gemma3-1b --batch $b --new 64 > gpurun_out/profgem$b.log 2>&1 || exit 1
  DB=$(find gpurun_out/profgem$b -name 'run_results.db' | head -n1)
  python3 bench/prof_summary.py $DB --steps 68 --top 30 > gpurun_out/profgem${b}_summary.txt || exit 1
  rm -rf gpurun_out/profgem$b
  head -n 36 gpurun_out/profgem${b}_summary.txt
done
