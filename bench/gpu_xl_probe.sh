# GPT-2 XL: native vs hipBLASLt weight-gradient GEMMs at the XL shapes, then a serial-stream
# kernel profile of the B=64 step (per-kernel cost without side-stream overlap)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench/wgrad_blas_ab.py --model gpt2-xl --iters 5 > gpurun_out/wgrad_xl.log 2>&1 || { tail -20 gpurun_out/wgrad_xl.log; exit 1; }
grep '^{' gpurun_out/wgrad_xl.log
PENROZ_WGRAD_STREAM=0 timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_xl -o run -- python3 bench.py --model gpt2-xl --batch 64 --steps 2 --warmup 1 --ref-steps 0 > gpurun_out/prof_xl_bench.log 2>&1 || { tail -20 gpurun_out/prof_xl_bench.log; exit 1; }
DB=$(find gpurun_out/prof_xl -name 'run_results.db' | head -n1)
python3 bench/prof_summary.py $DB --steps 3 > gpurun_out/prof_xl_summary.txt
head -n 20 gpurun_out/prof_xl_summary.txt | cut -c1-130
tail -1 gpurun_out/prof_xl_bench.log | cut -c1-300
