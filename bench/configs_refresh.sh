# Refresh of every secondary config (one box, one after the other) -> gpurun_out/bench_r6_configs.log
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
LOG=gpurun_out/bench_r6_configs.log
: > $LOG
run() {  # name, time limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/cfg_run.log 2>&1 || { echo "$name FAILED"; tail -20 gpurun_out/cfg_run.log; exit 1; }
  echo "$name $(grep '^{' gpurun_out/cfg_run.log | tail -1 | cut -c1-1500)" | tee -a $LOG | cut -c1-300
}
run headline 300 python bench.py --steps 20 --warmup 5
run gpt2-hf 300 python bench.py --model gpt2-hf --steps 10 --warmup 3 --ref-steps 0
run gpt2-hf-nodropout 300 env PENROZ_BENCH_HF_PDROP=0 python bench.py --model gpt2-hf --steps 10 --warmup 3 --ref-steps 0
run gpt2-xl 500 python bench.py --model gpt2-xl --steps 5 --warmup 2 --ref-steps 0
run via-runtime 500 python bench.py --steps 15 --warmup 3 --ref-steps 0 --via-runtime
run gemma3-1b-b8 400 python bench.py --model gemma3-1b --batch 8 --steps 5 --warmup 2 --ref-steps 0
run gemma4-e2b-b8 400 python bench.py --model gemma4-e2b --batch 8 --steps 5 --warmup 2 --ref-steps 0
for m in gpt2 gemma3-1b; do for b in 1 32 64; do
  run decode-$m-b$b 300 python bench/bench_decode.py --model $m --batch $b
done; done
run decode-gpt2-b1-ctx1k 300 python bench/bench_decode.py --model gpt2 --batch 1 --prompt 832 --new 128
run decode-gemma3-1b-b1-ctx4k 300 python bench/bench_decode.py --model gemma3-1b --batch 1 --prompt 3968 --new 128 --block 4096
timeout -k 10 300 python -u -m pytest tests/test_executor_parity_gpu.py -x -q -s --timeout 250 --timeout-method thread -k headline > gpurun_out/parity_s.log 2>&1; grep -E "parity|passed|failed" gpurun_out/parity_s.log | tee -a $LOG
