# (1) headline config through the runtime path (train_model) vs the executor loop;
# (2) GPT-2 XL (1.56 B params) batch sweep on one MI355X (288 GB HBM sizing)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --ref-steps 0 --via-runtime > gpurun_out/bench_runtime.log 2>&1; tail -1 gpurun_out/bench_runtime.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('executor', round(d['value']), 'runtime', d['via_runtime'])" || exit 1
for b in 16 32 64; do
  timeout -k 10 400 python bench.py --model gpt2-xl --batch $b --steps 4 --warmup 2 --ref-steps 0 > gpurun_out/bench_xl_b$b.log 2>&1
  rc=$?
  if [ $rc -eq 0 ]; then tail -1 gpurun_out/bench_xl_b$b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('xl B=$b', round(d['value']), 'tok/s', round(d['ms_per_step'],1), 'ms', 'mfu', round(d['mfu_bf16_dense'],3))"; 
  elif grep -q "OutOfMemoryError" gpurun_out/bench_xl_b$b.log; then echo "xl B=$b: out of memory"; else echo "xl B=$b failed rc=$rc"; tail -5 gpurun_out/bench_xl_b$b.log; exit $rc; fi
done
