# GPT-2 XL B=64: side stream for weight-gradient GEMMs on (default) vs off, alternating
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in 1 0 1 0; do
  timeout -k 10 300 env PENROZ_WGRAD_STREAM=$s python bench.py --model gpt2-xl --batch 64 --steps 4 --warmup 2 --ref-steps 0 > gpurun_out/xl_stream$s.log 2>&1 || { tail -20 gpurun_out/xl_stream$s.log; exit 1; }
  echo "xl wgrad_stream=$s: $(grep '^{' gpurun_out/xl_stream$s.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"], 1))')"
done
for s in 1 0; do
  timeout -k 10 300 env PENROZ_WGRAD_STREAM=$s python bench.py --steps 20 --warmup 5 --ref-steps 0 > gpurun_out/s_stream$s.log 2>&1 || { tail -20 gpurun_out/s_stream$s.log; exit 1; }
  echo "124m wgrad_stream=$s: $(grep '^{' gpurun_out/s_stream$s.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"], 2))')"
done
