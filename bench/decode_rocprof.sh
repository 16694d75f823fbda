# Kernel-trace stats of the graph-replayed decode step at batch 64 (GPT-2 124M and Gemma-3 1B):
# per-kernel time per step, for profiles/rocprof_r6_decode_*.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
cd /tmp && cd "$GRAFT_REPO_ROOT"
for m in gpt2 gemma3-1b; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/decprof/$m -o run -- \
    python3 bench/bench_decode.py --model $m --batch 64 > gpurun_out/decprof/$m.log 2>&1 || { tail -20 gpurun_out/decprof/$m.log; exit 1; }
done
