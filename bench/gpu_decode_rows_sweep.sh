# Decode step time vs batch rows with the fused add+LN+GEMM kernel on / off (threshold sizing).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in ${BATCHES:-1 4 8 16 32}; do for f in 0 1; do
  PENROZ_DECODE_FUSED=$f PENROZ_DECODE_FUSED_MAX_ROWS=64 timeout -k 10 300 python -u bench/bench_decode.py --batch $b --new 96 > gpurun_out/drs_b${b}_f$f.log 2>&1 || { tail -5 gpurun_out/drs_b${b}_f$f.log; exit 1; }
  echo "batch=$b fused=$f $(tail -1 gpurun_out/drs_b${b}_f$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), "ms/step", round(d["value"]), "tok/s")')"
done; done
