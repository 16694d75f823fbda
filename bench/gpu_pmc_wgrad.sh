# PMC passes (one counter group per run) for the native wgrad kernel (lm_head and qkv shapes) and
# the flash-attention kernels' memory traffic. Summaries -> gpurun_out/pmcw/summary.txt
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcw
run() { timeout -s KILL 60 rocprofv3 --pmc $1 --output-format csv -d gpurun_out/pmcw/$2 -o p -- python3 $3 > gpurun_out/pmcw/$2.log 2>&1; }
for shp in lm_head qkv; do
  run "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" ${shp}_a "bench/wgrad_one.py $shp" || exit 1
  run "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE" ${shp}_b "bench/wgrad_one.py $shp" || exit 1
  run "FETCH_SIZE" ${shp}_c "bench/wgrad_one.py $shp" || exit 1
  run "WRITE_SIZE" ${shp}_d "bench/wgrad_one.py $shp" || exit 1
done
run "FETCH_SIZE" attn_c "bench/attn_bench.py --iters 2" || exit 1
run "WRITE_SIZE" attn_d "bench/attn_bench.py --iters 2" || exit 1
python3 - > gpurun_out/pmcw/summary.txt <<'PY'
import csv, glob, collections, os
for d in sorted(glob.glob("gpurun_out/pmcw/*/")):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        continue
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    calls = collections.defaultdict(set)
    for r in csv.DictReader(open(f[0])):
        kn = r.get("Kernel_Name", "")
        key = next((k for k in ("wgrad256_ring16", "fa_fwd3", "fa_bwd_dkdv2", "fa_bwd_dq3", "fa_bwd_pre") if k in kn), None)
        if key is None:
            continue
        tot[key][r["Counter_Name"]] += float(r["Counter_Value"])
        calls[key].add(r.get("Dispatch_Id", ""))
    for k, c in tot.items():
        print(os.path.basename(d.rstrip("/")), k, f"dispatches={len(calls[k])}", " ".join(f"{n}={v:.4g}" for n, v in sorted(c.items())))
PY
cat gpurun_out/pmcw/summary.txt
