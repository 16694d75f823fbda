set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmca
run() { timeout -s KILL 90 rocprofv3 --pmc $1 --output-format csv -d gpurun_out/pmca/$2 -o p -- python3 bench/attn_bench.py --iters 3 > gpurun_out/pmca/$2.log 2>&1; }
run "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" a && \
run "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE" b
for d in a b; do f=$(find gpurun_out/pmca/$d -name '*counter_collection.csv' | head -n1); echo "== $d"; python3 - "$f" <<'PY'
import csv, sys, collections
tot = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    kn = r.get("Kernel_Name", "")
    for key in ("fa_fwd3", "fa_bwd_dkdv2", "fa_bwd_dq3", "fa_bwd_pre"):
        if key in kn:
            tot[key][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in tot.items():
    print(k, " ".join(f"{c}={v:.4g}" for c, v in sorted(d.items())))
PY
done
