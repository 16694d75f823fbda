set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
run() { timeout -s KILL 60 rocprofv3 --pmc $1 --output-format csv -d gpurun_out/pmc/$2 -o p -- python3 bench/gemm_one.py $3 $4 $5 > gpurun_out/pmc/$2.log 2>&1; }
run "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" fc2fwd fwd 3072 768 && \
run "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" fc2blas blas 3072 768 && \
run "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE" fc2fwd_b fwd 3072 768
for d in fc2fwd fc2blas fc2fwd_b; do f=$(find gpurun_out/pmc/$d -name '*counter_collection.csv' | head -n1); echo "== $d"; python3 - "$f" <<'PY'
import csv, sys, collections
tot = collections.defaultdict(float); names = {}
for r in csv.DictReader(open(sys.argv[1])):
    kn = r.get("Kernel_Name", "")
    if "gemm_kernel" not in kn and "Cijk" not in kn: continue
    tot[r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(tot.items()): print(f"{k:28s} {v:.4g}")
PY
done
