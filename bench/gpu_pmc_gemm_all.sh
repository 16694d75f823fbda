# Per-shape PMC evidence, native fwd GEMM (csrc/kernels/gemm.hip, off by default) vs hipBLASLt, at
# the five GPT-2 124M forward shapes (M = 65 536): four counter passes per (shape, kernel), each
# its own rocprofv3 run; summary table in gpurun_out/pmc_all/summary.txt
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_all
P1="SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
for shape in "qkv 768 2304" "proj 768 768" "fc 768 3072" "fc2 3072 768" "lm_head 768 50304"; do
  set -- $shape
  for mode in fwd blas; do
    i=0
    for P in "$P1" "$P2" "$P3" "$P4"; do
      i=$((i+1))
      timeout -s KILL 60 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc_all/$1_${mode}_p$i -o p -- python3 bench/gemm_one.py $mode $2 $3 3 > gpurun_out/pmc_all/$1_${mode}_$i.log 2>&1 || { echo "pmc pass failed: $1 $mode $i"; tail -5 gpurun_out/pmc_all/$1_${mode}_$i.log; exit 1; }
    done
  done
done
python3 bench/pmc_gemm_summary.py gpurun_out/pmc_all > gpurun_out/pmc_all/summary.txt
cat gpurun_out/pmc_all/summary.txt
