"""Summarise bench/gpu_pmc_gemm_all.sh: per (shape, kernel) MFMA busy, VALU/SALU per MFMA,
wait / LDS / conflict fractions and HBM bytes, from the rocprofv3 counter CSVs.

    python bench/pmc_gemm_summary.py gpurun_out/pmc_all
"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
rows = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    tag = os.path.relpath(f, root).split(os.sep)[0]  # <shape>_<mode>_p<i>
    shape, mode = tag.rsplit("_", 2)[0], tag.rsplit("_", 2)[1]
    n = collections.Counter()
    for r in csv.DictReader(open(f)):
        kn = r.get("Kernel_Name", "")
        if "gemm_kernel" not in kn and "Cijk" not in kn:
            continue
        rows[(shape, mode)][r["Counter_Name"]] += float(r["Counter_Value"])
print(f"{'shape':8s} {'kernel':6s} {'MFMA busy':>9s} {'VALU/MFMA':>9s} {'SALU/MFMA':>9s} {'wait/wave':>9s} "
      f"{'LDSwait':>8s} {'conflict':>9s} {'FETCH GB':>9s} {'WRITE GB':>9s}")
for (shape, mode), c in sorted(rows.items()):
    mf = c.get("SQ_INSTS_MFMA", 0) or 1
    busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(1.0, 1024 * c.get("GRBM_GUI_ACTIVE", 0) / 8)
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{shape:8s} {'native' if mode == 'fwd' else 'blaslt':6s} {busy:9.1%} {c.get('SQ_INSTS_VALU', 0) / mf:9.2f} "
          f"{c.get('SQ_INSTS_SALU', 0) / mf:9.2f} {c.get('SQ_WAIT_INST_ANY', 0) / wc:9.1%} "
          f"{c.get('SQ_WAIT_INST_LDS', 0) / wc:8.1%} {c.get('SQ_LDS_BANK_CONFLICT', 0):9.3g} "
          f"{c.get('FETCH_SIZE', 0) / 1e6:9.2f} {c.get('WRITE_SIZE', 0) / 1e6:9.2f}")
print("# 3 dispatches per pass; MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs);"
      " FETCH/WRITE_SIZE are KB counters (gfx950 half-count caveat: compare kernels, not absolutes)")
