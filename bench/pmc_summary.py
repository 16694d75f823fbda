"""Summarise the PMC passes of ``bench/gpu.sh pmc``: per kernel (name contains one of the given
substrings) the counters summed over dispatches, plus the derived rates the performance notes
quote: MFMA busy, VALU / MFMA, wait and LDS-wait fractions, bank conflicts per LDS instruction,
HBM bytes read / written.

    python bench/pmc_summary.py gpurun_out/pmc_attn fa_fwd3,fa_bwd_dkdv,fa_bwd_dq
"""
import collections
import csv
import glob
import os
import sys

root, keys = sys.argv[1], sys.argv[2].split(",")
tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        kn = r.get("Kernel_Name", "")
        key = next((k for k in keys if k in kn), None)
        if key is None:
            continue
        tot[key][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[key].add((f, r.get("Dispatch_Id", "")))
for k in keys:
    c = tot.get(k)
    if not c:
        print(f"{k}: no dispatches")
        continue
    mf = c.get("SQ_INSTS_MFMA", 0) or 1
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(1.0, 1024 * c.get("GRBM_GUI_ACTIVE", 0) / 8)
    lds = c.get("SQ_LDS_IDX_ACTIVE", 0) or 1
    print(f"{k}: dispatches/pass={len(disp[k]) // 4} MFMA_busy={busy:.1%} VALU/MFMA={c.get('SQ_INSTS_VALU', 0) / mf:.2f} "
          f"SALU/MFMA={c.get('SQ_INSTS_SALU', 0) / mf:.2f} wait_any={c.get('SQ_WAIT_ANY', 0) / wc:.1%} "
          f"wait_inst={c.get('SQ_WAIT_INST_ANY', 0) / wc:.1%} lds_wait={c.get('SQ_WAIT_INST_LDS', 0) / wc:.1%} "
          f"lds_conflict={c.get('SQ_LDS_BANK_CONFLICT', 0) / lds:.1%} "
          f"fetch_GB={c.get('FETCH_SIZE', 0) / 1e6:.3f} write_GB={c.get('WRITE_SIZE', 0) / 1e6:.3f}")
    print("   " + " ".join(f"{n}={v:.4g}" for n, v in sorted(c.items())))
