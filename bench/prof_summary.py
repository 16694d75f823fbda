"""Summarise a rocprofv3 kernel trace (``--kernel-trace`` SQLite ``*_results.db`` or the
``kernel_stats.csv`` of ``--stats --output-format csv``) into a per-kernel table.

    python bench/prof_summary.py gpurun_out/prof3/run_results.db --steps 8 [--top 40] [--csv out.csv]

``--steps`` divides totals into per-step figures (count every step the profiled run executed:
warmup + timed). Kernel names are shortened (template arguments and parameter lists dropped).
"""
from __future__ import annotations

import argparse
import collections
import csv
import re
import sqlite3
import sys


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\([^()]*\)$", "", name)
    if name.startswith("void "):
        name = name[5:]
    # drop namespaces and template arguments, keep a distinguishing prefix
    base = re.sub(r"<.*>", "<>", name)
    base = base.split("::")[-1] if "::" in base and not base.startswith("Cijk") else base
    return base[:90]


def load_db(path: str):
    c = sqlite3.connect(path)
    rows = c.execute("select name, duration, grid_x, workgroup_x, vgpr_count, accum_vgpr_count, lds_size from kernels")
    for name, dur, gx, wx, vg, ag, lds in rows:
        yield name, float(dur), int(gx or 0) // max(1, int(wx or 1)), int(vg or 0), int(ag or 0), int(lds or 0)


def load_csv(path: str):
    with open(path) as f:
        for r in csv.DictReader(f):
            yield r["Name"], float(r["TotalDurationNs"]), 0, 0, 0, 0


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--csv", default=None)
    ap.add_argument("--by-grid", action="store_true", help="one row per (kernel, workgroup count)")
    a = ap.parse_args(argv)
    src = load_db(a.path) if a.path.endswith(".db") else load_csv(a.path)
    agg = collections.defaultdict(lambda: [0, 0.0, 0, 0, 0, 0])
    for name, dur, wgs, vg, ag, lds in src:
        k = f"{short(name)} [{wgs}]" if a.by_grid else short(name)
        e = agg[k]
        e[0] += 1
        e[1] += dur
        e[2], e[3], e[4], e[5] = wgs, vg, ag, lds
    total = sum(e[1] for e in agg.values())
    items = sorted(agg.items(), key=lambda kv: -kv[1][1])
    out = [("kernel", "calls", "total_ms", "per_step_ms", "avg_us", "pct", "workgroups", "vgpr", "agpr", "lds")]
    for k, (n, t, wgs, vg, ag, lds) in items[: a.top]:
        out.append((k, n, f"{t / 1e6:.3f}", f"{t / 1e6 / a.steps:.3f}", f"{t / n / 1e3:.1f}", f"{100 * t / total:.1f}",
                    wgs, vg, ag, lds))
    print(f"# {a.path}: {sum(e[0] for e in agg.values())} dispatches, {total / 1e6:.2f} ms GPU kernel time, "
          f"{total / 1e6 / a.steps:.2f} ms/step over {a.steps} step(s)")
    w = [max(len(str(r[i])) for r in out) for i in range(len(out[0]))]
    for r in out:
        print("  ".join(str(v).ljust(w[i]) if i == 0 else str(v).rjust(w[i]) for i, v in enumerate(r)))
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            csv.writer(f).writerows(out)


if __name__ == "__main__":
    sys.exit(main())
