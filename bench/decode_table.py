"""Per-step kernel table of a graph-replayed decode run from a rocprofv3 ``--kernel-trace`` database
(rocpd SQLite, ``<dir>/run_results.db``; bench/decode_rocprof.sh writes them).

Steps are counted as the calls of one kernel that runs once per decode step (``--per-step``,
default the sampler's merge kernel). Prefill and warm-up kernels stay in the totals; they are the
rows with well under one call per step.

    python bench/decode_table.py gpurun_out/decprof/gemma3-1b/run_results.db
"""
from __future__ import annotations

import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--per-step", default="sample_merge_kernel")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, count(*), sum(end - start), max(grid_x * grid_y * grid_z / "
                     "(workgroup_x * workgroup_y * workgroup_z)) from kernels group by name").fetchall()
    steps = sum(n for name, n, _, _ in rows if a.per_step in name)
    if not steps:
        raise SystemExit(f"no kernel matching {a.per_step!r}")
    rows.sort(key=lambda r: -r[2])
    total = sum(r[2] for r in rows)
    print(f"# {a.db}: {steps} decode steps, {total / steps / 1e3:.1f} us of kernel time per step")
    print(" calls/step  us/step  us/call    WGs  kernel")
    for name, n, ns, wgs in rows[:a.top]:
        print(f"{n / steps:10.2f} {ns / steps / 1e3:8.1f} {ns / n / 1e3:8.2f} {wgs:6d}  {name[:100]}")


if __name__ == "__main__":
    main()
