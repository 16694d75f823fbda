"""Per-step timeline of a rocprofv3 kernel trace: wall time, per-queue busy time, overlap.

    python bench/timeline.py gpurun_out/prof2/run_results.db [--marker adam_flat_kernel]

Steps are delimited by the optimizer kernel (one per step). Reports, for each complete step:
wall (first kernel start -> optimizer end), busy time of each HW queue (union of its kernel
intervals), the union over all queues, and the top kernels by time on each queue.
"""
import argparse
import collections
import sqlite3


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="adam_flat_kernel")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, queue_id from kernels order by start").fetchall()
    ends = [i for i, r in enumerate(rows) if a.marker in r[0]]
    for k in range(1, len(ends)):
        seg = rows[ends[k - 1] + 1: ends[k] + 1]
        t0, t1 = seg[0][1], seg[-1][2]
        byq = collections.defaultdict(list)
        names = collections.defaultdict(lambda: collections.Counter())
        for n, s, e, q in seg:
            byq[q].append((s, e))
            short = n.split("(")[0].replace("void ", "")[:60]
            names[q][short] += e - s
        allu = union([(s, e) for _, s, e, _ in seg])
        print(f"step {k}: wall {(t1 - t0) / 1e6:.2f} ms, any-queue busy {allu / 1e6:.2f} ms")
        for q, iv in byq.items():
            top = ", ".join(f"{n} {t / 1e6:.2f}" for n, t in names[q].most_common(4))
            print(f"   queue {q}: {len(iv)} kernels, busy {union(iv) / 1e6:.2f} ms | {top}")


if __name__ == "__main__":
    main()
