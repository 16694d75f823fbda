"""Per-step timeline of a rocprofv3 kernel trace: wall time, per-queue busy time, overlap.

    python bench/timeline.py gpurun_out/prof2/run_results.db [--marker adam_flat_kernel]

Steps are delimited by a marker kernel (default: the optimizer kernel, one per step; with the
optimizer fused into the backward use the first forward kernel, e.g. ``--marker embed_fwd``).
``--tail N`` lists the last N kernels of the last complete step (the step's critical tail). Reports, for each complete step:
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
    ap.add_argument("--tail", type=int, default=0, help="also list the last N kernels (by end) of the last step")
    ap.add_argument("--window", type=float, nargs=2, default=None, metavar=("MS0", "MS1"),
                    help="list every kernel of the last step that overlaps [MS0, MS1] ms from its start")
    ap.add_argument("--gaps", type=float, default=0.0,
                    help="also list idle gaps >= this many µs of the busiest queue in the last step, with the "
                         "other queues' kernels running in them")
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
        if a.gaps and k == len(ends) - 1:
            mq = max(byq, key=lambda q: union(byq[q]))
            iv = sorted((s_, e) for _, s_, e, q in seg if q == mq)
            mk = sorted((s_, e, n) for n, s_, e, q in seg if q == mq)
            idle, cur, before = [], mk[0][1], {}
            prev_n = mk[0][2]
            for s_, e, n in mk[1:]:
                if s_ - cur >= a.gaps * 1e3:
                    idle.append((cur, s_))
                    before[(cur, s_)] = (prev_n, n)
                cur = max(cur, e)
                prev_n = n
            tot = sum(e - s_ for s_, e in idle)
            print(f"   queue {mq} idle gaps >= {a.gaps:g} us: {len(idle)}, {tot / 1e6:.2f} ms")
            for g0, g1 in idle:
                fill = collections.Counter()
                for n, s_, e, q in seg:
                    if q != mq and s_ < g1 and e > g0:
                        fill[n.split("(")[0].replace("void ", "")[:40]] += min(e, g1) - max(s_, g0)
                what = ", ".join(f"{n} {t / 1e3:.0f}us" for n, t in fill.most_common(3))
                pb, pa = (x.split("(")[0].replace("void ", "")[:40] for x in before[(g0, g1)])
                print(f"     {(g0 - t0) / 1e6:8.3f} +{(g1 - g0) / 1e3:7.1f} us | {what}\n"
                      f"              after {pb} / before {pa}")
        if a.window and k == len(ends) - 1:
            w0, w1 = (t0 + x * 1e6 for x in a.window)
            for n, s_, e, q in seg:
                if s_ < w1 and e > w0:
                    print(f"     {(s_ - t0) / 1e6:8.3f}-{(e - t0) / 1e6:8.3f}  q{q}  {n.split('(')[0].replace('void ', '')[:70]}")
        if a.tail and k == len(ends) - 1:  # the step's tail: what runs after the backward's bulk
            print(f"   last {a.tail} kernels of step {k} (ms from step start: start-end, queue):")
            for n, s_, e, q in sorted(seg, key=lambda r: r[2])[-a.tail:]:
                short = n.split("(")[0].replace("void ", "")[:56]
                print(f"     {(s_ - t0) / 1e6:8.3f}-{(e - t0) / 1e6:8.3f}  q{q}  {short}")


if __name__ == "__main__":
    main()
