"""Gradient all-reduce sweep over RCCL / xGMI: bucket size × wire dtype × transport.

    python bench/allreduce_bench.py --gpus 8 [--sizes-mb 1,4,16,25,64,128,256] [--wires fp32,bf16]
    python bench/allreduce_bench.py --gpus 2 --device cpu          # gloo plumbing rehearsal

Like ``bench.py`` it launches one rank per GPU itself (parent never touches the GPU) unless a
launcher already set ``WORLD_SIZE``. Each point: W warm-up + K timed in-place AVG all-reduces of
one bucket, bracketed by barrier + synchronize, max over ranks. Reported per point:
``ms``, ``algbw_GBps`` = bucket bytes / time, ``busbw_GBps`` = algbw · 2(n-1)/n (the per-rank
link traffic of a ring; compare against 7 xGMI links × ≈153 GB/s per MI355X).
Transports: ``c10d`` (torch ProcessGroupNCCL = RCCL) and ``native`` (``csrc/comm/rccl_comm.cpp``).
Also prints the bucket plan the executor would use for GPT-2 124M (652 MB of fp32 gradients)
and GPT-2 XL (6.55 GB) at the default bucket size, so the sweep can be read against it.
Rank 0 prints one JSON line per point and a summary line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def gpt2_segments(C: int, L: int, V: int = 50304, P: int = 1024) -> list[tuple[int, int]]:
    """Element ranges of the executor's flat gradient layout (backward order: head, blocks, embeddings)."""
    sizes = [[V * C + 2 * C]] + [[4 * C * C + C + 4 * C * C + 4 * C + 2 * C + C * C + C + 3 * C * C + 3 * C + 2 * C]
                                 for _ in range(L)] + [[P * C + V * C]]
    segs, off = [], 0
    for s in sizes:
        n = sum(s)
        segs.append((off, off + n))
        off += n
    return segs


def plan_summary(bucket_mb: float) -> dict:
    from penroz.parallel.reducer import plan_buckets
    out = {}
    for name, (C, L) in {"gpt2-124m": (768, 12), "gpt2-xl": (1600, 48)}.items():
        b = plan_buckets(gpt2_segments(C, L), bucket_mb * 2**20)
        mb = [(e - s) * 4 / 2**20 for s, e in b]
        out[name] = {"grad_mb": round(sum(mb), 1), "buckets": len(b), "min_mb": round(min(mb), 1),
                     "max_mb": round(max(mb), 1)}
    return out


def run_rank(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.device == "cuda":
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)
    else:
        dev = torch.device("cpu")
        dist.init_process_group("gloo", rank=rank, world_size=world)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    native = None
    transports = [t for t in args.transports.split(",") if t]
    if "native" in transports and dev.type == "cuda":
        from penroz.parallel.rccl import NativeComm
        native = NativeComm.get()
    results = []
    for wire in args.wires.split(","):
        dt = {"fp32": torch.float32, "bf16": torch.bfloat16}[wire]
        for mb in [float(x) for x in args.sizes_mb.split(",")]:
            n = int(mb * 2**20) // 4  # elements of the fp32 gradient bucket
            buf = torch.ones(n, device=dev, dtype=dt)
            for tr in transports:
                if tr == "native" and native is None:
                    continue

                def one():
                    if tr == "native":
                        native.all_reduce_avg_async(buf)
                        native.wait_all()
                    elif dev.type == "cuda":
                        dist.all_reduce(buf, op=dist.ReduceOp.AVG)
                    else:
                        dist.all_reduce(buf)
                for _ in range(args.warmup):
                    one()
                sync()
                dist.barrier()
                t0 = time.perf_counter()
                for _ in range(args.iters):
                    one()
                sync()
                dist.barrier()
                dt_s = torch.tensor([(time.perf_counter() - t0) / args.iters], dtype=torch.float64,
                                    device=dev if dev.type == "cuda" else "cpu")
                dist.all_reduce(dt_s, op=dist.ReduceOp.MAX)
                t = float(dt_s.item())
                nbytes = buf.numel() * buf.element_size()
                alg = nbytes / t / 1e9
                res = {"transport": tr, "wire": wire, "grad_bucket_mb": mb, "wire_mb": round(nbytes / 2**20, 2),
                       "ms": t * 1e3, "algbw_GBps": alg, "busbw_GBps": alg * 2 * (world - 1) / world if world > 1 else 0.0,
                       "n_ranks": world}
                results.append(res)
                if rank == 0:
                    print(json.dumps(res), flush=True)
            del buf
    if rank == 0:
        best = max(results, key=lambda r: r["busbw_GBps"]) if results else None
        ver = None
        if dev.type == "cuda":
            try:
                v = torch.cuda.nccl.version()
                ver = ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
            except Exception:
                pass
        print(json.dumps({"summary": True, "n_ranks": world, "rccl_version": ver, "best": best,
                          "bucket_plan_default": plan_summary(args.bucket_mb)}), flush=True)
    dist.destroy_process_group()


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    ap.add_argument("--sizes-mb", default="1,4,16,25,64,128,256")
    ap.add_argument("--wires", default="fp32,bf16")
    ap.add_argument("--transports", default="c10d,native")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--bucket-mb", type=float, default=float(os.environ.get("PENROZ_BUCKET_MB", "64")))
    args = ap.parse_args(argv)
    if "WORLD_SIZE" not in os.environ:
        import bench  # the same supervised self-launch as the headline benchmark
        if args.gpus > 1 or args.device == "cpu":
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.gpus > 1:
            sys.exit(bench.launch_ranks(args, argv, script=os.path.abspath(__file__)))
        os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(bench._free_port()))
    run_rank(args)


if __name__ == "__main__":
    main()
