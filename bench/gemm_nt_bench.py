"""Native NT GEMM (csrc/kernels/gemm_nt.hip) vs hipBLASLt (torch.addmm / mm with the shipped
TunableOp table, what the executors run) at the GPT-2 124M headline shapes, M = 65 536 tokens.
Interleaved rounds in one process, random operands; median µs and TF per shape, one JSON line per
shape. ``fc_gelu`` compares the fused bias + GELU epilogue with addmm + the HIP GELU kernel.

    python bench/gemm_nt_bench.py [--rounds 5] [--iters 10] [--shapes qkv,fc_gelu] [--grid G] [--group-m 8]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from penroz.ops import _ext  # noqa: E402
from penroz.ops import gemm as gemm_ops  # noqa: E402
from penroz.ops import activations as act_ops  # noqa: E402

M = 65536
# name: (N, K, bias, gelu)
SHAPES = {
    "qkv": (2304, 768, True, False), "proj": (768, 768, True, False), "fc_gelu": (3072, 768, True, True),
    "fc": (3072, 768, True, False), "fc2": (768, 3072, True, False), "fc2_dgrad": (3072, 768, False, False),
    "fc_dgrad": (768, 3072, False, False), "qkv_dgrad": (768, 2304, False, False),
    "proj_dgrad": (768, 768, False, False), "lm_head": (50304, 768, False, False),
    "lm_head_dgrad": (768, 50304, False, False),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--grid", type=int, default=0)
    ap.add_argument("--group-m", type=int, default=0)
    ap.add_argument("--arms", default="0", help="comma-separated native ablate values (bit 0: no stores, "
                    "bit 1: waves 4-7 at priority 1)")
    ap.add_argument("--groups", default="", help="comma-separated group_m values to compare (native, ablate 0)")
    args = ap.parse_args()
    k = _ext.kernels()
    gemm_ops.load_tuned_gemms()
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    for name in args.shapes.split(","):
        N, K, has_bias, gelu = SHAPES[name]
        a = torch.rand(M, K, device=dev, generator=g).sub_(0.5).to(torch.bfloat16)
        b = torch.rand(N, K, device=dev, generator=g).sub_(0.5).div_(K ** 0.5).to(torch.bfloat16)
        bias = torch.randn(N, device=dev, generator=g).to(torch.bfloat16) if has_bias else None
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        act = torch.empty_like(out) if gelu else None
        out2 = torch.empty_like(out)
        act2 = torch.empty_like(out) if gelu else None

        def native_arm(abl, gm):
            return lambda: k.gemm_nt(a, b, bias, out, act, 0, gm, args.grid, abl)

        def blas():
            if bias is not None:
                torch.addmm(bias, a, b.t(), out=out2)
            else:
                torch.mm(a, b.t(), out=out2)
            if gelu:
                act_ops.gelu_fwd(out2, "none", out=act2)

        arms = {"blas": blas}
        for abl in args.arms.split(","):
            arms["native" if abl == "0" else f"native_a{abl}"] = native_arm(int(abl), args.group_m)
        for gm in filter(None, args.groups.split(",")):
            arms[f"native_g{gm}"] = native_arm(0, int(gm))
        native = arms["native"] if "native" in arms else next(iter(arms.values()))
        times = {n: [] for n in arms}
        for f in arms.values():
            f()
        torch.cuda.synchronize()
        for _ in range(args.rounds):
            for n, f in arms.items():
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(args.iters):
                    f()
                e.record()
                e.synchronize()
                times[n].append(s.elapsed_time(e) * 1e3 / args.iters)
        native()
        blas()
        torch.cuda.synchronize()
        err = ((out.float() - out2.float()).norm() / out2.float().norm()).item()
        flop = 2.0 * M * N * K
        rec = {"shape": name, "M": M, "N": N, "K": K, "bias": has_bias, "gelu": gelu, "rel_err_vs_blas": round(err, 5)}
        for n, ts in times.items():
            med = statistics.median(ts)
            rec[f"{n}_us"] = round(med, 1)
            rec[f"{n}_tf"] = round(flop / med / 1e6, 1)
        rec["speedup"] = round(rec["blas_us"] / rec["native_us"], 3)
        print(json.dumps(rec), flush=True)
        del a, b, out, out2, act, act2


if __name__ == "__main__":
    main()
