"""Native 8-phase GEMM (csrc/kernels/gemm8.hip) vs hipBLASLt (TunableOp-tuned, as the executor runs it)
at the GPT-2 124M forward and dgrad shapes, M = 65 536 tokens, random operands.

    python bench/gemm8_bench.py [--iters 20]

Interleaved rounds in one process (native, library, native, ...): median TF per arm.
Forward: out[M, n_out] = x[M, k_in] · W[n_out, k_in]ᵀ (+ bias, + GELU for fc);
dgrad:   dx[M, k_in] = dy[M, n_out] · Wᵀ[k_in, n_out]ᵀ (the executor's transposed weight copy).
"""
import argparse
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from penroz.ops import _ext, gemm as G  # noqa: E402

SHAPES = {"qkv": (768, 2304), "proj": (768, 768), "fc": (768, 3072), "fc2": (3072, 768), "lm_head": (768, 50304)}


def timed(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters / 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--M", type=int, default=65536)
    args = ap.parse_args()
    k = _ext.kernels()
    G.load_tuned_gemms()
    M = args.M
    tot = {"native": 0.0, "blas": 0.0}
    for name, (kin, nout) in SHAPES.items():
        torch.manual_seed(0)
        x = (torch.rand(M, kin, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(nout, kin, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
        wt = w.t().contiguous()
        b = None if name == "lm_head" else (torch.rand(nout, device="cuda") - 0.5).to(torch.bfloat16)
        dy = (torch.rand(M, nout, device="cuda") * 2 - 1).to(torch.bfloat16)
        y = torch.empty(M, nout, device="cuda", dtype=torch.bfloat16)
        act = torch.empty_like(y) if name == "fc" else None
        dx = torch.empty(M, kin, device="cuda", dtype=torch.bfloat16)
        fl = 2 * M * kin * nout
        arms = {
            "fwd_native": lambda: k.gemm8_bf16(x, w, b, y, act, 0),
            "fwd_blas": (lambda: torch.addmm(b, x, w.t(), out=y)) if b is not None else (lambda: torch.mm(x, w.t(), out=y)),
            "dgrad_native": lambda: k.gemm8_bf16(dy, wt, None, dx),
            "dgrad_blas": lambda: torch.mm(dy, wt.t(), out=dx),  # the executor's call
        }
        if name == "fc":  # the library arm pays the standalone GELU kernel it needs
            from penroz.ops import activations as Ac
            arms["fwd_blas"] = lambda: (torch.addmm(b, x, w.t(), out=y), Ac.gelu_fwd(y, "none", out=act))
        # numerics (sampled rows)
        arms["fwd_native"]()
        arms["dgrad_native"]()
        torch.cuda.synchronize()
        rows = torch.randint(0, M, (128,), device="cuda")
        ref = x[rows].float() @ w.float().t() + (b.float() if b is not None else 0)
        ef = ((y[rows].float() - ref).norm() / ref.norm()).item()
        refd = dy[rows].float() @ w.float()
        ed = ((dx[rows].float() - refd).norm() / refd.norm()).item()
        for f in arms.values():
            f()
        res = {a: [] for a in arms}
        for _ in range(args.rounds):
            for a, f in arms.items():
                res[a].append(timed(f, args.iters))
        med = {a: statistics.median(v) for a, v in res.items()}
        out = {"shape": name, "M": M, "K_fwd": kin, "N_fwd": nout, "rel_err_fwd": ef, "rel_err_dgrad": ed}
        for a, t in med.items():
            out[a + "_us"] = round(t * 1e6, 1)
            out[a + "_TF"] = round(fl / t / 1e12, 1)
        out["fwd_speedup"] = round(med["fwd_blas"] / med["fwd_native"], 3)
        out["dgrad_speedup"] = round(med["dgrad_blas"] / med["dgrad_native"], 3)
        tot["native"] += med["fwd_native"] + med["dgrad_native"]
        tot["blas"] += med["fwd_blas"] + med["dgrad_blas"]
        print(json.dumps(out), flush=True)
    print(json.dumps({"per_layer_sum_us": {k2: round(v * 1e6, 1) for k2, v in tot.items()},
                      "speedup": round(tot["blas"] / tot["native"], 3)}), flush=True)


if __name__ == "__main__":
    main()
