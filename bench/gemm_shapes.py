"""Forward / data-gradient GEMMs of a fused executor step, one by one: hipBLASLt as the executor
calls it (TunableOp-tuned table loaded), median of interleaved rounds, TF per call and ms per step.

    python bench/gemm_shapes.py [--model gemma3-1b|gpt2] [--tokens N] [--iters 10]

fwd:   out[T, n] = x[T, k] · W[n, k]ᵀ
dgrad: dx[T, k] = dy[T, n] · W[n, k]   (W read through the executor's transposed copy Wᵀ[k, n])
"""
import argparse
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from penroz.ops import gemm as G  # noqa: E402

# (k = in_features, n = out_features, calls per step)
MODELS = {
    "gemma3-1b": {"tokens": 8192, "shapes": {"qkv": (1152, 1536, 26), "o": (1024, 1152, 26),
                                             "gate_up": (1152, 13824, 26), "down": (6912, 1152, 26),
                                             "lm_head": (1152, 262144, 1)}},
    "gpt2": {"tokens": 65536, "shapes": {"qkv": (768, 2304, 12), "proj": (768, 768, 12), "fc": (768, 3072, 12),
                                        "fc2": (3072, 768, 12), "lm_head": (768, 50304, 1)}},
}


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
    ap.add_argument("--model", default="gemma3-1b", choices=sorted(MODELS))
    ap.add_argument("--tokens", type=int, default=None)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    cfg = MODELS[a.model]
    T = a.tokens or cfg["tokens"]
    G.load_tuned_gemms()
    step = {"blas": 0.0}
    for name, (kin, nout, per_step) in cfg["shapes"].items():
        torch.manual_seed(0)
        x = (torch.rand(T, kin, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(nout, kin, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
        wt = w.t().contiguous()
        dy = (torch.rand(T, nout, device="cuda") * 2 - 1).to(torch.bfloat16)
        y = torch.empty(T, nout, device="cuda", dtype=torch.bfloat16)
        dx = torch.empty(T, kin, device="cuda", dtype=torch.bfloat16)
        arms = {"fwd_blas": lambda: torch.mm(x, w.t(), out=y),
                "dgrad_blas": lambda: torch.mm(dy, wt.t(), out=dx)}
        res = {k: [] for k in arms}
        for _ in range(a.rounds):
            for k, fn in arms.items():
                fn()
                res[k].append(timed(fn, a.iters))
        fl = 2.0 * T * kin * nout
        row = {"shape": name, "T": T, "k": kin, "n": nout}
        for k, v in res.items():
            t = statistics.median(v)
            row[k + "_us"] = round(t * 1e6, 1)
            row[k + "_TF"] = round(fl / t / 1e12, 1)
        for d in ("fwd", "dgrad"):
            step["blas"] += row[f"{d}_blas_us"] * per_step / 1e3
        print(json.dumps(row), flush=True)
    print(json.dumps({"ms_per_step": {k: round(v, 2) for k, v in step.items()}}), flush=True)


if __name__ == "__main__":
    main()
