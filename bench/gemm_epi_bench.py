"""Deferred-epilogue GEMM (csrc/kernels/gemm_epi.hip) vs hipBLASLt (TunableOp solutions, as the executor
runs it) and the gemm8 kernel, GPT-2 124M shapes at M = 65 536 tokens, random operands, interleaved
rounds in one process; median µs / TF per arm.

  fc_gelu : fc forward + GELU (library arm: addmm + the standalone GELU kernel)
  qkv / proj / fc2 / lm_head : plain forward GEMMs with bias (lm_head: none)
  fc2_dgrad / fc_dgrad : data-gradient shapes (A = dy, B = the transposed weight copy)

    python bench/gemm_epi_bench.py [--rounds 5] [--iters 20] [--flags 0]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from penroz.ops import _ext, gemm as G, activations as Ac  # noqa: E402


def timed(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--M", type=int, default=65536)
ap.add_argument("--shapes", default="fc_gelu,fc2_dgrad_dgelu,qkv,proj,fc2,fc2_dgrad,fc_dgrad,lm_head")
args = ap.parse_args()
k = _ext.kernels()
G.load_tuned_gemms()
M = args.M
SHAPES = {"fc_gelu": (768, 3072, True, True), "fc2_dgrad_dgelu": (768, 3072, False, "dgelu"), "qkv": (768, 2304, True, False), "proj": (768, 768, True, False),
          "fc2": (3072, 768, True, False), "fc2_dgrad": (768, 3072, False, False),
          "fc_dgrad": (3072, 768, False, False), "lm_head": (768, 50304, False, False)}
for name in args.shapes.split(","):
    K, N, has_bias, gelu = SHAPES[name]
    torch.manual_seed(0)
    a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    b = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
    bias = (torch.rand(N, device="cuda") - 0.5).to(torch.bfloat16) if has_bias else None
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    act = torch.empty_like(out) if gelu else None
    if gelu == "dgelu":  # fc2 dgrad through GELU': library GEMM + the GELU-backward / bias-column kernel
        pre = (torch.randn(M, N, device="cuda") * 2).to(torch.bfloat16)
        dbias = torch.zeros(N, device="cuda")
        arms = {"epi": lambda: k.gemm_epi_dgelu(a, b, pre, out, dbias, 0),
                "epi_nostore": lambda: k.gemm_epi_dgelu(a, b, pre, out, dbias, 0, 1),
                "blas": lambda: (torch.mm(a, b.t(), out=out), Ac.gelu_bwd(out, pre, "none", dbias, out=out))}
        res = {n: [] for n in arms}
        for _ in range(args.rounds):
            for n, f in arms.items():
                res[n].append(timed(f, args.iters))
        fl = 2 * M * K * N
        med = {n: statistics.median(v) for n, v in res.items()}
        print(json.dumps({"shape": name, "M": M, "K": K, "N": N,
                          **{n: {"us": round(t, 1), "TF": round(fl / t / 1e6, 1)} for n, t in med.items()},
                          "epi_vs_blas": round(med["blas"] / med["epi"], 3)}), flush=True)
        continue
    arms = {"epi": lambda: k.gemm_epi_bf16(a, b, bias, out, act, 0),
            "epi_nostore": lambda: k.gemm_epi_bf16(a, b, bias, out, act, 0, 1),
            "gemm8": lambda: k.gemm8_bf16(a, b, bias, out, act, 0, 32)}
    if gelu:
        arms["blas"] = lambda: (torch.addmm(bias, a, b.t(), out=out), Ac.gelu_fwd(out, "none", out=act))
    elif bias is not None:
        arms["blas"] = lambda: torch.addmm(bias, a, b.t(), out=out)
    else:
        arms["blas"] = lambda: torch.mm(a, b.t(), out=out)
    # numerics (sampled rows) of the native arm
    arms["epi"]()
    torch.cuda.synchronize()
    rows = torch.randint(0, M, (64,), device="cuda")
    ref = a[rows].float() @ b.float().t() + (bias.float() if bias is not None else 0)
    rel = ((out[rows].float() - ref).norm() / ref.norm()).item()
    res = {n: [] for n in arms}
    for _ in range(args.rounds):
        for n, f in arms.items():
            res[n].append(timed(f, args.iters))
    fl = 2 * M * K * N
    med = {n: statistics.median(v) for n, v in res.items()}
    print(json.dumps({"shape": name, "M": M, "K": K, "N": N, "rel_err": rel,
                      **{n: {"us": round(t, 1), "TF": round(fl / t / 1e6, 1)} for n, t in med.items()},
                      "epi_vs_blas": round(med["blas"] / med["epi"], 3)}), flush=True)
