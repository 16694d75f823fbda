"""Batched decode linears (csrc/kernels/decode_linear.hip) at GPT-2 124M decode shapes: µs per
launch inside a replayed graph, 12 weight copies cycled (the 12 layers: weights stream from HBM /
Infinity Cache as in a real step), with timing ablations (flags: 1 no activation reads, 2 no weight
reads, 4 no stores; LN GEMM also 8 no LayerNorm, 16 no MFMA) and hipBLASLt (torch.mm) at the same shape for reference.

    python bench/decode_linear_bench.py [--rows 64]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from penroz.ops._ext import kernels  # noqa: E402

L = 12


def timeit(fns, reps=8):
    for f in fns:
        f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            for f in fns:
                f()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / (3 * reps * len(fns)) * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=64)
    a = ap.parse_args()
    k = kernels()
    M, C = a.rows, 768
    dev = "cuda"
    if M <= 4:  # the batch-1..4 decode GEMV (decode_gemv), per GPT-2 shape and rows per wave
        resid = torch.randn(M, C, device=dev)
        gamma, beta = torch.ones(C, device=dev), torch.zeros(C, device=dev)
        for name, N, K, ln in (("qkv", 3 * C, C, True), ("fc", 4 * C, C, True), ("proj", C, C, False),
                               ("fc2", C, 4 * C, False), ("lm_head", 50304, C, True)):
            nl = 1 if name == "lm_head" else L
            ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(nl)]
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            row = {"kernel": "decode_gemv", "shape": name, "M": M, "N": N, "K": K, "ln": ln}
            for rpw in (2, 4, 8):
                if ln:
                    fns = [lambda w=w: k.decode_gemv(None, resid, None, None, None, gamma, beta, 1e-5, w, None, out, 0, rpw)
                           for w in ws]
                else:
                    fns = [lambda w=w: k.decode_gemv(x, None, None, None, None, None, None, 0.0, w, None, out, 0, rpw)
                           for w in ws]
                row[f"rpw{rpw}_us"] = round(timeit(fns), 2)
            print(json.dumps(row), flush=True)
        z = torch.zeros(1, device=dev)
        print(json.dumps({"kernel": "torch add_ (1 element)", "us": round(timeit([lambda: z.add_(1.0)] * L), 2)}))
        return
    resid = torch.randn(M, C, device=dev)
    gamma, beta = torch.ones(C, device=dev), torch.zeros(C, device=dev)
    for name, N, K in (("qkv", 3 * C, C), ("fc", 4 * C, C)):
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(L)]
        bs = [torch.zeros(N, device=dev, dtype=torch.bfloat16) for _ in range(L)]
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        y = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        row = {"kernel": "decode_ln_gemm", "shape": name, "M": M, "N": N, "K": K}
        for flags in (0, 1, 2, 4, 3, 7, 15, 23, 31):
            row[f"f{flags}_us"] = round(timeit([lambda w=w, b=b: k.decode_ln_gemm(resid, gamma, beta, 1e-5, w, b, out,
                                                                                   0, flags) for w, b in zip(ws, bs)]), 2)
        row["blas_mm_us"] = round(timeit([lambda w=w: torch.mm(y, w.t(), out=out) for w in ws]), 2)
        print(json.dumps(row), flush=True)
    for name, N, K in (("proj", C, C), ("fc2", C, 4 * C)):
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(L)]
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        r = torch.zeros(M, N, device=dev)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        row = {"kernel": "decode_gemm_acc", "shape": name, "M": M, "N": N, "K": K}
        for flags in (0, 1, 2, 4, 3, 7):
            row[f"f{flags}_us"] = round(timeit([lambda w=w: k.decode_gemm_acc(x, w, None, r, flags) for w in ws]), 2)
        row["blas_mm_us"] = round(timeit([lambda w=w: torch.mm(x, w.t(), out=out) for w in ws]), 2)
        print(json.dumps(row), flush=True)
    # an empty-ish kernel for the per-launch floor inside a graph
    z = torch.zeros(1, device=dev)
    print(json.dumps({"kernel": "torch add_ (1 element)", "us": round(timeit([lambda: z.add_(1.0)] * L), 2)}))


if __name__ == "__main__":
    main()
