"""Decode-shaped GEMM microbenchmark: native skinny GEMM vs torch (hipBLASLt) per weight shape
at M = 1 / 8 / 64 rows, reported as µs and effective weight-read bandwidth (TB/s).

    python bench/skinny_bench.py [--model gemma3-1b|gpt2] [--rows 1,8,64]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from penroz.ops import gemm as G  # noqa: E402

SHAPES = {
    "gemma3-1b": {"qkv": (1536, 1152), "o": (1152, 1024), "gate_up": (13824, 1152), "down": (1152, 6912),
                  "head": (262144, 1152)},
    "gpt2": {"qkv": (2304, 768), "proj": (768, 768), "fc": (3072, 768), "fc2": (768, 3072), "head": (50304, 768)},
}


def timeit(fn, iters=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gemma3-1b")
    ap.add_argument("--rows", default="1,8,64")
    a = ap.parse_args()
    ws, cnt = G.skinny_workspace(torch.device("cuda"))
    from penroz.ops._ext import kernels
    k = kernels()
    for name, (n, kk) in SHAPES[a.model].items():
        w = torch.randn(n, kk, device="cuda", dtype=torch.bfloat16) * 0.02
        for m in [int(r) for r in a.rows.split(",")]:
            x = torch.randn(m, kk, device="cuda", dtype=torch.bfloat16)
            out = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
            ref = (x.float() @ w.float().t())
            k.skinny_gemm(x, w, None, out, ws, cnt, 0)
            torch.cuda.synchronize()
            err = ((out.float() - ref).norm() / ref.norm()).item()
            tn = timeit(lambda: k.skinny_gemm(x, w, None, out, ws, cnt, 0))
            tb = timeit(lambda: torch.mm(x, w.t(), out=out))
            gb = n * kk * 2 / 1e9
            print(json.dumps({"shape": name, "N": n, "K": kk, "M": m, "native_us": round(tn * 1e6, 2),
                              "native_TBps": round(gb / tn / 1e3, 2), "blas_us": round(tb * 1e6, 2),
                              "blas_TBps": round(gb / tb / 1e3, 2), "rel_err": float(f"{err:.2e}")}), flush=True)
        del w


if __name__ == "__main__":
    main()
