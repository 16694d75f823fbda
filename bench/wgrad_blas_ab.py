"""Weight-gradient GEMM A/B at the GPT-2 124M (or ``--model gpt2-xl``) shapes (M = 65 536 tokens): the native kernel
(``wgrad_gemm``) vs hipBLASLt through ``torch.addmm(g, dy.t(), x, out_dtype=float32)`` with
the fp32 gradient accumulated in place (beta = 1). Run with PYTORCH_TUNABLEOP_ENABLED=1
PYTORCH_TUNABLEOP_TUNING=1 to let TunableOp search hipBLASLt/rocBLAS solutions for the library
side. One JSON line per shape.

    python bench/wgrad_blas_ab.py [--iters 10]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from penroz.ops import _ext  # noqa: E402

def shapes(C: int, L: int, V: int = 50304) -> tuple[dict, dict]:
    """(out, in) of every weight gradient of a GPT-2 layout of width C, and calls per step."""
    sh = {"qkv": (3 * C, C), "proj": (C, C), "fc": (4 * C, C), "fc2": (C, 4 * C), "lm_head": (V, C)}
    return sh, {"qkv": L, "proj": L, "fc": L, "fc2": L, "lm_head": 1}


MODELS = {"gpt2-124m": (768, 12), "gpt2-xl": (1600, 48)}


def timeit(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--tokens", type=int, default=65536)
    ap.add_argument("--model", default="gpt2-124m", choices=list(MODELS))
    a = ap.parse_args()
    SHAPES, per_layer = shapes(*MODELS[a.model])
    N = a.tokens
    k = _ext.kernels()
    tot = {"native_ms": 0.0, "blas_ms": 0.0}
    for name, (m, n) in SHAPES.items():
        torch.manual_seed(0)
        dy = (torch.rand(N, m, device="cuda") * 2 - 1).to(torch.bfloat16)
        x = (torch.rand(N, n, device="cuda") * 2 - 1).to(torch.bfloat16)
        g1 = torch.zeros(m, n, device="cuda")
        g2 = torch.zeros(m, n, device="cuda")
        k.wgrad_gemm(dy, x, g1)
        torch.addmm(g2, dy.t(), x, out_dtype=torch.float32, out=g2)
        torch.cuda.synchronize()
        err = ((g1 - g2).norm() / g2.norm()).item()
        tn = timeit(lambda: k.wgrad_gemm(dy, x, g1), a.iters)
        tb = timeit(lambda: torch.addmm(g2, dy.t(), x, out_dtype=torch.float32, out=g2), a.iters)
        wb = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        t16 = timeit(lambda: torch.mm(dy.t(), x, out=wb), a.iters)
        t16a = timeit(lambda: g2.add_(torch.mm(dy.t(), x, out=wb)), a.iters)
        fl = 2.0 * N * m * n
        tot["native_ms"] += per_layer[name] * tn * 1e3
        tot["blas_ms"] += per_layer[name] * tb * 1e3
        tot["blas_bf16out_add_ms"] = tot.get("blas_bf16out_add_ms", 0.0) + per_layer[name] * t16a * 1e3
        print(json.dumps({"shape": name, "native_us": round(tn * 1e6, 1), "native_TF": round(fl / tn / 1e12, 1),
                          "blas_us": round(tb * 1e6, 1), "blas_TF": round(fl / tb / 1e12, 1), "rel_err": err,
                          "blas_bf16out_us": round(t16 * 1e6, 1), "blas_bf16out_TF": round(fl / t16 / 1e12, 1),
                          "blas_bf16out_plus_add_us": round(t16a * 1e6, 1)}),
              flush=True)
        del dy, x, g1, g2, wb
    print(json.dumps({k2: round(v, 2) for k2, v in tot.items()} | {"per": f"{a.model} step"}), flush=True)


if __name__ == "__main__":
    main()
