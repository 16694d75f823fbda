"""Forward linear GEMMs at the GPT-2 124M executor shapes (M = 65 536): hipBLASLt with the bias
epilogue (torch.addmm) vs without (torch.mm), both with the executor's tuned solution table
loaded. Decides whether the bias can move into the consuming LayerNorm / GELU kernels.

    python bench/bias_mm_probe.py [--iters 20]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from penroz.ops import gemm as gemm_ops  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    gemm_ops.load_tuned_gemms()
    M = 65536
    tot = {"addmm_ms": 0.0, "mm_ms": 0.0}
    for name, (n_out, k_in) in {"qkv": (2304, 768), "proj": (768, 768), "fc": (3072, 768), "fc2": (768, 3072)}.items():
        x = torch.randn(M, k_in, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(n_out, k_in, device="cuda", dtype=torch.bfloat16) * 0.02
        b = torch.randn(n_out, device="cuda", dtype=torch.bfloat16)
        y = torch.empty(M, n_out, device="cuda", dtype=torch.bfloat16)
        ta = timeit(lambda: torch.addmm(b, x, w.t(), out=y), a.iters)
        tm = timeit(lambda: torch.mm(x, w.t(), out=y), a.iters)
        fl = 2.0 * M * n_out * k_in
        tot["addmm_ms"] += 12 * ta * 1e3
        tot["mm_ms"] += 12 * tm * 1e3
        print(json.dumps({"shape": name, "addmm_us": round(ta * 1e6, 1), "addmm_TF": round(fl / ta / 1e12, 1),
                          "mm_us": round(tm * 1e6, 1), "mm_TF": round(fl / tm / 1e12, 1)}), flush=True)
    print(json.dumps({k: round(v, 2) for k, v in tot.items()} | {"per": "GPT-2 124M step, 12 layers"}), flush=True)


if __name__ == "__main__":
    main()
