"""A/B of the native weight-gradient kernel variants at GPT-2 124M shapes (K = 65 536 tokens),
with a correctness check of every variant against the fp32 product.

    python bench/wgrad_variants.py [--variants 4,6] [--iters 10]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from penroz.ops import _ext  # noqa: E402

SHAPES = {"qkv": (2304, 768), "proj": (768, 768), "fc": (3072, 768), "fc2": (768, 3072), "lm_head": (50304, 768),
          "lm_head_hf": (50257, 768)}
PER_STEP = {"qkv": 12, "proj": 12, "fc": 12, "fc2": 12, "lm_head": 1, "lm_head_hf": 0}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="4,6")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--tokens", type=int, default=65536)
    a = ap.parse_args()
    k = _ext.kernels()
    N = a.tokens
    vs = [int(v) for v in a.variants.split(",")]
    step = {v: 0.0 for v in vs}
    for name, (m, n) in SHAPES.items():
        torch.manual_seed(0)
        ld = (m + 7) // 8 * 8
        dyb = (torch.rand(N, ld, device="cuda") * 2 - 1).to(torch.bfloat16)
        dy = dyb[:, :m]
        x = (torch.rand(N, n, device="cuda") * 2 - 1).to(torch.bfloat16)
        ref = dy.float().t() @ x.float()
        res = {"shape": name}
        for v in vs:
            g = torch.zeros(m, n, device="cuda")
            k.wgrad_gemm(dy, x, g, 256, v)
            torch.cuda.synchronize()
            err = ((g - ref).norm() / ref.norm()).item()
            for _ in range(2):
                k.wgrad_gemm(dy, x, g, 256, v)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                k.wgrad_gemm(dy, x, g, 256, v)
            torch.cuda.synchronize()
            t = (time.perf_counter() - t0) / a.iters
            res[f"v{v}_us"] = round(t * 1e6, 1)
            res[f"v{v}_TF"] = round(2.0 * N * m * n / t / 1e12, 1)
            res[f"v{v}_err"] = float(f"{err:.2e}")
            step[v] += PER_STEP[name] * t * 1e3
            assert err < 1e-4, (name, v, err)
        print(json.dumps(res), flush=True)
        del dyb, dy, x, ref
    print(json.dumps({f"v{v}_ms_per_step": round(t, 2) for v, t in step.items()}), flush=True)


if __name__ == "__main__":
    main()
