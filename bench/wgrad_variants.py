"""A/B of the native weight-gradient kernel variants against hipBLASLt (torch.mm with an fp32
output: into a temporary + add, or straight into a zero gradient) at GPT-2 124M (K = 65 536
tokens) or Gemma-3 1B shapes, with a correctness check of every variant against the fp32 product.

    python bench/wgrad_variants.py [--model gpt2|gemma3-1b] [--tokens N] [--variants 4,6] [--iters 10] [--blas]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from penroz.ops import _ext  # noqa: E402

MODELS = {
    "gpt2": ({"qkv": (2304, 768), "proj": (768, 768), "fc": (3072, 768), "fc2": (768, 3072), "lm_head": (50304, 768),
              "lm_head_hf": (50257, 768)},
             {"qkv": 12, "proj": 12, "fc": 12, "fc2": 12, "lm_head": 1, "lm_head_hf": 0}),
    "gemma3-1b": ({"qkv": (1536, 1152), "o": (1152, 1024), "gate_up": (13824, 1152), "down": (1152, 6912),
                   "lm_head": (262144, 1152)},
                  {"qkv": 26, "o": 26, "gate_up": 26, "down": 26, "lm_head": 1}),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="4,6")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--tokens", type=int, default=65536)
    ap.add_argument("--model", default="gpt2", choices=sorted(MODELS))
    ap.add_argument("--blas", action="store_true", help="also time torch.mm (hipBLASLt) with an fp32 output")
    a = ap.parse_args()
    SHAPES, PER_STEP = MODELS[a.model]
    k = _ext.kernels()
    N = a.tokens
    vs = [int(v) for v in a.variants.split(",")]
    step = {v: 0.0 for v in vs}
    if a.blas:
        step.update({"blas_tmp_add": 0.0, "blas_direct": 0.0})
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
        if a.blas:
            g = torch.zeros(m, n, device="cuda")
            fns = {"blas_tmp_add": lambda: g.add_(torch.mm(dy.t(), x, out_dtype=torch.float32)),
                   "blas_direct": lambda: torch.mm(dy.t(), x, out_dtype=torch.float32, out=g)}
            for key, fn in fns.items():
                for _ in range(2):
                    fn()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.iters):
                    fn()
                torch.cuda.synchronize()
                t = (time.perf_counter() - t0) / a.iters
                res[f"{key}_us"] = round(t * 1e6, 1)
                res[f"{key}_TF"] = round(2.0 * N * m * n / t / 1e12, 1)
                step[key] += PER_STEP[name] * t * 1e3
        print(json.dumps(res), flush=True)
        del dyb, dy, x, ref
    print(json.dumps({f"{v if isinstance(v, str) else 'v%d' % v}_ms_per_step": round(t, 2) for v, t in step.items()}),
          flush=True)


if __name__ == "__main__":
    main()
