"""One-off GPU environment probe: GEMM/SDPA throughput at GPT-2 shapes and API support.

Run on the MI355X box: ``python bench/probe_env.py``. Prints one line per measurement.
"""
import json
import time

import torch
import torch.nn.functional as F


def timeit(fn, iters=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    dev = "cuda"
    props = torch.cuda.get_device_properties(0)
    print(json.dumps({"device": props.name, "gcn": getattr(props, "gcnArchName", None),
                      "cus": props.multi_processor_count, "mem_gb": props.total_memory / 2**30}))
    N, C, V = 64 * 1024, 768, 50304
    x = torch.randn(N, C, device=dev, dtype=torch.bfloat16)
    res = {}
    for name, (m, k, n) in {"qkv": (N, C, 3 * C), "proj": (N, C, C), "fc": (N, C, 4 * C),
                            "fc2": (N, 4 * C, C), "lm_head": (N, C, V)}.items():
        a = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
        w = torch.randn(n, k, device=dev, dtype=torch.bfloat16)
        b = torch.randn(n, device=dev, dtype=torch.bfloat16)
        t = timeit(lambda: torch.addmm(b, a, w.t()))
        res[f"fwd_{name}_TF"] = 2 * m * k * n / t / 1e12
        g = torch.randn(m, n, device=dev, dtype=torch.bfloat16)
        t = timeit(lambda: torch.mm(g, w))
        res[f"dgrad_{name}_TF"] = 2 * m * k * n / t / 1e12
        t = timeit(lambda: torch.mm(g.t(), a))
        res[f"wgrad_{name}_TF"] = 2 * m * k * n / t / 1e12
        try:
            t = timeit(lambda: torch.mm(g.t(), a, out_dtype=torch.float32))
            res[f"wgrad_f32out_{name}_TF"] = 2 * m * k * n / t / 1e12
        except Exception as e:
            res[f"wgrad_f32out_{name}"] = repr(e)[:200]
        del a, w, b, g
    print(json.dumps(res))
    # SDPA causal at GPT-2 shapes
    B, H, T, D = 64, 12, 1024, 64
    q = torch.randn(B, H, T, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn_like(q, requires_grad=True)
    v = torch.randn_like(q, requires_grad=True)
    flops = 4 * B * H * T * T * D / 2
    t = timeit(lambda: F.scaled_dot_product_attention(q, k, v, is_causal=True))
    o = F.scaled_dot_product_attention(q, k, v, is_causal=True)
    do = torch.randn_like(o)
    tb = timeit(lambda: torch.autograd.grad(F.scaled_dot_product_attention(q, k, v, is_causal=True),
                                            (q, k, v), do))
    print(json.dumps({"sdpa_fwd_ms": t * 1e3, "sdpa_fwd_TF": flops / t / 1e12,
                      "sdpa_fwdbwd_ms": tb * 1e3, "sdpa_bwd_TF": 2.5 * flops / (tb - t) / 1e12}))
    # memory-bound reference: LayerNorm fp32 [N, C]
    xf = torch.randn(N, C, device=dev)
    ln = torch.nn.LayerNorm(C).to(dev)
    t = timeit(lambda: ln(xf))
    print(json.dumps({"ln_fwd_ms": t * 1e3, "ln_GBps": N * C * 8 / t / 1e9}))
    big = torch.empty(2**28, device=dev)
    t = timeit(lambda: big.mul_(1.0001))
    print(json.dumps({"stream_mul_TBps": 2 * big.numel() * 4 / t / 1e12}))


if __name__ == "__main__":
    main()
