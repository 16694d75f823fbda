"""Flash-attention microbenchmark for profiling (GPT-2 124M attention shape by default).

    python bench/attn_bench.py [--iters 20] [--B 64 --T 1024 --H 12 --D 64] [--which fwd,bwd]

Prints per-call time and TFLOP/s (causal FLOPs: fwd 2 GEMMs, bwd 2.5× fwd) for the native
kernels and for torch SDPA. Meant to run under ``rocprofv3 --pmc ... -- python3 bench/attn_bench.py``.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from penroz.ops import attention as A  # noqa: E402


def timeit(fn, iters):
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
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--H", type=int, default=12)
    ap.add_argument("--Hkv", type=int, default=0)
    ap.add_argument("--D", type=int, default=64)
    ap.add_argument("--which", default="fwd,bwd")
    ap.add_argument("--sdpa", action="store_true")
    ap.add_argument("--p", type=float, default=0.0, help="attention dropout probability")
    a = ap.parse_args()
    B, T, H, D = a.B, a.T, a.H, a.D
    Hkv = a.Hkv or H
    torch.manual_seed(0)
    qkv = torch.randn(B, T, (H + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    fl = 4.0 * B * H * T * T * D / 2
    res = {"B": B, "T": T, "H": H, "Hkv": Hkv, "D": D, "p": a.p}
    out, lse = A.flash_fwd(qkv, H, Hkv, D, a.p, 7)
    if "fwd" in a.which:
        from penroz.ops._ext import kernels
        k = kernels()
        variants = [1, 3] if (hasattr(k, "flash_fwd_variant") and D == 64) else [0]
        for v in variants:
            if v:
                prev = k.flash_fwd_variant(v)
            t = timeit(lambda: A.flash_fwd(qkv, H, Hkv, D, a.p, 7, out=out, lse=lse), a.iters)
            sfx = f"_v{v}" if v else ""
            res.update({f"fwd{sfx}_us": round(t * 1e6, 1), f"fwd{sfx}_TF": round(fl / t / 1e12, 1)})
            if v:
                k.flash_fwd_variant(prev)
    if "bwd" in a.which:
        from penroz.ops._ext import kernels
        k = kernels()
        dout = torch.randn_like(out)
        dq = torch.empty_like(qkv)
        t = timeit(lambda: A.flash_bwd(dout, qkv, out, lse, H, Hkv, D, a.p, 7, dqkv=dq), a.iters)
        res.update({"bwd_us": round(t * 1e6, 1), "bwd_TF": round(2.5 * fl / t / 1e12, 1)})
    if a.sdpa:
        q, k, v = qkv.split([H * D, Hkv * D, Hkv * D], dim=2)
        q = q.reshape(B, T, H, D).transpose(1, 2).detach().requires_grad_()
        k = k.reshape(B, T, Hkv, D).transpose(1, 2).detach().requires_grad_()
        v = v.reshape(B, T, Hkv, D).transpose(1, 2).detach().requires_grad_()
        gqa = Hkv != H
        t = timeit(lambda: F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=gqa), a.iters)
        res.update(sdpa_fwd_us=round(t * 1e6, 1), sdpa_fwd_TF=round(fl / t / 1e12, 1))
        o = F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=gqa)
        go = torch.randn_like(o)
        t = timeit(lambda: torch.autograd.grad(o, (q, k, v), go, retain_graph=True), a.iters)
        res.update(sdpa_bwd_us=round(t * 1e6, 1), sdpa_bwd_TF=round(2.5 * fl / t / 1e12, 1))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
