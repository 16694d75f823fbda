"""Micro-benchmarks of the penroz HIP kernels vs their PyTorch/hipBLASLt counterparts (one MI355X).

Prints one JSON line per measurement: GPT-2 124M shapes at B=64, T=1024.
"""
import json
import math
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
from penroz.ops import _ext, attention as A

def timeit(fn, iters=10, warmup=3):
    for _ in range(warmup): fn()
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(iters): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t0) / iters

def emit(**kw): print(json.dumps(kw), flush=True)

k = _ext.kernels()
N = 65536
which = sys.argv[1:] or ["wgrad", "attn"]
if "wgrad" in which:
    for name, (m, n) in {"qkv": (2304, 768), "proj": (768, 768), "fc": (3072, 768), "fc2": (768, 3072), "lm_head": (50304, 768)}.items():
        dy = torch.randn(N, m, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(N, n, device="cuda", dtype=torch.bfloat16)
        g = torch.zeros(m, n, device="cuda")
        fl = 2 * N * m * n
        tn = timeit(lambda: k.wgrad_gemm(dy, x, g))
        tr16 = timeit(lambda: k.wgrad_gemm(dy, x, g, 256, 4))
        t128 = timeit(lambda: k.wgrad_gemm(dy, x, g, 128))
        tt = timeit(lambda: g.add_(torch.mm(dy.t(), x, out_dtype=torch.float32)))
        emit(kernel="wgrad", shape=name, native_TF=round(fl / tn / 1e12, 1), ring16_TF=round(fl / tr16 / 1e12, 1),
             native128_TF=round(fl / t128 / 1e12, 1), hipblaslt_TF=round(fl / tt / 1e12, 1),
             native_us=round(tn * 1e6, 1), hipblaslt_us=round(tt * 1e6, 1))
if "attn" in which:
    B, T, H, D = 64, 1024, 12, 64
    qkv = torch.randn(B, T, 3 * H * D, device="cuda", dtype=torch.bfloat16)
    fl = 4 * B * H * T * T * D / 2
    out, lse = A.flash_fwd(qkv, H, H, D)
    tf = timeit(lambda: A.flash_fwd(qkv, H, H, D, out=out, lse=lse))
    dout = torch.randn_like(out)
    dq = torch.empty_like(qkv)
    tb = timeit(lambda: A.flash_bwd(dout, qkv, out, lse, H, H, D, dqkv=dq))
    q, kk, v = (t.view(B, T, H, D).transpose(1, 2) for t in qkv.split(H * D, dim=2))
    ts = timeit(lambda: F.scaled_dot_product_attention(q, kk, v, is_causal=True))
    emit(kernel="flash_fwd", native_us=round(tf * 1e6, 1), native_TF=round(fl / tf / 1e12, 1),
         sdpa_us=round(ts * 1e6, 1), sdpa_TF=round(fl / ts / 1e12, 1))
    emit(kernel="flash_bwd", native_us=round(tb * 1e6, 1), native_TF=round(2.5 * fl / tb / 1e12, 1))
if "ce" in which:
    from penroz.ops import fused as Fu
    V = 50304
    logits = (torch.randn(N, V, device="cuda") * 3).to(torch.bfloat16)
    tgt = torch.randint(0, V, (N,), device="cuda")
    buf = logits.clone()
    t = timeit(lambda: Fu.cross_entropy_fwd_bwd(buf, tgt, 1.0 / N), iters=5, warmup=2)
    emit(kernel="cross_entropy", us=round(t * 1e6, 1),
         TBps=round(2 * N * V * 2 / t / 1e12, 2))
if "adam" in which:
    n = 163_087_104
    p, g, m, v = (torch.randn(n, device="cuda") for _ in range(4))
    v.abs_()
    sh = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    t = timeit(lambda: k.adamw_step(p, g, m, v, sh, 6e-4, 0.9, 0.95, 1e-8, 0.01, 10, 1.0, False))
    emit(kernel="adamw_flat", n=n, us=round(t * 1e6, 1), TBps=round(30 * n / t / 1e12, 2))
    t = timeit(lambda: p.copy_(g))  # the same kind of traffic: 1 read + 1 write stream of fp32
    emit(kernel="torch_copy_fp32", n=n, us=round(t * 1e6, 1), TBps=round(8 * n / t / 1e12, 2))
if "stream" in which:
    # memory-bound streams at the fc activation shape [65536, 3072] bf16: GELU forward (read +
    # write), GELU backward fused with the fc bias-gradient column sum (2 reads + 1 write), the
    # plain column sum (1 read) — effective TB/s against a torch copy of the same bytes
    F_ = 3072
    x = torch.randn(N, F_, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(N, F_, device="cuda", dtype=torch.bfloat16)
    y = torch.empty_like(x)
    db = torch.zeros(F_, device="cuda")
    nb = x.numel() * 2
    t = timeit(lambda: k.gelu_fwd(x, 0, y), 20)
    emit(kernel="gelu_fwd", us=round(t * 1e6, 1), TBps=round(2 * nb / t / 1e12, 2))
    t = timeit(lambda: k.gelu_bwd(dy, x, 0, db, y), 20)
    emit(kernel="gelu_bwd_colsum", us=round(t * 1e6, 1), TBps=round(3 * nb / t / 1e12, 2))
    t = timeit(lambda: k.colsum(dy, db), 20)
    emit(kernel="colsum", us=round(t * 1e6, 1), TBps=round(nb / t / 1e12, 2))
    t = timeit(lambda: y.copy_(x), 20)
    emit(kernel="torch_copy", us=round(t * 1e6, 1), TBps=round(2 * nb / t / 1e12, 2))
