"""gemm8 timing ablations (results wrong in ablated modes): 1 = epilogue without global stores.
Interleaved rounds, median, GPT-2 K=768 shapes."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from penroz.ops import _ext  # noqa: E402

k = _ext.kernels()
M = 65536


def timed(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


for name, (K, N) in {"qkv_fwd": (768, 2304), "fc2_dgrad": (768, 3072), "lm_head_fwd": (768, 50304),
                     "fc_dgrad": (3072, 768)}.items():
    a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    res = {0: [], 1: [], "blas": []}
    for _ in range(5):
        for abl in (0, 1):
            res[abl].append(timed(lambda: k.gemm8_bf16(a, b, None, out, None, 0, abl)))
        res["blas"].append(timed(lambda: torch.mm(a, b.t(), out=out)))
    fl = 2 * M * K * N
    print(name, {str(kk): (round(statistics.median(v), 1), round(fl / statistics.median(v) / 1e6, 1))
                 for kk, v in res.items()}, flush=True)
