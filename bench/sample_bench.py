"""Microbench of the sampling kernel: B=64 rows of GPT-2's 50304-wide vocabulary.

python bench/sample_bench.py   (fp16 rows take the streaming kernel, bf16/fp32 the register one)
"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from penroz.ops._ext import kernels

K = kernels()


def t_us(fn, n=50):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


u = torch.rand(64, device="cuda")
for scale in (3.0, 0.05, 0.0):
    base = torch.randn(64, 50304, device="cuda") * scale
    for dt in (torch.bfloat16, torch.float32, torch.float16):
        lg = base.to(dt)
        r = [f"{t_us(lambda: K.sample_tokens(lg, u, T, k)):7.1f}" for T, k in ((0.0, 0), (1.0, 0), (1.0, 50))]
        print(f"scale={scale:<5} {str(dt)[6:]:9s} greedy/T=1/top50 us: {' '.join(r)}", flush=True)
