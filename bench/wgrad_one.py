"""Run the native wgrad kernel (default variant) a few times on one GPT-2 124M shape — a
target for rocprofv3 --pmc passes (bench/gpu_pmc_wgrad.sh).  python bench/wgrad_one.py lm_head"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from penroz.ops import _ext  # noqa: E402

SHAPES = {"qkv": (2304, 768), "proj": (768, 768), "fc": (3072, 768), "fc2": (768, 3072), "lm_head": (50304, 768)}
m, n = SHAPES[sys.argv[1] if len(sys.argv) > 1 else "lm_head"]
N = 65536
dy = (torch.rand(N, m, device="cuda") * 2 - 1).to(torch.bfloat16)
x = (torch.rand(N, n, device="cuda") * 2 - 1).to(torch.bfloat16)
g = torch.zeros(m, n, device="cuda")
for _ in range(3):
    _ext.kernels().wgrad_gemm(dy, x, g)
torch.cuda.synchronize()
