"""Diagnostic for gemm8: the GEMM on small shapes with debug ablation bits (2: global_load_lds DMA,
4: plain stores) to localise a wrong result."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from penroz.ops import _ext  # noqa: E402

k = _ext.kernels()
torch.manual_seed(0)
for (M, N, Kd) in ((256, 256, 128), (512, 512, 256)):
    a = (torch.rand(M, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(N, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
    ref = a.float() @ b.float().t()
    for abl in (0, 2, 4, 6):
        out = torch.full((M, N), 7.0, device="cuda", dtype=torch.bfloat16)
        k.gemm8_bf16(a, b, None, out, None, 0, abl)
        bad = (out.float() - ref).abs() > 0.05 * ref.abs().max()
        print(f"gemm {M}x{N}x{Kd} ablate={abl}: bad={bad.sum().item()} of {M * N}", flush=True)
        if bad.any() and abl == 0:
            # which k-slices are missing? solve out ~ a[:, ks] @ b[:, ks]^T for each 64-slice
            o = out.float()
            for s in range(0, Kd, 32):
                part = a[:, s:s + 32].float() @ b[:, s:s + 32].float().t()
                print(f"   corr with k-slice {s}: {torch.corrcoef(torch.stack([o.flatten(), part.flatten()]))[0, 1].item():.3f}")
