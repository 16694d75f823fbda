"""Phase anatomy of the D = 64 dK/dV backward kernel from in-kernel s_memtime stamps (diagnostic
build path, flash_bwd_stamps): mean shader cycles per ring iteration and wave spent issuing the
next slice's DMA, issuing the S / dP MFMAs, in the softmax-gradient + dV / dK part, waiting for
the DMA and at the barrier.

    python bench/attn_stamps.py [--B 64 --T 1024 --H 12]
    PENROZ_FA_STAMP_DIAG=1 (every DMA refetches one slice: cache-hot sources) / 2 (no DMA at all):
    ablations of the stamped build only, with wrong gradients
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from penroz.ops import attention as A  # noqa: E402
from penroz.ops._ext import kernels  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=64)
ap.add_argument("--T", type=int, default=1024)
ap.add_argument("--H", type=int, default=12)
ap.add_argument("--iters", type=int, default=5)
a = ap.parse_args()
torch.manual_seed(0)
B, T, H, D = a.B, a.T, a.H, 64
qkv = torch.randn(B, T, 3 * H * D, device="cuda", dtype=torch.bfloat16)
out, lse = A.flash_fwd(qkv, H, H, D)
dout = torch.randn_like(out)
dq = torch.empty_like(qkv)
k = kernels()
buf = torch.zeros(6, dtype=torch.int64, device="cuda")
A.flash_bwd(dout, qkv, out, lse, H, H, D, dqkv=dq)  # warm
k.flash_bwd_stamps(buf)
try:
    for _ in range(a.iters):
        A.flash_bwd(dout, qkv, out, lse, H, H, D, dqkv=dq)
    torch.cuda.synchronize()
finally:
    k.flash_bwd_stamps(None)
v = buf.tolist()
n = max(1, v[5])
names = ["dma_issue", "s_dp_mfma_issue", "grads_dv_dk", "dma_wait", "barrier"]
per = {nm: round(v[i] / n, 1) for i, nm in enumerate(names)}
per["total"] = round(sum(v[:5]) / n, 1)
print(json.dumps({"B": B, "T": T, "H": H, "wave_iterations": n, "cycles_per_iteration": per}))
