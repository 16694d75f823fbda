"""Run one native GEMM shape a few times (for rocprofv3 --pmc passes).
    python bench/gemm_one.py fwd|dgrad K_IN N_OUT [iters]"""
import os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from penroz.ops import _ext
k = _ext.kernels()
mode, kin, nout = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 5
M = 65536
x = torch.rand(M, kin, device="cuda", dtype=torch.bfloat16) * 2 - 1
w = (torch.rand(nout, kin, device="cuda", dtype=torch.bfloat16) * 2 - 1) * 0.05
dy = torch.rand(M, nout, device="cuda", dtype=torch.bfloat16) * 2 - 1
y = torch.empty(M, nout, device="cuda", dtype=torch.bfloat16)
dx = torch.empty(M, kin, device="cuda", dtype=torch.bfloat16)
for _ in range(iters):
    if mode == "fwd":
        k.gemm_bf16(x, w, False, None, y)
    elif mode == "blas":
        torch.mm(x, w.t(), out=y)
    else:
        k.gemm_bf16(dy, w, True, None, dx)
torch.cuda.synchronize()
print("done")
