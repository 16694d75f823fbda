"""Diagnose gemm_epi wrong outputs: which (row, col) blocks are wrong / unwritten."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from penroz.ops import _ext
k = _ext.kernels()
for (M, N, K) in [(256, 256, 768), (512, 512, 768)]:
    torch.manual_seed(0)
    a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    out = torch.full((M, N), 7.0, device="cuda", dtype=torch.bfloat16)
    k.gemm_epi_bf16(a, b, None, out, None, 0)
    torch.cuda.synchronize()
    ref = a.float() @ b.float().t()
    o = out.float()
    bad = (o - ref).abs() > 0.05 * ref.abs().max()
    unw = o == 7.0
    print(f"M{M} N{N} K{K}: bad {bad.float().mean():.4f} unwritten {unw.float().mean():.4f}")
    # per 32x32 block within the 256x256 tile
    bb = bad.view(M // 32, 32, N // 32, 32).float().mean(dim=(1, 3))
    print("bad fraction per 32x32 block (rows x cols):")
    print((bb * 100).round().int().cpu().numpy())
    # per row-in-block / col pattern in first block
    r = bad[:32, :32].float()
    print("first block rows bad:", r.mean(1).cpu().numpy().round(2))
    print("first block cols bad:", r.mean(0).cpu().numpy().round(2))
    # is the output a permutation/transpose of ref?
    if bad.any():
        t = (o[:256, :256] - ref[:256, :256].t()).abs().max().item() if M >= 256 and N >= 256 else None
        print("max |out - ref^T| on first tile:", t)
        i, j = bad.nonzero()[0].tolist()
        print("first bad", i, j, o[i, j].item(), ref[i, j].item())
        # look for where ref[i,j] appears in the output row
        row = o[i]
        cand = (row - ref[i, j]).abs().argmin().item()
        print("closest value in the same output row at col", cand, row[cand].item())
