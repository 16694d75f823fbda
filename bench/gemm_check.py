"""Full-output check of the native GEMM (locates wrong tiles)."""
import os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from penroz.ops import _ext
k = _ext.kernels()
M = 65536
torch.manual_seed(0)
for (kin, nout, bias, kn) in [(768, 2304, True, False), (768, 2304, False, False), (768, 768, True, False), (768, 3072, 'gelu', False), (768, 2304, False, True), (768, 50304, False, False), (3072, 768, True, False)]:
    x = torch.rand(M, kin, device="cuda", dtype=torch.bfloat16) * 2 - 1
    w = (torch.rand(nout, kin, device="cuda", dtype=torch.bfloat16) * 2 - 1) * 0.05
    b = torch.rand(nout, device="cuda", dtype=torch.bfloat16) - 0.5 if bias else None
    for rep in range(2):
        if kn:
            dy = torch.rand(M, nout, device="cuda", dtype=torch.bfloat16) * 2 - 1
            y = torch.full((M, kin), float('nan'), device="cuda", dtype=torch.bfloat16)
            k.gemm_bf16(dy, w, True, None, y)
            ref = dy.float() @ w.float()
        else:
            y = torch.full((M, nout), float('nan'), device="cuda", dtype=torch.bfloat16)
            y2 = torch.full((M, nout), float('nan'), device="cuda", dtype=torch.bfloat16) if bias == 'gelu' else None
            k.gemm_bf16(x, w, False, b, y, y2, 0)
            ref = x.float() @ w.float().t() + (b.float() if b is not None else 0)
            if y2 is not None:
                gref = torch.nn.functional.gelu(y.float())
                print("gelu bad", int((~((y2.float() - gref).abs() <= 0.01 + 0.01 * gref.abs())).sum()), flush=True)
        torch.cuda.synchronize()
        bad = ~((y.float() - ref).abs() <= 0.02 * ref.abs().max())
        nb = int(bad.sum())
        msg = f"kin={kin} nout={nout} bias={bias} kn={kn} rep={rep} bad={nb}"
        if nb:
            idx = bad.nonzero()
            tiles = sorted({(int(r) // 256, int(c) // 256) for r, c in idx[:20000].tolist()})
            msg += f" first={idx[0].tolist()} tiles={tiles[:20]} ntiles_bad={len(tiles)}"
            sub = bad[idx[0,0]//256*256:(idx[0,0]//256+1)*256, idx[0,1]//256*256:(idx[0,1]//256+1)*256]
            msg += f" rows_bad_in_tile={int(sub.any(1).sum())} cols_bad={int(sub.any(0).sum())}"
        print(msg, flush=True)
