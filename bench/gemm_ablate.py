"""Timing ablations of the native GEMM main loop (results are garbage in ablated modes)."""
import os, sys, time, json, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from penroz.ops import _ext
k = _ext.kernels()
def timeit(fn, iters=20, warmup=5):
    for _ in range(warmup): fn()
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(iters): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t0) / iters
M = 65536
for kin, nout in [(3072, 768), (768, 50304)]:
    x = torch.rand(M, kin, device="cuda", dtype=torch.bfloat16) * 2 - 1
    w = (torch.rand(nout, kin, device="cuda", dtype=torch.bfloat16) * 2 - 1) * 0.05
    y = torch.empty(M, nout, device="cuda", dtype=torch.bfloat16)
    fl = 2 * M * kin * nout
    res = {}
    for ab in [0, 16, 8, 0, 16]:
        res[ab] = round(fl / timeit(lambda: k.gemm_bf16(x, w, False, None, y, None, 0, ab)) / 1e12, 1)
    print(json.dumps({"K": kin, "N": nout, "TF_by_ablation": res}), flush=True)
