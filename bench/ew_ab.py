"""Streaming elementwise kernels (csrc/kernels/elementwise.hip) under PENROZ_EW_NT (non-temporal
loads / stores) x PENROZ_EW_GRID (workgroup cap) at the GPT-2 124M (B=64) and Gemma-3 1B (B=8)
step shapes; one JSON line per (kernel, variant) with the effective HBM bandwidth."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from penroz.ops import _ext  # noqa: E402

k = _ext.kernels()


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


bf = dict(device="cuda", dtype=torch.bfloat16)
x = torch.randn(65536, 3072, **bf)
y = torch.empty_like(x)
dy = torch.randn_like(x)
db = torch.empty(3072, device="cuda")
gu = torch.randn(8192, 13824, **bf)
g = torch.empty(8192, 6912, **bf)
dg = torch.randn(8192, 6912, **bf)
dgu = torch.empty_like(gu)
qkv = torch.randn(8, 1024, 1536, **bf)
qkv_out = torch.empty_like(qkv)
cosv = torch.randn(1024, 128, device="cuda")
sinv = torch.randn(1024, 128, device="cuda")
cases = {
    "rope_qkv_gemma": (lambda: k.rope_qkv(qkv, cosv, sinv, 4, 1, 256, False, qkv_out), 2 * qkv.numel() * 2),
    "gelu_fwd": (lambda: k.gelu_fwd(x, 0, y), 2 * x.numel() * 2),
    "gelu_bwd_colsum": (lambda: k.gelu_bwd(dy, x, 0, db, y), 3 * x.numel() * 2),
    "gated_packed": (lambda: k.gated_act_packed(gu, 1, g), (gu.numel() + g.numel()) * 2),
    "gated_bwd_packed": (lambda: k.gated_act_bwd_packed(dg, gu, dgu, 1), (dg.numel() + 2 * gu.numel()) * 2),
}
only = sys.argv[1:]
for rep in range(2):
    for name, (fn, nbytes) in cases.items():
        if only and name not in only:
            continue
        for nt in os.environ.get("EW_NTS", "0 1").split():
            for cap in os.environ.get("EW_CAPS", "2048 8192 1073741824").split():
                os.environ["PENROZ_EW_NT"], os.environ["PENROZ_EW_GRID"] = nt, cap
                t = timeit(fn)
                print(json.dumps({"kernel": name, "rep": rep, "nt": nt, "cap": cap, "us": round(t * 1e6, 1),
                                  "TBps": round(nbytes / t / 1e12, 2)}), flush=True)
