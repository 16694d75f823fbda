"""Flat AdamW variants (csrc/kernels/adamw.hip: PENROZ_ADAM_NT, PENROZ_ADAM_GRID) at the GPT-2 124M and
Gemma-3 1B flat-buffer sizes; one JSON line per (n, variant). Run on the GPU box."""
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


for n in (163_087_104, 1_000_000_000):
    p, g, m, v = (torch.randn(n, device="cuda") for _ in range(4))
    v.abs_()
    sh = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    for rep in range(2):
        for nt in ("0", "1", "2"):
            for grid in ("4096", "16384", "1000000000"):
                os.environ["PENROZ_ADAM_NT"], os.environ["PENROZ_ADAM_GRID"] = nt, grid
                t = timeit(lambda: k.adamw_step(p, g, m, v, sh, 6e-4, 0.9, 0.95, 1e-8, 0.01, 10, 1.0, False))
                print(json.dumps({"n": n, "rep": rep, "nt": nt, "grid": grid, "us": round(t * 1e6, 1),
                                  "TBps": round(30 * n / t / 1e12, 2)}), flush=True)
    del p, g, m, v, sh
    torch.cuda.empty_cache()
