"""Native forward/dgrad GEMM (csrc/kernels/gemm.hip) vs hipBLASLt at GPT-2 124M shapes.

Checks numerics against an fp32 reference on a row sample, then times both (random operands).
    python bench/gemm_bench.py [M]
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from penroz.ops import _ext  # noqa: E402


def timeit(fn, iters=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    k = _ext.kernels()
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    shapes = {"qkv": (768, 2304), "proj": (768, 768), "fc": (768, 3072), "fc2": (3072, 768), "lm_head": (768, 50304)}
    torch.manual_seed(0)
    tot = {"native_fwd": 0.0, "blas_fwd": 0.0, "native_dgrad": 0.0, "blas_dgrad": 0.0}
    for name, (kin, nout) in shapes.items():
        x = torch.rand(M, kin, device="cuda", dtype=torch.bfloat16) * 2 - 1
        w = (torch.rand(nout, kin, device="cuda", dtype=torch.bfloat16) * 2 - 1) * 0.05
        b = None if name == "lm_head" else torch.rand(nout, device="cuda", dtype=torch.bfloat16) - 0.5
        dy = torch.rand(M, nout, device="cuda", dtype=torch.bfloat16) * 2 - 1
        y = torch.empty(M, nout, device="cuda", dtype=torch.bfloat16)
        y2 = torch.empty_like(y) if name == "fc" else None
        dx = torch.empty(M, kin, device="cuda", dtype=torch.bfloat16)
        fl = 2 * M * kin * nout
        # numerics on a row sample
        k.gemm_bf16(x, w, False, b, y, y2, 0)
        k.gemm_bf16(dy, w, True, None, dx)
        torch.cuda.synchronize()
        rows = torch.randint(0, M, (256,), device="cuda")
        ref = x[rows].float() @ w.float().t() + (b.float() if b is not None else 0)
        err_f = ((y[rows].float() - ref).abs().max() / ref.abs().max()).item()
        refd = dy[rows].float() @ w.float()
        err_d = ((dx[rows].float() - refd).abs().max() / refd.abs().max()).item()
        err_g = 0.0
        if y2 is not None:
            refg = torch.nn.functional.gelu(y[rows].float())
            err_g = (y2[rows].float() - refg).abs().max().item()
        tn = timeit(lambda: k.gemm_bf16(x, w, False, b, y, y2, 0))
        if b is not None:
            tb = timeit(lambda: torch.addmm(b, x, w.t(), out=y))
        else:
            tb = timeit(lambda: torch.mm(x, w.t(), out=y))
        tnd = timeit(lambda: k.gemm_bf16(dy, w, True, None, dx))
        tbd = timeit(lambda: torch.mm(dy, w, out=dx))
        mult = 1 if name == "lm_head" else 12
        tot["native_fwd"] += tn * mult
        tot["blas_fwd"] += tb * mult
        tot["native_dgrad"] += tnd * mult
        tot["blas_dgrad"] += tbd * mult
        print(json.dumps({"shape": name, "M": M, "N": nout, "K": kin,
                          "fwd_native_TF": round(fl / tn / 1e12, 1), "fwd_blas_TF": round(fl / tb / 1e12, 1),
                          "dgrad_native_TF": round(fl / tnd / 1e12, 1), "dgrad_blas_TF": round(fl / tbd / 1e12, 1),
                          "err_fwd": err_f, "err_dgrad": err_d, "err_gelu": err_g}), flush=True)
    print(json.dumps({k2: round(v * 1e3, 2) for k2, v in tot.items()}), "ms per GPT-2 step", flush=True)


if __name__ == "__main__":
    main()
