"""gemm8 timing ablations (results wrong in ablated modes), interleaved rounds, median µs / TF, GPT-2 shapes.

ablate bits: 1 = epilogue without global stores; 4 = one workgroup per tile instead of one persistent
workgroup per CU (the dispatcher refills CUs as tiles finish); 8 = GELU epilogue with the branch-free
A&S erf; (ablate >> 4) & 3 = store cache policy (0 plain, 1 sc0, 2 nt, 3 sc0|nt); ablate >> 8 = odd
workgroups start that many `s_sleep 127` late (de-synchronised epilogues).

    python bench/gemm8_ablate.py [--arms 0,1,32,256,768]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from penroz.ops import _ext, gemm as G  # noqa: E402

k = _ext.kernels()
M = 65536


def timed(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


ap = argparse.ArgumentParser()
ap.add_argument("--arms", default="0,1,4,8,12,32,512,768,1024")
ap.add_argument("--rounds", type=int, default=5)
args = ap.parse_args()
arms = [int(a) for a in args.arms.split(",")]
G.load_tuned_gemms()
for name, (K, N, gelu) in {"qkv_fwd": (768, 2304, False), "fc_fwd_gelu": (768, 3072, True),
                           "fc2_dgrad": (768, 3072, False), "fc_dgrad": (3072, 768, False)}.items():
    a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    bias = (torch.rand(N, device="cuda") - 0.5).to(torch.bfloat16) if gelu else None
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    act = torch.empty_like(out) if gelu else None
    res = {str(x): [] for x in arms}
    res["blas"] = []
    for _ in range(args.rounds):
        for abl in arms:
            res[str(abl)].append(timed(lambda: k.gemm8_bf16(a, b, bias, out, act, 0, abl)))
        if gelu:
            from penroz.ops import activations as Ac
            res["blas"].append(timed(lambda: (torch.addmm(bias, a, b.t(), out=out), Ac.gelu_fwd(out, "none", out=act))))
        else:
            res["blas"].append(timed(lambda: torch.mm(a, b.t(), out=out)))
    fl = 2 * M * K * N
    print(name, {kk: (round(statistics.median(v), 1), round(fl / statistics.median(v) / 1e6, 1))
                 for kk, v in res.items()}, flush=True)
