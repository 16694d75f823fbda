"""Probe wgrad GEMM variants at GPT-2 shapes (N = 65536 tokens) on one MI355X."""
import json, os, sys, time
import torch

def timeit(fn, iters=10, warmup=3):
    for _ in range(warmup): fn()
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(iters): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t0) / iters

N = 65536
shapes = {"qkv": (768, 2304), "proj": (768, 768), "fc": (768, 3072), "fc2": (3072, 768), "lm_head": (768, 50304)}
res = {}
for name, (k_in, n_out) in shapes.items():
    x = torch.randn(N, k_in, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(N, n_out, device="cuda", dtype=torch.bfloat16)
    fl = 2 * N * k_in * n_out
    out = torch.empty(n_out, k_in, device="cuda")
    v = {}
    v["mm_bf16"] = timeit(lambda: torch.mm(dy.t(), x))
    v["mm_f32out"] = timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
    v["mmT_bf16"] = timeit(lambda: torch.mm(x.t(), dy))
    try:
        v["addmm_f32_acc"] = timeit(lambda: torch.addmm(out, dy.t(), x, out_dtype=torch.float32))
    except Exception as e:
        v["addmm_f32_acc"] = None
    # split the token dim into chunks (more parallel tiles per launch? no: sequential)
    res[name] = {k: (round(fl / t / 1e12, 1) if t else None) for k, t in v.items()}
    print(name, json.dumps(res[name]), flush=True)
try:
    torch.backends.cuda.preferred_blas_library("cublas")
    for name, (k_in, n_out) in shapes.items():
        x = torch.randn(N, k_in, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(N, n_out, device="cuda", dtype=torch.bfloat16)
        fl = 2 * N * k_in * n_out
        print("rocblas", name, round(fl / timeit(lambda: torch.mm(dy.t(), x)) / 1e12, 1),
              "fwd", round(fl / timeit(lambda: torch.mm(x, torch.randn(n_out, k_in, device='cuda', dtype=torch.bfloat16).t())) / 1e12, 1), flush=True)
except Exception as e:
    print("rocblas switch failed", e)
