"""Probe forward / dgrad GEMMs at GPT-2 124M shapes (M = 65536 tokens) on one MI355X.

Times torch.addmm / torch.mm (hipBLASLt heuristic pick) per shape, then the same calls with
PyTorch TunableOp searching hipBLASLt + rocBLAS solutions, and (if built) the native kernels.
    python bench/probe_fwd_gemm.py [--tunable]
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timeit(fn, iters=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


M = 65536
SHAPES = {"qkv": (768, 2304), "proj": (768, 768), "fc": (768, 3072), "fc2": (3072, 768), "lm_head": (768, 50304)}


def run(tag):
    res = {}
    torch.manual_seed(0)
    for name, (k_in, n_out) in SHAPES.items():
        x = torch.rand(M, k_in, device="cuda", dtype=torch.bfloat16) * 2 - 1
        w = (torch.rand(n_out, k_in, device="cuda", dtype=torch.bfloat16) * 2 - 1) * 0.05
        b = torch.rand(n_out, device="cuda", dtype=torch.bfloat16)
        dy = torch.rand(M, n_out, device="cuda", dtype=torch.bfloat16) * 2 - 1
        y = torch.empty(M, n_out, device="cuda", dtype=torch.bfloat16)
        dx = torch.empty(M, k_in, device="cuda", dtype=torch.bfloat16)
        fl = 2 * M * k_in * n_out
        if name == "lm_head":
            tf = timeit(lambda: torch.mm(x, w.t(), out=y))
        else:
            tf = timeit(lambda: torch.addmm(b, x, w.t(), out=y))
        td = timeit(lambda: torch.mm(dy, w, out=dx))
        res[name] = {"fwd_TF": round(fl / tf / 1e12, 1), "fwd_us": round(tf * 1e6, 1),
                     "dgrad_TF": round(fl / td / 1e12, 1), "dgrad_us": round(td * 1e6, 1)}
        print(tag, name, json.dumps(res[name]), flush=True)
    tot_f = sum(v["fwd_us"] for v in res.values())
    tot_d = sum(v["dgrad_us"] for v in res.values())
    print(tag, "per-step GEMM ms (12 layers + head):",
          json.dumps({"fwd": round((tot_f - res['lm_head']['fwd_us']) * 12 / 1e3 + res['lm_head']['fwd_us'] / 1e3, 2),
                      "dgrad": round((tot_d - res['lm_head']['dgrad_us']) * 12 / 1e3 + res['lm_head']['dgrad_us'] / 1e3, 2)}),
          flush=True)
    return res


if __name__ == "__main__":
    run("default")
    if "--tunable" in sys.argv:
        import torch.cuda.tunable as tunable
        tunable.enable(True)
        tunable.tuning_enable(True)
        tunable.set_max_tuning_duration(200)
        tunable.set_max_tuning_iterations(30)
        out = os.path.join(ROOT, "gpurun_out", "tunableop_results.csv")
        tunable.set_filename(out)
        run("tuning")
        tunable.tuning_enable(False)
        run("tuned")
        tunable.write_file()
