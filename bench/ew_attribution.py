"""Which aten ops launch stock-torch elementwise kernels inside a fused-executor training step?
Runs a few bench.py steps of a model under torch.profiler and attributes every kernel whose name
matches --kernel (default: torch's elementwise / reduce kernels) to the chain of CPU ops that
launched it (innermost three), with calls and GPU time per step.

    python bench/ew_attribution.py --model gemma4-e2b --batch 8 [--steps 3]
"""
from __future__ import annotations

import argparse
import collections
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gemma4-e2b")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--kernel", default="at::native")
    a = ap.parse_args()
    args = bench.parse_args(["--model", a.model, "--batch", str(a.batch)])
    cfg = bench.MODELS[a.model]
    dev = torch.device("cuda", 0)
    model, runner = bench._build(args, cfg, dev, "fused", 1)
    g = torch.Generator().manual_seed(0)
    pool = [torch.randint(0, cfg["V"], (a.batch, args.seq + 1), generator=g).pin_memory() for _ in range(4)]
    step = bench._make_step(runner, pool, dev)
    for i in range(3):
        step(i)
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts) as prof:
        for i in range(a.steps):
            step(i)
        torch.cuda.synchronize()
    calls = collections.Counter()
    us = collections.Counter()
    for e in prof.events():
        if e.device_type != torch.autograd.DeviceType.CPU or not e.kernels:
            continue
        chain, p = [], e
        while p is not None and len(chain) < 3:
            chain.append(p.name)
            p = p.cpu_parent
        key = " < ".join(chain)
        for k in e.kernels:
            if a.kernel in k.name:
                calls[key] += 1
                us[key] += k.duration
    tot = sum(us.values())
    print(f"# {a.model} B={a.batch}: kernels matching {a.kernel!r} per step, by launching op chain")
    print(" calls/step  us/step  op chain (innermost first)")
    for key, t in us.most_common(40):
        print(f"{calls[key] / a.steps:10.1f} {t / a.steps:8.1f}  {key}")
    print(f"total: {sum(calls.values()) / a.steps:.1f} kernels, {tot / a.steps / 1e3:.3f} ms per step")


if __name__ == "__main__":
    main()
