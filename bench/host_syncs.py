"""Host-side blocking calls inside a training step: runs a few bench.py steps of a model under
torch.profiler (CPU + GPU activity) and lists the HIP runtime calls that wait for the device
(stream / device / event synchronize, blocking copies) with the Python frames above them, plus
the per-step host time. A sync inside the step drains the GPU and shows up in a kernel trace as
an idle gap at the step boundary.

    python bench/host_syncs.py --model gemma3-1b --batch 8 [--steps 3]
"""
from __future__ import annotations

import argparse
import collections
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

BLOCKING = ("Synchronize", "hipMemcpy", "hipMemcpyWithStream", "hipMemcpyDtoH", "hipStreamQuery", "hipEventQuery",
            "hipMalloc", "hipFree", "hipHostMalloc", "hipHostFree")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gemma3-1b")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--steps", type=int, default=3)
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
    host = []
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, with_stack=True) as prof:
        for i in range(a.steps):
            t0 = time.perf_counter()
            step(i)
            host.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
    print(f"host time per step (ms): {[round(h * 1e3, 2) for h in host]}")
    calls = collections.defaultdict(lambda: [0, 0.0])
    for e in prof.events():
        if any(b in e.name for b in BLOCKING):
            stack = " <- ".join(f for f in (e.stack or [])[:6] if "penroz" in f or "bench" in f)[:400]
            k = (e.name, stack)
            calls[k][0] += 1
            calls[k][1] += e.cpu_time_total / 1e3
    for (name, stack), (n, ms) in sorted(calls.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"{ms / a.steps:9.3f} ms/step  {n / a.steps:6.1f}/step  {name}  | {stack}")
    # any single host event longer than 0.5 ms (a hidden wait), with its Python frames
    print("host events > 0.5 ms:")
    for e in sorted(prof.events(), key=lambda e: -e.cpu_time_total)[:60]:
        if e.device_type == torch.autograd.DeviceType.CPU and e.cpu_time_total > 500 and not e.name.startswith("ProfilerStep"):
            stack = " <- ".join(f for f in (e.stack or [])[:8] if "penroz" in f or "bench" in f)[:300]
            print(f"  {e.cpu_time_total / 1e3:8.3f} ms  {e.name[:60]}  | {stack}")


if __name__ == "__main__":
    main()
