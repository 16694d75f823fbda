"""Where does the runtime path (NeuralNetworkModel.train_model: Loader, per-epoch diagnostics,
progress) lose time against the bare executor step? Runs a few epochs of the GPT-2 124M headline
config through train_model under torch.profiler and reports, per epoch, the wall time, the GPU busy
time (union of kernel intervals) and the largest GPU idle gaps with the CPU ops running meanwhile.

    python bench/runtime_profile.py [--epochs 6] [--out gpurun_out/runtime_prof]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def summarize(prof, path, n, label):
    import collections
    prof.export_chrome_trace(path)
    ev = json.load(open(path))["traceEvents"]
    ks = [e for e in ev if e.get("cat") == "kernel"]
    iv = sorted((e["ts"], e["ts"] + e.get("dur", 0)) for e in ks)
    busy, cs, ce = 0.0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > ce:
            busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    span = iv[-1][1] - iv[0][0]
    per = collections.Counter()
    for e in ks:
        per[e["name"]] += e.get("dur", 0)
    print(f"{label}: {n} steps, span {span / 1e3 / n:.2f} ms/step, GPU busy (any kernel) {busy / 1e3 / n:.2f} ms/step, "
          f"{len(ks) / n:.0f} kernels/step, kernel-time sum {sum(per.values()) / 1e3 / n:.2f} ms/step")
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=6)
    ap.add_argument("--out", default="gpurun_out/runtime_prof")
    args = ap.parse_args()
    from penroz.models import model as model_mod
    from penroz.models.mapper import Mapper
    from penroz.models.model import NeuralNetworkModel
    from penroz.utils import loaders
    B, T, V = 64, 1024, 50304
    tmp = tempfile.mkdtemp(prefix="penroz_rt_prof_")
    loaders.DATA_FOLDER = os.path.join(tmp, "data")
    NeuralNetworkModel.SHM_PATH = os.path.join(tmp, "shm")
    model_mod.MODELS_FOLDER = os.path.join(tmp, "models")
    epochs = args.epochs + 3
    rng = np.random.default_rng(0)
    loaders.save_shard("bench", 0, rng.integers(0, V, epochs * B * T + 1), V)
    torch.manual_seed(1234)
    m = NeuralNetworkModel("prof", Mapper(bench.gpt2_layers(), {"adamw": {"lr": 6e-4, "betas": [0.9, 0.95]}}))
    m.to("cuda")
    os.environ["PENROZ_ENGINE"] = "fused"
    m.train_model("bench", 0, 3, B, T, B)  # warm up (executor, GEMM tables, allocator)
    os.makedirs(args.out, exist_ok=True)
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    # the bare executor step on the same model for comparison (bench.py's loop)
    from penroz.models.model import _make_runner
    runner = _make_runner(m, "fused", torch.device("cuda"), False)
    g = torch.Generator().manual_seed(0)
    pool = [torch.randint(0, V, (B, T + 1), generator=g).pin_memory() for _ in range(2)]
    step = bench._make_step(runner, pool, torch.device("cuda"))
    for i in range(3):
        step(i)
    torch.cuda.synchronize()
    with torch.profiler.profile(activities=acts) as pb:
        for i in range(args.epochs):
            step(i)
        torch.cuda.synchronize()
    runner.close()
    bk = summarize(pb, os.path.join(args.out, "bench_trace.json"), args.epochs, "bench loop")
    with torch.profiler.profile(activities=acts) as prof:
        m.train_model("bench", 0, args.epochs, B, T, B)
    rk = summarize(prof, os.path.join(args.out, "trace.json"), args.epochs, "train_model")
    print("per-epoch kernel time deltas (train_model - bench loop), ms:")
    for n in sorted(set(bk) | set(rk), key=lambda n: -abs(rk.get(n, 0) - bk.get(n, 0)))[:12]:
        print(f"  {(rk.get(n, 0) - bk.get(n, 0)) / 1e3 / args.epochs:+8.3f}  {n[:100]}")
    path = os.path.join(args.out, "trace.json")
    ev = json.load(open(path))["traceEvents"]
    kern = sorted((e["ts"], e["ts"] + e.get("dur", 0)) for e in ev if e.get("cat") == "kernel")
    cpu = [e for e in ev if e.get("cat") in ("cpu_op", "python_function", "user_annotation")]
    # gaps: GPU idle intervals > 200 us with the CPU ops active in them
    gaps, end = [], kern[0][1]
    for s, e in kern[1:]:
        if s - end > 200:
            gaps.append((end, s))
        end = max(end, e)
    print(f"kernels {len(kern)}, span {(kern[-1][1] - kern[0][0]) / 1e3:.1f} ms, "
          f"epochs {args.epochs}, progress tokensPerSec {[round(p['tokensPerSec']) for p in m.progress]}")
    tot = sum(b - a for a, b in gaps)
    print(f"GPU idle gaps > 0.2 ms: {len(gaps)}, total {tot / 1e3:.2f} ms")
    for a, b in sorted(gaps, key=lambda g: g[0] - g[1])[:12]:
        names = sorted({e["name"] for e in cpu if e["ts"] < b and e["ts"] + e.get("dur", 0) > a
                        and e.get("dur", 0) > 0.3 * (b - a)})
        print(f"  gap {(b - a) / 1e3:6.2f} ms at +{(a - kern[0][0]) / 1e3:8.1f} ms: {names[:8]}")


if __name__ == "__main__":
    main()
