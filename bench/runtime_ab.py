"""Runtime path (train_model) vs the bare executor loop, in either order within one process.

bench.py --via-runtime runs train_model AFTER the executor loop, on a second model: its ratio
(≈0.90) mixes the runtime's own cost with whatever a second executor in the same process costs
(new streams, a second set of HIP queues). This script runs the runtime first (``--order rb``) or
second (``--order br``) and prints both figures, so the two effects separate.

    python bench/runtime_ab.py --order rb --epochs 12
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def run_runtime(epochs: int, warm: int, B: int, T: int, V: int) -> float:
    from penroz.models import model as model_mod
    from penroz.models.mapper import Mapper
    from penroz.models.model import NeuralNetworkModel
    from penroz.utils import loaders
    tmp = tempfile.mkdtemp(prefix="penroz_rt_ab_")
    loaders.DATA_FOLDER = os.path.join(tmp, "data")
    NeuralNetworkModel.SHM_PATH = os.path.join(tmp, "shm")
    model_mod.MODELS_FOLDER = os.path.join(tmp, "models")
    n = warm + epochs + 1
    rng = np.random.default_rng(0)
    loaders.save_shard("bench", 0, rng.integers(0, V, n * B * T + 1), V)
    torch.manual_seed(1234)
    m = NeuralNetworkModel("ab", Mapper(bench.gpt2_layers(), {"adamw": {"lr": 6e-4, "betas": [0.9, 0.95]}}))
    m.to("cuda")
    os.environ["PENROZ_ENGINE"] = "fused"
    m.train_model("bench", 0, n, B, T, B)
    tps = [p["tokensPerSec"] for p in m.progress[warm:n - 1]]
    del m
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return B * T / (sum(tps) / len(tps)) * 1e3


def run_bench(steps: int, warm: int, B: int, T: int, V: int) -> float:
    args = bench.parse_args(["--steps", str(steps)])
    cfg = bench.MODELS["gpt2-124m"]
    dev = torch.device("cuda", 0)
    model, runner = bench._build(args, cfg, dev, "fused", 1)
    g = torch.Generator().manual_seed(0)
    pool = [torch.randint(0, V, (B, T + 1), generator=g).pin_memory() for _ in range(4)]
    step = bench._make_step(runner, pool, dev)
    for i in range(warm):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    ex = getattr(runner, "exec", None)
    if ex is not None:
        ex.end_training()
        ex.free_buffers()
    del runner, model
    torch.cuda.empty_cache()
    return ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--order", choices=["rb", "br", "rr", "bb"], default="rb")
    ap.add_argument("--epochs", type=int, default=12)
    args = ap.parse_args()
    B, T, V = 64, 1024, 50304
    out = {"order": args.order, "env": {k: v for k, v in os.environ.items() if k.startswith("PENROZ_")}}
    for i, c in enumerate(args.order):
        key = f"{i}_{'runtime' if c == 'r' else 'bench'}_ms"
        out[key] = run_runtime(args.epochs, 3, B, T, V) if c == "r" else run_bench(args.epochs, 3, B, T, V)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
