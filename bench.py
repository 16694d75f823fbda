"""Headline benchmark: whole-node training tokens/s, GPT-2 124M (reference example layout), DDP.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--engine fused|generic|reference]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

One process per GPU (RANK/LOCAL_RANK/WORLD_SIZE from the environment; backend nccl = RCCL).
Model: the reference's example GPT-2 layer list (``main.py:57-83``: V=50304, C=768, 12 layers,
12 heads, untied lm_head, 163.1 M params), AdamW(6e-4, (0.9, 0.95), 1e-8, wd 0.01), bf16 compute.
Data: synthetic uniform token ids of shape [B, T] per rank per step (random-init weights), copied
host->device every step like the runtime's loader path.  Weak scaling: B sequences of T=1024
tokens per GPU per step (default B=64 → 65,536 tokens/GPU/step, one micro-step).
Timed region: W untimed warmup steps, then exactly K full optimizer steps (forward, backward,
gradient all-reduce, fused AdamW) bracketed by barrier + synchronize; the max over ranks is
reported.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# Reference-semantics eager PyTorch on MI355X, same config (bench/ref_eager_gpt2.py, B=64, T=1024,
# measured on one MI355X this round: profiles/probe_env_r1.log).  BASELINE.md publishes no GPU
# number for the reference, so vs_baseline is null and this figure is reported separately.
REFERENCE_EAGER_TOK_S_PER_GPU = 482820.8


def gpt2_layers(V=50304, C=768, L=12, H=12, P=1024):
    std2 = 0.02 / math.sqrt(2 * L)
    layers = [{"summation": [{"embedding": {"num_embeddings": V, "embedding_dim": C}, "normal": {"mean": 0.0, "std": 0.02}},
                             {"position": {"num_embeddings": P, "embedding_dim": C}, "normal": {"mean": 0.0, "std": 0.02}}]},
              {"dropout": {"p": 0.0}}]
    for _ in range(L):
        layers.append({"residual": [
            {"sequential": [{"layernorm": {"normalized_shape": C}},
                            {"linear": {"in_features": C, "out_features": 3 * C}, "normal": {"mean": 0.0, "std": 0.02}, "zeros": {}},
                            {"attention": {"num_heads": H, "dropout": 0.0}},
                            {"linear": {"in_features": C, "out_features": C}, "normal": {"mean": 0.0, "std": std2}, "zeros": {}},
                            {"dropout": {"p": 0.0}}]},
            {"sequential": [{"layernorm": {"normalized_shape": C}},
                            {"linear": {"in_features": C, "out_features": 4 * C}, "normal": {"mean": 0.0, "std": 0.02}, "zeros": {}},
                            {"gelu": {}},
                            {"linear": {"in_features": 4 * C, "out_features": C}, "normal": {"mean": 0.0, "std": std2}, "zeros": {}},
                            {"dropout": {"p": 0.0}}]}]})
    layers += [{"layernorm": {"normalized_shape": C}},
               {"linear": {"in_features": C, "out_features": V, "bias": False}},
               {"softmaxlast": {"dim": -1}}]
    return layers


MODELS = {
    "gpt2-124m": dict(V=50304, C=768, L=12, H=12, P=1024),
    "gpt2-xl": dict(V=50304, C=1600, L=48, H=25, P=1024),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64, help="sequences per GPU per step")
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--engine", default="fused", choices=["fused", "generic", "reference"])
    ap.add_argument("--model", default="gpt2-124m", choices=list(MODELS))
    ap.add_argument("--profile", default=None, metavar="DIR",
                    help="after the timed steps, profile 3 more under torch.profiler into DIR "
                         "(Chrome trace + per-kernel table); set PENROZ_ROCTX=1 for roctx phase ranges")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} != WORLD_SIZE {world}")
    # PENROZ_BENCH_DEVICE / PENROZ_DIST_BACKEND: rehearsal knobs only (e.g. 2 ranks sharing the
    # one GPU of a test box over gloo); the headline runs use LOCAL_RANK and nccl (= RCCL).
    local = int(os.environ.get("PENROZ_BENCH_DEVICE", local))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        backend = os.environ.get("PENROZ_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)
    os.environ["PENROZ_ENGINE"] = args.engine

    from penroz.models.mapper import Mapper
    from penroz.models.model import NeuralNetworkModel, _make_runner

    cfg = MODELS[args.model]
    torch.manual_seed(1234)
    model = NeuralNetworkModel("bench", Mapper(gpt2_layers(**cfg),
                                               {"adamw": {"lr": 6e-4, "betas": [0.9, 0.95], "eps": 1e-8}}))
    model.to(device)
    runner = _make_runner(model, args.engine, device, distributed=world > 1)
    model.train()

    B, T, V = args.batch, args.seq, cfg["V"]
    g = torch.Generator().manual_seed(rank)
    pool = [torch.randint(0, V, (B, T + 1), generator=g).pin_memory() for _ in range(4)]

    def step(i):
        buf = pool[i % len(pool)].to(device, non_blocking=True)
        x, y = buf[:, :-1], buf[:, 1:]
        runner.zero_grad()
        loss = runner.micro_step(x.contiguous(), y.contiguous(), 1.0, first=True, last=True, capture=False)
        runner.step()
        return loss

    for i in range(args.warmup):
        step(i)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms = dt / args.steps * 1e3
    tok_s = world * B * T * args.steps / dt
    if rank == 0:
        flops_per_tok = 6 * (sum(p.numel() for p in model.parameters()) - cfg["V"] * cfg["C"] - cfg["P"] * cfg["C"]) \
            + 12 * cfg["L"] * cfg["C"] * T
        print(json.dumps({
            "metric": "tokens/sec (whole node) GPT-2 124M DDP train at 1/2/4/8 MI355X" if args.model == "gpt2-124m"
            else f"tokens/sec (whole node) {args.model} DDP train",
            "value": tok_s, "unit": "tokens/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "vs_reference_eager_same_gpu": tok_s / (world * REFERENCE_EAGER_TOK_S_PER_GPU) if args.model == "gpt2-124m" else None,
            "mfu_bf16_dense": tok_s / world * flops_per_tok / 2.5e15,
            "final_loss": float(loss.item()), "engine": args.engine,
            "dtype": "bf16", "data": "synthetic uniform tokens, random-init weights",
            "config": {"model": args.model, "global_batch": world * B, "seq_len": T, "micro_batch_per_gpu": B,
                       "tokens_per_step": world * B * T, "parallelism": f"dp{world}"},
        }), flush=True)
    if args.profile:  # outside the timed region
        from penroz.utils.profiling import profile_steps
        out = os.path.join(args.profile, f"rank{rank}")
        table = profile_steps(lambda: step(0), 3, out)
        if rank == 0:
            print(table, file=sys.stderr)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
