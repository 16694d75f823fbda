"""Headline benchmark: whole-node training tokens/s, GPT-2 124M (reference example layout), DDP.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--engine fused|generic|reference]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

One process per GPU (backend nccl = RCCL).  Under torchrun (or any launcher that sets
``WORLD_SIZE``) each process is one rank.  Started plainly with ``--gpus N > 1`` the script is
its own launcher, like the reference's ``ddp.py:43-73`` (one worker per visible device): the
parent never touches the GPU (``torch.cuda.device_count()`` does not initialise HIP), checks
that N devices are visible — failing loudly otherwise instead of silently measuring one GPU —
spawns N child ranks with ``RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
MASTER_PORT``, tears the group down if any rank fails, and exits with the first failing code.

Model: the reference's example GPT-2 layer list (``main.py:57-83``: V=50304, C=768, 12 layers,
12 heads, untied lm_head, 163.1 M params), AdamW(6e-4, (0.9, 0.95), 1e-8, wd 0.01), bf16 compute.
Data: synthetic uniform token ids of shape [B, T] per rank per step (random-init weights), copied
host->device every step like the runtime's loader path.  Weak scaling: B sequences of T=1024
tokens per GPU per step (default B=64 → 65,536 tokens/GPU/step, one micro-step).
Timed region: W untimed warmup steps, then exactly K full optimizer steps (forward, backward,
gradient all-reduce, fused AdamW) bracketed by barrier + synchronize; the max over ranks is
reported.  Rank 0 prints one JSON line.

Extra fields (outside the timed region):
  * ``comm``: bucket plan, wire dtype, transport, RCCL version, ranks seen by the communicator,
    and ``allreduce_exposed_ms`` = ms/step of the timed run minus ms/step of a few further
    steps with the gradient all-reduce switched off (the part of the collective NOT hidden
    behind the backward), and ``probe_busbw_GBps`` = ring bus bandwidth of bare all-reduces of
    one default-size bucket (RCCL over xGMI at N > 1; compare 7 links × ≈153 GB/s);
  * ``comm`` at N > 1 also holds the first-contact record made before the model is built
    (``penroz.parallel.commtune``): ``devices`` (every rank's PCI id; duplicate devices abort
    the run), ``sweep`` (bare all-reduce ms / busbw over bucket sizes 16-256 MB x fp32/bf16 wire x
    c10d/native transport, each result checked for the exact average; with
    ``PENROZ_COMM_SWEEP_ARMS=full`` also native channel count 8/16/32, forced protocol Simple /
    LL128 and forced algorithm Ring / Tree), ``plan`` (``commtune.plan``: transport + channel count +
    protocol + algorithm and bucket size the gradient reducer then uses — each transport judged at
    its own bucket size — and ``wire_recommendation``, bf16 when the predicted fp32 all-reduce
    exceeds the estimated backward; the wire itself stays fp32 unless the user sets it; user-set
    ``PENROZ_COMM`` / ``PENROZ_RCCL_CHANNELS`` / ``PENROZ_RCCL_PROTO`` / ``PENROZ_RCCL_ALGO`` /
    ``PENROZ_BUCKET_MB`` /
    ``PENROZ_GRAD_WIRE`` win) and ``rccl.coll_channels`` / ``rccl.nranks`` (parsed from RCCL's INIT
    log: what RCCL itself built for c10d's communicator). ``rccl_nranks`` is ``ncclCommCount`` of the
    native communicator when the gradients go through it. ``sweep_stats`` holds the sweep's wall time
    and the arms run / skipped (``commtune.SWEEP_BUDGET_S``) / failed. The forced channel / protocol /
    algorithm arms run only with ``PENROZ_COMM_SWEEP_ARMS=full``. The process group has an explicit timeout
    (``PENROZ_DIST_TIMEOUT``, 300 s), so a stuck rank fails the run instead of hanging it;
  * ``vs_reference_eager_same_gpu``: the same config through the ``reference`` engine (stock
    PyTorch eager + autocast + foreach AdamW, the reference's semantics) measured in this same
    process right after with the headline's own warmup / step counts (1 GPU only; ``--ref-steps
    0`` skips it).
``--device cpu`` (gloo, generic engine, pair it with ``--model tiny``) is the plumbing rehearsal
used by the CPU tests; the headline is always ``--device cuda``.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import subprocess
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC = "tokens/sec (whole node) GPT-2 124M DDP train at 1/2/4/8 MI355X"


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
    # the /import/ of HF "gpt2": V = 50257, tanh GELU, embd/resid/attn dropout 0.1, bf16 params
    # (reference mappers.py:122-176, neural_net_model.py:222); random init, no download
    "gpt2-hf": dict(V=50257, C=768, L=12, H=12, P=1024, hf=True),
    "tiny": dict(V=512, C=64, L=2, H=2, P=64),  # plumbing rehearsal only
    # google/gemma-3-1b-pt text shapes through Mapper.from_hf_config (RMSNorm, RoPE, GQA 4:1,
    # head_dim 256, gated GELU MLP, 262k vocab; random init, no checkpoint): the generic engine
    # (autograd over the HIP layers: flash attention D=256, RMSNorm, gated activation)
    "gemma3-1b": dict(V=262144, C=1152, L=26, H=4, P=32768, gemma=True, Hkv=1, D=256, F=6912),
    # a Gemma-4-class layer list through the reference's heterogeneous-layer mapping
    # (mappers.py:206-233; the E2B-sized text stack is not published offline, so the shape is
    # synthetic): sliding (head_dim 256) and full-attention (global_head_dim 512, one global KV
    # head) layers alternating, the last 8 layers KV-shared with double-wide gated MLPs,
    # 262k vocab, tied embedding. Exercises the D = 512 flash kernels in the fused executor.
    "gemma4-e2b": dict(V=262144, C=1536, L=20, H=8, P=32768, gemma=True, gemma4=True, Hkv=1, D=256, F=6144,
                       Dg=512, Hkv_g=1, shared=8),
}


def gemma3_1b_layers(L: int = 26) -> list[dict]:
    from types import SimpleNamespace
    from penroz.models.mapper import Mapper
    return Mapper.from_hf_config(SimpleNamespace(
        model_type="gemma3_text", vocab_size=262144, hidden_size=1152, intermediate_size=6912, num_hidden_layers=L,
        num_attention_heads=4, num_key_value_heads=1, head_dim=256, rms_norm_eps=1e-6, rope_theta=1e6,
        rope_local_base_freq=10000.0, attention_dropout=0.0, hidden_activation="gelu_pytorch_tanh",
        query_pre_attn_scalar=256, sliding_window=512))


def gemma4_config(cfg: dict):
    """The HF-style text config of a ``gemma4=True`` MODELS entry (Mapper.from_hf_config input)."""
    from types import SimpleNamespace
    return SimpleNamespace(
        model_type="gemma4_text", vocab_size=cfg["V"], hidden_size=cfg["C"], intermediate_size=cfg["F"],
        num_hidden_layers=cfg["L"], num_attention_heads=cfg["H"], num_key_value_heads=cfg["Hkv"],
        head_dim=cfg["D"], global_head_dim=cfg["Dg"], num_global_key_value_heads=cfg["Hkv_g"],
        layer_types=["sliding_attention", "full_attention"] * (cfg["L"] // 2) + ["sliding_attention"] * (cfg["L"] % 2),
        num_kv_shared_layers=cfg["shared"], use_double_wide_mlp=True, rms_norm_eps=1e-6, rope_theta=1e6,
        attention_dropout=0.0, hidden_activation="gelu_pytorch_tanh", query_pre_attn_scalar=cfg["D"])


def gemma_layer_shapes(cfg: dict) -> list[tuple[int, int, int]]:
    """Per layer (head_dim, KV heads, MLP width) of a gemma MODELS entry."""
    if not cfg.get("gemma4"):
        return [(cfg["D"], cfg["Hkv"], cfg["F"])] * cfg["L"]
    g = gemma4_config(cfg)
    first_shared = cfg["L"] - cfg["shared"]
    return [((cfg["Dg"], cfg["Hkv_g"]) if t == "full_attention" else (cfg["D"], cfg["Hkv"]))
            + ((2 * cfg["F"]) if i >= first_shared else cfg["F"],) for i, t in enumerate(g.layer_types)]


def hf_gpt2_layers(V, C, L, H, P, pdrop=None):
    # PENROZ_BENCH_HF_PDROP: A/B of the import layout's dropout (HF gpt2: 0.1 at all three sites)
    if pdrop is None:
        pdrop = float(os.environ.get("PENROZ_BENCH_HF_PDROP", "0.1"))
    from types import SimpleNamespace
    from penroz.models import hf
    cfg = SimpleNamespace(vocab_size=V, n_embd=C, n_head=H, n_layer=L, n_positions=P, activation_function="gelu_new",
                          resid_pdrop=pdrop, embd_pdrop=pdrop, attn_pdrop=pdrop, model_type="gpt2")
    return hf.gpt2_layers(cfg)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU); self-launched when WORLD_SIZE is unset")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None, help="sequences per GPU per step (default 64; tiny: 4)")
    ap.add_argument("--seq", type=int, default=None, help="tokens per sequence (default 1024; tiny: 32)")
    ap.add_argument("--engine", default=None, choices=["fused", "generic", "reference"],
                    help="default: fused on cuda, generic on cpu")
    ap.add_argument("--model", default="gpt2-124m", choices=list(MODELS))
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    ap.add_argument("--ref-steps", type=int, default=-1,
                    help="steps of the reference engine measured after the run for vs_reference_eager_same_gpu "
                         "(1 GPU, gpt2-124m only; default -1 = the headline's --steps after its --warmup; 0 = skip)")
    ap.add_argument("--comm-probe-iters", type=int, default=5,
                    help="world > 1: time this many bare all-reduces of one gradient bucket after the timed "
                         "run and report the bus bandwidth in comm (0 = skip)")
    ap.add_argument("--nocomm-steps", type=int, default=4,
                    help="steps without the gradient all-reduce, for allreduce_exposed_ms (world > 1; 0 = skip)")
    ap.add_argument("--no-comm-sweep", dest="comm_sweep", action="store_false",
                    help="world > 1: skip the first-contact all-reduce sweep (bucket size x wire x transport) "
                         "that picks the gradient transport before the timed run")
    ap.add_argument("--no-gemm-table-guard", dest="gemm_table_guard", action="store_false",
                    help="skip the pre-timing check that keeps the shipped GEMM solution table only if it is not "
                         "slower than hipBLASLt's heuristic on this step (reported as gemm_table)")
    ap.add_argument("--via-runtime", action="store_true",
                    help="also time the same config through NeuralNetworkModel.train_model (Loader over synthetic "
                         "shards, per-epoch diagnostics, checkpoints) and report its tokensPerSec progress figure")
    ap.add_argument("--data-ranks", type=int, default=1,
                    help="single process only: each step's batch is the concatenation of the synthetic batches "
                         "that ranks 0..N-1 of a --gpus N run would draw (with --batch B·N), so its losses and "
                         "parameters must match that N-rank data-parallel run (rehearsal check)")
    ap.add_argument("--profile", default=None, metavar="DIR",
                    help="after the timed steps, profile 3 more under torch.profiler into DIR "
                         "(Chrome trace + per-kernel table); set PENROZ_ROCTX=1 for roctx phase ranges")
    args = ap.parse_args(argv)
    tiny = args.model == "tiny"
    args.batch = args.batch or (4 if tiny else 64)
    args.seq = args.seq or (32 if tiny else 1024)
    args.engine = args.engine or ("fused" if args.device == "cuda" else "generic")
    if args.device == "cpu" and args.engine == "fused":
        raise SystemExit("the fused engine needs --device cuda")
    return args


# ------------------------------------------------------------------------------- self-launch
def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv: list[str], poll_s: float = 0.2, script: str | None = None) -> int:
    """Spawn ``args.gpus`` child ranks of ``script`` (default: this file) and supervise them
    (parent: no GPU use)."""
    n = args.gpus
    if args.device == "cuda":
        visible = torch.cuda.device_count()  # does not initialise HIP on this image
        if visible < n:
            print(f"bench.py: --gpus {n} requested but only {visible} GPU(s) are visible; refusing to "
                  f"report a {n}-GPU number from fewer devices", file=sys.stderr, flush=True)
            return 2
    port = _free_port()
    threads = max(1, (os.cpu_count() or 2) // n)
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                    "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                    "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
        if args.device == "cpu":
            env.setdefault("OMP_NUM_THREADS", str(threads))
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    try:
        live = list(procs)
        while live:
            time.sleep(poll_s)
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    print(f"bench.py: rank {procs.index(p)} exited with code {code}; stopping the group",
                          file=sys.stderr, flush=True)
                    for q in live:
                        q.terminate()
    finally:
        for p in procs:
            try:
                p.wait(timeout=60)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    return rc if rc >= 0 else 128 - rc


# ------------------------------------------------------------------------------- one rank
def _sync(device):
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def _comm_info(runner, world: int) -> dict:
    red = None
    ex = getattr(runner, "exec", None)
    if ex is not None:
        red = ex.reducer
    elif getattr(runner, "reducer", None) is not None:
        red = runner.reducer.reducer
    info = {"nranks": dist.get_world_size() if dist.is_initialized() else 1}
    native = getattr(red, "_native", None) if red is not None else None
    if native is not None:  # what RCCL itself reports for the communicator the gradients go through
        info["rccl_nranks"] = {"native": native.nranks, "native_rank": native.comm_rank,
                               "native_device": native.comm_device}
    try:
        v = torch.cuda.nccl.version()
        info["rccl_version"] = ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
    except Exception:  # no RCCL in this build
        info["rccl_version"] = None
    if ex is not None and hasattr(ex, "opt_overlap_mode"):
        info["optimizer_overlap"] = ex.opt_overlap_mode()
    if red is not None:
        sizes = [(e - s) * red.flat_grad.element_size() / 2**20 for s, e in red.buckets]
        info.update({"buckets": len(sizes), "bucket_mb": [round(x, 2) for x in sizes],
                     "wire": "bf16" if red._wire is not None else str(red.flat_grad.dtype).replace("torch.", ""),
                     "transport": "native-rccl" if red._native is not None else red.backend,
                     "grad_mb": round(sum(sizes), 2)})
    return info


def _reducer_of(runner):
    ex = getattr(runner, "exec", None)
    if ex is not None:
        return ex.reducer
    r = getattr(runner, "reducer", None)
    return r.reducer if r is not None else None


def _allreduce_probe(device, world: int, iters: int) -> dict:
    """Bare in-place AVG all-reduces of one default-size fp32 gradient bucket (RCCL over xGMI on
    the GPU; a 4 MB bucket over gloo on the CPU): ms per call and ring bus bandwidth
    (bytes · 2(n−1)/n per second, the per-rank link traffic), max over ranks."""
    from penroz.parallel.reducer import DEFAULT_BUCKET_MB
    mb = DEFAULT_BUCKET_MB if device.type == "cuda" else 4
    buf = torch.ones(int(mb * 2**20) // 4, device=device, dtype=torch.float32)
    op = dist.ReduceOp.AVG if device.type == "cuda" else dist.ReduceOp.SUM
    for _ in range(2):
        dist.all_reduce(buf, op=op)
    dt, _ = _timed(lambda i: dist.all_reduce(buf, op=op), iters, world, device)
    t = dt / iters
    return {"probe_allreduce_mb": mb, "probe_allreduce_ms": t * 1e3,
            "probe_busbw_GBps": buf.numel() * 4 * 2 * (world - 1) / world / t / 1e9}


def _grad_plan_inputs(args) -> tuple[int, float]:
    """(fp32 gradient bytes, estimated backward ms per rank) of the benchmarked model, before it
    is built: parameter count from the config (GPT: 12·L·C² blocks + untied wte/lm_head + wpe;
    Gemma: the layer list's linears), backward ≈ 2/3 of 6·params·tokens at a planning 1.0 PF/s."""
    cfg = MODELS[args.model]
    C, L, V = cfg["C"], cfg["L"], cfg["V"]
    if cfg.get("gemma"):  # q, o: H·D·C each; k, v: Hkv·D·C each; gate, up, down: C·F each; 4 RMSNorms per
        # layer + the final one; embedding + lm_head
        n = sum(C * (2 * cfg["H"] * D + 2 * Hkv * D) + 3 * C * F + 4 * C for D, Hkv, F in gemma_layer_shapes(cfg))
        n += 2 * V * C + C
    else:
        n = L * (12 * C * C + 13 * C) + 2 * V * C + cfg["P"] * C + 2 * C
    tokens = args.batch * args.seq
    return 4 * n, 4.0 * n * tokens / 1.0e15 * 1e3


def _first_contact(args, device, world: int, rccl_log) -> dict:
    """World > 1, before the model is built (outside the timed region): every rank's device
    identity (N distinct PCI devices, or fail), the all-reduce sweep over bucket size × wire dtype
    × transport × RCCL channel count (``penroz.parallel.commtune``), and the plan the reducer will
    use — transport + channels, bucket size, wire — each transport judged at its own bucket size
    (``commtune.plan``; any of ``PENROZ_COMM`` / ``PENROZ_RCCL_CHANNELS`` / ``PENROZ_BUCKET_MB`` /
    ``PENROZ_GRAD_WIRE`` set by the user wins), and the channel count RCCL picked."""
    from penroz.parallel import commtune
    devices = commtune.gather_identities(device)
    if device.type == "cuda" and "PENROZ_BENCH_DEVICE" not in os.environ:
        pcis = [d.get("pci") for d in devices]
        if len(set(pcis)) != len(pcis):
            raise SystemExit(f"bench.py: ranks share devices {pcis}; refusing to report a {world}-GPU number")
    out = {"devices": [d.get("pci", d.get("host")) for d in devices]}
    if args.comm_sweep:
        sizes = commtune.SWEEP_SIZES_MB if device.type == "cuda" else (1, 4)
        channels, protos, algos = commtune.sweep_arms() if device.type == "cuda" else ((0,), ("",), ("",))
        stats = {}
        transports = ("c10d", "native") if device.type == "cuda" else ("c10d",)  # native = RCCL only
        rows = commtune.sweep(device, sizes_mb=sizes, iters=args.comm_probe_iters or 3, channels=channels,
                              protos=protos, algos=algos, transports=transports, stats=stats)
        out["sweep"] = rows
        out["sweep_stats"] = stats
        grad_bytes, bwd_ms = _grad_plan_inputs(args)
        if device.type != "cuda":
            bwd_ms = None  # the 1 PF/s planning rate means nothing for the CPU plumbing config
        # the wire stays fp32 (the reference DDP's numerics); the plan only RECORDS whether a bf16
        # wire would pay (wire_recommendation) — PENROZ_GRAD_WIRE=bf16 is the user's opt-in
        pl = commtune.plan(rows, grad_bytes, bwd_ms, auto_bf16=False)
        pl["grad_bytes"], pl["backward_ms_estimate"] = grad_bytes, None if bwd_ms is None else round(bwd_ms, 4)
        # the gloo plumbing config keeps the reference DDP's 25 MB buckets and fp32 wire: the sweep's
        # sizes do not model its TCP transfers
        applied = {"PENROZ_COMM": pl["transport"]}
        if pl["transport"] == "native" and pl.get("channels"):
            applied["PENROZ_RCCL_CHANNELS"] = str(pl["channels"])
        if pl["transport"] == "native" and pl.get("proto"):
            applied["PENROZ_RCCL_PROTO"] = pl["proto"]
        if pl["transport"] == "native" and pl.get("algo"):
            applied["PENROZ_RCCL_ALGO"] = pl["algo"]
        if device.type == "cuda":
            if pl.get("bucket_mb") is not None:
                applied["PENROZ_BUCKET_MB"] = str(pl["bucket_mb"])
        for k, v in applied.items():
            if k in os.environ:
                pl.setdefault("user_set", {})[k] = os.environ[k]
            else:
                os.environ[k] = v
        # every rank must run the same reducer plan (bucket boundaries, transport): the sweep rows are
        # MAX/MIN-reduced so the plan is a pure function of identical inputs — checked, not assumed
        env = {k: os.environ.get(k) for k in sorted(applied)}
        seen = [None] * world
        dist.all_gather_object(seen, env)
        if any(e != env for e in seen):
            raise SystemExit(f"bench.py: ranks disagree on the gradient-sync plan: {seen}")
        pl["applied_env"], pl["agreed_ranks"] = env, world
        out["plan"] = pl
        if device.type == "cuda":
            from penroz.parallel import rccl
            native = os.environ["PENROZ_COMM"] == "native"
            keep = int(os.environ.get("PENROZ_RCCL_CHANNELS", "0") or 0) if native else -1
            rccl.NativeComm.release(keep=keep, keep_proto=os.environ.get("PENROZ_RCCL_PROTO", "") if native else "",
                                    keep_algo=os.environ.get("PENROZ_RCCL_ALGO", "") if native else "")
    out["rccl"] = commtune.rccl_channels(rccl_log)
    return out


def _timed(step, n, world, device):
    if world > 1:
        dist.barrier()
    _sync(device)
    t0 = time.perf_counter()
    loss = None
    for i in range(n):
        loss = step(i)
    _sync(device)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=device if device.type == "cuda" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt, loss


def _build(args, cfg, device, engine, world):
    from penroz.models.mapper import Mapper
    from penroz.models.model import NeuralNetworkModel, _make_runner
    os.environ["PENROZ_ENGINE"] = engine
    torch.manual_seed(1234)
    dims = {k: cfg[k] for k in ("V", "C", "L", "H", "P")}
    if cfg.get("gemma4"):
        from penroz.models.mapper import Mapper
        layers = Mapper.from_hf_config(gemma4_config(cfg))
    elif cfg.get("gemma"):
        layers = gemma3_1b_layers(cfg["L"])
    else:
        layers = hf_gpt2_layers(**dims) if cfg.get("hf") else gpt2_layers(**dims)
    model = NeuralNetworkModel("bench", Mapper(layers, {"adamw": {"lr": 6e-4, "betas": [0.9, 0.95], "eps": 1e-8}}))
    if cfg.get("hf"):
        for mod in model.modules():
            if isinstance(mod, (torch.nn.Linear, torch.nn.Embedding)):
                torch.nn.init.normal_(mod.weight, 0.0, 0.02)
    model.to(device)
    if (cfg.get("hf") or cfg.get("gemma")) and device.type == "cuda":
        model.to(dtype=torch.bfloat16)  # what /import/ produces
    runner = _make_runner(model, engine, device, distributed=world > 1)
    model.train()
    return model, runner


def _make_step(runner, pool, device, sync_grads=True):
    """One training step on pool batch i. On the GPU each step copies the NEXT step's batch on a
    copy stream after enqueuing its own work (the runtime's Loader path prefetches the same way,
    models/model.py): the host-to-device copy on the compute stream put the host behind the GPU
    at every step boundary (PENROZ_COPY_STREAM=0: the copy inline, A/B; the copy stream is the
    process-wide one the runtime's Loader path uses too, models/executor.py shared_stream)."""
    cuda = device.type == "cuda" and os.environ.get("PENROZ_COPY_STREAM", "1") != "0"
    if cuda:
        from penroz.models.executor import shared_stream
        cs = shared_stream(device, "copy")
    pending = {}

    def fetch(slot):
        with torch.cuda.stream(cs):
            buf = pool[slot].to(device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(cs)
        return buf, ev

    def step(i):
        slot = i % len(pool)
        if cuda:
            buf, ev = pending.pop(slot, None) or fetch(slot)
            pending.clear()
            cur = torch.cuda.current_stream(device)
            cur.wait_event(ev)
            buf.record_stream(cur)
        else:
            buf = pool[slot].to(device, non_blocking=True)
        x, y = buf[:, :-1], buf[:, 1:]
        runner.zero_grad()
        loss = runner.micro_step(x.contiguous(), y.contiguous(), 1.0, first=True, last=sync_grads, capture=False)
        runner.step()
        if cuda:
            nxt = (i + 1) % len(pool)
            pending[nxt] = fetch(nxt)
        return loss
    return step


def _reference_eager_tok_s(args, cfg, device, pool) -> float | None:
    """Same config through the reference-semantics engine, in this process (1 GPU)."""
    from penroz.ops import _ext
    try:
        model, runner = _build(args, cfg, device, "reference", 1)
        step = _make_step(runner, pool, device)
        steps = args.steps if args.ref_steps < 0 else args.ref_steps
        for i in range(args.warmup):  # the headline's own warmup / step counts
            step(i)
        dt, _ = _timed(step, steps, 1, device)
        del model, runner
        return args.batch * args.seq * steps / dt
    except torch.OutOfMemoryError:
        return None
    finally:
        _ext.FORCE_TORCH = False
        torch.cuda.empty_cache()


def _via_runtime(args, cfg, device, world, rank) -> dict:
    """``PUT /train/``'s worker path (``train_model``) on the same config: synthetic token shards on
    disk, the rank-strided Loader, per-epoch weight-update ratios and cost sync, checkpoints in a
    scratch directory. Returns the mean ``tokensPerSec`` of the timed epochs (the last epoch, which
    also captures stats, is excluded) — the runtime's own throughput figure."""
    import tempfile
    import numpy as np
    from penroz.models import model as model_mod
    from penroz.models.mapper import Mapper
    from penroz.models.model import NeuralNetworkModel
    from penroz.utils import checkpoint as ckpt
    from penroz.utils import loaders
    B, T = args.batch, args.seq
    epochs = args.warmup + args.steps + 1
    tmp = tempfile.mkdtemp(prefix="penroz_runtime_bench_")
    saved = (loaders.DATA_FOLDER, NeuralNetworkModel.SHM_PATH, model_mod.MODELS_FOLDER)
    loaders.DATA_FOLDER = os.path.join(tmp, "data")
    NeuralNetworkModel.SHM_PATH = os.path.join(tmp, "shm")
    model_mod.MODELS_FOLDER = os.path.join(tmp, "models")
    try:
        if rank == 0:
            rng = np.random.default_rng(0)
            loaders.save_shard("bench", 0, rng.integers(0, cfg["V"], epochs * B * T * world + 1), cfg["V"])
        if world > 1:
            dist.barrier()
        torch.manual_seed(1234)
        dims = {k: cfg[k] for k in ("V", "C", "L", "H", "P")}
        layers = hf_gpt2_layers(**dims) if cfg.get("hf") else gpt2_layers(**dims)
        m = NeuralNetworkModel("bench", Mapper(layers, {"adamw": {"lr": 6e-4, "betas": [0.9, 0.95], "eps": 1e-8}}))
        m.to(device)
        if cfg.get("hf"):
            m.to(dtype=torch.bfloat16)
        os.environ["PENROZ_ENGINE"] = args.engine
        m.train_model("bench", 0, epochs, B, T, B)
        prog = m.progress[args.warmup:epochs - 1]
        tps = [p["tokensPerSec"] for p in prog]
        out = {"epochs_timed": len(tps), "tokensPerSec_mean": sum(tps) / len(tps) if tps else None,
               "tokensPerSec_median": sorted(tps)[len(tps) // 2] if tps else None,
               "speedPerSec_mean": sum(p["speedPerSec"] for p in prog) / len(prog) if prog else None}
        del m
        torch.cuda.empty_cache() if device.type == "cuda" else None
        return out
    finally:
        ckpt.wait_flushes()
        loaders.DATA_FOLDER, NeuralNetworkModel.SHM_PATH, model_mod.MODELS_FOLDER = saved
        if rank == 0:
            import shutil
            shutil.rmtree(tmp, ignore_errors=True)


def run_rank(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} != WORLD_SIZE {world}")
    if args.device == "cuda":
        # PENROZ_BENCH_DEVICE / PENROZ_DIST_BACKEND: rehearsal knobs only (e.g. 2 ranks sharing the
        # one GPU of a test box over gloo); the headline runs use LOCAL_RANK and nccl (= RCCL).
        local = int(os.environ.get("PENROZ_BENCH_DEVICE", local))
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    first_contact = {}
    if world > 1:
        from penroz.parallel import commtune
        from penroz.parallel.dist import init_group
        backend = os.environ.get("PENROZ_DIST_BACKEND", "nccl" if args.device == "cuda" else "gloo")
        rccl_log = commtune.enable_rccl_init_log(rank) if backend == "nccl" else None
        init_group(backend, device)  # explicit timeout: a stuck rank fails the run, no silent hang
        first_contact = _first_contact(args, device, world, rccl_log)

    cfg = MODELS[args.model]
    B, T, V = args.batch, args.seq, cfg["V"]
    if T > cfg["P"]:
        raise SystemExit(f"--seq {T} exceeds the {args.model} position table ({cfg['P']})")
    model, runner = _build(args, cfg, device, args.engine, world)
    if args.data_ranks > 1:
        if world > 1 or B % args.data_ranks:
            raise SystemExit("--data-ranks N: one process, --batch a multiple of N")
        gens = [torch.Generator().manual_seed(r) for r in range(args.data_ranks)]
        b = B // args.data_ranks
        pool = [torch.cat([torch.randint(0, V, (b, T + 1), generator=gr) for gr in gens]) for _ in range(4)]
    else:
        g = torch.Generator().manual_seed(rank)
        pool = [torch.randint(0, V, (B, T + 1), generator=g) for _ in range(4)]
    if device.type == "cuda":
        pool = [p.pin_memory() for p in pool]
    step = _make_step(runner, pool, device)

    for i in range(args.warmup):
        step(i)
    gemm_table = {}
    if device.type == "cuda" and args.gemm_table_guard:  # before the timed region, never inside it
        from penroz.ops import gemm as gemm_ops
        # _timed MAX-reduces over ranks, so every rank keeps or drops the table together
        gemm_table = gemm_ops.guard_tuned_gemms(lambda n: _timed(step, n, world, device)[0])
    dt, loss = _timed(step, args.steps, world, device)
    ms = dt / args.steps * 1e3
    tok_s = world * B * T * args.steps / dt
    final_loss = float(loss.item())

    comm = _comm_info(runner, world)
    comm.update(first_contact)
    # the loss averaged over ranks (= the single-process loss of the concatenated batch) and a
    # parameter checksum: what the multi-rank rehearsal tests compare against a --data-ranks run
    gl = loss.detach().float().reshape(1).clone()
    if world > 1:
        gl = gl.to(device) if device.type == "cuda" else gl
        dist.all_reduce(gl, op=dist.ReduceOp.SUM)
        gl /= world
        # every rank must have built the same gradient buckets (boundaries decide which
        # elements each collective sums): gathered and compared, not assumed
        red = _reducer_of(runner)
        plan_b = [list(b) for b in red.buckets] if red is not None else None
        plans = [None] * world
        dist.all_gather_object(plans, plan_b)
        if any(p_ != plan_b for p_ in plans):
            raise SystemExit(f"bench.py: ranks built different gradient buckets: {plans}")
        comm["bucket_plans_agree"] = world
    global_loss = float(gl.item())
    with torch.no_grad():
        param_checksum = float(sum(p.detach().double().abs().sum() for p in model.parameters()))
    if world > 1 and args.nocomm_steps > 0:  # outside the timed region
        dt0, _ = _timed(_make_step(runner, pool, device, sync_grads=False), args.nocomm_steps, world, device)
        comm["ms_per_step_without_allreduce"] = dt0 / args.nocomm_steps * 1e3
        comm["allreduce_exposed_ms"] = max(0.0, ms - comm["ms_per_step_without_allreduce"])
    elif world == 1:
        comm["allreduce_exposed_ms"] = 0.0
    if world > 1 and args.comm_probe_iters > 0:  # outside the timed region
        comm.update(_allreduce_probe(device, world, args.comm_probe_iters))

    if args.profile:  # outside the timed region
        from penroz.utils.profiling import profile_steps
        out = os.path.join(args.profile, f"rank{rank}")
        table = profile_steps(lambda: step(0), 3, out)
        if rank == 0:
            print(table, file=sys.stderr)

    n_params = sum(p.numel() for p in model.parameters())
    n_linear = sum(m.weight.numel() for m in model.modules() if isinstance(m, torch.nn.Linear))
    runtime = None
    if args.via_runtime:
        ex = getattr(runner, "exec", None)
        if ex is not None:
            ex.end_training()
            ex.free_buffers()
        del runner, model
        if device.type == "cuda":
            torch.cuda.empty_cache()
        runtime = _via_runtime(args, cfg, device, world, rank)
        if runtime.get("tokensPerSec_mean"):
            runtime["ratio_vs_executor"] = runtime["tokensPerSec_mean"] / tok_s
    ref_tok_s = None
    if (world == 1 and device.type == "cuda" and args.engine == "fused" and args.ref_steps != 0
            and args.model == "gpt2-124m"):
        if not args.via_runtime:
            ex = getattr(runner, "exec", None)
            if ex is not None:
                ex.free_buffers()
            del runner, model
            torch.cuda.empty_cache()
        ref_tok_s = _reference_eager_tok_s(args, cfg, device, pool)

    if rank == 0:
        if cfg.get("gemma"):  # matmul weights (tied lm_head counted as the Linear it is) + attention
            flops_per_tok = 6 * n_linear + sum(12 * cfg["H"] * D * T for D, _, _ in gemma_layer_shapes(cfg))
        else:
            flops_per_tok = 6 * (n_params - cfg["V"] * cfg["C"] - cfg["P"] * cfg["C"]) + 12 * cfg["L"] * cfg["C"] * T
        print(json.dumps({
            "metric": METRIC if args.model == "gpt2-124m" else f"tokens/sec (whole node) {args.model} DDP train",
            "value": tok_s, "unit": "tokens/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "vs_reference_eager_same_gpu": (tok_s / ref_tok_s) if ref_tok_s else None,
            "reference_eager_tok_s": ref_tok_s,
            "mfu_bf16_dense": tok_s / world * flops_per_tok / 2.5e15 if device.type == "cuda" else None,
            "final_loss": final_loss, "final_loss_global": global_loss, "param_checksum": param_checksum,
            "engine": args.engine, "device": args.device,
            "dtype": "bf16" if device.type == "cuda" else "fp32",
            "data": "synthetic uniform tokens, random-init weights",
            "comm": comm,
            **({"gemm_table": gemm_table} if gemm_table else {}),
            **({"via_runtime": runtime} if runtime is not None else {}),
            "config": {"model": args.model, "global_batch": world * B, "seq_len": T, "micro_batch_per_gpu": B,
                       "tokens_per_step": world * B * T, "parallelism": f"dp{world}"},
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args, argv))
    run_rank(args)


if __name__ == "__main__":
    main()
