"""First-contact communicator tuning for the gradient all-reduce (RCCL over xGMI, or gloo).

The reference hands gradient synchronisation to DDP's C++ Reducer with fixed 25 MB buckets over
ProcessGroupNCCL (``/root/reference/neural_net_model.py:609``). Here the transport, the bucket
size and the wire dtype are choices, and the right ones depend on the node: an MI355X has seven
point-to-point xGMI links (≈153 GB/s each), so a ring collective's bus bandwidth depends on how
many channels RCCL spreads over them and on the message size. This module measures that on the
job's own group, outside any timed region:

* :func:`sweep` — bare in-place AVG all-reduces of one gradient bucket for every (transport,
  wire dtype, bucket size), each checked for the correct average (rank-valued input), reporting
  ``ms``, ``algbw`` and ``busbw`` (= algbw · 2(n−1)/n, the per-rank link traffic of a ring);
* :func:`choose` — the transport for training: the C++ communicator (``csrc/comm/rccl_comm.cpp``)
  only when it reduced correctly and beat torch's ProcessGroupNCCL by a margin at the bucket size
  the reducer will use; otherwise c10d;
* :func:`rccl_channels` — the channel count RCCL picked, parsed from its INIT/GRAPH log
  (``enable_rccl_init_log`` must run before the first communicator is created);
* :func:`gather_identities` — every rank's device PCI id, proving N distinct devices.
"""
from __future__ import annotations

import glob
import logging
import os
import re
import time

import torch
import torch.distributed as dist

log = logging.getLogger(__name__)

SWEEP_SIZES_MB = (16, 32, 64, 128, 256)
# native communicator arms. The default first contact builds ONE native communicator (RCCL's own
# channel count, protocol and algorithm). The forced arms below are opt-in
# (``PENROZ_COMM_SWEEP_ARMS=full``): a forced protocol / algorithm that RCCL cannot serve fails only
# at enqueue time, and no run with more than one GPU has exercised them yet.
# channel counts: an MI355X node has 7 xGMI links per GPU, so the useful counts are multiples of the
# rings RCCL lays over them (0 = RCCL's own choice)
SWEEP_CHANNELS = (0, 8, 16, 32)
# protocols forced at RCCL's own channel count ("" = RCCL's per-size choice): Simple (bandwidth) vs
# LL128 (latency / mid sizes); LL is for small messages, not buckets
SWEEP_PROTOS = ("", "Simple", "LL128")
# algorithms forced likewise (the per-communicator NCCL_ALGO): Ring (bandwidth-optimal over the
# point-to-point xGMI rings) vs Tree (fewer steps for latency-bound sizes)
SWEEP_ALGOS = ("", "Ring", "Tree")
# wall-clock budget of the whole first-contact sweep; arms not yet started when it is spent are
# skipped (agreed over the group, so every rank skips the same ones)
SWEEP_BUDGET_S = 90.0


def sweep_arms() -> tuple[tuple, tuple, tuple]:
    """(channels, protos, algos) the first contact sweeps: RCCL's defaults only, or every forced arm
    with ``PENROZ_COMM_SWEEP_ARMS=full``."""
    if os.environ.get("PENROZ_COMM_SWEEP_ARMS", "default") == "full":
        return SWEEP_CHANNELS, SWEEP_PROTOS, SWEEP_ALGOS
    return (0,), ("",), ("",)


_LOG_DIR = "/tmp"


def enable_rccl_init_log(rank: int) -> str | None:
    """Route RCCL's INIT/GRAPH info log to a per-rank file (only if the user set no NCCL_DEBUG).

    Must run before the first RCCL communicator of the process is created (RCCL reads these
    once). Returns the file pattern, or None when the user's own settings are kept."""
    if "NCCL_DEBUG" in os.environ:
        return None
    pattern = os.path.join(_LOG_DIR, f"penroz_rccl_r{rank}_{os.getpid()}.log")
    os.environ["NCCL_DEBUG"] = "INFO"
    os.environ["NCCL_DEBUG_SUBSYS"] = "INIT,GRAPH"
    os.environ["NCCL_DEBUG_FILE"] = pattern
    return pattern


_CHAN_RE = [re.compile(r"(\d+) coll channels"), re.compile(r"Channel \d+/(\d+)")]
# RCCL's "Init COMPLETE" / "comm ... rank r nranks n" lines: the clique size RCCL itself built
_NRANKS_RE = re.compile(r"\bn[Rr]anks[ =](\d+)")


def parse_rccl_log(text: str) -> dict:
    """{'coll_channels', 'nranks'} from RCCL INIT/GRAPH log text (None where absent). ``nranks`` is
    the largest clique size any communicator of the process reported."""
    n = None
    for rx in _CHAN_RE:
        vals = [int(v) for v in rx.findall(text)]
        if vals:
            n = max(vals)
            break
    ranks = [int(v) for v in _NRANKS_RE.findall(text)]
    return {"coll_channels": n, "nranks": max(ranks) if ranks else None}


def rccl_channels(pattern: str | None) -> dict:
    """{'coll_channels': n | None, 'nranks': n | None, 'log': path} from the INIT log written under
    ``pattern`` (``nranks``: what RCCL itself reported for its communicators, c10d's included)."""
    if not pattern:
        return {"coll_channels": None, "nranks": None, "log": None}
    files = sorted(glob.glob(pattern + "*")) or ([pattern] if os.path.exists(pattern) else [])
    out = {"coll_channels": None, "nranks": None}
    for f in files:
        try:
            text = open(f, errors="replace").read()
        except OSError:
            continue
        got = parse_rccl_log(text)
        for k, v in got.items():
            if v is not None and out[k] is None:
                out[k] = v
    out["log"] = files[0] if files else None
    return out


def gather_identities(device: torch.device) -> list[dict]:
    from penroz.parallel.dist import device_identity
    me = device_identity(device)
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, me)
    return out


def _sync(device):
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def _native_or_none(device, channels: int = 0, proto: str = "", algo: str = ""):
    """The C++ communicator (``channels`` > 0: built with exactly that many RCCL channels; ``proto`` /
    ``algo``: with that RCCL protocol / algorithm forced) on every rank, or None on every rank
    (agreed over the c10d group).

    A rank that refuses right away (module missing, duplicate device, init error) makes every
    rank fall back. A rank that BLOCKS inside ncclCommInitRank while another refused cannot be
    released: ncclCommInitRank has no timeout, so the guard timer ends that process with exit
    code 124 after ``PENROZ_DIST_TIMEOUT`` — the failure conditions that can be checked without
    RCCL (module import, distinct devices) are agreed on BEFORE any rank enters the init."""
    ok = torch.zeros(1, device=device)
    native = None
    # only where it can work: RCCL ranks (a gloo rehearsal of several ranks on one GPU makes RCCL
    # refuse the duplicate device — "invalid usage" — which must not end the run) on distinct GPUs
    if (device.type == "cuda" and os.environ.get("PENROZ_COMM_SWEEP_NATIVE", "1") != "0"
            and dist.get_backend() == "nccl"):
        try:
            from penroz.parallel import rccl
            rccl.load_module()
            ok += 1
        except Exception:  # module missing on this rank: nobody builds a communicator
            pass
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if ok.item() > 0:
        ids = [(d.get("host"), d.get("pci"), d.get("uuid")) for d in gather_identities(device)]
        if len(set(ids)) != len(ids):
            ok.zero_()
    if ok.item() > 0:
        import threading
        from penroz.parallel import rccl
        from penroz.parallel.dist import dist_timeout_s
        # ncclCommInitRank blocks until every rank has joined and has no timeout of its own:
        # a rank that never gets there must end the job, not hang it
        guard = threading.Timer(dist_timeout_s(), lambda: os._exit(124))
        guard.daemon = True
        guard.start()
        built = torch.zeros(1, device=device)
        try:
            native = rccl.NativeComm.get(channels=channels, proto=proto, algo=algo)
            built += 1
        except RuntimeError as e:  # refused right away on this rank: everybody falls back to c10d
            log.warning(f"native RCCL communicator ({channels or 'default'} channels, protocol "
                        f"{proto or 'default'}, algorithm {algo or 'default'}) unavailable: {e}")
        finally:
            guard.cancel()
        dist.all_reduce(built, op=dist.ReduceOp.MIN)
        if built.item() == 0:
            native = None
        else:
            native = _probe_native(device, native, channels, proto, algo)
    return native


def _probe_native(device, native, channels, proto, algo):
    """One small AVG all-reduce on a freshly built communicator before any timing: a forced
    protocol / algorithm that RCCL cannot serve fails at ENQUEUE time, not at init. The ranks first
    agree (MIN over the c10d group) that EVERY rank enqueued it — a rank whose enqueue failed leaves
    its peers' collective hanging, so they abort the communicator instead of waiting on it
     — then wait, check the average and agree again; a failed arm is dropped on every
    rank."""
    from penroz.parallel import rccl
    arm = (f"native RCCL arm ({channels or 'default'} channels, protocol {proto or 'default'}, "
           f"algorithm {algo or 'default'})")
    enq = torch.zeros(1, device=device)
    t = torch.full((4096,), float(dist.get_rank() + 1), device=device)
    try:
        native.all_reduce_avg_async(t)
        enq += 1
    except RuntimeError as e:
        log.warning(f"{arm} failed to enqueue its probe all-reduce: {e}")
    dist.all_reduce(enq, op=dist.ReduceOp.MIN)
    if enq.item() == 0:
        rccl.NativeComm.drop(channels=channels, proto=proto, algo=algo, abort=True)
        return None
    ok = torch.zeros(1, device=device)
    try:
        native.wait_all()
        _sync(device)
        if bool((t == (dist.get_world_size() + 1) / 2.0).all()):
            ok += 1
    except RuntimeError as e:
        log.warning(f"{arm} failed its probe all-reduce: {e}")
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if ok.item() > 0:
        return native
    rccl.NativeComm.drop(channels=channels, proto=proto, algo=algo)
    return None


def sweep(device: torch.device, sizes_mb=SWEEP_SIZES_MB, wires=("fp32", "bf16"), transports=("c10d", "native"),
          iters: int = 3, warmup: int = 1, channels=(0,), protos=("",), algos=("",),
          budget_s: float | None = None, stats: dict | None = None) -> list[dict]:
    """Time every (transport, wire, bucket size); max over ranks; correctness-checked.

    ``channels``: the native communicator is swept once per channel count (0 = RCCL's own
    choice; others build a communicator with exactly that many channels — the per-communicator
    form of ``NCCL_MIN/MAX_NCHANNELS``); ``protos``: at the first channel count, once more per
    forced protocol (the per-communicator form of ``NCCL_PROTO``) and per forced algorithm
    (``NCCL_ALGO``). The extra arms are swept at fp32 only. Every row says which (``channels`` /
    ``proto`` / ``algo``: None for c10d, "" = RCCL's).

    Arms run one after another: each native arm is built, probed (:func:`_probe_native`), timed at
    every size and — unless it is the first (RCCL-default) arm — destroyed right away, so at most
    two native communicators are alive at once. ``budget_s`` (default ``SWEEP_BUDGET_S``) caps the
    sweep's wall time: an arm that would start after it is spent is skipped on every rank (the
    elapsed time is MAX-agreed). ``stats`` (a dict) receives ``wall_s``, ``arms_run``,
    ``arms_skipped`` and ``arms_failed``.

    The input on rank r is r + 1 everywhere, so the average is (n + 1) / 2 exactly in fp32 and
    bf16 (n ≤ 255); ``ok`` records whether the result matched on every rank."""
    world, rank = dist.get_world_size(), dist.get_rank()
    gloo = dist.get_backend() != "nccl"
    budget = SWEEP_BUDGET_S if budget_s is None else budget_s
    t_start = time.perf_counter()
    st = stats if stats is not None else {}
    st.update(arms_run=[], arms_skipped=[], arms_failed=[])
    expect = (world + 1) / 2.0
    arms = [(tr, None) for tr in transports if tr != "native"]
    if "native" in transports:
        arms += [("native", (ch, protos[0], algos[0])) for ch in channels]
        arms += [("native", (channels[0], pr, algos[0])) for pr in protos[1:]]
        arms += [("native", (channels[0], protos[0], al)) for al in algos[1:]]
    default_arm = (channels[0], protos[0], algos[0])
    rows = []
    native_dead = False
    for tr, key in arms:
        label = tr if key is None else f"native:{key[0] or 'default'}/{key[1] or 'default'}/{key[2] or 'default'}"
        spent = torch.tensor([time.perf_counter() - t_start], dtype=torch.float64, device=device)
        dist.all_reduce(spent, op=dist.ReduceOp.MAX)
        if spent.item() > budget or (tr == "native" and native_dead):
            st["arms_skipped"].append(label)
            continue
        native = None
        if tr == "native":
            native = _native_or_none(device, *key)
            if native is None:
                st["arms_failed"].append(label)
                if key == default_arm:
                    native_dead = True  # the communicator cannot be built at all
                continue
        st["arms_run"].append(label)
        ch, pr, al = key if key is not None else (None, None, None)
        for wire in wires:
            if tr == "native" and wire != "fp32" and key != default_arm:
                continue
            dt = {"fp32": torch.float32, "bf16": torch.bfloat16}[wire]
            for mb in sizes_mb:
                n = int(mb * 2**20) // 4  # elements of an fp32 gradient bucket of that size
                buf = torch.empty(n, device=device, dtype=dt)

                def one():
                    if tr == "native":
                        native.all_reduce_avg_async(buf)
                        native.wait_all()
                    elif gloo:
                        dist.all_reduce(buf)
                        buf.div_(world)
                    else:
                        dist.all_reduce(buf, op=dist.ReduceOp.AVG)

                buf.fill_(rank + 1)
                one()
                _sync(device)
                good = torch.tensor([1.0 if bool((buf == expect).all()) else 0.0], device=device)
                for _ in range(max(0, warmup - 1)):
                    one()
                _sync(device)
                dist.barrier()
                t0 = time.perf_counter()
                for _ in range(iters):
                    one()
                _sync(device)
                dist.barrier()
                t = torch.tensor([(time.perf_counter() - t0) / iters], dtype=torch.float64, device=device)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                dist.all_reduce(good, op=dist.ReduceOp.MIN)
                sec = float(t.item())
                nbytes = buf.numel() * buf.element_size()
                alg = nbytes / sec / 1e9
                rows.append({"transport": tr, "channels": ch, "proto": pr, "algo": al, "wire": wire, "bucket_mb": mb,
                             "ms": round(sec * 1e3, 4),
                             "algbw_GBps": round(alg, 2), "busbw_GBps": round(alg * 2 * (world - 1) / world, 2),
                             "ok": bool(good.item() > 0)})
                del buf
        if tr == "native" and key != default_arm:
            from penroz.parallel import rccl
            del native
            rccl.NativeComm.drop(channels=key[0], proto=key[1], algo=key[2])
    st["wall_s"] = round(time.perf_counter() - t_start, 3)
    st["budget_s"] = budget
    return rows


def _arm_key(r) -> tuple:
    """A native row's arm: (channel count, protocol, algorithm); "" = RCCL's own choice."""
    return (r.get("channels", 0), r.get("proto") or "", r.get("algo") or "")


def _arm_rows(rows, transport, channels, wire="fp32", proto="", algo=""):
    return [r for r in rows if r["transport"] == transport and r["wire"] == wire and r["ok"]
            and (transport != "native" or _arm_key(r) == (channels, proto, algo))]


def plan(rows: list[dict], grad_bytes: int, backward_ms: float | None = None, margin: float = 1.03,
         bf16_gain: float = 1.2, auto_bf16: bool = False) -> dict:
    """The whole gradient-sync configuration from one sweep, each transport judged at ITS OWN size:

    1. every correct (transport, channel count) arm gets its bucket size from :func:`choose_bucket`'s
       rule (the smallest size within 90 % of that arm's best bus bandwidth);
    2. the native communicator wins only if its best arm's bus bandwidth, at that arm's size, is
       ≥ ``margin`` × c10d's at c10d's size (the channel count comes with the arm);
    3. the wire: always fp32 (the reference DDP's numerics) unless ``auto_bf16``. The bf16 wire is
       RECOMMENDED (``wire_recommendation``) when the predicted fp32 all-reduce of the whole
       gradient (``grad_bytes`` / algbw at the chosen size) exceeds ``backward_ms`` — it could not
       hide behind the backward — and the bf16 wire of the same transport, correct at that size,
       is ≥ ``bf16_gain`` × faster for the whole gradient; only ``auto_bf16`` applies it (the user
       opts in with ``PENROZ_GRAD_WIRE=bf16``; a bf16 wire changes gradient numerics).

    The native arms are (channel count, protocol, algorithm) triples; the winning arm brings all three.

    Returns {"transport", "channels", "proto", "algo", "bucket_mb", "wire", "predicted_fp32_ms", ...,
    "reason"}."""
    out = {"transport": "c10d", "channels": None, "proto": None, "algo": None, "bucket_mb": None, "wire": "fp32"}
    c_rows = _arm_rows(rows, "c10d", None)
    if not c_rows:
        out["reason"] = "no correct c10d rows"
        return out
    arms = {("c10d", None, None, None): c_rows}
    for ch, pr, al in sorted({_arm_key(r) for r in rows if r["transport"] == "native"}):
        nr = _arm_rows(rows, "native", ch, proto=pr, algo=al)
        if nr:
            arms[("native", ch, pr, al)] = nr
    picked = {}
    for key, ar in arms.items():
        best = max(r["busbw_GBps"] for r in ar)
        pick = min((r for r in ar if r["busbw_GBps"] >= 0.9 * best), key=lambda r: r["bucket_mb"])
        picked[key] = pick
    c = picked[("c10d", None, None, None)]
    nat = [(k, r) for k, r in picked.items() if k[0] == "native"]
    choice_key, choice = ("c10d", None, None, None), c
    if nat:
        nk, nr = max(nat, key=lambda kv: kv[1]["busbw_GBps"])
        if nr["busbw_GBps"] >= margin * c["busbw_GBps"]:
            choice_key, choice = nk, nr
        out["reason"] = (f"native ({nk[1] or 'default'} channels, protocol {nk[2] or 'default'}, algorithm "
                         f"{nk[3] or 'default'}) {nr['busbw_GBps']} GB/s at {nr['bucket_mb']} MB vs c10d "
                         f"{c['busbw_GBps']} GB/s at {c['bucket_mb']} MB")
    else:
        out["reason"] = "no correct native arm"
    out.update(transport=choice_key[0], channels=choice_key[1], proto=choice_key[2], algo=choice_key[3],
               bucket_mb=choice["bucket_mb"], busbw_GBps=choice["busbw_GBps"])
    fp32_ms = grad_bytes / (choice["algbw_GBps"] * 1e9) * 1e3
    out["predicted_fp32_ms"] = round(fp32_ms, 3)
    bf = [r for r in rows if r["transport"] == choice_key[0] and r["wire"] == "bf16" and r["ok"]
          and r["bucket_mb"] == choice["bucket_mb"]
          and (choice_key[0] != "native" or _arm_key(r) == choice_key[1:])]
    if bf:
        bf16_ms = (grad_bytes / 2) / (bf[0]["algbw_GBps"] * 1e9) * 1e3
        out["predicted_bf16_ms"] = round(bf16_ms, 3)
        if backward_ms is not None and fp32_ms > backward_ms and fp32_ms >= bf16_gain * bf16_ms:
            out["wire_recommendation"] = "bf16"
            if auto_bf16:
                out["wire"] = "bf16"
            out["wire_reason"] = (f"fp32 all-reduce {fp32_ms:.1f} ms > backward {backward_ms:.1f} ms; "
                                  f"bf16 {bf16_ms:.1f} ms")
    out.setdefault("wire_recommendation", "fp32")
    if "wire_reason" not in out:
        out["wire_reason"] = ("no backward estimate" if backward_ms is None else
                              f"fp32 all-reduce {fp32_ms:.1f} ms vs backward {backward_ms:.1f} ms")
    return out


def choose(rows: list[dict], bucket_mb: float, margin: float = 1.03) -> dict:
    """Transport for the fp32 gradient all-reduce at ``bucket_mb`` (the nearest swept size):
    native only if it was correct and ≥ ``margin`` × c10d's bus bandwidth there."""
    fp = [r for r in rows if r["wire"] == "fp32"]
    if not fp:
        return {"transport": "c10d", "reason": "no sweep"}
    size = min({r["bucket_mb"] for r in fp}, key=lambda s: abs(s - bucket_mb))
    at = {r["transport"]: r for r in fp if r["bucket_mb"] == size}
    c, n = at.get("c10d"), at.get("native")
    if c is None:
        return {"transport": "c10d", "reason": "c10d not swept"}
    if n is None:
        return {"transport": "c10d", "reason": "native communicator unavailable", "at_mb": size}
    if not n["ok"]:
        return {"transport": "c10d", "reason": "native all-reduce result wrong", "at_mb": size}
    if n["busbw_GBps"] >= margin * c["busbw_GBps"]:
        return {"transport": "native", "reason": f"native {n['busbw_GBps']} vs c10d {c['busbw_GBps']} GB/s",
                "at_mb": size}
    return {"transport": "c10d", "reason": f"native {n['busbw_GBps']} vs c10d {c['busbw_GBps']} GB/s", "at_mb": size}


def choose_bucket(rows: list[dict], transport: str, frac: float = 0.9) -> dict | None:
    """Gradient bucket size for ``transport``: the SMALLEST swept fp32 size whose bus bandwidth
    is within ``frac`` of the best one. On point-to-point xGMI a ring all-reduce is per-link bound,
    so past the size where the links saturate a bigger bucket only starts its collective later in
    the backward (and leaves more bytes exposed after it); below it, per-call latency dominates.
    The sweep's timings are MAX-reduced over ranks, so every rank picks the same size (the bucket
    plans must match). None when nothing correct was swept for ``transport``."""
    fp = [r for r in rows if r["wire"] == "fp32" and r["transport"] == transport and r["ok"]]
    if not fp:
        return None
    best = max(r["busbw_GBps"] for r in fp)
    pick = min((r for r in fp if r["busbw_GBps"] >= frac * best), key=lambda r: r["bucket_mb"])
    return {"bucket_mb": pick["bucket_mb"], "busbw_GBps": pick["busbw_GBps"], "best_busbw_GBps": best,
            "rule": f"smallest size within {frac:.0%} of the best bus bandwidth"}
