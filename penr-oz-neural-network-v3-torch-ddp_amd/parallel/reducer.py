"""Bucketed, backward-overlapped gradient all-reduce over a flat fp32 gradient buffer.

Replaces the reference's implicit C++ DDP ``Reducer`` (``neural_net_model.py:609``: 25 MB fp32
buckets, autograd hooks, all-reduce during backward).  Design for 8×MI355X / xGMI:

* gradients live in ONE flat buffer whose layout follows *backward completion order*
  (lm_head first … token embedding last), so a bucket is a contiguous slice and needs no
  pack/unpack copy;
* bucket boundaries fall on layer boundaries and default to ≥ 64 MB
  (``PENROZ_BUCKET_MB``): xGMI is 7 point-to-point links of ≈153 GB/s, so a ring collective is
  per-link bound and small buckets waste launches/latency; 64 MB keeps ~10 buckets in flight
  behind a GPT-2 124M backward;
* as soon as the executor (or the autograd hooks, for generic models) finishes the layers of
  a bucket, ``bucket_ready(i)`` launches its all-reduce asynchronously on the communicator's
  own stream (RCCL), ordered after the producing kernels by a stream event, so it overlaps
  the rest of the backward; ``finish()`` makes the compute stream wait for all of them
  before the optimizer step;
* ``no_sync`` micro-steps: the caller simply does not call ``bucket_ready`` until the last;
* optional bf16 wire format (``PENROZ_GRAD_WIRE=bf16``): a bucket is cast to a bf16 staging
  buffer on the compute stream, all-reduced in bf16 (half the xGMI bytes), and cast back into
  the fp32 gradient buffer in ``finish()``; accumulation and the optimizer stay fp32.

Transport: ``torch.distributed`` with the ``nccl`` backend (= RCCL on ROCm; the reference's
``ProcessGroupNCCL`` call pattern is *not* replicated — one async all-reduce per bucket with
``ReduceOp.AVG``) or ``gloo`` on CPU.  ``PENROZ_COMM=native`` selects the C++ RCCL
communicator (``csrc/comm/rccl_comm.cpp``: own ``ncclComm_t``, high-priority HIP stream).
"""
from __future__ import annotations

import logging
import os

import torch
import torch.distributed as dist

log = logging.getLogger(__name__)

DEFAULT_BUCKET_MB = float(os.environ.get("PENROZ_BUCKET_MB", "64"))
# gloo (CPU plumbing config): the reference DDP's 25 MB, so the first buckets' TCP transfers start
# early in the backward (64 MB buckets left ≈ 500 ms of a 1.9 s CPU step exposed, 25 MB ≈ 310 ms:
# profiles/bench_r3_cpu_gloo_ws2_t64.log)
GLOO_BUCKET_MB = float(os.environ.get("PENROZ_BUCKET_MB", "25"))


def default_bucket_mb(backend: str | None) -> float:
    """PENROZ_BUCKET_MB read at call time (the multi-GPU bench sets it from its first-contact
    all-reduce sweep, parallel/commtune.py: choose_bucket), else the per-backend default."""
    env = os.environ.get("PENROZ_BUCKET_MB")
    if env is not None:
        return float(env)
    return GLOO_BUCKET_MB if backend == "gloo" else DEFAULT_BUCKET_MB
WIRE_DTYPES = {"fp32": None, "bf16": torch.bfloat16}


def plan_buckets(segments: list[tuple[int, int]], bucket_bytes: float, elem_size: int = 4) -> list[tuple[int, int]]:
    """Group consecutive (start, end) element segments into buckets of >= ``bucket_bytes``."""
    buckets: list[tuple[int, int]] = []
    cur_start, cur_end = None, None
    for s, e in segments:
        if cur_start is None:
            cur_start, cur_end = s, e
        elif s != cur_end:
            buckets.append((cur_start, cur_end))
            cur_start, cur_end = s, e
        else:
            cur_end = e
        if (cur_end - cur_start) * elem_size >= bucket_bytes:
            buckets.append((cur_start, cur_end))
            cur_start = cur_end = None
    if cur_start is not None:
        buckets.append((cur_start, cur_end))
    return buckets


def split_last_bucket(buckets: list[tuple[int, int]], pieces: int, align: int = 64) -> list[tuple[int, int]]:
    """The last bucket (the token / position embeddings, produced by the final kernel of the
    backward, so its all-reduce cannot overlap anything) cut into ``pieces`` consecutive pieces
    (boundaries on ``align``-element multiples): the pieces' all-reduces pipeline with the
    optimizer passes of the pieces that have already landed."""
    if pieces <= 1 or not buckets:
        return list(buckets)
    s, e = buckets[-1]
    n = e - s
    step = max(align, -(-(-(-n // pieces)) // align) * align)  # ceil(ceil(n / pieces) / align) · align
    cuts = list(range(s, e, step)) + [e]
    return list(buckets[:-1]) + [(a, b) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]


def ready_map(buckets: list[tuple[int, int]], segments: list[tuple[int, int]]) -> dict[int, list[int]]:
    """segment index -> the buckets whose last element lies in that segment (a bucket may be
    all-reduced once the segment that completes it is done; every bucket appears once)."""
    out: dict[int, list[int]] = {}
    for i, (_, be) in enumerate(buckets):
        seg = next(j for j, (s, e) in enumerate(segments) if s <= be - 1 < e)
        out.setdefault(seg, []).append(i)
    return out


class GradReducer:
    def __init__(self, flat_grad: torch.Tensor, buckets: list[tuple[int, int]], group=None,
                 wire: str | None = None):
        self.flat_grad = flat_grad
        self.buckets = buckets
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.backend = dist.get_backend(group) if dist.is_initialized() else None
        self._works: list = []
        self._launched = [False] * len(buckets)
        self._native = None
        if self.world > 1 and flat_grad.is_cuda and os.environ.get("PENROZ_COMM", "c10d") == "native":
            from penroz.parallel import rccl
            self._native = rccl.NativeComm.get(group)
        wire = wire or os.environ.get("PENROZ_GRAD_WIRE", "fp32")
        if wire not in WIRE_DTYPES:
            raise ValueError(f"PENROZ_GRAD_WIRE must be one of {sorted(WIRE_DTYPES)}, got {wire!r}")
        wdt = WIRE_DTYPES[wire]
        self._wire = None
        if self.world > 1 and wdt is not None and wdt != flat_grad.dtype:
            self._wire = torch.empty(flat_grad.numel(), dtype=wdt, device=flat_grad.device)
        log.info(f"GradReducer: {len(buckets)} bucket(s) over {flat_grad.numel() * 4 / 2**20:.1f} MiB, "
                 f"world {self.world}, transport {'native-rccl' if self._native else self.backend}, wire {wire}")

    def bucket_of(self, elem_index: int) -> int:
        for i, (s, e) in enumerate(self.buckets):
            if s <= elem_index < e:
                return i
        raise IndexError(elem_index)

    def bucket_ready(self, i: int):
        if self.world == 1 or self._launched[i]:
            self._launched[i] = True
            return
        s, e = self.buckets[i]
        view = self.flat_grad[s:e]
        if self._wire is not None:
            self._wire[s:e].copy_(view)  # cast on the producing stream, then reduce the copy
            view = self._wire[s:e]
        self._launched[i] = True
        if self._native is not None:
            self._works.append(("native", self._native.all_reduce_avg_async(view)))
        elif self.backend == "nccl":
            self._works.append(dist.all_reduce(view, op=dist.ReduceOp.AVG, group=self.group, async_op=True))
        else:
            self._works.append((dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.group, async_op=True), view))

    def launch_remaining(self):
        """Launch every bucket not yet launched (no wait)."""
        for i in range(len(self.buckets)):
            if not self._launched[i]:
                self.bucket_ready(i)

    def per_bucket_waits(self) -> bool:
        """True when :meth:`wait_bucket` can wait for one bucket at a time (every bucket launched,
        in bucket order; c10d work objects or native RCCL completion events)."""
        return len(self._works) == len(self.buckets)

    def stream_waits(self) -> bool:
        """True when :meth:`wait_bucket` only makes the CURRENT STREAM wait (RCCL through c10d or
        the native communicator), so the host can enqueue a bucket's optimizer pass right after
        launching it; gloo waits block the host."""
        return self.world > 1 and (self._native is not None or self.backend == "nccl")

    def wait_bucket(self, i: int) -> tuple[int, int]:
        """Current stream waits for bucket ``i``'s all-reduce (launch order = bucket order);
        returns its element range, now holding the averaged gradient."""
        w = self._works[i]
        if isinstance(w, tuple) and w[0] == "native":
            self._native.wait(w[1])
        elif isinstance(w, tuple):
            w[0].wait()
            w[1].div_(self.world)
        else:
            w.wait()
        s, e = self.buckets[i]
        if self._wire is not None:
            self.flat_grad[s:e].copy_(self._wire[s:e])
        return s, e

    def reset(self):
        self._works.clear()
        self._launched = [False] * len(self.buckets)
        if self._native is not None:
            self._native.reset_handles()

    def finish(self):
        """Launch any bucket not yet launched, then wait for all of them."""
        for i in range(len(self.buckets)):
            if not self._launched[i]:
                self.bucket_ready(i)
        if self._native is not None:
            self._native.wait_all()
        for w in self._works:
            if isinstance(w, tuple) and w[0] == "native":
                continue
            if isinstance(w, tuple):
                w[0].wait()
                w[1].div_(self.world)
            else:
                w.wait()
        self._works.clear()
        if self._wire is not None:
            for s, e in self.buckets:
                self.flat_grad[s:e].copy_(self._wire[s:e])
        self._launched = [False] * len(self.buckets)

    def broadcast_params(self, flat_param: torch.Tensor, src: int = 0):
        """Rank-0 parameter broadcast at start (DDP ctor semantics, one collective)."""
        if self.world > 1:
            if self._native is not None:
                self._native.broadcast(flat_param, src)
            else:
                dist.broadcast(flat_param, src=src, group=self.group)


def row_sparse_tables(model: torch.nn.Module) -> list[torch.nn.Parameter]:
    """Embedding weights whose gradient is row-sparse: owned by one ``nn.Embedding`` (dense
    gradient) and used by no other module — a tied lm_head makes the table's gradient dense."""
    uses: dict[int, int] = {}
    for mod in model.modules():
        for p in mod.parameters(recurse=False):
            uses[id(p)] = uses.get(id(p), 0) + 1
    return [m.weight for m in model.modules()
            if isinstance(m, torch.nn.Embedding) and not m.sparse and m.max_norm is None
            and m.weight.requires_grad and uses.get(id(m.weight)) == 1]


def sparse_rows_enabled(backend: str | None) -> bool:
    """PENROZ_SPARSE_EMBED_GRAD=1/0 forces it; default on for gloo (host memory bandwidth and TCP
    make the dense 147 MB token table the largest single cost of the CPU plumbing step) and off
    for RCCL (at 64k tokens per rank nearly every row of a 50k vocabulary is touched)."""
    env = os.environ.get("PENROZ_SPARSE_EMBED_GRAD")
    if env is not None:
        return env != "0"
    return backend == "gloo"


class HookedReducer:
    """Generic-model reducer: autograd post-accumulate hooks mark parameters ready.

    Parameters' ``.grad`` are views of one flat buffer laid out in reverse registration order
    (≈ backward order); a bucket launches when all its parameters have accumulated.
    """

    def __init__(self, params: list[torch.nn.Parameter], bucket_mb: float | None = None, group=None,
                 sparse_rows: list[torch.nn.Parameter] | None = None):
        backend = dist.get_backend(group) if dist.is_initialized() else None
        if bucket_mb is None:
            bucket_mb = default_bucket_mb(backend)
        self.params = [p for p in params if p.requires_grad]
        order = list(reversed(self.params))
        total = sum(p.numel() for p in order)
        dev, dtype = order[0].device, order[0].dtype
        self.flat_grad = torch.zeros(total, device=dev, dtype=dtype)
        self.offsets = {}
        # row-sparse tables (embedding weights used by nothing else): reduced over the union of the
        # rows any rank touched instead of densely (see _reduce_rows); excluded from the buckets
        ids = {id(p) for p in (sparse_rows or [])}
        self.sparse = [p for p in order if id(p) in ids and p.dim() == 2]
        segments = []
        off = 0
        esz = self.flat_grad.element_size()
        # a parameter larger than a bucket is cut into bucket-sized pieces, each its own bucket
        # (the CPU plumbing config's 147 MB lm_head weight: one collective of that size held every
        # later bucket behind it); all pieces launch when the parameter's gradient lands
        piece = max(1, int(bucket_mb * 2**20) // esz)
        if os.environ.get("PENROZ_SPLIT_BIG_PARAMS", "1") == "0":  # A/B: whole parameters only
            piece = 1 << 62
        for p in order:
            n = p.numel()
            self.offsets[p] = off
            if not any(p is q for q in self.sparse):
                if n > piece:
                    segments.extend((s0, min(off + n, s0 + piece)) for s0 in range(off, off + n, piece))
                else:
                    segments.append((off, off + n))
            off += n
        self.reducer = GradReducer(self.flat_grad, plan_buckets(segments, bucket_mb * 2**20, esz), group)
        self.group = group
        self._param_bucket = {}  # parameter -> the buckets holding (pieces of) its gradient
        for p in order:
            if any(p is q for q in self.sparse):
                self._param_bucket[p] = []
                continue
            first = self.reducer.bucket_of(self.offsets[p])
            last = self.reducer.bucket_of(self.offsets[p] + p.numel() - 1)
            self._param_bucket[p] = list(range(first, last + 1))
        self._rows_pending: list = []
        self.sync = True
        self._handles = [p.register_post_accumulate_grad_hook(self._hook) for p in order]
        self.attach_grads()

    def attach_grads(self):
        for p in self.params:
            off = self.offsets[p]
            p.grad = self.flat_grad[off:off + p.numel()].view_as(p)
        self._reset_counts()

    def _reset_counts(self):
        self._pending = [0] * len(self.reducer.buckets)
        for p in self.params:
            for b in self._param_bucket[p]:
                self._pending[b] += 1

    def _hook(self, p):
        if not self.sync:
            return
        # (row-sparse tables hold no bucket: they reduce in finish(), same order on every rank)
        for b in self._param_bucket[p]:
            self._pending[b] -= 1
            if self._pending[b] == 0:
                self.reducer.bucket_ready(b)

    def _reduce_rows(self, p):
        """All-reduce only the rows of ``p.grad`` that some rank touched: one small all-reduce of
        the row mask, then the union rows packed into one buffer. Exact: a row no rank touched is
        zero everywhere. The token table of the CPU plumbing config (T = 64, B = 4) is 256 of 50304
        rows per rank, so its 147 MB of fp32 gradient go over gloo as ≈ 1.5 MB."""
        if self.reducer.world == 1:
            return
        g = self.flat_grad[self.offsets[p]:self.offsets[p] + p.numel()].view_as(p)
        mask = g.ne(0).any(dim=1).to(torch.int32)
        dist.all_reduce(mask, group=self.group)
        rows = mask.nonzero().squeeze(1)
        packed = g.index_select(0, rows)
        work = dist.all_reduce(packed, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        self._rows_pending.append((work, g, rows, packed))

    def finish(self):
        if self.sync:
            self.reducer.launch_remaining()
            for p in self.sparse:
                self._reduce_rows(p)
            self.reducer.finish()
            for work, g, rows, packed in self._rows_pending:
                work.wait()
                g.index_copy_(0, rows, packed.div_(self.reducer.world))
            self._rows_pending.clear()
        self._reset_counts()

    def zero_grad(self):
        self.flat_grad.zero_()
        for p in self.params:  # a set_to_none elsewhere must not detach the views
            off = self.offsets[p]
            if p.grad is None or p.grad.data_ptr() != self.flat_grad[off:].data_ptr():
                p.grad = self.flat_grad[off:off + p.numel()].view_as(p)

    def remove(self):
        for h in self._handles:
            h.remove()
