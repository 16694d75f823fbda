"""Fused GPT-2 training/eval executor for MI355X.

A layer list that matches the GPT-2 pattern of the reference's example/HF-import layout
(``main.py:57-83``, ``mappers.py:122-176``) is *lowered* to this executor while the
``nn.Module`` tree (and therefore every state_dict key) stays exactly as compiled.  Instead of
per-module autograd it runs an explicit forward and backward:

forward, per layer (N = B·T tokens, fp32 residual stream — the reference's autocast numerics)
  LN1 (HIP, → bf16) → QKV GEMM+bias (hipBLASLt) → flash attention (HIP, reads the fused QKV
  tensor, writes head-merged O + LSE) → proj GEMM+bias → residual-add+LN2 (one HIP pass)
  → fc GEMM+bias (hipBLASLt) → GELU (HIP elementwise kernel writing the activation; the
  pre-activation is kept for the backward) → fc2 GEMM+bias → (residual-add fused into the next LN)
head: final LN → lm_head GEMM → cross-entropy (HIP: one LDS-resident pass per row, writes
  the logits gradient in place, no fp32 logits). The head can run in token chunks
  (``_head_chunk_rows``: automatic above 8 GiB of logits, or ``PENROZ_HEAD_CHUNK`` rows):
  lm_head GEMM → CE → dgrad → wgrad per chunk over two rotating chunk buffers, so the [N, V]
  logits tensor is never materialised (the reference's ``F.cross_entropy`` over full logits,
  ``neural_net_model.py:263-267``).
backward mirrors it: dgrad/wgrad GEMMs (wgrad accumulated in fp32), GELU backward fused with
  the fc bias-gradient column sum, LayerNorm backward fused with dγ/dβ, the residual-gradient
  accumulation, its bf16 copy for the next GEMM, and the bias gradient of the preceding
  linear; flash-attention backward with the qkv bias gradient summed in its epilogues; embedding
  backward (dwte scatter, dwpe reduction).

Dropout (the HF GPT-2 import: embd/resid/attn_pdrop = 0.1, ``mappers.py:140-142`` in the
reference): attention dropout runs inside the flash kernels; embedding dropout inside the
embedding kernels; each residual branch's dropout inside the add+LayerNorm kernel that adds it
to the stream, and the LayerNorm backward applies the regenerated mask to the branch gradient.
Masks are hashed from (step seed, site, element) and never stored.

bf16-parameter models (``/import/`` loads HF weights in bf16, ``neural_net_model.py:222``) train
here too: the executor keeps fp32 master copies and makes the module parameters views of the
bf16 shadow the fused AdamW rewrites every step, so ``state_dict()`` stays bf16 (the checkpoint
dtype of the reference) while the update itself is fp32.

Parameters, gradients and AdamW moments live in flat fp32 buffers laid out in backward
completion order (lm_head … wte) so gradient buckets are contiguous slices: the reducer
launches each bucket's RCCL all-reduce as soon as the layers in it finish, overlapped with
the remaining backward.  A flat bf16 shadow of every parameter feeds the GEMMs and is
refreshed by the fused AdamW kernel in the same pass that updates the fp32 masters.
"""
from __future__ import annotations

import logging
import math
from dataclasses import dataclass, field

import torch
import torch.nn as nn
from torch import Tensor

from penroz.models import layers as L
from penroz.ops import attention as attn_ops
from penroz.ops import activations as act_ops
from penroz.ops import fused as fused_ops
from penroz.ops import norms as norm_ops
from penroz.ops import gemm as gemm_ops
from penroz.utils.profiling import trace_range
from penroz.ops import _ext

log = logging.getLogger(__name__)


@dataclass
class _Block:
    ln1: nn.LayerNorm
    qkv: nn.Linear
    attn: L.CausalSelfAttention
    proj: nn.Linear
    ln2: nn.LayerNorm
    fc: nn.Linear
    act: nn.GELU
    fc2: nn.Linear
    p_attn_res: float = 0.0  # dropout on the attention branch (after proj)
    p_mlp_res: float = 0.0   # dropout on the MLP branch (after fc2)


@dataclass
class GPTSpec:
    V: int
    C: int
    H: int
    D: int
    F: int
    P: int
    wte: nn.Embedding
    wpe: L.PositionEmbedding
    blocks: list = field(default_factory=list)
    lnf: nn.LayerNorm = None
    head: nn.Linear = None
    gelu_approx: str = "none"
    p_embd: float = 0.0
    param_dtype: torch.dtype = torch.float32


def _is(m, cls):
    return isinstance(m, cls)


def _dropout_ok(m) -> bool:
    return _is(m, nn.Dropout) and 0.0 <= m.p < 1.0


# residual-dropout mask streams: one per (step seed, site); attention dropout uses seed + layer
def _head_chunk_rows(N: int, V: int) -> int:
    """Token rows per lm_head/CE chunk.

    ``PENROZ_HEAD_CHUNK`` = rows (0 = one chunk of all N rows). Unset: one chunk while the bf16
    [N, V] logits fit in ``PENROZ_HEAD_CHUNK_AUTO_GB`` (default 8 GiB), else chunks of ≈ 2 GiB.
    Chunking trades time for memory on MI355X (GPT-2 124M headline, N = 65 536:
    ``profiles/head_chunk_r2_sweep.log``): 67.7 ms/step unchunked, 68.7 at 16 384 rows, 69.1 at
    8 192, 76.3 at 4 096 (per-chunk wgrad accumulation and untuned GEMM shapes), while the 6.6 GB
    logits are < 3 % of the 288 GB HBM, so the full tensor stays the default at that size.
    """
    import os
    env = os.environ.get("PENROZ_HEAD_CHUNK")
    if env is not None:
        c = int(env)
    else:
        row_bytes = ((V + 7) // 8 * 8) * 2
        limit = float(os.environ.get("PENROZ_HEAD_CHUNK_AUTO_GB", "8")) * 2**30
        c = 0 if N * row_bytes <= limit else max(1024, int(2 * 2**30 // row_bytes) // 1024 * 1024)
    return N if c <= 0 or c >= N else c


def _site_seed(seed: int, site: int) -> int:
    return (seed * 1_000_003 + 7_919 * (site + 1) + 0x5BD1E995) & 0x7FFFFFFFFFFFFFFF


def _minus(ranges, cut):
    """[(a, b)] ranges with the range ``cut`` (or None) removed."""
    if cut is None:
        return list(ranges)
    c0, c1 = cut
    out = []
    for a, b in ranges:
        if a < c0:
            out.append((a, min(b, c0)))
        if b > c1:
            out.append((max(a, c1), b))
    return [(a, b) for a, b in out if b > a]


def cu_mask_words(spec: str, n_cu: int) -> list[int]:
    """CU mask words for PENROZ_SIDE_CUS: ``stride:k[:o]`` = CUs i with i % k == o, ``first:n`` =
    CUs 0..n-1 (bit i of word i // 32 = CU i)."""
    kind, _, rest = spec.partition(":")
    if kind == "stride":
        k, _, o = rest.partition(":")
        sel = [i for i in range(n_cu) if i % int(k) == int(o or 0)]
    elif kind == "first":
        sel = list(range(min(int(rest), n_cu)))
    else:
        raise ValueError(f"PENROZ_SIDE_CUS: want stride:k[:o] or first:n, got {spec!r}")
    if not sel:
        raise ValueError(f"PENROZ_SIDE_CUS={spec!r} selects no CU")
    words = [0] * ((n_cu + 31) // 32)
    for i in sel:
        words[i // 32] |= 1 << (i % 32)
    return words


def _cu_masked_stream(device: torch.device, spec: str):
    """The side stream confined to a CU subset (A/B of critical-path GEMM interference)."""
    k = _ext.kernels()
    idx = device.index if device.index is not None else torch.cuda.current_device()
    ptr = k.cu_masked_stream(idx, cu_mask_words(spec, k.cu_count(idx)))
    return torch.cuda.ExternalStream(ptr, device=device)


_HP_STREAMS: dict = {}
_SHARED_STREAMS: dict = {}


def shared_stream(device: torch.device, role: str):
    """ONE stream per (device, role) for the whole process — the executors' weight-gradient side
    stream ("side"), the per-bucket optimizer stream ("opt") and the input-copy stream ("copy").
    Every extra stream drawn from torch's pool is mapped onto one of the device's few hardware
    queues (GPU_MAX_HW_QUEUES = 4), and which streams end up sharing a queue depends on how many
    were drawn before: a copy stream created before a second model's executor cut that model's
    step from 0.98 to 0.88 of the first's (bench.py --via-runtime, profiles/notes_r6.md). Shared
    streams keep a later executor on the first one's queues; sharing only adds ordering."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    st = _SHARED_STREAMS.get((idx, role))
    if st is None:
        st = _SHARED_STREAMS[(idx, role)] = torch.cuda.Stream(device=torch.device("cuda", idx))
    return st


def _high_priority_stream(device: torch.device):
    """ONE high-priority stream per device for every executor of the process. A second executor
    drawing a second stream from torch's high-priority pool (a later model in the same process —
    the server's worker, bench.py --via-runtime) ran the headline step at 65.4-65.5 ms instead of
    61.2-61.3: the second stream does not get the first one's queue priority, and the side stream's
    weight-gradient GEMMs then delay the dgrad chain (11 main-queue stalls of 0.3-0.56 ms before
    LayerNorm backward per step); with PENROZ_MAIN_PRIORITY=0 the second run matched the first
    (bench/runtime_ab.py, profiles/notes_r6.md). Sharing the stream only adds ordering between
    executors, never removes it."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    hp = _HP_STREAMS.get(idx)
    if hp is None:
        lo, hi = torch.cuda.Stream.priority_range()
        hp = _HP_STREAMS[idx] = torch.cuda.Stream(device=torch.device("cuda", idx), priority=min(lo, hi))
    return hp


class GPTExecutor:
    # ------------------------------------------------------------------ pattern match
    @staticmethod
    def match(model, require_fp32: bool = False) -> GPTSpec | None:
        """The GPT-2 block structure, with fp32 or bf16 parameters (one dtype for all; the
        executor keeps fp32 masters either way). ``require_fp32``: fp32 parameters only."""
        ls = list(model.layers)
        if len(ls) < 5:
            return None
        emb = ls[0]
        if not (_is(emb, L.Summation) and len(emb) == 2 and type(emb[0]) is nn.Embedding
                and _is(emb[1], L.PositionEmbedding)):
            return None
        if not _dropout_ok(ls[1]):
            return None
        tail = ls[-3:] if _is(ls[-1], L.SoftmaxOnLast) else ls[-2:]
        if len(tail) < 2 or not _is(tail[0], nn.LayerNorm) or not _is(tail[1], nn.Linear) or tail[1].bias is not None:
            return None
        body = ls[2:len(ls) - len(tail)]
        if not body:
            return None
        C = emb[0].embedding_dim
        spec = GPTSpec(V=emb[0].num_embeddings, C=C, H=0, D=0, F=0, P=emb[1].num_embeddings,
                       wte=emb[0], wpe=emb[1], lnf=tail[0], head=tail[1])
        approx = None
        for blk in body:
            if not (_is(blk, L.ResidualConnection) and len(blk) == 2):
                return None
            a, m = blk[0], blk[1]
            if not (_is(a, nn.Sequential) and len(a) == 5 and _is(m, nn.Sequential) and len(m) == 5):
                return None
            ln1, qkv, att, proj, d1 = a
            ln2, fc, act, fc2, d2 = m
            ok = (_is(ln1, nn.LayerNorm) and _is(qkv, nn.Linear) and _is(att, L.CausalSelfAttention)
                  and _is(proj, nn.Linear) and _dropout_ok(d1) and _is(ln2, nn.LayerNorm)
                  and _is(fc, nn.Linear) and _is(act, nn.GELU) and _is(fc2, nn.Linear) and _dropout_ok(d2))
            if not ok:
                return None
            if att.rope_theta is not None or att.num_kv_heads != att.num_heads or not 0.0 <= att.dropout < 1.0:
                return None
            H = att.num_heads
            D = C // H
            if (qkv.in_features, qkv.out_features) != (C, 3 * C) or (proj.in_features, proj.out_features) != (C, C):
                return None
            if fc.in_features != C or fc2.out_features != C or fc2.in_features != fc.out_features:
                return None
            if any(x.bias is None for x in (qkv, proj, fc, fc2)) or any(
                    x.weight is None or x.bias is None or tuple(x.normalized_shape) != (C,) for x in (ln1, ln2)):
                return None
            if approx is None:
                approx = act.approximate
            if act.approximate != approx:
                return None
            spec.H, spec.D, spec.F = H, D, fc.out_features
            spec.blocks.append(_Block(ln1, qkv, att, proj, ln2, fc, act, fc2, float(d1.p), float(d2.p)))
        if spec.D not in attn_ops.SUPPORTED_HEAD_DIMS or C % 64 != 0 or spec.F % 64 != 0:
            return None
        if tuple(spec.lnf.normalized_shape) != (C,) or spec.head.in_features != C:
            return None
        dtypes = {p.dtype for p in model.parameters()}
        if len(dtypes) != 1 or not dtypes <= ({torch.float32} if require_fp32 else {torch.float32, torch.bfloat16}):
            return None
        spec.param_dtype = dtypes.pop()
        spec.p_embd = float(ls[1].p)
        spec.gelu_approx = approx
        return spec

    # ------------------------------------------------------------------ setup
    def __init__(self, model, device):
        spec = self.match(model)
        if spec is None:
            raise ValueError("model does not match the GPT-2 pattern")
        _ext.kernels()  # hard requirement on GPU
        if device.type == "cuda":
            gemm_ops.load_tuned_gemms()
        self.model = model
        self.spec = spec
        self.device = device
        self.L = len(spec.blocks)
        self._flatten()
        self._acts_shape = None
        self.reducer = None
        self._captured = None
        self._step_seed = 0
        self._reduce_pending = False
        import os
        self._overlap_opt = os.environ.get("PENROZ_OVERLAP_OPT", "1") != "0"
        self._opt_apply, self._opt_done = None, False
        self._side_init()

    def _param_order(self):
        s = self.spec
        segs = [[s.head.weight, s.lnf.weight, s.lnf.bias]]
        for b in reversed(s.blocks):
            segs.append([b.fc2.weight, b.fc2.bias, b.fc.weight, b.fc.bias, b.ln2.weight, b.ln2.bias,
                         b.proj.weight, b.proj.bias, b.qkv.weight, b.qkv.bias, b.ln1.weight, b.ln1.bias])
        segs.append([s.wpe.weight, s.wte.weight])
        return segs

    def _flatten(self):
        """Re-point every parameter at a view of flat fp32 / grad / bf16-shadow buffers."""
        segs = self._param_order()
        params = [p for seg in segs for p in seg]
        if len({id(p) for p in params}) != len(params) or len(params) != len(list(self.model.parameters())):
            raise ValueError("executor needs every parameter exactly once (no tying)")
        # zero rows after the lm_head weight (V rounded up to HEAD_PAD): the head GEMMs run at the
        # padded width (the logit rows are padded anyway), the pad rows stay zero (zero gradient,
        # zero update) and the state_dict sees only the first V rows
        pad = {id(self.spec.head.weight): self.head_pad_rows() * self.spec.C} if self.head_pad_rows() else {}
        total = sum(p.numel() + pad.get(id(p), 0) for p in params)
        dev = self.device
        self.flat = torch.empty(total, dtype=torch.float32, device=dev)
        self.flat_grad = torch.zeros(total, dtype=torch.float32, device=dev)
        self.shadow = torch.empty(total, dtype=torch.bfloat16, device=dev)
        self.offsets = {}
        self.segments = []
        bf16_params = self.spec.param_dtype == torch.bfloat16
        off = 0
        for seg in segs:
            start = off
            for p in seg:
                n = p.numel()
                self.flat[off:off + n].copy_(p.data.reshape(-1))
                if bf16_params:
                    # the module sees the bf16 shadow (rewritten by every optimizer step); the
                    # fp32 masters and gradients stay internal (grad(p) / f32(p))
                    p.data = self.shadow[off:off + n].view_as(p)
                else:
                    p.data = self.flat[off:off + n].view_as(p)
                    p.grad = self.flat_grad[off:off + n].view_as(p)
                self.offsets[id(p)] = off
                off += n
                if pad.get(id(p)):
                    self.flat[off:off + pad[id(p)]].zero_()
                    off += pad[id(p)]
            self.segments.append((start, off))
        self.params_in_order = params
        self.refresh_shadow()
        self._init_transposed()
        opt = self.model.optimizer
        if hasattr(opt, "attach_flat") and len(opt.param_groups) == 1:
            opt.attach_flat(params, self.flat, self.flat_grad, self.shadow, [self.offsets[id(p)] for p in params])
            self._opt_flat = True
        else:
            self._opt_flat = False

    # the lm_head weight's rows are padded to a multiple of this (HF GPT-2 V = 50257 -> 50304, the
    # headline's width: hipBLASLt ran the 50257-wide lm_head forward 1.7 ms slower per step, and the
    # transposed dgrad copy needs widths % 64; profiles/notes_r6.md). PENROZ_HEAD_PAD=0: off
    HEAD_PAD = 128

    def head_pad_rows(self) -> int:
        import os
        m = int(os.environ.get("PENROZ_HEAD_PAD", self.HEAD_PAD))
        return (-self.spec.V) % m if m > 0 and self.device.type == "cuda" else 0

    @property
    def Vp(self) -> int:
        """Rows of the padded lm_head weight (= logit columns the head GEMMs produce)."""
        return self.spec.V + self.head_pad_rows()

    def head_w(self) -> Tensor:
        """The bf16 lm_head weight with its zero pad rows, [Vp, C]."""
        off = self.offsets[id(self.spec.head.weight)]
        return self.shadow[off:off + self.Vp * self.spec.C].view(self.Vp, self.spec.C)

    def head_grad(self) -> Tensor:
        off = self.offsets[id(self.spec.head.weight)]
        return self.flat_grad[off:off + self.Vp * self.spec.C].view(self.Vp, self.spec.C)

    def refresh_shadow(self):
        self.shadow.copy_(self.flat)
        # a shadow rebuilt outside the fused optimizer (a new session, weights loaded) makes every
        # transposed dgrad copy stale, including those rebuilt after the last segment AdamW pass
        if getattr(self, "_t_fresh", None):
            self._t_fresh.clear()

    # ---- transposed bf16 weight copies for the data-gradient GEMMs ----------------------------
    # dx = dy·W with W [out, in] as stored reaches 0.94-1.32 PF on hipBLASLt at GPT-2 shapes; with
    # W transposed ([in, out], so both operands are reduction-contiguous as in the forward) it
    # reaches 1.11-1.53 PF (profiles/dgrad_layout_r1.log). With the optimizer fused into the
    # backward, a segment's copies are rebuilt right after its optimizer pass on the side stream
    # (overlapping the rest of the backward; _t_fresh); otherwise — and for anything not yet
    # rebuilt — at the start of the micro-step on the side stream, and the backward's first dgrad
    # waits for them (Gemma-3 1B: the 1.1 ms of transposes sat between the step's last AdamW pass
    # and the next forward, profiles/notes_r5.md). PENROZ_DGRAD_T=0: off.
    def _init_transposed(self):
        import os
        self._tw, self._t_ready, self._t_fresh = {}, None, set()
        if self.device.type != "cuda" or os.environ.get("PENROZ_DGRAD_T", "1") == "0" or not _ext.available():
            return
        s = self.spec
        lins = [s.head] + [l for b in s.blocks for l in (b.qkv, b.proj, b.fc, b.fc2)]
        shape = {id(s.head.weight): (self.Vp, s.C)}  # the head's copy covers its pad rows
        ws = [l.weight for l in lins]
        ws = [w for w in ws if shape.get(id(w), w.shape)[0] % 64 == 0 and shape.get(id(w), w.shape)[1] % 64 == 0]
        self.shadow_t = torch.empty(sum(math.prod(shape.get(id(w), w.shape)) for w in ws), dtype=torch.bfloat16,
                                    device=self.device)
        off = 0
        for w in ws:
            r, c = shape.get(id(w), w.shape)
            self._tw[id(w)] = (w, self.shadow_t[off:off + r * c].view(c, r))
            off += r * c

    def _refresh_transposed(self):
        if not self._tw:
            return
        k = _ext.kernels()
        side = getattr(self, "_side", None)
        todo = [(key, e) for key, e in self._tw.items() if key not in self._t_fresh]
        self._t_fresh.clear()
        if side is None:
            for _, e in todo:
                k.transpose_bf16(self._tw_source(e), e[1])
            return
        if not todo:  # all rebuilt after their segments' optimizer passes (the main stream joined)
            return
        # the copies must see this step's weights: the side stream waits for everything the main
        # stream has queued (the optimizer's shadow refresh). The main stream is captured BEFORE
        # entering the side-stream context — inside it, current_stream() IS the side stream, and
        # waiting on it orders nothing (that was a race: transposes of a half-refreshed shadow)
        main = torch.cuda.current_stream(self.device)
        with torch.cuda.stream(side):
            side.wait_stream(main)
            for _, e in todo:
                k.transpose_bf16(self._tw_source(e), e[1])
            self._t_ready = torch.cuda.Event()
            self._t_ready.record(side)

    def _tw_source(self, entry) -> Tensor:
        return self.head_w() if entry[0] is self.spec.head.weight else self.bf16(entry[0])

    # rebuild a segment's transposed copies right after its optimizer pass: Gemma-3 1B B=8 −0.2 to
    # −0.3 ms, Gemma-4 e2b −0.4 ms; GPT-2 +0.16 / +0.19 ms (its start-of-step transposes already
    # overlap the forward), so the GPT executor keeps them at the step start
    SEGMENT_TRANSPOSE = False

    def _transpose_segment(self, s: int, e: int):
        """Rebuild the transposed dgrad copies of the parameters in flat range [s, e) on the current
        stream, right after that range's optimizer pass (their shadow is final for the next step)."""
        import os
        env = os.environ.get("PENROZ_SEGMENT_TRANSPOSE")  # (A/B: 1 / 0 overrides the class default)
        if not getattr(self, "_tw", None) or not (self.SEGMENT_TRANSPOSE if env is None else env == "1"):
            return
        k = _ext.kernels()
        for key, ent in self._tw.items():
            off = self.offsets.get(key)
            if off is not None and s <= off and off + ent[1].numel() <= e:  # the whole weight is final
                k.transpose_bf16(self._tw_source(ent), ent[1])
                self._t_fresh.add(key)

    def _dgrad_w(self, w: Tensor) -> Tensor:
        """The weight operand of dx = dy·W: the transposed copy (viewed back as [out, in]) or the shadow
        (the lm_head's with its pad rows)."""
        tw = self._tw.get(id(w)) if self._tw else None
        if tw is None:
            return self.head_w() if w is self.spec.head.weight else self.bf16(w)
        if self._t_ready is not None:
            torch.cuda.current_stream(self.device).wait_event(self._t_ready)
            self._t_ready = None
        return tw[1].t()

    def bf16(self, p: Tensor) -> Tensor:
        off = self.offsets[id(p)]
        return self.shadow[off:off + p.numel()].view(p.shape)

    def grad(self, p: Tensor) -> Tensor:
        off = self.offsets[id(p)]
        return self.flat_grad[off:off + p.numel()].view(p.shape)

    def f32(self, p: Tensor) -> Tensor:
        """The fp32 master of ``p`` (``p`` itself for fp32 models)."""
        off = self.offsets[id(p)]
        return self.flat[off:off + p.numel()].view(p.shape)

    # ------------------------------------------------------------------ buffers
    def _alloc(self, B: int, T: int):
        if self._acts_shape == (B, T):
            return
        s, dev = self.spec, self.device
        N, C, F, V = B * T, s.C, s.F, s.V
        bf, f32 = torch.bfloat16, torch.float32
        self.resid = [torch.empty(N, C, dtype=f32, device=dev) for _ in range(self.L + 1)]
        self.resid_mid = [torch.empty(N, C, dtype=f32, device=dev) for _ in range(self.L)]
        self.ln1 = [torch.empty(N, C, dtype=bf, device=dev) for _ in range(self.L)]
        self.ln2 = [torch.empty(N, C, dtype=bf, device=dev) for _ in range(self.L)]
        self.stats = [tuple(torch.empty(N, dtype=f32, device=dev) for _ in range(4)) for _ in range(self.L)]
        self.statsf = (torch.empty(N, dtype=f32, device=dev), torch.empty(N, dtype=f32, device=dev))
        self.qkv = [torch.empty(N, 3 * C, dtype=bf, device=dev) for _ in range(self.L)]
        self.att = [torch.empty(N, C, dtype=bf, device=dev) for _ in range(self.L)]
        self.lse = [torch.empty(B, s.H, T, dtype=f32, device=dev) for _ in range(self.L)]
        self.fcpre = [torch.empty(N, F, dtype=bf, device=dev) for _ in range(self.L)]
        self.fcact = [torch.empty(N, F, dtype=bf, device=dev) for _ in range(self.L)]
        self.lnf_out = torch.empty(N, C, dtype=bf, device=dev)
        # rows padded to a multiple of 8 elements (16 B): the GEMMs take the row stride, the CE
        # kernel's 16-B chunks stay inside the row (HF GPT-2: V = 50257 -> stride 50264)
        # training: two rotating [chunk, ld] buffers (lm_head → CE → dgrad/wgrad per token chunk);
        # the full [N, ld] logits only exist transiently for logits_for / diagnostics captures
        self.head_chunk = _head_chunk_rows(N, V)
        self._head_bufs = [torch.empty(self.head_chunk, self._logit_ld(), dtype=bf, device=dev)
                           for _ in range(2 if self.head_chunk < N else 1)]
        self.tmp_c = torch.empty(N, C, dtype=bf, device=dev)
        self.dresid = torch.empty(N, C, dtype=f32, device=dev)
        # gradient buffers read by the side-stream weight-gradient GEMMs rotate between two
        # copies, so the main stream can produce the next one while the side stream still reads
        self.dresid_bf2 = [torch.empty(N, C, dtype=bf, device=dev) for _ in range(2)]
        self.d_f2 = [torch.empty(N, F, dtype=bf, device=dev) for _ in range(2)]
        self.dqkv2 = [torch.empty(N, 3 * C, dtype=bf, device=dev) for _ in range(2)]
        self.d_c = torch.empty(N, C, dtype=bf, device=dev)
        self._acts_shape = (B, T)

    def free_buffers(self):
        for name in ("resid", "resid_mid", "ln1", "ln2", "qkv", "fcpre", "fcact", "lnf_out", "_head_bufs", "tmp_c",
                     "dresid", "dresid_bf2", "d_f2", "d_c", "dqkv2", "att", "lse", "stats", "statsf"):
            if hasattr(self, name):
                delattr(self, name)
        self._acts_shape = None

    # ------------------------------------------------------------------ forward
    def _linear(self, x: Tensor, lin: nn.Linear, out: Tensor | None = None) -> Tensor:
        w = self.bf16(lin.weight)
        if lin.bias is not None:
            return torch.addmm(self.bf16(lin.bias), x, w.t(), out=out) if out is not None else \
                torch.addmm(self.bf16(lin.bias), x, w.t())
        return torch.mm(x, w.t(), out=out) if out is not None else torch.mm(x, w.t())

    def _drop(self, training: bool, seed: int, l: int, branch: int) -> tuple[float, int]:
        """(p, mask seed) of residual-dropout site (layer l, branch 0 = attention / 1 = MLP)."""
        b = self.spec.blocks[l]
        p = (b.p_attn_res if branch == 0 else b.p_mlp_res) if training else 0.0
        return p, _site_seed(seed, 2 * l + branch)

    def _forward(self, idx: Tensor, training: bool, dropout_seed: int = 0):
        """Embedding … final LayerNorm (``self.lnf_out``); the lm_head runs in ``_head_*``."""
        s = self.spec
        B, T = idx.shape
        if T > s.P:
            raise ValueError(f"sequence length {T} exceeds the position table {s.P}")
        self._alloc(B, T)
        H, D, C = s.H, s.D, s.C
        f = self.f32
        fused_ops.embedding_fwd(idx, f(s.wte.weight), f(s.wpe.weight), s.wpe.position_offset, out=self.resid[0],
                                dropout_p=s.p_embd if training else 0.0,
                                dropout_seed=_site_seed(dropout_seed, -1))
        for l, b in enumerate(s.blocks):
            mean1, rstd1, mean2, rstd2 = self.stats[l]
            if l == 0:
                norm_ops.ln_fwd(self.resid[0], f(b.ln1.weight), f(b.ln1.bias), b.ln1.eps, y=self.ln1[0],
                                mean=mean1, rstd=rstd1)
            else:  # resid[l] = resid_mid[l-1] + drop(fc2(l-1)), LN1(l) in the same pass
                dp, ds = self._drop(training, dropout_seed, l - 1, 1)
                norm_ops.add_ln_fwd(self.resid_mid[l - 1], self.tmp_c, self.resid[l], f(b.ln1.weight),
                                    f(b.ln1.bias), b.ln1.eps, y=self.ln1[l], mean=mean1, rstd=rstd1,
                                    dropout_p=dp, dropout_seed=ds)
            self._linear(self.ln1[l], b.qkv, out=self.qkv[l])
            p = b.attn.dropout if training else 0.0
            attn_ops.flash_fwd(self.qkv[l].view(B, T, 3 * C), H, H, D, p, dropout_seed + l,
                               out=self.att[l].view(B, T, C), lse=self.lse[l])
            self._linear(self.att[l], b.proj, out=self.tmp_c)
            dp, ds = self._drop(training, dropout_seed, l, 0)
            norm_ops.add_ln_fwd(self.resid[l], self.tmp_c, self.resid_mid[l], f(b.ln2.weight), f(b.ln2.bias),
                                b.ln2.eps, y=self.ln2[l], mean=mean2, rstd=rstd2, dropout_p=dp, dropout_seed=ds)
            # fc: library GEMM + bias into the pre-activation, then the HIP GELU kernel writes the
            # activation (ops/gemm.py linear_gelu); the backward's dgrad_gelu is a library GEMM
            # followed by one GELU-backward + fc-bias column-sum kernel
            gemm_ops.linear_gelu(self.ln2[l], self.bf16(b.fc.weight), self.bf16(b.fc.bias), self.fcpre[l],
                                 self.fcact[l], s.gelu_approx)
            self._linear(self.fcact[l], b.fc2, out=self.tmp_c)
        Lc = self.L
        meanf, rstdf = self.statsf
        dp, ds = self._drop(training, dropout_seed, Lc - 1, 1)
        norm_ops.add_ln_fwd(self.resid_mid[Lc - 1], self.tmp_c, self.resid[Lc], f(s.lnf.weight), f(s.lnf.bias),
                            s.lnf.eps, y=self.lnf_out, mean=meanf, rstd=rstdf, dropout_p=dp, dropout_seed=ds)

    def _logit_ld(self) -> int:
        """Row stride of the logits buffers: the padded head width, and a multiple of 8 elements
        (16 B: the GEMMs take the stride, the CE kernel's 16-B chunks stay inside the row)."""
        return (self.Vp + 7) // 8 * 8

    def _head_logits(self, r0: int, r1: int, buf: Tensor) -> Tensor:
        """lm_head GEMM of token rows [r0, r1) into ``buf`` ([rows, ld]); returns the [rows, Vp]
        view (columns V..Vp-1 are the pad rows' exact zeros; slice [:, :V] for the logits)."""
        lg = buf[: r1 - r0, : self.Vp]
        torch.mm(self.lnf_out[r0:r1], self.head_w().t(), out=lg)
        return lg

    def _full_logits(self, padded: bool = False) -> Tensor:
        N = self.lnf_out.shape[0]
        buf = torch.empty(N, self._logit_ld(), dtype=torch.bfloat16, device=self.device)
        lg = self._head_logits(0, N, buf)
        return lg if padded else lg[:, : self.spec.V]

    # ------------------------------------------------------------------ public API
    @torch.no_grad()
    def eval_loss(self, idx: Tensor, targets: Tensor) -> Tensor:
        self._forward(idx, training=False)
        N, tg = self.lnf_out.shape[0], targets.reshape(-1)
        total = torch.zeros((), dtype=torch.float32, device=self.device)
        for r0 in range(0, N, self.head_chunk):
            r1 = min(N, r0 + self.head_chunk)
            total += fused_ops.cross_entropy_fwd_bwd(self._head_logits(r0, r1, self._head_bufs[0])[:, : self.spec.V],
                                                     tg[r0:r1], 0.0).sum()
        return total / N

    @torch.no_grad()
    def logits_for(self, idx: Tensor) -> Tensor:
        self._forward(idx, training=False)
        return self._full_logits().view(idx.shape[0], idx.shape[1], -1)

    # the last bucket (wpe + wte: 157 MB fp32 at GPT-2 124M, produced by the backward's final
    # kernel) is cut into this many pieces so its all-reduce pipelines with the optimizer passes of
    # the pieces already landed (PENROZ_TAIL_PIECES)
    TAIL_PIECES = 4

    def setup_training(self, distributed: bool):
        from penroz.parallel.reducer import GradReducer, plan_buckets, default_bucket_mb, ready_map, split_last_bucket
        import os
        import torch.distributed as dist
        self.refresh_shadow()
        self.reducer = None
        if distributed and dist.is_initialized() and dist.get_world_size() > 1:
            buckets = plan_buckets(self.segments, default_bucket_mb(dist.get_backend()) * 2**20)
            buckets = split_last_bucket(buckets, int(os.environ.get("PENROZ_TAIL_PIECES", self.TAIL_PIECES)))
            self.reducer = GradReducer(self.flat_grad, buckets)
            self.reducer.broadcast_params(self.flat)
            self.refresh_shadow()
            self._ready_at = ready_map(buckets, self.segments)

    def _per_bucket_opt_ok(self) -> bool:
        """World > 1: apply the fused AdamW to each gradient bucket inside the backward, on its own
        stream, as soon as that bucket's all-reduce has landed (PENROZ_OPT_PER_BUCKET=1 forces it on
        a host-blocking transport such as gloo, 0 disables it)."""
        import os
        env = os.environ.get("PENROZ_OPT_PER_BUCKET")
        if env == "0" or self.device.type != "cuda" or not self._buckets_tile_flat():
            return False
        return env == "1" or self.reducer.stream_waits()

    def opt_overlap_mode(self) -> str:
        """How the optimizer step overlaps the backward (reported by bench.py in ``comm``)."""
        if getattr(self, "_opt_mode", None):
            return self._opt_mode
        return "none"

    def end_training(self):
        if self.reducer is not None:
            self.wait_gradients()
        self.reducer = None

    def zero_grad(self):
        """Zero the gradients. Once a backward has shown which flat ranges only the weight-gradient
        GEMMs write (the linear weights: most of the buffer), those are left alone and the first
        GEMM into each writes instead of accumulating (``gemm_ops.wgrad(accumulate=False)``), so
        the step neither clears them nor reads them back (PENROZ_GRAD_OVERWRITE=0: clear all)."""
        self.wait_gradients()
        # a flat range the last backward left all-zero itself (the Gemma row-split embedding step)
        skip, self._zero_skip = getattr(self, "_zero_skip", None), None
        self._micro_since_zero = 0
        gaps = getattr(self, "_zero_gaps", None)
        if gaps is not None:
            key = (self.flat_grad.data_ptr(), skip)
            if getattr(self, "_zero_views_key", None) != key:  # views of THIS buffer
                self._zero_views = [self.flat_grad[a:b] for a, b in _minus(gaps, skip)]
                self._zero_views_key = key
            torch._foreach_zero_(self._zero_views)
            self._stale = {k: [r] for k, r in self._wgrad_ranges.items()}
        else:
            for a, b in _minus([(0, self.flat_grad.numel())], skip):
                self.flat_grad[a:b].zero_()
            self._stale = {}
        self._captured = None

    def _learn_wgrad_ranges(self):
        """After the first backward: the flat ranges outside the weight-gradient GEMMs' outputs,
        as views for one multi-tensor zero (neighbouring ranges merged)."""
        import os
        self._zero_gaps = None
        if (os.environ.get("PENROZ_GRAD_OVERWRITE", "1") == "0" or self.device.type != "cuda"
                or not getattr(self, "_wgrad_ranges", None) or getattr(self, "_wgrad_ranges_invalid", False)):
            return
        covered = sorted(self._wgrad_ranges.values())
        gaps, pos = [], 0
        for s, e in covered:
            if s < pos:  # overlapping outputs: not a partition, keep clearing everything
                return
            if s > pos:
                gaps.append((pos, s))
            pos = e
        if pos < self.flat_grad.numel():
            gaps.append((pos, self.flat_grad.numel()))
        self._zero_gaps = gaps

    def _segment_done(self, seg_index: int, sync: bool):
        if self._opt_apply is not None and sync and self.reducer is None:
            # optimizer inside the backward: this segment's gradients are final once the side
            # stream (its weight gradients, deferred dγ / bias reductions) has caught up with the
            # main stream (its other gradients); nothing later in this backward reads its weights
            s, e = self.segments[seg_index]
            if getattr(self, "_side", None) is None:
                self._opt_apply(s, e)
                self._transpose_segment(s, e)
                return
            main = torch.cuda.current_stream(self.device)
            with torch.cuda.stream(self._side):
                self._side.wait_stream(main)
                self._opt_apply(s, e)
                self._transpose_segment(s, e)
            return
        if self.reducer is None or not sync:
            return
        ready = self._ready_at.get(seg_index, ())
        if not ready:
            return
        if getattr(self, "_side", None) is None:
            for i in ready:
                self.reducer.bucket_ready(i)
        else:
            # the bucket's weight gradients come from the side stream, its bias / LayerNorm
            # gradients from the main stream: launch the collective from the side stream after
            # it has caught up with the main stream
            main = torch.cuda.current_stream(self.device)
            with torch.cuda.stream(self._side):
                self._side.wait_stream(main)
                for i in ready:
                    self.reducer.bucket_ready(i)
        if self._opt_bucketed:
            self._opt_buckets(ready)

    def _opt_buckets(self, ids):
        """Per-bucket optimizer (world > 1): on the optimizer stream, wait for each bucket's
        all-reduce (a stream wait, not a host wait) and apply the fused AdamW to its range, then
        rebuild the transposed dgrad copies of the weights wholly inside it (Gemma). Nothing later
        in the backward reads the parameters of a finished segment; the main stream joins this
        stream before the step returns (the next forward reads the new weights)."""
        ost = getattr(self, "_opt_stream", None)
        if ost is None:
            ost = self._opt_stream = shared_stream(self.device, "opt")
        with torch.cuda.stream(ost):
            for i in ids:
                if i in self._opt_buckets_done:
                    continue
                s, e = self.reducer.wait_bucket(i)
                self._opt_apply(s, e)
                self._transpose_segment(s, e)
                self._opt_buckets_done.add(i)

    # ---- weight gradients on a side HIP stream -------------------------------------------------
    # The weight-gradient GEMMs and the finishing kernels of every dγ / dβ / bias column reduction
    # (the qkv bias partials come from the attention-backward epilogues) are off the backward's
    # critical path (nothing in the
    # backward reads parameter gradients), so they run on a second stream and overlap the
    # main stream's dgrad GEMMs, LayerNorm / GELU backward, flash-attention backward. Ordering: the side stream waits on an event
    # recorded after each operand's producer; before the main stream overwrites a rotating
    # operand buffer it waits on the event recorded after that buffer's last side-stream reader;
    # gradient buckets are handed to the reducer from the side stream (after it has also waited
    # for the main stream's bias / LayerNorm gradients), and the main stream joins the side stream
    # before the step returns. PENROZ_WGRAD_STREAM=0 runs everything on one stream (A/B).
    def _side_init(self):
        import os
        self._side = None
        if self.device.type == "cuda" and os.environ.get("PENROZ_WGRAD_STREAM", "1") != "0":
            cus = os.environ.get("PENROZ_SIDE_CUS", "")
            self._side = _cu_masked_stream(self.device, cus) if cus else shared_stream(self.device, "side")
        self._buf_free = {}

    def _side_call(self, operand: Tensor, fn):
        """Run ``fn`` (gradient-only work reading ``operand``) on the side stream, or inline."""
        if getattr(self, "_side", None) is None:
            fn()
            return
        main = torch.cuda.current_stream(self.device)
        ready = torch.cuda.Event()
        ready.record(main)
        with torch.cuda.stream(self._side):
            self._side.wait_event(ready)
            fn()
            done = torch.cuda.Event()
            done.record(self._side)
        self._buf_free[operand.data_ptr()] = done

    def _wgrad(self, dy: Tensor, x: Tensor, p: Tensor):
        self._wgrad_into(id(p), dy, x, self.grad(p))

    def _wgrad_into(self, key: int, dy: Tensor, x: Tensor, g: Tensor):
        """g (+)= dyᵀ·x on the side stream: the first write of a range that zero_grad left alone
        overwrites it; the ranges are recorded during the first backward (see zero_grad).

        ``_stale[key]`` holds the parts of the key's learned range that zero_grad skipped and no
        write of this step has touched yet. A write covering exactly the whole stale learned range
        overwrites it; any other write (e.g. a chunked wgrad writing sub-ranges under one key)
        first clears the stale parts it overlaps and accumulates; parts still stale at the end of
        the backward are cleared by :meth:`_finish_wgrad_bookkeeping`. A range pattern that differs
        from the learned one also makes zero_grad clear everything from the next step on."""
        rec = getattr(self, "_wgrad_ranges", None)
        if rec is None:
            rec = self._wgrad_ranges = {}
        off = g.data_ptr() - self.flat_grad.data_ptr()
        rng = (off // 4, off // 4 + g.numel())
        if not getattr(self, "_ranges_learned", False):
            if rec.get(key, rng) != rng:  # one key, several sub-ranges: not a plain overwrite
                self._wgrad_ranges_invalid = True
            rec[key] = rng
        elif rec.get(key) != rng:
            self._wgrad_ranges_invalid = True
            self._zero_gaps = None
        stale = getattr(self, "_stale", None) or {}
        parts = stale.get(key)
        if parts and parts == [rng]:  # the whole learned range, untouched this step: overwrite
            del stale[key]
            self._side_call(dy, lambda: gemm_ops.wgrad(dy, x, g, False))
            return
        if parts:
            keep = []
            for s_, e_ in parts:
                a, b = max(s_, rng[0]), min(e_, rng[1])
                if a >= b:
                    keep.append((s_, e_))
                    continue
                view = self.flat_grad[a:b]
                self._side_call(dy, lambda v=view: v.zero_())
                if s_ < a:
                    keep.append((s_, a))
                if b < e_:
                    keep.append((b, e_))
            if keep:
                stale[key] = keep
            else:
                del stale[key]
        self._side_call(dy, lambda: gemm_ops.wgrad(dy, x, g, True))

    def _finish_wgrad_bookkeeping(self):
        """End of a backward: learn the ranges once; clear any part of a range zero_grad skipped
        that no GEMM wrote (not expected: every backward writes every linear weight's gradient)."""
        if not getattr(self, "_ranges_learned", False):
            self._ranges_learned = True
            self._learn_wgrad_ranges()
        stale = getattr(self, "_stale", None)
        if stale:
            log.warning(f"weight-gradient ranges not written by this backward: {len(stale)}; clearing them")
            self._join_side()
            for parts in stale.values():
                for s_, e_ in parts:
                    self.flat_grad[s_:e_].zero_()
            stale.clear()

    def _defer_reductions(self, on: bool):
        """LayerNorm / bias column-reduction finishing kernels go to the side stream (on) or not."""
        if getattr(self, "_side", None) is not None:
            _ext.kernels().set_deferred_reduce_stream(self._side.cuda_stream if on else 0, self.device.index or 0)

    def _reuse(self, buf: Tensor) -> Tensor:
        """Main stream: wait until the side stream no longer reads ``buf`` (before overwriting)."""
        ev = self._buf_free.pop(buf.data_ptr(), None) if getattr(self, "_side", None) is not None else None
        if ev is not None:
            torch.cuda.current_stream(self.device).wait_event(ev)
        return buf

    def _join_side(self):
        if getattr(self, "_side", None) is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._side)
            self._buf_free.clear()

    @torch.no_grad()
    def train_micro_step(self, idx: Tensor, targets: Tensor, scale: float, sync: bool = True,
                         capture: bool = False, fuse_optimizer: bool = False) -> Tensor:
        """Forward + backward of one micro-batch; gradients accumulate into the flat buffer.
        Returns the (scaled) mean loss as a device scalar.

        ``fuse_optimizer`` (the last micro-step of a step whose ``optimizer_step`` follows, single
        process): the fused AdamW updates each parameter segment inside the backward, on the side
        stream, as soon as that segment's gradients are final — the optimizer pass overlaps the
        rest of the backward instead of running after it (``optimizer_step`` then has nothing left
        to do). ``PENROZ_OPT_IN_BWD=0`` keeps the separate step."""
        import os
        self._opt_apply = None
        self._opt_bucketed = False
        if (fuse_optimizer and sync and not capture and self._opt_flat
                and os.environ.get("PENROZ_OPT_IN_BWD", "1") != "0"):
            if self.reducer is None:
                self._opt_apply = self.model.optimizer.begin_flat_ranges()
                self._opt_mode = "per-segment-in-backward" if self._opt_apply is not None else None
            elif self._per_bucket_opt_ok():
                self._opt_apply = self.model.optimizer.begin_flat_ranges()
                self._opt_bucketed = self._opt_apply is not None
                self._opt_buckets_done = set()
                self._opt_mode = "per-bucket-in-backward" if self._opt_bucketed else None
        hp = self._main_stream() if not capture else None
        try:
            if hp is None:
                loss = self._train_micro_step(idx, targets, scale, sync, capture)
            else:  # the step's critical path on a high-priority stream (PENROZ_MAIN_PRIORITY=1)
                cur = torch.cuda.current_stream(self.device)
                hp.wait_stream(cur)
                with torch.cuda.stream(hp):
                    loss = self._train_micro_step(idx, targets, scale, sync, capture)
                cur.wait_stream(hp)
        finally:
            self._opt_done = self._opt_apply is not None
            self._opt_apply = None
        return loss

    # the critical path on a high-priority stream. Round 5: GPT-2 headline 61.63 / 61.63 -> 61.19 /
    # 61.19 ms/step. Round 6, with one stream per role per process and the batch copy on its own
    # stream, the headline is faster WITHOUT it: 61.83 / 61.76 / 61.79 (high) vs 61.55 / 61.60 /
    # 61.63 (normal) and 60.45 / 60.54 vs 60.40 / 60.29 on a second box; the Gemma executors keep
    # it (faster there, profiles/notes_r6.md §15, §17)
    MAIN_PRIORITY_DEFAULT = False

    def _main_stream(self):
        """A high-priority stream for the forward / backward critical path, so the side stream's
        weight-gradient GEMMs yield the CUs to the dgrad / attention chain when both have work
        (PENROZ_MAIN_PRIORITY=1 / 0 overrides the executor's default)."""
        import os
        env = os.environ.get("PENROZ_MAIN_PRIORITY")
        on = self.MAIN_PRIORITY_DEFAULT if env is None else env == "1"
        if self.device.type != "cuda" or not on or getattr(self, "_side", None) is None:
            return None
        hp = getattr(self, "_hp_stream", None)
        if hp is None:
            hp = self._hp_stream = _high_priority_stream(self.device)
        return hp

    def _train_micro_step(self, idx: Tensor, targets: Tensor, scale: float, sync: bool, capture: bool) -> Tensor:
        s = self.spec
        B, T = idx.shape
        N, C = B * T, s.C
        seed = self._step_seed
        self._step_seed += 1000
        self._refresh_transposed()
        with trace_range("forward"):
            self._forward(idx, training=True, dropout_seed=seed)
        cap = capture and self._captured is None
        # ---- head, per token chunk: lm_head GEMM, CE (in place -> dlogits), dgrad, wgrad
        head_range = trace_range("backward.head")
        head_range.__enter__()
        self._defer_reductions(True)
        tg = targets.reshape(-1)
        V = s.V
        if cap:  # diagnostics want the whole logits / dlogits tensors: one transient chunk
            full = self._full_logits(padded=True)
            acts = [self.resid[0].view(B, T, C).clone()] * 2 + [r.view(B, T, C).clone() for r in self.resid[1:]] + \
                   [self.lnf_out.view(B, T, C).float().clone(), full[:, :V].reshape(B, T, V).clone()]
            chunks = [(0, N, full)]
        else:
            chunks = [(r0, min(N, r0 + self.head_chunk), None) for r0 in range(0, N, self.head_chunk)]
        loss = torch.zeros((), dtype=torch.float32, device=self.device)
        w_dgrad = self._dgrad_w(s.head.weight)
        for i, (r0, r1, lg) in enumerate(chunks):
            if lg is None:  # the side stream may still be reading this buffer (wgrad two chunks back)
                lg = self._head_logits(r0, r1, self._reuse(self._head_bufs[i % len(self._head_bufs)]))
            # CE rewrites the V real columns with dlogits; the pad columns stay the exact zeros of
            # the pad rows, so the padded dgrad / wgrad equal the unpadded ones (pad rows get 0)
            loss += fused_ops.cross_entropy_fwd_bwd(lg[:, :V], tg[r0:r1], scale / N).sum()
            torch.mm(lg[:, : w_dgrad.shape[0]], w_dgrad, out=self.d_c[r0:r1])
            self._wgrad_into(id(s.head.weight), lg, self.lnf_out[r0:r1], self.head_grad())
        loss *= scale / N
        mean, rstd = self.statsf
        last = s.blocks[-1]
        rb = 0  # rotating dresid_bf buffer index
        dp, ds = self._drop(True, seed, self.L - 1, 1)
        norm_ops.ln_bwd(self.d_c, self.resid[self.L], mean, rstd, self.f32(s.lnf.weight), self.dresid, False,
                        self._reuse(self.dresid_bf2[rb]), self.grad(s.lnf.weight), self.grad(s.lnf.bias),
                        self.grad(last.fc2.bias), dropout_p=dp, dropout_seed=ds)
        grads_cap = []
        if cap:
            grads_cap = [full[:, :V].reshape(B, T, V).clone(), self.d_c.view(B, T, C).float().clone(),
                         self.dresid.view(B, T, C).clone()]
        self._segment_done(0, sync)
        head_range.__exit__(None, None, None)
        for l in range(self.L - 1, -1, -1):
            layer_range = trace_range(f"backward.block{l}")
            layer_range.__enter__()
            b = s.blocks[l]
            d_f, dqkv = self._reuse(self.d_f2[l & 1]), self._reuse(self.dqkv2[l & 1])
            dres_bf = self.dresid_bf2[rb]
            # ---- MLP branch
            # fc2 data gradient, GELU backward and the fc bias gradient in one kernel (ops/gemm.py)
            gemm_ops.dgrad_gelu(dres_bf, self._dgrad_w(b.fc2.weight).t(), self.fcpre[l], d_f, self.grad(b.fc.bias),
                                s.gelu_approx)
            self._wgrad(dres_bf, self.fcact[l], b.fc2.weight)
            torch.mm(d_f, self._dgrad_w(b.fc.weight), out=self.d_c)
            self._wgrad(d_f, self.ln2[l], b.fc.weight)
            _, _, mean, rstd = self.stats[l]
            rb ^= 1
            dres_bf = self._reuse(self.dresid_bf2[rb])
            dp, ds = self._drop(True, seed, l, 0)
            norm_ops.ln_bwd(self.d_c, self.resid_mid[l], mean, rstd, self.f32(b.ln2.weight), self.dresid, True,
                            dres_bf, self.grad(b.ln2.weight), self.grad(b.ln2.bias), self.grad(b.proj.bias),
                            dropout_p=dp, dropout_seed=ds)
            # ---- attention branch
            torch.mm(dres_bf, self._dgrad_w(b.proj.weight), out=self.d_c)
            self._wgrad(dres_bf, self.att[l], b.proj.weight)
            # the qkv bias gradient comes out of the attention-backward epilogues (partials finished
            # on the side stream by the deferred reduction)
            attn_ops.flash_bwd(self.d_c.view(B, T, C), self.qkv[l].view(B, T, 3 * C), self.att[l].view(B, T, C),
                               self.lse[l], s.H, s.H, s.D, b.attn.dropout, seed + l, dqkv=dqkv.view(B, T, 3 * C),
                               dbias=self.grad(b.qkv.bias))
            torch.mm(dqkv, self._dgrad_w(b.qkv.weight), out=self.d_c)
            self._wgrad(dqkv, self.ln1[l], b.qkv.weight)
            mean, rstd, _, _ = self.stats[l]
            prev_bias = self.grad(s.blocks[l - 1].fc2.bias) if l > 0 else None
            rb ^= 1
            dp, ds = self._drop(True, seed, l - 1, 1) if l > 0 else (0.0, 0)
            norm_ops.ln_bwd(self.d_c, self.resid[l], mean, rstd, self.f32(b.ln1.weight), self.dresid, True,
                            self._reuse(self.dresid_bf2[rb]) if l > 0 else None, self.grad(b.ln1.weight),
                            self.grad(b.ln1.bias), prev_bias, dropout_p=dp, dropout_seed=ds)
            if cap:
                grads_cap.append(self.dresid.view(B, T, C).clone())
            self._segment_done(self.L - l, sync)
            layer_range.__exit__(None, None, None)
        fused_ops.embedding_bwd(self.dresid, idx, self.grad(s.wte.weight), self.grad(s.wpe.weight),
                                s.wpe.position_offset, dropout_p=s.p_embd, dropout_seed=_site_seed(seed, -1))
        self._segment_done(self.L + 1, sync)
        self._defer_reductions(False)
        self._finish_wgrad_bookkeeping()
        self._join_side()
        if sync and self.reducer is not None:
            # Overlap the tail: the last bucket (token embedding, produced by the final kernel of
            # the backward) is still reducing when the backward ends. If the optimizer step comes
            # next, it updates each bucket's slice as soon as that bucket's all-reduce has landed
            # (optimizer_step), instead of waiting for all of them here.
            self.reducer.launch_remaining()
            if self._opt_bucketed:  # every bucket's AdamW is queued on the optimizer stream
                self._opt_buckets(range(len(self.reducer.buckets)))
                torch.cuda.current_stream(self.device).wait_stream(self._opt_stream)
                self.reducer.reset()
            elif self._overlap_opt and not cap and self.reducer.per_bucket_waits():
                self._reduce_pending = True
            else:
                with trace_range("grad_allreduce.wait"):
                    self.reducer.finish()
        if cap:
            # grads_cap: [dlogits, d_lnf, d_resid[L], d_resid[L-1], ..., d_resid[0]]
            dlog, dlnf, dres = grads_cap[0], grads_cap[1], grads_cap[2:]
            dres = list(reversed(dres))  # d_resid[0] ... d_resid[L]
            act_grads = [dres[0], dres[0]] + dres[1:] + [dlnf, dlog]
            algos = [l.__class__.__name__.lower() for l in self.model.layers]
            pairs = list(zip(acts, act_grads))
            self._captured = (algos, pairs[:len(algos)])
        return loss

    def wait_gradients(self):
        """Make the current stream wait for every outstanding gradient all-reduce."""
        if self._reduce_pending:
            self._reduce_pending = False
            self.reducer.finish()

    def optimizer_step(self):
        opt = self.model.optimizer
        if getattr(self, "_opt_done", False):  # applied segment by segment inside the backward
            self._opt_done = False
            return
        with trace_range("optimizer"):
            if self._reduce_pending:
                self._reduce_pending = False
                red = self.reducer
                ranges = [(lambda i=i: red.wait_bucket(i)) for i in range(len(red.buckets))]
                if self._buckets_tile_flat() and self._opt_flat and opt.flat_step_ranges(ranges):
                    red.reset()
                    self._opt_mode = "per-bucket-after-backward"
                    return
                red.finish()
            opt.step()
            if not self._opt_flat:
                self.refresh_shadow()

    def _buckets_tile_flat(self) -> bool:
        """The ranged optimizer step needs the buckets to cover the flat buffer exactly once."""
        pos = 0
        for s, e in sorted(self.reducer.buckets):
            if s != pos:
                return False
            pos = e
        return pos == self.flat.numel()

    def captured(self):
        if self._captured is None:
            return [l.__class__.__name__.lower() for l in self.model.layers], []
        return self._captured
