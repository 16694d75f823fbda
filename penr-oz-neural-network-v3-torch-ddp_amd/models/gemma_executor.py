"""Fused Gemma-family training / eval executor for MI355X (the Gemma analogue of
:class:`penroz.models.executor.GPTExecutor`).

A layer list of the reference's Gemma layout (``mappers.py:179-262``: ScaledEmbedding →
TransformerBlock(RMSNorm → QKV → RoPE attention (GQA) → O; RMSNorm → GatedMLP; optional post-norms)
× L → RMSNorm → lm_head; blocks per ``neural_net_layers.py:144-225``) is lowered to an explicit
forward and backward over flat parameter buffers while the ``nn.Module`` tree and its state_dict
keys stay as compiled. Per block, N = B·T tokens, fp32 residual stream:

forward
  QKV GEMM (hipBLASLt, bf16 shadow) → RoPE (HIP, per-layer θ table) → flash attention (HIP,
  head_dim 64/128/256, GQA by index math) → O GEMM → [residual add + post-attention norm +
  pre-MLP norm] (one HIP pass, ``gemma_combine_fwd``; the Gemma 3 / Gemma 2 / Gemma 1 post-norm
  placements are its modes 0 / 1 / 2) → gate|up GEMM over the CONCATENATED weight (gate_proj and
  up_proj sit next to each other in the flat buffer, so their bf16 shadow slice is one [2F, C]
  matrix and their gradient slice one [2F, C] gradient) → gated activation on the packed halves
  (HIP) → down GEMM → [residual add + post-MLP norm + the NEXT block's input norm] (one pass; after
  the last block the next norm is the final norm, whose bf16 output feeds the lm_head).
head: lm_head GEMM → fused cross-entropy (HIP, logits gradient in place) → dgrad / wgrad, in token
  chunks when the [N, V] logits exceed 8 GiB (Gemma's 262 144-token vocabulary: 4 GiB at N = 8192).
backward mirrors it: every combine's backward is one HIP pass (RMSNorm backward of both norms,
  the residual-gradient accumulation, the bf16 branch gradient for the next dgrad GEMM, and the
  norm-weight gradients as deterministic partial-row reductions finished on the side stream);
  packed gated-activation backward; inverse RoPE; flash-attention backward; weight-gradient GEMMs
  on the side stream (fp32 accumulation into the flat gradient buffer), data-gradient GEMMs on
  transposed bf16 weight copies; embedding gradient (scaled scatter-add).

Parameters, gradients and AdamW moments live in flat fp32 buffers laid out in backward completion
order (lm_head … embedding) so gradient buckets are contiguous slices for the overlapped
all-reduce; a bf16 shadow feeds the GEMMs and is rewritten by the fused AdamW step (bf16-parameter
models — what ``/import/`` produces — train with fp32 masters while ``state_dict()`` stays bf16).
"""
from __future__ import annotations

import logging
from dataclasses import dataclass, field

import torch
import torch.nn as nn
from torch import Tensor

from penroz.models import layers as L
from penroz.models.executor import GPTExecutor, _head_chunk_rows, _is
from penroz.ops import _ext
from penroz.ops import attention as attn_ops
from penroz.ops import fused as fused_ops
from penroz.ops import gemm as gemm_ops
from penroz.ops import rope as rope_ops
from penroz.utils.profiling import trace_range

log = logging.getLogger(__name__)

_ACT_KIND = {"gelu": 0, "gelu_tanh": 1, "silu": 2}  # elementwise.hip act_f kinds


@dataclass
class _GBlock:
    in_norm: L.RMSNorm
    qkv: nn.Linear
    attn: L.CausalSelfAttention
    o: nn.Linear
    pre_mlp: L.RMSNorm
    mlp: L.GatedMLP
    post_attn: L.RMSNorm | None
    post_mlp: L.RMSNorm | None
    # this block's shapes: Gemma 4 layer lists are heterogeneous (full-attention layers with
    # global_head_dim / their own KV-head count, double-wide MLPs on KV-shared layers:
    # reference mappers.py:206-233)
    H: int = 0
    Hkv: int = 0
    D: int = 0
    F: int = 0


@dataclass
class GemmaSpec:
    V: int
    C: int
    emb: L.ScaledEmbedding
    norm_f: L.RMSNorm
    head: nn.Linear
    blocks: list = field(default_factory=list)
    mode: int = 2            # 0: post-norm on the residual (Gemma 3+), 1: on the branch (Gemma 2), 2: none
    H: int = 0               # the first block's shapes (every block's when ``uniform``)
    Hkv: int = 0
    D: int = 0
    F: int = 0
    uniform: bool = True
    act: int = 1
    param_dtype: torch.dtype = torch.float32

    # the GPTExecutor helpers read these names
    @property
    def lnf(self):
        return self.norm_f


class GemmaExecutor(GPTExecutor):
    # the critical path on the high-priority stream: round 5 measured it slightly slower at B = 8;
    # with one stream per role per process (round 6) it is faster: Gemma-3 1B B = 8 66.85 / 66.87
    # -> 66.30 / 66.29 ms (same box, profiles/notes_r6.md §15)
    MAIN_PRIORITY_DEFAULT = True
    # transposed dgrad copies rebuilt at the step start (as GPT) instead of after each segment's
    # AdamW: round 5 measured the segment rebuild −0.2 to −0.3 ms; with the high-priority critical
    # path and the shared streams (round 6) the step-start rebuild is faster: Gemma-3 1B B = 8
    # 65.86 / 65.86 -> 65.14 / 65.32 and 65.82 / 65.72 -> 65.09 / 65.06 ms on two boxes, Gemma-4 e2b
    # neutral (profiles/notes_r6.md §16; PENROZ_SEGMENT_TRANSPOSE=1 / 0 overrides)
    SEGMENT_TRANSPOSE = False

    # ------------------------------------------------------------------ pattern match
    @staticmethod
    def match(model, require_fp32: bool = False) -> GemmaSpec | None:
        ls = list(model.layers)
        if ls and _is(ls[-1], L.SoftmaxOnLast):
            ls = ls[:-1]
        if len(ls) < 4 or type(ls[0]) is not L.ScaledEmbedding or type(ls[-2]) is not L.RMSNorm:
            return None
        head = ls[-1]
        if type(head) is not nn.Linear or head.bias is not None:
            return None
        emb = ls[0]
        if head.weight is emb.weight:  # a tied head would be one parameter in two flat slots
            return None
        C = emb.embedding_dim
        if C % 8 or C > 6144 or head.in_features != C or ls[-2].weight.numel() != C:
            return None
        spec = GemmaSpec(V=emb.num_embeddings, C=C, emb=emb, norm_f=ls[-2], head=head)
        modes, shapes, acts = set(), set(), set()
        for blk in ls[1:-2]:
            if type(blk) is not L.TransformerBlock:
                return None
            ab, mb = list(blk.attn_block), list(blk.mlp_block)
            if not (len(ab) == 4 and type(ab[0]) is L.RMSNorm and type(ab[1]) is nn.Linear
                    and type(ab[2]) is L.CausalSelfAttention and type(ab[3]) is nn.Linear
                    and len(mb) == 2 and type(mb[0]) is L.RMSNorm and type(mb[1]) is L.GatedMLP):
                return None
            in_norm, qkv, attn, o = ab
            pre, mlp = mb
            if (blk.post_attn_norm is None) != (blk.post_mlp_norm is None):
                return None
            if blk.post_attn_norm is not None and not (type(blk.post_attn_norm) is L.RMSNorm
                                                       and type(blk.post_mlp_norm) is L.RMSNorm):
                return None
            mode = 2 if blk.post_attn_norm is None else (0 if blk.post_norm_on_residual else 1)
            H, Hkv = attn.num_heads, attn.num_kv_heads
            D = attn.head_dim if attn.head_dim is not None else qkv.out_features // (H + 2 * Hkv)
            F = mlp.gate_proj.out_features
            if (qkv.bias is not None or o.bias is not None or mlp.gate_proj.bias is not None
                    or mlp.up_proj.bias is not None or mlp.down_proj.bias is not None):
                return None
            if (qkv.in_features != C or qkv.out_features != (H + 2 * Hkv) * D or o.in_features != H * D
                    or o.out_features != C or mlp.gate_proj.in_features != C or mlp.up_proj.out_features != F
                    or mlp.down_proj.in_features != F or mlp.down_proj.out_features != C):
                return None
            if D not in attn_ops.SUPPORTED_HEAD_DIMS or H % Hkv or F % 64 or attn.rope_theta is None:
                return None
            if not 0.0 <= attn.dropout < 1.0:
                return None
            modes.add(mode)
            shapes.add((H, Hkv, D, F))
            acts.add(mlp.act_kind)
            spec.blocks.append(_GBlock(in_norm, qkv, attn, o, pre, mlp, blk.post_attn_norm, blk.post_mlp_norm,
                                       H, Hkv, D, F))
        if not spec.blocks or len(modes) != 1 or len(acts) != 1:
            return None
        spec.mode = modes.pop()
        b0 = spec.blocks[0]
        spec.H, spec.Hkv, spec.D, spec.F = b0.H, b0.Hkv, b0.D, b0.F
        spec.uniform = len(shapes) == 1
        spec.act = _ACT_KIND[acts.pop()]
        dtypes = {p.dtype for p in model.parameters()}
        if len(dtypes) != 1 or not dtypes <= ({torch.float32} if require_fp32 else {torch.float32, torch.bfloat16}):
            return None
        spec.param_dtype = dtypes.pop()
        return spec

    # ------------------------------------------------------------------ setup
    def __init__(self, model, device):
        spec = self.match(model)
        if spec is None:
            raise ValueError("model does not match the Gemma pattern")
        _ext.kernels()
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
        self._rope_tables = {}

    def _param_order(self):
        s = self.spec
        segs = [[s.head.weight, s.norm_f.weight]]
        for b in reversed(s.blocks):
            seg = [b.mlp.down_proj.weight, b.mlp.gate_proj.weight, b.mlp.up_proj.weight, b.pre_mlp.weight]
            if b.post_mlp is not None:
                seg += [b.post_mlp.weight, b.post_attn.weight]
            seg += [b.o.weight, b.qkv.weight, b.in_norm.weight]
            segs.append(seg)
        segs.append([s.emb.weight])
        return segs

    def gu_bf16(self, b: _GBlock) -> Tensor:
        """The [gate; up] bf16 weight [2F, C] (adjacent in the flat buffer)."""
        off = self.offsets[id(b.mlp.gate_proj.weight)]
        F, C = b.F, self.spec.C
        return self.shadow[off:off + 2 * F * C].view(2 * F, C)

    def gu_grad(self, b: _GBlock) -> Tensor:
        off = self.offsets[id(b.mlp.gate_proj.weight)]
        F, C = b.F, self.spec.C
        return self.flat_grad[off:off + 2 * F * C].view(2 * F, C)

    # ---- transposed bf16 weight copies for the data-gradient GEMMs (see GPTExecutor) ---------
    def _init_transposed(self):
        import os
        self._tw, self._t_ready, self._t_fresh = {}, None, set()
        if self.device.type != "cuda" or os.environ.get("PENROZ_DGRAD_T", "1") == "0" or not _ext.available():
            return
        s = self.spec
        srcs = [(id(s.head.weight), lambda: self.bf16(s.head.weight))]
        for b in s.blocks:
            srcs += [(id(b.qkv.weight), lambda b=b: self.bf16(b.qkv.weight)),
                     (id(b.o.weight), lambda b=b: self.bf16(b.o.weight)),
                     (id(b.mlp.gate_proj.weight), lambda b=b: self.gu_bf16(b)),
                     (id(b.mlp.down_proj.weight), lambda b=b: self.bf16(b.mlp.down_proj.weight))]
        srcs = [(k, f) for k, f in srcs if f().shape[0] % 64 == 0 and f().shape[1] % 64 == 0]
        self.shadow_t = torch.empty(sum(f().numel() for _, f in srcs), dtype=torch.bfloat16, device=self.device)
        off = 0
        for key, f in srcs:
            w = f()
            n = w.numel()
            self._tw[key] = (f, self.shadow_t[off:off + n].view(w.shape[1], w.shape[0]))
            off += n

    def _refresh_transposed(self):
        if not self._tw:
            return
        k = _ext.kernels()
        side = getattr(self, "_side", None)
        if side is None:
            for key, (f, t) in self._tw.items():
                if key not in self._t_fresh:
                    k.transpose_bf16(f(), t)
            self._t_fresh.clear()
            return
        todo = [(f, t) for key, (f, t) in self._tw.items() if key not in self._t_fresh]
        self._t_fresh.clear()
        if not todo:  # all rebuilt after their segments' optimizer passes (the main stream joined)
            return
        main = torch.cuda.current_stream(self.device)
        with torch.cuda.stream(side):
            side.wait_stream(main)
            for f, t in todo:
                k.transpose_bf16(f(), t)
            self._t_ready = torch.cuda.Event()
            self._t_ready.record(side)

    def _tw_source(self, entry) -> Tensor:
        return entry[0]()

    def _dgrad(self, key_param: Tensor, src: Tensor) -> Tensor:
        """The weight operand of dx = dy·W: the transposed copy (viewed back as [out, in]) or ``src``."""
        tw = self._tw.get(id(key_param)) if self._tw else None
        if tw is None:
            return src
        if self._t_ready is not None:
            torch.cuda.current_stream(self.device).wait_event(self._t_ready)
            self._t_ready = None
        return tw[1].t()

    # ------------------------------------------------------------------ buffers
    def _alloc(self, B: int, T: int):
        if self._acts_shape == (B, T):
            return
        s, dev = self.spec, self.device
        N, C, V = B * T, s.C, s.V
        bs = s.blocks
        bf, f32 = torch.bfloat16, torch.float32
        Lc = self.L
        e = lambda *shape, dt=bf: torch.empty(*shape, dtype=dt, device=dev)  # noqa: E731
        qkv_w = lambda b: (b.H + 2 * b.Hkv) * b.D  # noqa: E731
        # resid[l]: block l input (fp32); mid[l]: after the attention combine
        self.resid = [e(N, C, dt=f32) for _ in range(Lc + 1)]
        self.mid = [e(N, C, dt=f32) for _ in range(Lc)]
        self.y_in = [e(N, C) for _ in range(Lc)]       # input norm outputs (QKV GEMM inputs)
        self.y_mlp = [e(N, C) for _ in range(Lc)]      # pre-MLP norm outputs (gate|up inputs)
        self.qkv = [e(N, qkv_w(b)) for b in bs]         # post-RoPE (attention inputs)
        self.att = [e(N, b.H * b.D) for b in bs]
        self.lse = [e(B, b.H, T, dt=f32) for b in bs]
        self.gu = [e(N, 2 * b.F) for b in bs]
        self.g = [e(N, b.F) for b in bs]
        mode = s.mode
        # norm statistics: r_in[l] (input norm of block l), r_pa / r_pre (attention combine),
        # r_pm (post-MLP combine's post-norm); the post-norm inputs the backward re-reads
        self.r_in = [e(N, dt=f32) for _ in range(Lc)]
        self.r_pre = [e(N, dt=f32) for _ in range(Lc)]
        self.r_pa = [e(N, dt=f32) for _ in range(Lc)] if mode in (0, 1) else None
        self.r_pm = [e(N, dt=f32) for _ in range(Lc)] if mode in (0, 1) else None
        self.r_f = e(N, dt=f32)
        if mode == 0:
            self.s_attn = [e(N, C, dt=f32) for _ in range(Lc)]
            self.s_mlp = [e(N, C, dt=f32) for _ in range(Lc)]
        elif mode == 1:
            self.s_attn = [e(N, C) for _ in range(Lc)]   # the branch outputs a (bf16)
            self.s_mlp = [e(N, C) for _ in range(Lc)]
        else:
            self.s_attn = self.s_mlp = None
        self.lnf_out = e(N, C)
        self.head_chunk = _head_chunk_rows(N, V)
        self._head_bufs = [e(self.head_chunk, (V + 7) // 8 * 8) for _ in range(2 if self.head_chunk < N else 1)]
        self.tmp_c = e(N, C)                               # branch outputs (O / down GEMMs)
        # per-block scratch shared by all blocks: flat buffers sized for the widest block, viewed
        # per block as [N, width] (``_rows``); a view keeps the buffer's data_ptr, so the
        # side-stream reuse events (``_reuse``) still key on the buffer
        QKV, A, F = max(qkv_w(b) for b in bs), max(b.H * b.D for b in bs), max(b.F for b in bs)
        self.qkv_raw = e(N * QKV)                          # QKV GEMM output before RoPE
        self.dresid = e(N, C, dt=f32)
        # rotating, read by side-stream wgrads: 4 deep — the side stream starts the backward ~7 ms
        # behind (lm_head wgrad, head-segment AdamW), and with 2 buffers the main stream stalled
        # 2.9 ms at block L-1 for the reader of its reuse (profiles/notes_r5.md, timeline gaps)
        self.d_branch2 = [e(N, C) for _ in range(4)]
        self.d_g = e(N * F)
        self.d_gu2 = [e(N * 2 * F) for _ in range(2)]
        self.d_att2 = [e(N * A) for _ in range(2)]
        self.d_qkv = e(N * QKV)
        self.d_qkv_raw2 = [e(N * QKV) for _ in range(2)]
        self.d_c = e(N, C)
        self._acts_shape = (B, T)

    @staticmethod
    def _rows(buf: Tensor, N: int, width: int) -> Tensor:
        """[N, width] view of the front of a flat per-block scratch buffer."""
        return buf[: N * width].view(N, width)

    def free_buffers(self):
        for name in ("resid", "mid", "y_in", "y_mlp", "qkv", "att", "lse", "gu", "g", "r_in", "r_pre", "r_pa",
                     "r_pm", "r_f", "s_attn", "s_mlp", "lnf_out", "_head_bufs", "tmp_c", "qkv_raw", "dresid",
                     "d_branch2", "d_g", "d_gu2", "d_att2", "d_qkv", "d_qkv_raw2", "d_c"):
            if hasattr(self, name):
                delattr(self, name)
        self._acts_shape = None

    def _rope(self, b: _GBlock, T: int):
        a = b.attn
        key = (a.rope_theta, b.D, T)
        tab = self._rope_tables.get(key)
        if tab is None:
            inv = a._inv_freq(b.D, self.device)
            tab = self._rope_tables[key] = rope_ops.rope_table(inv, 0, T, self.device)
        return tab

    def _mm(self, x: Tensor, w: Tensor, out: Tensor) -> Tensor:
        return torch.mm(x, w.t(), out=out)

    # ---- row-split AdamW of the embedding table ------------------------------------------------
    # The table's gradient is zero on every row this step's tokens do not touch (8k of 262k rows
    # at Gemma-3 1B B=8), and those rows' AdamW update does not depend on the backward. With the
    # optimizer fused into the backward and one micro-step per optimizer step, the untouched rows
    # are updated on the side stream while the forward runs (no gradient read); the touched rows
    # follow the embedding backward, which leaves the table's gradient all-zero again, so zero_grad
    # skips the 1.2 GB range. Bitwise the same update as the dense step. PENROZ_EMB_ROW_ADAM=0: off.
    def _row_split_begin(self, idx: Tensor):
        import os
        self._row_split = None
        app = self._opt_apply
        side = getattr(self, "_side", None)
        C = self.spec.C
        # (world > 1: a row untouched here may be touched on another rank — the averaged table
        # gradient is dense, so the per-bucket optimizer updates the table as a whole)
        if (app is None or not hasattr(app, "rows") or side is None or self._micro_since_zero != 1
                or self.reducer is not None
                or C % 4 or os.environ.get("PENROZ_EMB_ROW_ADAM", "1") == "0"):
            return
        es, ee = self.segments[self.L + 1]
        V = self.spec.V
        if (ee - es) != V * C or es % 4:
            return
        if getattr(self, "_emb_mask", None) is None:
            self._emb_mask = torch.zeros(V, dtype=torch.int32, device=self.device)
        rows = idx.reshape(-1).to(torch.int64)
        main = torch.cuda.current_stream(self.device)
        with torch.cuda.stream(side):
            side.wait_stream(main)
            self._emb_mask.zero_()
            self._emb_mask.index_fill_(0, rows, 1)
            app.rows(es, ee, C, self._emb_mask, None, 0)
        rows.record_stream(side)
        self._row_split = (es, ee, rows)

    def _segment_done(self, seg_index: int, sync: bool):
        rs = getattr(self, "_row_split", None)
        if rs is None or seg_index != self.L + 1 or self._opt_apply is None or not sync:
            return super()._segment_done(seg_index, sync)
        es, ee, rows = rs
        main = torch.cuda.current_stream(self.device)
        with torch.cuda.stream(self._side):
            self._side.wait_stream(main)
            self._opt_apply.rows(es, ee, self.spec.C, self._emb_mask, rows, 1)
        self._row_split = None
        self._zero_skip = (es, ee)  # the touched rows' gradient was cleared by the kernel

    # ------------------------------------------------------------------ forward
    def _combine_fwd(self, mode, x, a, w1, w2, eps1, eps2, h_out, y_out, s_save, r1, r2):
        _ext.kernels().gemma_combine_fwd(mode, x, a, w1, w2, float(eps1), float(eps2), h_out, y_out, s_save, r1, r2)

    def _forward(self, idx: Tensor, training: bool, dropout_seed: int = 0):
        s = self.spec
        B, T = idx.shape
        self._alloc(B, T)
        C, mode = s.C, s.mode
        N = B * T
        f = self.f32
        k = _ext.kernels()
        # scaled embedding (fp32 rows of the master table)
        torch.mul(torch.nn.functional.embedding(idx.reshape(-1), f(s.emb.weight)), s.emb.scale, out=self.resid[0])
        b0 = s.blocks[0]
        self._combine_fwd(3, self.resid[0], None, None, f(b0.in_norm.weight), 0.0, b0.in_norm.eps, None,
                          self.y_in[0], None, None, self.r_in[0])
        for l, b in enumerate(s.blocks):
            H, Hkv, D = b.H, b.Hkv, b.D
            qkv_raw = self._rows(self.qkv_raw, N, (H + 2 * Hkv) * D)
            self._mm(self.y_in[l], self.bf16(b.qkv.weight), qkv_raw)
            cos, sin = self._rope(b, T)
            k.rope_qkv(qkv_raw.view(B, T, -1), cos, sin, H, Hkv, D, False, self.qkv[l])
            p = b.attn.dropout if training else 0.0
            attn_ops.flash_fwd(self.qkv[l].view(B, T, -1), H, Hkv, D, p, dropout_seed + l,
                               out=self.att[l].view(B, T, H * D), lse=self.lse[l])
            self._mm(self.att[l], self.bf16(b.o.weight), self.tmp_c)
            post = b.post_attn
            if mode == 1:
                self.s_attn[l].copy_(self.tmp_c)
            self._combine_fwd(mode, self.resid[l], self.tmp_c, f(post.weight) if post is not None else None,
                              f(b.pre_mlp.weight), post.eps if post is not None else 0.0, b.pre_mlp.eps, self.mid[l],
                              self.y_mlp[l], self.s_attn[l] if mode == 0 else None,
                              self.r_pa[l] if self.r_pa is not None else None, self.r_pre[l])
            self._mm(self.y_mlp[l], self.gu_bf16(b), self.gu[l])
            k.gated_act_packed(self.gu[l], s.act, self.g[l])
            self._mm(self.g[l], self.bf16(b.mlp.down_proj.weight), self.tmp_c)
            last = l + 1 == self.L
            nxt = s.norm_f if last else s.blocks[l + 1].in_norm
            pm = b.post_mlp
            if mode == 1:
                self.s_mlp[l].copy_(self.tmp_c)
            self._combine_fwd(mode, self.mid[l], self.tmp_c, f(pm.weight) if pm is not None else None,
                              f(nxt.weight), pm.eps if pm is not None else 0.0, nxt.eps, self.resid[l + 1],
                              self.lnf_out if last else self.y_in[l + 1], self.s_mlp[l] if mode == 0 else None,
                              self.r_pm[l] if self.r_pm is not None else None,
                              self.r_f if last else self.r_in[l + 1])

    # ------------------------------------------------------------------ backward
    def _combine_bwd(self, mode, dy, dh_in, h, s_save, r1, r2, w1, w2, dx, da, dw1, dw2, dh_save=None):
        _ext.kernels().gemma_combine_bwd(mode, dy, dh_in, h, s_save if mode == 0 else None,
                                         s_save if mode == 1 else None, r1, r2, w1, w2, dx, da, dw1, dw2, dh_save)

    def _train_micro_step(self, idx: Tensor, targets: Tensor, scale: float, sync: bool, capture: bool) -> Tensor:
        s = self.spec
        B, T = idx.shape
        N, C, mode = B * T, s.C, s.mode
        seed = self._step_seed
        self._step_seed += 1000
        f, gr = self.f32, self.grad
        k = _ext.kernels()
        self._refresh_transposed()
        self._micro_since_zero = getattr(self, "_micro_since_zero", 0) + 1
        self._row_split_begin(idx)
        with trace_range("forward"):
            self._forward(idx, training=True, dropout_seed=seed)
        cap = capture and self._captured is None
        head_range = trace_range("backward.head")
        head_range.__enter__()
        self._defer_reductions(True)
        tg = targets.reshape(-1)
        if cap:
            full = self._full_logits()
            acts = [self.resid[0].view(B, T, C).clone()] + [r.view(B, T, C).clone() for r in self.resid[1:]] + \
                   [self.lnf_out.view(B, T, C).float().clone(), full.view(B, T, -1).clone()]
            chunks = [(0, N, full)]
            dh_caps = [torch.empty(N, C, dtype=torch.float32, device=self.device) for _ in range(self.L + 1)]
        else:
            chunks = [(r0, min(N, r0 + self.head_chunk), None) for r0 in range(0, N, self.head_chunk)]
            dh_caps = None
        loss = torch.zeros((), dtype=torch.float32, device=self.device)
        w_head = self._dgrad(s.head.weight, self.bf16(s.head.weight))
        for i, (r0, r1, lg) in enumerate(chunks):
            if lg is None:
                lg = self._head_logits(r0, r1, self._reuse(self._head_bufs[i % len(self._head_bufs)]))
            loss += fused_ops.cross_entropy_fwd_bwd(lg, tg[r0:r1], scale / N).sum()
            torch.mm(lg, w_head, out=self.d_c[r0:r1])
            self._wgrad(lg, self.lnf_out[r0:r1], s.head.weight)
        loss *= scale / N
        if cap:
            grads_cap = [full.view(B, T, -1).clone(), self.d_c.view(B, T, C).float().clone()]
        # final combine (last block's MLP side + the final norm): dh_in none
        lb = s.blocks[-1]
        pm = lb.post_mlp
        db = self._reuse(self.d_branch2[0])
        self._combine_bwd(mode, self.d_c, None, self.resid[self.L], self.s_mlp[-1] if self.s_mlp else None,
                          self.r_pm[-1] if self.r_pm else None, self.r_f, f(pm.weight) if pm is not None else None,
                          f(s.norm_f.weight), self.dresid, db, gr(pm.weight) if pm is not None else None,
                          gr(s.norm_f.weight), dh_save=dh_caps[self.L] if cap else None)
        self._segment_done(0, sync)
        head_range.__exit__(None, None, None)
        rb = 0
        for l in range(self.L - 1, -1, -1):
            layer_range = trace_range(f"backward.block{l}")
            layer_range.__enter__()
            b = s.blocks[l]
            H, Hkv, D = b.H, b.Hkv, b.D
            QKV = (H + 2 * Hkv) * D
            db = self.d_branch2[rb]
            # ---- MLP: down dgrad / wgrad, packed gated backward, gate|up dgrad / wgrad
            d_g = self._rows(self.d_g, N, b.F)
            torch.mm(db, self._dgrad(b.mlp.down_proj.weight, self.bf16(b.mlp.down_proj.weight)), out=d_g)
            self._wgrad(db, self.g[l], b.mlp.down_proj.weight)
            dgu = self._rows(self._reuse(self.d_gu2[l & 1]), N, 2 * b.F)
            k.gated_act_bwd_packed(d_g, self.gu[l], dgu, s.act)
            torch.mm(dgu, self._dgrad(b.mlp.gate_proj.weight, self.gu_bf16(b)), out=self.d_c)
            self._wgrad_into(id(b.mlp.gate_proj.weight), dgu, self.y_mlp[l], self.gu_grad(b))
            # ---- attention combine: dy = d(pre-MLP norm output), dh_in = dresid (grad of mid[l])
            pa = b.post_attn
            rb = (rb + 1) % len(self.d_branch2)
            db = self._reuse(self.d_branch2[rb])
            self._combine_bwd(mode, self.d_c, self.dresid, self.mid[l], self.s_attn[l] if self.s_attn else None,
                              self.r_pa[l] if self.r_pa else None, self.r_pre[l],
                              f(pa.weight) if pa is not None else None, f(b.pre_mlp.weight), self.dresid, db,
                              gr(pa.weight) if pa is not None else None, gr(b.pre_mlp.weight))
            # ---- attention: O dgrad / wgrad, flash backward, inverse RoPE, QKV dgrad / wgrad
            datt = self._rows(self._reuse(self.d_att2[l & 1]), N, H * D)
            torch.mm(db, self._dgrad(b.o.weight, self.bf16(b.o.weight)), out=datt)
            self._wgrad(db, self.att[l], b.o.weight)
            d_qkv = self._rows(self.d_qkv, N, QKV)
            attn_ops.flash_bwd(datt.view(B, T, H * D), self.qkv[l].view(B, T, -1), self.att[l].view(B, T, H * D),
                               self.lse[l], H, Hkv, D, b.attn.dropout, seed + l, dqkv=d_qkv.view(B, T, -1))
            cos, sin = self._rope(b, T)
            dqr = self._rows(self._reuse(self.d_qkv_raw2[l & 1]), N, QKV)
            k.rope_qkv(d_qkv.view(B, T, -1), cos, sin, H, Hkv, D, True, dqr)
            torch.mm(dqr, self._dgrad(b.qkv.weight, self.bf16(b.qkv.weight)), out=self.d_c)
            self._wgrad(dqr, self.y_in[l], b.qkv.weight)
            # ---- the combine that produced y_in[l]: block l-1's MLP combine (or the embedding norm)
            if l > 0:
                pb = s.blocks[l - 1]
                pm = pb.post_mlp
                rb = (rb + 1) % len(self.d_branch2)
                db = self._reuse(self.d_branch2[rb])
                self._combine_bwd(mode, self.d_c, self.dresid, self.resid[l],
                                  self.s_mlp[l - 1] if self.s_mlp else None, self.r_pm[l - 1] if self.r_pm else None,
                                  self.r_in[l], f(pm.weight) if pm is not None else None, f(b.in_norm.weight),
                                  self.dresid, db, gr(pm.weight) if pm is not None else None, gr(b.in_norm.weight),
                                  dh_save=dh_caps[l] if cap else None)
            else:
                self._combine_bwd(3, self.d_c, self.dresid, self.resid[0], None, None, self.r_in[0], None,
                                  f(b.in_norm.weight), self.dresid, None, None, gr(b.in_norm.weight),
                                  dh_save=dh_caps[0] if cap else None)
            self._segment_done(self.L - l, sync)
            layer_range.__exit__(None, None, None)
        # embedding: dW[idx] += scale · dx0
        gw = gr(s.emb.weight)
        gw.index_add_(0, idx.reshape(-1), self.dresid, alpha=float(s.emb.scale))
        self._segment_done(self.L + 1, sync)
        self._defer_reductions(False)
        self._finish_wgrad_bookkeeping()
        self._join_side()
        if sync and self.reducer is not None:
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
            # block outputs' gradients: dh of the combine that produced each resid[l]
            act_grads = [dh_caps[0].view(B, T, C)] + [dh_caps[l].view(B, T, C) for l in range(1, self.L + 1)] + \
                        [grads_cap[1], grads_cap[0]]
            algos = [m.__class__.__name__.lower() for m in self.model.layers]
            pairs = list(zip(acts, act_grads))
            self._captured = (algos, pairs[:len(algos)])
        return loss
