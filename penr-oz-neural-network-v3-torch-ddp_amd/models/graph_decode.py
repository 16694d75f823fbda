"""Graph-captured incremental decoding: one HIP graph replays a whole decode step.

The reference decodes one token per Python iteration through every layer module
(``neural_net_model.py:360-406, 457-514``) and grows its KV cache with ``torch.cat``. At
batch 64 on MI355X that per-token path is launch-bound: ~150 kernel launches plus Python
dispatch per token cost ~2.9 ms while the actual work (weights + cache read once) is ~0.2 ms.

Here the decode step — the model's own module forward (so numerics are the eager path's:
same LayerNorm / GELU / decode-attention kernels, same GEMMs), KV append, sampling, and the
feedback of the sampled token into the next step's input — is captured ONCE per
(rows, block size, sampling settings) into a ``torch.cuda.CUDAGraph`` (a hipGraph on ROCm) and
replayed. Everything that changes between steps lives on the device:

* ``StaticKVCache.pos_t`` / ``len_t``: the slot this step writes and the cache length after it;
  the decode-attention kernel reads q in place and ``len_t`` at run time, and appends this step's
  K/V (read in place from the fused QKV rows, int8-quantised for TurboQuant) at slot
  ``len_t - 1 = pos_t`` itself (``csrc/kernels/decode_attn.hip``: ``k_new``, ``seq_len_dev``);
* ``PositionEmbedding.position_offset_tensor``: the learned position gathered at ``pos_t``;
* the sampler hashes its uniforms on the device from (seed of the generate call, absolute token
  index, row) and writes the token straight into the next step's input and the burst output
  buffer; one tiny kernel then advances the position / length / step counters. Streaming and
  non-streaming calls therefore draw identical tokens under the same ``torch.manual_seed``;
* the step's ``nn.Linear`` GEMMs (M = rows ≤ 64) run on the decode-shaped MFMA kernel
  (``csrc/kernels/skinny_gemm.hip``): called explicitly by the decode programs, or — for the
  module-forward fallback — through ``ops/gemm.py: decode_gemms(model)``, which re-routes only
  that model's own ``nn.Linear`` instances for the capture.

The host only tracks the cache length (one per replay) to switch to the reference's
sliding-window re-prefill when the window is full, and copies each burst of tokens back once
(stop-token checks per burst). Prefill and re-prefill run eagerly. RoPE models (Gemma) rotate
with a cos/sin table computed on the device from ``pos_t`` once per step
(``_GraphMode.rope_table``); their head_dim 256 runs on the same decode-attention kernel.
"""
from __future__ import annotations

import gc
import logging
import os
import weakref

import torch
from torch import Tensor

from penroz.models import kv_cache as kvc
from penroz.ops import _ext
from penroz.ops import activations as act_ops
from penroz.ops import attention as attn_ops
from penroz.ops import fused as fused_ops
from penroz.ops import gemm as gemm_ops
from penroz.ops import norms as norm_ops
from penroz.ops import rope as rope_ops
from penroz.ops import sampling as samp_ops

log = logging.getLogger(__name__)

GRAPH_DECODE = os.environ.get("PENROZ_GRAPH_DECODE", "1") != "0"
# GPT-2-pattern bf16 models: the captured step is the explicit program below instead of the
# module forward ("0": module forward, numerically identical to the eager decode path)
DECODE_PROGRAM = os.environ.get("PENROZ_DECODE_PROGRAM", "1") != "0"
# the decode-attention kernel appends the step's K/V itself (one kernel less per layer); "0":
# separate kv_append kernel
FUSED_APPEND = os.environ.get("PENROZ_FUSED_APPEND", "1") != "0"
# decode rows up to which the linears use the decode-shaped MFMA kernel instead of hipBLASLt
# (measured: a win at batch 1, none at batch 64 — profiles/bench_r1_decode_graph.log)
SKINNY_MAX_ROWS = int(os.environ.get("PENROZ_SKINNY_MAX_ROWS", "16"))
# Gemma program: RoPE and the gated activation in the skinny GEMM epilogues ("1", default) or the
# separate RoPE / packed-activation kernels after plain skinny GEMMs ("0": same-box A/B switch)
DECODE_EPILOGUES = os.environ.get("PENROZ_DECODE_EPILOGUES", "1") != "0"
# GPT decode program: residual add + LayerNorm fused in front of the QKV and fc GEMMs (and GELU
# behind fc) in one decode-shaped kernel (csrc/kernels/skinny_gemm.hip decode_ln_linear); "0":
# separate add+LN, GEMM and GELU kernels
FUSED_LN_LINEAR = os.environ.get("PENROZ_DECODE_FUSED", "1") != "0"
# ... up to this many decode rows: every workgroup normalises all rows itself, which pays off
# while the rows are few (batch 1 / 4 / 8: -8 / -10 / -3 %) and loses from 16 rows on (+14 % at 16,
# +69 % at 64): profiles/decode_fused_rows_r2.log
FUSED_MAX_ROWS = int(os.environ.get("PENROZ_DECODE_FUSED_MAX_ROWS", "8"))
# ... above that: the batched block (csrc/kernels/decode_linear.hip) — 5 kernels per block, the
# fp32 residual updated in place by the proj / fc2 epilogues, LayerNorm recomputed per 16-row
# block inside the QKV / fc GEMMs; "0": add+LN, GEMM, GELU kernels (8 per block)
BATCHED_BLOCK = os.environ.get("PENROZ_DECODE_BATCHED", "1") != "0"
# ... and up to this many rows (batch 1-4) every linear of the GPT block — the LN-fused QKV and
# fc(+GELU), proj, fc2 and the lm_head — runs as the one-wave-per-workgroup decode GEMV
# (csrc/kernels/decode_linear.hip decode_gemv: one memory round trip, no LDS, no barrier, no
# split-K hand-off); "0": decode_ln_linear + skinny GEMMs
GEMV_MAX_ROWS = int(os.environ.get("PENROZ_DECODE_GEMV_MAX_ROWS", "4"))
# decode_gemv's reduction limit (256 lanes × 32 values, decode_linear.hip); wider linears take the
# skinny GEMM
GEMV_MAX_K = 8192
# the sampler's last row advances the step counters itself (sample_step with adv_a / adv_b / done:
# one launch less per token); "0": the separate decode_advance kernel
FUSED_ADVANCE = os.environ.get("PENROZ_DECODE_FUSED_ADVANCE", "1") != "0"


class _GraphMode:
    """Mixin: ``attend`` switches to device-positioned append + attention while capturing."""

    graph_mode = False

    def init_graph_state(self, device):
        self.pos_t = torch.zeros(1, dtype=torch.long, device=device)  # slot written by the step
        self.len_t = torch.ones(1, dtype=torch.long, device=device)   # cache length after it
        self._rope_tables: dict = {}

    def begin_step(self):
        self._rope_tables.clear()

    def rope_table(self, key, inv_freq: Tensor, T: int):
        """cos / sin for positions pos_t..pos_t+T-1, computed on the device once per step and
        ``key`` = (theta, head_dim): layers with the same rotary setup share it."""
        key = (*key, T)
        tab = self._rope_tables.get(key)
        if tab is None:
            tab = self._rope_tables[key] = rope_ops.rope_table(inv_freq, 0, T, inv_freq.device, offset_dev=self.pos_t)
        return tab

    def attend(self, layer_idx: int, q: Tensor, k: Tensor, v: Tensor) -> Tensor:
        if not self.graph_mode:
            return super().attend(layer_idx, q, k, v)
        return self._attend_graph(layer_idx, q, k, v)


class StaticKVCache(_GraphMode, kvc.KVCache):
    def _attend_graph(self, l: int, q: Tensor, k: Tensor, v: Tensor) -> Tensor:
        # k, v, q are views into this layer's fused QKV rows: one kernel appends K/V at pos_t,
        # the decode kernel reads q in place and the cache length from len_t
        kc, vc = self._k[l], self._v[l]
        if FUSED_APPEND:
            return attn_ops.decode_attention(q, kc, vc, kc.shape[2], seq_len_dev=self.len_t, k_new=k, v_new=v)
        _ext.kernels().kv_append(k, v, kc, vc, None, None, self.pos_t, 0)
        return attn_ops.decode_attention(q, kc, vc, kc.shape[2], seq_len_dev=self.len_t)


    def rope_attend_ok(self, B: int, H: int, Hkv: int, D: int) -> bool:
        """``attend_rope`` applies: opted in (PENROZ_DECODE_ROPE_IN_ATTN=1), graph mode with the
        fused append, the small decode kernel. Off by default: Gemma-3 1B batch 32 / 64 measured
        2.108 / 2.100 and 2.442 / 2.445 ms/step with it vs 2.074 / 2.077 and 2.425 / 2.433 ms with
        the separate RoPE pass (profiles/negative_r6_rope_in_decode_attn.log)."""
        kc = self._k[0]
        return (os.environ.get("PENROZ_DECODE_ROPE_IN_ATTN", "0") == "1" and self.graph_mode and FUSED_APPEND
                and _ext.available()
                and attn_ops.decode_rope_fusable(B, H, Hkv, D, kc.shape[2], kc.dtype))

    def attend_rope(self, l: int, q: Tensor, k: Tensor, v: Tensor, cos: Tensor, sin: Tensor) -> Tensor:
        """``attend`` with q / k unrotated: the decode kernel applies RoPE (cos / sin [1, D/2]) to
        q and to the key it appends, in place of a separate RoPE pass over the QKV rows."""
        kc, vc = self._k[l], self._v[l]
        return attn_ops.decode_attention(q, kc, vc, kc.shape[2], seq_len_dev=self.len_t, k_new=k, v_new=v,
                                         rope=(cos.view(-1), sin.view(-1)))


class StaticTurboKVCache(_GraphMode, kvc.TurboQuantKVCache):
    def _attend_graph(self, l: int, q: Tensor, k: Tensor, v: Tensor) -> Tensor:
        # same per-token int8 quantiser as the eager append (kv_quantize)
        self._dtype[l] = k.dtype
        if FUSED_APPEND:
            return attn_ops.decode_attention(q, self._k[l], self._v[l], self._k[l].shape[2], self._sk[l],
                                             self._sv[l], seq_len_dev=self.len_t, k_new=k, v_new=v)
        _ext.kernels().kv_append(k, v, self._k[l], self._v[l], self._sk[l], self._sv[l], self.pos_t, 0)
        return attn_ops.decode_attention(q, self._k[l], self._v[l], self._k[l].shape[2], self._sk[l], self._sv[l],
                                         seq_len_dev=self.len_t)


class GPTDecodeProgram:
    """One decode step of a GPT-2-pattern bf16 model as an explicit kernel sequence.

    The module forward costs ~12 kernels per block at decode shapes (residual adds and dtype
    glue included) and every kernel has a fixed ~4-5 µs cost in a replayed graph at batch 64 —
    more than most of them compute. Per block this runs 9: [add-residual + fc2 bias + LN1] →
    QKV GEMM+bias → KV append → decode attention → proj GEMM → [add-residual + proj bias + LN2]
    → fc GEMM+bias → GELU → fc2 GEMM, with the residual stream kept in fp32 (the training executor's
    numerics; the module path rounds it to bf16 after every add). The embedding reads the
    position from the device.
    """

    def __init__(self, model, spec):
        self.spec = spec
        dev = spec.wte.weight.device
        # LayerNorm kernels take fp32 affine parameters
        self.ln = [(b.ln1.weight.float(), b.ln1.bias.float(), b.ln1.eps, b.ln2.weight.float(), b.ln2.bias.float(),
                    b.ln2.eps) for b in spec.blocks]
        self.lnf = (spec.lnf.weight.float(), spec.lnf.bias.float(), spec.lnf.eps)
        # proj / fc2 biases are added by the following add+LN kernel (fp32), so those two GEMMs
        # run without a bias epilogue (hipBLASLt's pick for fc2 at M = 64 has none: torch then
        # launches an extra bias-broadcast copy per call)
        self.out_bias = [(b.proj.bias.float(), b.fc2.bias.float()) for b in spec.blocks]
        self.device = dev

    @staticmethod
    def build(model):
        if not DECODE_PROGRAM:
            return None
        from penroz.models.executor import GPTExecutor
        spec = GPTExecutor.match(model)
        if spec is None or any(p.dtype != torch.bfloat16 for p in model.parameters()):
            return None
        return GPTDecodeProgram(model, spec)

    def _linear(self, x: Tensor, lin, bias: bool = True) -> Tensor:
        b = lin.bias if bias else None
        if x.shape[0] <= SKINNY_MAX_ROWS and gemm_ops.skinny_ok(x, lin.weight):
            return gemm_ops.skinny_linear(x, lin.weight, b)
        if b is not None:
            return torch.addmm(b, x, lin.weight.t())
        return torch.mm(x, lin.weight.t())

    def _gemv_ok(self, rows: int) -> bool:
        sp = self.spec
        return (1 <= rows <= min(4, GEMV_MAX_ROWS) and sp.C % 8 == 0 and sp.C <= 1024
                and sp.blocks[0].fc.out_features % 8 == 0 and sp.gelu_approx in ("none", "tanh") and _ext.available())

    def _fused_ok(self, rows: int) -> bool:
        sp = self.spec
        return (FUSED_LN_LINEAR and 1 <= rows <= min(64, FUSED_MAX_ROWS) and sp.C % 32 == 0 and sp.C <= 1024
                and sp.gelu_approx in ("none", "tanh") and _ext.available())

    def _batched_ok(self, rows: int) -> bool:
        sp = self.spec
        return (BATCHED_BLOCK and rows > FUSED_MAX_ROWS and sp.C % 32 == 0 and sp.C <= 1024
                and sp.blocks[0].fc.out_features % 32 == 0 and sp.gelu_approx in ("none", "tanh")
                and _ext.available())

    def forward(self, idx: Tensor, cache) -> Tensor:
        """idx [rows, 1] -> logits [rows, V] (bf16); appends this step's K/V at cache.pos_t."""
        sp = self.spec
        rows, C, H, D = idx.shape[0], sp.C, sp.H, sp.D
        if (rows == 1 and self._gemv_ok(rows) and sp.wte.weight.dtype == torch.bfloat16
                and sp.wpe.weight.dtype == torch.bfloat16):
            # the first block's LN + QKV GEMV reads the embedding row itself (no embedding kernel):
            # B = 1 0.3548 / 0.3564 -> 0.3520 / 0.3544 ms; at 4 rows every workgroup's four-row
            # gather cost more than the launch it saves (0.535 -> 0.551), profiles/decode_r5.md
            x = torch.empty(rows, C, dtype=torch.float32, device=idx.device)
            return self._forward_gemv(x, torch.empty_like(x), rows, cache, emb=(idx.reshape(-1).contiguous(), cache.pos_t))
        x = fused_ops.embedding_fwd(idx, sp.wte.weight, sp.wpe.weight, 0, pos_dev=cache.pos_t)  # fp32 [rows, C]
        if self._batched_ok(rows):
            return self._forward_batched(x, rows, cache)
        x2 = torch.empty_like(x)  # the residual stream ping-pongs between x and x2 (no aliasing)
        if self._gemv_ok(rows):
            return self._forward_gemv(x, x2, rows, cache)
        if self._fused_ok(rows):
            return self._forward_fused(x, x2, rows, cache)

        def add_ln(delta, w, b, eps, dbias=None):
            nonlocal x, x2
            y, _, _ = norm_ops.add_ln_fwd(x, delta, x2, w, b, eps, delta_bias=dbias)
            x, x2 = x2, x
            return y

        delta = dbias = None
        for l, blk in enumerate(sp.blocks):
            w1, b1, e1, w2, b2, e2 = self.ln[l]
            pb, fb = self.out_bias[l]
            if delta is None:
                y, _, _ = norm_ops.ln_fwd(x, w1, b1, e1)
            else:
                y = add_ln(delta, w1, b1, e1, dbias)
            qkv = self._linear(y, blk.qkv).view(rows, 1, 3 * C)
            q = qkv[:, :, :C].view(rows, 1, H, D)
            k = qkv[:, :, C:2 * C].view(rows, 1, H, D)
            v = qkv[:, :, 2 * C:].view(rows, 1, H, D)
            o = cache._attend_graph(l, q, k, v)
            d = self._linear(o.view(rows, C), blk.proj, bias=False)
            y = add_ln(d, w2, b2, e2, pb)
            h = self._linear(y, blk.fc)
            h = act_ops.gelu_fwd(h, sp.gelu_approx, out=h)
            delta, dbias = self._linear(h, blk.fc2, bias=False), fb
        wf, bf, ef = self.lnf
        return self._linear(add_ln(delta, wf, bf, ef, dbias), sp.head)

    def _forward_fused(self, x: Tensor, x2: Tensor, rows: int, cache) -> Tensor:
        """Per block: [add + LN1 + QKV GEMM + bias] → decode attention (K/V append fused) → proj
        GEMM → [add + proj bias + LN2 + fc GEMM + bias + GELU] → fc2 GEMM: 5 kernels instead of 8."""
        sp = self.spec
        K = _ext.kernels()
        C, H, D = sp.C, sp.H, sp.D
        act = 2 if sp.gelu_approx == "tanh" else 1
        delta = dbias = None
        for l, blk in enumerate(sp.blocks):
            w1, b1, e1, w2, b2, e2 = self.ln[l]
            pb, fb = self.out_bias[l]
            qkv = torch.empty(rows, 3 * C, dtype=torch.bfloat16, device=x.device)
            if delta is None:
                K.decode_ln_linear(x, None, None, None, w1, b1, e1, blk.qkv.weight, blk.qkv.bias, qkv, 0)
            else:
                K.decode_ln_linear(x, delta, dbias, x2, w1, b1, e1, blk.qkv.weight, blk.qkv.bias, qkv, 0)
                x, x2 = x2, x
            qkv = qkv.view(rows, 1, 3 * C)
            q = qkv[:, :, :C].view(rows, 1, H, D)
            k = qkv[:, :, C:2 * C].view(rows, 1, H, D)
            v = qkv[:, :, 2 * C:].view(rows, 1, H, D)
            o = cache._attend_graph(l, q, k, v)
            d = self._linear(o.view(rows, C), blk.proj, bias=False)
            h = torch.empty(rows, blk.fc.out_features, dtype=torch.bfloat16, device=x.device)
            K.decode_ln_linear(x, d, pb, x2, w2, b2, e2, blk.fc.weight, blk.fc.bias, h, act)
            x, x2 = x2, x
            delta, dbias = self._linear(h, blk.fc2, bias=False), fb
        wf, bf, ef = self.lnf
        y, _, _ = norm_ops.add_ln_fwd(x, delta, x2, wf, bf, ef, delta_bias=dbias)
        return self._linear(y, sp.head)


    def _forward_gemv(self, x: Tensor, x2: Tensor, rows: int, cache, emb=None) -> Tensor:
        """Batch 1-4, per block: [add + LN1 + QKV GEMV + bias] → decode attention (K/V append fused)
        → proj GEMV → [add + proj bias + LN2 + fc GEMV + bias + GELU] → fc2 GEMV; then the final
        add + LN and the lm_head GEMV — every linear one decode_gemv launch. ``emb`` = (token ids,
        device position): the first GEMV builds the residual rows wte[tok] + wpe[pos] itself and
        writes them to ``x`` (one kernel less per token)."""
        sp = self.spec
        K = _ext.kernels()
        C, H, D = sp.C, sp.H, sp.D
        act = 2 if sp.gelu_approx == "tanh" else 1
        delta = dbias = None
        for l, blk in enumerate(sp.blocks):
            w1, b1, e1, w2, b2, e2 = self.ln[l]
            pb, fb = self.out_bias[l]
            qkv = torch.empty(rows, 3 * C, dtype=torch.bfloat16, device=x.device)
            if delta is None and emb is not None:
                K.decode_gemv(None, None, None, None, x, w1, b1, e1, blk.qkv.weight, blk.qkv.bias, qkv, 0,
                              emb_idx=emb[0], emb_wte=sp.wte.weight, emb_wpe=sp.wpe.weight, emb_pos=emb[1])
            elif delta is None:
                K.decode_gemv(None, x, None, None, None, w1, b1, e1, blk.qkv.weight, blk.qkv.bias, qkv, 0)
            else:
                K.decode_gemv(None, x, delta, dbias, x2, w1, b1, e1, blk.qkv.weight, blk.qkv.bias, qkv, 0)
                x, x2 = x2, x
            qkv = qkv.view(rows, 1, 3 * C)
            q = qkv[:, :, :C].view(rows, 1, H, D)
            k = qkv[:, :, C:2 * C].view(rows, 1, H, D)
            v = qkv[:, :, 2 * C:].view(rows, 1, H, D)
            o = cache._attend_graph(l, q, k, v).view(rows, C)
            d = torch.empty(rows, C, dtype=torch.bfloat16, device=x.device)
            K.decode_gemv(o, None, None, None, None, None, None, 0.0, blk.proj.weight, None, d, 0)
            h = torch.empty(rows, blk.fc.out_features, dtype=torch.bfloat16, device=x.device)
            K.decode_gemv(None, x, d, pb, x2, w2, b2, e2, blk.fc.weight, blk.fc.bias, h, act)
            x, x2 = x2, x
            delta = torch.empty(rows, C, dtype=torch.bfloat16, device=x.device)
            K.decode_gemv(h, None, None, None, None, None, None, 0.0, blk.fc2.weight, None, delta, 0)
            dbias = fb
        wf, bf, ef = self.lnf
        logits = torch.empty(rows, sp.head.weight.shape[0], dtype=torch.bfloat16, device=x.device)
        K.decode_gemv(None, x, delta, dbias, x2, wf, bf, ef, sp.head.weight, None, logits, 0)
        return logits

    def _forward_batched(self, x: Tensor, rows: int, cache) -> Tensor:
        """Per block: [LN1 + QKV GEMM + bias] → decode attention (K/V append fused) → [proj GEMM +
        bias, added into the fp32 residual in place] → [LN2 + fc GEMM + bias + GELU] → [fc2 GEMM +
        bias, added into the residual]: 5 kernels instead of 8."""
        sp = self.spec
        K = _ext.kernels()
        C, H, D = sp.C, sp.H, sp.D
        act = 2 if sp.gelu_approx == "tanh" else 1
        for l, blk in enumerate(sp.blocks):
            w1, b1, e1, w2, b2, e2 = self.ln[l]
            qkv = torch.empty(rows, 3 * C, dtype=torch.bfloat16, device=x.device)
            K.decode_ln_gemm(x, w1, b1, e1, blk.qkv.weight, blk.qkv.bias, qkv, 0)
            qkv = qkv.view(rows, 1, 3 * C)
            q = qkv[:, :, :C].view(rows, 1, H, D)
            k = qkv[:, :, C:2 * C].view(rows, 1, H, D)
            v = qkv[:, :, 2 * C:].view(rows, 1, H, D)
            o = cache._attend_graph(l, q, k, v)
            K.decode_gemm_acc(o.view(rows, C), blk.proj.weight, blk.proj.bias, x)
            h = torch.empty(rows, blk.fc.out_features, dtype=torch.bfloat16, device=x.device)
            K.decode_ln_gemm(x, w2, b2, e2, blk.fc.weight, blk.fc.bias, h, act)
            K.decode_gemm_acc(h, blk.fc2.weight, blk.fc2.bias, x)
        wf, bf, ef = self.lnf
        y, _, _ = norm_ops.ln_fwd(x, wf, bf, ef)
        return self._linear(y, sp.head)


def _packed_gate_up(mlp):
    """The [gate; up] weight of one gated MLP as one contiguous tensor, built once per weight
    version and cached on the module, so every decoder of the model shares one copy (no autograd
    graph: built under no_grad)."""
    g, u = mlp.gate_proj.weight, mlp.up_proj.weight
    key = (g.data_ptr(), g._version, u.data_ptr(), u._version)
    hit = mlp.__dict__.get("_packed_gu")
    if hit is not None and hit[0] == key:
        return hit[1]
    with torch.no_grad():
        gu = torch.cat([g, u]).contiguous()
    mlp.__dict__["_packed_gu"] = (key, gu)
    return gu


class GemmaDecodeProgram:
    """One decode step of a Gemma-family bf16 model (``models/hf.py`` layer list) as an explicit
    kernel sequence.

    The module forward runs ~16 kernels per block at decode shapes (four RMSNorms, two residual
    adds, separate gate and up GEMMs). Per block this runs 6 (+1 split-K combine): QKV GEMM with
    RoPE (device-offset table) in its epilogue (``skinny_qkv_rope``) → decode attention with fused K/V append → O GEMM →
    [residual add + post-attention norm + pre-MLP norm] → gate|up GEMM (one concatenated weight)
    with the gated activation in its epilogue (``skinny_gated``) → down GEMM → [residual add +
    post-MLP norm + the next block's input norm]. Rounding follows the module path (bf16 residual stream, torch's rounding
    points), so only the GEMM accumulation order of the fused gate|up projection can differ.
    Reference block semantics: ``neural_net_layers.py:188-225``.
    """

    def __init__(self, emb, blocks, norm_f, head):
        self.emb, self.norm_f, self.head = emb, norm_f, head
        self.blocks = []
        for b in blocks:
            in_norm, qkv, attn, o = list(b.attn_block)
            pre_mlp, mlp = list(b.mlp_block)
            if b.post_attn_norm is None:
                mode = 2
            else:
                mode = 0 if b.post_norm_on_residual else 1
            self.blocks.append(dict(
                in_norm=in_norm, qkv=qkv.weight, attn=attn, o=o.weight, pre_mlp=pre_mlp, mode=mode,
                post_attn=b.post_attn_norm, post_mlp=b.post_mlp_norm,
                gu=_packed_gate_up(mlp), down=mlp.down_proj.weight,
                kind=act_ops._GATED[mlp.act_kind], inter=mlp.gate_proj.out_features))

    @staticmethod
    def build(model):
        if not DECODE_PROGRAM:
            return None
        from torch import nn
        from penroz.models import layers as L
        mods = list(model.layers)
        if mods and isinstance(mods[-1], L.SoftmaxOnLast):
            mods = mods[:-1]
        if (len(mods) < 4 or not isinstance(mods[0], L.ScaledEmbedding) or not isinstance(mods[-2], L.RMSNorm)
                or not isinstance(mods[-1], nn.Linear) or mods[-1].bias is not None):
            return None
        if any(p.dtype != torch.bfloat16 for p in model.parameters()):
            return None
        C = mods[0].embedding_dim
        if C % 8 or C > 6144:
            return None
        for b in mods[1:-2]:
            if not isinstance(b, L.TransformerBlock) or (b.post_attn_norm is None) != (b.post_mlp_norm is None):
                return None
            ab, mb = list(b.attn_block), list(b.mlp_block)
            if not (len(ab) == 4 and isinstance(ab[0], L.RMSNorm) and isinstance(ab[1], nn.Linear)
                    and isinstance(ab[2], L.CausalSelfAttention) and isinstance(ab[3], nn.Linear)
                    and len(mb) == 2 and isinstance(mb[0], L.RMSNorm) and isinstance(mb[1], L.GatedMLP)):
                return None
            a, mlp = ab[2], mb[1]
            if (ab[1].bias is not None or ab[3].bias is not None or mlp.gate_proj.bias is not None
                    or mlp.down_proj.bias is not None or a.head_dim not in attn_ops.DECODE_HEAD_DIMS
                    or mlp.gate_proj.out_features % 8):
                return None
            norms = [ab[0], mb[0]] + ([b.post_attn_norm, b.post_mlp_norm] if b.post_attn_norm is not None else [])
            if any(not isinstance(n, L.RMSNorm) for n in norms):
                return None
        return GemmaDecodeProgram(mods[0], mods[1:-2], mods[-2], mods[-1])

    def _gemv_ok(self, rows: int, C: int) -> bool:
        """Batch 1-4: every projection as one decode GEMV (decode_gemv / decode_gemv_pair:
        one wave per workgroup, one memory round trip; RoPE and the gated activation in the
        paired-row epilogues)."""
        # decode_gemv reads K <= 8192 (decode_linear.hip); the O and down projections read K = H·D
        # and the intermediate size (12288 on Gemma-4 e2b's KV-shared double-wide MLPs)
        return (1 <= rows <= min(4, GEMV_MAX_ROWS) and C % 8 == 0 and C <= 1792 and _ext.available()
                and all(b["o"].shape[1] <= GEMV_MAX_K and b["down"].shape[1] <= GEMV_MAX_K for b in self.blocks))

    def forward(self, idx: Tensor, cache) -> Tensor:
        """idx [rows, 1] -> logits [rows, V] (bf16); appends this step's K/V at cache.pos_t."""
        K = _ext.kernels()
        rows = idx.shape[0]
        gemv = self._gemv_ok(rows, self.emb.embedding_dim)

        def lin(x: Tensor, w: Tensor) -> Tensor:
            if gemv and w.shape[1] % 8 == 0 and w.shape[1] <= GEMV_MAX_K:
                out = torch.empty(rows, w.shape[0], device=x.device, dtype=torch.bfloat16)
                K.decode_gemv(x.contiguous(), None, None, None, None, None, None, 0.0, w, None, out, 0)
                return out
            return _linear(x, w)

        x = torch.nn.functional.embedding(idx.view(rows), self.emb.weight) * self.emb.scale
        first = self.blocks[0]["in_norm"]
        y = K.rmsnorm_fwd(x, first.weight, first.eps)[0]
        if gemv and DECODE_EPILOGUES and all(b["attn"].rope_theta is not None and b["attn"].head_dim % 2 == 0
                                             for b in self.blocks):
            return self._forward_gemv(K, rows, x, y, cache)
        for l, b in enumerate(self.blocks):
            a = b["attn"]
            H, Hkv, D = a.num_heads, a.num_kv_heads, a.head_dim
            if a.rope_theta is not None:
                inv = a._inv_freq(D, y.device)
                cos, sin = cache.rope_table((a.rope_theta, D), inv, 1)
                if gemv and DECODE_EPILOGUES and D % 2 == 0:
                    qkv = torch.empty(rows, b["qkv"].shape[0], device=y.device, dtype=torch.bfloat16)
                    K.decode_gemv_pair(y.contiguous(), b["qkv"], qkv, 2, 0, D, H + Hkv, cos, sin)
                    qkv = qkv.view(rows, 1, -1)
                elif DECODE_EPILOGUES and rows <= SKINNY_MAX_ROWS and gemm_ops.skinny_qkv_rope_ok(y, b["qkv"], D):
                    qkv = gemm_ops.skinny_qkv_rope(y, b["qkv"], cos, sin, D, H + Hkv).view(rows, 1, -1)
                elif getattr(cache, "rope_attend_ok", None) is not None and cache.rope_attend_ok(rows, H, Hkv, D):
                    # 17-64 rows: q and the new key rotated inside the decode attention kernel
                    qkv = _linear(y, b["qkv"]).view(rows, 1, -1)
                    q, k, v = qkv.split([H * D, Hkv * D, Hkv * D], dim=2)
                    att = cache.attend_rope(l, q.reshape(rows, 1, H, D), k.view(rows, 1, Hkv, D),
                                            v.view(rows, 1, Hkv, D), cos, sin)
                    qkv = None
                else:
                    qkv = rope_ops.apply_rope_qkv(_linear(y, b["qkv"]).view(rows, 1, -1), H, Hkv, D, inv, 0,
                                                  table=(cos, sin))
            else:
                qkv = lin(y, b["qkv"]).view(rows, 1, -1)
            if qkv is not None:
                q, k, v = qkv.split([H * D, Hkv * D, Hkv * D], dim=2)
                att = cache.attend(l, q.reshape(rows, 1, H, D), k.view(rows, 1, Hkv, D), v.view(rows, 1, Hkv, D))
            o = lin(att.view(rows, H * D), b["o"])
            pa, pm, pre = b["post_attn"], b["post_mlp"], b["pre_mlp"]
            h, y = K.rms_residual(x, o, pa.weight if pa is not None else None, pre.weight, b["mode"],
                                  pa.eps if pa is not None else 0.0, pre.eps)
            if gemv and DECODE_EPILOGUES:
                g = torch.empty(rows, b["inter"], device=y.device, dtype=torch.bfloat16)
                K.decode_gemv_pair(y.contiguous(), b["gu"], g, 1, b["kind"])
            else:
                g = _gated(y, b["gu"], b["kind"])
            d = lin(g, b["down"])
            nxt = self.blocks[l + 1]["in_norm"] if l + 1 < len(self.blocks) else self.norm_f
            x, y = K.rms_residual(h, d, pm.weight if pm is not None else None, nxt.weight, b["mode"],
                                  pm.eps if pm is not None else 0.0, nxt.eps)
        return lin(y, self.head.weight)

    def _forward_gemv(self, K, rows: int, x: Tensor, y: Tensor, cache) -> Tensor:
        """Batch 1-4: QKV + RoPE, O, gate|up + activation, down and the lm_head as decode GEMVs (one
        wave per workgroup, one memory round trip); the residual adds + RMSNorms stay the
        rms_residual kernel (as the GEMVs' prologue — every workgroup normalising the rows itself —
        it measured neutral: Gemma-3 1B B=1 1.576 / 1.579 vs 1.571 / 1.571 ms, profiles/decode_r5.md)."""
        for l, b in enumerate(self.blocks):
            a = b["attn"]
            H, Hkv, D = a.num_heads, a.num_kv_heads, a.head_dim
            cos, sin = cache.rope_table((a.rope_theta, D), a._inv_freq(D, x.device), 1)
            qkv = torch.empty(rows, b["qkv"].shape[0], device=x.device, dtype=torch.bfloat16)
            K.decode_gemv_pair(y.contiguous(), b["qkv"], qkv, 2, 0, D, H + Hkv, cos, sin)
            qkv = qkv.view(rows, 1, -1)
            q, k, v = qkv.split([H * D, Hkv * D, Hkv * D], dim=2)
            att = cache.attend(l, q.reshape(rows, 1, H, D), k.view(rows, 1, Hkv, D), v.view(rows, 1, Hkv, D))
            o = torch.empty(rows, b["o"].shape[0], device=x.device, dtype=torch.bfloat16)
            K.decode_gemv(att.reshape(rows, H * D).contiguous(), None, None, None, None, None, None, 0.0, b["o"], None, o, 0)
            pa, pm, pre = b["post_attn"], b["post_mlp"], b["pre_mlp"]
            h, y = K.rms_residual(x, o, pa.weight if pa is not None else None, pre.weight, b["mode"],
                                  pa.eps if pa is not None else 0.0, pre.eps)
            g = torch.empty(rows, b["inter"], device=x.device, dtype=torch.bfloat16)
            K.decode_gemv_pair(y, b["gu"], g, 1, b["kind"])
            d = torch.empty(rows, b["down"].shape[0], device=x.device, dtype=torch.bfloat16)
            K.decode_gemv(g, None, None, None, None, None, None, 0.0, b["down"], None, d, 0)
            nxt = self.blocks[l + 1]["in_norm"] if l + 1 < len(self.blocks) else self.norm_f
            x, y = K.rms_residual(h, d, pm.weight if pm is not None else None, nxt.weight, b["mode"],
                                  pm.eps if pm is not None else 0.0, nxt.eps)
        logits = torch.empty(rows, self.head.weight.shape[0], device=x.device, dtype=torch.bfloat16)
        K.decode_gemv(y, None, None, None, None, None, None, 0.0, self.head.weight, None, logits, 0)
        return logits


# 17-32 rows: decode_linear.hip decode_gemm (16 rows × 16 columns per workgroup, K split over its
# waves) instead of hipBLASLt, whose picks for these skinny shapes ran 36-216 workgroups
# (profiles/notes_r6.md §13); up to this many output columns (the lm_head keeps hipBLASLt).
# PENROZ_DECODE_GEMM=0: hipBLASLt (A/B)
DECODE_GEMM = os.environ.get("PENROZ_DECODE_GEMM", "1") != "0"
DECODE_GEMM_MAX_ROWS, DECODE_GEMM_MAX_N = 32, 32768


def _decode_gemm_ok(x: Tensor, w: Tensor, gated: bool = False) -> bool:
    """decode_gemm takes 17-32 rows (Gemma-3 1B B = 17 / 32: 2.20 -> 1.92 / 2.22 -> 2.07
    ms/step). At 64 rows every mix measured slower than hipBLASLt's step (2.42 ms: 2.60-2.88;
    the narrow O / down projections ran 19 vs 8-12 µs), so those keep hipBLASLt
    (profiles/notes_r6.md §13)."""
    n = w.shape[0] // 2 if gated else w.shape[0]
    return (DECODE_GEMM and SKINNY_MAX_ROWS < x.shape[0] <= DECODE_GEMM_MAX_ROWS and x.is_cuda
            and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.dim() == 2 and x.stride(1) == 1
            and x.stride(0) % 8 == 0 and x.data_ptr() % 16 == 0 and w.is_contiguous() and w.data_ptr() % 16 == 0
            and w.shape[1] == x.shape[1] and x.shape[1] % 32 == 0 and n % 16 == 0 and n <= DECODE_GEMM_MAX_N
            and _ext.available())


def _gated(x: Tensor, gu: Tensor, kind: int) -> Tensor:
    """act(x·Wgᵀ) ⊙ (x·Wuᵀ) from the packed gate|up weight: one fused launch with the activation
    in the GEMM epilogue (the skinny kernel up to SKINNY_MAX_ROWS rows, decode_gemm up to 64), else
    GEMM + packed activation."""
    if DECODE_EPILOGUES and x.shape[0] <= SKINNY_MAX_ROWS and gemm_ops.skinny_ok(x, gu):
        return gemm_ops.skinny_gated(x, gu, kind)
    if DECODE_EPILOGUES and _decode_gemm_ok(x, gu, gated=True):
        out = torch.empty(x.shape[0], gu.shape[0] // 2, device=x.device, dtype=torch.bfloat16)
        _ext.kernels().decode_gemm(x, gu, out, kind)
        return out
    return _ext.kernels().gated_act_packed(_linear(x, gu), kind)


def _linear(x: Tensor, w: Tensor) -> Tensor:
    """x [M, K] · wᵀ without bias: the decode-shaped MFMA kernels up to 64 rows."""
    if x.shape[0] <= SKINNY_MAX_ROWS and gemm_ops.skinny_ok(x, w):
        return gemm_ops.skinny_linear(x, w, None)
    if _decode_gemm_ok(x, w):
        out = torch.empty(x.shape[0], w.shape[0], device=x.device, dtype=torch.bfloat16)
        _ext.kernels().decode_gemm(x, w, out, -1)
        return out
    return torch.mm(x, w.t())


def applicable(model) -> bool:
    if not GRAPH_DECODE or not torch.cuda.is_available():
        return False
    p = next(model.parameters(), None)
    if p is None or not p.is_cuda:
        return False
    attn = model._find_attention_layers()
    if not attn:
        return False
    # the captured step appends K/V and attends inside the decode kernel, so every layer's head_dim
    # must have one (HF Gemma builders set head_dim; GPT-pattern models derive it from C / H)
    gpt_d = None
    if any(a.head_dim is None for a in attn):
        from penroz.models.executor import GPTExecutor
        spec = GPTExecutor.match(model)
        gpt_d = spec.D if spec is not None else None
    for a in attn:
        d = a.head_dim if a.head_dim is not None else gpt_d
        if d is not None and d not in attn_ops.DECODE_HEAD_DIMS:
            return False
        if d is None and a.rope_theta is not None:
            return False
    return True


class GraphDecoder:
    """Static decode state + the captured step graph for ``rows`` sequences."""

    def __init__(self, model, rows: int, capacity: int, temperature: float, top_k: int | None):
        # weak: the model caches its decoders (model.__dict__), so a strong reference would make a
        # cycle that only the cyclic GC frees — and a collection that runs while ANOTHER graph is
        # being captured destroys this one's graph mid-capture (a hard abort)
        self._model = weakref.ref(model)
        self.device = next(model.parameters()).device
        self.attn = model._find_attention_layers()
        self.pos_layers = model._find_position_embeddings()
        cls = StaticTurboKVCache if kvc.TURBO_QUANT_ENABLED else StaticKVCache
        self.cache = cls(len(self.attn), capacity)
        self.cache.init_graph_state(self.device)
        self.rows, self.capacity = rows, capacity
        self.temperature, self.top_k = float(temperature), top_k
        self.idx = torch.zeros(rows, 1, dtype=torch.long, device=self.device)
        self.out = torch.zeros(rows, capacity, dtype=torch.long, device=self.device)
        self.step_t = torch.zeros(1, dtype=torch.long, device=self.device)
        self.seed_t = torch.zeros(1, dtype=torch.long, device=self.device)  # per-run sampling salt
        self.graph: torch.cuda.CUDAGraph | None = None
        gemm_ops.skinny_workspace(self.device)  # zeroed counters exist before any capture
        attn_ops.decode_counters(self.device)  # (the decode attention's split-merge counters too)
        gemm_ops.load_tuned_gemms()  # measured hipBLASLt solutions for the decode-shaped GEMMs too
        self.program = GPTDecodeProgram.build(model) or GemmaDecodeProgram.build(model)

    # ------------------------------------------------------------------ cache attachment
    def attach(self):
        for i, a in enumerate(self.attn):
            a.set_kv_cache(self.cache, i)

    def detach(self):
        for a in self.attn:
            a.set_kv_cache(None, 0)
        for p in self.pos_layers:
            p.position_offset = 0
            p.position_offset_tensor = None

    # ------------------------------------------------------------------ the step
    def _step(self):
        for p in self.pos_layers:
            p.position_offset_tensor = self.cache.pos_t
        self.cache.graph_mode = True
        self.cache.begin_step()
        try:
            if self.program is not None:
                last = self.program.forward(self.idx, self.cache)
            else:
                model = self._model()
                with gemm_ops.decode_gemms(model, max_rows=SKINNY_MAX_ROWS):
                    acts, _ = model(self.idx, skip_softmax=True)
                logits = acts[-1]
                last = logits[:, -1, :] if logits.ndim == 3 else logits
            if _ext.available() and last.is_cuda:
                # one sampler kernel writes the token into the next step's input and the burst
                # buffer (uniforms hashed on the device), one kernel advances the counters
                V = last.shape[-1]
                k = 0 if self.top_k is None or self.top_k >= V else int(self.top_k)
                if FUSED_ADVANCE:  # the sampler's last row advances the counters itself
                    if getattr(self, "_done_t", None) is None:
                        self._done_t = torch.zeros(1, dtype=torch.int32, device=last.device)
                    _ext.kernels().sample_step(last.contiguous(), self.temperature, k, self.seed_t, self.step_t,
                                               self.idx, self.out, self.cache.pos_t, self.cache.len_t, self._done_t)
                else:
                    _ext.kernels().sample_step(last.contiguous(), self.temperature, k, self.seed_t, self.step_t,
                                               self.idx, self.out)
                    _ext.kernels().decode_advance(self.cache.pos_t, self.cache.len_t, self.step_t)
            else:
                nxt = samp_ops.sample(last, self.temperature, self.top_k, device_rng=True)
                torch.add(nxt, 0, out=self.idx)  # a kernel, not a memcpy node
                self.out.index_copy_(1, self.step_t, nxt)
                self.cache.pos_t.add_(1)
                self.cache.len_t.add_(1)
                self.step_t.add_(1)
        finally:
            self.cache.graph_mode = False
            for p in self.pos_layers:
                p.position_offset_tensor = None

    # The sampler kernel hashes each uniform from (seed_t, step_t, row) as
    #   seed + G·(step + 1) + R·(row + 1)  (mod 2^64, csrc/kernels/sampling.hip),
    # with step_t counting from 0 inside a burst. Loading seed_t = run_seed + G·start for a burst
    # that starts at absolute token index ``start`` makes every draw a function of
    # (run seed, absolute index, row) alone: how the tokens are cut into bursts (streaming = bursts
    # of 1, non-streaming = one long burst), and whether the graph was captured in this call or
    # reused, no longer changes them.
    _HASH_STEP = 0x9E3779B97F4A7C15

    def begin(self, run_seed: int):
        """Once per generate call: the seed every burst of this call derives from."""
        self.run_seed = int(run_seed) & (2 ** 64 - 1)

    def _burst_seed(self, start: int) -> int:
        v = (getattr(self, "run_seed", 0) + self._HASH_STEP * int(start)) & (2 ** 64 - 1)
        return v - 2 ** 64 if v >= 2 ** 63 else v

    def _set_state(self, last_tok: Tensor, cache_len: int, start: int = 0):
        self.seed_t.fill_(self._burst_seed(start))
        self.idx.copy_(last_tok)
        self.cache.pos_t.fill_(cache_len)
        self.cache.len_t.fill_(cache_len + 1)
        self.step_t.zero_()

    def _capture(self, last_tok: Tensor, cache_len: int, start: int = 0):
        # warm-up run on a side stream (lazy allocations, kernel loading), then capture. The
        # warm-up really executes a step, so it must start from the true state: it then writes
        # exactly the cache slot the first real step rewrites.
        self._set_state(last_tok, cache_len, start)
        from penroz.models.executor import shared_stream
        side = shared_stream(self.device, "side")  # (no new pool stream per capture)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            self._step()
        torch.cuda.current_stream(self.device).wait_stream(side)
        self._set_state(last_tok, cache_len, start)
        g = torch.cuda.CUDAGraph()
        # no cyclic GC inside the capture: a collection there can free objects that own HIP
        # resources (another decoder's graph, events), which is illegal while capturing
        gc_on = gc.isenabled()
        gc.disable()
        try:
            with torch.cuda.graph(g):
                self._step()
        finally:
            if gc_on:
                gc.enable()
        self.graph = g
        self._set_state(last_tok, cache_len, start)  # capture does not execute; state is as before
        log.info(f"captured decode graph: rows={self.rows} block={self.capacity} "
                 f"temperature={self.temperature} top_k={self.top_k}")

    @torch.inference_mode()
    def run(self, last_tok: Tensor, n_steps: int, start: int = 0) -> Tensor:
        """Decode ``n_steps`` tokens after ``last_tok`` [rows, 1] from the current cache; returns
        the [rows, n_steps] new tokens (device). ``start``: absolute index (within this generate
        call) of the first of them. The cache must have room for n_steps more."""
        cache_len = self.cache.seq_len()
        assert 0 < cache_len and cache_len + n_steps <= self.capacity, (cache_len, n_steps, self.capacity)
        if self.graph is None:
            self._capture(last_tok, cache_len, start)
        else:
            self._set_state(last_tok, cache_len, start)
        for _ in range(n_steps):
            self.graph.replay()
        self.cache._len = [cache_len + n_steps] * self.cache.num_layers
        return self.out[:, :n_steps]


def get_decoder(model, rows: int, block_size: int, temperature: float, top_k: int | None) -> GraphDecoder | None:
    """Cached per model and (rows, block size, sampling settings, weights identity); None when the
    model does not qualify (CPU, no attention, RoPE head_dim without a decode kernel) or ``PENROZ_GRAPH_DECODE=0``."""
    if not applicable(model):
        return None
    p = next(model.parameters())
    # weights identity AND version: in-place updates (training) re-capture, so nothing captured
    # (e.g. LayerNorm's cached fp32 weight copies for bf16 models) can go stale
    version = sum(q._version for q in model.parameters())
    key = (rows, block_size, float(temperature), top_k if temperature else None, kvc.TURBO_QUANT_ENABLED,
           p.data_ptr(), p.dtype, version)
    cache = model.__dict__.setdefault("_graph_decoders", {})
    dec = cache.get(key)
    if dec is None:
        while len(cache) >= 2:  # bounded: each holds a KV cache and a graph memory pool
            cache.pop(next(iter(cache)))
        dec = GraphDecoder(model, rows, block_size, temperature, top_k)
        cache[key] = dec
    return dec
