"""Causal self-attention over a fused QKV tensor, and KV-cache (decode) attention.

GPU: hand-written CDNA4 flash attention — ``csrc/kernels/flash_attn.hip`` (head_dim 64, GPT-2)
and ``csrc/kernels/flash_attn_gen.hip`` (head_dim 128 / 256 / 512, Gemma; the same algebra over
64-column LDS panels, D = 512 split over column parts):
  * forward reads Q/K/V straight out of the fused ``[B, T, (H + 2·Hkv)·D]`` projection (no
    split/transpose copies), keeps Q in registers, stages K/V tiles through XOR-swizzled LDS,
    computes Sᵀ = K·Qᵀ with ``v_mfma_f32_32x32x16_bf16`` so each lane owns one query row's
    scores (softmax in registers, one cross-half exchange), feeds P straight from the
    accumulators into Oᵀ = Vᵀ·Pᵀ (V read with ``ds_read_b64_tr_b16``), and writes O already
    head-merged ``[B, T, H·D]`` plus the row log-sum-exp;
  * backward keeps each wave's 32 keys (K, V, dKᵀ, dVᵀ) in registers while sweeping the query
    slices of every query head of its KV group; a second, forward-shaped kernel keeps 32 query
    rows (Q, dO, dQᵀ) in registers while sweeping the key tiles — deterministic, no atomics.
  GQA is handled by index math (kv head = q head // group) — K/V are never expanded.
  Dropout (``attn_pdrop``) uses a counter-based hash RNG regenerated in the backward pass.
CPU: ``torch.nn.functional.scaled_dot_product_attention`` (math) with GQA expansion.

Replaces the reference's SDPA call (``neural_net_layers.py:59-95``).
"""
from __future__ import annotations

import math
import os

import torch
from torch import Tensor
import torch.nn.functional as F

from penroz.ops._ext import use_kernels, kernels

# head dims with a native kernel: prefill / training flash attention (flash_attn.hip: 64;
# flash_attn_gen.hip: 128, 256 and Gemma-4's global_head_dim 512 — whose O accumulator alone (32
# query rows × 512 fp32 per wave) would fill a wave's whole register file, so the 512 kernels split
# D over column parts: grid z) and decode attention (csrc/kernels/decode_attn.hip: also 32).
# Prefill / training at any other head dim <= 512 runs the next wider kernel on zero-padded heads
# (see _padded_dim); only heads wider than 512 fall back to torch SDPA.
SUPPORTED_HEAD_DIMS = (64, 128, 256, 512)
DECODE_HEAD_DIMS = (32, 64, 128, 256, 512)


def _padded_dim(D: int) -> int | None:
    """The native flash-attention width that serves head_dim ``D`` (None: no native kernel)."""
    for n in SUPPORTED_HEAD_DIMS:
        if D <= n:
            return n
    return None


def reference_causal_attention_qkv(qkv: Tensor, H: int, Hkv: int, D: int, dropout_p: float = 0.0) -> Tensor:
    B, T, _ = qkv.shape
    q, k, v = qkv.split([H * D, Hkv * D, Hkv * D], dim=2)
    q = q.reshape(B, T, H, D).transpose(1, 2)
    k = k.reshape(B, T, Hkv, D).transpose(1, 2)
    v = v.reshape(B, T, Hkv, D).transpose(1, 2)
    if Hkv < H:
        rep = H // Hkv
        k = k.repeat_interleave(rep, dim=1)
        v = v.repeat_interleave(rep, dim=1)
    o = F.scaled_dot_product_attention(q, k, v, dropout_p=dropout_p, is_causal=True)
    return o.transpose(1, 2).reshape(B, T, H * D)


def reference_attention_lse(qkv: Tensor, H: int, Hkv: int, D: int):
    """fp32 math reference returning (out [B,T,H*D], lse [B,H,T]) for kernel parity tests."""
    B, T, _ = qkv.shape
    q, k, v = qkv.float().split([H * D, Hkv * D, Hkv * D], dim=2)
    q = q.reshape(B, T, H, D).transpose(1, 2)
    k = k.reshape(B, T, Hkv, D).transpose(1, 2).repeat_interleave(H // Hkv, dim=1)
    v = v.reshape(B, T, Hkv, D).transpose(1, 2).repeat_interleave(H // Hkv, dim=1)
    s = (q @ k.transpose(-1, -2)) / math.sqrt(D)
    mask = torch.ones(T, T, dtype=torch.bool, device=qkv.device).triu(1)
    s = s.masked_fill(mask, float("-inf"))
    lse = torch.logsumexp(s, dim=-1)
    p = torch.softmax(s, dim=-1)
    o = p @ v
    return o.transpose(1, 2).reshape(B, T, H * D), lse


def flash_fwd(qkv: Tensor, H: int, Hkv: int, D: int, dropout_p: float = 0.0, seed: int = 0,
              out: Tensor | None = None, lse: Tensor | None = None):
    """bf16 qkv [B,T,(H+2Hkv)D] -> (out bf16 [B,T,H*D], lse f32 [B,H,T])."""
    B, T, _ = qkv.shape
    out = torch.empty(B, T, H * D, dtype=torch.bfloat16, device=qkv.device) if out is None else out
    lse = torch.empty(B, H, T, dtype=torch.float32, device=qkv.device) if lse is None else lse
    fn = kernels().flash_attn_fwd if D == 64 else kernels().flash_attn_gen_fwd
    fn(qkv, out, lse, H, Hkv, D, 1.0 / math.sqrt(D), float(dropout_p), int(seed))
    return out, lse


def flash_bwd(dout: Tensor, qkv: Tensor, out: Tensor, lse: Tensor, H: int, Hkv: int, D: int,
              dropout_p: float = 0.0, seed: int = 0, dqkv: Tensor | None = None,
              dbias: Tensor | None = None) -> Tensor:
    """-> dqkv bf16 [B,T,(H+2Hkv)D] (written into ``dqkv`` when given).

    ``dbias`` (fp32 [(H+2Hkv)D]): += the column sums of dqkv, i.e. the fused QKV projection's bias
    gradient. At head_dim 64 the dK/dV and dQ kernels produce them in their epilogues (no second
    pass over the 2304-wide gradient); other head dims run the column-sum kernel afterwards."""
    dqkv = torch.empty_like(qkv) if dqkv is None else dqkv
    scale = 1.0 / math.sqrt(D)
    if D == 64:
        kernels().flash_attn_bwd(dout, qkv, out, lse, dqkv, H, Hkv, D, scale, float(dropout_p), int(seed), dbias)
    else:
        kernels().flash_attn_gen_bwd(dout, qkv, out, lse, dqkv, H, Hkv, D, scale, float(dropout_p), int(seed))
        if dbias is not None:
            kernels().colsum(dqkv.view(-1, dqkv.shape[-1]), dbias)
    return dqkv


def new_seed() -> int:
    return int(torch.randint(0, 2**31 - 1, (1,)).item())


class _FlashAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, H, Hkv, D, dropout_p):
        in_dtype = qkv.dtype
        x = qkv.to(torch.bfloat16).contiguous()
        seed = new_seed() if dropout_p > 0 else 0
        out, lse = flash_fwd(x, H, Hkv, D, dropout_p, seed)
        ctx.save_for_backward(x, out, lse)
        ctx.meta = (H, Hkv, D, dropout_p, seed, in_dtype)
        return out if in_dtype == torch.bfloat16 else out.to(in_dtype)

    @staticmethod
    def backward(ctx, dout):
        x, out, lse = ctx.saved_tensors
        H, Hkv, D, p, seed, in_dtype = ctx.meta
        dqkv = flash_bwd(dout.to(torch.bfloat16).contiguous(), x, out, lse, H, Hkv, D, p, seed)
        return dqkv.to(in_dtype), None, None, None, None


class _PaddedFlashAttnFn(torch.autograd.Function):
    """Head dim D without its own kernel: every head zero-padded to the kernel width Dp. The
    scores are unchanged (the padded columns contribute 0 to Q·Kᵀ; the scale stays 1/√D), the
    output's padded columns are P·0 = 0, and in the backward dQ, dK, dV vanish on them (dO is
    padded with zeros), so slicing them off is exact."""

    @staticmethod
    def forward(ctx, qkv, H, Hkv, D, Dp, dropout_p):
        in_dtype = qkv.dtype
        B, T, _ = qkv.shape
        x = torch.zeros(B, T, H + 2 * Hkv, Dp, dtype=torch.bfloat16, device=qkv.device)
        x[..., :D] = qkv.view(B, T, H + 2 * Hkv, D)
        x = x.view(B, T, -1)
        seed = new_seed() if dropout_p > 0 else 0
        out = torch.empty(B, T, H * Dp, dtype=torch.bfloat16, device=qkv.device)
        lse = torch.empty(B, H, T, dtype=torch.float32, device=qkv.device)
        fn = kernels().flash_attn_fwd if Dp == 64 else kernels().flash_attn_gen_fwd
        fn(x, out, lse, H, Hkv, Dp, 1.0 / math.sqrt(D), float(dropout_p), int(seed))
        ctx.save_for_backward(x, out, lse)
        ctx.meta = (H, Hkv, D, Dp, dropout_p, seed, in_dtype)
        o = out.view(B, T, H, Dp)[..., :D].reshape(B, T, H * D)
        return o.to(in_dtype)

    @staticmethod
    def backward(ctx, dout):
        x, out, lse = ctx.saved_tensors
        H, Hkv, D, Dp, p, seed, in_dtype = ctx.meta
        B, T, _ = x.shape
        dp = torch.zeros(B, T, H, Dp, dtype=torch.bfloat16, device=x.device)
        dp[..., :D] = dout.view(B, T, H, D)
        dqkv = torch.empty_like(x)
        scale = 1.0 / math.sqrt(D)
        dpv = dp.view(B, T, H * Dp)
        if Dp == 64:
            kernels().flash_attn_bwd(dpv, x, out, lse, dqkv, H, Hkv, Dp, scale, float(p), int(seed), None)
        else:
            kernels().flash_attn_gen_bwd(dpv, x, out, lse, dqkv, H, Hkv, Dp, scale, float(p), int(seed))
        g = dqkv.view(B, T, H + 2 * Hkv, Dp)[..., :D].reshape(B, T, (H + 2 * Hkv) * D)
        return g.to(in_dtype), None, None, None, None, None


def causal_attention_qkv(qkv: Tensor, H: int, Hkv: int, D: int, dropout_p: float = 0.0) -> Tensor:
    """Causal attention of a fused-QKV tensor ``[B, T, (H + 2·Hkv)·D]`` -> ``[B, T, H·D]``."""
    if use_kernels(qkv):
        if D in SUPPORTED_HEAD_DIMS:
            return _FlashAttnFn.apply(qkv, H, Hkv, D, dropout_p)
        Dp = _padded_dim(D)
        if Dp is not None and D % 8 == 0:
            return _PaddedFlashAttnFn.apply(qkv, H, Hkv, D, Dp, dropout_p)
    return reference_causal_attention_qkv(qkv, H, Hkv, D, dropout_p)


# --------------------------------------------------------------------------- decode / cache
def reference_cache_attention(q: Tensor, k: Tensor, v: Tensor, q_offset: int) -> Tensor:
    """q [B,Tq,H,D], k/v [B,Hkv,S,D] (S = q_offset + Tq); query i sits at q_offset + i."""
    B, Tq, H, D = q.shape
    Hkv, S = k.shape[1], k.shape[2]
    qh = q.transpose(1, 2).float()
    kh = k.float().repeat_interleave(H // Hkv, dim=1)
    vh = v.float().repeat_interleave(H // Hkv, dim=1)
    s = (qh @ kh.transpose(-1, -2)) / math.sqrt(D)
    qpos = torch.arange(q_offset, q_offset + Tq, device=q.device).unsqueeze(1)
    kpos = torch.arange(S, device=q.device).unsqueeze(0)
    s = s.masked_fill(kpos > qpos, float("-inf"))
    o = torch.softmax(s, dim=-1) @ vh
    return o.transpose(1, 2).reshape(B, Tq, H * D).to(q.dtype)


# arrival counters of the decode kernel's in-launch split merge (csrc/kernels/decode_attn.hip):
# zeroed once per device, outside any graph capture (every launch leaves them zero again), so a
# captured step reuses them. PENROZ_DECODE_MERGE=0: no counters — the separate combine launch.
DECODE_COUNTERS = 1 << 13
_decode_counters: dict = {}


def decode_counters(device: torch.device) -> Tensor | None:
    """The device's split-merge counters, created on first use — unless that use is inside a
    stream capture (the zeroing would become part of the graph): then None, the combine launch."""
    if os.environ.get("PENROZ_DECODE_MERGE", "1") == "0" or device.type != "cuda":
        return None
    idx = device.index if device.index is not None else torch.cuda.current_device()
    cnt = _decode_counters.get(idx)
    if cnt is None and not torch.cuda.is_current_stream_capturing():
        cnt = _decode_counters[idx] = torch.zeros(DECODE_COUNTERS, dtype=torch.int32, device=torch.device("cuda", idx))
    return cnt


def decode_rope_fusable(B: int, H: int, Hkv: int, D: int, cap: int, cache_dtype: torch.dtype) -> bool:
    """The decode kernel can rotate q and the appended key itself (``decode_attention(rope=)``):
    the one-workgroup-per-(batch, KV head) kernel over a bf16 cache of ``cap`` slots."""
    return (cache_dtype == torch.bfloat16 and D % 16 == 0 and D <= 256
            and kernels().decode_small_applies(B, 1, H, Hkv, D, cap))


def decode_attention(q: Tensor, k_cache: Tensor, v_cache: Tensor, seq_len: int,
                     k_scale: Tensor | None = None, v_scale: Tensor | None = None,
                     seq_len_dev: Tensor | None = None, k_new: Tensor | None = None,
                     v_new: Tensor | None = None, rope: tuple[Tensor, Tensor] | None = None) -> Tensor:
    """Attention of ``q [B, Tq, H, D]`` against the first ``seq_len`` cache slots.

    Cache layout ``[B, Hkv, cap, D]`` (bf16/fp16/fp32, or int8 with per-token fp32 scales
    ``[B, Hkv, cap]`` — TurboQuant; dequantisation fused into the kernel).
    GPU: split-K decode kernel (``csrc/kernels/decode_attn.hip``). ``seq_len_dev`` (device int64
    [1], GPU only): the kernel reads the cache length at run time (``seq_len`` is then the
    capacity bound) — the form a captured HIP graph replays at every position.
    ``k_new`` / ``v_new`` ([B, 1, Hkv, D], GPU kernel only): this step's K / V, appended at slot
    ``seq_len - 1`` by the attention kernel itself (int8 caches: quantised as ``kv_quantize_into``).
    ``rope`` (fp32 cos / sin [D/2] of this step's single position; with ``k_new`` / ``v_new``): q and
    the new key arrive unrotated and the kernel applies rotate-half RoPE itself — only where
    ``decode_rope_fusable`` says so.
    """
    Tq = q.shape[1]
    if rope is not None and (k_new is None or not use_kernels(q)):
        raise ValueError("in-kernel RoPE needs the decode kernel's fused append")
    if use_kernels(q) and q.shape[-1] in DECODE_HEAD_DIMS:
        # a view into the fused QKV rows is read in place (packed heads, uniform row stride)
        if not (q.stride(3) == 1 and q.stride(2) == q.shape[3]
                and (Tq == 1 or q.stride(0) == q.shape[1] * q.stride(1))):
            q = q.contiguous()
        return kernels().decode_attn(q, k_cache, v_cache, k_scale, v_scale, int(seq_len),
                                     int(seq_len - Tq), 1.0 / math.sqrt(q.shape[-1]), seq_len_dev, k_new, v_new,
                                     decode_counters(q.device), *(rope if rope is not None else (None, None)))
    if k_new is not None:
        raise ValueError("fused KV append needs the decode kernel")
    if seq_len_dev is not None:
        seq_len = int(seq_len_dev.item())
    k = k_cache[:, :, :seq_len]
    v = v_cache[:, :, :seq_len]
    if k_scale is not None:
        k = k.float() * k_scale[:, :, :seq_len, None]
        v = v.float() * v_scale[:, :, :seq_len, None]
    return reference_cache_attention(q, k, v, seq_len - Tq)
