"""Next-token selection (greedy / temperature / top-k) and int8 KV quantisation.

Reference semantics (``neural_net_model.py:393-405``): temperature 0 → argmax of the last
position; ``top_k`` → softmax over the top-k logits / T then multinomial; otherwise softmax
over logits / T then multinomial.  (The reference's top-k runs over every position and its
non-softmax-model path crashes — bugs 2 and 5 of SURVEY §7.4 — both fixed here.)

GPU: ``csrc/kernels/sampling.hip`` — one workgroup per row: temperature scale, top-k by a
radix-select threshold in LDS, softmax and inverse-CDF draw from one uniform per row, all in
a single pass over the row (no sort, no host round trip).
``kv_quantize``: per-token absmax/127 int8 (``kv_cache.py:114-125``), written straight into
the preallocated cache slot.
"""
from __future__ import annotations

import torch
from torch import Tensor

from penroz.ops._ext import use_kernels, kernels


def reference_sample(logits: Tensor, temperature: float, top_k: int | None, uniform: Tensor) -> Tensor:
    """logits [B, V] -> token ids [B, 1] using the given uniforms [B] (inverse-CDF draw)."""
    lf = logits.float()
    if temperature == 0.0:
        return lf.argmax(dim=-1, keepdim=True)
    lf = lf / temperature
    if top_k is not None and top_k < lf.shape[-1]:
        vals, idx = lf.topk(top_k, dim=-1)
    else:
        vals, idx = lf.sort(dim=-1, descending=True)
    probs = torch.softmax(vals, dim=-1)
    cdf = probs.cumsum(-1)
    choice = torch.searchsorted(cdf, (uniform.float() * cdf[:, -1]).unsqueeze(-1).contiguous())
    choice = choice.clamp(max=vals.shape[-1] - 1)
    return idx.gather(1, choice)


def sample(logits: Tensor, temperature: float, top_k: int | None, generator: torch.Generator | None = None,
           device_rng: bool = False) -> Tensor:
    """logits [B, V] -> [B, 1] int64 next-token ids. ``device_rng``: draw the uniforms on the
    device (required inside a captured HIP graph; the host-drawn default matches CPU runs)."""
    B = logits.shape[0]
    if temperature == 0.0:
        if use_kernels(logits):
            return kernels().sample_tokens(logits.contiguous(), None, 0.0, 0)
        return logits.argmax(dim=-1, keepdim=True)
    if device_rng:
        uniform = torch.rand(B, device=logits.device)
    else:
        uniform = torch.rand(B, generator=generator, device="cpu").to(logits.device)
    if use_kernels(logits):
        k = 0 if top_k is None or top_k >= logits.shape[-1] else int(top_k)
        return kernels().sample_tokens(logits.contiguous(), uniform, float(temperature), k)
    return reference_sample(logits, temperature, top_k, uniform)


def reference_quantize(x: Tensor) -> tuple[Tensor, Tensor]:
    """x [..., D] -> (int8 [..., D], scale [..., 1]) per-token absmax / 127."""
    abs_max = x.abs().amax(dim=-1, keepdim=True)
    scale = abs_max / 127.0
    scale = torch.where(scale == 0, torch.ones_like(scale), scale)
    q = (x / scale).round().clamp(-128, 127).to(torch.int8)
    return q, scale


def kv_quantize_into(x: Tensor, q_out: Tensor, s_out: Tensor, pos: int) -> None:
    """x [B, T, Hkv, D] -> q_out[:, :, pos:pos+T] (int8 [B,Hkv,cap,D]), s_out[:, :, pos:pos+T] (f32)."""
    if use_kernels(x):
        kernels().kv_quantize(x.contiguous(), q_out, s_out, int(pos))
        return
    T = x.shape[1]
    q, s = reference_quantize(x.float().transpose(1, 2))
    q_out[:, :, pos:pos + T] = q
    s_out[:, :, pos:pos + T] = s.squeeze(-1)


def kv_store_into(x: Tensor, out: Tensor, pos: int) -> None:
    """x [B, T, Hkv, D] -> out[:, :, pos:pos+T] (layout [B, Hkv, cap, D])."""
    out[:, :, pos:pos + x.shape[1]] = x.transpose(1, 2).to(out.dtype)
