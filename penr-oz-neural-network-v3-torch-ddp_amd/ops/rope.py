"""Rotary position embedding applied to the Q and K parts of a fused QKV tensor.

Reference math (``neural_net_layers.py:33-57``): ``x*cos + rotate_half(x)*sin`` with
``freqs = outer(t, inv_freq)`` duplicated over both halves.  GPU: ``csrc/kernels/rope.hip``
reads a cos/sin table ``[T, D/2]`` (computed once per call on the device — no per-element
trig in the kernel) and rotates Q and K in one pass; V is copied through.  The backward is
the same kernel with the rotation inverted.
"""
from __future__ import annotations

import torch
from torch import Tensor

from penroz.ops._ext import use_kernels, kernels


def rope_table(inv_freq: Tensor, offset: int, T: int, device, offset_dev: Tensor | None = None) -> tuple[Tensor, Tensor]:
    """cos / sin [T, D/2] for positions offset..offset+T-1; ``offset_dev`` (device int64 [1])
    supplies the offset at run time instead (graph-replayed decode)."""
    if offset_dev is not None:
        t = offset_dev.to(torch.float32) + torch.arange(T, device=device, dtype=torch.float32)
    else:
        t = torch.arange(offset, offset + T, device=device, dtype=torch.float32)
    freqs = torch.outer(t, inv_freq.to(device=device, dtype=torch.float32))
    return freqs.cos().contiguous(), freqs.sin().contiguous()


def _rotate_half(x: Tensor) -> Tensor:
    x1, x2 = x[..., : x.shape[-1] // 2], x[..., x.shape[-1] // 2:]
    return torch.cat((-x2, x1), dim=-1)


def reference_apply_rope_qkv(qkv: Tensor, H: int, Hkv: int, D: int, inv_freq: Tensor, offset: int) -> Tensor:
    B, T, _ = qkv.shape
    q, k, v = qkv.split([H * D, Hkv * D, Hkv * D], dim=2)
    cos, sin = rope_table(inv_freq, offset, T, qkv.device)
    cos = torch.cat([cos, cos], -1).to(qkv.dtype)[None, :, None, :]
    sin = torch.cat([sin, sin], -1).to(qkv.dtype)[None, :, None, :]
    q = q.reshape(B, T, H, D)
    k = k.reshape(B, T, Hkv, D)
    q = q * cos + _rotate_half(q) * sin
    k = k * cos + _rotate_half(k) * sin
    return torch.cat([q.reshape(B, T, H * D), k.reshape(B, T, Hkv * D), v], dim=2)


class _RopeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, H, Hkv, D, cos, sin):
        ctx.save_for_backward(cos, sin)
        ctx.meta = (H, Hkv, D)
        return kernels().rope_qkv(qkv.contiguous(), cos, sin, H, Hkv, D, False)

    @staticmethod
    def backward(ctx, dy):
        cos, sin = ctx.saved_tensors
        H, Hkv, D = ctx.meta
        return kernels().rope_qkv(dy.contiguous(), cos, sin, H, Hkv, D, True), None, None, None, None, None


def apply_rope_qkv(qkv: Tensor, H: int, Hkv: int, D: int, inv_freq: Tensor, offset: int,
                   table: tuple[Tensor, Tensor] | None = None) -> Tensor:
    """``table``: a precomputed (cos, sin) for these positions (graph-replayed decode shares one
    device-offset table between the layers of a step)."""
    if use_kernels(qkv) and D % 2 == 0:
        cos, sin = table if table is not None else rope_table(inv_freq, offset, qkv.shape[1], qkv.device)
        return _RopeFn.apply(qkv, H, Hkv, D, cos, sin)
    if table is not None:
        raise ValueError("a precomputed RoPE table needs the HIP kernel")
    return reference_apply_rope_qkv(qkv, H, Hkv, D, inv_freq, offset)
