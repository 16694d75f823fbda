"""GELU (erf / tanh) and the gated-MLP activation ``act(gate) * up``.

GPU: ``csrc/kernels/elementwise.hip`` — 16-byte vectorised bf16/fp32 grid-stride kernels
(memory-bound; one read + one write per element).  The fused GPT executor calls the raw
``gelu_fwd``/``gelu_bwd`` entry points directly.
Reference semantics: ``{"gelu": {}}`` is the erf GELU, ``{"gelu": {"approximate": "tanh"}}``
is HF's ``gelu_new`` (``mappers.py:139``); GatedMLP's silu / gelu_pytorch_tanh / gelu
(``neural_net_layers.py:158-174``).
"""
from __future__ import annotations

import torch
from torch import Tensor
import torch.nn.functional as F

from penroz.ops._ext import use_kernels, kernels

_APPROX = {"none": 0, "tanh": 1}
_GATED = {"gelu": 0, "gelu_tanh": 1, "silu": 2}


def reference_gelu(x: Tensor, approximate: str = "none") -> Tensor:
    return F.gelu(x, approximate=approximate)


def reference_gelu_bwd(dy: Tensor, x: Tensor, approximate: str = "none") -> Tensor:
    xf = x.float().detach().requires_grad_(True)
    with torch.enable_grad():
        y = F.gelu(xf, approximate=approximate)
        (g,) = torch.autograd.grad(y, xf, dy.float())
    return g


def reference_gated_act(gate: Tensor, up: Tensor, kind: str) -> Tensor:
    if kind == "silu":
        a = F.silu(gate)
    elif kind == "gelu_tanh":
        a = F.gelu(gate, approximate="tanh")
    else:
        a = F.gelu(gate)
    return a * up


def gelu_fwd(x: Tensor, approximate: str = "none", out: Tensor | None = None) -> Tensor:
    out = torch.empty_like(x) if out is None else out
    kernels().gelu_fwd(x, _APPROX[approximate], out)
    return out


def gelu_bwd(dy: Tensor, x: Tensor, approximate: str = "none", dbias: Tensor | None = None,
             out: Tensor | None = None) -> Tensor:
    """dx = dy * GELU'(x) (``out`` may alias ``dy``); if ``dbias`` (fp32 [cols], 2-D input) is
    given, the column sums of dx are accumulated into it in the same pass."""
    out = torch.empty_like(x) if out is None else out
    kernels().gelu_bwd(dy, x, _APPROX[approximate], dbias, out)
    return out


class _GeluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, approximate):
        xc = x.contiguous()
        ctx.save_for_backward(xc)
        ctx.approximate = approximate
        return gelu_fwd(xc, approximate)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        return gelu_bwd(dy.contiguous().to(x.dtype), x, ctx.approximate).to(x.dtype), None


def gelu(x: Tensor, approximate: str = "none") -> Tensor:
    if use_kernels(x) and x.dtype in (torch.bfloat16, torch.float32, torch.float16):
        return _GeluFn.apply(x, approximate)
    return reference_gelu(x, approximate)


class _GatedActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gate, up, kind):
        g, u = gate.contiguous(), up.contiguous()
        ctx.save_for_backward(g, u)
        ctx.kind = kind
        return kernels().gated_act_fwd(g, u, _GATED[kind])

    @staticmethod
    def backward(ctx, dy):
        g, u = ctx.saved_tensors
        dg, du = kernels().gated_act_bwd(dy.contiguous().to(g.dtype), g, u, _GATED[ctx.kind])
        return dg, du, None


def gated_act(gate: Tensor, up: Tensor, kind: str) -> Tensor:
    if use_kernels(gate) and gate.dtype == up.dtype and gate.shape == up.shape:
        return _GatedActFn.apply(gate, up, kind)
    return reference_gated_act(gate, up, kind)
