"""LayerNorm / fused residual-add LayerNorm / RMSNorm.

GPU: HIP kernels in ``csrc/kernels/layernorm.hip`` and ``rmsnorm.hip`` — one 64-lane wave
per row, the row held in registers (float4 loads), fp32 statistics, bf16/fp32 output; the
backward fuses dγ/dβ partial sums, the residual-gradient accumulation and the preceding
linear's bias gradient (column sum) into one pass.
CPU: the torch reference math (``reference_*``) that the GPU parity tests compare against.

Replaces ATen ``layer_norm`` under autocast (fp32 stats) used by the reference's
``layernorm`` algo (``mappers.py:31``) and the reference RMSNorm (``neural_net_layers.py:144-155``).
"""
from __future__ import annotations

import torch
from torch import Tensor

from penroz.ops._ext import use_kernels, kernels


# --------------------------------------------------------------------------- references
def reference_layer_norm(x: Tensor, w: Tensor, b: Tensor, eps: float):
    xf = x.float()
    mean = xf.mean(-1, keepdim=True)
    var = xf.var(-1, unbiased=False, keepdim=True)
    rstd = torch.rsqrt(var + eps)
    y = (xf - mean) * rstd * w.float() + (b.float() if b is not None else 0.0)
    return y, mean.squeeze(-1), rstd.squeeze(-1)


def reference_layer_norm_bwd(dy: Tensor, x: Tensor, mean: Tensor, rstd: Tensor, w: Tensor):
    xf, dyf = x.float(), dy.float()
    xhat = (xf - mean.unsqueeze(-1)) * rstd.unsqueeze(-1)
    wdy = dyf * w.float()
    c1 = wdy.mean(-1, keepdim=True)
    c2 = (wdy * xhat).mean(-1, keepdim=True)
    dx = (wdy - c1 - xhat * c2) * rstd.unsqueeze(-1)
    dw = (dyf * xhat).reshape(-1, x.shape[-1]).sum(0)
    db = dyf.reshape(-1, x.shape[-1]).sum(0)
    return dx, dw, db


def reference_rms_norm(x: Tensor, w: Tensor, eps: float):
    dtype = x.dtype
    xf = x.float()
    norm = xf.pow(2).mean(-1, keepdim=True).add(eps).rsqrt()
    return (xf * norm).to(dtype) * w


# --------------------------------------------------------------------------- GPU entry points
def ln_fwd(x2d: Tensor, w: Tensor, b: Tensor, eps: float, out_dtype=torch.bfloat16,
           y: Tensor | None = None, mean: Tensor | None = None, rstd: Tensor | None = None):
    """[N, C] -> (y [N, C], mean [N] f32, rstd [N] f32); outputs written into given buffers."""
    N, C = x2d.shape
    y = torch.empty(N, C, dtype=out_dtype, device=x2d.device) if y is None else y
    mean = torch.empty(N, dtype=torch.float32, device=x2d.device) if mean is None else mean
    rstd = torch.empty(N, dtype=torch.float32, device=x2d.device) if rstd is None else rstd
    kernels().layernorm_fwd(x2d, w, b, float(eps), y, mean, rstd)
    return y, mean, rstd


def add_ln_fwd(resid_in: Tensor, delta: Tensor, resid_out: Tensor, w: Tensor, b: Tensor, eps: float,
               y: Tensor | None = None, mean: Tensor | None = None, rstd: Tensor | None = None,
               delta_bias: Tensor | None = None, dropout_p: float = 0.0, dropout_seed: int = 0):
    """``resid_out = resid_in + drop(delta (+ delta_bias))`` (fp32 stream, bf16 delta, fp32 bias
    [C]) and LayerNorm(resid_out) -> bf16 y. ``drop`` = inverted dropout with a mask hashed from
    (``dropout_seed``, element index); ``ln_bwd`` regenerates it."""
    N, C = resid_in.shape
    y = torch.empty(N, C, dtype=torch.bfloat16, device=resid_in.device) if y is None else y
    mean = torch.empty(N, dtype=torch.float32, device=resid_in.device) if mean is None else mean
    rstd = torch.empty(N, dtype=torch.float32, device=resid_in.device) if rstd is None else rstd
    kernels().add_layernorm_fwd(resid_in, delta, resid_out, w, b, float(eps), y, mean, rstd, delta_bias,
                                float(dropout_p), int(dropout_seed))
    return y, mean, rstd


def ln_bwd(dy: Tensor, x: Tensor, mean: Tensor, rstd: Tensor, w: Tensor, dresid: Tensor,
           accumulate: bool, dresid_bf16: Tensor | None, dw: Tensor, db: Tensor,
           dbias_prev: Tensor | None, dropout_p: float = 0.0, dropout_seed: int = 0):
    """Fused LayerNorm backward.

    ``dresid (+)= dx``; optionally writes ``dresid_bf16`` (the next dgrad GEMM's operand);
    ``dw += Σ dy·x̂``, ``db += Σ dy``; optionally ``dbias_prev += Σ_rows dresid`` (bias grad of
    the linear that produced the residual branch feeding this norm). With ``dropout_p`` (the
    branch's dropout in the forward's ``add_ln_fwd``) the bf16 copy and the bias sum carry the
    regenerated mask; the fp32 residual gradient does not.
    """
    kernels().layernorm_bwd(dy, x, mean, rstd, w, dresid, accumulate, dresid_bf16, dw, db, dbias_prev,
                            float(dropout_p), int(dropout_seed))


# --------------------------------------------------------------------------- autograd front-ends
class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        out_dtype = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
        # autocast keeps layer_norm in fp32 (reference semantics): output fp32 under autocast
        if torch.is_autocast_enabled("cuda"):
            out_dtype = torch.float32
        y, mean, rstd = ln_fwd(x2, w.float(), b.float(), eps, out_dtype)
        ctx.save_for_backward(x2, w, mean, rstd)
        ctx.has_b = b is not None
        ctx.shape = shape
        return y.view(shape)

    @staticmethod
    def backward(ctx, dy):
        x2, w, mean, rstd = ctx.saved_tensors
        dy2 = dy.reshape(-1, x2.shape[-1]).contiguous()
        dx = torch.empty(x2.shape, dtype=torch.float32, device=x2.device)
        dw = torch.zeros(w.shape, dtype=torch.float32, device=w.device)
        db = torch.zeros(w.shape, dtype=torch.float32, device=w.device)
        ln_bwd(dy2, x2, mean, rstd, w.float(), dx, False, None, dw, db, None)
        return (dx.to(x2.dtype).view(ctx.shape), dw.to(w.dtype), db.to(w.dtype) if ctx.has_b else None, None)


def layer_norm(x: Tensor, w: Tensor, b: Tensor, eps: float) -> Tensor:
    if use_kernels(x) and x.shape[-1] % 4 == 0 and b is not None:
        return _LayerNormFn.apply(x, w, b, eps)
    return torch.nn.functional.layer_norm(x, (x.shape[-1],), w, b, eps)


class _RMSNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, eps):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        y, rstd = kernels().rmsnorm_fwd(x2, w, eps)
        ctx.save_for_backward(x2, w, rstd)
        ctx.shape = shape
        return y.view(shape)

    @staticmethod
    def backward(ctx, dy):
        x2, w, rstd = ctx.saved_tensors
        dx, dw = kernels().rmsnorm_bwd(dy.reshape(-1, x2.shape[-1]).contiguous(), x2, w, rstd)
        return dx.view(ctx.shape), dw.to(w.dtype), None


def rms_norm(x: Tensor, w: Tensor, eps: float) -> Tensor:
    """``(x_f32 * rsqrt(mean(x²) + eps)).to(x.dtype) * w`` — reference semantics. Autocast does not
    change that expression (the statistics are fp32 already; the product follows type promotion),
    so the HIP kernel (fp32 statistics, output dtype = promote(x, w)) serves both modes."""
    if use_kernels(x) and x.shape[-1] % 4 == 0 and x.shape[-1] <= RMS_BWD_MAX_C:
        return _RMSNormFn.apply(x, w, eps)
    return reference_rms_norm(x, w, eps)


RMS_BWD_MAX_C = 10240  # the HIP backward keeps 4 waves x C fp32 dγ partials in LDS (rmsnorm.hip)
