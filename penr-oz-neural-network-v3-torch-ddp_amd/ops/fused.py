"""Fused training-step kernels used by the GPT executor and the runtime.

* ``embedding_fwd/bwd`` — token + learned position gather/add (fp32 residual stream out);
  backward: dwte by a sort-free deterministic per-token-row scatter (atomics on fp32 rows,
  256-B contiguous per wave instruction) and dwpe by a column reduction over the batch.
  Replaces ATen ``embedding``/``embedding_dense_backward`` (``mappers.py:20``,
  ``neural_net_layers.py:98-118``).
* ``cross_entropy_fwd_bwd`` — one workgroup per logits row: the row (V·2 B ≤ 160 KiB) is
  staged once in LDS, max / log-sum-exp / loss computed, and the gradient
  ``(softmax − onehot)·scale`` written back **in place** as bf16: no fp32 logits, no second
  HBM read.  Replaces ``log_softmax`` + ``nll_loss`` (``neural_net_model.py:263-267``).
* ``adamw_step`` — multi-tensor fused AdamW over flat fp32 buffers (param, grad, m, v) that
  also refreshes the bf16 shadow weights the GEMMs read; torch ``AdamW`` math (decoupled
  decay, bias correction).  Replaces ``torch.optim.AdamW`` foreach (``mappers.py:55``).
* ``colsum`` — fp32 column sums of a bf16 matrix (bias gradients).
* ``tensor_stats`` — mean / std / min / max + density histogram on device for diagnostics
  (replaces ``torch.histogram(a.cpu())`` of ``neural_net_model.py:735-777``).
"""
from __future__ import annotations

import torch
from torch import Tensor

from penroz.ops._ext import kernels, use_kernels


# --------------------------------------------------------------------------- embedding
def reference_embedding_fwd(idx: Tensor, wte: Tensor, wpe: Tensor, pos_offset: int = 0) -> Tensor:
    B, T = idx.shape
    pos = torch.arange(pos_offset, pos_offset + T, device=idx.device)
    return (wte[idx].float() + wpe[pos].float().unsqueeze(0)).reshape(B * T, -1)


def embedding_fwd(idx: Tensor, wte: Tensor, wpe: Tensor, pos_offset: int = 0, out: Tensor | None = None,
                  pos_dev: Tensor | None = None, dropout_p: float = 0.0, dropout_seed: int = 0) -> Tensor:
    """idx [B,T] int64 -> fp32 [B*T, C] = drop(wte[idx] + wpe[offset + t]); ``pos_dev`` (device
    int64 [1]) supplies the offset at run time instead (graph-replayed decode; clamped to the
    table). ``dropout_p``: inverted dropout, mask hashed from (``dropout_seed``, element index)."""
    B, T = idx.shape
    out = torch.empty(B * T, wte.shape[1], dtype=torch.float32, device=idx.device) if out is None else out
    kernels().embedding_fwd(idx, wte, wpe, int(pos_offset), out, pos_dev, float(dropout_p), int(dropout_seed))
    return out


def embedding_bwd(dout: Tensor, idx: Tensor, dwte: Tensor, dwpe: Tensor, pos_offset: int = 0,
                  dropout_p: float = 0.0, dropout_seed: int = 0):
    """Accumulate (+=) into fp32 dwte [V, C] and dwpe [P, C] from dout fp32 [B*T, C] (times the
    forward's regenerated dropout mask when ``dropout_p`` > 0)."""
    kernels().embedding_bwd(dout, idx, dwte, dwpe, int(pos_offset), float(dropout_p), int(dropout_seed))


# --------------------------------------------------------------------------- cross entropy
def reference_cross_entropy(logits: Tensor, targets: Tensor) -> tuple[Tensor, Tensor]:
    """-> (per-row loss fp32 [N], dlogits fp32 [N, V] for d(sum of losses))."""
    lf = logits.float()
    lse = torch.logsumexp(lf, dim=-1)
    loss = lse - lf.gather(1, targets.view(-1, 1)).squeeze(1)
    grad = torch.softmax(lf, dim=-1)
    grad[torch.arange(lf.shape[0], device=lf.device), targets] -= 1.0
    return loss, grad


def cross_entropy_fwd_bwd(logits: Tensor, targets: Tensor, grad_scale: float, ignore_index: int = -100) -> Tensor:
    """In place: ``logits`` bf16 [N, V] becomes ``grad_scale·(softmax − onehot)``.

    Returns per-row loss fp32 [N] (0 for ignored rows).  ``grad_scale=0`` skips the gradient
    (evaluation: the logits are left untouched).
    """
    return kernels().cross_entropy_fwd_bwd(logits, targets, float(grad_scale), int(ignore_index))


class _FusedCrossEntropyFn(torch.autograd.Function):
    """Mean cross-entropy over the non-ignored rows of bf16 logits [N, V]: one kernel pass computes
    the per-row loss (fp32 statistics) and, when a gradient will be needed, the gradient of the
    summed loss into a separate buffer; backward scales it by grad_output / n_valid on the device
    (no host sync). Every target ignored gives NaN, as ``F.cross_entropy`` does (0 / 0)."""

    @staticmethod
    def forward(ctx, logits, targets, ignore_index):
        n_valid = (targets != ignore_index).sum().to(torch.float32)
        if not ctx.needs_input_grad[0]:  # no_grad / eval (evaluate_model, /output): loss only
            rows = kernels().cross_entropy_fwd_bwd(logits, targets, 0.0, int(ignore_index))
            return rows.sum() / n_valid
        grad = torch.empty_like(logits)
        rows = kernels().cross_entropy_fwd_bwd(logits, targets, 1.0, int(ignore_index), grad)
        ctx.save_for_backward(grad, n_valid.clamp_min(1))
        return rows.sum() / n_valid

    @staticmethod
    def backward(ctx, g):
        grad, n_valid = ctx.saved_tensors
        return grad.mul_((g / n_valid).to(grad.dtype)), None, None


def cross_entropy(logits: Tensor, targets: Tensor, ignore_index: int = -100) -> Tensor:
    """``F.cross_entropy(logits, targets)`` (mean over non-ignored rows). GPU bf16 logits whose rows
    are 16-B aligned take the fused HIP kernel (replaces autocast's fp32 cast + log_softmax + nll +
    their backward: ~60 GB of traffic at a 262k vocabulary, B·T = 8k); anything else runs torch —
    fp16 logits included: under fp16 + GradScaler the gradient must be scaled in fp32 before it is
    rounded to fp16 (small probabilities would flush), which torch's autocast CE does."""
    if (use_kernels(logits) and logits.dim() == 2 and logits.dtype == torch.bfloat16
            and logits.stride(1) == 1 and logits.shape[1] % 8 == 0 and logits.is_contiguous()
            and targets.dtype == torch.int64 and targets.dim() == 1):
        return _FusedCrossEntropyFn.apply(logits, targets, ignore_index)
    return torch.nn.functional.cross_entropy(logits, targets, ignore_index=ignore_index)


# --------------------------------------------------------------------------- optimizer
def reference_adamw(p, g, m, v, lr, b1, b2, eps, wd, step):
    p.mul_(1 - lr * wd)
    m.lerp_(g, 1 - b1)
    v.mul_(b2).addcmul_(g, g, value=1 - b2)
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    denom = (v.sqrt() / (bc2 ** 0.5)).add_(eps)
    p.addcdiv_(m, denom, value=-lr / bc1)


def adamw_step(params: Tensor, grads: Tensor, exp_avg: Tensor, exp_avg_sq: Tensor,
               shadow: Tensor | None, lr: float, beta1: float, beta2: float, eps: float,
               weight_decay: float, step: int, grad_scale: float = 1.0, maximize: bool = False):
    """Flat-buffer AdamW (all fp32 [numel]); ``shadow`` (bf16 [numel]) refreshed when given."""
    kernels().adamw_step(params, grads, exp_avg, exp_avg_sq, shadow, float(lr), float(beta1),
                         float(beta2), float(eps), float(weight_decay), int(step), float(grad_scale),
                         bool(maximize))


def adam_rows_step(params: Tensor, grads: Tensor, exp_avg: Tensor, exp_avg_sq: Tensor, shadow: Tensor | None,
                   C: int, mask: Tensor, rows: Tensor | None, mode: int, lr: float, beta1: float, beta2: float,
                   eps: float, weight_decay: float, step: int, grad_scale: float = 1.0, maximize: bool = False,
                   decoupled: bool = True):
    """Row-split Adam(W) of an embedding table held in flat fp32 buffers ([R·C]): mode 0 updates
    the rows with ``mask == 0`` as for a zero gradient (no gradient read); mode 1 the rows listed
    in ``rows`` whose mask is 1 (each claimed once, mask -> 2), then clears their gradient."""
    kernels().adam_rows_step(params, grads, exp_avg, exp_avg_sq, shadow, int(C), mask, rows, int(mode), float(lr),
                             float(beta1), float(beta2), float(eps), float(weight_decay), int(step),
                             float(grad_scale), bool(maximize), bool(decoupled))


def adam_step(params, grads, exp_avg, exp_avg_sq, shadow, lr, beta1, beta2, eps, weight_decay, step,
              grad_scale: float = 1.0, maximize: bool = False):
    """Flat-buffer Adam (L2 weight decay added to the gradient, torch ``Adam`` semantics)."""
    kernels().adam_step(params, grads, exp_avg, exp_avg_sq, shadow, float(lr), float(beta1),
                        float(beta2), float(eps), float(weight_decay), int(step), float(grad_scale),
                        bool(maximize))


# --------------------------------------------------------------------------- reductions
def colsum(x: Tensor, out: Tensor) -> None:
    """out (fp32 [M]) += x.sum(0) for x bf16/fp32 [N, M]."""
    kernels().colsum(x, out)


def tensor_stats(x: Tensor, bins: int = 100):
    """-> (mean, std, min, max, hist fp32 [bins], edges fp32 [bins+1]) with density hist."""
    if use_kernels(x):
        s = kernels().tensor_stats(x.contiguous(), int(bins))
        return s
    xf = x.detach().float().reshape(-1)
    h = torch.histogram(xf.cpu(), bins=bins, density=True)
    return (xf.mean(), xf.std(), xf.min(), xf.max(), h.hist, h.bin_edges)
