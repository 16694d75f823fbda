"""GEMM entry points.

* ``wgrad(dy, x, grad)`` — ``grad += dyᵀ·x`` for weight gradients (bf16 operands, fp32
  accumulate into the flat gradient buffer). GPU: the hand-written MFMA split-K kernel in
  ``csrc/kernels/gemm_wgrad.hip`` (256×256 tile, LDS-DMA staging, transposed LDS reads,
  wave-quantisation-aware split-K, deterministic slab reduction fused with the accumulate).
  Measured at GPT-2 124M shapes (K = 65 536 tokens, profiles/kernel_bench_r1_wgrad_ring16.log): 800–1100 TF
  vs hipBLASLt's 270–950 TF on the same calls. Forward / dgrad GEMMs stay on hipBLASLt through
  ``torch.addmm``/``torch.mm`` (measured ≈0.9–1.4 PF at these shapes).
"""
from __future__ import annotations

import os

import torch
from torch import Tensor

from penroz.ops._ext import use_kernels, kernels

# "auto"/"1": the native kernel (faster than hipBLASLt on every measured GPT-2 shape);
# "0": hipBLASLt (A/B switch for benchmarking).
NATIVE_WGRAD = os.environ.get("PENROZ_NATIVE_WGRAD", "auto")


def _native_ok(m: int, n: int) -> bool:
    return NATIVE_WGRAD != "0" and m % 8 == 0 and n % 8 == 0


def reference_wgrad(dy: Tensor, x: Tensor, grad: Tensor) -> None:
    grad.add_(dy.float().t() @ x.float())


def wgrad(dy: Tensor, x: Tensor, grad: Tensor) -> None:
    if (use_kernels(dy) and _native_ok(dy.shape[1], x.shape[1]) and dy.dtype == torch.bfloat16
            and x.dtype == torch.bfloat16 and dy.stride(0) % 8 == 0 and x.stride(0) % 8 == 0):
        kernels().wgrad_gemm(dy, x, grad)
    elif dy.is_cuda:
        grad.add_(torch.mm(dy.t(), x, out_dtype=torch.float32))
    else:
        reference_wgrad(dy, x, grad)


# ---- forward / dgrad GEMMs (csrc/kernels/gemm.hip) ------------------------------------------
# EXPERIMENTAL native path: persistent 256×256-tile MFMA kernel (LDS-DMA double-buffered 64-deep
# chunks, ping-pong wave groups) with fused bias / bias+GELU epilogues. Measured slower than
# hipBLASLt on every GPT-2 shape (profiles/gemm_native_r1.log: 0.78-0.92× fwd, 0.85-0.95× dgrad),
# so it is OFF by default; PENROZ_NATIVE_GEMM=1 routes linear_fwd / linear_dgrad through it.
NATIVE_GEMM = os.environ.get("PENROZ_NATIVE_GEMM", "0")


def _gemm_ok(a: Tensor, b: Tensor, n: int) -> bool:
    return (NATIVE_GEMM == "1" and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16
            and a.shape[1] % 32 == 0 and a.shape[1] >= 128 and n % 8 == 0 and a.stride(1) == 1 and b.stride(1) == 1
            and a.stride(0) % 8 == 0 and b.stride(0) % 8 == 0)


def linear_fwd(x: Tensor, w: Tensor, bias: Tensor | None, out: Tensor, act: Tensor | None = None,
               gelu_approx: str = "none") -> Tensor:
    """out = x·wᵀ (+ bias); with ``act``: out = pre-activation, act = GELU(out) (one pass)."""
    if use_kernels(x) and _gemm_ok(x, w, w.shape[0]):
        kernels().gemm_bf16(x, w, False, bias, out, act, 1 if gelu_approx == "tanh" else 0)
        return out
    if bias is not None:
        torch.addmm(bias, x, w.t(), out=out)
    else:
        torch.mm(x, w.t(), out=out)
    if act is not None:
        act.copy_(torch.nn.functional.gelu(out.float(), approximate=gelu_approx))
    return out


def linear_dgrad(dy: Tensor, w: Tensor, out: Tensor) -> Tensor:
    """out = dy·w (input gradient of y = x·wᵀ)."""
    if use_kernels(dy) and _gemm_ok(dy, w, w.shape[1]):
        kernels().gemm_bf16(dy, w, True, None, out)
        return out
    return torch.mm(dy, w, out=out)
