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
