"""GEMM entry points.

* ``wgrad(dy, x, grad)`` — ``grad += dyᵀ·x`` for weight gradients (bf16 operands, fp32
  accumulate into the flat gradient buffer). GPU: the hand-written MFMA split-K kernel in
  ``csrc/kernels/gemm_wgrad.hip`` (both operands row-major in tokens, transposed LDS reads,
  deterministic slab reduction fused with the accumulate). Forward / dgrad GEMMs stay on
  hipBLASLt through ``torch.addmm``/``torch.mm`` (measured ≈0.9–1.4 PF at these shapes).
"""
from __future__ import annotations

import os

import torch
from torch import Tensor

from penroz.ops._ext import use_kernels, kernels

# "auto": the native kernel where it measured faster than hipBLASLt (small M×N outputs, e.g.
# the 768×768 attention projection: 334 vs 281 TF); "1" always; "0" never.
NATIVE_WGRAD = os.environ.get("PENROZ_NATIVE_WGRAD", "auto")


def _native_ok(m: int, n: int) -> bool:
    if NATIVE_WGRAD == "1":
        return True
    if NATIVE_WGRAD == "0":
        return False
    return m * n <= 1 << 20


def reference_wgrad(dy: Tensor, x: Tensor, grad: Tensor) -> None:
    grad.add_(dy.float().t() @ x.float())


def wgrad(dy: Tensor, x: Tensor, grad: Tensor) -> None:
    if use_kernels(dy) and _native_ok(dy.shape[1], x.shape[1]):
        kernels().wgrad_gemm(dy, x, grad)
    elif dy.is_cuda:
        grad.add_(torch.mm(dy.t(), x, out_dtype=torch.float32))
    else:
        reference_wgrad(dy, x, grad)
