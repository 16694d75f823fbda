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
# pipeline variant of the 256-tile kernel (csrc/kernels/gemm_wgrad.hip): 8 (fragment prefetch), 6,
# 4 — A/B knob. Unset: 8 for long token dimensions (GPT-2 B=64: K = 65 536), 6 for K <= 16 384,
# where the prefetch's extra prologue does not pay (Gemma-3 1B B=8, K = 8192: 67.05 / 67.11 ->
# 66.62 / 66.66 ms; GPT-2: 8 beats 6, 61.28 / 61.35 vs 61.49 / 61.43 ms; profiles/knobs_ab_r4.log)
_WGRAD_VARIANT_ENV = os.environ.get("PENROZ_WGRAD_VARIANT")
WGRAD_VARIANT = int(_WGRAD_VARIANT_ENV) if _WGRAD_VARIANT_ENV else 0  # 0: by K
WGRAD_SHORT_K = 16384


def _wgrad_variant(k: int) -> int:
    if WGRAD_VARIANT:
        return WGRAD_VARIANT
    return 6 if k <= WGRAD_SHORT_K else 8


def _native_ok(m: int, n: int, lda: int | None = None) -> bool:
    """m need not be a multiple of 8 when dy's rows are padded to it (lda >= round_up(m, 8))."""
    return NATIVE_WGRAD != "0" and n % 8 == 0 and (m % 8 == 0 or (lda is not None and lda >= (m + 7) // 8 * 8))


def reference_wgrad(dy: Tensor, x: Tensor, grad: Tensor, accumulate: bool = True) -> None:
    if accumulate:
        grad.add_(dy.float().t() @ x.float())
    else:
        grad.copy_(dy.float().t() @ x.float())


def wgrad(dy: Tensor, x: Tensor, grad: Tensor, accumulate: bool = True) -> None:
    """grad += dyᵀ·x, or grad = dyᵀ·x with accumulate=False (the first weight-gradient write of a
    step whose zero_grad skipped this range)."""
    if (use_kernels(dy) and _native_ok(dy.shape[1], x.shape[1], dy.stride(0)) and dy.dtype == torch.bfloat16
            and x.dtype == torch.bfloat16 and dy.stride(0) % 8 == 0 and x.stride(0) % 8 == 0):
        kernels().wgrad_gemm(dy, x, grad, 256, _wgrad_variant(dy.shape[0]), accumulate)
    elif dy.is_cuda:
        prod = torch.mm(dy.t(), x, out_dtype=torch.float32)
        grad.add_(prod) if accumulate else grad.copy_(prod)
    else:
        reference_wgrad(dy, x, grad, accumulate)


# ---- library GEMM solution choice (hipBLASLt / rocBLAS through torch) -----------------------
# The forward / dgrad GEMMs stay library calls; which hipBLASLt (or rocBLAS) solution runs each
# shape is measured, not left to the heuristic: bench/tune_gemms.sh runs PyTorch TunableOp's
# solution search over every GEMM the executor issues at the GPT-2 headline shapes (and the HF
# import layout) and ops/tuned/tunableop_gfx950.csv ships the winners (validated against the
# PyTorch / HIP / hipBLASLt / rocBLAS versions and the gfx950 arch at load; a mismatch is refused
# by torch and the heuristic picks stay). Loaded read-only (no tuning at run time; shapes not in
# the file keep the default solution). PENROZ_TUNED_GEMMS=0 disables.
TUNED_GEMM_FILE = os.environ.get("PENROZ_TUNED_GEMM_FILE") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "tuned", "tunableop_gfx950.csv")
_tuned_state: dict = {}


def load_tuned_gemms() -> bool:
    """Enable TunableOp in read-only mode with the shipped results (once per process)."""
    if "loaded" in _tuned_state:
        return _tuned_state["loaded"]
    ok = False
    if (os.environ.get("PENROZ_TUNED_GEMMS", "1") != "0" and os.environ.get("PYTORCH_TUNABLEOP_TUNING") != "1"
            and torch.cuda.is_available() and os.path.exists(TUNED_GEMM_FILE)):
        import torch.cuda.tunable as tunable
        tunable.enable(True)
        tunable.tuning_enable(False)
        tunable.record_untuned_enable(False)
        ok = bool(tunable.read_file(TUNED_GEMM_FILE))
        if not ok:
            tunable.enable(False)
    _tuned_state["loaded"] = ok
    return ok


def set_tuned_gemms(on: bool) -> bool:
    """Switch the loaded table's solutions on or off at run time (off: hipBLASLt's own heuristic
    for every shape). Returns whether the table is now in use."""
    if not _tuned_state.get("loaded"):
        return False
    import torch.cuda.tunable as tunable
    tunable.enable(bool(on))
    _tuned_state["active"] = bool(on)
    return bool(on)


def guard_tuned_gemms(run_steps, steps: int = 3, rounds: int = 2, margin: float = 1.0, agree=None) -> dict:
    """The shipped table must never cost time (it once drifted to 1 ms/step SLOWER than
    hipBLASLt's heuristic and nothing noticed). Times ``run_steps(steps)`` (returns seconds) with the
    table off and on, ``rounds`` interleaved times each, keeps the table only if its best time is
    <= ``margin`` × the heuristic's best, and leaves that choice switched on. ``agree`` (optional)
    maps a local time to the group's (MAX over ranks) so every rank decides the same.
    {} when no table is loaded."""
    if not _tuned_state.get("loaded"):
        return {}
    best = {False: float("inf"), True: float("inf")}
    for _ in range(rounds):
        for on in (False, True):
            set_tuned_gemms(on)
            dt = run_steps(steps)
            if agree is not None:
                dt = agree(dt)
            best[on] = min(best[on], dt / steps)
    keep = best[True] <= margin * best[False]
    set_tuned_gemms(keep)
    return {"table": os.path.basename(TUNED_GEMM_FILE), "with_table_ms": round(best[True] * 1e3, 3),
            "heuristic_ms": round(best[False] * 1e3, 3), "table_kept": keep}


# ---- linear + GELU / GELU backward (library GEMM + the HIP GELU kernels) -------------------
# Two native fused designs were built and measured against this pair (round 3-4): an 8-phase
# persistent MFMA GEMM with a bias/GELU epilogue and a 4-wave deferred-epilogue GEMM whose
# stores (and GELU' / bias-column work) stream inside the next tile. Both lost on every GPT-2
# shape and on the headline step (profiles/gemm_epi_r4.log, profiles/native_gemm_r4.md), so the
# forward / dgrad GEMMs are hipBLASLt and the GELU work stays in elementwise.hip.
def linear_gelu(x: Tensor, w: Tensor, bias: Tensor, pre: Tensor, act: Tensor, approximate: str = "none"):
    """pre = x·wᵀ + bias (library GEMM), act = GELU(pre) (bf16; ``approximate`` "none" = erf,
    "tanh" = gelu_new; the HIP GELU kernel)."""
    torch.addmm(bias, x, w.t(), out=pre)
    if use_kernels(pre):
        from penroz.ops import activations as act_ops
        act_ops.gelu_fwd(pre, approximate, out=act)
    else:
        act.copy_(torch.nn.functional.gelu(pre.float(), approximate=approximate))
    return pre, act


def dgrad_gelu(dy: Tensor, wt: Tensor, pre: Tensor, out: Tensor, dbias: Tensor | None, approximate: str = "none"):
    """Data gradient into a GELU's input: out = bf16(dy·wtᵀ) (library GEMM; ``wt`` = the
    transposed weight copy, [in, out] row-major), then out *= GELU'(pre) and dbias (fp32) += the
    column sums of out in one HIP kernel. The GPT executor's fc2 data gradient + GELU backward +
    fc bias gradient."""
    torch.mm(dy, wt.t(), out=out)
    from penroz.ops import activations as act_ops
    act_ops.gelu_bwd(out, pre, approximate, dbias, out=out)
    return out


# ---- decode-shaped GEMMs (csrc/kernels/skinny_gemm.hip) --------------------------------------
# out[M<=64, N] = x·Wᵀ (+ bias), bf16: one 16-column MFMA slice per workgroup over all rows,
# K split across the 4 waves (and across workgroups, with an in-launch slab reduction, when the
# output is narrow). Used for the graph-captured decode step (models/graph_decode.py), where a
# library GEMM tile at M = 64 leaves most CUs idle (~10 µs for a 3.5 MB weight read).
SKINNY_GEMM = os.environ.get("PENROZ_SKINNY_GEMM", "1") != "0"
_skinny_ws: dict = {}


def skinny_workspace(device: torch.device) -> tuple[Tensor, Tensor]:
    """Per-device split-K workspace and arrival counters (zeroed once, outside any graph
    capture; every launch leaves the counters zero again)."""
    key = (device.type, device.index if device.index is not None else torch.cuda.current_device())
    buf = _skinny_ws.get(key)
    if buf is None:
        dev = torch.device(*key)
        buf = (torch.empty(1 << 19, device=dev, dtype=torch.float32), torch.zeros(1 << 12, device=dev, dtype=torch.int32))
        _skinny_ws[key] = buf
    return buf


def skinny_ok(x: Tensor, w: Tensor) -> bool:
    if not (SKINNY_GEMM and x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16):
        return False
    K = x.shape[-1]
    rows = x.numel() // K if K else 0
    return (0 < rows <= 64 and K % 32 == 0 and w.is_contiguous() and w.shape[1] == K and w.data_ptr() % 16 == 0
            and use_kernels(x))


def skinny_linear(x: Tensor, w: Tensor, bias: Tensor | None) -> Tensor:
    """nn.Linear forward for ≤ 64 rows of bf16 activations (any leading shape)."""
    K, N = x.shape[-1], w.shape[0]
    x2 = x.reshape(-1, K)
    if x2.stride(1) != 1 or x2.stride(0) % 8 or x2.data_ptr() % 16:
        x2 = x2.contiguous()
    out = torch.empty(x2.shape[0], N, device=x.device, dtype=x.dtype)
    ws, cnt = skinny_workspace(x.device)
    kernels().skinny_gemm(x2, w, bias if bias is None or bias.dtype == torch.bfloat16 else bias.to(torch.bfloat16),
                          out, ws, cnt)
    return out.view(*x.shape[:-1], N)


def skinny_gated(x: Tensor, gu: Tensor, kind: int) -> Tensor:
    """Gated-MLP decode projection in one launch: act(x·gu[:I]ᵀ) ⊙ (x·gu[I:]ᵀ) for ≤ 64 rows,
    ``gu`` the packed [gate; up] weight [2I, K]; kind 0 gelu, 1 gelu_tanh, 2 silu. Bit-identical to
    ``skinny_linear`` + the packed gated-activation kernel (csrc/kernels/skinny_gemm.hip)."""
    out = torch.empty(x.shape[0], gu.shape[0] // 2, device=x.device, dtype=x.dtype)
    kernels().skinny_gated(x, gu, out, kind)
    return out


def skinny_qkv_rope_ok(x: Tensor, w: Tensor, D: int) -> bool:
    """The fused QKV + RoPE decode kernel applies: skinny shapes, whole heads of D % 32 == 0, and
    its split-K slabs fit the shared workspace."""
    if not (skinny_ok(x, w) and D % 32 == 0 and w.shape[0] % D == 0):
        return False
    return qkv_rope_plan_fits(x.numel() // x.shape[-1], w.shape[0], x.shape[-1])


def qkv_rope_plan_fits(rows: int, n: int, k: int) -> bool:
    """The kernel's own split-K plan (csrc/kernels/skinny_gemm.hip skinny_qkv_rope_plan: the rule
    its launcher applies) fits the shared workspace and counters of ``skinny_workspace``."""
    _, ws_floats, counters = kernels().skinny_qkv_rope_plan(rows, n, k)
    return ws_floats <= (1 << 19) and counters <= (1 << 12)


def skinny_qkv_rope(x: Tensor, w: Tensor, cos: Tensor, sin: Tensor, D: int, nrot: int) -> Tensor:
    """Decode QKV projection with RoPE (one position's cos / sin [D/2]) applied to the first
    ``nrot`` heads in the GEMM epilogue (csrc/kernels/skinny_gemm.hip); ≤ 64 rows."""
    out = torch.empty(x.shape[0], w.shape[0], device=x.device, dtype=x.dtype)
    ws, cnt = skinny_workspace(x.device)
    kernels().skinny_qkv_rope(x, w, cos, sin, D, nrot, out, ws, cnt)
    return out


class decode_gemms:
    """Context: the ``nn.Linear`` modules of ``model`` run decode-shaped inputs through the skinny
    kernel (others keep ``F.linear``). Entered by the graph decoder around the captured step of a
    model without a decode program. Only that model's own Linear instances are re-routed (an
    instance-level ``forward``, removed on exit): other models, and other threads serving them,
    are untouched; the serving lock keeps concurrent requests off the same model."""

    def __init__(self, model: torch.nn.Module, max_rows: int = 64):
        self.model = model
        self.max_rows = max_rows
        self._patched: list[torch.nn.Linear] = []

    def __enter__(self):
        if not (SKINNY_GEMM and self.max_rows > 0):
            return self
        max_rows = self.max_rows
        for mod in self.model.modules():
            if type(mod) is not torch.nn.Linear or "forward" in mod.__dict__:
                continue

            def forward(x, mod=mod):
                if (x.numel() <= max_rows * x.shape[-1] and skinny_ok(x, mod.weight)
                        and (mod.bias is None or mod.bias.is_contiguous())):
                    return skinny_linear(x, mod.weight, mod.bias)
                return torch.nn.functional.linear(x, mod.weight, mod.bias)

            mod.forward = forward
            self._patched.append(mod)
        return self

    def __exit__(self, *exc):
        for mod in self._patched:
            mod.__dict__.pop("forward", None)
        self._patched.clear()
        return False
