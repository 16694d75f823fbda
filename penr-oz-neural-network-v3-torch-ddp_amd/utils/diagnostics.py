"""Training diagnostics for the dashboard: weight-update ratios and layer/weight statistics.

Schema parity with the reference (``neural_net_model.py:690-700, 735-777``):
``weight_upd_ratio`` = std(Δw)/(std(w)+1e-8) per 2-D weight (None otherwise);
stats = ``{"layers": [{algo, activation: {mean, std, saturated, histogram: {x, y}},
gradient: {mean, std, histogram} | None}], "weights": [{shape, data: {mean, std},
gradient: {mean, std, histogram}} | None]}`` with 100-bin density histograms and the same
per-algo saturation rules.

MI355X-first: every statistic is computed on the device (``tensor_stats`` HIP kernel: one
fused moments + min/max pass and one histogram pass) and copied back in ONE transfer per
tensor; the reference does ``torch.histogram(a.cpu())`` — including a full copy of the
``[B, T, V]`` logits to the host — and one ``.item()`` sync per weight.
"""
from __future__ import annotations

import torch
from torch import Tensor

from penroz.ops import fused as fused_ops


@torch.no_grad()
def start_update_ratios(prev: list, weights: list):
    """Device-side part of :func:`weight_update_ratios`: std(w − prev) and std(w) of every weight,
    stacked on the device and copied to pinned host memory without waiting (the training loop
    reads them one epoch later with :func:`finish_update_ratios`)."""
    pairs = [(i, w.detach(), pw) for i, (pw, w) in enumerate(zip(prev, weights)) if pw is not None and w is not None]
    idx = [i for i, _, _ in pairs]
    if not pairs:
        return (len(weights), idx, None)
    from penroz.ops._ext import use_kernels, kernels
    ws, ps = [w for _, w, _ in pairs], [p for _, _, p in pairs]
    if (use_kernels(ws[0]) and len({(w.dtype, p.dtype) for w, p in zip(ws, ps)}) == 1
            and ws[0].dtype in (torch.float32, torch.bfloat16) and all(w.is_contiguous() and p.is_contiguous()
                                                                      for w, p in zip(ws, ps))):
        dev = kernels().update_moments(ws, ps)  # one chunked launch + one fold (csrc/kernels/adamw.hip)
    else:
        dev = torch.stack([torch.stack([(w - pw).float().std(), w.float().std()]) for w, pw in zip(ws, ps)])
    host = torch.empty(dev.shape, dtype=dev.dtype, pin_memory=dev.is_cuda)
    host.copy_(dev, non_blocking=dev.is_cuda)
    return (len(weights), idx, host)


def finish_update_ratios(started) -> list:
    """The per-weight update ratios of :func:`start_update_ratios` (after its work completed)."""
    n, idx, host = started
    out: list = [None] * n
    if host is not None:
        for i, (d, s) in zip(idx, host.tolist()):
            out[i] = d / (s + 1e-8)
    return out


def weight_update_ratios(prev: list, weights: list) -> list:
    vals = []
    idx = []
    for i, (pw, w) in enumerate(zip(prev, weights)):
        if pw is None or w is None:
            continue
        vals.append(torch.stack([(w - pw).float().std(), w.float().std()]))
        idx.append(i)
    out: list = [None] * len(weights)
    if vals:
        host = torch.stack(vals).cpu().tolist()
        for i, (d, s) in zip(idx, host):
            out[i] = d / (s + 1e-8)
    return out


def _hist(x: Tensor, bins: int = 100):
    mean, std, mn, mx, hist, edges = fused_ops.tensor_stats(x, bins)
    return float(mean), float(std), edges[:-1].tolist(), hist.tolist()


@torch.no_grad()
def _saturation(algo: str, a: Tensor) -> float:
    a = a.float()
    if algo == "embedding":
        sat = torch.norm(a, dim=-1) > 5.0
    elif algo == "batchnorm1d":
        sat = a.abs() > 3.0
    elif algo in ("tanh", "sigmoid"):
        sat = a.abs() > 0.97
    elif algo == "relu":
        sat = a <= 0
    elif algo == "softmax":
        sat = a.max(dim=-1).values > 0.97
    else:
        sat = a.abs() > 5.0
    return float(sat.float().mean())


@torch.no_grad()
def training_stats(algos: list[str], acts: list, weights: list, grad_of=None) -> dict:
    """``grad_of(w)``: the gradient of weight ``w`` when it is not ``w.grad`` (the fused executor
    keeps bf16-parameter models' fp32 gradients in its flat buffer)."""
    layers = []
    for algo, pair in zip(algos, acts):
        a, g = pair
        mean, std, hx, hy = _hist(a)
        entry = {"algo": algo, "activation": {"mean": mean, "std": std, "saturated": _saturation(algo, a),
                                               "histogram": {"x": hx, "y": hy}},
                 "gradient": None}
        if g is not None:
            gm, gs, gx, gy = _hist(g)
            entry["gradient"] = {"mean": gm, "std": gs, "histogram": {"x": gx, "y": gy}}
        layers.append(entry)
    wstats = []
    for w in weights:
        if w is None:
            wstats.append(None)
            continue
        wm, ws = float(w.float().mean()), float(w.float().std())
        grad = {"mean": None, "std": None, "histogram": {"x": [], "y": []}}
        g = grad_of(w) if grad_of is not None else w.grad
        if g is not None:
            gm, gs, gx, gy = _hist(g)
            grad = {"mean": gm, "std": gs, "histogram": {"x": gx, "y": gy}}
        wstats.append({"shape": str(tuple(w.shape)), "data": {"mean": wm, "std": ws}, "gradient": grad})
    return {"layers": layers, "weights": wstats}
