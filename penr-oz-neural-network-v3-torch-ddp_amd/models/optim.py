"""Fused Adam / AdamW: ``torch.optim`` subclasses whose GPU step is one HIP launch family.

State-dict format is exactly torch's (``state[p] = {step, exp_avg, exp_avg_sq}``, one param
group), so reference checkpoints load and ours load in the reference.  On GPU:
  * *flat mode* — when every parameter of the group is a view of one contiguous fp32 buffer
    (set up by :meth:`FusedAdamW.attach_flat`, used by the fused GPT executor), the step is a
    single grid-stride kernel over (param, grad, m, v) that also rewrites the bf16 shadow
    weights the GEMMs read (``csrc/kernels/adamw.hip``);
  * *list mode* — otherwise a multi-tensor kernel walks a chunk table of the group's tensors
    (fp32, or bf16 parameters with bf16 state as torch keeps it, updated in fp32 registers).
On CPU (or amsgrad / differentiable / capturable options) the stock torch step runs.
Replaces the reference's ``torch.optim.AdamW`` foreach step (``mappers.py:53-57``,
``neural_net_model.py:677``).
"""
from __future__ import annotations

import torch
from torch import Tensor

from penroz.ops import _ext
from penroz.ops import fused as fused_ops


class _FusedMixin:
    _decoupled = True

    def _init_fused(self):
        self._flat = None  # dict with flat buffers when attached

    # ------------------------------------------------------------------ flat buffers
    def attach_flat(self, params: list[Tensor], flat_param: Tensor, flat_grad: Tensor,
                    flat_shadow: Tensor | None, offsets: list[int]):
        """Register that ``params`` are views of ``flat_param`` at ``offsets``.

        Allocates flat ``exp_avg`` / ``exp_avg_sq`` buffers, copies any existing state into them
        and re-points each param's state tensors at views, so ``state_dict()`` is unchanged.
        """
        n = flat_param.numel()
        m = torch.zeros(n, dtype=torch.float32, device=flat_param.device)
        v = torch.zeros(n, dtype=torch.float32, device=flat_param.device)
        steps = set()
        for p, off in zip(params, offsets):
            st = self.state[p]
            k = p.numel()
            if "exp_avg" in st:
                m[off:off + k].copy_(st["exp_avg"].reshape(-1))
                v[off:off + k].copy_(st["exp_avg_sq"].reshape(-1))
            st["exp_avg"] = m[off:off + k].view_as(p)
            st["exp_avg_sq"] = v[off:off + k].view_as(p)
            if "step" not in st:
                st["step"] = torch.tensor(0.0)
            steps.add(float(st["step"]))
        if len(steps) > 1:
            raise ValueError(f"flat AdamW needs a common step count, got {sorted(steps)}")
        self._flat = {"params": list(params), "param": flat_param, "grad": flat_grad, "m": m, "v": v,
                      "shadow": flat_shadow, "ids": {id(p) for p in params}}

    def detach_flat(self):
        self._flat = None

    def load_state_dict(self, state_dict):
        flat = self._flat
        super().load_state_dict(state_dict)
        if flat is not None:  # keep state tensors as views of the flat buffers
            offs = []
            base = flat["param"].data_ptr()
            for p in flat["params"]:
                offs.append((p.data_ptr() - base) // p.element_size())
            self.attach_flat(flat["params"], flat["param"], flat["grad"], flat["shadow"], offs)

    # ------------------------------------------------------------------ step
    def _group_fused_ok(self, group) -> bool:
        if group.get("amsgrad") or group.get("differentiable") or group.get("capturable"):
            return False
        ps = [p for p in group["params"] if p.grad is not None]
        return bool(ps) and all(p.is_cuda and p.dtype in (torch.float32, torch.bfloat16) and p.grad.dtype == p.dtype
                                for p in ps) and _ext.available()

    @staticmethod
    def _group_cpu_fused_ok(group) -> bool:
        if group.get("differentiable") or group.get("capturable"):
            return False
        ps = [p for p in group["params"] if p.grad is not None]
        return bool(ps) and all(p.device.type == "cpu" and not p.grad.is_sparse and p.grad.dtype == p.dtype
                                and p.dtype in (torch.float32, torch.float64, torch.bfloat16) for p in ps)

    @torch.no_grad()
    def step(self, closure=None, grad_scale: float = 1.0):
        """One optimizer step; ``grad_scale`` multiplies every gradient (e.g. 1/num_steps)."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if len(self.param_groups) == 1 and self._flat is not None and \
                {id(p) for p in self.param_groups[0]["params"]} == self._flat["ids"]:
            self._step_flat(self.param_groups[0], grad_scale)
            return loss
        fallback = []
        for group in self.param_groups:
            if self._group_fused_ok(group):
                self._step_list(group, grad_scale)
            else:
                fallback.append(group)
        if fallback:
            if grad_scale != 1.0:
                for g in fallback:
                    for p in g["params"]:
                        if p.grad is not None:
                            p.grad.mul_(grad_scale)
            # host parameters: torch's single-pass vectorised CPU kernel (6x the per-tensor loop at
            # the GPT-2 124M plumbing config: 76 vs 461 ms per step with 4 threads)
            cpu_fused = [g for g in fallback if self._group_cpu_fused_ok(g)]
            for g in cpu_fused:
                g["fused"] = True
            saved = self.param_groups
            self.param_groups = fallback
            try:
                super().step()
            finally:
                self.param_groups = saved
                for g in cpu_fused:
                    g["fused"] = None
        return loss

    def _hyper(self, group):
        b1, b2 = group["betas"]
        lr = group["lr"]
        lr = float(lr) if not isinstance(lr, Tensor) else float(lr.item())
        return lr, float(b1), float(b2), float(group["eps"]), float(group["weight_decay"]), \
            bool(group.get("maximize", False))

    def _step_flat(self, group, grad_scale, ranges=None):
        f = self._flat
        lr, b1, b2, eps, wd, maximize = self._hyper(group)
        step = None
        for p in f["params"]:
            st = self.state[p]
            st["step"] += 1
            step = int(st["step"].item()) if step is None else step
        fn = fused_ops.adamw_step if self._decoupled else fused_ops.adam_step
        if ranges is None:
            fn(f["param"], f["grad"], f["m"], f["v"], f["shadow"], lr, b1, b2, eps, wd, step, grad_scale, maximize)
            return
        sh = f["shadow"]
        for r in ranges:  # (s, e) pairs, or a callable returning one (it may wait for the range first)
            s, e = r() if callable(r) else r
            fn(f["param"][s:e], f["grad"][s:e], f["m"][s:e], f["v"][s:e], sh[s:e] if sh is not None else None,
               lr, b1, b2, eps, wd, step, grad_scale, maximize)

    def begin_flat_ranges(self, grad_scale: float = 1.0):
        """Start a flat step whose ranges are applied later, one call per range, e.g. each
        parameter segment as soon as its gradients are final inside the backward. Returns
        ``apply(s, e)`` or None when the flat path does not apply. The step counter advances now,
        once; the caller must cover the flat buffer exactly once before the next step."""
        if not (len(self.param_groups) == 1 and self._flat is not None
                and {id(p) for p in self.param_groups[0]["params"]} == self._flat["ids"]):
            return None
        f, group = self._flat, self.param_groups[0]
        lr, b1, b2, eps, wd, maximize = self._hyper(group)
        step = None
        for p in f["params"]:
            st = self.state[p]
            st["step"] += 1
            step = int(st["step"].item()) if step is None else step
        fn = fused_ops.adamw_step if self._decoupled else fused_ops.adam_step
        sh = f["shadow"]

        def apply(s: int, e: int):
            fn(f["param"][s:e], f["grad"][s:e], f["m"][s:e], f["v"][s:e], sh[s:e] if sh is not None else None,
               lr, b1, b2, eps, wd, step, grad_scale, maximize)

        def apply_rows(s: int, e: int, C: int, mask, rows, mode: int):
            """[s, e) as an embedding table of width C: fused_ops.adam_rows_step (same math)."""
            fused_ops.adam_rows_step(f["param"][s:e], f["grad"][s:e], f["m"][s:e], f["v"][s:e],
                                     sh[s:e] if sh is not None else None, C, mask, rows, mode, lr, b1, b2, eps, wd,
                                     step, grad_scale, maximize, self._decoupled)
        apply.rows = apply_rows
        return apply

    def flat_step_ranges(self, ranges, grad_scale: float = 1.0) -> bool:
        """Flat step applied range by range (``ranges`` must cover the flat buffer exactly once);
        False (nothing done) when the flat path does not apply."""
        if not (len(self.param_groups) == 1 and self._flat is not None
                and {id(p) for p in self.param_groups[0]["params"]} == self._flat["ids"]):
            return False
        self._step_flat(self.param_groups[0], grad_scale, ranges)
        return True

    def _step_list(self, group, grad_scale):
        lr, b1, b2, eps, wd, maximize = self._hyper(group)
        by_step: dict[int, list] = {}
        for p in group["params"]:
            if p.grad is None:
                continue
            st = self.state[p]
            if len(st) == 0:
                st["step"] = torch.tensor(0.0)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["step"] += 1
            by_step.setdefault((int(st["step"].item()), p.dtype), []).append(p)
        k = _ext.kernels()
        for (step, _), ps in by_step.items():
            k.multi_tensor_adam([p.data for p in ps], [p.grad for p in ps],
                                [self.state[p]["exp_avg"] for p in ps], [self.state[p]["exp_avg_sq"] for p in ps],
                                lr, b1, b2, eps, wd, step, float(grad_scale), maximize, self._decoupled)


class FusedAdamW(_FusedMixin, torch.optim.AdamW):
    """``torch.optim.AdamW`` (defaults: lr 1e-3, betas (0.9, 0.999), eps 1e-8, weight_decay 0.01)."""
    _decoupled = True

    def __init__(self, params, *args, **kwargs):
        kwargs.pop("fused", None)
        kwargs.pop("foreach", None)
        torch.optim.AdamW.__init__(self, params, *args, **kwargs)
        self._init_fused()


class FusedAdam(_FusedMixin, torch.optim.Adam):
    """``torch.optim.Adam`` (L2 weight decay added to the gradient)."""
    _decoupled = False

    def __init__(self, params, *args, **kwargs):
        kwargs.pop("fused", None)
        kwargs.pop("foreach", None)
        torch.optim.Adam.__init__(self, params, *args, **kwargs)
        self._init_fused()
