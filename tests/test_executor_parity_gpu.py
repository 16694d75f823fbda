"""Fused executor parity at the headline shape and over a 100-step training run (MI355X).

* one step of the full GPT-2 124M example layout (C=768, 12 layers, V=50304, T=1024) against the
  same model run as plain fp32 PyTorch ops on the GPU (the fp32 reference of every kernel);
* 100 AdamW steps from one initialisation against the ``reference`` engine (stock eager PyTorch +
  bf16 autocast + torch.optim.AdamW — the reference's own training semantics): the loss curves
  must agree.
"""
import copy
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

import bench
from penroz.models.executor import GPTExecutor
from penroz.models.mapper import Mapper
from penroz.models.model import NeuralNetworkModel, _make_runner
from penroz.ops import _ext


def _gpt2(V=50304, C=768, L=12, H=12, P=1024, seed=0):
    torch.manual_seed(seed)
    return NeuralNetworkModel("p", Mapper(bench.gpt2_layers(V=V, C=C, L=L, H=H, P=P),
                                          {"adamw": {"lr": 6e-4, "betas": [0.9, 0.95], "eps": 1e-8}}))


def test_headline_shape_one_step_matches_fp32():
    m = _gpt2().cuda()
    ref = copy.deepcopy(m)
    B, T = 4, 1024
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randint(0, 50304, (B, T), device="cuda", generator=g)
    y = torch.randint(0, 50304, (B, T), device="cuda", generator=g)
    _ext.FORCE_TORCH = True  # plain fp32 torch ops: the reference of every HIP kernel
    try:
        _, loss_ref = ref(x, y, skip_softmax=True)
        loss_ref.backward()
    finally:
        _ext.FORCE_TORCH = False
    ex = GPTExecutor(m, torch.device("cuda"))
    ex.setup_training(False)
    ex.zero_grad()
    loss = ex.train_micro_step(x, y, 1.0)
    assert abs(loss.item() - loss_ref.item()) < 2e-2, (loss.item(), loss_ref.item())
    worst = 0.0
    for (n, p), (_, r) in zip(m.named_parameters(), ref.named_parameters()):
        rel = ((ex.grad(p) - r.grad).norm() / (r.grad.norm() + 1e-12)).item()
        worst = max(worst, rel)
        # measured worst over all parameters: 0.0104 (round 6, profiles/bench_r6_configs_final.log);
        # 2 % is that plus a margin — a regression to the former 5 % bound would now fail
        assert rel < 2e-2, f"{n}: rel grad err {rel}"
    print(f"headline-shape parity: loss {loss.item():.5f} vs {loss_ref.item():.5f}, worst rel grad err {worst:.4f}")


def _curve(engine, steps, data, seed=0):
    m = _gpt2(C=384, L=6, H=6, P=256, seed=seed).cuda()
    runner = _make_runner(m, engine, torch.device("cuda"), False)
    m.train()
    losses = []
    for i in range(steps):
        x, y = data[i % len(data)]
        runner.zero_grad()
        losses.append(float(runner.micro_step(x, y, 1.0, True, True, False)))
        runner.step()
    _ext.FORCE_TORCH = False
    return losses


def test_loss_curve_matches_reference_engine_over_100_steps():
    g = torch.Generator(device="cuda").manual_seed(2)
    base = torch.randint(0, 2000, (4, 257), device="cuda", generator=g)  # a small, learnable corpus
    data = [(base[:, :-1].contiguous(), base[:, 1:].contiguous())]
    fused = _curve("fused", 100, data)
    eager = _curve("reference", 100, data)
    assert fused[0] == pytest.approx(eager[0], abs=2e-2)
    assert fused[-1] < fused[0] - 3.0 and eager[-1] < eager[0] - 3.0  # both actually train
    for i in range(0, 100, 10):
        assert abs(fused[i] - eager[i]) < 0.05 * max(1.0, eager[i]) + 0.05, (i, fused[i], eager[i])
    assert abs(fused[-1] - eager[-1]) < 0.1 + 0.05 * eager[-1], (fused[-1], eager[-1])
    print("loss every 10 steps  fused:", [round(v, 3) for v in fused[::10]], " reference:", [round(v, 3) for v in eager[::10]])


@pytest.mark.parametrize("gemma", [False, True])
def test_grad_overwrite_matches_full_zeroing(monkeypatch, gemma):
    """zero_grad leaves the weight-gradient GEMMs' outputs alone after the first backward and
    their first write of the step overwrites (no clear, no read-back): gradients must equal those
    of clearing the whole buffer, over steps with gradient accumulation (2 micro-steps) and a
    chunked lm_head (several GEMMs into one gradient: the first overwrites, the rest add)."""
    monkeypatch.setenv("PENROZ_HEAD_CHUNK", "96")

    def run(overwrite: bool):
        monkeypatch.setenv("PENROZ_GRAD_OVERWRITE", "1" if overwrite else "0")
        torch.manual_seed(3)
        if gemma:
            from penroz.models.gemma_executor import GemmaExecutor
            layers = bench.gemma3_1b_layers(2)
            m = NeuralNetworkModel("g", Mapper(layers, {"adamw": {"lr": 1e-3}})).cuda()
            ex = GemmaExecutor(m, torch.device("cuda"))
            V = 262144
        else:
            m = _gpt2(V=1024, C=256, L=2, H=4, P=256, seed=3).cuda()
            ex = GPTExecutor(m, torch.device("cuda"))
            V = 1024
        ex.setup_training(False)
        g = torch.Generator(device="cuda").manual_seed(5)
        grads = []
        for step in range(3):
            ex.zero_grad()
            for micro in range(2):
                x = torch.randint(0, V, (2, 128), device="cuda", generator=g)
                ex.train_micro_step(x, torch.roll(x, -1, 1), 0.5, sync=micro == 1)
            torch.cuda.synchronize()
            grads.append(ex.flat_grad.clone())
            ex.optimizer_step()
        if overwrite:
            assert getattr(ex, "_zero_gaps", None) is not None, "overwrite mode never engaged"
        return grads

    # (the embedding backward's atomics make two runs differ in the last bits, so after the first
    # optimizer step everything differs slightly: compare with a tight relative tolerance — a range
    # left uncleared or accumulated onto stale values is off by O(1))
    for a, b in zip(run(True), run(False)):
        assert torch.isfinite(a).all()
        rel = ((a - b).norm() / b.norm()).item()
        assert rel < 1e-4, rel
