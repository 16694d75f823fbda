"""Fused GPT executor vs a pure-PyTorch fp32 reference of the same model (MI355X)."""
import copy
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from penroz.models.mapper import Mapper
from penroz.models.model import NeuralNetworkModel
from penroz.models.executor import GPTExecutor
from penroz.ops import _ext
import bench


def tiny(V=512, C=256, L=2, H=4, P=256, gelu=None):
    layers = bench.gpt2_layers(V=V, C=C, L=L, H=H, P=P)
    if gelu:
        for blk in layers[2:2 + L]:
            blk["residual"][1]["sequential"][2] = {"gelu": {"approximate": gelu}}
    return NeuralNetworkModel("t", Mapper(layers, {"adamw": {"lr": 1e-3, "betas": [0.9, 0.95]}}))


@pytest.mark.parametrize("gelu", [None, "tanh"])
def test_executor_matches_fp32_reference(gelu):
    torch.manual_seed(0)
    m = tiny(gelu=gelu).cuda()
    ref = copy.deepcopy(m)
    assert GPTExecutor.match(m) is not None
    B, T = 4, 128
    x = torch.randint(0, 512, (B, T), device="cuda")
    y = torch.randint(0, 512, (B, T), device="cuda")
    _ext.FORCE_TORCH = True
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
    for (n, p), (_, r) in zip(m.named_parameters(), ref.named_parameters()):
        rel = (p.grad - r.grad).norm() / (r.grad.norm() + 1e-12)
        assert rel < 5e-2, f"{n}: rel grad err {rel}"


def test_executor_trains_and_keeps_state_dict_keys():
    torch.manual_seed(0)
    m = tiny().cuda()
    keys = list(m.state_dict().keys())
    ex = GPTExecutor(m, torch.device("cuda"))
    ex.setup_training(False)
    x = torch.randint(0, 512, (8, 64), device="cuda")
    y = torch.roll(x, -1, 1)
    losses = []
    for _ in range(30):
        ex.zero_grad()
        losses.append(ex.train_micro_step(x, y, 1.0).item())
        ex.optimizer_step()
    assert losses[-1] < losses[0] - 1.0, losses
    assert list(m.state_dict().keys()) == keys
    # module forward (generic path) agrees with executor eval on the updated weights
    with torch.no_grad():
        _, c_mod = m(x, y, skip_softmax=True)
        c_ex = ex.eval_loss(x, y)
    assert abs(c_mod.item() - c_ex.item()) < 5e-2
    # optimizer state is torch-AdamW-shaped and serialisable
    sd = m.optimizer.state_dict()
    assert {"step", "exp_avg", "exp_avg_sq"} <= set(sd["state"][0].keys())


def _hf_gpt2(C=256, L=2, H=4, V=512, P=256, pdrop=0.1):
    """The /import/ layout of an HF GPT-2 (tanh GELU, dropouts from the config), random init."""
    from types import SimpleNamespace
    cfg = SimpleNamespace(vocab_size=V, n_embd=C, n_head=H, n_layer=L, n_positions=P,
                          activation_function="gelu_new", resid_pdrop=pdrop, embd_pdrop=pdrop, attn_pdrop=pdrop,
                          model_type="gpt2")
    torch.manual_seed(0)
    m = NeuralNetworkModel("hf", Mapper(Mapper.from_hf_config(cfg), {"adamw": {"lr": 1e-3, "betas": [0.9, 0.95]}}))
    for mod in m.modules():
        if isinstance(mod, (torch.nn.Linear, torch.nn.Embedding)):
            torch.nn.init.normal_(mod.weight, 0.0, 0.02)
    return m


def test_executor_accepts_hf_import_layout_bf16_with_dropout():
    """The reference's import -> train flow: bf16 params (neural_net_model.py:222), dropout 0.1
    (mappers.py:140-142). The executor must take it (fp32 masters internally) and train."""
    m = _hf_gpt2().cuda().to(dtype=torch.bfloat16)
    spec = GPTExecutor.match(m)
    assert spec is not None and spec.param_dtype == torch.bfloat16 and spec.p_embd == 0.1
    assert all(b.p_attn_res == 0.1 and b.p_mlp_res == 0.1 for b in spec.blocks)
    keys = {k: v.dtype for k, v in m.state_dict().items()}
    ex = GPTExecutor(m, torch.device("cuda"))
    ex.setup_training(False)
    x = torch.randint(0, 512, (8, 64), device="cuda")
    y = torch.roll(x, -1, 1)
    m.train()
    losses = []
    for _ in range(40):
        ex.zero_grad()
        losses.append(ex.train_micro_step(x, y, 1.0).item())
        ex.optimizer_step()
    assert all(math.isfinite(v) for v in losses)
    assert losses[-1] < losses[0] - 1.0, losses
    # state dict keeps keys AND bf16 dtype (the checkpoint format of an imported model) and the
    # module weights follow the optimizer (views of the bf16 shadow)
    assert {k: v.dtype for k, v in m.state_dict().items()} == keys
    w = m.layers[2][0][1].weight
    assert w.dtype == torch.bfloat16 and torch.equal(w.float(), ex.f32(w).to(torch.bfloat16).float())
    assert ex.grad(w).abs().sum() > 0


def test_executor_hf_vocab_not_multiple_of_8_matches_reference():
    """HF GPT-2's V = 50257 (here 509): padded logits rows; loss/grads vs fp32 eager (no dropout)."""
    torch.manual_seed(0)
    m = _hf_gpt2(V=509, pdrop=0.0).cuda()
    ref = copy.deepcopy(m)
    x = torch.randint(0, 509, (4, 128), device="cuda")
    y = torch.randint(0, 509, (4, 128), device="cuda")
    _ext.FORCE_TORCH = True
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
    for (n, p), (_, r) in zip(m.named_parameters(), ref.named_parameters()):
        rel = (ex.grad(p) - r.grad).norm() / (r.grad.norm() + 1e-12)
        assert rel < 5e-2, f"{n}: rel grad err {rel}"


def test_executor_dropout_masks_are_consistent_between_fwd_and_bwd():
    """Directional derivative check with dropout active: with the masks fixed by the step seed,
    (L(θ+εv) - L(θ-εv)) / 2ε must match <∇L, v> from the executor's backward."""
    m = _hf_gpt2(pdrop=0.2).cuda()
    ex = GPTExecutor(m, torch.device("cuda"))
    ex.setup_training(False)
    x = torch.randint(0, 512, (4, 64), device="cuda")
    y = torch.roll(x, -1, 1)
    seed0 = ex._step_seed
    ex.zero_grad()
    loss = ex.train_micro_step(x, y, 1.0)
    g = ex.flat_grad.clone()
    gen = torch.Generator(device="cuda").manual_seed(5)
    v = torch.randn(ex.flat.numel(), device="cuda", generator=gen)
    v /= v.norm()
    base = ex.flat.clone()
    eps = 0.05

    def loss_at(delta):
        ex.flat.copy_(base + delta)
        ex.refresh_shadow()
        ex._step_seed = seed0  # same masks
        ex.zero_grad()
        return ex.train_micro_step(x, y, 1.0).item()

    fd = (loss_at(eps * v) - loss_at(-eps * v)) / (2 * eps)
    an = float((g * v).sum())
    ex.flat.copy_(base)
    ex.refresh_shadow()
    assert math.isfinite(loss.item())
    assert abs(fd - an) <= 0.1 * abs(an) + 2e-3, (fd, an)
    # and the masks matter: a different seed gives a different loss
    ex._step_seed = seed0 + 1000
    ex.zero_grad()
    assert abs(ex.train_micro_step(x, y, 1.0).item() - loss.item()) > 1e-4


@pytest.mark.parametrize("V", [512, 509])
def test_executor_chunked_head_matches_one_chunk(monkeypatch, V):
    """Token-chunked lm_head/CE (PENROZ_HEAD_CHUNK rows, two rotating buffers, wgrad per chunk
    on the side stream) gives the loss and gradients of the single-chunk head."""
    torch.manual_seed(0)
    m = tiny(V=V).cuda()
    m2 = copy.deepcopy(m)
    B, T = 4, 128
    x = torch.randint(0, V, (B, T), device="cuda")
    y = torch.randint(0, V, (B, T), device="cuda")
    out = []
    for model, chunk in ((m, "0"), (m2, "96")):  # 96 does not divide 512: a ragged last chunk
        monkeypatch.setenv("PENROZ_HEAD_CHUNK", chunk)
        ex = GPTExecutor(model, torch.device("cuda"))
        ex.setup_training(False)
        ex.zero_grad()
        loss = ex.train_micro_step(x, y, 1.0)
        ev = ex.eval_loss(x, y)
        torch.cuda.synchronize()
        assert len(ex._head_bufs) == (1 if chunk == "0" else 2)
        out.append((loss.item(), ev.item(), ex.flat_grad.clone()))
    (l1, e1, g1), (l2, e2, g2) = out
    assert abs(l1 - l2) < 1e-4 and abs(e1 - e2) < 1e-4, (l1, l2, e1, e2)
    rel = (g1 - g2).norm() / g1.norm()
    assert rel < 1e-3, rel


def test_transposed_dgrad_weights_follow_the_main_stream():
    """The side-stream transposes of the bf16 shadow (dgrad operands) are ordered after every
    shadow write queued on the main stream (regression: the side stream once waited on itself,
    so the copies could be taken from a half-refreshed shadow)."""
    torch.manual_seed(0)
    m = tiny().cuda()
    ex = GPTExecutor(m, torch.device("cuda"))
    ex.setup_training(False)
    assert ex._tw, "transposed dgrad weights expected on the GPU"
    torch.cuda.synchronize()
    torch.cuda._sleep(200_000_000)  # keep the main stream busy, then rewrite the shadow behind it
    ex.shadow.mul_(2.0)
    ex._refresh_transposed()
    torch.cuda.synchronize()
    for w, t in ex._tw.values():
        assert torch.equal(t, ex.bf16(w).t()), "transpose ran before the main stream's shadow write"


def test_executors_share_one_high_priority_stream(monkeypatch):
    """Every executor of the process runs its critical path on ONE high-priority stream per
    device: a second stream from torch's high-priority pool lost the queue priority and slowed the
    second model's step by ≈4 ms (bench/runtime_ab.py)."""
    from penroz.models import executor as ex_mod
    dev = torch.device("cuda", torch.cuda.current_device())
    a = ex_mod._high_priority_stream(dev)
    b = ex_mod._high_priority_stream(torch.device("cuda"))
    assert a is b
    lo, hi = torch.cuda.Stream.priority_range()
    assert a.priority == min(lo, hi)
    monkeypatch.setenv("PENROZ_MAIN_PRIORITY", "1")  # (GPT's default runs without it since round 6)
    m1, m2 = tiny().cuda(), tiny().cuda()
    e1, e2 = GPTExecutor(m1, torch.device("cuda")), GPTExecutor(m2, torch.device("cuda"))
    s1, s2 = e1._main_stream(), e2._main_stream()
    assert s1 is s2 is a
    assert e1._side is e2._side  # one side stream per device and process too
