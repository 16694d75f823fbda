"""Fused Gemma executor (models/gemma_executor.py) vs the module path (MI355X).

* pattern match for the Gemma 3 / Gemma 2 / Gemma 1 layer lists of ``Mapper.from_hf_config``
  (post-norm on the residual / on the branch / none: combine modes 0 / 1 / 2);
* one fp32 step against the same model run as plain fp32 PyTorch ops (``FORCE_TORCH``: the fp32
  reference of every kernel), loss and every parameter gradient, per mode;
* the combine kernels against autograd of their fp32 definitions;
* 100 AdamW steps from one initialisation against the generic engine (module forward over the
  HIP layers + autograd): the loss curves agree;
* bf16 parameters (what ``/import/`` produces) train with fp32 masters and keep the state_dict.
"""
import copy
from types import SimpleNamespace

import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from penroz.models.gemma_executor import GemmaExecutor
from penroz.models.mapper import Mapper
from penroz.models.model import NeuralNetworkModel, _make_runner
from penroz.ops import _ext

DEV = "cuda"


def _gemma(model_type="gemma3_text", V=512, C=256, L=2, H=4, Hkv=2, D=64, F=512, seed=0, act="gelu_pytorch_tanh",
           **extra):
    torch.manual_seed(seed)
    cfg = SimpleNamespace(model_type=model_type, vocab_size=V, hidden_size=C, intermediate_size=F, num_hidden_layers=L,
                          num_attention_heads=H, num_key_value_heads=Hkv, head_dim=D, rms_norm_eps=1e-6,
                          rope_theta=10000.0, rope_local_base_freq=10000.0, attention_dropout=0.0,
                          hidden_activation=act, query_pre_attn_scalar=D, sliding_window=512, **extra)
    m = NeuralNetworkModel("g", Mapper(Mapper.from_hf_config(cfg), {"adamw": {"lr": 1e-3, "betas": [0.9, 0.95]}}))
    with torch.no_grad():  # non-trivial norm weights, so every dγ path carries signal
        for n, p in m.named_parameters():
            if p.dim() == 1:
                p.add_(torch.randn_like(p) * 0.2)
            else:
                p.normal_(0.0, 0.05)
    return m


@pytest.mark.parametrize("model_type,mode", [("gemma3_text", 0), ("gemma2", 1), ("gemma", 2)])
def test_match_modes(model_type, mode):
    spec = GemmaExecutor.match(_gemma(model_type))
    assert spec is not None and spec.mode == mode and (spec.H, spec.Hkv, spec.D, spec.F) == (4, 2, 64, 512)


@pytest.mark.parametrize("model_type", ["gemma3_text", "gemma2", "gemma"])
def test_one_step_matches_fp32_reference(model_type):
    m = _gemma(model_type).to(DEV)
    ref = copy.deepcopy(m)
    B, T = 4, 128
    g = torch.Generator(device=DEV).manual_seed(1)
    x = torch.randint(0, 512, (B, T), device=DEV, generator=g)
    y = torch.randint(0, 512, (B, T), device=DEV, generator=g)
    _ext.FORCE_TORCH = True
    try:
        _, loss_ref = ref(x, y, skip_softmax=True)
        loss_ref.backward()
    finally:
        _ext.FORCE_TORCH = False
    ex = GemmaExecutor(m, torch.device(DEV))
    ex.setup_training(False)
    ex.zero_grad()
    loss = ex.train_micro_step(x, y, 1.0)
    assert abs(loss.item() - loss_ref.item()) < 2e-2, (loss.item(), loss_ref.item())
    worst = 0.0
    for (n, p), (_, r) in zip(m.named_parameters(), ref.named_parameters()):
        rel = ((ex.grad(p) - r.grad).norm() / (r.grad.norm() + 1e-12)).item()
        worst = max(worst, rel)
        assert rel < 5e-2, f"{model_type} {n}: rel grad err {rel}"
    print(f"{model_type}: loss {loss.item():.5f} vs {loss_ref.item():.5f}, worst rel grad err {worst:.4f}")


# Gemma-4-like heterogeneous layer list (reference mappers.py:206-233): alternating sliding / full
# attention, the full layers with global_head_dim and their own KV-head count, the last two layers
# KV-shared with double-wide MLPs
GEMMA4 = dict(layer_types=["sliding_attention", "full_attention", "sliding_attention", "full_attention"],
              global_head_dim=512, num_global_key_value_heads=1, num_kv_shared_layers=2, use_double_wide_mlp=True)


def test_match_heterogeneous_gemma4_layer_list():
    spec = GemmaExecutor.match(_gemma("gemma4", L=4, F=256, **GEMMA4))
    assert spec is not None and not spec.uniform and spec.mode == 0
    assert [(b.H, b.Hkv, b.D, b.F) for b in spec.blocks] == [(4, 2, 64, 256), (4, 1, 512, 256), (4, 2, 64, 512),
                                                            (4, 1, 512, 512)]


def test_heterogeneous_gemma4_one_step_matches_fp32_reference():
    m = _gemma("gemma4", L=4, F=256, **GEMMA4).to(DEV)
    ref = copy.deepcopy(m)
    B, T = 2, 128
    g = torch.Generator(device=DEV).manual_seed(3)
    x = torch.randint(0, 512, (B, T), device=DEV, generator=g)
    y = torch.randint(0, 512, (B, T), device=DEV, generator=g)
    _ext.FORCE_TORCH = True
    try:
        _, loss_ref = ref(x, y, skip_softmax=True)
        loss_ref.backward()
    finally:
        _ext.FORCE_TORCH = False
    ex = GemmaExecutor(m, torch.device(DEV))
    ex.setup_training(False)
    ex.zero_grad()
    loss = ex.train_micro_step(x, y, 1.0)
    assert abs(loss.item() - loss_ref.item()) < 2e-2, (loss.item(), loss_ref.item())
    for (n, p), (_, r) in zip(m.named_parameters(), ref.named_parameters()):
        rel = ((ex.grad(p) - r.grad).norm() / (r.grad.norm() + 1e-12)).item()
        assert rel < 5e-2, f"gemma4 {n}: rel grad err {rel}"


def test_no_sdpa_for_gemma4_head_dims(monkeypatch):
    """Every head dim of the Gemma-4 layer list (64 sliding, 512 full) runs a native flash kernel:
    torch SDPA is never called in the fused step (nor in the generic engine's forward/backward)."""
    import torch.nn.functional as Fn
    calls = []
    real = Fn.scaled_dot_product_attention
    monkeypatch.setattr(Fn, "scaled_dot_product_attention", lambda *a, **k: calls.append(1) or real(*a, **k))
    m = _gemma("gemma4", L=4, F=256, **GEMMA4).to(DEV)
    x = torch.randint(0, 512, (2, 64), device=DEV)
    ex = GemmaExecutor(m, torch.device(DEV))
    ex.setup_training(False)
    ex.zero_grad()
    ex.train_micro_step(x, torch.roll(x, -1, 1), 1.0)
    _, c = m(x, torch.roll(x, -1, 1), skip_softmax=True)
    c.backward()
    torch.cuda.synchronize()
    assert not calls


def test_heterogeneous_gemma4_loss_curve_matches_generic_engine():
    g = torch.Generator(device=DEV).manual_seed(4)
    base = torch.randint(0, 400, (2, 129), device=DEV, generator=g)
    data = [(base[:, :-1].contiguous(), base[:, 1:].contiguous())]
    curves = {}
    for engine in ("fused", "generic"):
        m = _gemma("gemma4", L=4, F=256, seed=1, **GEMMA4).to(DEV)
        runner = _make_runner(m, engine, torch.device(DEV), False)
        if engine == "fused":
            assert isinstance(runner.exec, GemmaExecutor)
        m.train()
        losses = []
        for i in range(100):
            x, y = data[0]
            runner.zero_grad()
            losses.append(float(runner.micro_step(x, y, 1.0, True, True, False)))
            runner.step()
        curves[engine] = losses
    fused, generic = curves["fused"], curves["generic"]
    assert fused[-1] < fused[0] - 2.0 and generic[-1] < generic[0] - 2.0
    for i in range(0, 100, 10):
        assert abs(fused[i] - generic[i]) < 0.05 * max(1.0, generic[i]) + 0.05, (i, fused[i], generic[i])


def _rms(v, w, eps):
    return v * torch.rsqrt(v.pow(2).mean(-1, keepdim=True) + eps) * w


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
@pytest.mark.parametrize("C", [256, 1152, 100 * 4])
def test_combine_kernels_match_autograd(mode, C):
    torch.manual_seed(mode + C)
    N = 300
    k = _ext.kernels()
    x = torch.randn(N, C, device=DEV, requires_grad=True)
    a = torch.randn(N, C, device=DEV).to(torch.bfloat16).float().requires_grad_()
    w1 = (1 + 0.3 * torch.randn(C, device=DEV)).requires_grad_()
    w2 = (1 + 0.3 * torch.randn(C, device=DEV)).requires_grad_()
    e1, e2 = 1e-6, 1e-5
    if mode == 0:
        h = _rms(x + a, w1, e1)
    elif mode == 1:
        h = x + _rms(a, w1, e1)
    elif mode == 2:
        h = x + a
    else:
        h = x
    yv = _rms(h, w2, e2)
    h_out = torch.empty(N, C, device=DEV)
    y_out = torch.empty(N, C, device=DEV, dtype=torch.bfloat16)
    s_save = torch.empty(N, C, device=DEV)
    r1, r2 = torch.empty(N, device=DEV), torch.empty(N, device=DEV)
    ab = a.detach().to(torch.bfloat16)
    k.gemma_combine_fwd(mode, x.detach(), ab if mode != 3 else None, w1.detach() if mode < 2 else None, w2.detach(),
                        e1, e2, h_out if mode != 3 else None, y_out, s_save if mode == 0 else None,
                        r1 if mode < 2 else None, r2)
    if mode != 3:
        assert (h_out - h).abs().max().item() < 1e-4
    assert ((y_out.float() - yv).abs().max() / yv.abs().max()).item() < 1e-2
    # backward: dy (bf16) into y, dh_in into h (not for mode 3's h = x, which is the input)
    dy = torch.randn(N, C, device=DEV).to(torch.bfloat16)
    dh_in = torch.randn(N, C, device=DEV) if mode != 3 else None
    loss = (yv * dy.float()).sum() + ((h * dh_in).sum() if dh_in is not None else 0.0)
    loss.backward()
    dx = torch.empty(N, C, device=DEV)
    da = torch.empty(N, C, device=DEV, dtype=torch.bfloat16)
    dw1, dw2 = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    k.gemma_combine_bwd(mode, dy, dh_in, h_out if mode != 3 else x.detach(), s_save if mode == 0 else None,
                        ab if mode == 1 else None, r1 if mode < 2 else None, r2, w1.detach() if mode < 2 else None,
                        w2.detach(), dx, da if mode != 3 else None, dw1 if mode < 2 else None, dw2)

    def rel(p, r):
        return ((p.float() - r).norm() / (r.norm() + 1e-12)).item()

    assert rel(dx, x.grad) < 1e-4, rel(dx, x.grad)
    if mode != 3:
        assert rel(da, a.grad) < 1e-2, rel(da, a.grad)
    assert rel(dw2, w2.grad) < 1e-4
    if mode < 2:
        assert rel(dw1, w1.grad) < 1e-4


@pytest.mark.parametrize("N,F", [(77, 512), (1100, 6912)])  # the second: several grid trips, unrolled
def test_gated_bwd_packed_matches_unpacked(N, F):
    torch.manual_seed(0)
    k = _ext.kernels()
    gu = torch.randn(N, 2 * F, device=DEV).to(torch.bfloat16)
    dy = torch.randn(N, F, device=DEV).to(torch.bfloat16)
    for kind in (0, 1, 2):
        dg, du = k.gated_act_bwd(dy, gu[:, :F].contiguous(), gu[:, F:].contiguous(), kind)
        dgu = torch.empty_like(gu)
        k.gated_act_bwd_packed(dy, gu, dgu, kind)
        assert torch.equal(dgu[:, :F], dg) and torch.equal(dgu[:, F:], du)
        y = torch.empty(N, F, device=DEV, dtype=torch.bfloat16)
        k.gated_act_packed(gu, kind, y)
        assert torch.equal(y, k.gated_act_packed(gu, kind))
        ref = k.gated_act_fwd(gu[:, :F].contiguous(), gu[:, F:].contiguous(), kind)
        assert torch.equal(y, ref)


def _curve(engine, steps, data, seed=0):
    m = _gemma("gemma3_text", C=256, L=3, seed=seed).to(DEV)
    runner = _make_runner(m, engine, torch.device(DEV), False)
    m.train()
    losses = []
    for i in range(steps):
        x, y = data[i % len(data)]
        runner.zero_grad()
        losses.append(float(runner.micro_step(x, y, 1.0, True, True, False)))
        runner.step()
    _ext.FORCE_TORCH = False
    return losses


def test_loss_curve_matches_generic_engine_over_100_steps():
    g = torch.Generator(device=DEV).manual_seed(2)
    base = torch.randint(0, 400, (4, 129), device=DEV, generator=g)
    data = [(base[:, :-1].contiguous(), base[:, 1:].contiguous())]
    fused = _curve("fused", 100, data)
    generic = _curve("generic", 100, data)
    assert fused[0] == pytest.approx(generic[0], abs=3e-2)
    assert fused[-1] < fused[0] - 2.0 and generic[-1] < generic[0] - 2.0  # both actually train
    for i in range(0, 100, 10):
        assert abs(fused[i] - generic[i]) < 0.05 * max(1.0, generic[i]) + 0.05, (i, fused[i], generic[i])
    print("loss every 10 steps  fused:", [round(v, 3) for v in fused[::10]],
          " generic:", [round(v, 3) for v in generic[::10]])


def test_bf16_params_train_and_keep_state_dict():
    m = _gemma("gemma3_text").to(DEV).to(torch.bfloat16)
    keys = list(m.state_dict().keys())
    assert m._engine(torch.device(DEV)) == "fused" and isinstance(m._get_executor(torch.device(DEV)), GemmaExecutor)
    ex = m._get_executor(torch.device(DEV))
    ex.setup_training(False)
    x = torch.randint(0, 512, (4, 64), device=DEV)
    y = torch.roll(x, -1, 1)
    losses = []
    for _ in range(20):
        ex.zero_grad()
        losses.append(ex.train_micro_step(x, y, 1.0).item())
        ex.optimizer_step()
    assert losses[-1] < losses[0] - 1.0, losses
    assert list(m.state_dict().keys()) == keys
    assert all(p.dtype == torch.bfloat16 for p in m.parameters())
    with torch.no_grad():
        _, c_mod = m(x, y, skip_softmax=True)
        c_ex = ex.eval_loss(x, y)
    assert abs(c_mod.item() - c_ex.item()) < 0.1, (c_mod.item(), c_ex.item())


def _train(m, steps, fuse, micro=1):
    from penroz.models.model import _FusedRunner
    runner = _FusedRunner(m, torch.device(DEV), False)
    g = torch.Generator(device=DEV).manual_seed(7)
    data = torch.randint(0, 512, (steps * micro, 2, 65), device=DEV, generator=g)
    losses = []
    for i in range(steps):
        runner.zero_grad()
        tot = 0.0
        for j in range(micro):
            b = data[i * micro + j]
            tot += float(runner.exec.train_micro_step(b[:, :-1].contiguous(), b[:, 1:].contiguous(), 1.0 / micro,
                                                      sync=j == micro - 1, fuse_optimizer=fuse and j == micro - 1))
        runner.step()
        losses.append(tot)
    return losses


@pytest.mark.parametrize("micro", [1, 2])
def test_optimizer_in_backward_matches_the_separate_step(micro):
    """The fused AdamW applied per segment inside the backward == the step after it (same
    kernel, same values; only the launch order differs), with and without grad accumulation.
    Bitwise except the embedding table, whose gradient is a scatter-add (atomic order)."""
    a, b = _gemma("gemma3_text", seed=3).to(DEV), _gemma("gemma3_text", seed=3).to(DEV)
    la, lb = _train(a, 3, False, micro), _train(b, 3, True, micro)
    assert la == pytest.approx(lb, abs=1e-5)
    for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
        if n == "layers.0.weight":
            assert torch.allclose(p, q, rtol=0, atol=1e-5), n
        else:
            assert torch.equal(p, q), n


@pytest.mark.parametrize("V,steps", [(512, 3), (16384, 8)])
def test_row_split_embedding_adamw_matches_dense(monkeypatch, V, steps):
    """The embedding table's AdamW split into untouched rows (during the forward, zero gradient)
    and touched rows (after the embedding backward, gradient cleared) == the dense fused step; the
    gradient buffer's table range stays zero between steps (zero_grad skips it). Rows no token
    touches (the training tokens are < 512) are BITWISE equal — only the scatter order of touched
    rows may differ; at V = 16384 the untouched-row update (side stream) runs while the forward
    is still executing."""
    from penroz.models.model import _FusedRunner
    a, b = _gemma("gemma3_text", V=V, seed=4).to(DEV), _gemma("gemma3_text", V=V, seed=4).to(DEV)
    monkeypatch.setenv("PENROZ_EMB_ROW_ADAM", "0")
    la = _train(a, steps, True)
    monkeypatch.setenv("PENROZ_EMB_ROW_ADAM", "1")
    lb = _train(b, steps, True)
    assert la == pytest.approx(lb, abs=1e-5)
    for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
        if n == "layers.0.weight":  # scatter-add order of the table gradient on the touched rows
            assert torch.equal(p[512:], q[512:]), "untouched rows must match bitwise"
            assert torch.allclose(p[:512], q[:512], rtol=0, atol=1e-5), n
        else:
            assert torch.equal(p, q), n
    if V != 512:
        return
    runner = _FusedRunner(b, torch.device(DEV), False)
    ex = runner.exec
    x = torch.randint(0, 512, (2, 64), device=DEV)
    runner.zero_grad()
    ex.train_micro_step(x, x, 1.0, fuse_optimizer=True)
    torch.cuda.synchronize()
    assert getattr(ex, "_zero_skip", None) is not None, "row-split path not taken"
    es, ee = ex._zero_skip
    assert ex.flat_grad[es:ee].abs().max().item() == 0.0


def test_capture_returns_activation_and_gradient_pairs():
    m = _gemma("gemma2").to(DEV)
    ex = GemmaExecutor(m, torch.device(DEV))
    ex.setup_training(False)
    x = torch.randint(0, 512, (2, 32), device=DEV)
    ex.zero_grad()
    ex.train_micro_step(x, torch.roll(x, -1, 1), 1.0, capture=True)
    algos, pairs = ex.captured()
    assert algos[0] == "scaledembedding" and algos.count("transformerblock") == 2
    assert len(pairs) == len(algos) - 1  # no pair for the softmax head
    for act, grad in pairs:
        assert act.shape[:2] == (2, 32) and act.shape == grad.shape
        assert torch.isfinite(act).all() and torch.isfinite(grad).all()


def test_new_session_after_segment_transposes_uses_fresh_weights(monkeypatch):
    """the transposed dgrad copies rebuilt after each segment's AdamW pass are marked
    fresh; a new session that rebuilds the shadow from other weights (loaded after training) must
    rebuild them too, or its first step's data gradients use the old weights. Gradients of the
    first step after the reload == an executor without transposed copies (PENROZ_DGRAD_T=0)."""
    from penroz.models.model import _FusedRunner
    monkeypatch.setenv("PENROZ_SEGMENT_TRANSPOSE", "1")  # (the default rebuilds at the step start)
    m = _gemma("gemma3_text", seed=6).to(DEV)
    _train(m, 2, True)
    ex = m._get_executor(torch.device(DEV))
    other = _gemma("gemma3_text", seed=7).to(DEV)
    with torch.no_grad():
        for p, q in zip(m.parameters(), other.parameters()):
            p.data.copy_(q.data)  # fp32 parameters are views of the executor's flat masters
    runner = _FusedRunner(m, torch.device(DEV), False)  # new session: shadow rebuilt from flat
    assert runner.exec is ex
    g = torch.Generator(device=DEV).manual_seed(8)
    x = torch.randint(0, 512, (2, 64), device=DEV, generator=g)
    y = torch.randint(0, 512, (2, 64), device=DEV, generator=g)
    ex.zero_grad()
    ex.train_micro_step(x, y, 1.0)
    monkeypatch.setenv("PENROZ_DGRAD_T", "0")
    ref = GemmaExecutor(other, torch.device(DEV))
    ref.setup_training(False)
    ref.zero_grad()
    ref.train_micro_step(x, y, 1.0)
    torch.cuda.synchronize()
    for (n, p), (_, q) in zip(m.named_parameters(), other.named_parameters()):
        a, b = ex.grad(p), ref.grad(q)
        rel = ((a - b).norm() / (b.norm() + 1e-12)).item()
        assert rel < 1e-2, f"{n}: rel grad err {rel}"
