"""GPT pattern lowering (CPU): which layer lists the fused executor accepts."""
import copy

import pytest

import bench
from penroz.models.executor import GPTExecutor
from penroz.models.mapper import Mapper
from penroz.models.model import NeuralNetworkModel


def _model(layers):
    return NeuralNetworkModel("x", Mapper(layers, {"adamw": {"lr": 1e-3}}))


def test_reference_example_layout_matches():
    spec = GPTExecutor.match(_model(bench.gpt2_layers(V=128, C=128, L=2, H=2, P=64)))
    assert spec is not None and (spec.C, spec.H, spec.D, spec.F, spec.V, spec.P) == (128, 2, 64, 512, 128, 64)
    assert len(spec.blocks) == 2 and spec.gelu_approx == "none"


def test_hf_style_layouts():
    from transformers import GPT2Config
    from penroz.models import hf
    cfg = GPT2Config(vocab_size=128, n_positions=64, n_embd=128, n_layer=1, n_head=2)
    spec = GPTExecutor.match(_model(hf.gpt2_layers(cfg)))  # HF default dropout 0.1: fused kernels
    assert spec is not None and spec.p_embd == 0.1 and spec.blocks[0].p_attn_res == spec.blocks[0].p_mlp_res == 0.1
    bf = _model(hf.gpt2_layers(cfg)).to(dtype=__import__("torch").bfloat16)  # /import/ loads bf16 weights
    assert GPTExecutor.match(bf).param_dtype == __import__("torch").bfloat16
    assert GPTExecutor.match(bf, require_fp32=True) is None
    cfg = GPT2Config(vocab_size=128, n_positions=64, n_embd=128, n_layer=1, n_head=2, resid_pdrop=0.0,
                     embd_pdrop=0.0, attn_pdrop=0.1)
    spec = GPTExecutor.match(_model(hf.gpt2_layers(cfg)))
    assert spec is not None and spec.gelu_approx == "tanh"  # attention dropout runs in the flash kernel


def test_non_matching_layouts():
    base = bench.gpt2_layers(V=128, C=128, L=1, H=2, P=64)
    rope = copy.deepcopy(base)
    rope[2]["residual"][0]["sequential"][2]["attention"]["rope_theta"] = 10000.0
    assert GPTExecutor.match(_model(rope)) is None
    odd_head = copy.deepcopy(base)
    odd_head[2]["residual"][0]["sequential"][2]["attention"]["num_heads"] = 4  # D = 32
    assert GPTExecutor.match(_model(odd_head)) is None
    mlp = [{"linear": {"in_features": 4, "out_features": 4}}, {"relu": {}}, {"linear": {"in_features": 4, "out_features": 2}}]
    assert GPTExecutor.match(_model(mlp)) is None


def test_head_chunk_policy(monkeypatch):
    from penroz.models.executor import _head_chunk_rows
    monkeypatch.delenv("PENROZ_HEAD_CHUNK", raising=False)
    assert _head_chunk_rows(65536, 50304) == 65536          # 6.6 GB of logits: one chunk
    c = _head_chunk_rows(4 * 65536, 50304)                   # 26 GB: ~2 GiB chunks
    assert c % 1024 == 0 and 1024 <= c < 4 * 65536 and c * 50304 * 2 <= 2 * 2**30
    monkeypatch.setenv("PENROZ_HEAD_CHUNK", "8192")
    assert _head_chunk_rows(65536, 50304) == 8192
    monkeypatch.setenv("PENROZ_HEAD_CHUNK", "0")
    assert _head_chunk_rows(4 * 65536, 50304) == 4 * 65536


def test_gemma_executor_pattern_match_modes():
    """The fused Gemma executor's pattern match (CPU): Gemma 3 / 2 / 1 layer lists map to the
    combine modes 0 / 1 / 2; a tied head or a GPT layer list does not match."""
    from types import SimpleNamespace
    from penroz.models.gemma_executor import GemmaExecutor
    from penroz.models.mapper import Mapper
    from penroz.models.model import NeuralNetworkModel
    for mt, mode in (("gemma3_text", 0), ("gemma2", 1), ("gemma", 2)):
        cfg = SimpleNamespace(model_type=mt, vocab_size=64, hidden_size=64, intermediate_size=128, num_hidden_layers=2,
                              num_attention_heads=2, num_key_value_heads=1, head_dim=64, rms_norm_eps=1e-6,
                              rope_theta=10000.0, attention_dropout=0.0, hidden_activation="gelu_pytorch_tanh")
        m = NeuralNetworkModel("g", Mapper(Mapper.from_hf_config(cfg), {"adamw": {"lr": 1e-3}}))
        spec = GemmaExecutor.match(m)
        assert spec is not None and spec.mode == mode and spec.F == 128 and spec.act == 1
        m.layers[-2].weight = m.layers[0].weight  # tied head: not lowered
        assert GemmaExecutor.match(m) is None
    import bench
    g = NeuralNetworkModel("t", Mapper(bench.gpt2_layers(V=64, C=64, L=1, H=1, P=32), {"adamw": {"lr": 1e-3}}))
    assert GemmaExecutor.match(g) is None


def test_gemma_executor_matches_heterogeneous_gemma4_layer_list():
    """Gemma 4 layer lists (reference mappers.py:206-233) lower to the fused executor with
    per-block shapes: global_head_dim / KV heads on full-attention layers, double-wide MLPs on
    KV-shared layers; C up to 6144 (Gemma-3 27B: 5376)."""
    from types import SimpleNamespace
    from penroz.models.gemma_executor import GemmaExecutor
    from penroz.models.mapper import Mapper
    from penroz.models.model import NeuralNetworkModel
    cfg = SimpleNamespace(model_type="gemma4", vocab_size=64, hidden_size=64, intermediate_size=128,
                          num_hidden_layers=4, num_attention_heads=2, num_key_value_heads=2, head_dim=64,
                          rms_norm_eps=1e-6, rope_theta=10000.0, attention_dropout=0.0,
                          hidden_activation="gelu_pytorch_tanh",
                          layer_types=["sliding_attention", "full_attention"] * 2, global_head_dim=128,
                          num_global_key_value_heads=1, num_kv_shared_layers=2, use_double_wide_mlp=True)
    m = NeuralNetworkModel("g4", Mapper(Mapper.from_hf_config(cfg), {"adamw": {"lr": 1e-3}}))
    spec = GemmaExecutor.match(m)
    assert spec is not None and not spec.uniform
    assert [(b.H, b.Hkv, b.D, b.F) for b in spec.blocks] == [(2, 2, 64, 128), (2, 1, 128, 128), (2, 2, 64, 256),
                                                            (2, 1, 128, 256)]
    wide = SimpleNamespace(**{**vars(cfg), "hidden_size": 5376, "num_hidden_layers": 1, "layer_types": None,
                              "intermediate_size": 64, "vocab_size": 16})
    assert GemmaExecutor.match(NeuralNetworkModel("w", Mapper(Mapper.from_hf_config(wide), {"adamw": {}}))) is not None


def _range_exec(monkeypatch):
    """A bare executor with only the weight-gradient bookkeeping live: flat fp32 buffer, wgrad
    done eagerly on the CPU (g = dyᵀ·x or g += dyᵀ·x), no side stream."""
    import types
    import torch
    from penroz.models import executor as E
    ex = object.__new__(GPTExecutor)
    ex.flat_grad = torch.zeros(64)
    ex.device = types.SimpleNamespace(type="cuda", index=0)  # range learning is a GPU-path feature
    ex._side = None
    ex.wait_gradients = lambda: None

    def wgrad(dy, x, g, acc):
        r = dy.t() @ x
        if acc:
            g.add_(r)
        else:
            g.copy_(r)
    monkeypatch.setattr(E.gemm_ops, "wgrad", wgrad)
    return ex


def test_wgrad_ranges_chunked_after_learning(monkeypatch):
    """after the ranges are learned, a key that writes sub-ranges (chunked wgrad) must
    never accumulate onto last step's data — whether its first chunk is a sub-range, the whole
    learned range, or some parts are never written."""
    import torch
    ex = _range_exec(monkeypatch)
    torch.manual_seed(0)
    A = ex.flat_grad[0:32].view(8, 4)    # weight A's gradient
    Bg = ex.flat_grad[40:56].view(4, 4)  # weight B's gradient; [32:40) and [56:64) are other grads
    dyA, xA = torch.randn(5, 8), torch.randn(5, 4)
    dyB, xB = torch.randn(5, 4), torch.randn(5, 4)
    # learning step: whole-range writes
    ex.zero_grad()
    ex._wgrad_into(1, dyA, xA, A)
    ex._wgrad_into(2, dyB, xB, Bg)
    ex._finish_wgrad_bookkeeping()
    assert ex._zero_gaps == [(0 + 32, 40), (56, 64)]
    assert torch.allclose(A, dyA.t() @ xA)

    def step(writes_a, learned_ranges_skipped=False):
        ex.flat_grad.fill_(123.0)  # last step's values everywhere
        ex.zero_grad()
        assert torch.all(ex.flat_grad[32:40] == 0)
        if learned_ranges_skipped:
            assert torch.all(ex.flat_grad[40:56] == 123.0) and torch.all(ex.flat_grad[0:32] == 123.0)
        for r0, r1, dy, x in writes_a:
            ex._wgrad_into(1, dy[:, r0:r1], x, A[r0:r1])
        ex._wgrad_into(2, dyB, xB, Bg)
        ex._finish_wgrad_bookkeeping()
        assert torch.allclose(Bg, dyB.t() @ xB)

    d1, d2 = torch.randn(5, 8), torch.randn(5, 8)
    # sub-ranges first, one range accumulated twice (two token chunks), the rest once
    step([(0, 4, d1, xA), (0, 4, d2, xA), (4, 8, d1, xA)], learned_ranges_skipped=True)
    want = torch.cat([(d1[:, :4] + d2[:, :4]).t() @ xA, d1[:, 4:].t() @ xA])
    assert torch.allclose(A, want, atol=1e-5)
    # the whole learned range first (overwrite), then a sub-range accumulates onto it; with the
    # pattern changed zero_grad now clears everything, so re-arm the skip to test the stale path
    assert ex._zero_gaps is None
    ex._zero_gaps = [(32, 40), (56, 64)]
    step([(0, 8, d1, xA), (2, 6, d2, xA)], learned_ranges_skipped=True)
    want = d1.t() @ xA
    want[2:6] += d2[:, 2:6].t() @ xA
    assert torch.allclose(A, want, atol=1e-5)
    # a part never written this step ends up zero, not stale
    ex._zero_gaps = [(32, 40), (56, 64)]
    step([(0, 3, d1, xA)], learned_ranges_skipped=True)
    assert torch.allclose(A[0:3], d1[:, :3].t() @ xA, atol=1e-5) and torch.all(A[3:] == 0)
    # the changed pattern makes zero_grad clear everything from now on
    assert ex._wgrad_ranges_invalid and ex._zero_gaps is None


def test_side_stream_cu_mask_words():
    from penroz.models.executor import cu_mask_words
    w = cu_mask_words("stride:4", 256)
    assert len(w) == 8 and all(x == 0x11111111 for x in w)
    w = cu_mask_words("stride:8:1", 256)
    assert all(x == 0x02020202 for x in w)
    assert cu_mask_words("first:40", 256)[:2] == [0xFFFFFFFF, 0xFF] and cu_mask_words("first:40", 256)[2:] == [0] * 6
    with pytest.raises(ValueError):
        cu_mask_words("half", 256)


def test_zero_gap_minus_skip_range():
    from penroz.models.executor import _minus
    assert _minus([(0, 10), (20, 30)], None) == [(0, 10), (20, 30)]
    assert _minus([(0, 10), (20, 30)], (5, 25)) == [(0, 5), (25, 30)]
    assert _minus([(0, 10)], (0, 10)) == []
    assert _minus([(0, 100)], (40, 60)) == [(0, 40), (60, 100)]
    assert _minus([(10, 20)], (30, 40)) == [(10, 20)]
