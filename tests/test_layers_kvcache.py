"""Layer library and KV cache (CPU reference paths)."""
import importlib

import pytest
import torch
import torch.nn.functional as F

from penroz.models import layers as L
from penroz.models import kv_cache as KV
from penroz.models.mapper import Mapper
from penroz.models.model import NeuralNetworkModel


def test_attention_matches_sdpa_and_gqa():
    torch.manual_seed(0)
    B, T, H, Hkv, D = 2, 7, 4, 2, 8
    att = L.CausalSelfAttention(num_heads=H, num_kv_heads=Hkv)
    qkv = torch.randn(B, T, (H + 2 * Hkv) * D)
    out = att(qkv)
    q, k, v = qkv.split([H * D, Hkv * D, Hkv * D], dim=2)
    q = q.view(B, T, H, D).transpose(1, 2)
    k = k.view(B, T, Hkv, D).transpose(1, 2).repeat_interleave(2, 1)
    v = v.view(B, T, Hkv, D).transpose(1, 2).repeat_interleave(2, 1)
    ref = F.scaled_dot_product_attention(q, k, v, is_causal=True).transpose(1, 2).reshape(B, T, H * D)
    assert torch.allclose(out, ref, atol=1e-5)


def test_simple_layers():
    x = torch.randint(0, 10, (2, 5))
    pe = L.PositionEmbedding(8, 4)
    assert pe(x).shape == (5, 4)
    pe.position_offset = 3
    assert torch.equal(pe(x[:, :2]), pe.weight[3:5])
    with pytest.raises(ValueError):
        pe(torch.zeros(1, 6, dtype=torch.long))
    s = L.Summation(torch.nn.Embedding(10, 4), L.PositionEmbedding(8, 4))
    assert s(x).shape == (2, 5, 4)
    r = L.ResidualConnection(torch.nn.Identity(), torch.nn.Identity())
    assert torch.equal(r(torch.ones(2)), torch.full((2,), 4.0))
    assert L.SoftmaxOnLast(dim=-1)(torch.randn(2, 5, 3)).shape == (2, 3)
    rms = L.RMSNorm(6)
    y = rms(torch.randn(3, 6).to(torch.bfloat16))
    assert y.dtype == torch.float32  # bf16 x * fp32 weight promotes (reference semantics)
    mlp = L.GatedMLP(6, 12, activation="silu")
    assert mlp(torch.randn(2, 6)).shape == (2, 6)
    se = L.ScaledEmbedding(10, 4, scale=3.0)
    assert torch.allclose(se(x), se.weight[x] * 3.0)


def _rope_model(n_layer=3):
    C, H, Hkv, D = 16, 4, 2, 4
    blk = lambda: {"transformerblock": {
        "attn_block": {"sequential": [{"rmsnorm": {"normalized_shape": C}},
                                      {"linear": {"in_features": C, "out_features": (H + 2 * Hkv) * D, "bias": False}},
                                      {"attention": {"num_heads": H, "num_kv_heads": Hkv, "rope_theta": 10000.0,
                                                     "head_dim": D}},
                                      {"linear": {"in_features": H * D, "out_features": C, "bias": False}}]},
        "mlp_block": {"sequential": [{"rmsnorm": {"normalized_shape": C}},
                                     {"gatedmlp": {"in_features": C, "intermediate_size": 32}}]},
        "post_attn_norm": {"rmsnorm": {"normalized_shape": C}},
        "post_mlp_norm": {"rmsnorm": {"normalized_shape": C}}}}
    layers = [{"scaledembedding": {"num_embeddings": 50, "embedding_dim": C, "scale": 4.0}}] + \
             [blk() for _ in range(n_layer)] + \
             [{"rmsnorm": {"normalized_shape": C}}, {"linear": {"in_features": C, "out_features": 50, "bias": False}},
              {"softmaxlast": {"dim": -1}}]
    torch.manual_seed(0)
    return NeuralNetworkModel("rope", Mapper(layers, {"adamw": {"lr": 1e-3}}))


def _gpt_model():
    import bench
    torch.manual_seed(0)
    return NeuralNetworkModel("gpt", Mapper(bench.gpt2_layers(V=50, C=16, L=3, H=2, P=64), {"adamw": {"lr": 1e-3}}))


@pytest.mark.parametrize("make", [_gpt_model, _rope_model])
def test_kv_cache_decode_matches_full_recompute(make):
    """Incremental decode logits == full-context logits at every step (multi-layer, RoPE, GQA)."""
    model = make().eval()
    ctx = torch.randint(0, 50, (2, 5))
    cache, pos = model._attach_kv_cache(capacity=4)  # forces a capacity growth too
    try:
        with torch.no_grad():
            acts, _ = model(ctx, skip_softmax=True)
            for step in range(6):
                nxt = acts[-1][:, -1:].argmax(-1)
                full, _ = model._forward_nocache(torch.cat([ctx, nxt], 1))
                for p in pos:
                    p.position_offset = cache.seq_len()
                acts, _ = model(nxt, skip_softmax=True)
                assert torch.allclose(acts[-1][:, -1], full[-1][:, -1], atol=1e-4), step
                ctx = torch.cat([ctx, nxt], 1)
        assert all(cache.seq_len(i) == 11 for i in range(cache.num_layers))
    finally:
        model._detach_kv_cache(pos)


def test_kv_cache_api():
    c = KV.KVCache(2)
    k, v = torch.randn(1, 2, 3, 4), torch.randn(1, 2, 3, 4)
    fk, fv = c.append(0, k, v)
    assert torch.equal(fk, k) and c.seq_len(0) == 3 and c.seq_len(1) == 0
    k2 = torch.randn(1, 2, 1, 4)
    fk, fv = c.append(0, k2, k2)
    assert fk.shape == (1, 2, 4, 4) and torch.equal(fk[:, :, 3:], k2)
    assert c.get(1) == (None, None)
    m = c.metrics
    assert m.num_appends == 2 and m.total_entries == 4 and m.compression_ratio == 1.0
    c.log_metrics()
    c.clear()
    assert c.seq_len(0) == 0 and c.metrics.num_appends == 0


def test_turboquant_roundtrip_dtype_and_ratio():
    c = KV.TurboQuantKVCache(1)
    k = (torch.randn(2, 3, 5, 64) * 2).to(torch.bfloat16)
    fk, fv = c.append(0, k, k)
    assert fk.dtype == torch.bfloat16, "dequantised cache keeps the model dtype (reference bug 4)"
    rel = (fk.float() - k.float()).abs().max() / k.float().abs().max()
    assert rel < 0.02
    assert c._k[0].dtype == torch.int8
    assert c.metrics.compression_ratio > 1.5
    q, s = KV.TurboQuantKVCache._quantize(torch.zeros(1, 1, 1, 4))
    assert torch.all(s == 1) and torch.all(q == 0)


def test_factory_env_flag(monkeypatch):
    monkeypatch.setattr(KV, "TURBO_QUANT_ENABLED", True)
    assert isinstance(KV.create_kv_cache(2), KV.TurboQuantKVCache)
    monkeypatch.setattr(KV, "TURBO_QUANT_ENABLED", False)
    assert type(KV.create_kv_cache(2)) is KV.KVCache


def test_turboquant_generation_runs_bf16():
    model = _gpt_model().to(dtype=torch.bfloat16)
    import penroz.models.model as M
    orig = M.create_kv_cache
    M.create_kv_cache = lambda n, cap=None: KV.TurboQuantKVCache(n, cap)
    try:
        toks = model.generate_tokens([[1, 2, 3]], 16, 5, temperature=0.0)
    finally:
        M.create_kv_cache = orig
    assert len(toks) == 8
