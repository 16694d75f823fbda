"""KV cache and TurboQuant int8 cache behaviour on CPU (reference: test_kv_cache.py, 18 tests),
plus the MI355X-design properties: preallocated storage, in-place appends, capacity growth,
per-layer lengths, dtype preservation."""
import pytest
import torch

from penroz.models import kv_cache as KC


def _kv(B=2, H=3, S=4, D=8, dtype=torch.float32, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(B, H, S, D, generator=g).to(dtype), torch.randn(B, H, S, D, generator=g).to(dtype))


def test_init_creates_empty_cache():
    c = KC.KVCache(num_layers=2)
    assert c.seq_len(0) == 0 and c.seq_len(1) == 0
    assert c.get(0) == (None, None)
    assert c.metrics.num_appends == 0


def test_append_single_step_returns_full_views():
    c = KC.KVCache(num_layers=1)
    k, v = _kv(S=1)
    fk, fv = c.append(0, k, v)
    assert fk.shape == (2, 3, 1, 8) and torch.equal(fk, k) and torch.equal(fv, v)
    assert c.seq_len(0) == 1


def test_append_multiple_steps_concatenates():
    c = KC.KVCache(num_layers=1)
    k1, v1 = _kv(S=3, seed=1)
    k2, v2 = _kv(S=2, seed=2)
    c.append(0, k1, v1)
    fk, fv = c.append(0, k2, v2)
    assert torch.equal(fk, torch.cat([k1, k2], dim=2)) and torch.equal(fv, torch.cat([v1, v2], dim=2))


def test_get_returns_cached_tensors():
    c = KC.KVCache(num_layers=1)
    k, v = _kv()
    c.append(0, k, v)
    gk, gv = c.get(0)
    assert torch.equal(gk, k) and torch.equal(gv, v)


def test_clear_resets_lengths_and_metrics():
    c = KC.KVCache(num_layers=2)
    k, v = _kv()
    c.append(0, k, v)
    c.append(1, k, v)
    c.clear()
    assert c.seq_len(0) == c.seq_len(1) == 0 and c.get(0) == (None, None)
    assert c.metrics.total_entries == 0


def test_metrics_updated_on_append():
    c = KC.KVCache(num_layers=1)
    k, v = _kv(S=5)
    c.append(0, k, v)
    m = c.metrics
    assert m.num_appends == 1 and m.total_entries == 5
    assert m.memory_bytes == 2 * k.nelement() * 4 and m.compression_ratio == 1.0
    assert m.last_append_latency_ms >= 0


def test_multi_layer_cache_independent_lengths():
    c = KC.KVCache(num_layers=3)
    k, v = _kv(S=4)
    c.append(0, k, v)
    c.append(2, k[:, :, :1], v[:, :, :1])
    assert [c.seq_len(i) for i in range(3)] == [4, 0, 1]


def test_storage_is_preallocated_and_written_in_place():
    c = KC.KVCache(num_layers=1, capacity=64)
    k, v = _kv(S=2)
    c.append(0, k, v)
    store = c._k[0]
    assert store.shape[2] == 64
    c.append(0, k, v)
    assert c._k[0].data_ptr() == store.data_ptr()  # no reallocation, no re-concatenation


def test_capacity_doubles_when_outgrown():
    c = KC.KVCache(num_layers=1, capacity=4)
    k, v = _kv(S=3, seed=3)
    c.append(0, k, v)
    k2, v2 = _kv(S=3, seed=4)
    fk, _ = c.append(0, k2, v2)
    assert c._k[0].shape[2] == 8
    assert torch.equal(fk, torch.cat([k, k2], dim=2))


def test_reserve_sets_first_allocation():
    c = KC.KVCache(num_layers=1)
    c.reserve(100)
    k, v = _kv(S=1)
    c.append(0, k, v)
    assert c._k[0].shape[2] == 100


def test_shape_change_resets_layer():
    c = KC.KVCache(num_layers=1)
    k, v = _kv(B=2)
    c.append(0, k, v)
    k1, v1 = _kv(B=1)
    fk, _ = c.append(0, k1, v1)
    assert fk.shape[0] == 1 and c.seq_len(0) == k1.shape[2]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_dtype_preserved(dtype):
    c = KC.KVCache(num_layers=1)
    k, v = _kv(dtype=dtype)
    fk, fv = c.append(0, k, v)
    assert fk.dtype == dtype and fv.dtype == dtype


# ----------------------------------------------------------------------------- TurboQuant
def test_turbo_init_creates_empty_cache():
    c = KC.TurboQuantKVCache(num_layers=2)
    assert c.get(0) == (None, None) and c.seq_len(1) == 0


def test_turbo_append_returns_dequantized_close_to_input():
    c = KC.TurboQuantKVCache(num_layers=1)
    k, v = _kv(S=6)
    fk, fv = c.append(0, k, v)
    assert fk.shape == k.shape and fk.dtype == k.dtype
    assert (fk - k).abs().max() <= k.abs().amax(-1, keepdim=True).max() / 127 + 1e-6
    assert (fv - v).abs().max() <= v.abs().amax(-1, keepdim=True).max() / 127 + 1e-6


def test_turbo_stored_as_int8_with_fp32_scales():
    c = KC.TurboQuantKVCache(num_layers=1)
    k, v = _kv()
    c.append(0, k, v)
    assert c._k[0].dtype == torch.int8 and c._v[0].dtype == torch.int8
    assert c._sk[0].dtype == torch.float32 and c._sk[0].shape[:2] == (2, 3)


def test_turbo_compression_ratio_greater_than_one():
    c = KC.TurboQuantKVCache(num_layers=1)
    k, v = _kv(D=64)
    c.append(0, k, v)
    assert c.metrics.compression_ratio > 3.0  # fp32 -> int8 + one fp32 scale per token


def test_turbo_append_multiple_steps():
    c = KC.TurboQuantKVCache(num_layers=1)
    k1, v1 = _kv(S=2, seed=5)
    k2, v2 = _kv(S=3, seed=6)
    c.append(0, k1, v1)
    fk, _ = c.append(0, k2, v2)
    assert fk.shape[2] == 5
    ref = torch.cat([k1, k2], dim=2)
    assert torch.allclose(fk, ref, atol=ref.abs().max().item() / 100)


def test_turbo_clear_resets():
    c = KC.TurboQuantKVCache(num_layers=1)
    k, v = _kv()
    c.append(0, k, v)
    c.clear()
    assert c.get(0) == (None, None) and c.metrics.num_appends == 0


def test_quantize_dequantize_roundtrip():
    x = torch.randn(4, 16, 32)
    q, s = KC.TurboQuantKVCache._quantize(x)
    assert q.dtype == torch.int8
    back = KC.TurboQuantKVCache._dequantize(q, s)
    assert (back - x).abs().max() <= (x.abs().amax(-1, keepdim=True) / 127).max() + 1e-6


def test_quantize_zero_tensor_is_safe():
    q, s = KC.TurboQuantKVCache._quantize(torch.zeros(2, 3, 8))
    back = KC.TurboQuantKVCache._dequantize(q, s)
    assert torch.isfinite(back).all() and back.abs().max() == 0


def test_per_token_scales_preserve_accuracy_across_appends():
    """A large-magnitude append must not degrade earlier small-magnitude tokens."""
    c = KC.TurboQuantKVCache(num_layers=1)
    small = torch.randn(1, 1, 4, 16) * 1e-3
    big = torch.randn(1, 1, 4, 16) * 1e3
    c.append(0, small, small)
    fk, _ = c.append(0, big, big)
    rel = ((fk[:, :, :4] - small).abs().max() / small.abs().max()).item()
    assert rel < 0.02


def test_turbo_keeps_bf16_dtype():
    c = KC.TurboQuantKVCache(num_layers=1)
    k, v = _kv(dtype=torch.bfloat16)
    fk, fv = c.append(0, k, v)
    gk, gv = c.get(0)
    assert fk.dtype == gk.dtype == torch.bfloat16


# ----------------------------------------------------------------------------- factory
def test_factory_default_creates_basic_cache(monkeypatch):
    monkeypatch.setattr(KC, "TURBO_QUANT_ENABLED", False)
    c = KC.create_kv_cache(2)
    assert type(c) is KC.KVCache and c.num_layers == 2


def test_factory_env_flag_creates_turbo_cache(monkeypatch):
    monkeypatch.setattr(KC, "TURBO_QUANT_ENABLED", True)
    assert isinstance(KC.create_kv_cache(2), KC.TurboQuantKVCache)


def test_attend_matches_reference_attention():
    from penroz.ops import attention as A
    c = KC.KVCache(num_layers=1)
    g = torch.Generator().manual_seed(0)
    B, H, Hkv, D = 1, 4, 2, 16
    outs = []
    ks, vs = [], []
    for t in range(3):
        q = torch.randn(B, 1, H, D, generator=g)
        k = torch.randn(B, 1, Hkv, D, generator=g)
        v = torch.randn(B, 1, Hkv, D, generator=g)
        ks.append(k)
        vs.append(v)
        out = c.attend(0, q, k, v)
        kk = torch.cat(ks, 1).transpose(1, 2)
        vv = torch.cat(vs, 1).transpose(1, 2)
        ref = A.reference_cache_attention(q, kk, vv, t)
        assert torch.allclose(out, ref, atol=1e-5)
