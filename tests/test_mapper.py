"""Config compiler, optimizer factory, HF config/state-dict mapping (CPU)."""
import copy
from types import SimpleNamespace

import pytest
import torch
import torch.nn as nn

from penroz.models import layers as L
from penroz.models.mapper import Mapper
from penroz.models.model import NeuralNetworkModel
from penroz.models.optim import FusedAdamW, FusedAdam


ALL_ALGOS = [
    ({"embedding": {"num_embeddings": 10, "embedding_dim": 4}}, nn.Embedding),
    ({"linear": {"in_features": 4, "out_features": 3}}, nn.Linear),
    ({"flatten": {}}, nn.Flatten),
    ({"batchnorm1d": {"num_features": 4}}, nn.BatchNorm1d),
    ({"relu": {}}, nn.ReLU),
    ({"gelu": {"approximate": "tanh"}}, nn.GELU),
    ({"sigmoid": {}}, nn.Sigmoid),
    ({"softmax": {"dim": -1}}, nn.Softmax),
    ({"tanh": {}}, nn.Tanh),
    ({"dropout": {"p": 0.1}}, nn.Dropout),
    ({"sequential": [{"relu": {}}, {"tanh": {}}]}, nn.Sequential),
    ({"layernorm": {"normalized_shape": 4}}, nn.LayerNorm),
    ({"attention": {"num_heads": 2}}, L.CausalSelfAttention),
    ({"summation": [{"linear": {"in_features": 4, "out_features": 4}}, {"relu": {}}]}, L.Summation),
    ({"residual": [{"linear": {"in_features": 4, "out_features": 4}}]}, L.ResidualConnection),
    ({"position": {"num_embeddings": 8, "embedding_dim": 4}}, L.PositionEmbedding),
    ({"softmaxlast": {"dim": -1}}, L.SoftmaxOnLast),
    ({"rmsnorm": {"normalized_shape": 4}}, L.RMSNorm),
    ({"gatedmlp": {"in_features": 4, "intermediate_size": 8}}, L.GatedMLP),
    ({"scaledembedding": {"num_embeddings": 10, "embedding_dim": 4, "scale": 2.0}}, L.ScaledEmbedding),
]


@pytest.mark.parametrize("cfg,cls", ALL_ALGOS)
def test_every_algo_compiles(cfg, cls):
    (m,) = Mapper([cfg], {"sgd": {"lr": 0.1}}).to_layers()
    assert isinstance(m, cls)


def test_transformerblock_compiles_without_mutating_config():
    block = {"transformerblock": {
        "attn_block": {"sequential": [{"rmsnorm": {"normalized_shape": 8}},
                                      {"linear": {"in_features": 8, "out_features": 24, "bias": False}},
                                      {"attention": {"num_heads": 2, "rope_theta": 10000.0, "head_dim": 4}},
                                      {"linear": {"in_features": 8, "out_features": 8, "bias": False}}]},
        "mlp_block": {"sequential": [{"rmsnorm": {"normalized_shape": 8}},
                                     {"gatedmlp": {"in_features": 8, "intermediate_size": 16}}]},
        "post_attn_norm": {"rmsnorm": {"normalized_shape": 8}},
        "post_mlp_norm": {"rmsnorm": {"normalized_shape": 8}},
        "post_norm_on_residual": False}}
    before = copy.deepcopy(block)
    (m,) = Mapper([block], {"sgd": {"lr": 0.1}}).to_layers()
    assert isinstance(m, L.TransformerBlock) and not m.post_norm_on_residual
    assert block == before, "the layer config must not be mutated (reference bug 14)"
    assert m(torch.randn(2, 5, 8)).shape == (2, 5, 8)


def test_inits_and_confidence():
    torch.manual_seed(0)
    layers = [{"linear": {"in_features": 50, "out_features": 40}, "xavier_uniform": {}, "zeros": {}, "confidence": 0.5},
              {"linear": {"in_features": 40, "out_features": 40}, "normal": {"mean": 1.0, "std": 0.0}},
              {"linear": {"in_features": 40, "out_features": 40, "bias": False}, "kaiming_uniform": {}, "zeros": {}}]
    a, b, c = Mapper(layers, {"sgd": {"lr": 0.1}}).to_layers()
    bound = 0.5 * (6 / 90) ** 0.5
    assert a.weight.abs().max() <= bound + 1e-6 and torch.all(a.bias == 0)
    assert torch.all(b.weight == 1.0)
    assert c.bias is None


def test_optimizers():
    params = [nn.Parameter(torch.zeros(3))]
    o = Mapper([], {"adamw": {"lr": 6e-4, "betas": [0.9, 0.95], "eps": 1e-8}}).to_optimizer(params)
    assert isinstance(o, FusedAdamW) and isinstance(o, torch.optim.AdamW)
    assert o.param_groups[0]["betas"] == (0.9, 0.95) and o.param_groups[0]["weight_decay"] == 0.01
    assert isinstance(Mapper([], {"adam": {"lr": 1e-3}}).to_optimizer(params), FusedAdam)
    assert isinstance(Mapper([], {"sgd": {"lr": 1e-3, "momentum": 0.9}}).to_optimizer(params), torch.optim.SGD)


def test_fused_optimizer_cpu_matches_torch():
    torch.manual_seed(0)
    p1 = nn.Parameter(torch.randn(5, 4))
    p2 = nn.Parameter(p1.detach().clone())
    o1 = FusedAdamW([p1], lr=1e-2, weight_decay=0.1)
    o2 = torch.optim.AdamW([p2], lr=1e-2, weight_decay=0.1)
    for _ in range(3):
        g = torch.randn(5, 4)
        p1.grad, p2.grad = g.clone(), g.clone()
        o1.step()
        o2.step()
    assert torch.allclose(p1, p2)
    o3 = torch.optim.AdamW([nn.Parameter(torch.zeros(5, 4))], lr=1e-2)
    o3.load_state_dict(o1.state_dict())  # torch can read our state dict
    assert o1.param_groups[0]["fused"] is None  # the CPU fused kernel is chosen per step, not saved
    # and we resume from torch's (non-fused) state: the CPU fused kernel takes over its step tensors
    p4 = nn.Parameter(p2.detach().clone())
    o4 = FusedAdamW([p4], lr=1e-2, weight_decay=0.1)
    o4.load_state_dict(copy.deepcopy(o2.state_dict()))  # (torch's state_dict shares its state tensors)
    g = torch.randn(5, 4)
    p4.grad, p2.grad = g.clone(), g.clone()
    o4.step(grad_scale=0.5)
    p2.grad.mul_(0.5)
    o2.step()
    assert torch.allclose(p4, p2)


def test_fused_adam_cpu_matches_torch():
    torch.manual_seed(1)
    p1 = nn.Parameter(torch.randn(7, 3))
    p2 = nn.Parameter(p1.detach().clone())
    o1 = FusedAdam([p1], lr=1e-2, weight_decay=0.05, betas=(0.8, 0.9))
    o2 = torch.optim.Adam([p2], lr=1e-2, weight_decay=0.05, betas=(0.8, 0.9))
    for _ in range(4):
        g = torch.randn(7, 3)
        p1.grad, p2.grad = g.clone(), g.clone()
        o1.step()
        o2.step()
    assert torch.allclose(p1, p2, atol=1e-6)


def test_unsupported():
    with pytest.raises(ValueError):
        Mapper([{"bogus": {}}], {"sgd": {"lr": 1}}).to_layers()
    with pytest.raises(ValueError):
        Mapper([], {"bogus": {}}).to_optimizer([nn.Parameter(torch.zeros(1))])


# ---------------------------------------------------------------------------- HuggingFace GPT-2
def _hf_gpt2(n_layer=2, act="gelu_new"):
    from transformers import GPT2Config, GPT2LMHeadModel
    cfg = GPT2Config(vocab_size=120, n_positions=64, n_embd=32, n_layer=n_layer, n_head=4,
                     activation_function=act, resid_pdrop=0.0, embd_pdrop=0.0, attn_pdrop=0.0)
    torch.manual_seed(0)
    return cfg, GPT2LMHeadModel(cfg).eval()


def test_gpt2_config_to_layers():
    cfg, _ = _hf_gpt2(3)
    layers = Mapper.from_hf_config(cfg)
    assert len(layers) == 2 + 3 + 3
    assert layers[0]["summation"][0]["embedding"] == {"num_embeddings": 120, "embedding_dim": 32}
    assert layers[2]["residual"][1]["sequential"][2] == {"gelu": {"approximate": "tanh"}}
    assert layers[-2]["linear"]["bias"] is False and "softmaxlast" in layers[-1]
    layers = Mapper.from_hf_config(_hf_gpt2(1, act="gelu")[0])
    assert layers[2]["residual"][1]["sequential"][2] == {"gelu": {}}


def test_gpt2_import_logit_parity():
    cfg, hf = _hf_gpt2(2)
    sd = hf.state_dict()
    n = Mapper.detect_hf_n_layer(sd)
    assert n == 2
    model = NeuralNetworkModel("hf", Mapper(Mapper.from_hf_config(cfg, n), {"adamw": {"lr": 1e-3}}))
    mapped = Mapper.map_hf_state_dict_to_custom(sd, n, cfg)
    assert set(mapped) == set(model.state_dict())
    model.load_state_dict(mapped, strict=True)
    x = torch.randint(0, 120, (2, 17))
    with torch.no_grad():
        ref = hf(x).logits
        acts, _ = model(x, skip_softmax=True)
    assert torch.allclose(acts[-1], ref, atol=1e-4), (acts[-1] - ref).abs().max()


def test_gpt2_mapping_falls_back_to_tied_embedding():
    cfg, hf = _hf_gpt2(1)
    sd = {k: v for k, v in hf.state_dict().items() if k != "lm_head.weight"}
    mapped = Mapper.map_hf_state_dict_to_custom(sd, 1, cfg)
    assert torch.equal(mapped["layers.4.weight"], sd["transformer.wte.weight"])
    assert torch.equal(mapped["layers.2.0.1.weight"], sd["transformer.h.0.attn.c_attn.weight"].t())


# ---------------------------------------------------------------------------- Gemma family
def _gemma_cfg(model_type, n_layer=2, **extra):
    tc = SimpleNamespace(vocab_size=64, hidden_size=16, num_attention_heads=4, num_key_value_heads=2, head_dim=8,
                         num_hidden_layers=n_layer, intermediate_size=32, rms_norm_eps=1e-6, rope_theta=10000.0,
                         attention_dropout=0.0, hidden_activation="gelu_pytorch_tanh", **extra)
    if model_type in ("gemma3", "gemma4"):
        return SimpleNamespace(model_type=model_type, text_config=tc)
    tc.model_type = model_type
    return tc


def _gemma_sd(cfg, n_layer, prefix="model", drop_kv_for=()):
    tc = getattr(cfg, "text_config", cfg)
    C, H, Hkv = tc.hidden_size, tc.num_attention_heads, tc.num_key_value_heads
    types = getattr(tc, "layer_types", None) or ["sliding_attention"] * n_layer
    sd = {f"{prefix}.embed_tokens.weight": torch.randn(tc.vocab_size, C), f"{prefix}.norm.weight": torch.randn(C)}
    for i in range(n_layer):
        D = getattr(tc, "global_head_dim", tc.head_dim) if types[i] == "full_attention" else tc.head_dim
        hkv = (getattr(tc, "num_global_key_value_heads", None) or Hkv) if types[i] == "full_attention" else Hkv
        p = f"{prefix}.layers.{i}"
        sd[f"{p}.self_attn.q_proj.weight"] = torch.randn(H * D, C)
        if i not in drop_kv_for:
            sd[f"{p}.self_attn.k_proj.weight"] = torch.randn(hkv * D, C)
            sd[f"{p}.self_attn.v_proj.weight"] = torch.randn(hkv * D, C)
        sd[f"{p}.self_attn.o_proj.weight"] = torch.randn(C, H * D)
        for n in ("input_layernorm", "post_attention_layernorm", "pre_feedforward_layernorm", "post_feedforward_layernorm"):
            sd[f"{p}.{n}.weight"] = torch.randn(C)
        wide = 2 if getattr(tc, "use_double_wide_mlp", False) and i >= n_layer - (getattr(tc, "num_kv_shared_layers", 0) or 0) else 1
        sd[f"{p}.mlp.gate_proj.weight"] = torch.randn(tc.intermediate_size * wide, C)
        sd[f"{p}.mlp.up_proj.weight"] = torch.randn(tc.intermediate_size * wide, C)
        sd[f"{p}.mlp.down_proj.weight"] = torch.randn(C, tc.intermediate_size * wide)
    return sd


@pytest.mark.parametrize("mt,prefix", [("gemma", "model"), ("gemma2", "model"), ("gemma3_text", "model"),
                                       ("gemma3", "model.language_model")])
def test_gemma_mapping_keys_and_norm_offset(mt, prefix):
    cfg = _gemma_cfg(mt)
    layers = Mapper.from_hf_config(cfg)
    assert "scaledembedding" in layers[0] and layers[0]["scaledembedding"]["scale"] == 4.0
    blk = layers[1]["transformerblock"]
    assert ("post_attn_norm" in blk) == (mt != "gemma")
    if mt != "gemma":
        assert blk["post_norm_on_residual"] == (mt != "gemma2")
    model = NeuralNetworkModel("g", Mapper(layers, {"adamw": {"lr": 1e-3}}))
    sd = _gemma_sd(cfg, 2, prefix)
    mapped = Mapper.map_hf_state_dict_to_custom(sd, 2, cfg)
    assert set(mapped) == set(model.state_dict())
    model.load_state_dict(mapped, strict=True)
    assert torch.allclose(mapped["layers.1.attn_block.0.weight"], sd[f"{prefix}.layers.0.input_layernorm.weight"] + 1)
    y, _ = model(torch.randint(0, 64, (1, 6)), skip_softmax=True)
    assert y[-1].shape == (1, 6, 64)


def test_gemma4_heterogeneous_and_kv_shared_layers():
    types = ["sliding_attention", "full_attention", "sliding_attention", "full_attention"]
    cfg = _gemma_cfg("gemma4", 4, layer_types=types, global_head_dim=16, num_global_key_value_heads=1,
                     num_kv_shared_layers=2, use_double_wide_mlp=True)
    layers = Mapper.from_hf_config(cfg)
    att1 = layers[2]["transformerblock"]["attn_block"]["sequential"][2]["attention"]
    assert att1["head_dim"] == 16 and att1["num_kv_heads"] == 1
    assert layers[4]["transformerblock"]["mlp_block"]["sequential"][1]["gatedmlp"]["intermediate_size"] == 64
    sd = _gemma_sd(cfg, 4, "model.language_model", drop_kv_for=(2, 3))
    mapped = Mapper.map_hf_state_dict_to_custom(sd, 4, cfg)
    model = NeuralNetworkModel("g4", Mapper(layers, {"adamw": {"lr": 1e-3}}))
    model.load_state_dict(mapped, strict=True)
    # shared layer 3 (full) takes K/V from layer 1, layer 2 (sliding) from layer 0
    q3 = sd["model.language_model.layers.3.self_attn.q_proj.weight"]
    k1 = sd["model.language_model.layers.1.self_attn.k_proj.weight"]
    assert torch.equal(mapped["layers.4.attn_block.1.weight"][q3.shape[0]:q3.shape[0] + k1.shape[0]], k1)


def test_detect_n_layer():
    assert Mapper.detect_hf_n_layer({"transformer.h.3.attn.c_attn.weight": 0}) == 4
    assert Mapper.detect_hf_n_layer({"model.layers.5.self_attn.q_proj.weight": 0}) == 6
    assert Mapper.detect_hf_n_layer({"model.language_model.embed_tokens.weight": 0,
                                     "model.language_model.layers.1.self_attn.q_proj.weight": 0}) == 2
    assert Mapper.detect_hf_n_layer({}) == 0
