"""Every algo of the layer-config vocabulary: construction through the Mapper and forward output
shapes on CPU (reference: test_neural_net_layers.py — constructors and forward shapes)."""
import pytest
import torch
import torch.nn as nn

from penroz.models import layers as L
from penroz.models.mapper import Mapper

ADAM = {"adam": {"lr": 1e-3}}


def build(layer_cfg: dict) -> nn.Module:
    return Mapper([layer_cfg], ADAM).to_layers()[0]


CTOR_CASES = [
    ({"embedding": {"num_embeddings": 10, "embedding_dim": 4}}, nn.Embedding),
    ({"linear": {"in_features": 4, "out_features": 3}}, nn.Linear),
    ({"linear": {"in_features": 4, "out_features": 3, "bias": False}}, nn.Linear),
    ({"flatten": {}}, nn.Flatten),
    ({"batchnorm1d": {"num_features": 4}}, nn.BatchNorm1d),
    ({"relu": {}}, nn.ReLU),
    ({"gelu": {}}, L.GELU),
    ({"gelu": {"approximate": "tanh"}}, L.GELU),
    ({"sigmoid": {}}, nn.Sigmoid),
    ({"softmax": {"dim": -1}}, nn.Softmax),
    ({"tanh": {}}, nn.Tanh),
    ({"dropout": {"p": 0.1}}, nn.Dropout),
    ({"sequential": [{"linear": {"in_features": 4, "out_features": 4}}, {"relu": {}}]}, nn.Sequential),
    ({"layernorm": {"normalized_shape": 4}}, L.LayerNorm),
    ({"attention": {"num_heads": 2}}, L.CausalSelfAttention),
    ({"attention": {"num_heads": 4, "num_kv_heads": 2, "rope_theta": 10000.0, "head_dim": 8}}, L.CausalSelfAttention),
    ({"summation": [{"embedding": {"num_embeddings": 10, "embedding_dim": 4}},
                    {"position": {"num_embeddings": 8, "embedding_dim": 4}}]}, L.Summation),
    ({"residual": [{"linear": {"in_features": 4, "out_features": 4}}]}, L.ResidualConnection),
    ({"position": {"num_embeddings": 8, "embedding_dim": 4}}, L.PositionEmbedding),
    ({"softmaxlast": {"dim": -1}}, L.SoftmaxOnLast),
    ({"rmsnorm": {"normalized_shape": 4}}, L.RMSNorm),
    ({"gatedmlp": {"in_features": 4, "intermediate_size": 8}}, L.GatedMLP),
    ({"gatedmlp": {"in_features": 4, "intermediate_size": 8, "activation": "silu"}}, L.GatedMLP),
    ({"scaledembedding": {"num_embeddings": 10, "embedding_dim": 4, "scale": 2.0}}, L.ScaledEmbedding),
]


@pytest.mark.parametrize("cfg,cls", CTOR_CASES, ids=[next(iter(c)) + str(i) for i, (c, _) in enumerate(CTOR_CASES)])
def test_layer_construction(cfg, cls):
    assert isinstance(build(cfg), cls)


def test_attention_rejects_indivisible_kv_heads():
    with pytest.raises(ValueError):
        L.CausalSelfAttention(num_heads=3, num_kv_heads=2)


def test_init_and_confidence_applied_recursively():
    torch.manual_seed(0)
    # init functions are top-level keys of the layer dict (weight: normal / xavier_uniform /
    # kaiming_uniform, bias: zeros), applied to every submodule that has the attribute
    m = build({"sequential": [{"linear": {"in_features": 8, "out_features": 8}}],
               "normal": {"std": 0.02}, "zeros": {}, "confidence": 0.5})
    lin = m[0]
    assert torch.all(lin.bias == 0)
    assert 0.004 < lin.weight.std().item() < 0.02  # normal(0.02) scaled by 0.5


B, T = 2, 6
FWD_CASES = [
    ("embedding", {"embedding": {"num_embeddings": 10, "embedding_dim": 4}}, lambda: torch.randint(0, 10, (B, T)), (B, T, 4)),
    ("linear", {"linear": {"in_features": 4, "out_features": 3}}, lambda: torch.randn(B, T, 4), (B, T, 3)),
    ("flatten", {"flatten": {}}, lambda: torch.randn(B, 3, 4), (B, 12)),
    ("batchnorm1d", {"batchnorm1d": {"num_features": 4}}, lambda: torch.randn(5, 4), (5, 4)),
    ("relu", {"relu": {}}, lambda: torch.randn(B, 4), (B, 4)),
    ("gelu", {"gelu": {}}, lambda: torch.randn(B, T, 8), (B, T, 8)),
    ("gelu_tanh", {"gelu": {"approximate": "tanh"}}, lambda: torch.randn(B, T, 8), (B, T, 8)),
    ("sigmoid", {"sigmoid": {}}, lambda: torch.randn(B, 4), (B, 4)),
    ("softmax", {"softmax": {"dim": -1}}, lambda: torch.randn(B, 4), (B, 4)),
    ("tanh", {"tanh": {}}, lambda: torch.randn(B, 4), (B, 4)),
    ("dropout", {"dropout": {"p": 0.5}}, lambda: torch.randn(B, 4), (B, 4)),
    ("layernorm", {"layernorm": {"normalized_shape": 8}}, lambda: torch.randn(B, T, 8), (B, T, 8)),
    ("attention_mha", {"attention": {"num_heads": 2}}, lambda: torch.randn(B, T, 3 * 16), (B, T, 16)),
    ("attention_gqa_rope", {"attention": {"num_heads": 4, "num_kv_heads": 2, "rope_theta": 10000.0, "head_dim": 8}},
     lambda: torch.randn(B, T, (4 + 2 * 2) * 8), (B, T, 32)),
    ("summation", {"summation": [{"embedding": {"num_embeddings": 10, "embedding_dim": 4}},
                                 {"position": {"num_embeddings": 8, "embedding_dim": 4}}]},
     lambda: torch.randint(0, 10, (B, T)), (B, T, 4)),
    ("residual", {"residual": [{"linear": {"in_features": 4, "out_features": 4}},
                               {"linear": {"in_features": 4, "out_features": 4}}]}, lambda: torch.randn(B, T, 4), (B, T, 4)),
    ("position", {"position": {"num_embeddings": 8, "embedding_dim": 4}}, lambda: torch.randint(0, 10, (B, T)), (T, 4)),
    ("softmaxlast", {"softmaxlast": {"dim": -1}}, lambda: torch.randn(B, T, 10), (B, 10)),
    ("rmsnorm", {"rmsnorm": {"normalized_shape": 8}}, lambda: torch.randn(B, T, 8), (B, T, 8)),
    ("gatedmlp", {"gatedmlp": {"in_features": 8, "intermediate_size": 16}}, lambda: torch.randn(B, T, 8), (B, T, 8)),
    ("scaledembedding", {"scaledembedding": {"num_embeddings": 10, "embedding_dim": 4, "scale": 3.0}},
     lambda: torch.randint(0, 10, (B, T)), (B, T, 4)),
    ("sequential_mlp", {"sequential": [{"linear": {"in_features": 8, "out_features": 16}}, {"gelu": {}},
                                       {"linear": {"in_features": 16, "out_features": 8}}]},
     lambda: torch.randn(B, T, 8), (B, T, 8)),
]


@pytest.mark.parametrize("name,cfg,make_input,shape", FWD_CASES, ids=[c[0] for c in FWD_CASES])
def test_forward_shapes(name, cfg, make_input, shape):
    torch.manual_seed(0)
    m = build(cfg)
    m.eval()
    with torch.no_grad():
        out = m(make_input())
    assert tuple(out.shape) == shape
    assert torch.isfinite(out).all()


def test_transformer_block_forward_and_post_norm_variants():
    torch.manual_seed(0)
    C = 16
    def blk(on_residual):
        attn = nn.Sequential(L.RMSNorm(C), nn.Linear(C, 3 * C, bias=False), L.CausalSelfAttention(num_heads=2),
                             nn.Linear(C, C, bias=False))
        mlp = nn.Sequential(L.RMSNorm(C), L.GatedMLP(C, 32))
        return L.TransformerBlock(attn, mlp, L.RMSNorm(C), L.RMSNorm(C), post_norm_on_residual=on_residual)
    x = torch.randn(B, T, C)
    for on_res in (True, False):
        out = blk(on_res)(x)
        assert out.shape == x.shape and torch.isfinite(out).all()


def test_scaled_embedding_scales():
    e = L.ScaledEmbedding(10, 4, scale=3.0)
    idx = torch.tensor([[1, 2]])
    assert torch.allclose(e(idx), nn.functional.embedding(idx, e.weight) * 3.0)


def test_position_embedding_offset_and_bounds():
    p = L.PositionEmbedding(8, 4)
    p.position_offset = 5
    out = p(torch.zeros(1, 3, dtype=torch.long))
    assert torch.equal(out, p.weight[5:8])
    with pytest.raises(Exception):
        p(torch.zeros(1, 4, dtype=torch.long))  # 5 + 4 > 8 positions


def test_residual_adds_each_child_in_turn():
    r = L.ResidualConnection(nn.Identity(), nn.Identity())
    x = torch.ones(2, 3)
    assert torch.equal(r(x), 4 * x)  # x + x = 2x, then 2x + 2x


def test_softmaxlast_uses_last_position():
    s = L.SoftmaxOnLast(dim=-1)
    x = torch.randn(2, 5, 7)
    assert torch.allclose(s(x), torch.softmax(x[:, -1, :], dim=-1))


def test_rmsnorm_matches_formula():
    n = L.RMSNorm(8)
    with torch.no_grad():
        n.weight.uniform_(0.5, 1.5)
    x = torch.randn(3, 8)
    ref = x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + n.eps) * n.weight
    assert torch.allclose(n(x), ref, atol=1e-6)


@pytest.mark.parametrize("act,fn", [("silu", nn.functional.silu),
                                    ("gelu_pytorch_tanh", lambda t: nn.functional.gelu(t, approximate="tanh")),
                                    ("gelu", nn.functional.gelu)])
def test_gatedmlp_activation_variants(act, fn):
    torch.manual_seed(0)
    m = L.GatedMLP(8, 16, activation=act)
    x = torch.randn(2, 8)
    ref = m.down_proj(fn(m.gate_proj(x)) * m.up_proj(x))
    assert torch.allclose(m(x), ref, atol=1e-6)


def test_packed_gate_up_is_shared_and_tracks_weight_versions():
    """The Gemma decode program's fused [gate; up] weight is built once per weight version and
    shared by every decoder of the model (advisor: one copy per decoder)."""
    import torch
    from penroz.models import layers as L
    from penroz.models.graph_decode import _packed_gate_up
    mlp = L.GatedMLP(16, 32)
    a = _packed_gate_up(mlp)
    assert not a.requires_grad and a.shape == (64, 16)
    assert _packed_gate_up(mlp) is a
    torch.testing.assert_close(a, torch.cat([mlp.gate_proj.weight, mlp.up_proj.weight]).detach())
    with torch.no_grad():
        mlp.up_proj.weight.add_(1.0)  # an optimizer step bumps the version
    b = _packed_gate_up(mlp)
    assert b is not a
    torch.testing.assert_close(b[32:], mlp.up_proj.weight.detach())
