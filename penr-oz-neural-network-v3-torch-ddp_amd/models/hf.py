"""HuggingFace config -> layer list, and HF state dict -> internal state-dict keys.

Behaviour follows the reference (``mappers.py:102-262`` configs, ``:276-448`` weights):

GPT-2 family: ``summation(embedding, position)``, embd dropout, L residual blocks of
``[layernorm, linear(C,3C), attention, linear(C,C), dropout]`` +
``[layernorm, linear(C,4C), gelu, linear(4C,C), dropout]``, final layernorm, untied lm_head,
``softmaxlast``.  ``gelu_new`` -> tanh GELU; dropouts from ``embd/resid/attn_pdrop``.
HF's Conv1D weights are transposed; ``lm_head`` falls back to the tied ``wte``.

Gemma family (gemma, gemma2, gemma3(_text), gemma4(_text)): ``scaledembedding`` (×sqrt(C)),
``transformerblock`` per layer (RMSNorm → fused QKV → GQA/RoPE attention → o_proj;
RMSNorm → gated MLP), post-norms for Gemma 2+ (on the branch for Gemma 2, after the residual
add for 3+), Gemma 4 heterogeneous full/sliding layers and KV-shared layers (K/V weights
copied from the last earlier layer of the same type), double-wide MLP on shared layers.
Gemma's ``1 + w`` RMSNorm weights are converted to plain weights (+1).
"""
from __future__ import annotations

import logging

import torch

log = logging.getLogger(__name__)

GEMMA_MODEL_TYPES = frozenset({"gemma", "gemma2", "gemma3", "gemma3_text", "gemma4", "gemma4_text"})


def _first_attr(cfg, *names, default=None):
    for n in names:
        v = getattr(cfg, n, None)
        if v is not None:
            return v
    return default


def is_gemma(hf_config) -> bool:
    mt = getattr(hf_config, "model_type", None)
    return isinstance(mt, str) and mt in GEMMA_MODEL_TYPES


def layers_from_hf_config(hf_config, n_layer_override: int = None) -> list[dict]:
    layers = gemma_layers(hf_config, n_layer_override) if is_gemma(hf_config) else gpt2_layers(hf_config, n_layer_override)
    log.info("Built %d layers from HuggingFace config (model_type=%s)", len(layers),
             getattr(hf_config, "model_type", None))
    return layers


# --------------------------------------------------------------------------- GPT-2
def gpt2_layers(cfg, n_layer_override: int = None) -> list[dict]:
    vocab = cfg.vocab_size
    C = _first_attr(cfg, "n_embd", "hidden_size")
    H = _first_attr(cfg, "n_head", "num_attention_heads")
    L = n_layer_override if n_layer_override is not None else _first_attr(cfg, "n_layer", "num_hidden_layers")
    P = _first_attr(cfg, "n_positions", "max_position_embeddings")
    act = getattr(cfg, "activation_function", "gelu_new")
    gelu = {"gelu": {"approximate": "tanh"}} if act == "gelu_new" else {"gelu": {}}
    p_resid = getattr(cfg, "resid_pdrop", 0.0)
    p_embd = getattr(cfg, "embd_pdrop", 0.0)
    p_attn = getattr(cfg, "attn_pdrop", 0.0)

    def attn_branch():
        return {"sequential": [{"layernorm": {"normalized_shape": C}},
                               {"linear": {"in_features": C, "out_features": 3 * C}},
                               {"attention": {"num_heads": H, "dropout": p_attn}},
                               {"linear": {"in_features": C, "out_features": C}},
                               {"dropout": {"p": p_resid}}]}

    def mlp_branch():
        return {"sequential": [{"layernorm": {"normalized_shape": C}},
                               {"linear": {"in_features": C, "out_features": 4 * C}},
                               dict(gelu),
                               {"linear": {"in_features": 4 * C, "out_features": C}},
                               {"dropout": {"p": p_resid}}]}

    out = [{"summation": [{"embedding": {"num_embeddings": vocab, "embedding_dim": C}},
                          {"position": {"num_embeddings": P, "embedding_dim": C}}]},
           {"dropout": {"p": p_embd}}]
    out += [{"residual": [attn_branch(), mlp_branch()]} for _ in range(L)]
    out += [{"layernorm": {"normalized_shape": C}},
            {"linear": {"in_features": C, "out_features": vocab, "bias": False}},
            {"softmaxlast": {"dim": -1}}]
    return out


# --------------------------------------------------------------------------- Gemma
def _rope_theta(tc) -> float:
    theta = getattr(tc, "rope_theta", None)
    if theta is not None:
        return theta
    scaling = getattr(tc, "rope_scaling", None)
    if isinstance(scaling, dict) and "sliding_attention" in scaling:
        return scaling["sliding_attention"].get("rope_theta", 10000.0)
    return 10000.0


def gemma_layers(cfg, n_layer_override: int = None) -> list[dict]:
    mt = cfg.model_type
    tc = getattr(cfg, "text_config", cfg)
    vocab, C = tc.vocab_size, tc.hidden_size
    H = tc.num_attention_heads
    Hkv = getattr(tc, "num_key_value_heads", H)
    D = getattr(tc, "head_dim", C // H)
    L = n_layer_override if n_layer_override is not None else tc.num_hidden_layers
    inter = getattr(tc, "intermediate_size", 4 * C)
    eps = getattr(tc, "rms_norm_eps", 1e-6)
    theta = _rope_theta(tc)
    p_attn = getattr(tc, "attention_dropout", 0.0)
    act = getattr(tc, "hidden_activation", None) or getattr(tc, "hidden_act", "gelu_pytorch_tanh")
    post_norms = mt != "gemma"
    on_residual = mt != "gemma2"
    layer_types = getattr(tc, "layer_types", None)
    D_global = getattr(tc, "global_head_dim", D)
    Hkv_global = getattr(tc, "num_global_key_value_heads", None) or Hkv
    double_wide = getattr(tc, "use_double_wide_mlp", False)
    n_shared = getattr(tc, "num_kv_shared_layers", 0) or 0
    first_shared = L - n_shared if n_shared > 0 else L

    def rms():
        return {"rmsnorm": {"normalized_shape": C, "eps": eps}}

    out: list[dict] = [{"scaledembedding": {"num_embeddings": vocab, "embedding_dim": C, "scale": float(C ** 0.5)}}]
    for i in range(L):
        full = bool(layer_types) and i < len(layer_types) and layer_types[i] == "full_attention"
        d = D_global if full else D
        hkv = Hkv_global if full else Hkv
        mlp_width = inter * 2 if (double_wide and i >= first_shared) else inter
        block = {
            "attn_block": {"sequential": [
                rms(),
                {"linear": {"in_features": C, "out_features": H * d + 2 * hkv * d, "bias": False}},
                {"attention": {"num_heads": H, "num_kv_heads": hkv, "dropout": p_attn,
                               "rope_theta": theta, "head_dim": d}},
                {"linear": {"in_features": H * d, "out_features": C, "bias": False}},
            ]},
            "mlp_block": {"sequential": [
                rms(),
                {"gatedmlp": {"in_features": C, "intermediate_size": mlp_width, "bias": False,
                              "activation": act}},
            ]},
        }
        if post_norms:
            block["post_attn_norm"] = rms()
            block["post_mlp_norm"] = rms()
            block["post_norm_on_residual"] = on_residual
        out.append({"transformerblock": block})
    out += [rms(), {"linear": {"in_features": C, "out_features": vocab, "bias": False}},
            {"softmaxlast": {"dim": -1}}]
    return out


# --------------------------------------------------------------------------- state dicts
def _gemma_prefix(sd: dict) -> str:
    return "model.language_model" if "model.language_model.embed_tokens.weight" in sd else "model"


def detect_n_layer(sd: dict) -> int:
    pfx = _gemma_prefix(sd)
    idx_pos = pfx.count(".") + 2
    gemma = [int(k.split(".")[idx_pos]) for k in sd
             if k.startswith(f"{pfx}.layers.") and k.endswith(".self_attn.q_proj.weight")]
    if gemma:
        return max(gemma) + 1
    gpt2 = [int(k.split(".")[2]) for k in sd if k.startswith("transformer.h.") and k.endswith(".attn.c_attn.weight")]
    return max(gpt2) + 1 if gpt2 else 0


def map_state_dict(sd: dict, n_layer: int, hf_config=None) -> dict:
    if hf_config is not None and is_gemma(hf_config):
        return _map_gemma(sd, n_layer, hf_config)
    return _map_gpt2(sd, n_layer)


# (internal suffix, HF suffix, transpose?) for one GPT-2 block; "0" = attention branch,
# "1" = MLP branch; positions inside each Sequential follow gpt2_layers above.
_GPT2_BLOCK = [
    ("0.0.weight", "ln_1.weight", False), ("0.0.bias", "ln_1.bias", False),
    ("0.1.weight", "attn.c_attn.weight", True), ("0.1.bias", "attn.c_attn.bias", False),
    ("0.3.weight", "attn.c_proj.weight", True), ("0.3.bias", "attn.c_proj.bias", False),
    ("1.0.weight", "ln_2.weight", False), ("1.0.bias", "ln_2.bias", False),
    ("1.1.weight", "mlp.c_fc.weight", True), ("1.1.bias", "mlp.c_fc.bias", False),
    ("1.3.weight", "mlp.c_proj.weight", True), ("1.3.bias", "mlp.c_proj.bias", False),
]


def _map_gpt2(sd: dict, n_layer: int) -> dict:
    out = {"layers.0.0.weight": sd["transformer.wte.weight"],
           "layers.0.1.weight": sd["transformer.wpe.weight"]}
    for i in range(n_layer):
        for ours, theirs, transpose in _GPT2_BLOCK:
            w = sd[f"transformer.h.{i}.{theirs}"]
            out[f"layers.{2 + i}.{ours}"] = w.t().contiguous() if transpose else w  # HF Conv1D is [in, out]
    lnf = 2 + n_layer
    out[f"layers.{lnf}.weight"] = sd["transformer.ln_f.weight"]
    out[f"layers.{lnf}.bias"] = sd["transformer.ln_f.bias"]
    out[f"layers.{lnf + 1}.weight"] = sd.get("lm_head.weight", sd["transformer.wte.weight"])
    return out


def _kv_reference_layers(tc, n_layer: int) -> dict[int, int]:
    n_shared = getattr(tc, "num_kv_shared_layers", 0) or 0
    types = getattr(tc, "layer_types", None)
    refs: dict[int, int] = {}
    if n_shared <= 0 or not types or len(types) < n_layer:
        return refs
    first = n_layer - n_shared
    for i in range(first, n_layer):
        for j in range(first - 1, -1, -1):  # last earlier non-shared layer of the same type
            if types[j] == types[i]:
                refs[i] = j
                break
    return refs


def _map_gemma(sd: dict, n_layer: int, cfg) -> dict:
    post_norms = cfg.model_type != "gemma"
    pfx = _gemma_prefix(sd)
    found = detect_n_layer(sd)
    if found != n_layer:
        log.warning("HF state dict has %d text layers but config says %d; using detected count", found, n_layer)
        n_layer = found
    refs = _kv_reference_layers(getattr(cfg, "text_config", cfg), n_layer)
    one = lambda key: sd[key] + 1  # Gemma RMSNorm stores (w - 1)

    out = {"layers.0.weight": sd[f"{pfx}.embed_tokens.weight"]}
    for i in range(n_layer):
        blk, hf = f"layers.{1 + i}", f"{pfx}.layers.{i}"
        kv_src = f"{pfx}.layers.{refs[i]}" if i in refs else hf
        out[f"{blk}.attn_block.0.weight"] = one(f"{hf}.input_layernorm.weight")
        out[f"{blk}.attn_block.1.weight"] = torch.cat([sd[f"{hf}.self_attn.q_proj.weight"],
                                                       sd[f"{kv_src}.self_attn.k_proj.weight"],
                                                       sd[f"{kv_src}.self_attn.v_proj.weight"]], dim=0)
        out[f"{blk}.attn_block.3.weight"] = sd[f"{hf}.self_attn.o_proj.weight"]
        if post_norms:
            out[f"{blk}.post_attn_norm.weight"] = one(f"{hf}.post_attention_layernorm.weight")
            out[f"{blk}.mlp_block.0.weight"] = one(f"{hf}.pre_feedforward_layernorm.weight")
            out[f"{blk}.post_mlp_norm.weight"] = one(f"{hf}.post_feedforward_layernorm.weight")
        else:  # Gemma 1: post_attention_layernorm is the pre-MLP norm
            out[f"{blk}.mlp_block.0.weight"] = one(f"{hf}.post_attention_layernorm.weight")
        for proj in ("gate_proj", "up_proj", "down_proj"):
            out[f"{blk}.mlp_block.1.{proj}.weight"] = sd[f"{hf}.mlp.{proj}.weight"]
    lnf = 1 + n_layer
    out[f"layers.{lnf}.weight"] = one(f"{pfx}.norm.weight")
    out[f"layers.{lnf + 1}.weight"] = sd.get("lm_head.weight", sd[f"{pfx}.embed_tokens.weight"])
    return out
