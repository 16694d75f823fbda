"""Layer library for the JSON layer vocabulary.

Behavioural parity with the reference's custom modules (``neural_net_layers.py:7-225``):
``CausalSelfAttention``, ``PositionEmbedding``, ``Summation``, ``ResidualConnection``,
``SoftmaxOnLast``, ``RMSNorm``, ``GatedMLP``, ``ScaledEmbedding``, ``TransformerBlock``.
Parameter names and module nesting are identical, so state_dict keys match the reference's
checkpoints (``mappers.py:326-353``).

What differs (MI355X-first):
  * attention goes through ``penroz.ops.attention`` — the hand-written CDNA4 flash-attention
    kernels on GPU (fused QKV read, head merge in the epilogue, GQA by index math, no expand);
    torch SDPA math on CPU only;
  * the KV cache is preallocated and written in place, stores the *KV* heads (the reference
    expands GQA before caching, ``neural_net_layers.py:76-88``) and each layer reads its own
    cache length for the RoPE offset (reference bug: layer 0's length for every layer, ``:72``);
  * RMSNorm / RoPE / gated-MLP activation / LayerNorm / GELU use HIP kernels on GPU.
"""
from __future__ import annotations

import torch
from torch import Tensor
import torch.nn as nn

from penroz.ops import attention as attn_ops
from penroz.ops import norms as norm_ops
from penroz.ops import activations as act_ops
from penroz.ops import rope as rope_ops


class CausalSelfAttention(nn.Module):
    """Causal self-attention over a fused QKV input ``[B, T, (H + 2*Hkv) * D]``.

    Mirrors ``neural_net_layers.py:7-95``: optional RoPE (``rope_theta``), grouped-query
    attention (``num_kv_heads``), attention dropout while training, optional KV cache.
    """

    def __init__(self, num_heads: int, dropout: float = 0.0,
                 num_kv_heads: int = None, rope_theta: float = None,
                 head_dim: int = None):
        super().__init__()
        self.num_heads = num_heads
        self.num_kv_heads = num_kv_heads if num_kv_heads is not None else num_heads
        if self.num_heads % self.num_kv_heads != 0:
            raise ValueError(f"num_heads {num_heads} not divisible by num_kv_heads {self.num_kv_heads}")
        self.dropout = dropout
        self.rope_theta = rope_theta
        self.head_dim = head_dim
        self._kv_cache = None
        self._layer_idx = 0
        if rope_theta is not None and head_dim is not None:
            inv_freq = 1.0 / (rope_theta ** (torch.arange(0, head_dim, 2, dtype=torch.float32) / head_dim))
            self.register_buffer("inv_freq", inv_freq, persistent=False)

    def set_kv_cache(self, kv_cache, layer_idx: int):
        """Attach (or detach with ``None``) a KV cache slot for incremental decoding."""
        self._kv_cache = kv_cache
        self._layer_idx = layer_idx

    def _inv_freq(self, head_dim: int, device) -> Tensor:
        if hasattr(self, "inv_freq"):
            return self.inv_freq.to(device)
        return 1.0 / (self.rope_theta ** (torch.arange(0, head_dim, 2, device=device,
                                                       dtype=torch.float32) / head_dim))

    def forward(self, query_key_value: Tensor) -> Tensor:
        batch_size, block_size, total_dim = query_key_value.size()
        head_dim = total_dim // (self.num_heads + 2 * self.num_kv_heads)
        q_dim = self.num_heads * head_dim
        kv_dim = self.num_kv_heads * head_dim

        cache = self._kv_cache
        offset = cache.seq_len(self._layer_idx) if cache is not None else 0

        if self.rope_theta is not None:
            inv_freq = self._inv_freq(head_dim, query_key_value.device)
            # graph-replayed decode: positions come from the cache's device counter (one table per
            # (theta, head_dim) and step, shared by the layers)
            table = (cache.rope_table((self.rope_theta, head_dim), inv_freq, block_size)
                     if getattr(cache, "graph_mode", False) else None)
            qkv = rope_ops.apply_rope_qkv(query_key_value, self.num_heads, self.num_kv_heads, head_dim,
                                          inv_freq, offset, table=table)
        else:
            qkv = query_key_value

        if cache is None:
            dropout = self.dropout if self.training else 0.0
            return attn_ops.causal_attention_qkv(qkv, self.num_heads, self.num_kv_heads, head_dim,
                                                 dropout_p=dropout)

        # Incremental path: append this step's K/V (KV heads only) in place, attend over the cache.
        q, k, v = qkv.split([q_dim, kv_dim, kv_dim], dim=2)
        k = k.view(batch_size, block_size, self.num_kv_heads, head_dim)
        v = v.view(batch_size, block_size, self.num_kv_heads, head_dim)
        q = q.reshape(batch_size, block_size, self.num_heads, head_dim)
        return cache.attend(self._layer_idx, q, k, v)


class PositionEmbedding(nn.Embedding):
    """Learned absolute positions ``arange(offset, offset + T)`` (``neural_net_layers.py:98-118``)."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self._position_offset = 0
        self.position_offset_tensor: Tensor | None = None  # device int64 [1] (graph-replayed decode)

    @property
    def position_offset(self) -> int:
        return self._position_offset

    @position_offset.setter
    def position_offset(self, value: int):
        self._position_offset = value

    def forward(self, input_data: Tensor) -> Tensor:
        _, num_positions = input_data.shape
        if self.position_offset_tensor is not None:  # offset read on the device (caller bounds it)
            positions = self.position_offset_tensor + torch.arange(num_positions, dtype=torch.long,
                                                                   device=input_data.device)
            return super().forward(positions)
        if self._position_offset + num_positions > self.num_embeddings:
            raise ValueError(f"positions {self._position_offset}..{self._position_offset + num_positions} "
                             f"exceed the position table ({self.num_embeddings})")
        positions = torch.arange(self._position_offset, self._position_offset + num_positions,
                                 dtype=torch.long, device=input_data.device)
        return super().forward(positions)


class Summation(nn.Sequential):
    """Sum of every child applied to the same input (token + position embedding)."""

    def forward(self, input_data: Tensor) -> Tensor:
        forwarded = self[0](input_data)
        for layer in self[1:]:
            forwarded = forwarded + layer(input_data)
        return forwarded


class ResidualConnection(nn.Sequential):
    """``x = x + child(x)`` for each child in order."""

    def forward(self, forwarded: Tensor) -> Tensor:
        for layer in self:
            forwarded = forwarded + layer(forwarded)
        return forwarded


class SoftmaxOnLast(nn.Softmax):
    """Softmax over the last position's logits ``logits[:, -1, :]``."""

    def forward(self, logits: Tensor) -> Tensor:
        return super().forward(logits[:, -1, :])


class LayerNorm(nn.LayerNorm):
    """``nn.LayerNorm`` whose GPU path is the HIP LayerNorm kernel (fp32 statistics).

    Same parameters/keys as ``nn.LayerNorm``; the ``layernorm`` algo compiles to this class.
    """

    def forward(self, x: Tensor) -> Tensor:
        if len(self.normalized_shape) == 1 and self.elementwise_affine:
            w, b = self.weight, self.bias
            if w.dtype != torch.float32 and b is not None and not torch.is_grad_enabled():
                w, b = self._fp32_affine()  # inference on bf16 weights: no per-call casts
            return norm_ops.layer_norm(x, w, b, self.eps)
        return super().forward(x)

    def _fp32_affine(self):
        """fp32 copies of (weight, bias) — the kernel's parameter dtype — cached until the
        parameters change (storage or in-place version)."""
        key = (self.weight.data_ptr(), self.weight._version, self.bias.data_ptr(), self.bias._version)
        c = self.__dict__.get("_fp32_cache")
        if c is None or c[0] != key:
            c = (key, self.weight.detach().float(), self.bias.detach().float())
            self.__dict__["_fp32_cache"] = c
        return c[1], c[2]


class GELU(nn.GELU):
    """``nn.GELU`` (erf or tanh) whose GPU path is the vectorised HIP GELU kernel."""

    def forward(self, x: Tensor) -> Tensor:
        return act_ops.gelu(x, self.approximate)


class RMSNorm(nn.Module):
    """Root-mean-square norm computed in fp32 (``neural_net_layers.py:144-155``)."""

    def __init__(self, normalized_shape: int, eps: float = 1e-6):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(normalized_shape))
        self.eps = eps

    def forward(self, x: Tensor) -> Tensor:
        return norm_ops.rms_norm(x, self.weight, self.eps)


class GatedMLP(nn.Module):
    """``down(act(gate(x)) * up(x))`` with silu / gelu_tanh / gelu (``neural_net_layers.py:158-174``)."""

    def __init__(self, in_features: int, intermediate_size: int,
                 bias: bool = False, activation: str = "gelu_pytorch_tanh"):
        super().__init__()
        self.gate_proj = nn.Linear(in_features, intermediate_size, bias=bias)
        self.up_proj = nn.Linear(in_features, intermediate_size, bias=bias)
        self.down_proj = nn.Linear(intermediate_size, in_features, bias=bias)
        if activation in ("silu", "swish"):
            self.act_kind = "silu"
            self.act = nn.SiLU()
        elif activation == "gelu_pytorch_tanh":
            self.act_kind = "gelu_tanh"
            self.act = nn.GELU(approximate="tanh")
        else:
            self.act_kind = "gelu"
            self.act = nn.GELU()

    def forward(self, x: Tensor) -> Tensor:
        return self.down_proj(act_ops.gated_act(self.gate_proj(x), self.up_proj(x), self.act_kind))


class ScaledEmbedding(nn.Embedding):
    """Embedding whose output is multiplied by a fixed ``scale`` (Gemma: sqrt(hidden))."""

    def __init__(self, num_embeddings: int, embedding_dim: int, scale: float = 1.0, **kwargs):
        super().__init__(num_embeddings, embedding_dim, **kwargs)
        self.scale = scale

    def forward(self, input_data: Tensor) -> Tensor:
        return super().forward(input_data) * self.scale


class TransformerBlock(nn.Module):
    """Decoder block with optional post-norms (``neural_net_layers.py:188-225``).

    ``post_norm_on_residual=True`` (Gemma 3+): ``h = post_norm(x + attn(x))``;
    ``False`` (Gemma 2): ``h = x + post_norm(attn(x))``.
    """

    def __init__(self, attn_block: nn.Module, mlp_block: nn.Module,
                 post_attn_norm: nn.Module = None, post_mlp_norm: nn.Module = None,
                 post_norm_on_residual: bool = True):
        super().__init__()
        self.attn_block = attn_block
        self.mlp_block = mlp_block
        self.post_attn_norm = post_attn_norm
        self.post_mlp_norm = post_mlp_norm
        self.post_norm_on_residual = post_norm_on_residual

    def forward(self, x: Tensor) -> Tensor:
        attn_out = self.attn_block(x)
        if self.post_attn_norm is not None and not self.post_norm_on_residual:
            attn_out = self.post_attn_norm(attn_out)
        h = x + attn_out
        if self.post_attn_norm is not None and self.post_norm_on_residual:
            h = self.post_attn_norm(h)
        mlp_out = self.mlp_block(h)
        if self.post_mlp_norm is not None and not self.post_norm_on_residual:
            mlp_out = self.post_mlp_norm(mlp_out)
        out = h + mlp_out
        if self.post_mlp_norm is not None and self.post_norm_on_residual:
            out = self.post_mlp_norm(out)
        return out
