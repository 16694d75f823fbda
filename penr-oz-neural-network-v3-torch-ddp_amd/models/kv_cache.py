"""Preallocated KV cache for incremental decoding, plus the int8 "TurboQuant" variant.

API parity with the reference (``kv_cache.py:14-206``): ``KVCacheMetrics``, ``KVCache.append /
get / clear / seq_len / log_metrics``, ``TurboQuantKVCache`` (per-token absmax/127 int8 with
fp32 scales), ``create_kv_cache`` keyed on ``TURBO_QUANT_KV_CACHE=1``.

MI355X-first differences:
  * storage is preallocated ``[B, Hkv, capacity, D]`` per layer and written in place (the
    reference re-``torch.cat``s the whole cache every token — O(S) copies per step);
    capacity doubles only if a sequence outgrows it;
  * only the KV heads are stored (no GQA expansion before caching);
  * ``attend`` runs the decode-attention HIP kernel directly on the cache — for the int8
    cache the dequantisation is fused into the kernel, so the full cache is never
    materialised in fp32 (the reference dequantises the *whole* cache every step and returns
    fp32, which also breaks bf16 models — SURVEY §7.4 bug 4);
  * ``seq_len(layer_idx)`` is per layer, so each layer's RoPE offset is its own.
"""
from __future__ import annotations

import logging
import os
import time
from dataclasses import dataclass

import torch
from torch import Tensor

from penroz.ops import attention as attn_ops
from penroz.ops import sampling as samp_ops

log = logging.getLogger(__name__)

TURBO_QUANT_ENABLED = os.environ.get("TURBO_QUANT_KV_CACHE", "0") == "1"
DEFAULT_CAPACITY = 256


@dataclass
class KVCacheMetrics:
    num_appends: int = 0
    total_entries: int = 0
    memory_bytes: int = 0
    compressed_memory_bytes: int = 0
    compression_ratio: float = 1.0
    last_append_latency_ms: float = 0.0


class KVCache:
    """Per-layer preallocated key/value storage."""

    def __init__(self, num_layers: int = 0, capacity: int | None = None):
        self.num_layers = num_layers
        self._capacity_hint = capacity
        self._k: list[Tensor | None] = [None] * num_layers
        self._v: list[Tensor | None] = [None] * num_layers
        self._len: list[int] = [0] * num_layers
        self._metrics = KVCacheMetrics()

    # ------------------------------------------------------------------ bookkeeping
    @property
    def metrics(self) -> KVCacheMetrics:
        return self._metrics

    def reserve(self, capacity: int):
        """Capacity to allocate on first use (e.g. the generation block size)."""
        self._capacity_hint = capacity

    def seq_len(self, layer_idx: int = 0) -> int:
        return self._len[layer_idx]

    def clear(self):
        """Forget every cached token (storage is kept for reuse)."""
        self._len = [0] * self.num_layers
        self._metrics = KVCacheMetrics()

    def _record(self, t0: float, new_tokens: int, raw_bytes: int, stored_bytes: int):
        m = self._metrics
        m.num_appends += 1
        m.total_entries += new_tokens
        m.memory_bytes += raw_bytes
        m.compressed_memory_bytes += stored_bytes
        m.compression_ratio = (m.memory_bytes / m.compressed_memory_bytes
                               if m.compressed_memory_bytes > 0 else 1.0)
        m.last_append_latency_ms = (time.monotonic() - t0) * 1000

    def log_metrics(self):
        m = self._metrics
        log.info(f"KVCache metrics: entries={m.total_entries}, memory={m.memory_bytes / 1024:.1f}KB, "
                 f"compression_ratio={m.compression_ratio:.2f}, last_append={m.last_append_latency_ms:.3f}ms")

    # ------------------------------------------------------------------ storage
    def _alloc(self, like: Tensor, B: int, Hkv: int, cap: int, D: int, dtype=None):
        return torch.empty(B, Hkv, cap, D, dtype=dtype or like.dtype, device=like.device)

    def _ensure(self, layer_idx: int, like: Tensor, B: int, Hkv: int, D: int, new_tokens: int):
        """Make room for ``new_tokens`` more (a shape / device change resets the layer first)."""
        k = self._k[layer_idx]
        if k is not None and (k.shape[0] != B or k.shape[1] != Hkv or k.shape[3] != D
                              or k.device != like.device):
            k = None
            self._len[layer_idx] = 0
        needed = self._len[layer_idx] + new_tokens
        if k is None:
            cap = max(needed, self._capacity_hint or DEFAULT_CAPACITY)
            self._k[layer_idx] = self._alloc(like, B, Hkv, cap, D)
            self._v[layer_idx] = self._alloc(like, B, Hkv, cap, D)
        elif k.shape[2] < needed:
            cap = max(needed, 2 * k.shape[2])
            n = self._len[layer_idx]
            for store in (self._k, self._v):
                new = self._alloc(store[layer_idx], B, Hkv, cap, D)
                new[:, :, :n] = store[layer_idx][:, :, :n]
                store[layer_idx] = new

    def _write(self, layer_idx: int, k_bthd: Tensor, v_bthd: Tensor) -> int:
        """Store k/v given as [B, T, Hkv, D]; returns the new length."""
        B, T, Hkv, D = k_bthd.shape
        self._ensure(layer_idx, k_bthd, B, Hkv, D, T)
        pos = self._len[layer_idx]
        samp_ops.kv_store_into(k_bthd, self._k[layer_idx], pos)
        samp_ops.kv_store_into(v_bthd, self._v[layer_idx], pos)
        self._len[layer_idx] = pos + T
        return pos + T

    # ------------------------------------------------------------------ reference API
    def append(self, layer_idx: int, key: Tensor, value: Tensor) -> tuple[Tensor, Tensor]:
        """Append ``key``/``value`` of shape (B, Hkv, S_new, D); return the full (B, Hkv, S, D) views."""
        t0 = time.monotonic()
        raw = key.nelement() * key.element_size() + value.nelement() * value.element_size()
        n = self._write(layer_idx, key.transpose(1, 2), value.transpose(1, 2))
        self._record(t0, key.shape[2], raw, raw)
        return self._k[layer_idx][:, :, :n], self._v[layer_idx][:, :, :n]

    def get(self, layer_idx: int) -> tuple[Tensor | None, Tensor | None]:
        n = self._len[layer_idx]
        if n == 0:
            return None, None
        return self._k[layer_idx][:, :, :n], self._v[layer_idx][:, :, :n]

    # ------------------------------------------------------------------ decode attention
    def attend(self, layer_idx: int, q: Tensor, k: Tensor, v: Tensor) -> Tensor:
        """Append k/v ([B, T, Hkv, D]) then attend q ([B, T, H, D]) over the cache -> [B, T, H*D]."""
        t0 = time.monotonic()
        raw = k.nelement() * k.element_size() + v.nelement() * v.element_size()
        n = self._write(layer_idx, k, v)
        self._record(t0, k.shape[1], raw, raw)
        return attn_ops.decode_attention(q, self._k[layer_idx], self._v[layer_idx], n)


class TurboQuantKVCache(KVCache):
    """int8 KV cache with per-token fp32 scales (``kv_cache.py:101-195``)."""

    def __init__(self, num_layers: int = 0, capacity: int | None = None):
        super().__init__(num_layers, capacity)
        self._sk: list[Tensor | None] = [None] * num_layers
        self._sv: list[Tensor | None] = [None] * num_layers
        self._dtype: list[torch.dtype | None] = [None] * num_layers

    # per-token quantisation helpers kept with the reference's names for parity tests
    @staticmethod
    def _quantize(tensor: Tensor) -> tuple[Tensor, Tensor]:
        return samp_ops.reference_quantize(tensor)

    @staticmethod
    def _dequantize(quantized: Tensor, scale: Tensor) -> Tensor:
        return quantized.float() * scale

    def _ensure(self, layer_idx: int, like: Tensor, B: int, Hkv: int, D: int, new_tokens: int):
        """Make room for ``new_tokens`` more (a shape / device change resets the layer first)."""
        k = self._k[layer_idx]
        if k is not None and (k.shape[0] != B or k.shape[1] != Hkv or k.shape[3] != D
                              or k.device != like.device):
            k = None
            self._len[layer_idx] = 0
        needed = self._len[layer_idx] + new_tokens
        if k is None:
            cap = max(needed, self._capacity_hint or DEFAULT_CAPACITY)
            self._k[layer_idx] = self._alloc(like, B, Hkv, cap, D, torch.int8)
            self._v[layer_idx] = self._alloc(like, B, Hkv, cap, D, torch.int8)
            self._sk[layer_idx] = torch.ones(B, Hkv, cap, dtype=torch.float32, device=like.device)
            self._sv[layer_idx] = torch.ones(B, Hkv, cap, dtype=torch.float32, device=like.device)
        elif k.shape[2] < needed:
            cap = max(needed, 2 * k.shape[2])
            n = self._len[layer_idx]
            for store in (self._k, self._v):
                new = self._alloc(store[layer_idx], B, Hkv, cap, D, torch.int8)
                new[:, :, :n] = store[layer_idx][:, :, :n]
                store[layer_idx] = new
            for store in (self._sk, self._sv):
                new = torch.ones(B, Hkv, cap, dtype=torch.float32, device=like.device)
                new[:, :, :n] = store[layer_idx][:, :, :n]
                store[layer_idx] = new

    def _write(self, layer_idx: int, k_bthd: Tensor, v_bthd: Tensor) -> int:
        B, T, Hkv, D = k_bthd.shape
        self._ensure(layer_idx, k_bthd, B, Hkv, D, T)
        pos = self._len[layer_idx]
        samp_ops.kv_quantize_into(k_bthd, self._k[layer_idx], self._sk[layer_idx], pos)
        samp_ops.kv_quantize_into(v_bthd, self._v[layer_idx], self._sv[layer_idx], pos)
        self._dtype[layer_idx] = k_bthd.dtype
        self._len[layer_idx] = pos + T
        return pos + T

    def _stored_bytes(self, k: Tensor) -> int:
        n_tok = k.nelement() // k.shape[-1]
        return 2 * (k.nelement() * 1 + n_tok * 4)

    def append(self, layer_idx: int, key: Tensor, value: Tensor) -> tuple[Tensor, Tensor]:
        """Quantise and append (B, Hkv, S_new, D); return the dequantised full cache in key's dtype."""
        t0 = time.monotonic()
        raw = key.nelement() * key.element_size() + value.nelement() * value.element_size()
        n = self._write(layer_idx, key.transpose(1, 2), value.transpose(1, 2))
        self._record(t0, key.shape[2], raw, self._stored_bytes(key))
        k = self._dequantize(self._k[layer_idx][:, :, :n], self._sk[layer_idx][:, :, :n, None])
        v = self._dequantize(self._v[layer_idx][:, :, :n], self._sv[layer_idx][:, :, :n, None])
        return k.to(key.dtype), v.to(value.dtype)

    def get(self, layer_idx: int) -> tuple[Tensor | None, Tensor | None]:
        n = self._len[layer_idx]
        if n == 0:
            return None, None
        dt = self._dtype[layer_idx] or torch.float32
        return (self._dequantize(self._k[layer_idx][:, :, :n], self._sk[layer_idx][:, :, :n, None]).to(dt),
                self._dequantize(self._v[layer_idx][:, :, :n], self._sv[layer_idx][:, :, :n, None]).to(dt))

    def get_quantized(self, layer_idx: int):
        n = self._len[layer_idx]
        return self._k[layer_idx], self._v[layer_idx], self._sk[layer_idx], self._sv[layer_idx], n

    def attend(self, layer_idx: int, q: Tensor, k: Tensor, v: Tensor) -> Tensor:
        t0 = time.monotonic()
        raw = k.nelement() * k.element_size() + v.nelement() * v.element_size()
        n = self._write(layer_idx, k, v)
        self._record(t0, k.shape[1], raw, self._stored_bytes(k))
        return attn_ops.decode_attention(q, self._k[layer_idx], self._v[layer_idx], n,
                                         self._sk[layer_idx], self._sv[layer_idx])


def create_kv_cache(num_layers: int, capacity: int | None = None) -> KVCache:
    """``TurboQuantKVCache`` when ``TURBO_QUANT_KV_CACHE=1`` (module constant), else ``KVCache``."""
    if TURBO_QUANT_ENABLED:
        log.info("TurboQuant KV cache enabled (TURBO_QUANT_KV_CACHE=1)")
        return TurboQuantKVCache(num_layers, capacity)
    return KVCache(num_layers, capacity)
