"""JSON layer-list compiler (the model "config language") and optimizer factory.

API and vocabulary parity with the reference ``Mapper`` (``mappers.py:18-99, 264-274``):
21 layer algos, weight inits ``xavier_uniform / kaiming_uniform / normal``, bias init
``zeros``, ``confidence`` weight scaling, optimizers ``adam / adamw / sgd`` with torch
defaults (AdamW weight_decay 0.01 on *all* params, one param group).  HF config/state-dict
mapping lives in :mod:`penroz.models.hf` and is re-exported here as classmethods.

Differences on purpose:
  * the config is never mutated (the reference compiles ``transformerblock`` by writing
    ``nn.Module`` objects back into the caller's dict, so modules end up pickled in the
    checkpoint — SURVEY §7.4 bug 14);
  * ``layernorm`` / ``gelu`` compile to subclasses whose GPU path is a HIP kernel (same
    parameters and keys as ``nn.LayerNorm`` / ``nn.GELU``);
  * ``adam`` / ``adamw`` compile to fused-kernel subclasses of ``torch.optim.Adam/AdamW``
    (identical ``state_dict`` format, one multi-tensor HIP launch per step on GPU).
"""
from __future__ import annotations

import copy
import logging
from typing import Any, Iterable, Tuple

import torch
import torch.nn as nn
from torch.optim import Optimizer

from penroz.models import layers as L
from penroz.models import optim as fused_optim

log = logging.getLogger(__name__)


class Mapper:
    _algo_to_func = {
        "embedding": nn.Embedding,
        "linear": nn.Linear,
        "flatten": nn.Flatten,
        "batchnorm1d": nn.BatchNorm1d,
        "relu": nn.ReLU,
        "gelu": L.GELU,
        "sigmoid": nn.Sigmoid,
        "softmax": nn.Softmax,
        "tanh": nn.Tanh,
        "dropout": nn.Dropout,
        "sequential": nn.Sequential,
        "layernorm": L.LayerNorm,
        "attention": L.CausalSelfAttention,
        "summation": L.Summation,
        "residual": L.ResidualConnection,
        "position": L.PositionEmbedding,
        "softmaxlast": L.SoftmaxOnLast,
        "rmsnorm": L.RMSNorm,
        "gatedmlp": L.GatedMLP,
        "scaledembedding": L.ScaledEmbedding,
        "transformerblock": L.TransformerBlock,
    }

    _init_weight_to_func = {
        "xavier_uniform": nn.init.xavier_uniform_,
        "kaiming_uniform": nn.init.kaiming_uniform_,
        "normal": nn.init.normal_,
    }

    _init_bias_to_func = {
        "zeros": nn.init.zeros_,
    }

    _optim_to_func = {
        "adam": fused_optim.FusedAdam,
        "adamw": fused_optim.FusedAdamW,
        "sgd": torch.optim.SGD,
    }

    def __init__(self, layers: list[dict], optimizer: dict):
        self.layers = layers
        self.optimizer = optimizer

    # ------------------------------------------------------------------ compiler
    @staticmethod
    def _unpack_func_and_args(k_to_args: dict, k_to_func: dict) -> Tuple[Any, Any]:
        for k, v in k_to_args.items():
            if k in k_to_func:
                return k_to_func[k], v
        return None, None

    @staticmethod
    def _apply_confidence(module: nn.Module, confidence: float):
        weight = getattr(module, "weight", None)
        if isinstance(weight, torch.Tensor):
            with torch.no_grad():
                weight.mul_(confidence)

    @classmethod
    def _to_layer(cls, layer: dict) -> nn.Module:
        layer_func, raw_args = cls._unpack_func_and_args(layer, cls._algo_to_func)
        if layer_func is None:
            raise ValueError(f"Unsupported layer: {layer}")
        if isinstance(raw_args, dict):
            args = {k: (cls._to_layer(v) if isinstance(v, dict) else copy.deepcopy(v))
                    for k, v in raw_args.items()}
            module: nn.Module = layer_func(**args)
        elif isinstance(raw_args, list):
            args = [cls._to_layer(a) if isinstance(a, dict) else a for a in raw_args]
            module = layer_func(*args)
        elif raw_args is None:
            module = layer_func()
        else:
            raise ValueError(f"Unsupported layer arguments: {layer}")

        init_w, init_w_args = cls._unpack_func_and_args(layer, cls._init_weight_to_func)
        if init_w is not None:
            module.apply(lambda m: init_w(m.weight, **init_w_args)
                         if isinstance(getattr(m, "weight", None), torch.Tensor) else None)
        init_b, init_b_args = cls._unpack_func_and_args(layer, cls._init_bias_to_func)
        if init_b is not None:
            module.apply(lambda m: init_b(m.bias, **init_b_args)
                         if isinstance(getattr(m, "bias", None), torch.Tensor) else None)
        confidence = layer.get("confidence")
        if confidence is not None:
            module.apply(lambda m: cls._apply_confidence(m, confidence))
        return module

    def to_layers(self) -> list[nn.Module]:
        return [self._to_layer(layer) for layer in self.layers]

    def to_optimizer(self, params: Iterable[torch.Tensor]) -> Optimizer:
        optim_func, optim_args = self._unpack_func_and_args(self.optimizer, self._optim_to_func)
        if optim_func is None:
            raise ValueError(f"Unsupported optimizer: {self.optimizer}")
        kwargs = dict(optim_args or {})
        if "betas" in kwargs:
            kwargs["betas"] = tuple(kwargs["betas"])
        return optim_func(params, **kwargs)

    # ------------------------------------------------------------------ HuggingFace mapping
    @classmethod
    def from_hf_config(cls, hf_config, n_layer_override: int = None) -> list[dict]:
        from penroz.models import hf
        return hf.layers_from_hf_config(hf_config, n_layer_override)

    @staticmethod
    def detect_hf_n_layer(hf_sd: dict) -> int:
        from penroz.models import hf
        return hf.detect_n_layer(hf_sd)

    @classmethod
    def map_hf_state_dict_to_custom(cls, hf_sd: dict, n_layer: int, hf_config=None) -> dict:
        from penroz.models import hf
        return hf.map_state_dict(hf_sd, n_layer, hf_config)
