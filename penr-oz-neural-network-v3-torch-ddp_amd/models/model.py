"""Model runtime: create / persist / import / forward / evaluate / generate / train / diagnose.

API parity with the reference ``NeuralNetworkModel`` (``neural_net_model.py:28-779``) so the
service layer and checkpoints interoperate: same constructor, attributes (``progress``,
``avg_cost``, ``avg_cost_history``, ``stats``, ``status``), ``serialize / deserialize /
delete / from_huggingface``, ``forward(input, target, skip_softmax) -> (activations, cost)``,
``compute_output``, ``evaluate_model``, ``generate_tokens[_stream]``,
``train_model_on_device`` (distributed worker entry) and ``train_model``.

Training engines (``PENROZ_ENGINE``, default ``auto``):
  * ``fused`` — GPT-2-pattern models on GPU lower to :class:`penroz.models.executor.GPTExecutor`,
    Gemma-pattern models to :class:`penroz.models.gemma_executor.GemmaExecutor` (hand-written HIP
    kernels + hipBLASLt GEMMs, explicit backward, flat fp32 master/grad buffers, fused AdamW,
    bucketed RCCL all-reduce overlapped with backward);
  * ``generic`` — any layer list: module forward (HIP kernels through autograd), bf16 autocast
    on GPU, our bucketed reducer for DDP;
  * ``reference`` — stock PyTorch eager + autocast + ``torch.nn.parallel.DDP`` + foreach AdamW
    (the reference's exact semantics; used as the on-device baseline).
``auto`` = fused when the pattern matches on GPU, else generic.

Semantics kept: ``num_steps = max(1, B·T // (step_size·T·world))`` micro-steps, loss = mean of
micro-step losses all-reduced as an average, rank data stride ``B·T·rank`` /
``B·T·world``, progress/stats schemas and caps, status codes, ``speedPerSec = B·T/epoch_secs``
(rank-0 micro-step view, kept for compatibility) plus a true whole-job ``tokensPerSec``.
"""
from __future__ import annotations

import logging
import os
import random
import time
from contextlib import nullcontext
from datetime import datetime as dt
from typing import Optional, Tuple

import numpy as np
import torch
import torch.nn as nn
from torch import Tensor
import torch.distributed as dist

from penroz.models.kv_cache import KVCache, create_kv_cache
from penroz.models.layers import CausalSelfAttention, PositionEmbedding, SoftmaxOnLast
from penroz.models.mapper import Mapper
from penroz.ops import sampling as samp_ops
from penroz.ops import fused as fused_ops
from penroz.parallel import dist as ddp
from penroz.parallel.launcher import maybe_inject_fault
from penroz.utils import checkpoint as ckpt
from penroz.utils import diagnostics

log = logging.getLogger(__name__)
MODELS_FOLDER = ckpt.MODELS_FOLDER


def _status(code: str, message: str) -> dict:
    return {"code": code, "dt": dt.now().isoformat(), "message": message}


class NeuralNetworkModel(nn.Module):
    _detect_shm_path = staticmethod(ckpt.detect_shm_path)
    SHM_PATH = ckpt.detect_shm_path()

    def __init__(self, model_id: str, mapper: Mapper):
        super().__init__()
        self.model_id = model_id
        self.mapper = mapper
        self.layers = nn.ModuleList(self.mapper.to_layers())
        self._is_softmax_last = isinstance(self.layers[-1], nn.Softmax)
        self.optimizer = self.mapper.to_optimizer(self.parameters())
        self.progress = []
        self.avg_cost = None
        self.avg_cost_history = []
        self.stats = None
        self.status = _status("Created", "Model created but not yet trained.")
        self._executor = None

    # ------------------------------------------------------------------ properties
    @property
    def _weights(self) -> list[Tensor | None]:
        return [p if p.ndim == 2 else None for p in self.parameters()]

    @torch.no_grad()
    def _snapshot_weights(self) -> list[Tensor | None]:
        """The weights before an epoch, for its weight-update ratios (reference
        ``neural_net_model.py:684-703``): copied into one buffer kept across epochs by a single
        multi-tensor copy, instead of one allocation + copy kernel per weight every epoch."""
        ws = self._weights
        live = [w for w in ws if w is not None]
        key = tuple((w.dtype, w.device, w.numel()) for w in live)
        cache = self.__dict__.get("_snap")
        if cache is None or cache[0] != key:
            bufs = {}
            views = []
            for w in live:
                k = (w.dtype, w.device)
                bufs[k] = bufs.get(k, 0) + w.numel()
            flat = {k: torch.empty(n, dtype=k[0], device=k[1]) for k, n in bufs.items()}
            off = dict.fromkeys(flat, 0)
            for w in live:
                k = (w.dtype, w.device)
                views.append(flat[k][off[k]:off[k] + w.numel()].view_as(w))
                off[k] += w.numel()
            cache = self.__dict__["_snap"] = (key, views)
        views = cache[1]
        if live:
            torch._foreach_copy_(views, [w.detach() for w in live])
        it = iter(views)
        return [next(it) if w is not None else None for w in ws]

    @property
    def num_params(self) -> int:
        return sum(p.numel() for p in self.parameters())

    def to(self, device: str = None, dtype: torch.dtype = None):
        if device is not None:
            if ddp.is_ddp() and device == "cuda":
                device = f"cuda:{ddp.ddp_local_rank()}"
                torch.cuda.set_device(device)
            super().to(device)
        if dtype is not None:
            super().to(dtype=dtype)
        return self

    # ------------------------------------------------------------------ persistence
    @classmethod
    def get_model_path(cls, model_id):
        return os.path.join(MODELS_FOLDER, f"model_{model_id}.pth")

    def _progress_doc(self) -> dict:
        return {"progress": self.progress, "average_cost": self.avg_cost,
                "average_cost_history": self.avg_cost_history, "status": self.status}

    def serialize(self):
        os.makedirs(MODELS_FOLDER, exist_ok=True)
        model_path = self.get_model_path(self.model_id)
        shm_path = os.path.join(self.SHM_PATH, model_path)
        data = {
            "layers": self.mapper.layers,
            "state": {k: v.detach().cpu() for k, v in self.state_dict().items()},
            "optim": self.mapper.optimizer,
            "optim_state": _optim_state_to_cpu(self.optimizer.state_dict()),
            "progress": self.progress,
            "average_cost": self.avg_cost,
            "average_cost_history": self.avg_cost_history,
            "stats": self.stats,
            "status": self.status,
        }
        if ddp.master_proc():
            log.info(f"Caching model to {shm_path}...")
        ckpt.atomic_torch_save(data, shm_path)
        for base in (shm_path, model_path):  # small JSON sidecars: /progress and /stats never load weights
            ckpt.atomic_json(self._progress_doc(), ckpt.sidecar_path(base))
            ckpt.atomic_json({"stats": self.stats}, ckpt.sidecar_path(base, "stats"))
        ckpt.flush_async(shm_path, model_path)

    @classmethod
    def _ensure_cached(cls, model_id: str) -> str:
        model_path = cls.get_model_path(model_id)
        shm_path = os.path.join(cls.SHM_PATH, model_path)
        if not os.path.exists(shm_path):
            if ddp.master_proc():
                log.info(f"Cache miss: copying from {model_path}")
                ckpt.atomic_copy(model_path, shm_path)
                side = ckpt.sidecar_path(model_path)
                if os.path.exists(side):
                    ckpt.atomic_copy(side, ckpt.sidecar_path(shm_path))
            if ddp.is_ddp() and dist.is_available() and dist.is_initialized():
                dist.barrier()
        return shm_path

    @classmethod
    def deserialize(cls, model_id: str):
        try:
            shm_path = cls._ensure_cached(model_id)
            data = ckpt.load(shm_path)
        except FileNotFoundError as e:
            log.error(f"File not found error occurred: {e}")
            raise KeyError(f"Model {model_id} not created yet.")
        model = cls(model_id, Mapper(data["layers"], data["optim"]))
        saved_dtype = next((v.dtype for v in data["state"].values()
                            if isinstance(v, Tensor) and v.is_floating_point()), None)
        if saved_dtype is not None and saved_dtype != torch.float32:
            model.to(dtype=saved_dtype)
        model.load_state_dict(data["state"])
        model.optimizer.load_state_dict(data["optim_state"])
        model.progress = data["progress"]
        model.avg_cost = data["average_cost"]
        model.avg_cost_history = data["average_cost_history"]
        model.stats = data["stats"]
        model.status = data["status"]
        return model

    @classmethod
    def read_progress(cls, model_id: str) -> dict:
        """Progress/status without loading weights (sidecar), falling back to the checkpoint."""
        model_path = cls.get_model_path(model_id)
        for p in (ckpt.sidecar_path(os.path.join(cls.SHM_PATH, model_path)), ckpt.sidecar_path(model_path)):
            if os.path.exists(p):
                import json
                with open(p) as f:
                    return json.load(f)
        m = cls.deserialize(model_id)
        return m._progress_doc()

    @classmethod
    def read_stats(cls, model_id: str):
        """Training stats from the stats sidecar, falling back to the checkpoint."""
        model_path = cls.get_model_path(model_id)
        for p in (ckpt.sidecar_path(os.path.join(cls.SHM_PATH, model_path), "stats"),
                  ckpt.sidecar_path(model_path, "stats")):
            if os.path.exists(p):
                import json
                with open(p) as f:
                    return json.load(f)["stats"]
        return cls.deserialize(model_id).stats

    @classmethod
    def mark_status(cls, model_id: str, code: str, message: str):
        """Rewrite a stored model's status (e.g. ``Error`` after a worker crash)."""
        model = cls.deserialize(model_id)
        model.status = _status(code, message)
        model.serialize()
        ckpt.wait_flushes()

    @classmethod
    def delete(cls, model_id: str):
        model_path = cls.get_model_path(model_id)
        shm_path = os.path.join(cls.SHM_PATH, model_path)
        for p in (shm_path, ckpt.sidecar_path(shm_path), ckpt.sidecar_path(shm_path, "stats"), model_path,
                  ckpt.sidecar_path(model_path), ckpt.sidecar_path(model_path, "stats")):
            try:
                os.remove(p)
            except FileNotFoundError as e:
                if p == shm_path:
                    log.warning(f"Failed to delete: {e}")

    @classmethod
    def from_huggingface(cls, model_id: str, hf_repo_id: str, revision: Optional[str] = None,
                         device: str = "cpu") -> "NeuralNetworkModel":
        from transformers import AutoConfig, AutoModelForCausalLM
        log.info(f"Fetching HuggingFace config for {hf_repo_id} (revision={revision})")
        hf_config = AutoConfig.from_pretrained(hf_repo_id, revision=revision)
        hf_model = AutoModelForCausalLM.from_pretrained(hf_repo_id, revision=revision, dtype=torch.bfloat16,
                                                        low_cpu_mem_usage=True)
        hf_sd = hf_model.state_dict()
        del hf_model
        n_layer = Mapper.detect_hf_n_layer(hf_sd)
        if n_layer == 0:
            tc = getattr(hf_config, "text_config", hf_config)
            n_layer = getattr(tc, "n_layer", None) or getattr(tc, "num_hidden_layers", None)
        layers = Mapper.from_hf_config(hf_config, n_layer_override=n_layer)
        mapper = Mapper(layers, {"adamw": {"lr": 6e-4, "betas": [0.9, 0.95], "eps": 1e-8}})
        model = cls(model_id, mapper)
        model.to(dtype=torch.bfloat16)
        model.to(device)
        model.load_state_dict(Mapper.map_hf_state_dict_to_custom(hf_sd, n_layer, hf_config), strict=True)
        model.status = _status("Imported", f"Model imported from HuggingFace: {hf_repo_id}")
        model.serialize()
        return model

    # ------------------------------------------------------------------ forward
    def forward(self, input_tensor: Tensor, target: Tensor = None, skip_softmax=False) -> Tuple[list[Tensor], Tensor]:
        activations = []
        x = prev = input_tensor
        layers = self.layers[:-1] if skip_softmax and self._is_softmax_last else self.layers
        for layer in layers:
            prev = x
            x = layer(prev)
            activations.append(x)
        if target is None:
            cost = torch.empty(0)
        elif self._is_softmax_last:
            logits = x if skip_softmax else prev
            if logits.ndim > 2 and target.ndim > 1:
                logits = logits.reshape(-1, logits.size(-1))
                target = target.reshape(-1)
            cost = fused_ops.cross_entropy(logits, target)  # F.cross_entropy semantics; fused HIP on GPU bf16
        else:
            cost = nn.functional.mse_loss(x, target)
        return activations, cost

    @torch.no_grad()
    def compute_output(self, input_data: list, target: list | int | None = None) -> Tuple[list, float | None]:
        self.eval()
        p0 = next(self.parameters())
        x = torch.tensor(input_data, device=p0.device)
        if x.is_floating_point():
            x = x.to(p0.dtype)
        if target is not None:
            target = torch.tensor(target, device=p0.device)
            if target.is_floating_point():
                target = target.to(p0.dtype)
        activations, cost = self(x, target)
        return activations[-1].float().tolist(), (cost.item() if cost.numel() > 0 else None)

    # ------------------------------------------------------------------ evaluation
    @torch.no_grad()
    def evaluate_model(self, dataset_id: str, target_dataset_id: str | None, shard: int,
                       epochs: int, batch_size: int, block_size: int, step_size: int) -> float:
        from penroz.utils.loaders import Loader
        self.eval()
        buffer_size = batch_size * block_size
        world = ddp.ddp_world_size()
        num_steps = max(1, buffer_size // (step_size * block_size * world))
        begin_idx, idx_offset = buffer_size * ddp.ddp_rank(), buffer_size * world
        loader = Loader(dataset_id, shard, begin_idx, buffer_size, idx_offset)
        target_loader = Loader(target_dataset_id, shard, begin_idx, buffer_size, idx_offset) \
            if target_dataset_id is not None else None
        device = next(self.parameters()).device
        executor = self._get_executor(device)
        total = torch.zeros((), device=device, dtype=torch.float32)
        for _ in range(epochs):
            if target_loader is None:
                inp, tgt = loader.next_batch()
            else:
                inp, _ = loader.next_batch(target_offset=0)
                tgt, _ = target_loader.next_batch(target_offset=0)
            x = torch.as_tensor(np.asarray(inp), dtype=torch.long).view(batch_size, block_size).to(device)
            y = torch.as_tensor(np.asarray(tgt), dtype=torch.long).view(batch_size, block_size).to(device)
            for _ in range(num_steps):
                if executor is not None:
                    step_cost = executor.eval_loss(x, y)
                else:
                    with self._autocast(device):
                        _, step_cost = self(x, y, skip_softmax=True)
                total += step_cost.float() / (epochs * num_steps)
        if ddp.use_ddp(device.type) and dist.is_initialized():
            ddp.ddp_all_reduce(total)
        avg = total.item()
        if ddp.master_proc():
            log.info(f"Model {self.model_id}: For {epochs} evaluation(s) Avg Cost: {avg:.4f}")
        return avg

    # ------------------------------------------------------------------ generation
    def _find_attention_layers(self) -> list[CausalSelfAttention]:
        return [m for m in self.modules() if isinstance(m, CausalSelfAttention)]

    def _find_position_embeddings(self) -> list[PositionEmbedding]:
        return [m for m in self.modules() if isinstance(m, PositionEmbedding)]

    def _attach_kv_cache(self, capacity: int | None = None) -> tuple[KVCache | None, list[PositionEmbedding]]:
        attn = self._find_attention_layers()
        pos = self._find_position_embeddings()
        if not attn:
            return None, pos
        cache = create_kv_cache(len(attn), capacity)
        for i, a in enumerate(attn):
            a.set_kv_cache(cache, i)
        return cache, pos

    def _forward_nocache(self, x: Tensor):
        """Full-context forward with any attached KV cache temporarily detached (testing aid)."""
        attn = self._find_attention_layers()
        pos = self._find_position_embeddings()
        saved = [(a._kv_cache, a._layer_idx) for a in attn]
        offs = [p.position_offset for p in pos]
        for a in attn:
            a.set_kv_cache(None, 0)
        for p in pos:
            p.position_offset = 0
        try:
            return self(x, skip_softmax=True)
        finally:
            for a, (c, i) in zip(attn, saved):
                a.set_kv_cache(c, i)
            for p, o in zip(pos, offs):
                p.position_offset = o

    def _detach_kv_cache(self, pos_embeddings=None):
        for a in self._find_attention_layers():
            a.set_kv_cache(None, 0)
        for p in (pos_embeddings or self._find_position_embeddings()):
            p.position_offset = 0

    def _prepare_generation(self, input_context: list, max_new_tokens: int, temperature: float, top_k: int | None):
        self.eval()
        device = next(self.parameters()).device
        context = torch.tensor(input_context, dtype=torch.long, device=device)
        if context.ndim == 1:
            context = context.unsqueeze(0)
        top_k_msg = "" if top_k is None else f" top {top_k}"
        log.info(f"Generating at most {max_new_tokens}{top_k_msg} tokens with {temperature} temperature "
                 f"using device {device}")
        softmax_layer = self.layers[-1] if self._is_softmax_last else SoftmaxOnLast(dim=-1)
        return context, softmax_layer

    @torch.inference_mode()
    def _generate_next_token(self, context: Tensor, block_size: int, temperature: float, top_k: int | None,
                             softmax_layer=None, kv_cache: KVCache | None = None,
                             pos_embeddings: list[PositionEmbedding] | None = None) -> Tensor:
        if kv_cache is not None and kv_cache.seq_len() > 0:
            if kv_cache.seq_len() >= block_size:
                # sliding window: clear and re-prefill the last block_size tokens
                kv_cache.clear()
                model_input = context[:, -block_size:]
                for p in (pos_embeddings or []):
                    p.position_offset = 0
            else:
                model_input = context[:, -1:]
                for p in (pos_embeddings or []):
                    p.position_offset = kv_cache.seq_len()
        else:
            model_input = context[:, -block_size:]
        activations, _ = self(model_input, skip_softmax=True)
        logits = activations[-1]
        last = logits[:, -1, :] if logits.ndim == 3 else logits
        return samp_ops.sample(last, temperature, top_k)

    @torch.inference_mode()
    def generate_tokens(self, input_context: list, block_size: int, max_new_tokens: int,
                        temperature=1.0, top_k: int | None = None, stop_token: int | None = None) -> list:
        return [t for t in self._generate(input_context, block_size, max_new_tokens, temperature, top_k,
                                          stop_token, full_context=True)][-1]

    @torch.inference_mode()
    def generate_tokens_stream(self, input_context: list, block_size: int, max_new_tokens: int,
                               temperature=1.0, top_k: int | None = None, stop_token: int | None = None):
        log.info("Streaming token generation started")
        for tok in self._generate(input_context, block_size, max_new_tokens, temperature, top_k, stop_token,
                                  full_context=False):
            yield tok
        log.info("Streaming token generation completed")

    def _token_bursts(self, context: Tensor, block_size: int, max_new_tokens: int, temperature, top_k,
                      softmax_layer, burst: int):
        """Yield [rows, k] blocks of new tokens (device). On the GPU the decode steps replay a
        captured HIP graph (``graph_decode.py``); prefill and the sliding-window re-prefill
        (cache full) run eagerly, exactly as the per-token path."""
        from penroz.models import graph_decode
        rows = context.shape[0]
        dec = graph_decode.get_decoder(self, rows, block_size, temperature, top_k)
        if dec is None:
            cache, pos = self._attach_kv_cache(capacity=block_size)
        else:
            # one seed per generate call, drawn from torch's generator before any token: graph-
            # sampled tokens depend on (seed, absolute index, row) only (graph_decode.begin)
            dec.begin(int(torch.randint(0, 2 ** 62, (1,)).item()) if temperature else 0)
            dec.attach()
            cache, pos = dec.cache, dec.pos_layers
            cache.clear()
        try:
            remaining = max_new_tokens
            produced = 0
            last = None
            while remaining > 0:
                n = cache.seq_len() if cache is not None else 0
                if dec is None or n == 0 or n >= block_size:
                    new = self._generate_next_token(context, block_size, temperature, top_k, softmax_layer, cache,
                                                    pos)
                    for p in pos:
                        p.position_offset = 0
                else:
                    k = min(remaining, block_size - n, burst)
                    new = dec.run(last, k, start=produced)
                context = torch.cat((context, new.to(context.device)), dim=1)
                last = context[:, -1:]
                remaining -= new.shape[1]
                produced += new.shape[1]
                yield new
        finally:
            if cache is not None:
                cache.log_metrics()
            if dec is None:
                self._detach_kv_cache(pos)
            else:
                dec.detach()

    def _generate(self, input_context, block_size, max_new_tokens, temperature, top_k, stop_token, full_context):
        context, softmax_layer = self._prepare_generation(input_context, max_new_tokens, temperature, top_k)
        rows = context.shape[0]
        generated = []
        done = torch.zeros(rows, dtype=torch.bool)
        burst = 1 if (not full_context or stop_token is not None) else max_new_tokens
        stopped = False
        with torch.inference_mode():
            for new in self._token_bursts(context, block_size, max_new_tokens, temperature, top_k, softmax_layer,
                                          burst):
                toks = new.tolist()
                for j in range(new.shape[1]):
                    col = [r[j] for r in toks]
                    context = torch.cat((context, new[:, j:j + 1].to(context.device)), dim=1)
                    generated.append(col[0])
                    if not full_context:
                        yield col[0]
                    if stop_token is not None:
                        done |= torch.tensor([t == stop_token for t in col])
                        if bool(done[0]) and (rows == 1 or bool(done.all())):
                            stopped = True
                            break
                if stopped:
                    break
        if full_context:
            yield context[0].tolist()

    def _generate_eager(self, input_context, block_size, max_new_tokens, temperature, top_k, stop_token,
                        full_context):
        """Per-token path (kept for A/B and as the reference-shaped loop)."""
        context, softmax_layer = self._prepare_generation(input_context, max_new_tokens, temperature, top_k)
        cache, pos = self._attach_kv_cache(capacity=block_size)
        rows = context.shape[0]
        generated = []
        done = torch.zeros(rows, dtype=torch.bool)
        try:
            with torch.inference_mode():
                for _ in range(max_new_tokens):
                    nxt = self._generate_next_token(context, block_size, temperature, top_k, softmax_layer, cache, pos)
                    context = torch.cat((context, nxt.to(context.device)), dim=1)
                    toks = nxt.view(-1).tolist()
                    generated.append(toks[0])
                    if not full_context:
                        yield toks[0]
                    if stop_token is not None:
                        done |= torch.tensor([t == stop_token for t in toks])
                        if bool(done[0]) and (rows == 1 or bool(done.all())):
                            break
        finally:
            if cache is not None:
                cache.log_metrics()
            self._detach_kv_cache(pos)
        if full_context:
            yield context[0].tolist()

    @torch.inference_mode()
    def generate_batch(self, input_context: list, block_size: int, max_new_tokens: int, temperature=1.0,
                       top_k: int | None = None, stop_token: int | None = None) -> list[list[int]]:
        """All rows' contexts (the reference returns row 0 only — bug 5)."""
        context, sm = self._prepare_generation(input_context, max_new_tokens, temperature, top_k)
        burst = 32 if stop_token is not None else max_new_tokens
        for new in self._token_bursts(context, block_size, max_new_tokens, temperature, top_k, sm, burst):
            if stop_token is not None:
                hit = (new == stop_token).all(dim=0).nonzero()
                if hit.numel():
                    context = torch.cat((context, new[:, :int(hit[0]) + 1].to(context.device)), dim=1)
                    break
            context = torch.cat((context, new.to(context.device)), dim=1)
        return context.tolist()

    # ------------------------------------------------------------------ training
    @classmethod
    def train_model_on_device(cls, model_id: str, device: str, dataset_id: str, shard: int,
                              epochs: int, batch_size: int, block_size: int, step_size: int):
        if ddp.is_ddp():
            ddp.reconfig_logging()
            log.info(f"DDP local rank {ddp.ddp_local_rank()} - training model {model_id} on device {device} "
                     f"with backend {ddp.backend_for(device)}")
            if str(device).startswith("cuda"):
                torch.cuda.set_device(ddp.ddp_local_rank())
            ddp.init_process_group(device)
        model = cls.deserialize(model_id)
        model.to(device)
        actual = next(model.parameters()).device
        for state in model.optimizer.state.values():
            for k, v in state.items():
                if isinstance(v, Tensor) and k != "step":
                    state[k] = v.to(actual)
        try:
            model.train_model(dataset_id, shard, epochs, batch_size, block_size, step_size)
        finally:
            ckpt.wait_flushes()
            if ddp.is_ddp() and dist.is_initialized():
                dist.destroy_process_group()

    @staticmethod
    def amp_dtype(device) -> torch.dtype | None:
        """Autocast dtype on the GPU, as the reference picks it (``neural_net_model.py:570-575``):
        bf16 where the device supports it (every MI355X), else fp16 with a GradScaler.
        ``PENROZ_AMP_DTYPE=fp16`` forces the fp16 + GradScaler path (generic engine) for parity
        runs of that fallback; ``bf16`` forces bf16."""
        if device.type != "cuda":
            return None
        env = os.environ.get("PENROZ_AMP_DTYPE", "auto").lower()
        if env in ("fp16", "float16", "half"):
            return torch.float16
        if env in ("bf16", "bfloat16"):
            return torch.bfloat16
        return torch.bfloat16 if torch.cuda.is_bf16_supported() else torch.float16

    @staticmethod
    def _autocast(device):
        dtype = NeuralNetworkModel.amp_dtype(device)
        if dtype is not None:
            return torch.amp.autocast("cuda", dtype=dtype)
        return nullcontext()

    def _engine(self, device) -> str:
        eng = os.environ.get("PENROZ_ENGINE", "auto")
        if self.amp_dtype(device) == torch.float16:
            return "reference" if eng == "reference" else "generic"  # the fused executor is bf16-only
        if eng == "auto":
            return "fused" if device.type == "cuda" and self._executor_class() is not None else "generic"
        return eng

    def _executor_class(self):
        """The fused executor this layer list lowers to (GPT-2 or Gemma pattern), or None."""
        from penroz.models.executor import GPTExecutor
        from penroz.models.gemma_executor import GemmaExecutor
        for cls in (GPTExecutor, GemmaExecutor):
            if cls.match(self) is not None:
                return cls
        return None

    def _get_executor(self, device):
        if device.type != "cuda" or self._engine(device) != "fused":
            return None
        if self._executor is None or self._executor.device != device:
            cls = self._executor_class()
            if cls is None:
                raise ValueError("PENROZ_ENGINE=fused needs a GPT-2 or Gemma pattern layer list")
            self._executor = cls(self, device)
        return self._executor

    def train_model(self, dataset_id: str, shard: int, epochs: int, batch_size: int, block_size: int,
                    step_size: int):
        from penroz.utils.loaders import Loader
        device = next(self.parameters()).device
        engine = self._engine(device)
        if ddp.master_proc():
            log.info(f"Training model using device {device} (engine {engine})")
        world = ddp.ddp_world_size()
        buffer_size = batch_size * block_size
        num_steps = max(1, buffer_size // (step_size * block_size * world))
        begin_idx, idx_offset = buffer_size * ddp.ddp_rank(), buffer_size * world
        log.info(f"Training starts from idx {begin_idx} of ds {dataset_id} at shard {shard} offset every {idx_offset}")
        loader = Loader(dataset_id, begin_shard=shard, begin_idx=begin_idx, buffer_size=buffer_size,
                        idx_offset=idx_offset)

        self.progress = []
        self.stats = None
        self.status = _status("Training", "Model is currently being trained.")
        last_serialized = None
        if ddp.master_proc():
            self.serialize()
            last_serialized = time.time()

        distributed = ddp.use_ddp(device.type) and dist.is_initialized()
        runner = _make_runner(self, engine, device, distributed)
        self.train()

        copy_stream = None
        if device.type == "cuda" and os.environ.get("PENROZ_COPY_STREAM", "1") != "0":
            from penroz.models.executor import shared_stream
            copy_stream = shared_stream(device, "copy")

        def fetch():
            """The next micro-batch on the device. Called right after the previous micro-step is
            enqueued, so the host-side shard read / pin / copy overlaps the GPU executing that step
            (profiles/notes_r6.md). On the GPU the copy runs on its own stream: on the compute stream
            it would wait behind the step just enqueued and then hold the next step's first kernel
            for the copy's own latency (Gemma-3 1B bench: 70.09 -> 69.75 ms/step). The batch order
            is the loader's, unchanged."""
            inp, tgt = loader.next_batch()
            x = torch.as_tensor(np.asarray(inp), dtype=torch.long).view(batch_size, block_size)
            y = torch.as_tensor(np.asarray(tgt), dtype=torch.long).view(batch_size, block_size)
            if copy_stream is None and device.type == "cuda":
                return x.pin_memory().to(device, non_blocking=True), y.pin_memory().to(device, non_blocking=True), None
            if device.type == "cuda":
                with torch.cuda.stream(copy_stream):
                    xd = x.pin_memory().to(device, non_blocking=True)
                    yd = y.pin_memory().to(device, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(copy_stream)
                return xd, yd, ev
            return x.to(device), y.to(device), None

        def ready(batch):
            """A fetched batch for the compute stream (which waits for its copy)."""
            x, y, ev = batch
            if ev is not None:
                cur = torch.cuda.current_stream(device)
                cur.wait_event(ev)
                x.record_stream(cur)
                y.record_stream(cur)
            return x, y

        # GPU: an epoch's bookkeeping (cost, weight-update ratios, duration) is read back one epoch
        # LATER, from pinned copies and events recorded behind its step, so the host never drains
        # the device between epochs: the next epoch's work is already queued while the previous
        # one's numbers are finalised (a per-epoch synchronize left the GPU idle ≈ 3-5 ms per
        # epoch: the --via-runtime ratio 0.91, profiles/notes_r6.md). PENROZ_EPOCH_SYNC=1: the
        # synchronous loop. Durations are then GPU-timeline epoch spans (event to event).
        lazy = device.type == "cuda" and os.environ.get("PENROZ_EPOCH_SYNC", "0") != "1"
        every = max(1, epochs // 100)
        pend = None

        def finish(pd):
            """Record one finished epoch (waits for that epoch's events only)."""
            ep, ev0, ev1, cost_h, rat, t_host = pd
            if ev1 is not None:
                ev1.synchronize()
                secs = max(ev0.elapsed_time(ev1) / 1e3, 1e-9)
            else:
                secs = t_host
            progress_cost = float(cost_h.item())
            if ep % every == 0:
                self.progress.append({
                    "dt": dt.now().isoformat(), "epoch": ep + 1, "durationInSecs": secs,
                    "speedPerSec": buffer_size / secs,
                    "tokensPerSec": num_steps * world * buffer_size / secs,
                    "cost": progress_cost,
                    "weight_upd_ratio": diagnostics.finish_update_ratios(rat) if rat is not None else [],
                })
            log.info(f"Model {self.model_id}: Training Epoch {ep + 1}, Cost: {progress_cost:.4f}, "
                     f"Duration: {secs:.2f} secs, Speed: {buffer_size / secs:.2f} tokens/sec")

        nxt = fetch() if epochs > 0 else None
        for epoch in range(epochs):
            t0 = time.time()
            long_training = last_serialized is not None and (t0 - last_serialized >= 10)
            capture = ddp.master_proc() and (epoch + 1 == epochs or long_training)
            record = ddp.master_proc() and epoch % every == 0
            ev0 = None
            if lazy and ddp.master_proc():
                ev0 = torch.cuda.Event(enable_timing=True)
                ev0.record()
            prev = self._snapshot_weights() if record and os.environ.get("PENROZ_DIAG_SNAPSHOT", "1") != "0" \
                else []
            runner.zero_grad()
            cost = torch.zeros((), device=device, dtype=torch.float32)
            try:
                for step in range(num_steps):
                    maybe_inject_fault(epoch * num_steps + step)
                    x, y = ready(nxt)
                    cost += runner.micro_step(x, y, 1.0 / num_steps, first=step == 0,
                                              last=step == num_steps - 1, capture=capture)
                    if epoch + 1 < epochs or step + 1 < num_steps:
                        nxt = fetch()
            except Exception as exc:
                if ddp.master_proc():
                    if pend is not None:  # the previous epoch's record is complete: keep it
                        try:
                            finish(pend)
                        except Exception:  # the device may be in a failed state
                            pass
                        pend = None
                    log.error(f"Model {self.model_id}: Training Epoch {epoch + 1} failed: {exc}")
                    self.status = _status("Error", f"Training epoch {epoch + 1} failed: {exc}")
                    self.serialize()
                raise
            if distributed:
                ddp.ddp_all_reduce(cost)
            runner.step()
            if lazy:
                if ddp.master_proc():
                    # the ratios of this epoch's update, on the device behind its step; host copies
                    # land in pinned memory, read by finish() one epoch later
                    rat = diagnostics.start_update_ratios(prev, self._weights) if record and prev else None
                    cost_h = torch.empty((), dtype=torch.float32, pin_memory=True)
                    cost_h.copy_(cost, non_blocking=True)
                    ev1 = torch.cuda.Event(enable_timing=True)
                    ev1.record()
                    if pend is not None:
                        finish(pend)
                    pend = (epoch, ev0, ev1, cost_h, rat, None)
            else:
                if device.type == "cuda":
                    torch.cuda.synchronize()
                if ddp.master_proc():
                    rat = diagnostics.start_update_ratios(prev, self._weights) if record and prev else None
                    finish((epoch, None, None, cost.detach().cpu(), rat, time.time() - t0))
            if ddp.master_proc() and long_training:
                if pend is not None:
                    finish(pend)
                    pend = None
                self._record_training_overall_progress(runner.captured(), runner.grad_of)
                self.serialize()
                last_serialized = time.time()
        if pend is not None:
            finish(pend)

        if ddp.master_proc():
            self.status = _status("Trained", f"Model trained for {epochs} epochs.")
            log.info(f"Model {self.model_id}: Done training for {epochs} epochs.")
            self._record_training_overall_progress(runner.captured(), runner.grad_of)
            self.serialize()
        runner.close()
        ckpt.wait_flushes()  # the disk copy is complete when training returns

    @torch.no_grad()
    def _record_training_overall_progress(self, captured, grad_of=None):
        costs = [p["cost"] for p in self.progress]
        avg_progress_cost = sum(costs) / len(costs) if costs else 0.0
        self.avg_cost = ((self.avg_cost or avg_progress_cost) + avg_progress_cost) / 2.0
        self.avg_cost_history.append(self.avg_cost)
        if len(self.avg_cost_history) > 100:
            self.avg_cost_history.pop(random.randint(1, 98))
        algos, acts = captured
        self.stats = diagnostics.training_stats(algos, acts, self._weights, grad_of)
        log.info(f"Model {self.model_id} - Cost: {avg_progress_cost:.4f} Overall Cost: {self.avg_cost:.4f}")


def _optim_state_to_cpu(sd: dict) -> dict:
    out = {"state": {}, "param_groups": sd["param_groups"]}
    for k, st in sd["state"].items():
        out["state"][k] = {n: (v.detach().cpu().clone() if isinstance(v, Tensor) else v) for n, v in st.items()}
    return out


# ---------------------------------------------------------------------------- step runners
class _GenericRunner:
    """Module forward + autograd backward (+ our bucketed reducer under DDP)."""

    def __init__(self, model: NeuralNetworkModel, device, distributed: bool, reference: bool = False):
        self.model = model
        self.device = device
        self.reference = reference
        self.amp = NeuralNetworkModel._autocast(device)
        # fp16 autocast needs loss scaling (reference neural_net_model.py:573-575, 650-675)
        self.scaler = torch.amp.GradScaler("cuda") if NeuralNetworkModel.amp_dtype(device) == torch.float16 else None
        self.reducer = None
        self.ddp_model = None
        if distributed:
            if reference:
                self.ddp_model = nn.parallel.DistributedDataParallel(model)
            else:
                from penroz.parallel.reducer import HookedReducer, row_sparse_tables, sparse_rows_enabled
                self._broadcast_params()
                sparse = row_sparse_tables(model) if sparse_rows_enabled(dist.get_backend()) else None
                self.reducer = HookedReducer(list(model.parameters()), sparse_rows=sparse)
        self._acts: list[Tensor] = []
        self._algos = [l.__class__.__name__.lower() for l in model.layers]

    def _broadcast_params(self):
        for p in self.model.parameters():
            dist.broadcast(p.data, src=0)

    def zero_grad(self):
        if self.reducer is not None:
            self.reducer.zero_grad()
        else:
            self.model.optimizer.zero_grad()
        self._acts = []

    def micro_step(self, x, y, scale, first, last, capture):
        fwd = self.ddp_model if self.ddp_model is not None else self.model
        if self.ddp_model is not None:
            self.ddp_model.require_backward_grad_sync = last
        if self.reducer is not None:
            self.reducer.sync = last
        with self.amp if self.device.type == "cuda" else nullcontext():
            acts, loss = fwd(x, y, skip_softmax=True)
            scaled = loss * scale if scale != 1.0 else loss
        if capture and not self._acts:  # stats use the first micro-step's activations
            for a in acts:
                a.retain_grad()
            self._acts.extend(acts)
        (self.scaler.scale(scaled) if self.scaler is not None else scaled).backward()
        if last and self.reducer is not None:
            self.reducer.finish()
        return scaled.detach().float()

    def step(self):
        if self.scaler is None:
            self.model.optimizer.step()
            return
        # unscale + inf/nan check, skipped step on overflow; the captured activation gradients
        # (dashboard stats) were scaled too: unscale them with the scale of this step
        self.scaler.step(self.model.optimizer)
        inv = 1.0 / self.scaler.get_scale()
        for a in self._acts:
            if a.grad is not None:
                a.grad.mul_(inv)
        self.scaler.update()

    @staticmethod
    def grad_of(p):
        return p.grad

    def captured(self):
        return self._algos, [(a, a.grad) for a in self._acts]

    def close(self):
        if self.reducer is not None:
            self.reducer.remove()


class _FusedRunner:
    def __init__(self, model: NeuralNetworkModel, device, distributed: bool):
        self.model = model
        self.exec = model._get_executor(device)
        self.exec.setup_training(distributed)

    def zero_grad(self):
        self.exec.zero_grad()

    def micro_step(self, x, y, scale, first, last, capture):
        # the last micro-step's backward may apply the optimizer per parameter segment (step()
        # always follows it in the training loop and the bench)
        return self.exec.train_micro_step(x, y, scale, sync=last, capture=capture, fuse_optimizer=last)

    def step(self):
        self.exec.optimizer_step()

    def grad_of(self, p):
        return self.exec.grad(p)

    def captured(self):
        return self.exec.captured()

    def close(self):
        self.exec.end_training()


def _make_runner(model, engine, device, distributed):
    from penroz.ops import _ext
    _ext.FORCE_TORCH = engine == "reference"
    if engine == "fused":
        return _FusedRunner(model, device, distributed)
    return _GenericRunner(model, device, distributed, reference=(engine == "reference"))
