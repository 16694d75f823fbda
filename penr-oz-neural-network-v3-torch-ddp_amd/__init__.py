"""penroz — an MI355X-native neural-network training and serving engine.

Capabilities follow ``derinworks/penr-oz-neural-network-v3-torch-ddp`` (JSON-layer models,
GPT-2/Gemma import, data-parallel training, KV-cache generation, a FastAPI service), while
the compute path is hand-written HIP for CDNA4 (gfx950) and gradient sync is RCCL over xGMI.

Layout:
  models/    layer library, JSON config compiler, HF import, model runtime, fused GPT executor
  ops/       Python front-ends of the HIP kernels (``penroz_kernels`` extension) + torch refs
  parallel/  rank helpers, process launcher, RCCL communicator and bucketed gradient reducer
  utils/     token shards / loaders, tokenizers, checkpoint IO, logging, diagnostics
  serve/     FastAPI application and dashboard
"""
__version__ = "0.1.0"
