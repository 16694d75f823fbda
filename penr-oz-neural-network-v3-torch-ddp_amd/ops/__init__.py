"""Python front-ends of the HIP/CDNA4 kernels (``penroz_kernels`` extension).

Every op has two implementations: the HIP kernel (taken whenever an operand is a GPU tensor;
missing extension => hard error) and a pure-torch reference used on CPU and by the GPU parity
tests.  Modules: ``norms``, ``activations``, ``attention``, ``rope``, ``fused`` (embedding,
cross-entropy, AdamW, reductions, stats), ``sampling`` (+ int8 KV quantisation).
"""
from penroz.ops._ext import available, kernels  # noqa: F401
