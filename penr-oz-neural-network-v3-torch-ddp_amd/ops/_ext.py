"""Loader for the in-tree HIP extension ``penroz_kernels`` (built for gfx950 by ``setup.py``).

GPU tensors MUST go through the extension: if a CUDA (= HIP) tensor reaches an op and the
extension is not importable, :func:`kernels` raises instead of silently falling back to eager
PyTorch.  CPU tensors use the pure-torch reference implementations that the GPU parity tests
compare against.
"""
from __future__ import annotations

import importlib
import os
import sys

import torch

_REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# PENROZ_EXT_DIR: load the extension from another in-tree build (same-box A/B benchmarking)
_BUILD_DIR = os.environ.get("PENROZ_EXT_DIR") or os.path.join(_REPO_ROOT, "build_ext")

_mod = None
_err: Exception | None = None


def _load():
    global _mod, _err
    if _mod is not None or _err is not None:
        return _mod
    if _BUILD_DIR not in sys.path:
        sys.path.insert(0, _BUILD_DIR)
    try:
        # torch must be imported first so libc10_hip / libamdhip64 are already mapped
        _mod = importlib.import_module("penroz_kernels")
    except Exception as e:  # pragma: no cover - exercised on boxes without a build
        _err = e
    return _mod


def available() -> bool:
    return _load() is not None


def kernels():
    """Return the compiled kernel module or raise loudly."""
    mod = _load()
    if mod is None:
        raise RuntimeError(
            "penroz_kernels HIP extension is not built/importable "
            f"({_err!r}); run `python setup.py build_ext` (gfx950) before using GPU tensors")
    return mod


def on_gpu(*tensors) -> bool:
    return any(isinstance(t, torch.Tensor) and t.is_cuda for t in tensors)


# Set by the ``reference`` engine only (stock-PyTorch baseline for speedup claims).
FORCE_TORCH = False


def use_kernels(*tensors) -> bool:
    """True when the HIP path must be taken (any operand on the GPU)."""
    if FORCE_TORCH:
        return False
    if on_gpu(*tensors):
        kernels()  # raises if missing
        return True
    return False
