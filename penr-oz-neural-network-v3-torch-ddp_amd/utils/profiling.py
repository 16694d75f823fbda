"""Tracing and profiling hooks (SURVEY §5.1 — the reference has none).

* ``trace_range(name)`` — a roctx range (ROCm's marker API, loaded from the ROCm runtime with
  ctypes: ``librocprofiler-sdk-roctx`` first, the legacy ``libroctx64`` otherwise). Ranges
  show up in ``rocprofv3 --marker-trace`` timelines around the executor's forward, backward,
  gradient all-reduce and optimizer phases. Enabled by ``PENROZ_ROCTX=1``; otherwise a no-op
  that costs one attribute check.
* ``profile_steps(step_fn, steps, out_dir)`` — runs ``step_fn`` under ``torch.profiler`` with
  CPU + GPU activities and writes a Chrome trace plus a per-kernel table (used by
  ``bench.py --profile DIR``).

Per-kernel GPU timings for committed profiles come from ``rocprofv3 --kernel-trace`` and
``bench/prof_summary.py``; hardware counters from ``rocprofv3 --pmc``.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

import torch

ENABLED = os.environ.get("PENROZ_ROCTX", "0") == "1"
_lib = None
_lib_tried = False


def _roctx():
    global _lib, _lib_tried
    if not _lib_tried:
        _lib_tried = True
        rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
        for name in ("librocprofiler-sdk-roctx.so.1", "libroctx64.so.4", "libroctx64.so"):
            for path in (os.path.join(rocm, "lib", name), name):
                try:
                    lib = ctypes.CDLL(path)
                    lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    lib.roctxRangePushA.restype = ctypes.c_int
                    lib.roctxRangePop.restype = ctypes.c_int
                    lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                    _lib = lib
                    return _lib
                except (OSError, AttributeError):
                    continue
    return _lib


def available() -> bool:
    return _roctx() is not None


@contextlib.contextmanager
def trace_range(name: str):
    if not ENABLED:
        yield
        return
    lib = _roctx()
    if lib is None:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()


def mark(name: str) -> None:
    if ENABLED and _roctx() is not None:
        _lib.roctxMarkA(name.encode())


def profile_steps(step_fn, steps: int, out_dir: str, row_limit: int = 40) -> str:
    """Run ``step_fn()`` ``steps`` times under torch.profiler; return the kernel table text."""
    os.makedirs(out_dir, exist_ok=True)
    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    with torch.profiler.profile(activities=acts, record_shapes=False) as prof:
        for _ in range(steps):
            step_fn()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    prof.export_chrome_trace(os.path.join(out_dir, "trace.json"))
    sort_key = "cuda_time_total" if torch.cuda.is_available() else "cpu_time_total"
    table = prof.key_averages().table(sort_by=sort_key, row_limit=row_limit)
    with open(os.path.join(out_dir, "kernels.txt"), "w") as f:
        f.write(table)
    return table
