"""Checkpoint IO: atomic writes, shared-memory cache, background disk flush, progress sidecar.

Format parity with the reference (``neural_net_model.py:98-174``): ``torch.save`` (default pickle protocol) of a dict
with ``layers, state, optim, optim_state, progress, average_cost, average_cost_history,
stats, status`` at ``models/model_{id}.pth``, cached under ``{SHM}/models/``.

Fixes (SURVEY §5.2/§7.4 bug 10): every write goes to a temp file + ``os.replace`` (readers
never see a torn checkpoint); the disk flush copies atomically on a background *thread*
(never a fork of a GPU-initialised process); a small JSON sidecar carries progress/status so
``/progress`` does not ``torch.load`` a multi-GB file.  Loads use ``weights_only=True``.
"""
from __future__ import annotations

import json
import logging
import os
import platform
import shutil
import tempfile
import threading
import uuid

import torch

log = logging.getLogger(__name__)

MODELS_FOLDER = "models"


def detect_shm_path() -> str:
    override = os.environ.get("PENROZ_SHM_PATH")
    if override:
        return override
    system = platform.system()
    if system == "Linux":
        if os.path.isdir("/dev/shm") and os.access("/dev/shm", os.W_OK):
            return "/dev/shm"
    elif system == "Darwin":
        if os.path.isdir("/Volumes/RAMDisk") and os.access("/Volumes/RAMDisk", os.W_OK):
            return "/Volumes/RAMDisk"
    return tempfile.gettempdir()


def _atomic_write(path: str, writer):
    d = os.path.dirname(path) or "."
    os.makedirs(d, exist_ok=True)
    tmp = f"{path}.tmp-{os.getpid()}-{threading.get_ident()}-{uuid.uuid4().hex[:8]}"
    try:
        writer(tmp)
        os.replace(tmp, path)
    except BaseException:
        if os.path.exists(tmp):
            os.remove(tmp)
        raise


def atomic_torch_save(obj, path: str):
    # torch's default pickle protocol (2): the only one the weights_only loader accepts (the
    # reference writes protocol 5, which `torch.load(weights_only=True)` rejects)
    _atomic_write(path, lambda tmp: torch.save(obj, tmp))


def atomic_copy(src: str, dst: str):
    _atomic_write(dst, lambda tmp: shutil.copyfile(src, tmp))


def atomic_json(obj, path: str):
    def w(tmp):
        with open(tmp, "w") as f:
            json.dump(obj, f)
    _atomic_write(path, w)


_flush_lock = threading.Lock()
_flush_dst: dict[str, dict] = {}   # absolute destination -> {"gen", "lock"}
_flushers: list[threading.Thread] = []


def _flush_one(src: str, dst: str, st: dict, gen: int):
    with st["lock"]:  # one copy at a time per destination, in queue order
        if st["gen"] != gen:
            return  # a newer save of this destination is queued behind us: its copy wins
        try:
            atomic_copy(src, dst)
        except FileNotFoundError:  # the cached file was deleted (model deleted) before the flush
            log.warning(f"flush skipped: {src} no longer exists")


def flush_async(src: str, dst: str) -> threading.Thread:
    """Copy ``src`` to ``dst`` atomically on a background thread.

    Paths are made absolute when the flush is queued (a later ``chdir`` cannot redirect it).
    Flushes to one destination are serialised and carry a generation number: a flush whose
    save has been superseded before it starts copying is skipped, so the disk copy can only
    move forward to the newest snapshot, never back to an older one."""
    src, dst = os.path.abspath(src), os.path.abspath(dst)
    with _flush_lock:
        st = _flush_dst.setdefault(dst, {"gen": 0, "lock": threading.Lock()})
        st["gen"] += 1
        gen = st["gen"]
        t = threading.Thread(target=_flush_one, args=(src, dst, st, gen), name=f"flush-{os.path.basename(dst)}")
        _flushers[:] = [x for x in _flushers if x.is_alive()]
        _flushers.append(t)
    t.start()
    return t


def wait_flushes():
    with _flush_lock:
        pending = list(_flushers)
    for t in pending:
        t.join()
    with _flush_lock:
        _flushers[:] = [x for x in _flushers if x.is_alive()]


def sidecar_path(pth_path: str, kind: str = "progress") -> str:
    """``model_x.pth`` -> ``model_x.progress.json`` (progress/status) or ``model_x.stats.json``."""
    base = pth_path[:-4] if pth_path.endswith(".pth") else pth_path
    return f"{base}.{kind}.json"


def load(path: str) -> dict:
    """Safe load (``weights_only=True``). Legacy pickle-5 checkpoints written by the reference can
    only be read with ``PENROZ_TRUSTED_CHECKPOINTS=1`` (an explicit opt-in to full unpickling)."""
    try:
        return torch.load(path, weights_only=True, map_location="cpu")
    except Exception:
        if os.environ.get("PENROZ_TRUSTED_CHECKPOINTS") == "1":
            log.warning(f"loading {path} with full unpickling (PENROZ_TRUSTED_CHECKPOINTS=1)")
            return torch.load(path, weights_only=False, map_location="cpu")
        raise
