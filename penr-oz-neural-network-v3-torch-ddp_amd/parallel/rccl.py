"""Python side of the native RCCL communicator (``csrc/comm/rccl_comm.cpp``).

Rank 0 creates an RCCL unique id and publishes it through the ``torch.distributed`` TCPStore;
every rank then builds its own ``ncclComm_t`` bound to its GPU and a high-priority HIP stream.
Used by :class:`penroz.parallel.reducer.GradReducer` when ``PENROZ_COMM=native``.
"""
from __future__ import annotations

import importlib
import os
import sys

import torch
import torch.distributed as dist

_REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
_BUILD_DIR = os.path.join(_REPO_ROOT, "build_ext")


def load_module():
    if _BUILD_DIR not in sys.path:
        sys.path.insert(0, _BUILD_DIR)
    return importlib.import_module("penroz_comm")


class NativeComm:
    _instances: dict = {}

    def __init__(self, group=None, key: str = "penroz_rccl_uid", channels: int = 0):
        mod = load_module()
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        store = dist.distributed_c10d._get_default_store()
        key = f"{key}_c{channels}"  # one unique id per communicator
        if rank == 0:
            store.set(key, mod.RcclComm.unique_id())
        uid = store.get(key)
        self.comm = mod.RcclComm(bytes(uid), rank, world, torch.cuda.current_device(), channels)
        self.rank, self.world, self.channels = rank, world, channels

    @staticmethod
    def default_channels() -> int:
        """Channel count for :meth:`get` without an explicit one: ``PENROZ_RCCL_CHANNELS`` (set
        by the first-contact sweep when a fixed count beat RCCL's own choice), else 0 = RCCL's."""
        return int(os.environ.get("PENROZ_RCCL_CHANNELS", "0") or 0)

    @classmethod
    def get(cls, group=None, channels: int | None = None) -> "NativeComm":
        ch = cls.default_channels() if channels is None else channels
        k = (id(group), ch)
        if k not in cls._instances:
            cls._instances[k] = NativeComm(group, channels=ch)
        return cls._instances[k]

    @classmethod
    def release(cls, group=None, keep: int | None = None):
        """Destroy this group's communicators except the one with ``keep`` channels (the sweep
        builds one per channel count; only the chosen one stays alive)."""
        for k in [k for k in cls._instances if k[0] == id(group) and k[1] != keep]:
            del cls._instances[k]

    def all_reduce_avg_async(self, t: torch.Tensor) -> int:
        """Launch; returns the handle :meth:`wait` takes."""
        return self.comm.all_reduce_avg_async(t)

    def wait(self, handle: int):
        """The current stream waits for that one collective."""
        self.comm.wait(handle)

    def reset_handles(self):
        self.comm.reset_handles()

    def wait_all(self):
        self.comm.wait_all()

    def broadcast(self, t: torch.Tensor, root: int = 0):
        self.comm.broadcast(t, root)
