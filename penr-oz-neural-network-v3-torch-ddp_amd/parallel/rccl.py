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

    def __init__(self, group=None, key: str = "penroz_rccl_uid", channels: int = 0, proto: str = ""):
        mod = load_module()
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        store = dist.distributed_c10d._get_default_store()
        key = f"{key}_c{channels}_p{proto or 'default'}"  # one unique id per communicator
        if rank == 0:
            store.set(key, mod.RcclComm.unique_id())
        uid = store.get(key)
        # the protocol (Simple / LL / LL128) is fixed per communicator: RCCL reads NCCL_PROTO while
        # tuning a communicator at init, so it is set for this init only (a user's own NCCL_PROTO
        # is left alone when no protocol is asked for)
        prev = os.environ.get("NCCL_PROTO")
        if proto:
            os.environ["NCCL_PROTO"] = proto
        try:
            self.comm = mod.RcclComm(bytes(uid), rank, world, torch.cuda.current_device(), channels)
        finally:
            if proto:
                if prev is None:
                    os.environ.pop("NCCL_PROTO", None)
                else:
                    os.environ["NCCL_PROTO"] = prev
        self.rank, self.world, self.channels, self.proto = rank, world, channels, proto

    @staticmethod
    def default_channels() -> int:
        """Channel count for :meth:`get` without an explicit one: ``PENROZ_RCCL_CHANNELS`` (set
        by the first-contact sweep when a fixed count beat RCCL's own choice), else 0 = RCCL's."""
        return int(os.environ.get("PENROZ_RCCL_CHANNELS", "0") or 0)

    @staticmethod
    def default_proto() -> str:
        """Protocol for :meth:`get` without an explicit one: ``PENROZ_RCCL_PROTO`` (set by the
        first-contact sweep when a forced protocol beat RCCL's per-size choice), else "" = RCCL's."""
        return os.environ.get("PENROZ_RCCL_PROTO", "")

    @classmethod
    def get(cls, group=None, channels: int | None = None, proto: str | None = None) -> "NativeComm":
        ch = cls.default_channels() if channels is None else channels
        pr = cls.default_proto() if proto is None else proto
        k = (id(group), ch, pr)
        if k not in cls._instances:
            cls._instances[k] = NativeComm(group, channels=ch, proto=pr)
        return cls._instances[k]

    @classmethod
    def release(cls, group=None, keep: int | None = None, keep_proto: str = ""):
        """Destroy this group's communicators except the one with ``keep`` channels and protocol
        ``keep_proto`` (the sweep builds one per arm; only the chosen one stays alive)."""
        for k in [k for k in cls._instances if k[0] == id(group) and (k[1], k[2]) != (keep, keep_proto)]:
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
