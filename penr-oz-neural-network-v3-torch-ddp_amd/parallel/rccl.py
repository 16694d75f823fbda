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

    def __init__(self, group=None, key: str = "penroz_rccl_uid", channels: int = 0, proto: str = "", algo: str = ""):
        mod = load_module()
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        store = dist.distributed_c10d._get_default_store()
        key = f"{key}_c{channels}_p{proto or 'default'}_a{algo or 'default'}"  # one unique id per communicator
        if rank == 0:
            store.set(key, mod.RcclComm.unique_id())
        uid = store.get(key)
        # the protocol (Simple / LL / LL128) and algorithm (Ring / Tree) are fixed per communicator:
        # RCCL reads NCCL_PROTO / NCCL_ALGO while tuning a communicator at init, so they are set for
        # this init only (a user's own setting is left alone when nothing is asked for).
        # Threading assumption: setenv is not safe against a concurrent getenv in another thread.
        # Forced arms are opt-in (PENROZ_COMM_SWEEP_ARMS=full, commtune.sweep_arms) and are built in the
        # first-contact sweep, before training starts, with no collective in flight on any other
        # communicator of this process (the sweep's own c10d agreement calls have returned).
        # That leaves only RCCL's idle proxy threads, which read NCCL_PROTO / NCCL_ALGO at init only.
        forced = {k: v for k, v in (("NCCL_PROTO", proto), ("NCCL_ALGO", algo)) if v}
        prev = {k: os.environ.get(k) for k in forced}
        os.environ.update(forced)
        try:
            self.comm = mod.RcclComm(bytes(uid), rank, world, torch.cuda.current_device(), channels)
        finally:
            for k, v in prev.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        self.rank, self.world, self.channels, self.proto, self.algo = rank, world, channels, proto, algo

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

    @staticmethod
    def default_algo() -> str:
        """Algorithm for :meth:`get` without an explicit one: ``PENROZ_RCCL_ALGO`` (set by the
        first-contact sweep when a forced algorithm beat RCCL's per-size choice), else "" = RCCL's."""
        return os.environ.get("PENROZ_RCCL_ALGO", "")

    @classmethod
    def get(cls, group=None, channels: int | None = None, proto: str | None = None,
            algo: str | None = None) -> "NativeComm":
        ch = cls.default_channels() if channels is None else channels
        pr = cls.default_proto() if proto is None else proto
        al = cls.default_algo() if algo is None else algo
        k = (id(group), ch, pr, al)
        if k not in cls._instances:
            cls._instances[k] = NativeComm(group, channels=ch, proto=pr, algo=al)
        return cls._instances[k]

    @classmethod
    def release(cls, group=None, keep: int | None = None, keep_proto: str = "", keep_algo: str = ""):
        """Destroy this group's communicators except the one with ``keep`` channels, protocol
        ``keep_proto`` and algorithm ``keep_algo`` (the sweep builds one per arm; only the chosen
        one stays alive)."""
        for k in [k for k in cls._instances if k[0] == id(group) and k[1:] != (keep, keep_proto, keep_algo)]:
            del cls._instances[k]

    @classmethod
    def drop(cls, group=None, channels: int = 0, proto: str = "", algo: str = "", abort: bool = False):
        """Destroy the one communicator of this group with that (channels, protocol, algorithm);
        ``abort``: ncclCommAbort first (a collective may be in flight that will never complete)."""
        c = cls._instances.pop((id(group), channels, proto, algo), None)
        if c is not None and abort:
            c.abort()

    @property
    def nranks(self) -> int:
        """The clique size RCCL reports for this communicator (``ncclCommCount``), not the world
        size the caller passed in."""
        return int(self.comm.nranks)

    @property
    def comm_rank(self) -> int:
        """This member's rank as RCCL reports it (``ncclCommUserRank``)."""
        return int(self.comm.comm_rank)

    @property
    def comm_device(self) -> int:
        """The HIP device RCCL bound this communicator to (``ncclCommCuDevice``)."""
        return int(self.comm.comm_device)

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

    def abort(self):
        """ncclCommAbort: drop the communicator without waiting for collectives in flight."""
        self.comm.abort()

    def broadcast(self, t: torch.Tensor, root: int = 0):
        self.comm.broadcast(t, root)
