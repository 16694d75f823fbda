"""Single-node multi-process launcher: one worker per GPU (or a CPU split), TCPStore rendezvous.

Replaces the reference's torchelastic agent (``ddp.py:38-73``: ``elastic_launch`` with
``min/max_nodes=1, rdzv c10d, max_restarts=0, monitor_interval=5``) with a small native-first
design:
  * workers are spawned (``multiprocessing`` *spawn* context — a fresh interpreter, never a
    fork of a GPU-initialised process) with ``RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
    MASTER_PORT`` set; ``torch.distributed`` env:// rendezvous uses the TCPStore on rank 0;
  * ``OMP_NUM_THREADS`` is split across CPU workers (the reference's elastic launch left it
    unset: 7× slower CPU DDP at world_size 2);
  * a monitor polls worker exit codes; the first failure tears the group down and is
    *returned* (and reported through ``on_failure``) so the caller can mark the model
    ``Error`` instead of leaving it ``Training`` forever (reference bug 9);
  * rendezvous on the loopback interface: 127.0.0.1 on Linux; off Linux (macOS / Windows
    development boxes) the address family that actually works — ``::1`` when an IPv6 loopback
    socket connects, else 127.0.0.1 — with ``GLOO_USE_IPV6`` (and ``GLOO_SOCKET_IFNAME=lo0`` for
    IPv6 on macOS) set to match, as the reference does (``ddp.py:22-36, 59-68``); ``mps`` runs
    get ``PYTORCH_ENABLE_MPS_FALLBACK=1`` so collectives MPS lacks fall back to the CPU
    (``ddp.py:39-42``);
  * fault injection for tests: ``PENROZ_FAULT_RANK`` / ``PENROZ_FAULT_STEP`` make that rank
    exit with code 13 at that training step (checked in the runtime's loop).
"""
from __future__ import annotations

import logging
import multiprocessing as mp
from multiprocessing import connection as mp_connection
import os
import socket
import sys
import time
import traceback
from typing import Callable

import torch

log = logging.getLogger(__name__)

FAULT_EXIT_CODE = 13


def free_port(host: str = "127.0.0.1") -> int:
    family = socket.AF_INET6 if ":" in host else socket.AF_INET
    with socket.socket(family, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def detect_active_ip_family() -> str:
    """"ipv6" when a datagram socket can be connected to the IPv6 loopback, else "ipv4"."""
    if not socket.has_ipv6:
        return "ipv4"
    try:
        with socket.socket(socket.AF_INET6, socket.SOCK_DGRAM) as s:
            s.settimeout(0.5)
            s.connect(("::1", 1))
        return "ipv6"
    except OSError:
        return "ipv4"


def rendezvous_env(device: str, platform: str | None = None) -> tuple[str, dict]:
    """(loopback address, extra worker environment) for a single-node run on this platform."""
    platform = platform or sys.platform
    env: dict = {}
    if device == "mps":
        env["PYTORCH_ENABLE_MPS_FALLBACK"] = "1"
        log.warning("MPS device: PYTORCH_ENABLE_MPS_FALLBACK=1, so ops MPS lacks (e.g. c10d::allgather_) "
                    "fall back to the CPU")
    if platform.startswith("linux"):
        return "127.0.0.1", env
    ipv6 = detect_active_ip_family() == "ipv6"
    env["GLOO_USE_IPV6"] = "1" if ipv6 else "0"
    if ipv6 and platform == "darwin":
        env["GLOO_SOCKET_IFNAME"] = "lo0"
    return ("::1" if ipv6 else "127.0.0.1"), env


def default_nproc(device: str) -> int:
    if str(device).startswith("cuda"):
        return max(1, torch.cuda.device_count())  # device_count() does not initialise HIP
    if device == "mps":
        return max(1, torch.mps.device_count()) if hasattr(torch, "mps") else 1
    return max(1, (os.cpu_count() or 2) // 2)


def _worker_entry(env: dict, worker_op: Callable, args: tuple):
    os.environ.update(env)
    try:
        worker_op(*args)
    except SystemExit:
        raise
    except BaseException:
        traceback.print_exc()
        os._exit(1)


def launch_single_node_ddp(run_id: str, device: str, worker_op: Callable[..., None], *args,
                           nproc: int | None = None, on_failure: Callable[[int, int], None] | None = None,
                           monitor_interval: float = 0.5, extra_env: dict | None = None) -> int:
    """Run ``worker_op(*args)`` in ``nproc`` ranks; return 0 or the first failing exit code."""
    nproc = nproc or default_nproc(device)
    addr, rdzv_env = rendezvous_env(str(device))
    port = free_port(addr)
    threads = max(1, (os.cpu_count() or 1) // nproc)
    log.info(f"Launching run {run_id}: {nproc} worker(s) on {device}, rendezvous [{addr}]:{port}")
    ctx = mp.get_context("spawn")
    procs = []
    for rank in range(nproc):
        env = {
            "RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(nproc),
            "LOCAL_WORLD_SIZE": str(nproc), "GROUP_RANK": "0",
            "MASTER_ADDR": addr, "MASTER_PORT": str(port),
            "PENROZ_RUN_ID": str(run_id), "HSA_ENABLE_IPC_MODE_LEGACY": "0",
            **rdzv_env,
        }
        if not str(device).startswith("cuda"):
            env["OMP_NUM_THREADS"] = str(threads)
        if extra_env:
            env.update(extra_env)
        p = ctx.Process(target=_worker_entry, args=(env, worker_op, args), name=f"{run_id}-rank{rank}")
        p.start()
        procs.append(p)

    failed_rank, failed_code = None, 0
    alive = {p.sentinel: (rank, p) for rank, p in enumerate(procs)}
    try:
        # wait on process sentinels: the first process to exit is seen first, so a rank that
        # dies of a peer's crash ("connection reset") is not blamed for it
        while alive and failed_rank is None:
            ready = mp_connection.wait(list(alive), timeout=monitor_interval)
            for s in sorted(ready, key=lambda x: alive[x][0]):
                rank, p = alive.pop(s)
                p.join()
                if p.exitcode != 0 and failed_rank is None:
                    failed_rank, failed_code = rank, p.exitcode
    finally:
        if failed_rank is not None:
            log.error(f"Run {run_id}: rank {failed_rank} exited with code {failed_code}; stopping the group")
            for p in procs:
                if p.exitcode is None:
                    p.terminate()
        for p in procs:
            p.join(timeout=30)
            if p.exitcode is None:
                p.kill()
                p.join()
    if failed_rank is not None and on_failure is not None:
        on_failure(failed_rank, failed_code)
    return failed_code if failed_rank is not None else 0


def maybe_inject_fault(step: int):
    """Test hook: exit this rank with ``FAULT_EXIT_CODE`` at ``PENROZ_FAULT_STEP``."""
    fr, fs = os.environ.get("PENROZ_FAULT_RANK"), os.environ.get("PENROZ_FAULT_STEP")
    if fr is None or fs is None:
        return
    if int(os.environ.get("RANK", 0)) == int(fr) and step == int(fs):
        log.error(f"Injected fault on rank {fr} at step {fs}")
        os._exit(FAULT_EXIT_CODE)
