"""Rank/env helpers and small collectives (parity with the reference's ``ddp.py:13-17, 75-85``).

Processes are launched one per GPU by :mod:`penroz.parallel.launcher` (or ``torchrun``) with
``RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT`` in the environment.  The
process group backend is ``nccl`` (= RCCL on ROCm) for GPU work and ``gloo`` for CPU.
"""
from __future__ import annotations

import json
import logging
import logging.config
import os
import sys
from pathlib import Path

import torch
import torch.distributed as dist

log = logging.getLogger(__name__)

is_ddp = lambda: int(os.environ.get("RANK", -1)) != -1  # noqa: E731
ddp_rank = lambda: int(os.environ.get("RANK", 0))  # noqa: E731
ddp_local_rank = lambda: int(os.environ.get("LOCAL_RANK", 0))  # noqa: E731
ddp_world_size = lambda: int(os.environ.get("WORLD_SIZE", 1))  # noqa: E731
master_proc = lambda: ddp_rank() == 0  # noqa: E731


def running_on_linux() -> bool:
    return sys.platform.startswith("linux")


def backend_for(device: str) -> str:
    return "nccl" if str(device).startswith("cuda") else "gloo"


def use_ddp(device: str) -> bool:
    """DDP is on whenever launched distributed (single-process MPS excluded, as the reference)."""
    if is_ddp() and ddp_world_size() == 1 and device == "mps":
        return False
    return is_ddp()


def dist_timeout_s() -> float:
    """Collective / rendezvous timeout (``PENROZ_DIST_TIMEOUT`` seconds, default 300).

    torch's default is 10 min for NCCL (30 for gloo); a dead or stuck rank should instead fail
    the job with a non-zero exit well inside a benchmark driver's budget. On the nccl (RCCL)
    backend the ProcessGroupNCCL watchdog aborts the communicator and tears the process down
    when a collective exceeds it (``TORCH_NCCL_ASYNC_ERROR_HANDLING=1``, set here unless the
    caller chose otherwise); on gloo the blocked collective raises."""
    return float(os.environ.get("PENROZ_DIST_TIMEOUT", "300"))


def init_group(backend: str, device: torch.device | None = None, timeout_s: float | None = None):
    """``dist.init_process_group`` with an explicit timeout (and ``device_id`` binding on nccl)."""
    import datetime
    if not (dist.is_available() and not dist.is_initialized()):
        return dist.group.WORLD
    timeout = datetime.timedelta(seconds=timeout_s if timeout_s is not None else dist_timeout_s())
    kwargs = {"timeout": timeout}
    if backend == "nccl":
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        if device is not None:
            kwargs["device_id"] = device
    dist.init_process_group(backend=backend, **kwargs)
    return dist.group.WORLD


def init_process_group(device: str):
    """Initialise the default group once (env:// rendezvous on MASTER_ADDR/PORT)."""
    backend = backend_for(device)
    return init_group(backend, torch.device(f"cuda:{ddp_local_rank()}") if backend == "nccl" else None)


def device_identity(device: torch.device) -> dict:
    """What identifies this rank's device: PCI domain:bus:device and UUID (GPU), or the host."""
    if device.type != "cuda":
        import socket
        return {"device": "cpu", "host": socket.gethostname(), "pid": os.getpid()}
    p = torch.cuda.get_device_properties(device)
    pci = f"{getattr(p, 'pci_domain_id', 0):04x}:{getattr(p, 'pci_bus_id', 0):02x}:{getattr(p, 'pci_device_id', 0):02x}"
    return {"device": str(device), "pci": pci, "uuid": str(getattr(p, "uuid", "")), "name": p.name}


def ddp_all_reduce(tensor: torch.Tensor):
    """In-place mean over ranks (AVG on nccl/RCCL, SUM + divide on gloo)."""
    if dist.get_backend() == "nccl":
        dist.all_reduce(tensor, op=dist.ReduceOp.AVG)
    else:
        dist.all_reduce(tensor, op=dist.ReduceOp.SUM)
        tensor.div_(ddp_world_size())


def max_over_ranks(value: float, device) -> float:
    if not (dist.is_available() and dist.is_initialized()):
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


LOG_CONFIG_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                               "log_config.json")


def load_log_config() -> dict:
    with open(LOG_CONFIG_PATH) as f:
        return json.load(f)


def reconfig_logging():
    """Apply ``log_config.json`` in a worker; add a per-rank rotating file off Linux."""
    cfg = load_log_config()
    if is_ddp() and not running_on_linux():
        log_dir = Path("logs")
        log_dir.mkdir(parents=True, exist_ok=True)
        cfg["handlers"]["ddp_file"] = {
            "level": "INFO", "class": "logging.handlers.RotatingFileHandler", "formatter": "default",
            "filename": str(log_dir / f"ddp_rank{ddp_rank():02d}.log"), "maxBytes": 10_485_760, "backupCount": 3,
        }
        if "ddp_file" not in cfg["root"]["handlers"]:
            cfg["root"]["handlers"].append("ddp_file")
    logging.config.dictConfig(cfg)
