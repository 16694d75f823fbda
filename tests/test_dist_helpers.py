"""Rank/env helpers, collectives and launcher plumbing (reference: test_ddp.py, 24 tests, all
mocked). Real multi-process behaviour is covered separately in test_distributed.py."""
import logging
import os
from unittest import mock

import pytest
import torch

from penroz.parallel import dist as D
from penroz.parallel import launcher as LA


@pytest.fixture
def clean_env(monkeypatch):
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "PENROZ_FAULT_RANK", "PENROZ_FAULT_STEP"):
        monkeypatch.delenv(k, raising=False)
    return monkeypatch


def test_is_ddp_false_without_rank(clean_env):
    assert not D.is_ddp()


def test_is_ddp_true_with_rank(clean_env):
    clean_env.setenv("RANK", "0")
    assert D.is_ddp()


@pytest.mark.parametrize("fn,var,default", [(D.ddp_rank, "RANK", 0), (D.ddp_local_rank, "LOCAL_RANK", 0),
                                            (D.ddp_world_size, "WORLD_SIZE", 1)])
def test_rank_helpers_default(clean_env, fn, var, default):
    assert fn() == default


@pytest.mark.parametrize("fn,var", [(D.ddp_rank, "RANK"), (D.ddp_local_rank, "LOCAL_RANK"),
                                    (D.ddp_world_size, "WORLD_SIZE")])
def test_rank_helpers_set(clean_env, fn, var):
    clean_env.setenv(var, "3")
    assert fn() == 3


@pytest.mark.parametrize("rank,expected", [(None, True), ("0", True), ("2", False)])
def test_master_proc(clean_env, rank, expected):
    if rank is not None:
        clean_env.setenv("RANK", rank)
    assert D.master_proc() is expected


@pytest.mark.parametrize("device,backend", [("cuda", "nccl"), ("cuda:3", "nccl"), ("cpu", "gloo"), ("mps", "gloo")])
def test_backend_for(device, backend):
    assert D.backend_for(device) == backend


@pytest.mark.parametrize("rank,world,device,expected", [
    (None, None, "cuda", False),   # not launched distributed
    ("0", "2", "cuda", True),
    ("0", "2", "cpu", True),
    ("0", "1", "mps", False),      # single-process MPS: no DDP (reference semantics)
    ("0", "2", "mps", True),
])
def test_use_ddp_matrix(clean_env, rank, world, device, expected):
    if rank is not None:
        clean_env.setenv("RANK", rank)
        clean_env.setenv("WORLD_SIZE", world)
    assert D.use_ddp(device) is expected


def test_ddp_all_reduce_nccl_uses_avg(clean_env):
    t = torch.ones(3)
    with mock.patch.object(D.dist, "get_backend", return_value="nccl"), \
            mock.patch.object(D.dist, "all_reduce") as ar:
        D.ddp_all_reduce(t)
    assert ar.call_args.kwargs["op"] == D.dist.ReduceOp.AVG
    assert torch.equal(t, torch.ones(3))


def test_ddp_all_reduce_gloo_sums_then_divides(clean_env):
    clean_env.setenv("WORLD_SIZE", "4")
    t = torch.full((2,), 8.0)
    with mock.patch.object(D.dist, "get_backend", return_value="gloo"), \
            mock.patch.object(D.dist, "all_reduce") as ar:
        D.ddp_all_reduce(t)
    assert ar.call_args.kwargs["op"] == D.dist.ReduceOp.SUM
    assert torch.equal(t, torch.full((2,), 2.0))


def test_max_over_ranks_without_group_is_identity():
    assert D.max_over_ranks(1.5, "cpu") == 1.5


def test_reconfig_logging_applies_dictconfig(clean_env):
    with mock.patch.object(D.logging.config, "dictConfig") as dc:
        D.reconfig_logging()
    cfg = dc.call_args.args[0]
    assert cfg["version"] == 1 and "ddp_file" not in cfg["handlers"]


def test_reconfig_logging_adds_rank_file_off_linux(clean_env, tmp_path):
    clean_env.setenv("RANK", "1")
    clean_env.chdir(tmp_path)
    with mock.patch.object(D, "running_on_linux", return_value=False), \
            mock.patch.object(D.logging.config, "dictConfig") as dc:
        D.reconfig_logging()
    cfg = dc.call_args.args[0]
    h = cfg["handlers"]["ddp_file"]
    assert h["filename"].endswith("ddp_rank01.log") and h["maxBytes"] == 10 * 1024 * 1024
    assert "ddp_file" in cfg["root"]["handlers"]
    assert (tmp_path / "logs").is_dir()


def test_free_port_is_bindable():
    import socket
    p = LA.free_port()
    s = socket.socket()
    s.bind(("127.0.0.1", p))
    s.close()


def test_default_nproc_cpu_splits_cores():
    with mock.patch.object(LA.os, "cpu_count", return_value=16):
        assert LA.default_nproc("cpu") == 8


def test_default_nproc_cuda_counts_devices():
    with mock.patch.object(LA.torch.cuda, "device_count", return_value=8):
        assert LA.default_nproc("cuda") == 8


class _FakeProc:
    instances = []

    def __init__(self, target, args, name):
        self.target, self.args, self.name = target, args, name
        self.exitcode = 0
        r, w = os.pipe()
        os.close(w)  # the read end is immediately "ready" (EOF), like an exited process sentinel
        self.sentinel = r
        _FakeProc.instances.append(self)

    def start(self):
        pass

    def join(self, timeout=None):
        pass

    def terminate(self):
        pass

    def kill(self):
        pass


def test_launcher_env_per_rank_and_omp_split():
    _FakeProc.instances = []
    ctx = mock.Mock()
    ctx.Process.side_effect = lambda target, args, name: _FakeProc(target, args, name)
    with mock.patch.object(LA.mp, "get_context", return_value=ctx), \
            mock.patch.object(LA.os, "cpu_count", return_value=8):
        code = LA.launch_single_node_ddp("run42", "cpu", print, nproc=2)
    assert code == 0
    envs = [p.args[0] for p in _FakeProc.instances]
    assert [e["RANK"] for e in envs] == ["0", "1"]
    assert all(e["WORLD_SIZE"] == "2" and e["MASTER_ADDR"] == "127.0.0.1" for e in envs)
    assert all(e["OMP_NUM_THREADS"] == "4" and e["PENROZ_RUN_ID"] == "run42" for e in envs)
    assert envs[0]["MASTER_PORT"] == envs[1]["MASTER_PORT"]
    for p in _FakeProc.instances:
        os.close(p.sentinel)


def test_launcher_gpu_env_keeps_omp_and_ipc_mode():
    _FakeProc.instances = []
    ctx = mock.Mock()
    ctx.Process.side_effect = lambda target, args, name: _FakeProc(target, args, name)
    with mock.patch.object(LA.mp, "get_context", return_value=ctx):
        LA.launch_single_node_ddp("r", "cuda", print, nproc=2)
    envs = [p.args[0] for p in _FakeProc.instances]
    assert all("OMP_NUM_THREADS" not in e and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" for e in envs)
    for p in _FakeProc.instances:
        os.close(p.sentinel)


def test_launcher_reports_first_failure():
    _FakeProc.instances = []
    ctx = mock.Mock()

    def make(target, args, name):
        p = _FakeProc(target, args, name)
        p.exitcode = 13 if name.endswith("rank1") else 0
        return p
    ctx.Process.side_effect = make
    seen = []
    with mock.patch.object(LA.mp, "get_context", return_value=ctx):
        code = LA.launch_single_node_ddp("r", "cpu", print, nproc=2, on_failure=lambda r, c: seen.append((r, c)))
    assert code == 13 and seen == [(1, 13)]
    for p in _FakeProc.instances:
        os.close(p.sentinel)


def test_fault_injection_only_on_matching_rank_and_step(clean_env):
    clean_env.setenv("PENROZ_FAULT_RANK", "1")
    clean_env.setenv("PENROZ_FAULT_STEP", "3")
    clean_env.setenv("RANK", "1")
    with mock.patch.object(LA.os, "_exit") as ex:
        LA.maybe_inject_fault(2)
        ex.assert_not_called()
        LA.maybe_inject_fault(3)
        ex.assert_called_once_with(LA.FAULT_EXIT_CODE)
    clean_env.setenv("RANK", "0")
    with mock.patch.object(LA.os, "_exit") as ex:
        LA.maybe_inject_fault(3)
        ex.assert_not_called()


def test_fault_injection_disabled_by_default(clean_env):
    with mock.patch.object(LA.os, "_exit") as ex:
        LA.maybe_inject_fault(0)
        ex.assert_not_called()


def test_bucket_plan_gpt2_xl_gradients():
    """6.55 GB of XL fp32 gradients: contiguous buckets covering every element once, each at
    least the target (except the tail) and never splitting a layer."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench"))
    import allreduce_bench as ab
    from penroz.parallel.reducer import plan_buckets
    segs = ab.gpt2_segments(1600, 48)
    total = segs[-1][1]
    assert abs(total * 4 / 1e9 - 6.55) < 0.05
    for mb in (25, 64, 128, 256):
        b = plan_buckets(segs, mb * 2**20)
        assert b[0][0] == 0 and b[-1][1] == total
        assert all(b[i][1] == b[i + 1][0] for i in range(len(b) - 1))
        bounds = {s for s, _ in segs} | {total}
        assert all(s in bounds and e in bounds for s, e in b)  # layer boundaries only
        assert all((e - s) * 4 >= mb * 2**20 for s, e in b[:-1])
    plan = ab.plan_summary(64)
    assert plan["gpt2-xl"]["buckets"] < plan["gpt2-xl"]["grad_mb"] / 64 + 2


@pytest.mark.slow
def test_allreduce_bench_cpu_rehearsal():
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench", "allreduce_bench.py"), "--gpus", "2", "--device", "cpu",
                        "--sizes-mb", "1", "--wires", "fp32,bf16", "--iters", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 3 and lines[-1]["summary"] and lines[-1]["n_ranks"] == 2
    assert {l["wire"] for l in lines[:2]} == {"fp32", "bf16"} and lines[1]["wire_mb"] == 0.5


# ---- loopback rendezvous per platform / address family (reference ddp.py:22-36, 39-42, 59-68)

def test_rendezvous_linux_is_ipv4_loopback_without_gloo_overrides():
    addr, env = LA.rendezvous_env("cpu", platform="linux")
    assert addr == "127.0.0.1" and env == {}


@pytest.mark.parametrize("platform,family,addr,ifname", [
    ("darwin", "ipv6", "::1", "lo0"), ("darwin", "ipv4", "127.0.0.1", None),
    ("win32", "ipv6", "::1", None), ("win32", "ipv4", "127.0.0.1", None)])
def test_rendezvous_off_linux_follows_the_active_family(platform, family, addr, ifname):
    with mock.patch.object(LA, "detect_active_ip_family", return_value=family):
        got, env = LA.rendezvous_env("cpu", platform=platform)
    assert got == addr
    assert env["GLOO_USE_IPV6"] == ("1" if family == "ipv6" else "0")
    assert env.get("GLOO_SOCKET_IFNAME") == ifname


def test_rendezvous_mps_enables_cpu_fallback(caplog):
    with caplog.at_level(logging.WARNING):
        _, env = LA.rendezvous_env("mps", platform="linux")
    assert env["PYTORCH_ENABLE_MPS_FALLBACK"] == "1"
    assert "PYTORCH_ENABLE_MPS_FALLBACK" in caplog.text


def test_detect_active_ip_family_falls_back_to_ipv4_when_ipv6_connect_fails():
    class Refusing:
        def __init__(self, *a, **k):
            pass

        def __enter__(self):
            return self

        def __exit__(self, *exc):
            return False

        def settimeout(self, t):
            pass

        def connect(self, addr):
            raise OSError("no ipv6")

    with mock.patch.object(LA.socket, "socket", Refusing), mock.patch.object(LA.socket, "has_ipv6", True):
        assert LA.detect_active_ip_family() == "ipv4"
    with mock.patch.object(LA.socket, "has_ipv6", False):
        assert LA.detect_active_ip_family() == "ipv4"


def test_launch_passes_the_rendezvous_env_to_every_rank():
    seen = []

    class FakeProc:
        exitcode = 0
        sentinel = None

        def __init__(self, target, args, name):
            seen.append(args[0])
            self.sentinel = object()

        def start(self):
            pass

        def join(self, timeout=None):
            pass

    class Ctx:
        Process = FakeProc

    with mock.patch.object(LA, "rendezvous_env", return_value=("127.0.0.1", {"GLOO_USE_IPV6": "0"})), \
            mock.patch.object(LA.mp, "get_context", return_value=Ctx()), \
            mock.patch.object(LA.mp_connection, "wait", side_effect=lambda objs, timeout: objs):
        assert LA.launch_single_node_ddp("r", "cpu", print, nproc=2) == 0
    assert len(seen) == 2
    assert all(e["GLOO_USE_IPV6"] == "0" and e["MASTER_ADDR"] == "127.0.0.1" for e in seen)
