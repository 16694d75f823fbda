"""Real multi-process data parallelism on CPU (gloo, world_size 2) — the reference only mocks this."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
from penroz.parallel import launcher
from penroz.parallel.reducer import GradReducer, HookedReducer, plan_buckets


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _reducer_worker(rank, world, port, out):
    _init(rank, world, port)
    g = torch.arange(10, dtype=torch.float32) * (rank + 1)
    red = GradReducer(g, plan_buckets([(0, 3), (3, 7), (7, 10)], 20))
    assert len(red.buckets) == 2
    red.bucket_ready(1)
    red.finish()
    torch.save(g, f"{out}/g{rank}.pt")
    dist.destroy_process_group()


def test_grad_reducer_averages(tmp_path):
    mp.spawn(_reducer_worker, args=(2, _port(), str(tmp_path)), nprocs=2)
    want = torch.arange(10, dtype=torch.float32) * 1.5
    for r in range(2):
        assert torch.allclose(torch.load(tmp_path / f"g{r}.pt"), want)


def _wire_worker(rank, world, port, out):
    _init(rank, world, port)
    torch.manual_seed(7)
    base = torch.randn(1000)
    g = base * (rank + 1)
    red = GradReducer(g, plan_buckets([(0, 400), (400, 1000)], 1000), wire="bf16")
    assert red._wire is not None and red._wire.dtype == torch.bfloat16
    red.bucket_ready(0)
    red.finish()  # launches bucket 1, waits, casts back to fp32
    assert g.dtype == torch.float32
    torch.save(g, f"{out}/w{rank}.pt")
    dist.destroy_process_group()


def test_grad_reducer_bf16_wire(tmp_path):
    mp.spawn(_wire_worker, args=(2, _port(), str(tmp_path)), nprocs=2)
    torch.manual_seed(7)
    want = torch.randn(1000) * 1.5
    for r in range(2):
        got = torch.load(tmp_path / f"w{r}.pt")
        assert torch.allclose(got, want, rtol=2e-2, atol=2e-2)
        assert not torch.equal(got, want)  # really went through bf16


def test_grad_reducer_rejects_unknown_wire():
    with pytest.raises(ValueError):
        GradReducer(torch.zeros(4), [(0, 4)], wire="fp8")


def _hooked_worker(rank, world, port, out, sparse=False):
    _init(rank, world, port)
    from penroz.models.mapper import Mapper
    from penroz.models.model import NeuralNetworkModel
    from penroz.parallel.reducer import row_sparse_tables
    torch.manual_seed(0)
    m = NeuralNetworkModel("h", Mapper(bench.gpt2_layers(V=32, C=16, L=1, H=2, P=16), {"sgd": {"lr": 0.1}}))
    tables = row_sparse_tables(m) if sparse else None
    if sparse:
        assert len(tables) == 2  # token + position tables (the lm_head is untied)
    red = HookedReducer(list(m.parameters()), bucket_mb=0.001, sparse_rows=tables)
    # ~1 KB buckets: parameters larger than a bucket are cut into several (their pieces reduce
    # as separate collectives once the parameter's gradient lands)
    assert any(len(bs) > 1 for bs in red._param_bucket.values())
    torch.manual_seed(100 + rank)
    for micro in range(2):  # grad accumulation: the row union covers both micro-steps
        red.sync = micro == 1
        x = torch.randint(0, 32, (2, 4 + 4 * micro))
        _, loss = m(x, torch.roll(x, -1, 1), skip_softmax=True)
        loss.backward()
    red.finish()
    torch.save({n: p.grad.clone() for n, p in m.named_parameters()}, f"{out}/grads{rank}.pt")
    dist.destroy_process_group()


@pytest.mark.parametrize("sparse", [False, True])
def test_hooked_reducer_matches_mean_of_local_grads(tmp_path, sparse):
    mp.spawn(_hooked_worker, args=(2, _port(), str(tmp_path), sparse), nprocs=2)
    from penroz.models.mapper import Mapper
    from penroz.models.model import NeuralNetworkModel
    local = []
    for rank in range(2):
        torch.manual_seed(0)
        m = NeuralNetworkModel("h", Mapper(bench.gpt2_layers(V=32, C=16, L=1, H=2, P=16), {"sgd": {"lr": 0.1}}))
        torch.manual_seed(100 + rank)
        for micro in range(2):
            x = torch.randint(0, 32, (2, 4 + 4 * micro))
            _, loss = m(x, torch.roll(x, -1, 1), skip_softmax=True)
            loss.backward()
        local.append({n: p.grad for n, p in m.named_parameters()})
    g0, g1 = torch.load(tmp_path / "grads0.pt"), torch.load(tmp_path / "grads1.pt")
    for n in g0:
        assert torch.allclose(g0[n], g1[n]), n
        assert torch.allclose(g0[n], (local[0][n] + local[1][n]) / 2, atol=1e-6), n


@pytest.fixture
def sandbox(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    (tmp_path / "data").mkdir()
    (tmp_path / "shm").mkdir()
    monkeypatch.setenv("PENROZ_DATA_FOLDER", str(tmp_path / "data"))
    monkeypatch.setenv("PENROZ_SHM_PATH", str(tmp_path / "shm"))
    import penroz.utils.loaders as loaders
    from penroz.models.model import NeuralNetworkModel
    monkeypatch.setattr(loaders, "DATA_FOLDER", str(tmp_path / "data"))
    monkeypatch.setattr(NeuralNetworkModel, "SHM_PATH", str(tmp_path / "shm"))
    return tmp_path


def _make_model(model_id):
    from penroz.models.mapper import Mapper
    from penroz.models.model import NeuralNetworkModel
    from penroz.utils import checkpoint as ckpt
    torch.manual_seed(0)
    m = NeuralNetworkModel(model_id, Mapper(bench.gpt2_layers(V=64, C=32, L=2, H=2, P=32),
                                            {"adamw": {"lr": 3e-3, "betas": [0.9, 0.95]}}))
    m.serialize()
    ckpt.wait_flushes()
    return m


@pytest.mark.slow
def test_launcher_two_rank_training(sandbox):
    from penroz.models.model import NeuralNetworkModel
    from penroz.utils import loaders
    loaders.synthetic_shards("ds", 2, 8192, 64)
    _make_model("dp2")
    code = launcher.launch_single_node_ddp("dp2", "cpu", NeuralNetworkModel.train_model_on_device, "dp2", "cpu", "ds",
                                           0, 4, 4, 16, 2, nproc=2)
    assert code == 0
    m = NeuralNetworkModel.deserialize("dp2")
    assert m.status["code"] == "Trained" and len(m.progress) == 4
    p = m.progress[-1]
    assert p["tokensPerSec"] == pytest.approx(2 * p["speedPerSec"], rel=1e-6)  # world * micro-steps(1) * B*T
    assert m.stats is not None


@pytest.mark.slow
def test_launcher_fault_marks_error(sandbox):
    from penroz.models.model import NeuralNetworkModel
    from penroz.serve import app as A
    from penroz.utils import loaders
    loaders.synthetic_shards("ds", 1, 4096, 64)
    _make_model("flt")
    failures = []
    code = launcher.launch_single_node_ddp(
        "flt", "cpu", NeuralNetworkModel.train_model_on_device, "flt", "cpu", "ds", 0, 5, 2, 16, 2, nproc=2,
        on_failure=lambda r, c: (failures.append((r, c)), A._mark_failed("flt", r, c)),
        extra_env={"PENROZ_FAULT_RANK": "1", "PENROZ_FAULT_STEP": "1"})
    assert code == launcher.FAULT_EXIT_CODE and failures == [(1, launcher.FAULT_EXIT_CODE)]
    st = NeuralNetworkModel.read_progress("flt")["status"]
    assert st["code"] == "Error" and "rank 1" in st["message"]


class _FakeNative:
    """Stands in for the native RCCL communicator in the probe: rank 1's enqueue fails."""

    def __init__(self, rank, log):
        self.rank, self.log = rank, log
        self.enqueued = False

    def all_reduce_avg_async(self, t):
        if self.rank == 1:
            raise RuntimeError("forced protocol refused at enqueue")
        self.enqueued = True
        return 0

    def wait_all(self):
        # the real communicator would hang here: rank 1 never enqueued its half
        raise AssertionError("waited on a collective a peer never enqueued")


def _probe_worker(rank, world, port, out):
    _init(rank, world, port)
    from penroz.parallel import commtune, rccl
    calls = []
    rccl.NativeComm.drop = classmethod(lambda cls, **kw: calls.append(kw))
    fake = _FakeNative(rank, calls)
    res = commtune._probe_native(torch.device("cpu"), fake, 0, "LL128", "")
    torch.save({"res": res is None, "calls": calls, "enq": fake.enqueued}, f"{out}/p{rank}.pt")
    dist.destroy_process_group()


def test_native_probe_agrees_on_enqueue_before_waiting(tmp_path):
    """when one rank's enqueue fails, no rank waits on the probe collective; every rank
    drops the arm, aborting (not destroying) the communicator."""
    mp.spawn(_probe_worker, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        d = torch.load(tmp_path / f"p{r}.pt")
        assert d["res"], "the arm must be dropped on every rank"
        assert d["calls"] == [{"channels": 0, "proto": "LL128", "algo": "", "abort": True}]
    assert torch.load(tmp_path / "p0.pt")["enq"] and not torch.load(tmp_path / "p1.pt")["enq"]
