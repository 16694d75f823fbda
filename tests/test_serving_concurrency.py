"""Concurrency of the serving path and the checkpoint flusher (CPU).

The reference rebuilt a private model per request (``main.py:401-434``); here a cached model is
one shared module tree, so every request holds that model's serving lock (``serve/app.py``)."""
import os
import threading
import time
from concurrent.futures import ThreadPoolExecutor

import pytest
import torch
from fastapi.testclient import TestClient

import bench
import main
from penroz.models.mapper import Mapper
from penroz.models.model import NeuralNetworkModel
from penroz.serve import app as A
from penroz.utils import checkpoint as ckpt


@pytest.fixture
def served_model(workdir, monkeypatch):
    monkeypatch.setenv("PENROZ_SERVE_DEVICE", "cpu")
    monkeypatch.setattr(A, "_model_cache", {})
    torch.manual_seed(3)
    m = NeuralNetworkModel("conc", Mapper(bench.gpt2_layers(V=64, C=32, L=2, H=2, P=32), {"sgd": {"lr": 0.1}}))
    m.serialize()
    ckpt.wait_flushes()
    return m


def test_concurrent_generate_and_output_match_serial(served_model):
    client = TestClient(main.app, raise_server_exceptions=True)
    ctxs = [[[1, 2, 3]], [[5, 9]], [[4, 4, 4, 4]]]

    def gen(i, stream=False):
        body = {"model_id": "conc", "input": ctxs[i % 3], "block_size": 16, "max_new_tokens": 24,
                "temperature": 0.0, "stream": stream}
        r = client.post("/generate/", json=body)
        assert r.status_code == 200
        return r.text if stream else r.json()["tokens"]

    def out(i):
        r = client.post("/output/", json={"model_id": "conc", "input": ctxs[i % 3]})
        assert r.status_code == 200
        return r.json()["output"]

    serial = {("g", i): gen(i) for i in range(3)}
    serial.update({("s", i): gen(i, True) for i in range(3)})
    serial.update({("o", i): out(i) for i in range(3)})
    assert len(A._model_cache) == 1  # every request above ran on ONE cached module tree

    jobs = [(kind, i) for _ in range(4) for kind in ("g", "s", "o") for i in range(3)]
    with ThreadPoolExecutor(max_workers=9) as pool:
        futs = {pool.submit(gen if k == "g" else (lambda j: gen(j, True)) if k == "s" else out, i): (k, i)
                for k, i in jobs}
        for f, key in futs.items():
            assert f.result(timeout=120) == serial[key], key


def test_serving_lock_is_per_model(served_model):
    m = A.load_for_serving("conc")
    assert A.serving_lock(m) is A.serving_lock(m)
    other = NeuralNetworkModel("x", Mapper([{"linear": {"in_features": 2, "out_features": 2}}], {"sgd": {}}))
    assert A.serving_lock(other) is not A.serving_lock(m)


def test_stream_releases_lock_when_client_stops_early(served_model):
    m = A.load_for_serving("conc")
    lk = A.serving_lock(m)
    client = TestClient(main.app)
    with client.stream("POST", "/generate/", json={"model_id": "conc", "input": [[1]], "block_size": 16,
                                                     "max_new_tokens": 50, "temperature": 0.0, "stream": True}) as r:
        first = next(r.iter_lines())
        assert first.strip().isdigit()
    for _ in range(100):  # the abandoned generator is closed when collected
        if not lk.locked():
            break
        import gc
        gc.collect()
        time.sleep(0.05)
    assert not lk.locked()


def test_flushes_to_one_destination_never_regress(tmp_path, monkeypatch):
    """An older flush that finishes last must not overwrite a newer snapshot."""
    src, dst = tmp_path / "shm.pth", tmp_path / "disk.pth"
    orig = ckpt.atomic_copy
    calls = []

    def slow_first(s, d):
        data = open(s, "rb").read()  # snapshot the source now, publish later
        calls.append(data)
        if len(calls) == 1:
            time.sleep(0.4)
        ckpt._atomic_write(d, lambda tmp: open(tmp, "wb").write(data))

    monkeypatch.setattr(ckpt, "atomic_copy", slow_first)
    src.write_bytes(b"v1")
    ckpt.flush_async(str(src), str(dst))
    time.sleep(0.05)  # v1's copy is in flight
    src.write_bytes(b"v2")
    ckpt.flush_async(str(src), str(dst))
    src.write_bytes(b"v3")
    ckpt.flush_async(str(src), str(dst))
    ckpt.wait_flushes()
    assert dst.read_bytes() == b"v3"
    assert b"v2" not in calls  # the superseded middle flush was skipped
    monkeypatch.setattr(ckpt, "atomic_copy", orig)


def test_flush_paths_are_absolute_at_queue_time(tmp_path, monkeypatch):
    a, b = tmp_path / "a", tmp_path / "b"
    a.mkdir(), b.mkdir()
    monkeypatch.chdir(a)
    (a / "src.bin").write_bytes(b"payload")
    gate = threading.Event()
    orig = ckpt._flush_one

    def gated(*args):
        gate.wait(5)
        orig(*args)

    monkeypatch.setattr(ckpt, "_flush_one", gated)
    ckpt.flush_async("src.bin", "dst.bin")
    os.chdir(b)  # a later chdir must not redirect the queued flush
    gate.set()
    ckpt.wait_flushes()
    assert (a / "dst.bin").read_bytes() == b"payload" and not (b / "dst.bin").exists()


def test_stats_served_from_sidecar(served_model, monkeypatch):
    served_model.stats = {"layers": [], "weights": []}
    served_model.serialize()
    ckpt.wait_flushes()
    monkeypatch.setattr(NeuralNetworkModel, "deserialize", classmethod(lambda cls, mid: (_ for _ in ()).throw(
        AssertionError("/stats must not load the checkpoint"))))
    client = TestClient(main.app, raise_server_exceptions=True)
    assert client.get("/stats/?model_id=conc").json() == {"layers": [], "weights": []}


def test_abandoned_stream_releases_the_model(served_model, monkeypatch):
    """A client that reads one chunk of a streaming /generate and goes away: the response's
    background task closes the token generator, which releases the serving lock at once (not at
    garbage collection), so the next request runs; a request that cannot get the lock within
    PENROZ_SERVE_LOCK_TIMEOUT gets 503 instead of queueing forever."""
    import asyncio
    from penroz.serve.app import GenerateRequest
    model = A.load_for_serving("conc")
    resp = A.model_generate(GenerateRequest(model_id="conc", input=[[1, 2, 3]], block_size=16, max_new_tokens=24,
                                            temperature=0.0, stream=True))
    lock = A.serving_lock(model)

    async def one_chunk_then_drop():
        it = resp.body_iterator.__aiter__()
        first = await it.__anext__()
        assert first.strip().isdigit()
        assert lock.locked()  # held while the stream is open
        await resp.background()  # what Starlette runs after a disconnect

    asyncio.run(one_chunk_then_drop())
    assert not lock.locked()
    client = TestClient(main.app, raise_server_exceptions=True)
    r = client.post("/generate/", json={"model_id": "conc", "input": [[1, 2, 3]], "block_size": 16,
                                        "max_new_tokens": 4, "temperature": 0.0})
    assert r.status_code == 200
    monkeypatch.setenv("PENROZ_SERVE_LOCK_TIMEOUT", "0.2")
    assert lock.acquire(timeout=1)
    try:
        r = client.post("/generate/", json={"model_id": "conc", "input": [[1, 2, 3]], "block_size": 16,
                                            "max_new_tokens": 4, "temperature": 0.0, "stream": True})
        assert r.status_code == 503
        r = client.post("/output/", json={"model_id": "conc", "input": [[1, 2, 3]]})
        assert r.status_code == 503
    finally:
        lock.release()
