"""HTTP API: routes, schemas, error mapping, locks, gzip, streaming (CPU, mocked heavy work)."""
import asyncio
import gzip
import json
from unittest.mock import MagicMock, patch

import pytest
from fastapi.testclient import TestClient

import main
from penroz.serve import app as A

client = TestClient(main.app, raise_server_exceptions=False)


@pytest.fixture
def served():
    m = MagicMock()
    with patch.object(A, "load_for_serving", return_value=m):
        yield m


@pytest.fixture
def no_tasks():
    def consume(coro):
        coro.close()
    with patch.object(A, "create_task", side_effect=consume) as ct:
        yield ct


def test_root_redirects_and_dashboard():
    r = client.get("/")
    assert r.status_code == 200 and r.url.path == "/dashboard"
    assert "penroz" in r.text
    assert client.get("/static/dashboard.js").status_code == 200


def test_create_model():
    with patch.object(A, "NeuralNetworkModel") as M:
        r = client.post("/model/", json={"model_id": "t", "layers": [{"linear": {"in_features": 2, "out_features": 2}}],
                                         "optimizer": {"sgd": {"lr": 0.1}}})
    assert r.status_code == 200 and r.json() == {"message": "Model t created and saved successfully"}
    M.return_value.serialize.assert_called_once()


def test_create_model_unsupported_layer_is_400(workdir):
    r = client.post("/model/", json={"model_id": "t", "layers": [{"bogus": {}}], "optimizer": {"sgd": {"lr": 0.1}}})
    assert r.status_code == 400


def test_schema_errors_are_422():
    assert client.post("/model/", json={"model_id": "t"}).status_code == 422
    assert client.post("/generate/", json={"model_id": "t", "input": [[0]]}).status_code == 422


@pytest.mark.parametrize("target,cost", [(None, None), ([0.0, 1.0], 1.5), (1, 0.5)])
def test_output(served, target, cost):
    served.compute_output.return_value = ([0.1, 0.9], cost)
    r = client.post("/output/", json={"model_id": "t", "input": [0.0, 0.0], "target": target})
    assert r.status_code == 200 and r.json() == {"output": [0.1, 0.9], "cost": cost}


def test_output_gzip(served):
    served.compute_output.return_value = ([1.0], None)
    body = gzip.compress(json.dumps({"model_id": "t", "input": [0.0]}).encode())
    r = client.post("/output/", content=body, headers={"Content-Encoding": "gzip", "Content-Type": "application/json"})
    assert r.status_code == 200 and r.json()["output"] == [1.0]


def test_evaluate(served):
    served.evaluate_model.return_value = 1.25
    r = client.post("/evaluate/", json={"model_id": "t", "dataset_id": "d", "shard": 0, "epochs": 2,
                                        "batch_size": 2, "block_size": 16, "step_size": 1, "target_dataset_id": "x"})
    assert r.json() == {"cost": 1.25}
    served.evaluate_model.assert_called_once_with("d", "x", 0, 2, 2, 16, 1)


def test_generate_json_and_stream(served):
    served.generate_tokens.return_value = [1, 2, 3]
    r = client.post("/generate/", json={"model_id": "t", "input": [[1]], "block_size": 8, "max_new_tokens": 2})
    assert r.json() == {"tokens": [1, 2, 3]}
    served.generate_tokens_stream.return_value = iter([4, 5])
    r = client.post("/generate/", json={"model_id": "t", "input": [[1]], "block_size": 8, "max_new_tokens": 2,
                                        "stream": True})
    assert r.headers["content-type"].startswith("text/plain") and r.text == "4\n5\n"


def test_error_mapping(served):
    served.compute_output.side_effect = KeyError("missing")
    assert client.post("/output/", json={"model_id": "t", "input": [0]}).status_code == 404
    served.compute_output.side_effect = ValueError("bad")
    assert client.post("/output/", json={"model_id": "t", "input": [0]}).status_code == 400
    served.compute_output.side_effect = RuntimeError("boom")
    r = client.post("/output/", json={"model_id": "t", "input": [0]})
    assert r.status_code == 500 and r.json() == {"detail": "Please refer to server logs"}


def test_unknown_model_is_404(workdir):
    A._model_cache.clear()
    assert client.post("/output/", json={"model_id": "nope", "input": [0]}).status_code == 404
    assert client.get("/progress/?model_id=nope").status_code == 404


def test_train_accepted_and_conflict(no_tasks):
    body = {"model_id": "tr", "device": "cpu", "dataset_id": "d", "shard": 0, "epochs": 1, "batch_size": 2,
            "block_size": 8, "step_size": 1}
    r = client.put("/train/", json=body)
    assert r.status_code == 202 and r.json() == {"message": "Training for model tr started asynchronously."}
    lock = A.model_locks["tr"]

    async def hold():
        await lock.acquire()
    asyncio.run(hold())
    try:
        r = client.put("/train/", json=body)
        assert r.status_code == 409
    finally:
        lock.release()


def test_train_job_failure_marks_error():
    with patch.object(A.launcher, "launch_single_node_ddp") as launch, \
            patch.object(A.NeuralNetworkModel, "mark_status") as mark:
        def fake(run_id, device, op, *args, on_failure=None, **kw):
            on_failure(1, 13)
            return 13
        launch.side_effect = fake
        assert A.run_training_job("m", "cpu", "d", 0, 1, 2, 8, 1) == 13
        mark.assert_called_once()
        assert mark.call_args[0][1] == "Error"


def test_dataset_routes(no_tasks, workdir):
    from penroz.utils import loaders
    loaders.synthetic_shards("ds", 2, 10, 50)
    assert client.get("/dataset/?dataset_id=ds").json() == {"files": ["ds_000000.npy", "ds_000001.npy"]}
    with patch.object(A, "Downloader"):
        r = client.post("/dataset/", json={"dataset_id": "ds", "encoding": "x", "path": "p", "name": "n",
                                           "split": "train", "shard_size": 100})
    assert r.status_code == 202
    assert client.delete("/dataset/?dataset_id=ds").status_code == 204
    assert client.get("/dataset/?dataset_id=ds").json() == {"files": []}


def test_tokenize_decode():
    tok = MagicMock()
    tok.tokenize.return_value = [1, 2]
    tok.decode.return_value = "hi"
    with patch.object(A, "Tokenizer", return_value=tok):
        assert client.post("/tokenize/", json={"encoding": "e", "text": "hi"}).json() == {"encoding": "e", "tokens": [1, 2]}
        assert client.post("/decode/", json={"encoding": "e", "tokens": [1]}).json() == {"encoding": "e", "text": "hi"}


def test_import_and_conflict():
    with patch.object(A.NeuralNetworkModel, "from_huggingface") as fh:
        r = client.post("/import/", json={"hf_repo_id": "openai-community/gpt2", "model_id": "g"})
    assert r.status_code == 200 and r.json()["status"] == "imported"
    fh.assert_called_once_with("g", "openai-community/gpt2", None, "cpu")


def test_progress_stats_delete_roundtrip(workdir):
    import bench
    from penroz.models.mapper import Mapper
    from penroz.models.model import NeuralNetworkModel
    m = NeuralNetworkModel("p", Mapper(bench.gpt2_layers(V=32, C=16, L=1, H=2, P=16), {"sgd": {"lr": 0.1}}))
    m.serialize()
    r = client.get("/progress/?model_id=p").json()
    assert r["status"]["code"] == "Created" and r["progress"] == [] and r["average_cost"] is None
    assert client.get("/stats/?model_id=p").json() is None
    A._model_cache.clear()
    with patch.dict("os.environ", {"PENROZ_SERVE_DEVICE": "cpu"}):
        out = client.post("/generate/", json={"model_id": "p", "input": [[1, 2]], "block_size": 8,
                                              "max_new_tokens": 3, "temperature": 0.0}).json()
    assert len(out["tokens"]) == 5
    assert client.delete("/model/?model_id=p").status_code == 204
    assert client.get("/progress/?model_id=p").status_code == 404
