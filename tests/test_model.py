"""Model runtime on CPU: persistence, output, evaluation, generation, training, diagnostics."""
import json
import os
from unittest.mock import patch

import numpy as np
import pytest
import torch

import bench
from penroz.models.mapper import Mapper
from penroz.models.model import NeuralNetworkModel
from penroz.utils import checkpoint as ckpt
from penroz.utils import loaders

MLP = [{"linear": {"in_features": 9, "out_features": 9}, "xavier_uniform": {}, "confidence": 0.9},
       {"sigmoid": {}},
       {"linear": {"in_features": 9, "out_features": 3}},
       {"softmax": {"dim": -1}}]


def gpt(V=64, C=32, L=2, H=2, P=32, opt=None):
    torch.manual_seed(0)
    return NeuralNetworkModel("gpt", Mapper(bench.gpt2_layers(V=V, C=C, L=L, H=H, P=P),
                                            opt or {"adamw": {"lr": 3e-3, "betas": [0.9, 0.95]}}))


def test_construction_and_weights():
    m = NeuralNetworkModel("m", Mapper(MLP, {"sgd": {"lr": 0.1}}))
    assert m.status["code"] == "Created" and m.progress == [] and m.avg_cost is None
    assert m.num_params == 9 * 9 + 9 + 9 * 3 + 3
    assert [w is not None for w in m._weights] == [True, False, True, False]
    g = gpt()
    assert g.num_params == sum(p.numel() for p in g.parameters())


def test_serialize_roundtrip_and_sidecar(workdir):
    m = gpt()
    m.progress = [{"epoch": 1, "cost": 1.0}]
    m.serialize()
    ckpt.wait_flushes()
    assert os.path.exists("models/model_gpt.pth")
    assert os.path.exists(os.path.join(NeuralNetworkModel.SHM_PATH, "models/model_gpt.pth"))
    m2 = NeuralNetworkModel.deserialize("gpt")
    for (k, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), k
    assert m2.progress == m.progress and m2.status == m.status
    assert NeuralNetworkModel.read_progress("gpt")["progress"] == m.progress
    # cache miss: SHM copy removed -> restored from disk
    os.remove(os.path.join(NeuralNetworkModel.SHM_PATH, "models/model_gpt.pth"))
    NeuralNetworkModel.deserialize("gpt")
    # torch can read the checkpoint with the safe loader
    data = torch.load("models/model_gpt.pth", weights_only=True)
    assert set(data) == {"layers", "state", "optim", "optim_state", "progress", "average_cost",
                         "average_cost_history", "stats", "status"}


def test_deserialize_missing_and_delete(workdir):
    with pytest.raises(KeyError):
        NeuralNetworkModel.deserialize("nope")
    m = gpt()
    m.serialize()
    ckpt.wait_flushes()
    NeuralNetworkModel.delete("gpt")
    assert not os.path.exists("models/model_gpt.pth")
    NeuralNetworkModel.delete("gpt")  # missing files only logged


def test_bf16_dtype_restored(workdir):
    m = gpt().to(dtype=torch.bfloat16)
    m.serialize()
    ckpt.wait_flushes()
    m2 = NeuralNetworkModel.deserialize("gpt")
    assert next(m2.parameters()).dtype == torch.bfloat16


@pytest.mark.parametrize("inp,target,has_cost", [([0.0] * 9, None, False), ([0.0] * 9, [0.0, 0.0, 1.0], True),
                                                 ([[0.0] * 9] * 2, [1, 2], True)])
def test_compute_output(inp, target, has_cost):
    m = NeuralNetworkModel("m", Mapper(MLP, {"sgd": {"lr": 0.1}}))
    out, cost = m.compute_output(inp, target)
    assert np.asarray(out).shape[-1] == 3
    assert (cost is not None) == has_cost


def test_compute_output_bf16_converts_float_input():
    m = NeuralNetworkModel("m", Mapper(MLP, {"sgd": {"lr": 0.1}})).to(dtype=torch.bfloat16)
    out, _ = m.compute_output([0.5] * 9)
    assert len(out) == 3


def _shards(dataset, n=2, size=4000, vocab=64, seed=0):
    return loaders.synthetic_shards(dataset, n, size, vocab, seed)


def test_evaluate_with_and_without_target_dataset(workdir):
    _shards("ds")
    _shards("tgt", seed=1)
    m = gpt()
    c1 = m.evaluate_model("ds", None, 0, 2, 2, 16, 1)
    c2 = m.evaluate_model("ds", "tgt", 0, 2, 2, 16, 1)  # reference crashed here (bug 1)
    assert 2.0 < c1 < 6.0 and 2.0 < c2 < 6.0


def test_generate_greedy_stream_and_stop():
    m = gpt()
    toks = m.generate_tokens([[1, 2, 3]], 8, 10, temperature=0.0)
    assert len(toks) == 13 and toks[:3] == [1, 2, 3]
    streamed = list(m.generate_tokens_stream([[1, 2, 3]], 8, 10, temperature=0.0))
    assert streamed == toks[3:]
    torch.manual_seed(5)
    a = m.generate_tokens([[1, 2]], 8, 6, temperature=1.0, top_k=5)
    torch.manual_seed(5)
    b = [1, 2] + list(m.generate_tokens_stream([[1, 2]], 8, 6, temperature=1.0, top_k=5))
    assert a == b
    stop = toks[4]
    short = m.generate_tokens([[1, 2, 3]], 8, 10, temperature=0.0, stop_token=stop)
    assert short[-1] == stop and len(short) < 13
    assert len(m.generate_batch([[1, 2], [3, 4]], 8, 3, temperature=0.0)) == 2


def test_generation_without_softmax_layer_and_bf16():
    m = NeuralNetworkModel("m", Mapper(bench.gpt2_layers(V=64, C=32, L=1, H=2, P=32)[:-1], {"sgd": {"lr": 0.1}}))
    assert len(m.generate_tokens([[1]], 8, 3, temperature=0.8)) == 4  # reference crashed (bug 2)
    mb = gpt().to(dtype=torch.bfloat16)
    assert len(mb.generate_tokens([[1]], 8, 3, temperature=1.0, top_k=4)) == 4


def test_train_cpu_generic(workdir):
    _shards("ds", n=2, size=8192)
    m = gpt()
    m.serialize()
    m.train_model("ds", 0, 12, 4, 16, 2)
    ckpt.wait_flushes()
    assert m.status["code"] == "Trained"
    costs = [p["cost"] for p in m.progress]
    assert len(costs) == 12 and costs[-1] < costs[0]
    p0 = m.progress[0]
    assert {"dt", "epoch", "durationInSecs", "speedPerSec", "tokensPerSec", "cost", "weight_upd_ratio"} <= set(p0)
    assert len(p0["weight_upd_ratio"]) == len(list(m.parameters()))
    st = m.stats
    assert len(st["layers"]) == len(m.layers) - 1 and st["layers"][0]["algo"] == "summation"
    hist = st["layers"][2]["activation"]["histogram"]
    assert len(hist["x"]) == 100 and st["layers"][2]["gradient"] is not None
    assert st["weights"][0]["shape"] == "(64, 32)"
    m2 = NeuralNetworkModel.deserialize("gpt")
    assert m2.status["code"] == "Trained" and m2.avg_cost is not None
    json.dumps(m2.stats)


def test_train_error_marks_status(workdir):
    _shards("ds")
    m = gpt()
    with patch.object(NeuralNetworkModel, "forward", side_effect=RuntimeError("boom")):
        with pytest.raises(RuntimeError):
            m.train_model("ds", 0, 2, 2, 16, 1)
    ckpt.wait_flushes()
    assert NeuralNetworkModel.deserialize("gpt").status["code"] == "Error"
    NeuralNetworkModel.mark_status("gpt", "Error", "worker died")
    assert "worker died" in NeuralNetworkModel.read_progress("gpt")["status"]["message"]


def test_micro_steps_match_single_step(workdir):
    """num_steps micro-steps with loss/num_steps == one step on the same tokens (grad accumulation)."""
    _shards("ds", n=1, size=8192)
    a, b = gpt(opt={"sgd": {"lr": 0.1}}), gpt(opt={"sgd": {"lr": 0.1}})
    a.train_model("ds", 0, 1, 4, 16, 4)   # 1 micro-step of B=4
    b.train_model("ds", 0, 1, 4, 16, 1)   # 4 micro-steps (each its own B=4 window)
    assert a.progress[0]["cost"] > 0 and b.progress[0]["cost"] > 0


def test_shm_detection(monkeypatch):
    import platform
    monkeypatch.setattr(platform, "system", lambda: "Plan9")
    assert ckpt.detect_shm_path() == __import__("tempfile").gettempdir()


def test_amp_dtype_selection(monkeypatch):
    """bf16 where supported, fp16 (+ GradScaler in the generic runner) otherwise, as the reference
    (neural_net_model.py:570-575); PENROZ_AMP_DTYPE overrides; CPU has no autocast."""
    import torch
    from penroz.models.model import NeuralNetworkModel as M
    cuda = torch.device("cuda")
    assert M.amp_dtype(torch.device("cpu")) is None
    monkeypatch.setattr(torch.cuda, "is_bf16_supported", lambda *a, **k: True)
    assert M.amp_dtype(cuda) == torch.bfloat16
    monkeypatch.setattr(torch.cuda, "is_bf16_supported", lambda *a, **k: False)
    assert M.amp_dtype(cuda) == torch.float16
    monkeypatch.setenv("PENROZ_AMP_DTYPE", "bf16")
    assert M.amp_dtype(cuda) == torch.bfloat16
    monkeypatch.setenv("PENROZ_AMP_DTYPE", "fp16")
    monkeypatch.setattr(torch.cuda, "is_bf16_supported", lambda *a, **k: True)
    assert M.amp_dtype(cuda) == torch.float16
