"""FastAPI service: create / import / train / evaluate / generate / diagnose models.

Route and schema parity with the reference service (``main.py:21-506``): ``/``, ``/dashboard``,
``/static``, ``POST /model/``, ``POST /import/``, ``GET|POST|DELETE /dataset/``,
``POST /tokenize/``, ``POST /output/``, ``POST /evaluate/``, ``POST /generate/`` (JSON or
``text/plain`` token stream), ``POST /decode/``, ``PUT /train/``, ``GET /progress/``,
``GET /stats/``, ``DELETE /model/``; gzip request bodies; ``KeyError``→404, ``ValueError``→400,
other exceptions→500; per-id locks (409 while a job holds them).

MI355X-first differences:
  * serving runs on the GPU (``PENROZ_SERVE_DEVICE``, default ``cuda`` when present) with a small
    model cache keyed on the checkpoint's mtime, instead of rebuilding the model on the CPU for
    every request (``/generate`` uses the preallocated KV cache + decode-attention kernel);
  * ``/train/`` runs the launcher (one worker per GPU, RCCL) and checks its exit code: a failed
    run marks the model ``Error`` instead of leaving it ``Training`` (reference bug 9);
  * ``/progress/`` reads a small sidecar JSON instead of ``torch.load``-ing the checkpoint.
"""
from __future__ import annotations

import asyncio
import gzip
import logging
import math
import os
import threading
from asyncio import Lock, create_task
from typing import Dict

from fastapi import Body, FastAPI, HTTPException, Request
from fastapi.concurrency import run_in_threadpool
from fastapi.params import Query
from fastapi.responses import HTMLResponse, JSONResponse, RedirectResponse, Response, StreamingResponse
from fastapi.staticfiles import StaticFiles
from pydantic import BaseModel, Field

from penroz.models.mapper import Mapper
from penroz.models.model import NeuralNetworkModel
from penroz.parallel import launcher
from penroz.utils.loaders import Downloader, Loader
from penroz.utils.tokenizers import Tokenizer

log = logging.getLogger(__name__)

HERE = os.path.dirname(os.path.abspath(__file__))

app = FastAPI(title="penroz — MI355X neural network model API",
              description="Create, import, train, evaluate, generate with and diagnose neural network models "
                          "on AMD Instinct MI355X.",
              version="0.1.0")
app.mount("/static", StaticFiles(directory=os.path.join(HERE, "static")), name="static")

dataset_locks: Dict[str, Lock] = {}
model_locks: Dict[str, Lock] = {}


def _gpt2_example_layers(V=50304, C=768, L=12, H=12, P=1024) -> list[dict]:
    std2 = 0.02 / math.sqrt(2 * L)
    def lin(i, o, std):
        return {"linear": {"in_features": i, "out_features": o}, "normal": {"mean": 0.0, "std": std}, "zeros": {}}
    blocks = [{"residual": [
        {"sequential": [{"layernorm": {"normalized_shape": C}}, lin(C, 3 * C, 0.02),
                        {"attention": {"num_heads": H, "dropout": 0.0}}, lin(C, C, std2), {"dropout": {"p": 0.0}}]},
        {"sequential": [{"layernorm": {"normalized_shape": C}}, lin(C, 4 * C, 0.02), {"gelu": {}},
                        lin(4 * C, C, std2), {"dropout": {"p": 0.0}}]}]} for _ in range(L)]
    return ([{"summation": [{"embedding": {"num_embeddings": V, "embedding_dim": C}, "normal": {"mean": 0.0, "std": 0.02}},
                            {"position": {"num_embeddings": P, "embedding_dim": C}, "normal": {"mean": 0.0, "std": 0.02}}]},
             {"dropout": {"p": 0.0}}] + blocks +
            [{"layernorm": {"normalized_shape": C}}, {"linear": {"in_features": C, "out_features": V, "bias": False}},
             {"softmaxlast": {"dim": -1}}])


# ------------------------------------------------------------------------------ schemas
class ModelRequest(BaseModel):
    model_id: str = Field(..., examples=["gpt-example"], description="The unique identifier for the model.")


class ModelOnDeviceRequest(ModelRequest):
    device: str = Field("cpu", examples=["cpu", "cuda"], description="Device to run on (cuda = every GPU, RCCL)")


class CreateModelRequest(ModelRequest):
    layers: list[dict] = Field(..., examples=[_gpt2_example_layers()],
                               description="Layer list: each item maps an algo (and init keys) to its args.")
    optimizer: dict = Field(..., examples=[{"adamw": {"lr": 6e-4, "betas": [0.9, 0.95], "eps": 1e-8}}],
                            description="Optimizer name mapped to its args (adam, adamw, sgd).")


class DatasetRequest(BaseModel):
    dataset_id: str = Field(..., examples=["tiny-shakespeare"], description="The unique identifier for the dataset")


class TokenizerRequest(BaseModel):
    encoding: str = Field(..., examples=["tiktoken/gpt2"],
                          description="tiktoken encoding (prefix 'tiktoken/') or HuggingFace tokenizer name")


class DownloadDatasetRequest(DatasetRequest, TokenizerRequest):
    path: str = Field(..., examples=["andriotis/tiny-shakespeare-karpathy"])
    name: str = Field(..., examples=["default"])
    split: str = Field(..., examples=["train"])
    shard_size: int = Field(..., examples=[100000], description="Tokens per shard")


class TrainingRequest(ModelOnDeviceRequest, DatasetRequest):
    shard: int = Field(..., examples=[1], description="Dataset shard to begin from")
    epochs: int = Field(..., examples=[4], description="Number of training epochs")
    batch_size: int = Field(..., examples=[2], description="Sequences per rank per micro-step")
    block_size: int = Field(..., examples=[1024], description="Sequence length")
    step_size: int = Field(..., examples=[2], description="Sequences per accumulation step")


class EvaluateRequest(TrainingRequest):
    target_dataset_id: str | None = Field(None, examples=[None], description="Separate target dataset (optional)")
    shard: int = Field(..., examples=[0])
    epochs: int = Field(..., examples=[2])
    step_size: int = Field(..., examples=[1])


class TokenizeTextRequest(TokenizerRequest):
    text: str = Field(..., examples=["PENR-OZ:\nI say Hello world!"])


class OutputRequest(ModelRequest):
    input: list = Field(..., examples=[[[0]]], description="The initial input context")
    target: list | int | None = Field(None, examples=[None], description="Expected target (optional)")


class GenerateRequest(ModelRequest):
    input: list = Field(..., examples=[[[0]]], description="The initial input context")
    block_size: int = Field(..., examples=[1024], description="Context block size")
    max_new_tokens: int = Field(..., examples=[10])
    temperature: float = Field(1.0, examples=[1.0])
    top_k: int | None = Field(None, examples=[None])
    stop_token: int | None = Field(None, examples=[None], description="Token id that halts generation")
    stream: bool = Field(False, examples=[False], description="Stream tokens as text/plain lines")


class DecodeTokensRequest(TokenizerRequest):
    tokens: list[int] = Field(..., examples=[[0]])


class ImportModelRequest(BaseModel):
    hf_repo_id: str = Field(..., examples=["openai-community/gpt2", "google/gemma-3-1b"])
    model_id: str = Field(..., examples=["gpt2-imported"])
    revision: str | None = Field(None, examples=[None])
    device: str = Field("cpu", examples=["cpu", "cuda"])


class ModelIdQuery(Query):
    description = "The unique identifier for the model"


class DatasetIdQuery(Query):
    description = "The unique identifier for the dataset"


# ------------------------------------------------------------------------------ middleware / errors
@app.middleware("http")
async def gzip_decompression_middleware(request: Request, call_next):
    if request.headers.get("Content-Encoding", "").lower() == "gzip":
        body = gzip.decompress(await request.body())
        request._body = body

        async def receive():  # pragma: no cover - exercised through Starlette
            return {"type": "http.request", "body": body, "more_body": False}
        request._receive = receive
    return await call_next(request)


@app.exception_handler(Exception)
async def generic_exception_handler(_: Request, e: Exception):
    log.error(f"An error occurred: {e}")
    return JSONResponse(status_code=500, content={"detail": "Please refer to server logs"})


@app.exception_handler(KeyError)
async def key_error_handler(_: Request, e: KeyError):
    raise HTTPException(status_code=404, detail=f"Not found error occurred: {e}")


@app.exception_handler(ValueError)
async def value_error_handler(_: Request, e: ValueError):
    raise HTTPException(status_code=400, detail=f"Value error occurred: {e}")


# ------------------------------------------------------------------------------ serving cache
def serve_device() -> str:
    dev = os.environ.get("PENROZ_SERVE_DEVICE")
    if dev:
        return dev
    try:
        import torch
        return "cuda" if torch.cuda.is_available() else "cpu"
    except Exception:  # pragma: no cover
        return "cpu"


_cache_lock = threading.Lock()
_model_cache: dict[str, tuple[float, NeuralNetworkModel]] = {}


def serving_lock(model: NeuralNetworkModel) -> threading.Lock:
    """The lock every request holds while it runs on ``model``.

    A cached serving model is ONE module tree shared by all requests; generation attaches its
    KV cache / graph decoder to that tree and moves position offsets, so two requests must never
    run on it at once (the reference rebuilt a private model per request, ``main.py:401-434``).
    A plain ``Lock`` (not ``RLock``): a streaming response acquires it on the threadpool thread
    of its first chunk and may release it on another."""
    lk = model.__dict__.get("_serve_lock")
    if lk is None:
        with _cache_lock:
            lk = model.__dict__.setdefault("_serve_lock", threading.Lock())
    return lk


def _lock_timeout_s() -> float:
    return float(os.environ.get("PENROZ_SERVE_LOCK_TIMEOUT", "120"))


class _Held:
    """``with _Held(model):`` — the model's serving lock, waited for at most
    ``PENROZ_SERVE_LOCK_TIMEOUT`` seconds (then 503: busy), never indefinitely."""

    def __init__(self, model):
        self.lock = serving_lock(model)

    def __enter__(self):
        if not self.lock.acquire(timeout=_lock_timeout_s()):
            raise HTTPException(status_code=503, detail="Model is busy serving another request; retry later.")
        return self

    def __exit__(self, *exc):
        self.lock.release()


class _LockedStream:
    """A token stream that owns the model's serving lock from before the response starts until
    the stream is finished OR abandoned. The response's background task (run by Starlette after
    the body, also when the client disconnected mid-stream) closes the generator — retrying
    while a threadpool thread is still inside it producing a token — so its ``finally`` releases
    the lock at once instead of whenever the abandoned generator is garbage-collected."""

    def __init__(self, model, tokens):
        self.lock = serving_lock(model)
        if not self.lock.acquire(timeout=_lock_timeout_s()):
            raise HTTPException(status_code=503, detail="Model is busy serving another request; retry later.")
        self._released = False
        self._guard = threading.Lock()
        self.gen = self._run(tokens)

    def _release(self):
        with self._guard:
            if not self._released:
                self._released = True
                self.lock.release()

    def _run(self, tokens):
        try:
            for token in tokens:
                yield f"{token}\n"
        finally:
            self._release()

    def close(self):
        import time
        deadline = time.monotonic() + _lock_timeout_s()
        while True:
            try:
                self.gen.close()  # suspended at a yield (or finished): runs the finally now
                break
            except ValueError:  # "generator already executing" on a threadpool thread
                if time.monotonic() > deadline:
                    return
                time.sleep(0.005)
        self._release()  # never started: the finally never ran


def _checkpoint_mtime(model_id: str) -> float | None:
    p = os.path.join(NeuralNetworkModel.SHM_PATH, NeuralNetworkModel.get_model_path(model_id))
    if not os.path.exists(p):
        p = NeuralNetworkModel.get_model_path(model_id)
    return os.path.getmtime(p) if os.path.exists(p) else None


def load_for_serving(model_id: str) -> NeuralNetworkModel:
    """Deserialize (or reuse) a model and place it on the serving device."""
    if os.environ.get("PENROZ_SERVE_CACHE", "1") != "1":
        model = NeuralNetworkModel.deserialize(model_id)
        dev = serve_device()
        return model.to(dev) if dev != "cpu" and hasattr(model, "to") else model
    mtime = _checkpoint_mtime(model_id)
    with _cache_lock:
        hit = _model_cache.get(model_id)
        if hit is not None and mtime is not None and hit[0] == mtime:
            return hit[1]
    model = NeuralNetworkModel.deserialize(model_id)
    dev = serve_device()
    if dev != "cpu":
        model.to(dev)
    with _cache_lock:
        if mtime is not None:
            while len(_model_cache) >= int(os.environ.get("PENROZ_SERVE_CACHE_SIZE", "2")):
                _model_cache.pop(next(iter(_model_cache)))
            _model_cache[model_id] = (mtime, model)
    return model


def _evict(model_id: str):
    with _cache_lock:
        _model_cache.pop(model_id, None)


# ------------------------------------------------------------------------------ routes
@app.get("/", include_in_schema=False)
def redirect_to_dashboard():
    return RedirectResponse(url="/dashboard")


@app.get("/dashboard", response_class=HTMLResponse, include_in_schema=False)
async def dashboard():
    with open(os.path.join(HERE, "templates", "dashboard.html")) as f:
        return HTMLResponse(f.read())


@app.post("/model/")
def create_model(body: CreateModelRequest = Body(...)):
    model_id = body.model_id
    log.info(f"Requesting creation of model {model_id}")
    model = NeuralNetworkModel(model_id, Mapper(body.layers, body.optimizer))
    model.serialize()
    _evict(model_id)
    return {"message": f"Model {model_id} created and saved successfully"}


@app.post("/import/")
async def import_from_huggingface(body: ImportModelRequest = Body(...)):
    model_id = body.model_id
    lock = model_locks.setdefault(model_id, Lock())
    if lock.locked():
        raise HTTPException(status_code=409, detail=f"Operation already in progress for model {model_id}.")
    async with lock:
        await run_in_threadpool(NeuralNetworkModel.from_huggingface, model_id, body.hf_repo_id, body.revision,
                                body.device)
    _evict(model_id)
    return {"model_id": model_id, "status": "imported",
            "message": f"Model imported from HuggingFace ({body.hf_repo_id}) and ready for use"}


@app.get("/dataset/")
def list_dataset(dataset_id: str = DatasetIdQuery(...)):
    return {"files": Loader(dataset_id).list()}


@app.post("/dataset/")
async def download_dataset(body: DownloadDatasetRequest = Body(...)):
    dataset_id = body.dataset_id
    lock = dataset_locks.setdefault(dataset_id, Lock())
    if lock.locked():
        raise HTTPException(status_code=409, detail=f"Downloading dataset {dataset_id} already in progress.")
    downloader = Downloader(dataset_id, body.shard_size, body.encoding)

    async def download():
        async with lock:
            await run_in_threadpool(downloader.download, body.path, body.name, body.split)

    create_task(download())
    return JSONResponse(content={"message": f"Downloading Dataset {dataset_id} asynchronously."}, status_code=202)


@app.delete("/dataset/")
def delete_dataset(dataset_id: str = DatasetIdQuery(...)):
    Loader(dataset_id).delete()
    return Response(status_code=204)


@app.post("/tokenize/")
def tokenize_text(body: TokenizeTextRequest = Body(...)):
    return {"encoding": body.encoding, "tokens": Tokenizer(body.encoding).tokenize(body.text)}


@app.post("/output/")
def compute_model_output(body: OutputRequest = Body(...)):
    model = load_for_serving(body.model_id)
    with _Held(model):
        output, cost = model.compute_output(body.input, body.target)
    return {"output": output, "cost": cost}


@app.post("/evaluate/")
def evaluate_model(body: EvaluateRequest = Body(...)):
    model = load_for_serving(body.model_id)
    with _Held(model):
        cost = model.evaluate_model(body.dataset_id, body.target_dataset_id, body.shard, body.epochs,
                                    body.batch_size, body.block_size, body.step_size)
    return {"cost": cost}


@app.post("/generate/")
def model_generate(body: GenerateRequest = Body(...)):
    model = load_for_serving(body.model_id)
    if body.stream:
        # the lock is held for the stream's whole lifetime (the KV cache stays attached between
        # chunks) and released by the background task even when the client goes away mid-stream
        from starlette.background import BackgroundTask
        st = _LockedStream(model, model.generate_tokens_stream(body.input, body.block_size, body.max_new_tokens,
                                                              body.temperature, body.top_k, body.stop_token))
        return StreamingResponse(st.gen, media_type="text/plain", background=BackgroundTask(st.close))
    with _Held(model):
        tokens = model.generate_tokens(body.input, body.block_size, body.max_new_tokens, body.temperature,
                                       body.top_k, body.stop_token)
    return {"tokens": tokens}


@app.post("/decode/")
def decode_tokens(body: DecodeTokensRequest = Body(...)):
    return {"encoding": body.encoding, "text": Tokenizer(body.encoding).decode(body.tokens)}


def _mark_failed(model_id: str, rank: int, code: int):
    try:
        NeuralNetworkModel.mark_status(model_id, "Error", f"Training worker rank {rank} exited with code {code}")
    except Exception as e:  # pragma: no cover - best effort
        log.error(f"could not mark model {model_id} as failed: {e}")


def run_training_job(model_id: str, device: str, dataset_id: str, shard: int, epochs: int, batch_size: int,
                     block_size: int, step_size: int) -> int:
    """Blocking: launch the distributed workers and return the launcher's exit code."""
    code = launcher.launch_single_node_ddp(
        model_id, device, NeuralNetworkModel.train_model_on_device, model_id, device, dataset_id, shard, epochs,
        batch_size, block_size, step_size, on_failure=lambda r, c: _mark_failed(model_id, r, c))
    _evict(model_id)
    return code


@app.put("/train/")
async def train_model(body: TrainingRequest = Body(...)):
    model_id = body.model_id
    lock = model_locks.setdefault(model_id, Lock())
    if lock.locked():
        raise HTTPException(status_code=409, detail=f"Training already in progress for model {model_id}.")

    async def _launch():
        async with lock:
            code = await run_in_threadpool(run_training_job, model_id, body.device, body.dataset_id, body.shard,
                                           body.epochs, body.batch_size, body.block_size, body.step_size)
            log.info(f"Distributed training for model {model_id} finished with exit code {code}")

    create_task(_launch())
    return JSONResponse(content={"message": f"Training for model {model_id} started asynchronously."}, status_code=202)


@app.get("/progress/")
def model_progress(model_id: str = ModelIdQuery(...)):
    doc = NeuralNetworkModel.read_progress(model_id)
    return {"progress": doc["progress"], "average_cost": doc["average_cost"],
            "average_cost_history": doc["average_cost_history"], "status": doc["status"]}


@app.get("/stats/")
def model_stats(model_id: str = ModelIdQuery(...)):
    return NeuralNetworkModel.read_stats(model_id)


@app.delete("/model/")
def delete_model(model_id: str = ModelIdQuery(...)):
    NeuralNetworkModel.delete(model_id)
    _evict(model_id)
    return Response(status_code=204)


def main():  # pragma: no cover - process entry point
    import uvicorn
    from penroz.parallel.dist import load_log_config
    uvicorn.run(app, host=os.environ.get("PENROZ_HOST", "127.0.0.1"), port=int(os.environ.get("PENROZ_PORT", "8000")),
                log_config=load_log_config())


if __name__ == "__main__":  # pragma: no cover
    main()
