"""Two ranks of the fused GPT executor on ONE MI355X (gloo over GPU tensors): rehearses the
data-parallel path of the headline bench (bucketed, backward-overlapped gradient all-reduce in
the executor, rank-0 parameter broadcast) without a second GPU. The RCCL transport itself is
exercised by the driver's multi-GPU bench; everything above the collective call is shared.

Check: the all-reduced gradient of two ranks (each with its own micro-batch) equals the gradient
of one process on the concatenated batch, and both ranks hold identical parameters afterwards.
"""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - CPU runner
    pytest.skip("needs a GPU", allow_module_level=True)

import torch.distributed as dist
import torch.multiprocessing as mp

import bench


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(dev):
    from penroz.models.mapper import Mapper
    from penroz.models.model import NeuralNetworkModel
    torch.manual_seed(123)
    m = NeuralNetworkModel("ddp_gpu", Mapper(bench.gpt2_layers(V=512, C=128, L=2, H=2, P=128),
                                             {"adamw": {"lr": 1e-3, "betas": [0.9, 0.95]}}))
    m.to(dev)
    return m


def _batch(rank):
    g = torch.Generator().manual_seed(1000 + rank)
    b = torch.randint(0, 512, (4, 129), generator=g)
    return b[:, :-1].contiguous(), b[:, 1:].contiguous()


def _worker(rank, world, port, out, bucket_mb, overlap):
    per_bucket = overlap == "per_bucket"
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", PENROZ_BUCKET_MB=str(bucket_mb),
                      PENROZ_OVERLAP_OPT=str(1 if per_bucket else overlap),
                      PENROZ_OPT_PER_BUCKET="1" if per_bucket else "0")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import penroz.parallel.reducer as R
    R.DEFAULT_BUCKET_MB = R.GLOO_BUCKET_MB = bucket_mb  # several buckets for this small model
    from penroz.models.executor import GPTExecutor
    dev = torch.device("cuda", 0)
    model = _model(dev)
    if rank == 1:  # different init on rank 1: the rank-0 broadcast must overwrite it
        with torch.no_grad():
            for p in model.parameters():
                p.add_(0.01)
    ex = GPTExecutor(model, dev)
    ex.setup_training(True)
    assert ex.reducer is not None and len(ex.reducer.buckets) > 1
    x, y = _batch(rank)
    ex.zero_grad()
    if per_bucket:
        # the fused AdamW of each bucket runs inside the backward, on the optimizer stream, as soon
        # as the bucket's all-reduce has landed; the embedding bucket is cut into pieces
        assert len(ex.reducer.buckets) >= 4
        ex.train_micro_step(x.to(dev), y.to(dev), 1.0, sync=True, fuse_optimizer=True)
        assert ex.opt_overlap_mode() == "per-bucket-in-backward" and ex._opt_done
        assert ex._opt_buckets_done == set(range(len(ex.reducer.buckets)))
        ex.optimizer_step()  # nothing left to do
        torch.cuda.synchronize()
        torch.save(ex.flat_grad.cpu(), f"{out}/grad{rank}.pt")
        torch.save(ex.flat.cpu(), f"{out}/param{rank}.pt")
        dist.barrier()
        dist.destroy_process_group()
        return
    ex.train_micro_step(x.to(dev), y.to(dev), 1.0, sync=True)
    assert ex._reduce_pending == bool(overlap)  # overlap: the last buckets are still reducing
    if rank == 0:  # the optimizer consumes the in-flight buckets one by one
        ex.optimizer_step()
        ex.wait_gradients()
    else:          # explicit wait first
        ex.wait_gradients()
        ex.optimizer_step()
    torch.cuda.synchronize()
    torch.save(ex.flat_grad.cpu(), f"{out}/grad{rank}.pt")
    torch.cuda.synchronize()
    torch.save(ex.flat.cpu(), f"{out}/param{rank}.pt")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("overlap", [0, 1, "per_bucket"])
def test_fused_executor_two_ranks_match_single_process(tmp_path, overlap):
    mp.spawn(_worker, args=(2, _port(), str(tmp_path), 0.05, overlap), nprocs=2, join=True)
    from penroz.models.executor import GPTExecutor
    dev = torch.device("cuda", 0)
    model = _model(dev)
    ex = GPTExecutor(model, dev)
    ex.setup_training(False)
    x0, y0 = _batch(0)
    x1, y1 = _batch(1)
    ex.zero_grad()
    ex.train_micro_step(torch.cat([x0, x1]).to(dev), torch.cat([y0, y1]).to(dev), 1.0, sync=True)
    torch.cuda.synchronize()
    ref = ex.flat_grad.cpu()
    ex.optimizer_step()
    torch.cuda.synchronize()
    ref_p = ex.flat.cpu()
    g0, g1 = torch.load(tmp_path / "grad0.pt"), torch.load(tmp_path / "grad1.pt")
    assert torch.equal(g0, g1), "ranks disagree after the all-reduce"
    rel = (g0 - ref).norm() / ref.norm()
    assert rel < 1e-3, f"all-reduced gradient differs from the single-process gradient: {rel}"
    p0, p1 = torch.load(tmp_path / "param0.pt"), torch.load(tmp_path / "param1.pt")
    assert torch.equal(p0, p1), "parameters diverged across ranks"
    # one AdamW step from identical weights agrees with the single-process step (the first Adam
    # update is ~lr·sign(g): only gradients at rounding level may flip, bounded by 2·lr)
    diff = (p0 - ref_p).abs()
    assert diff.max() <= 2.1e-3 and (diff > 1e-5).float().mean() < 1e-3, (diff.max(), (diff > 1e-5).float().mean())
