"""Deferred-epilogue forward GEMM (csrc/kernels/gemm_epi.hip) vs an fp32 torch reference.

The kernel is persistent (one workgroup per CU walking several 256x256 tiles) and stores tile t's
output during tile t+1's main loop: shapes with more tiles than CUs (8192x3072, 16384x768,
777x50304) exercise the hand-over of the deferred units, the first tile (nothing to store yet) and
the flush after the last tile; ragged M / N (rows past M dropped by the panel resource, columns
past N by the per-store column check), K from the minimum 640 up to 3072, every epilogue (none,
bias, bias + erf / tanh GELU writing both outputs) and padded row strides.
Operands are random (not zero-filled) and B is asymmetric, so a transposed or misplaced store shows."""
import pytest
import torch

from penroz.ops import _ext

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref(a, b, bias):
    r = a.float() @ b.float().t()
    return r + bias.float() if bias is not None else r


@pytest.mark.parametrize("M,N,K", [(512, 512, 768), (300, 264, 640), (1024, 2304, 768), (4096, 768, 3072),
                                   (777, 50304, 768), (256, 8, 1280), (8192, 3072, 768), (16384, 768, 768),
                                   (65536 // 8, 3072, 768)])
@pytest.mark.parametrize("epi", ["none", "bias", "gelu", "gelu_tanh"])
def test_gemm_epi_matches_fp32(M, N, K, epi):
    torch.manual_seed(M + N + K)
    a = (torch.rand(M, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    b = ((torch.rand(N, K, device=DEV) * 2 - 1) * 0.1 + torch.arange(N, device=DEV).view(-1, 1) * 1e-3).to(torch.bfloat16)
    bias = (torch.rand(N, device=DEV) - 0.5).to(torch.bfloat16) if epi != "none" else None
    out = torch.full((M, N), 7.0, device=DEV, dtype=torch.bfloat16)
    act = torch.full((M, N), 7.0, device=DEV, dtype=torch.bfloat16) if epi.startswith("gelu") else None
    _ext.kernels().gemm_epi_bf16(a, b, bias, out, act, 1 if epi == "gelu_tanh" else 0)
    torch.cuda.synchronize()
    ref = _ref(a, b, bias)
    err = (out.float() - ref).abs().max().item()
    assert err <= 0.02 * max(1.0, ref.abs().max().item()), err
    rel = ((out.float() - ref).norm() / ref.norm()).item()
    assert rel < 4e-3, rel
    if act is not None:
        want = torch.nn.functional.gelu(out.float(), approximate="tanh" if epi == "gelu_tanh" else "none")
        assert (act.float() - want).abs().max().item() <= 0.02 * max(1.0, want.abs().max().item())
        # the GELU epilogue reads the bf16-rounded pre-activation, like the unfused pair: after
        # rounding to bf16 it matches torch's GELU of that tensor to within one bf16 ulp
        ulp = (act.float() - want.to(torch.bfloat16).float()).abs() / want.abs().clamp_min(1e-3)
        assert ulp.max().item() < 1.6e-2


def test_gemm_epi_strided_operands_and_output():
    """Padded row strides (the executor's lm_head logits buffer: V = 50257 rows padded to 50264)."""
    M, N, K = 600, 1000, 768
    abuf = (torch.rand(M, K + 64, device=DEV) * 2 - 1).to(torch.bfloat16)
    bbuf = (torch.rand(N, K + 8, device=DEV) * 2 - 1).to(torch.bfloat16)
    obuf = torch.zeros(M, 1008, device=DEV, dtype=torch.bfloat16)
    a, b, out = abuf[:, :K], bbuf[:, :K], obuf[:, :N]
    _ext.kernels().gemm_epi_bf16(a, b, None, out)
    torch.cuda.synchronize()
    ref = _ref(a, b, None)
    assert ((out.float() - ref).norm() / ref.norm()).item() < 4e-3
    assert torch.all(obuf[:, N:] == 0), "columns past N must not be written"


def test_gemm_epi_repeatable():
    """Same inputs, same bits (no data race between the DMA stream and the deferred stores)."""
    M, N, K = 8192, 3072, 768
    a = (torch.rand(M, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(N, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    bias = (torch.rand(N, device=DEV) - 0.5).to(torch.bfloat16)
    outs = []
    for _ in range(3):
        o, g = torch.empty(M, N, device=DEV, dtype=torch.bfloat16), torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        _ext.kernels().gemm_epi_bf16(a, b, bias, o, g, 0)
        outs.append((o, g))
    torch.cuda.synchronize()
    for o, g in outs[1:]:
        assert torch.equal(o, outs[0][0]) and torch.equal(g, outs[0][1])


def test_gemm_epi_rejects_bad_shapes():
    k = _ext.kernels()
    assert not k.gemm_epi_supported(512, 512, 512) and not k.gemm_epi_supported(512, 500, 768)
    assert k.gemm_epi_supported(512, 512, 768)
    a = torch.zeros(64, 512, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        k.gemm_epi_bf16(a, torch.zeros(64, 512, device=DEV, dtype=torch.bfloat16), None,
                        torch.empty(64, 64, device=DEV, dtype=torch.bfloat16))


@pytest.mark.parametrize("M,N,K", [(512, 512, 768), (300, 264, 640), (4096, 3072, 768), (777, 1000, 768),
                                   (8192, 3072, 768)])
@pytest.mark.parametrize("approx", [0, 1])
def test_gemm_epi_dgelu_matches_unfused(M, N, K, approx):
    """out = bf16(dy·wtᵀ)·GELU'(pre) and dbias += column sums of out, against the unfused pair
    (fp32 GEMM rounded to bf16, then the GELU backward in fp32, rounded to bf16)."""
    torch.manual_seed(M + N + K + approx)
    dy = (torch.rand(M, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    wt = ((torch.rand(N, K, device=DEV) * 2 - 1) * 0.1 + torch.arange(N, device=DEV).view(-1, 1) * 1e-3).to(torch.bfloat16)
    pre = (torch.randn(M, N, device=DEV) * 2).to(torch.bfloat16)
    out = torch.full((M, N), 7.0, device=DEV, dtype=torch.bfloat16)
    dbias = torch.full((N,), 0.5, device=DEV)
    _ext.kernels().gemm_epi_dgelu(dy, wt, pre, out, dbias, approx)
    torch.cuda.synchronize()
    dact = (dy.float() @ wt.float().t()).to(torch.bfloat16).float()
    x = pre.float().requires_grad_()
    torch.nn.functional.gelu(x, approximate="tanh" if approx else "none").backward(dact)
    ref = x.grad
    rel = ((out.float() - ref).norm() / ref.norm()).item()
    assert rel < 8e-3, rel
    want_b = 0.5 + out.float().sum(0)  # the kernel sums the values it stored
    assert ((dbias - want_b).abs().max() / want_b.abs().max()).item() < 1e-4
