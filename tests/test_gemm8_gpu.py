"""Native 8-phase forward / dgrad GEMM (csrc/kernels/gemm8.hip) vs an fp32 torch reference.

The kernel is persistent (one workgroup per CU walking several tiles, the DMA stream running on
into the next tile): shapes with more tiles than CUs (8192x3072, 16384x768, 777x50304) exercise
the tile hand-over, the epilogue-store accounting in the counted waits and the bias ring.

Operands are random (not zero-filled: a swapped C-write or a wrong k-order shows), B is asymmetric,
and the shapes cover ragged M and N (rows / columns past the matrix edge are clamped in the DMA
and never stored), K from the minimum 128 to the GPT-2 fc2 / qkv-dgrad depths, every epilogue
(none, bias, bias + GELU erf / tanh writing both outputs) and strided (padded-row) operands."""
import pytest
import torch

from penroz.ops import _ext

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref(a, b, bias):
    r = a.float() @ b.float().t()
    return r + bias.float() if bias is not None else r


@pytest.mark.parametrize("M,N,K", [(512, 512, 128), (300, 264, 256), (1024, 2304, 768), (4096, 768, 3072),
                                   (777, 50304, 768), (256, 8, 384), (8192, 3072, 768), (16384, 768, 2304)])
@pytest.mark.parametrize("epi", ["none", "bias", "gelu", "gelu_tanh"])
def test_gemm8_matches_fp32(M, N, K, epi):
    torch.manual_seed(M + N + K)
    a = (torch.rand(M, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    b = ((torch.rand(N, K, device=DEV) * 2 - 1) * 0.1 + torch.arange(N, device=DEV).view(-1, 1) * 1e-3).to(torch.bfloat16)
    bias = (torch.rand(N, device=DEV) - 0.5).to(torch.bfloat16) if epi != "none" else None
    out = torch.full((M, N), 7.0, device=DEV, dtype=torch.bfloat16)
    act = torch.full((M, N), 7.0, device=DEV, dtype=torch.bfloat16) if epi.startswith("gelu") else None
    _ext.kernels().gemm8_bf16(a, b, bias, out, act, 1 if epi == "gelu_tanh" else 0)
    ref = _ref(a, b, bias)
    err = (out.float() - ref).abs().max().item()
    assert err <= 0.02 * max(1.0, ref.abs().max().item()), err
    rel = ((out.float() - ref).norm() / ref.norm()).item()
    assert rel < 4e-3, rel
    if act is not None:
        want = torch.nn.functional.gelu(out.float(), approximate="tanh" if epi == "gelu_tanh" else "none")
        assert (act.float() - want).abs().max().item() <= 0.02 * max(1.0, want.abs().max().item())


def test_gemm8_strided_operands_and_output():
    """Padded row strides (the executor's lm_head logits buffer: V = 50257 rows padded to 50264)."""
    M, N, K = 512, 1000, 256
    abuf = (torch.rand(M, K + 64, device=DEV) * 2 - 1).to(torch.bfloat16)
    bbuf = (torch.rand(N, K + 8, device=DEV) * 2 - 1).to(torch.bfloat16)
    obuf = torch.zeros(M, 1008, device=DEV, dtype=torch.bfloat16)
    a, b, out = abuf[:, :K], bbuf[:, :K], obuf[:, :N]
    _ext.kernels().gemm8_bf16(a, b, None, out)
    ref = _ref(a, b, None)
    assert ((out.float() - ref).norm() / ref.norm()).item() < 4e-3
    assert torch.all(obuf[:, N:] == 0), "columns past N must not be written"


def test_gemm8_rejects_bad_shapes():
    a = torch.zeros(64, 96, device=DEV, dtype=torch.bfloat16)
    b = torch.zeros(64, 96, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="K % 128"):
        _ext.kernels().gemm8_bf16(a, b, None, torch.empty(64, 64, device=DEV, dtype=torch.bfloat16))


def test_gemm8_dma_path_probe():
    """The GEMM's LDS-DMA primitive (buffer_load_dwordx4 ... lds through a buffer resource): lands
    lane-linear at low and high LDS offsets (past 64 KiB), honours soffset, and reads 0 past the
    resource's size (how the kernel zero-fills rows beyond the matrix edge)."""
    k = _ext.kernels()
    src = torch.arange(8192, device=DEV, dtype=torch.int32).view(torch.bfloat16)
    words = src.view(torch.int32)
    for lds_off in (0, 65536, 133120):
        out = k.gemm8_dma_probe(src, 32768, lds_off, 0).view(-1)
        assert torch.equal(out[:512], words[:512]), lds_off
    out = k.gemm8_dma_probe(src, 32768, 0, 4096).view(-1)
    assert torch.equal(out[:512], words[1024:1536])
    out = k.gemm8_dma_probe(src, 1024, 0, 0).view(-1)
    assert torch.equal(out[:256], words[:256]) and int(out[256:512].abs().sum()) == 0
