"""Native NT GEMM (csrc/kernels/gemm_nt.hip) against a plain PyTorch fp32 reference of the same op:
out = a·bᵀ (+ bias) (→ GELU), bf16 in / out. Covers the persistent multi-tile path (small grids),
the store-pending vmcnt bookkeeping (many tiles per workgroup), ragged N (the last column tile
half full), strided A rows, and both GELU forms."""
import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from penroz.ops import _ext

DEV = "cuda"


def _ref(a, b, bias, gelu):
    y = a.float() @ b.float().t()
    if bias is not None:
        y = y + bias.float()
    pre = y.to(torch.bfloat16)
    if gelu is None:
        return pre, None
    return pre, torch.nn.functional.gelu(pre.float(), approximate=gelu).to(torch.bfloat16)


def _close(got, ref, tol=1e-2):
    rel = ((got.float() - ref.float()).norm() / ref.float().norm()).item()
    assert rel < tol, rel
    # element-wise: at most a couple of bf16 ulps apart (fp32 accumulation order differs)
    d = (got.float() - ref.float()).abs()
    assert (d <= 2e-2 * ref.float().abs() + 2e-2).float().mean().item() > 0.999


@pytest.mark.parametrize("M,N,K,grid", [(512, 256, 160, 0), (1024, 768, 768, 0), (2048, 768, 256, 8),
                                        (512, 384, 256, 0), (768, 640, 192, 16), (4096, 2304, 768, 0),
                                        (256, 1152, 256, 0)])
@pytest.mark.parametrize("mode", ["plain", "bias", "gelu", "gelu_tanh"])
def test_gemm_nt_matches_fp32(M, N, K, grid, mode):
    k = _ext.kernels()
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    a = torch.randn(M, K, device=DEV, generator=g).to(torch.bfloat16)
    b = (torch.randn(N, K, device=DEV, generator=g) / K ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, device=DEV, generator=g).to(torch.bfloat16) if mode != "plain" else None
    gelu = {"gelu": "none", "gelu_tanh": "tanh"}.get(mode)
    assert k.gemm_nt_supported(M, N, K)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    act = torch.empty_like(out) if gelu else None
    k.gemm_nt(a, b, bias, out, act, 1 if gelu == "tanh" else 0, 0, grid)
    pre, ref_act = _ref(a, b, bias, gelu)
    _close(out, pre)
    if gelu:
        _close(act, ref_act)


def test_gemm_nt_strided_a_and_out():
    """A rows with a stride > K (a view into a wider buffer) and an output with padded rows."""
    k = _ext.kernels()
    g = torch.Generator(device=DEV).manual_seed(3)
    big = torch.randn(1024, 1024, device=DEV, generator=g).to(torch.bfloat16)
    a = big[:, 128:128 + 512]
    b = (torch.randn(512, 512, device=DEV, generator=g) / 20).to(torch.bfloat16)
    obuf = torch.full((1024, 520), 7.0, device=DEV, dtype=torch.bfloat16)
    out = obuf[:, :512]
    k.gemm_nt(a, b, None, out)
    _close(out, _ref(a, b, None, None)[0])
    assert (obuf[:, 512:] == 7.0).all(), "wrote past the row"


def test_gemm_nt_many_tiles_per_workgroup_deterministic():
    """grid 8: every workgroup walks 96 tiles (the DMA ring crosses 95 tile boundaries); two
    launches agree bitwise."""
    k = _ext.kernels()
    g = torch.Generator(device=DEV).manual_seed(5)
    a = torch.randn(8192, 768, device=DEV, generator=g).to(torch.bfloat16)
    b = (torch.randn(3072, 768, device=DEV, generator=g) / 28).to(torch.bfloat16)
    bias = torch.randn(3072, device=DEV, generator=g).to(torch.bfloat16)
    o1 = torch.empty(8192, 3072, device=DEV, dtype=torch.bfloat16)
    o2 = torch.empty_like(o1)
    k.gemm_nt(a, b, bias, o1, None, 0, 0, 8)
    k.gemm_nt(a, b, bias, o2, None, 0, 4, 0)
    _close(o1, _ref(a, b, bias, None)[0])
    assert torch.equal(o1, o2)
