"""Host-side launch plans of the HIP extension (no GPU needed: the built extension imports on the
CPU runner): the fused decode QKV + RoPE kernel's split-K plan is exported by the kernel's own
source and the Python admission check reads it instead of re-deriving the rule."""
import pytest

from penroz.ops import _ext, gemm as G

pytestmark = pytest.mark.skipif(not _ext.available(), reason="HIP extension not built")


@pytest.mark.parametrize("M,N,K", [(1, 1536, 1152), (64, 1536, 1152), (16, 6144, 5376), (1, 2304, 768),
                                   (64, 8192, 2048), (32, 4096 + 512, 4096)])
def test_qkv_rope_plan_matches_launch_rule(M, N, K):
    split, ws, counters = _ext.kernels().skinny_qkv_rope_plan(M, N, K)
    ntiles, steps = N // 32, K // 32
    assert 1 <= split <= max(1, min(16, steps))
    assert split == 1 or ntiles < 128  # wide outputs never split
    assert split == 1 or ntiles * split >= 192 or split == min(steps // 4, 16)  # ~192 workgroups
    mb = 1 if M <= 16 else 2 if M <= 32 else 4
    assert ws == (split * ntiles * mb * 512 if split > 1 else 0)
    assert counters == (ntiles if split > 1 else 0)
    assert G.qkv_rope_plan_fits(M, N, K) == (ws <= 1 << 19 and counters <= 1 << 12)


def test_qkv_rope_plan_admission_over_every_split():
    """Every split the launcher would pick is admitted exactly when its slabs fit the shared
    workspace; at 64 rows some narrow outputs do not (95 tiles split 3 ways: 583 680 floats), and
    those fall back before any graph capture instead of throwing inside it."""
    refused = []
    for tiles in range(1, 128):
        split, ws, counters = _ext.kernels().skinny_qkv_rope_plan(64, 32 * tiles, 32 * 4096)
        assert G.qkv_rope_plan_fits(64, 32 * tiles, 32 * 4096) == (ws <= 1 << 19)
        if ws > 1 << 19:
            refused.append(tiles)
    assert 95 in refused
    split, ws, _ = _ext.kernels().skinny_qkv_rope_plan(64, 32 * 16, 32 * 64)
    assert split == 12 and ws == 12 * 16 * 4 * 512
