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


def _tiles(qb, BM, BN, T):
    return (min(T, (qb + 1) * BM) + BN - 1) // BN


@pytest.mark.parametrize("mode", ["1", "2"])
@pytest.mark.parametrize("nblk,nvh,slots,BM,T", [(8, 32, 256, 128, 1024), (16, 32, 512, 64, 1024), (8, 64, 256, 128, 1024),
                                                 (3, 2, 256, 128, 300), (40, 8, 512, 64, 2560), (1, 4, 256, 128, 100)])
def test_attn_work_plan_covers_every_tile_once(monkeypatch, mode, nblk, nvh, slots, BM, T):
    """flash_attn_gen.hip's causal work list: every query block's key tiles are covered exactly
    once (whole, or as the two halves [0, n/2) and [n/2, n)), split blocks are exactly those at or
    above split0, and items come heaviest first (the dispatch order the balance relies on)."""
    monkeypatch.setenv("PENROZ_ATTN_KV_SPLIT", mode)
    r = _ext.kernels().attn_work_plan(nblk, nvh, slots, BM, 32, T, 256, 2.7)
    n, split0, items = r[0], r[1], r[2:]
    if split0 >= nblk:  # nothing split: the kernel walks the blocks heaviest first by formula
        assert n == nblk and items == []
        return
    if mode == "2":
        assert split0 == 1
    assert n == len(items) == nblk + (nblk - split0)
    covered = {}
    sizes = []
    for e in items:
        qb, part = e & 0xFFFF, e >> 16
        nt = _tiles(qb, BM, 32, T)
        lo, hi = {0: (0, nt), 1: (0, nt // 2), 2: (nt // 2, nt)}[part]
        assert (part == 0) == (qb < split0)
        covered.setdefault(qb, []).append((lo, hi))
        sizes.append(hi - lo)
    for qb in range(nblk):
        spans = sorted(covered[qb])
        assert spans[0][0] == 0 and spans[-1][1] == _tiles(qb, BM, 32, T)
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    assert sizes == sorted(sizes, reverse=True)


def test_attn_work_plan_off_and_many_rounds(monkeypatch):
    """PENROZ_ATTN_KV_SPLIT=0 never splits; grids of several rounds are not split either."""
    monkeypatch.setenv("PENROZ_ATTN_KV_SPLIT", "0")
    assert _ext.kernels().attn_work_plan(8, 32, 256, 128, 32, 1024, 256, 2.7)[:2] == [8, 8]
    monkeypatch.setenv("PENROZ_ATTN_KV_SPLIT", "1")
    assert _ext.kernels().attn_work_plan(8, 768, 256, 128, 32, 1024, 256, 2.7)[:2] == [8, 8]
    r = _ext.kernels().attn_work_plan(8, 32, 256, 128, 32, 1024, 256, 2.7)
    assert r[1] < 8  # the Gemma-3 1B B=8 forward grid (one round) is split
