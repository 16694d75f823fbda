// Host-side launch planning shared by the HIP launch wrappers — plain C++ (no HIP headers), so
// the same code is also compiled into tests/native/host_plan_test.cpp and run under the host
// AddressSanitizer / UndefinedBehaviorSanitizer (tests/test_host_sanitizers.py).
#pragma once
#include <algorithm>
#include <cstdint>

namespace penroz {

struct SplitK {
  int splits;  // workgroups per output tile along K
  int klen;    // K range of one split (multiple of bk)
};

// Split-K count for the weight-gradient GEMM from a wave-quantisation cost model: the launch runs
// ceil(ntiles·s / slots) waves of workgroups, each 1/s of the K loop long, plus the fp32 slab
// round trip (s slabs written and read once) priced against the per-workgroup MFMA time.
// slots = resident workgroups (1 per CU for the 256-tile kernel, 2 for the 128-tile one).
inline SplitK plan_wgrad_splits(int M, int N, int K, int tile, int n_cu, int bk) {
  SplitK r{1, 0};
  if (M <= 0 || N <= 0 || K <= 0 || tile <= 0 || bk <= 0) return r;
  const int64_t tiles_m = (M + tile - 1) / tile, tiles_n = (N + tile - 1) / tile;
  const int64_t ntiles = tiles_m * tiles_n;
  const int64_t slots = tile == 256 ? std::max(1, n_cu) : 2 * (int64_t)std::max(1, n_cu);
  const double wg_full_k = (double)tile * tile * 2.0 * K / (tile == 256 ? 2.3e12 : 1.1e12);  // seconds
  double best = 1e30;
  const int smax = std::min(64, std::max(1, K / 512));
  for (int s = 1; s <= smax; ++s) {
    const double waves = (double)((ntiles * s + slots - 1) / slots);
    const double slab = s > 1 ? (double)s * M * N * 8.0 / 4.0e12 : 0.0;
    const double cost = waves * wg_full_k / s + slab;
    if (cost < best * 0.995) best = cost, r.splits = s;
  }
  const int64_t per = ((int64_t)K + r.splits - 1) / r.splits;
  r.klen = (int)((per + bk - 1) / bk * bk);
  r.splits = (int)(((int64_t)K + r.klen - 1) / r.klen);
  return r;
}

// Weight-gradient launch plan with a split TAIL: when the output tiles take more than one round of
// workgroups (one per CU) and the last round is mostly empty, the tiles of the full rounds run
// unsplit (direct read-add-write of the gradient, no slab) and only the last round's tiles are
// split along K, so that round is as full as the CUs allow and takes 1/tail_splits of a tile's
// time. GPT-2 lm_head (591 tiles): 2 + 1/3 rounds instead of 3 (or 5 half-rounds plus two
// full-size slabs). Falls back to the uniform plan above whenever that prices lower.
struct WgradPlan {
  int main_tiles;   // tiles [0, main_tiles): main_splits each
  int main_splits;  // 1 = direct into the gradient, > 1 = full-size fp32 slabs
  int main_klen;
  int tail_splits;  // tiles [main_tiles, ntiles): tail_splits each into per-tile slabs (0: none)
  int tail_klen;
};

inline WgradPlan plan_wgrad(int M, int N, int K, int tile, int n_cu, int bk) {
  const SplitK u = plan_wgrad_splits(M, N, K, tile, n_cu, bk);
  WgradPlan r{0, u.splits, u.klen, 0, 0};
  if (M <= 0 || N <= 0 || K <= 0 || tile != 256 || bk <= 0) {
    r.main_tiles = (M > 0 && N > 0 && tile > 0) ? (int)(((int64_t)(M + tile - 1) / tile) * ((N + tile - 1) / tile)) : 0;
    return r;
  }
  const int64_t ntiles = (int64_t)((M + tile - 1) / tile) * ((N + tile - 1) / tile);
  r.main_tiles = (int)ntiles;
  const int64_t slots = std::max(1, n_cu);
  if (ntiles <= slots) return r;
  const double wg_full_k = (double)tile * tile * 2.0 * K / 2.3e12;
  auto uniform_cost = [&](int s) {
    const double waves = (double)((ntiles * s + slots - 1) / slots);
    return waves * wg_full_k / s + (s > 1 ? (double)s * M * N * 8.0 / 4.0e12 : 0.0);
  };
  const int64_t rounds = (ntiles + slots - 1) / slots;
  const int64_t tail = ntiles - (rounds - 1) * slots;
  const int st = (int)std::min<int64_t>({64, slots / tail, std::max(1, K / 512)});
  if (st < 2) return r;
  const double tail_cost = (double)(rounds - 1) * wg_full_k + wg_full_k / st +
                           (double)tail * st * tile * tile * 8.0 / 4.0e12;
  if (tail_cost >= uniform_cost(u.splits) * 0.995) return r;
  r.main_tiles = (int)(ntiles - tail);
  r.main_splits = 1;
  r.main_klen = (int)(((int64_t)K + bk - 1) / bk * bk);
  const int64_t per = ((int64_t)K + st - 1) / st;
  r.tail_klen = (int)((per + bk - 1) / bk * bk);
  r.tail_splits = (int)(((int64_t)K + r.tail_klen - 1) / r.tail_klen);
  return r;
}

// Slices of the two-stage deterministic column reduction (reduce.h): ~sqrt(G) balances stages.
inline int reduce_slices(int G) {
  int s = 1;
  while ((int64_t)s * s < G) ++s;
  return s;
}

}  // namespace penroz
