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

// Slices of the two-stage deterministic column reduction (reduce.h): ~sqrt(G) balances stages.
inline int reduce_slices(int G) {
  int s = 1;
  while ((int64_t)s * s < G) ++s;
  return s;
}

}  // namespace penroz
