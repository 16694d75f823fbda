// Host-side unit test of the launch planners in csrc/kernels/host_plan.h, built and run by
// tests/test_host_sanitizers.py with -fsanitize=address,undefined (any report aborts the run).
#include "host_plan.h"

#include <cstdio>
#include <cstdlib>

using penroz::plan_wgrad_splits;

static int fails = 0;
#define EXPECT(c)                                                   \
  do {                                                              \
    if (!(c)) {                                                     \
      std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);      \
      ++fails;                                                      \
    }                                                               \
  } while (0)

int main() {
  // GPT-2 124M / XL weight-gradient shapes (K = tokens per step) and edge cases
  const int shapes[][3] = {{2304, 768, 65536}, {768, 768, 65536}, {3072, 768, 65536}, {768, 3072, 65536},
                           {50304, 768, 65536}, {50257, 768, 65536}, {4800, 1600, 65536}, {6400, 1600, 16384},
                           {8, 8, 1}, {200, 136, 1000}, {1, 1, 511}, {65536, 65536, 2147483647 / 2}};
  for (auto& s : shapes) {
    for (int tile : {128, 256}) {
      for (int bk : {32, 64}) {
        const auto p = plan_wgrad_splits(s[0], s[1], s[2], tile, 256, bk);
        EXPECT(p.splits >= 1 && p.splits <= 64);
        EXPECT(p.klen > 0 && p.klen % bk == 0);
        EXPECT((long long)p.klen * p.splits >= s[2]);              // covers K
        EXPECT((long long)p.klen * (p.splits - 1) < s[2]);         // no empty split
      }
    }
  }
  // split-tail plans: every tile covered once, the tail's splits cover K without an empty one
  const int tshapes[][3] = {{50304, 768, 65536}, {50257, 768, 65536}, {13824, 1152, 8192}, {262144, 1152, 8192},
                            {1152, 6912, 8192}, {6400, 1600, 16384}, {8, 8, 1}, {1 << 20, 768, 4096}};
  for (auto& s : tshapes) {
    const auto p = penroz::plan_wgrad(s[0], s[1], s[2], 256, 256, 32);
    const long long nt = (long long)((s[0] + 255) / 256) * ((s[1] + 255) / 256);
    EXPECT(p.main_tiles >= 0 && p.main_tiles <= nt);
    EXPECT(p.main_splits >= 1 && p.main_klen > 0 && p.main_klen % 32 == 0);
    EXPECT((long long)p.main_klen * p.main_splits >= s[2]);
    if (p.tail_splits > 0) {
      EXPECT(p.main_splits == 1 && p.main_tiles < nt && p.tail_splits >= 2);
      EXPECT(p.tail_klen % 32 == 0 && (long long)p.tail_klen * p.tail_splits >= s[2]);
      EXPECT((long long)p.tail_klen * (p.tail_splits - 1) < s[2]);
      EXPECT((nt - p.main_tiles) * p.tail_splits <= 256);  // the tail fits one round
    } else {
      EXPECT(p.main_tiles == nt);
    }
  }
  {  // GPT-2 lm_head: 591 tiles -> 512 direct + 79 tiles split 3 ways
    const auto p = penroz::plan_wgrad(50304, 768, 65536, 256, 256, 32);
    EXPECT(p.main_tiles == 512 && p.tail_splits == 3);
  }
  // degenerate inputs never divide by zero or overflow
  for (int bad : {0, -1}) {
    const auto p = plan_wgrad_splits(bad, 768, 1024, 256, 256, 64);
    EXPECT(p.splits == 1);
    const auto q = plan_wgrad_splits(768, 768, bad, 256, 0, 64);
    EXPECT(q.splits == 1);
    const auto w = penroz::plan_wgrad(768, bad, 1024, 256, 0, 32);
    EXPECT(w.tail_splits == 0 && w.main_splits >= 1);
  }
  for (int g : {0, 1, 2, 1024, 1 << 20, 2147483647}) {
    const int s = penroz::reduce_slices(g);
    EXPECT(s >= 1 && (long long)s * s >= g && (long long)(s - 1) * (s - 1) < (g > 1 ? g : 2));
  }
  std::printf("host_plan_test: %s (%d failures)\n", fails ? "FAILED" : "ok", fails);
  return fails ? 1 : 0;
}
