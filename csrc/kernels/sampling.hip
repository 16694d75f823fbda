// Next-token selection, one 1024-thread workgroup per row of logits [B, V]:
//   temperature == 0  -> argmax (first index on ties, like torch.argmax);
//   top_k > 0         -> radix-select the k-th largest (4 × 8-bit passes, LDS histograms) and
//                        keep logits >= it;
//   then softmax of (logit / T) over the kept set and an inverse-CDF draw with the row's
//   uniform u: thread-major order (thread t owns elements t, t+1024, …), one block scan of
//   the per-thread sums finds the owning thread, which walks its own elements.
// The whole decision stays on the device (no sort, no host round trip per token).
// sample_reg_kernel (default for V % 8 == 0, V <= 64 Ki) keeps the row in registers; wider rows
// and batches of >= 16 rows (greedy / top-k <= 64, V <= 256 Ki) go through the two-stage
// sample_part_kernel + sample_merge_kernel.
#include "common.h"
#include <cstdlib>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

namespace penroz {

constexpr int kST = 1024;

// Where a row's uniform comes from and where its token goes. Default: uni[row] in, out[row] out.
// The graph-replayed decode step (sample_step) instead hashes the uniform from (*seed, *step, row)
// on the device and also writes the token into out2[row, *step] — the sampler then is the whole
// token feedback (no RNG kernel, no copy / index kernels).
struct SampleIO {
  const float* uni;
  const int64_t* seed;
  const int64_t* step;
  int64_t* out;
  int64_t* out2;
  int64_t out2_stride;
  // graph decode (sample_step with advance): the writer of the LAST row to finish also advances
  // the step counters (+1 on *adv_a, *adv_b, *step) — every row has read *step by then — and
  // re-arms the arrival counter: one launch less per decoded token
  int64_t* adv_a = nullptr;
  int64_t* adv_b = nullptr;
  unsigned* done = nullptr;
  int nrows = 0;
  __device__ __forceinline__ float uniform(int row) const {
    if (uni) return uni[row];
    uint64_t z = (uint64_t)*seed + 0x9E3779B97F4A7C15ull * (uint64_t)(*step + 1) + 0xD1B54A32D192ED03ull * (uint64_t)(row + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;  // splitmix64 finaliser
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (float)(z >> 40) * (1.f / 16777216.f);  // 24 bits: [0, 1)
  }
  __device__ __forceinline__ void write(int row, int64_t tok) const {
    out[row] = tok;
    if (out2) out2[(size_t)row * out2_stride + *step] = tok;
    if (done) {
      __threadfence();  // this row's reads of *step and its stores come before its arrival
      if (atomicAdd(done, 1u) == (unsigned)nrows - 1u) {
        ++*adv_a;
        ++*adv_b;
        ++*const_cast<int64_t*>(step);
        *done = 0u;
        __threadfence();
      }
    }
  }
};

__device__ __forceinline__ uint32_t order_key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Radix-select digit pick over a 256-bin histogram, in parallel (a serial scan of the bins by
// one thread costs ~10 µs per pass in LDS latency): threads t < 256 scan the bins from the top
// (d = 255 - t) and the one bin d with S(d+1) < kk <= S(d), S(d) = Σ_{b≥d} bins[b], records the
// digit (d = 0 when fewer than kk keys remain). Every thread of the block must call it; the
// caller synchronises before (bins complete) and after (selection visible).
__device__ __forceinline__ void pick_digit(const uint32_t* bins, uint32_t* wtot, int shift, uint32_t pre,
                                           uint32_t msk, int kk, uint32_t* sel_prefix, uint32_t* sel_mask,
                                           int* sel_k) {
  const int t = threadIdx.x, lane = t & 63;
  uint32_t c = 0, incl = 0;
  if (t < 256) {
    c = bins[255 - t];
    incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t n = __shfl_up(incl, o, 64);
      if (lane >= o) incl += n;
    }
    if (lane == 63) wtot[t >> 6] = incl;
  }
  __syncthreads();
  if (t < 256) {
    for (int i = 0; i < (t >> 6); ++i) incl += wtot[i];
    const int d = 255 - t;
    const uint32_t above = incl - c;
    if ((int)above < kk && ((int)incl >= kk || d == 0)) {
      *sel_k = kk - (int)above;
      *sel_prefix = pre | ((uint32_t)d << shift);
      *sel_mask = msk | (255u << shift);
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(kST) sample_kernel(const T* __restrict__ logits, const SampleIO io, int V,
                                                     float temperature, int top_k) {
  __shared__ float fred[kST / 64];
  __shared__ int ired[kST / 64];
  __shared__ uint32_t hist[256];
  __shared__ uint32_t wtot[4];
  __shared__ float scan[kST];
  __shared__ uint32_t sel_prefix, sel_mask;
  __shared__ int sel_k;
  __shared__ int64_t result;
  const int row = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const T* lp = logits + (size_t)row * V;

  // ---- argmax (also the fallback draw)
  float bm = -INFINITY;
  int bi = 0x7fffffff;
  for (int i = t; i < V; i += kST) {
    const float v = to_f(lp[i]);
    if (v > bm || (v == bm && i < bi)) { bm = v; bi = i; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(bm, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (om > bm || (om == bm && oi < bi)) { bm = om; bi = oi; }
  }
  if (lane == 0) { fred[w] = bm; ired[w] = bi; }
  __syncthreads();
  if (t == 0) {
    float m = fred[0];
    int ix = ired[0];
    for (int i = 1; i < kST / 64; ++i)
      if (fred[i] > m || (fred[i] == m && ired[i] < ix)) { m = fred[i]; ix = ired[i]; }
    result = ix;
    fred[0] = m;
  }
  __syncthreads();
  const float gmax = fred[0];
  if (temperature == 0.f) {
    if (t == 0) io.write(row, result);
    return;
  }

  // ---- top-k threshold by radix select over order-preserving keys
  uint32_t thr = 0;
  if (top_k > 0 && top_k < V) {
    if (t == 0) { sel_prefix = 0; sel_mask = 0; sel_k = top_k; }
    for (int shift = 24; shift >= 0; shift -= 8) {
      for (int b = t; b < 256; b += kST) hist[b] = 0;
      __syncthreads();
      const uint32_t pre = sel_prefix, msk = sel_mask;
      const int kk = sel_k;
      for (int i = t; i < V; i += kST) {
        const uint32_t k = order_key(to_f(lp[i]));
        if ((k & msk) == pre) atomicAdd(&hist[(k >> shift) & 255u], 1u);
      }
      __syncthreads();
      pick_digit(hist, wtot, shift, pre, msk, kk, &sel_prefix, &sel_mask, &sel_k);
      __syncthreads();
    }
    thr = sel_prefix;
  }

  // ---- softmax weights (unnormalised) and per-thread sums
  const float invT = 1.f / temperature;
  const float m = gmax * invT;
  float s = 0.f;
  for (int i = t; i < V; i += kST) {
    const float v = to_f(lp[i]);
    if (thr == 0 || order_key(v) >= thr) s += __expf(v * invT - m);
  }
  scan[t] = s;
  __syncthreads();
  // inclusive Hillis-Steele scan over 1024 partial sums
  for (int o = 1; o < kST; o <<= 1) {
    const float add = t >= o ? scan[t - o] : 0.f;
    __syncthreads();
    scan[t] += add;
    __syncthreads();
  }
  const float total = scan[kST - 1];
  const float target = io.uniform(row) * total;
  const float before = t > 0 ? scan[t - 1] : 0.f;
  if (s > 0.f && target >= before && target < before + s) {
    float acc = before;
    int pick = -1;
    for (int i = t; i < V; i += kST) {
      const float v = to_f(lp[i]);
      if (thr != 0 && order_key(v) < thr) continue;
      acc += __expf(v * invT - m);
      pick = i;
      if (acc > target) break;
    }
    if (pick >= 0) result = pick;
  }
  __syncthreads();
  if (t == 0) io.write(row, result);
}

// Register-resident variant (V % 8 == 0, V <= 8·1024·CPT): the row is read from memory ONCE
// (8 elements per 16-B chunk, chunk k of thread t covers elements 8·(t + 512·k)), then argmax,
// the four radix passes, the softmax sums and the draw all run on registers. The radix
// histograms are lane-private ([bin][32] copies, lanes l and l+32 share one): the first pass
// puts almost every logit into one or two bins (sign + exponent bits), and a single shared
// histogram then serialises tens of thousands of LDS atomics on one address.
constexpr int kRT = 512;  // 256 VGPRs per thread: room for a 104-logit slice

template <int CPT, typename T>
__global__ void __launch_bounds__(kRT) sample_reg_kernel(const T* __restrict__ logits, const SampleIO io, int V,
                                                         float temperature, int top_k) {
  __shared__ uint32_t hist[256 * 32];
  __shared__ uint32_t bins[256];
  __shared__ uint32_t wtot[4];
  __shared__ float fred[kRT / 64];
  __shared__ int ired[kRT / 64];
  __shared__ float wsum[kRT / 64];
  __shared__ uint32_t sel_prefix, sel_mask;
  __shared__ int sel_k;
  __shared__ float total_s;
  __shared__ int64_t result;
  const int row = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const T* lp = logits + (size_t)row * V;
  // the 16-B chunks stay packed (bf16: 4 VGPRs per 8 logits) and are widened on use, so a
  // 104-logit slice per thread (GPT-2's padded 50304 vocab) fits next to the histogram / scan state without spilling
  constexpr int H = (int)sizeof(T) / 2;
  uint4 raw[CPT][H];
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    const int c = 8 * (t + kRT * k);
#pragma unroll
    for (int h = 0; h < H; ++h)
      raw[k][h] = c < V ? *reinterpret_cast<const uint4*>(lp + c + 4 * h)
                        : make_uint4(0xff80ff80u, 0xff80ff80u, 0xff80ff80u, 0xff80ff80u);  // masked by i < V
  }
  auto val = [&](int k, int j) -> float {
    if constexpr (H == 1) {
      const uint4 r = raw[k][0];
      const int q = j >> 1;
      const uint32_t x = q == 0 ? r.x : q == 1 ? r.y : q == 2 ? r.z : r.w;
      return __uint_as_float((j & 1) ? (x & 0xffff0000u) : (x << 16));
    } else {
      const uint4 r = raw[k][j >> 2];
      const int q = j & 3;
      const uint32_t x = q == 0 ? r.x : q == 1 ? r.y : q == 2 ? r.z : r.w;
      return __uint_as_float(x);
    }
  };
  // each pass re-widens from the packed registers: without this barrier the compiler hoists the
  // widened values / order keys out of the radix loop and keeps them all live (spills)
  auto opaque = [&]() {
#pragma unroll
    for (int k = 0; k < CPT; ++k)
#pragma unroll
      for (int h = 0; h < H; ++h) asm volatile("" : "+v"(raw[k][h].x), "+v"(raw[k][h].y), "+v"(raw[k][h].z), "+v"(raw[k][h].w));
  };
  // ---- argmax (first index on ties, like torch.argmax)
  float bm = -INFINITY;
  int bi = 0x7fffffff;
#pragma unroll
  for (int k = 0; k < CPT; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = 8 * (t + kRT * k) + j;
      const float x = val(k, j);
      if (i < V && x > bm) { bm = x; bi = i; }
    }
  const uint32_t tkey = order_key(bm);  // this thread's max (order key of -inf when empty)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(bm, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (om > bm || (om == bm && oi < bi)) { bm = om; bi = oi; }
  }
  if (lane == 0) { fred[w] = bm; ired[w] = bi; }
  __syncthreads();
  if (t == 0) {
    float m = fred[0];
    int ix = ired[0];
    for (int i = 1; i < kRT / 64; ++i)
      if (fred[i] > m || (fred[i] == m && ired[i] < ix)) { m = fred[i]; ix = ired[i]; }
    result = ix;
    fred[0] = m;
  }
  __syncthreads();
  const float gmax = fred[0];
  if (temperature == 0.f) {
    if (t == 0) io.write(row, result);
    return;
  }
  // ---- top-k, k <= 512: rank by counting. (1) The k-th largest of the 512 per-thread maxima,
  // L, bounds the row's k-th largest from below (k maxima, so k elements, are >= L); each
  // thread ranks its maximum against the other 511 (LDS broadcast reads). (2) The elements >= L —
  // typically not many more than k — are compacted into LDS in index order, ranked the same way
  // (value descending, index ascending), and the k best are laid out in rank order. (3) Softmax
  // and the inverse-CDF draw run over those k in rank order (the reference's sorted top-k order).
  // More than 512 candidates (heavy ties): the radix select below.
  if (top_k > 0 && top_k < V && top_k <= kRT) {
    uint32_t* ck = hist;                                       // [512] candidate keys (first: maxima)
    int* ci = reinterpret_cast<int*>(hist + kRT);              // [512] candidate indices
    float* pr = reinterpret_cast<float*>(hist + 2 * kRT);      // [512] weights in rank order
    int* pix = reinterpret_cast<int*>(hist + 3 * kRT);         // [512] indices in rank order
    ck[t] = tkey;
    __syncthreads();
    int rk = 0;  // 16-B broadcast reads, 8 in flight (a serial 4-B loop waits out the LDS latency)
    const uint4* ck4 = reinterpret_cast<const uint4*>(ck);
#pragma unroll 8
    for (int j4 = 0; j4 < kRT / 4; ++j4) {
      const uint4 o = ck4[j4];
      const int j = 4 * j4;
      rk += (o.x > tkey) || (o.x == tkey && j < t);
      rk += (o.y > tkey) || (o.y == tkey && j + 1 < t);
      rk += (o.z > tkey) || (o.z == tkey && j + 2 < t);
      rk += (o.w > tkey) || (o.w == tkey && j + 3 < t);
    }
    if (rk == top_k - 1) sel_prefix = tkey;
    __syncthreads();
    const uint32_t lo = sel_prefix;
    opaque();
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < CPT; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) cnt += (8 * (t + kRT * k) + j < V && order_key(val(k, j)) >= lo) ? 1 : 0;
    int incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int n = __shfl_up(incl, o, 64);
      if (lane >= o) incl += n;
    }
    if (lane == 63) ired[w] = incl;
    __syncthreads();
    if (t == 0) {
      int run = 0;
      for (int i = 0; i < kRT / 64; ++i) {
        const int x = ired[i];
        ired[i] = run;
        run += x;
      }
      sel_k = run;
    }
    __syncthreads();
    const int ncand = sel_k;
    if (ncand <= kRT) {
      int off = ired[w] + incl - cnt;
      opaque();
#pragma unroll
      for (int k = 0; k < CPT; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int i = 8 * (t + kRT * k) + j;
          const uint32_t key = order_key(val(k, j));
          if (i < V && key >= lo) {
            ck[off] = key;
            ci[off] = i;
            ++off;
          }
        }
      const int npad = (ncand + 31) & ~31;  // key 0 ranks below every real key
      if (t >= ncand && t < npad) ck[t] = 0;
      __syncthreads();
      const float invT = 1.f / temperature;
      const float m = gmax * invT;
      if (t < ncand) {
        const uint32_t mk = ck[t];
        const int mi = ci[t];
        int r = 0;
        for (int j4 = 0; j4 < npad / 4; j4 += 8) {
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const uint4 o = ck4[j4 + u];
            const int j = 4 * (j4 + u);
            r += (o.x > mk) || (o.x == mk && ci[j] < mi);
            r += (o.y > mk) || (o.y == mk && ci[j + 1] < mi);
            r += (o.z > mk) || (o.z == mk && ci[j + 2] < mi);
            r += (o.w > mk) || (o.w == mk && ci[j + 3] < mi);
          }
        }
        if (r < top_k) {
          const uint32_t bits = (mk & 0x80000000u) ? (mk & 0x7fffffffu) : ~mk;  // order_key⁻¹
          pr[r] = __expf(__uint_as_float(bits) * invT - m);
          pix[r] = mi;
        }
      }
      __syncthreads();
      const float pv = t < top_k ? pr[t] : 0.f;
      float inc = pv;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const float n = __shfl_up(inc, o, 64);
        if (lane >= o) inc += n;
      }
      if (lane == 63) wsum[w] = inc;
      __syncthreads();
      if (t == 0) {
        float run = 0.f;
        for (int i = 0; i < kRT / 64; ++i) {
          const float x = wsum[i];
          wsum[i] = run;
          run += x;
        }
        total_s = run;
      }
      __syncthreads();
      const float cum = wsum[w] + inc;
      const float target = io.uniform(row) * total_s;
      if (t < top_k && pv > 0.f && cum > target && cum - pv <= target) result = pix[t];
      __syncthreads();
      if (t == 0) io.write(row, result);
      return;
    }
  }
  // ---- top-k threshold: radix select over order-preserving keys (4 × 8-bit digits). Counting
  // every logit costs 4·V LDS atomics, and those that hit one bin serialise (~80 µs per 50 K
  // row), so the select runs twice over small sets instead: (1) over the 512 per-thread maxima,
  // whose k-th largest L is a lower bound of the row's k-th largest (k maxima, k elements ≥ L),
  // then (2) over the elements ≥ L only — typically barely more than k of them.
  auto radix_select = [&](auto&& visit, int kk0) -> uint32_t {
    if (t == 0) { sel_prefix = 0; sel_mask = 0; sel_k = kk0; }
    for (int shift = 24; shift >= 0; shift -= 8) {
      for (int i = t; i < 256 * 32; i += kRT) hist[i] = 0;
      __syncthreads();
      const uint32_t pre = sel_prefix, msk = sel_mask;
      const int kk = sel_k;
      opaque();
      visit([&](uint32_t key) {
        if ((key & msk) == pre) atomicAdd(&hist[((key >> shift) & 255u) * 32 + (lane & 31)], 1u);
      });
      __syncthreads();
      if (t < 256) {  // rotated reads: the 32 copies of bin t sit on 32 banks
        uint32_t c = 0;
        for (int i = 0; i < 32; ++i) c += hist[t * 32 + ((i + t) & 31)];
        bins[t] = c;
      }
      __syncthreads();
      pick_digit(bins, wtot, shift, pre, msk, kk, &sel_prefix, &sel_mask, &sel_k);
      __syncthreads();
    }
    return sel_prefix;
  };
  uint32_t thr = 0;
  if (top_k > 0 && top_k < V) {
    uint32_t lo = 0;
    if (top_k <= kRT) lo = radix_select([&](auto&& add) { add(tkey); }, top_k);
    thr = radix_select([&](auto&& add) {
#pragma unroll
      for (int k = 0; k < CPT; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t key = order_key(val(k, j));
          if (8 * (t + kRT * k) + j < V && key >= lo) add(key);
        }
    }, top_k);
  }
  // ---- unnormalised softmax weights of the kept set; block scan of per-thread sums
  const float invT = 1.f / temperature;
  const float m = gmax * invT;
  float s = 0.f;
  opaque();
#pragma unroll
  for (int k = 0; k < CPT; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float x = val(k, j);
      if (8 * (t + kRT * k) + j < V && (thr == 0 || order_key(x) >= thr)) s += __expf(x * invT - m);
    }
  float incl = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float n = __shfl_up(incl, o, 64);
    if (lane >= o) incl += n;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  if (t == 0) {
    float run = 0.f;
    for (int i = 0; i < kRT / 64; ++i) {
      const float x = wsum[i];
      wsum[i] = run;
      run += x;
    }
    total_s = run;
  }
  __syncthreads();
  const float before = wsum[w] + incl - s;
  const float target = io.uniform(row) * total_s;
  if (s > 0.f && target >= before && target < before + s) {
    float acc = before;
    int pick = -1;
    bool done = false;
    opaque();
#pragma unroll
    for (int k = 0; k < CPT; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = 8 * (t + kRT * k) + j;
        const float x = val(k, j);
        if (done || i >= V || (thr != 0 && order_key(x) < thr)) continue;
        acc += __expf(x * invT - m);
        pick = i;
        if (acc > target) done = true;
      }
    if (pick >= 0) result = pick;
  }
  __syncthreads();
  if (t == 0) io.write(row, result);
}


// ------------------------------------------------------------------------------------------
// Two-stage form for wide rows (V > 64 Ki: Gemma's 262 144-token vocabulary), greedy or
// top-k <= kPartK = 64. One 1024-thread workgroup per row reads the row seven times; here the row is
// split into <= 64 parts of 4096 logits (V <= 256 Ki), one 256-thread workgroup each (16 logits per thread in
// registers, read once):
//   stage 1 (grid parts x rows): the part's argmax, and its top-k by a 4-pass radix select on
//     the registers; every logit > the part's k-th largest, then the ties at it, go to a
//     candidate list (<= kPartC per part: only ties at the threshold can be dropped).
//     Every element >= the row's k-th largest is >= its part's k-th largest, so the candidates
//     hold the row's whole top-k (ties included) and its k-th largest key is the row's.
//   stage 2 (one workgroup per row): argmax merge; radix select over the candidates; the kept
//     ones are ranked by token index (the draw order of the one-stage kernels), softmax(v/T),
//     inverse-CDF draw with the row's uniform.
constexpr int kMergeBatch = 8;  // sample_merge_kernel: candidate slots per thread loaded together
constexpr int kPartN = 4096, kPartK = 64, kPartC = 128, kPartKeep = 1024, kPartMaxP = 64,
              kPartLds = kPartMaxP * kPartC;  // every part's candidates fit: none dropped in the merge

__device__ __forceinline__ float key_value(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

template <typename T>
__global__ void __launch_bounds__(256) sample_part_kernel(const T* __restrict__ logits, int V, int P, int top_k,
                                                          float* __restrict__ pval, int* __restrict__ pidx,
                                                          uint32_t* __restrict__ ckey, int* __restrict__ cidx,
                                                          int* __restrict__ cnt) {
  __shared__ uint32_t hist[256];
  __shared__ uint32_t wtot[4];
  __shared__ float fred[4];
  __shared__ int ired[4];
  __shared__ uint32_t sel_prefix, sel_mask;
  __shared__ int sel_k, ncand;
  const int part = blockIdx.x, row = blockIdx.y, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const T* lp = logits + (size_t)row * V;
  const int base = part * kPartN;
  float v[2][8];
  bool ok[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int e0 = base + 8 * (t + 256 * c);
    ok[c] = e0 < V;  // V % 8 == 0: a chunk is all in or all out
    Vec8<T>::load(lp + (ok[c] ? e0 : 0), v[c]);
  }
  float bm = -INFINITY;
  int bi = 0x7fffffff;
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int i = base + 8 * (t + 256 * c) + e;
      if (ok[c] && (v[c][e] > bm || (v[c][e] == bm && i < bi))) { bm = v[c][e]; bi = i; }
    }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(bm, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (om > bm || (om == bm && oi < bi)) { bm = om; bi = oi; }
  }
  if (lane == 0) { fred[w] = bm; ired[w] = bi; }
  __syncthreads();
  if (t == 0) {
    float m = fred[0];
    int ix = ired[0];
    for (int i = 1; i < 4; ++i)
      if (fred[i] > m || (fred[i] == m && ired[i] < ix)) { m = fred[i]; ix = ired[i]; }
    pval[(size_t)row * P + part] = m;
    pidx[(size_t)row * P + part] = ix;
  }
  if (top_k <= 0) return;
  uint32_t key[2][8];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int e = 0; e < 8; ++e) key[c][e] = ok[c] ? order_key(v[c][e]) : 0u;
  if (t == 0) { sel_prefix = 0; sel_mask = 0; sel_k = top_k; ncand = 0; }
  for (int shift = 24; shift >= 0; shift -= 8) {
    hist[t] = 0;
    __syncthreads();
    const uint32_t pre = sel_prefix, msk = sel_mask;
    const int kk = sel_k;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (ok[c] && (key[c][e] & msk) == pre) atomicAdd(&hist[(key[c][e] >> shift) & 255u], 1u);
    __syncthreads();
    pick_digit(hist, wtot, shift, pre, msk, kk, &sel_prefix, &sel_mask, &sel_k);
    __syncthreads();
  }
  const uint32_t thr = sel_prefix;
  const size_t cb = ((size_t)row * P + part) * kPartC;
  // the < k logits above the threshold first (always kept), then the ties at it
  for (int tie = 0; tie < 2; ++tie) {
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (ok[c] && (tie ? key[c][e] == thr : key[c][e] > thr)) {
          const int slot = atomicAdd(&ncand, 1);
          if (slot < kPartC) {
            ckey[cb + slot] = key[c][e];
            cidx[cb + slot] = base + 8 * (t + 256 * c) + e;
          }
        }
    __syncthreads();
  }
  if (t == 0) cnt[(size_t)row * P + part] = min(ncand, kPartC);
}

__global__ void __launch_bounds__(256) sample_merge_kernel(const SampleIO io, int P, float temperature, int top_k,
                                                           const float* __restrict__ pval, const int* __restrict__ pidx,
                                                           const uint32_t* __restrict__ ckey,
                                                           const int* __restrict__ cidx, const int* __restrict__ cnt) {
  __shared__ uint32_t hist[256];
  __shared__ uint32_t wtot[4];
  __shared__ float fred[4];
  __shared__ int ired[4];
  __shared__ uint32_t sel_prefix, sel_mask;
  __shared__ int sel_k, nkeep;
  __shared__ float kval[kPartKeep];
  __shared__ int kidx[kPartKeep];
  __shared__ float sval[kPartKeep];
  __shared__ int sidx[kPartKeep];
  extern __shared__ __attribute__((aligned(16))) uint32_t dyn_lds[];  // kPartLds keys + indices (64 KB)
  uint32_t* lkey = dyn_lds;
  int* lidx = reinterpret_cast<int*>(dyn_lds + kPartLds);
  __shared__ int coff[256], ccnt[256];
  __shared__ int ctot;
  const int row = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
  // this thread's part candidate count, fetched with the argmax operands (one memory round trip)
  const int c_own = (cnt != nullptr && t < P) ? cnt[(size_t)row * P + t] : 0;
  float bm = -INFINITY;
  int bi = 0x7fffffff;
  for (int p = t; p < P; p += 256) {
    const float pv = pval[(size_t)row * P + p];
    const int pi = pidx[(size_t)row * P + p];
    if (pv > bm || (pv == bm && pi < bi)) { bm = pv; bi = pi; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(bm, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (om > bm || (om == bm && oi < bi)) { bm = om; bi = oi; }
  }
  if (lane == 0) { fred[w] = bm; ired[w] = bi; }
  __syncthreads();
  float gmax = fred[0];
  int gidx = ired[0];
  for (int i = 1; i < 4; ++i)
    if (fred[i] > gmax || (fred[i] == gmax && ired[i] < gidx)) { gmax = fred[i]; gidx = ired[i]; }
  if (temperature == 0.f || top_k <= 0) {
    if (t == 0) io.write(row, gidx);
    return;
  }
  __syncthreads();  // fred / ired are reused below
  // compact the valid candidates of all parts into LDS (part order), then work from there
  const int c = c_own;
  int incl = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) ired[w] = incl;
  __syncthreads();
  for (int i = 0; i < w; ++i) incl += ired[i];
  if (t < P) {
    coff[t] = incl - c;
    ccnt[t] = c;
  }
  if (t == 255) ctot = min(incl, kPartLds);
  __syncthreads();
  // all of a thread's candidate slots are read before any is kept (slots past a part's count
  // hold stale values and are dropped): one memory round trip per kMergeBatch slots
  const int NCg = P * kPartC;
  for (int f0 = t; f0 < NCg; f0 += 256 * kMergeBatch) {
    uint32_t kb[kMergeBatch];
    int ib[kMergeBatch];
#pragma unroll
    for (int u = 0; u < kMergeBatch; ++u) {
      const int f = f0 + 256 * u;
      if (f < NCg) {
        kb[u] = ckey[(size_t)row * NCg + f];
        ib[u] = cidx[(size_t)row * NCg + f];
      }
    }
#pragma unroll
    for (int u = 0; u < kMergeBatch; ++u) {
      const int f = f0 + 256 * u;
      if (f >= NCg) break;
      const int p = f / kPartC, j = f - p * kPartC;
      if (j < ccnt[p] && coff[p] + j < kPartLds) {
        lkey[coff[p] + j] = kb[u];
        lidx[coff[p] + j] = ib[u];
      }
    }
  }
  const int NC = ctot;
  const uint32_t* kr = lkey;
  const int* ir = lidx;
  if (t == 0) { sel_prefix = 0; sel_mask = 0; sel_k = top_k; nkeep = 0; }
  for (int shift = 24; shift >= 0; shift -= 8) {
    hist[t] = 0;
    __syncthreads();
    const uint32_t pre = sel_prefix, msk = sel_mask;
    const int kk = sel_k;
    for (int f = t; f < NC; f += 256) {
      const uint32_t k = kr[f];
      if ((k & msk) == pre) atomicAdd(&hist[(k >> shift) & 255u], 1u);
    }
    __syncthreads();
    pick_digit(hist, wtot, shift, pre, msk, kk, &sel_prefix, &sel_mask, &sel_k);
    __syncthreads();
  }
  const uint32_t thr = sel_prefix;
  for (int tie = 0; tie < 2; ++tie) {  // above the threshold first, then the ties at it
    for (int f = t; f < NC; f += 256) {
      if (tie ? kr[f] != thr : kr[f] <= thr) continue;
      const int slot = atomicAdd(&nkeep, 1);
      if (slot < kPartKeep) {
        kval[slot] = key_value(kr[f]);
        kidx[slot] = ir[f];
      }
    }
    __syncthreads();
  }
  const int n = min(nkeep, kPartKeep);
  const float invT = 1.f / temperature;
  float part_sum = 0.f;
  for (int e = t; e < n; e += 256) {  // rank by token index: the draw walks the kept set in index order
    const int ix = kidx[e];
    int r = 0;
    for (int j = 0; j < n; ++j) r += kidx[j] < ix;
    const float wgt = __expf((kval[e] - gmax) * invT);
    sval[r] = wgt;
    sidx[r] = ix;
    part_sum += wgt;
  }
  part_sum = wave_sum(part_sum);
  if (lane == 0) fred[w] = part_sum;
  __syncthreads();
  if (w != 0) return;
  const float total = (fred[0] + fred[1]) + (fred[2] + fred[3]);
  const float target = io.uniform(row) * total;
  float carry = 0.f;
  int pick = n > 0 ? sidx[n - 1] : gidx;
  for (int b0 = 0; b0 < n; b0 += 64) {
    const int e = b0 + lane;
    float incl = e < n ? sval[e] : 0.f;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    const uint64_t hit = __ballot(e < n && carry + incl > target);
    if (hit) {
      pick = sidx[b0 + __ffsll((unsigned long long)hit) - 1];
      break;
    }
    carry += __shfl(incl, 63, 64);
  }
  if (lane == 0) io.write(row, pick);
}
}  // namespace penroz

using namespace penroz;

static void launch_sample(const torch::Tensor& logits, const SampleIO& io, double temperature, int64_t top_k) {
  TORCH_CHECK(logits.is_cuda() && logits.is_contiguous() && logits.dim() == 2);
  const int B = logits.size(0), V = logits.size(1);
  auto stream = at::hip::getCurrentHIPStream();
  int chunks = (V / 8 + kRT - 1) / kRT;
  for (int c : {1, 2, 3, 4, 6, 8, 10, 13, 16})  // instantiated slice sizes
    if (chunks <= c) { chunks = c; break; }
  const bool fits = chunks <= (logits.scalar_type() == torch::kBFloat16 ? 16 : 8);
  const float tt = (float)temperature;
  const int kk = (int)top_k;
  // the two-stage form for rows too wide for registers, and for any number of rows from
  // kTwoStageMinRows on (P x B part workgroups spread a row over P CUs where one workgroup per row
  // leaves most of the chip idle: a batch-64 decode step, and a batch-1 step whose single-workgroup
  // register sampler took ~38 µs of a ~600 µs GPT-2 token). PENROZ_SAMPLE_TWO_STAGE_MIN_ROWS
  // moves the switch (A/B; the register kernel serves the rows below it)
  static const int kTwoStageMinRows = [] {
    const char* e = std::getenv("PENROZ_SAMPLE_TWO_STAGE_MIN_ROWS");
    return e ? std::atoi(e) : 1;
  }();
  if (V % 8 == 0 && (!fits || B >= kTwoStageMinRows) && logits.scalar_type() != torch::kFloat16 &&
      V <= kPartMaxP * kPartN && (temperature == 0.0 || (top_k > 0 && top_k <= kPartK))) {
    const int P = (V + kPartN - 1) / kPartN;
    const bool topk = temperature != 0.0;
    auto opt = logits.options();
    auto pval = torch::empty({B, P}, opt.dtype(torch::kFloat32));
    auto pidx = torch::empty({B, P}, opt.dtype(torch::kInt32));
    torch::Tensor ckey, cidx, cnt;
    if (topk) {
      ckey = torch::empty({B, P, kPartC}, opt.dtype(torch::kInt32));
      cidx = torch::empty({B, P, kPartC}, opt.dtype(torch::kInt32));
      cnt = torch::empty({B, P}, opt.dtype(torch::kInt32));
    }
    uint32_t* ckp = topk ? reinterpret_cast<uint32_t*>(ckey.data_ptr()) : nullptr;
    int* cip = topk ? cidx.data_ptr<int>() : nullptr;
    int* cnp = topk ? cnt.data_ptr<int>() : nullptr;
    const int kpart = topk ? kk : 0;
    if (logits.scalar_type() == torch::kBFloat16)
      hipLaunchKernelGGL(sample_part_kernel<bf16>, dim3(P, B), dim3(256), 0, stream,
                         reinterpret_cast<const bf16*>(logits.data_ptr()), V, P, kpart, pval.data_ptr<float>(),
                         pidx.data_ptr<int>(), ckp, cip, cnp);
    else
      hipLaunchKernelGGL(sample_part_kernel<float>, dim3(P, B), dim3(256), 0, stream, logits.data_ptr<float>(), V, P,
                         kpart, pval.data_ptr<float>(), pidx.data_ptr<int>(), ckp, cip, cnp);
    static bool lds_set = [] {  // > 64 KB of LDS per workgroup must be requested
      return hipFuncSetAttribute(reinterpret_cast<const void*>(sample_merge_kernel),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, kPartLds * 8) == hipSuccess;
    }();
    TORCH_CHECK(lds_set, "sample_merge_kernel: LDS request refused");
    hipLaunchKernelGGL(sample_merge_kernel, dim3(B), dim3(256), kPartLds * 8, stream, io, P, tt, kpart, pval.data_ptr<float>(),
                       pidx.data_ptr<int>(), ckp, cip, cnp);
    return;
  }
  if (V % 8 == 0 && fits && logits.scalar_type() != torch::kFloat16) {
    auto launch = [&](auto tag) {
      using T = decltype(tag);
      const T* lp = reinterpret_cast<const T*>(logits.data_ptr());
#define PENROZ_SAMPLE_REG(C) \
  case C: hipLaunchKernelGGL((sample_reg_kernel<C, T>), dim3(B), dim3(kRT), 0, stream, lp, io, V, tt, kk); break;
      switch (chunks) {
        PENROZ_SAMPLE_REG(1) PENROZ_SAMPLE_REG(2) PENROZ_SAMPLE_REG(3) PENROZ_SAMPLE_REG(4) PENROZ_SAMPLE_REG(6)
        PENROZ_SAMPLE_REG(8)
        default:
          if constexpr (sizeof(T) == 2) {
            switch (chunks) { PENROZ_SAMPLE_REG(10) PENROZ_SAMPLE_REG(13) PENROZ_SAMPLE_REG(16) }
          }
      }
#undef PENROZ_SAMPLE_REG
    };
    if (logits.scalar_type() == torch::kBFloat16) launch(bf16{});
    else launch(float{});
    return;
  }
  if (logits.scalar_type() == torch::kBFloat16)
    hipLaunchKernelGGL(sample_kernel<bf16>, dim3(B), dim3(kST), 0, stream,
                       reinterpret_cast<const bf16*>(logits.data_ptr()), io, V, tt, kk);
  else if (logits.scalar_type() == torch::kFloat32)
    hipLaunchKernelGGL(sample_kernel<float>, dim3(B), dim3(kST), 0, stream, logits.data_ptr<float>(), io, V, tt, kk);
  else if (logits.scalar_type() == torch::kFloat16)
    hipLaunchKernelGGL(sample_kernel<__half>, dim3(B), dim3(kST), 0, stream,
                       reinterpret_cast<const __half*>(logits.data_ptr()), io, V, tt, kk);
  else TORCH_CHECK(false, "unsupported logits dtype");
}

torch::Tensor sample_tokens(torch::Tensor logits, c10::optional<torch::Tensor> uniform, double temperature,
                            int64_t top_k) {
  TORCH_CHECK(logits.is_cuda() && logits.is_contiguous() && logits.dim() == 2);
  const int B = logits.size(0);
  auto out = torch::empty({B, 1}, logits.options().dtype(torch::kInt64));
  torch::Tensor u;
  if (uniform.has_value() && uniform->defined()) u = uniform->to(torch::kFloat32).contiguous();
  else u = torch::zeros({B}, logits.options().dtype(torch::kFloat32));
  TORCH_CHECK(u.numel() == B && u.is_cuda());
  launch_sample(logits, SampleIO{u.data_ptr<float>(), nullptr, nullptr, out.data_ptr<int64_t>(), nullptr, 0}, temperature,
                top_k);
  return out;
}

// Graph-replayed decode: token of row r -> idx_out[r] and out_buf[r, *step]; uniforms hashed
// from (seed, *step, r) on the device. Then one tiny kernel advances the step counters.
void sample_step(torch::Tensor logits, double temperature, int64_t top_k, torch::Tensor seed, torch::Tensor step,
                 torch::Tensor idx_out, torch::Tensor out_buf, c10::optional<torch::Tensor> adv_a,
                 c10::optional<torch::Tensor> adv_b, c10::optional<torch::Tensor> done) {
  TORCH_CHECK(logits.dim() == 2 && step.is_cuda() && step.scalar_type() == torch::kInt64 && step.numel() == 1);
  TORCH_CHECK(seed.is_cuda() && seed.scalar_type() == torch::kInt64 && seed.numel() == 1, "seed: device int64 [1]");
  const int B = logits.size(0);
  TORCH_CHECK(idx_out.scalar_type() == torch::kInt64 && idx_out.numel() == B && idx_out.is_contiguous());
  TORCH_CHECK(out_buf.scalar_type() == torch::kInt64 && out_buf.dim() == 2 && out_buf.size(0) == B &&
              out_buf.stride(1) == 1, "out_buf [B, n] int64");
  SampleIO io{nullptr, seed.data_ptr<int64_t>(), step.data_ptr<int64_t>(), idx_out.data_ptr<int64_t>(),
               out_buf.data_ptr<int64_t>(), out_buf.stride(0)};
  if (done.has_value() && done->defined()) {  // fused counter advance (see SampleIO)
    TORCH_CHECK(adv_a.has_value() && adv_b.has_value(), "sample_step: advance needs both counters");
    for (const torch::Tensor* t : {&*adv_a, &*adv_b})
      TORCH_CHECK(t->is_cuda() && t->scalar_type() == torch::kInt64 && t->numel() == 1, "advance counters: int64 [1]");
    TORCH_CHECK(done->is_cuda() && done->scalar_type() == torch::kInt32 && done->numel() == 1, "done: int32 [1] (zero)");
    io.adv_a = adv_a->data_ptr<int64_t>();
    io.adv_b = adv_b->data_ptr<int64_t>();
    io.done = reinterpret_cast<unsigned*>(done->data_ptr<int>());
    io.nrows = B;
  }
  launch_sample(logits, io, temperature, top_k);
}

__global__ void decode_advance_kernel(int64_t* a, int64_t* b, int64_t* c) {
  if (threadIdx.x == 0) {
    ++*a;
    ++*b;
    ++*c;
  }
}

// +1 on three device int64 scalars (cache position, cache length, burst step) in one launch
void decode_advance(torch::Tensor a, torch::Tensor b, torch::Tensor c) {
  for (const auto* t : {&a, &b, &c})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == torch::kInt64 && t->numel() == 1, "decode_advance: int64 [1]");
  hipLaunchKernelGGL(decode_advance_kernel, dim3(1), dim3(64), 0, at::hip::getCurrentHIPStream(),
                     a.data_ptr<int64_t>(), b.data_ptr<int64_t>(), c.data_ptr<int64_t>());
}
