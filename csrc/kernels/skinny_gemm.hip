// Decode-shaped GEMMs: out[M, N] = x[M, K] · W[N, K]ᵀ (+ bias) for M <= 64 rows (one token per
// sequence of a decode batch), bf16 operands, fp32 accumulate — nn.Linear's layout.
//
// At these shapes a GEMM is latency-bound, not FLOP- or bandwidth-bound: GPT-2's QKV projection
// at M = 64 reads 3.5 MB of weights (0.7 µs of HBM time) and does 0.2 GFLOP, yet a library tile
// (hipBLASLt MT32x64x64, 96 workgroups) takes ~10 µs. What matters is how many independent loads
// are in flight per CU and how many CUs take part. So:
//   * a workgroup owns a 16-column slice of the output for ALL M rows: one 16x16x32 MFMA
//     column block, MB = ceil(M/16) row blocks; ceil(N/16) workgroups (144 for N = 2304);
//   * its 4 waves split the K range four ways (reduced through LDS at the end), and narrow
//     outputs (N = 768: 48 slices) also split K across workgroups (split-K with an in-launch
//     slab reduction: agent-scope release, arrival counter, the last arriver sums the slabs —
//     the counter is reset by that last arriver, so a captured graph can replay the kernel);
//   * operands go straight from global memory to MFMA fragments (A = W rows, B = x rows, 16 B
//     per lane per k-step) — every k-step's loads of a wave are issued before its first MFMA;
//     an LDS round trip would only add latency for operands nobody else in the workgroup reads.
// C/D layout of mfma_f32_16x16x32_bf16: col = lane & 15 (row m of x), row = 4·(lane >> 4) + r
// (output column n), so each lane ends with 4 consecutive outputs of one row.
#include "common.h"
#include <vector>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

namespace penroz {

typedef short sk_bf16x8 __attribute__((ext_vector_type(8)));
typedef float sk_f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t sk_u32x4 __attribute__((ext_vector_type(4)));

constexpr int kSkU = 8;  // k-steps (of 32) whose loads are issued together

template <int MB>
__global__ void __launch_bounds__(256) skinny_gemm_kernel(const bf16* __restrict__ x, int64_t x_rs,
                                                          const bf16* __restrict__ w, const bf16* __restrict__ bias,
                                                          bf16* __restrict__ out, int64_t o_rs, int M, int N, int K,
                                                          int splitk, float* __restrict__ ws, int* __restrict__ cnt) {
  // the 4 waves' partial tiles, then (split-K) the "last arriver" flag: ONE LDS object
  __shared__ __attribute__((aligned(16))) float red[4 * MB * 64 * 4 + 4];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int ntiles = gridDim.x / splitk;
  const int tile = blockIdx.x / splitk, split = blockIdx.x % splitk;
  const int n0 = tile * 16;
  const int steps = K / 32;
  const int sb0 = (int)((int64_t)steps * split / splitk), sb1 = (int)((int64_t)steps * (split + 1) / splitk);
  const int nsb = sb1 - sb0;
  const int s0 = sb0 + nsb * wid / 4, s1 = sb0 + nsb * (wid + 1) / 4;

  const int r16 = lane & 15, kq = 8 * (lane >> 4);
  const bf16* wp = w + (size_t)min(n0 + r16, N - 1) * K + kq;  // rows past N: clamped, never stored
  const bf16* xp[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int m = mb * 16 + r16;
    xp[mb] = x + (size_t)(m < M ? m : 0) * x_rs + kq;  // rows past M: only feed unstored outputs
  }
  sk_f32x4 acc[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) acc[mb] = (sk_f32x4){0.f, 0.f, 0.f, 0.f};

  for (int s = s0; s < s1; s += kSkU) {
    // all loads of the group first (addresses clamped to the last valid step: no per-load
    // branches), then the MFMAs of the steps that exist
    sk_u32x4 wa[kSkU], xb[kSkU][MB];
#pragma unroll
    for (int u = 0; u < kSkU; ++u) {
      const size_t ko = (size_t)min(s + u, s1 - 1) * 32;
      wa[u] = *reinterpret_cast<const sk_u32x4*>(wp + ko);
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) xb[u][mb] = *reinterpret_cast<const sk_u32x4*>(xp[mb] + ko);
    }
#pragma unroll
    for (int u = 0; u < kSkU; ++u) {
      if (s + u < s1) {
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
          acc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(sk_bf16x8, wa[u]),
                                                            __builtin_bit_cast(sk_bf16x8, xb[u][mb]), acc[mb], 0, 0, 0);
      }
    }
  }

  sk_f32x4* r4 = reinterpret_cast<sk_f32x4*>(red);
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) r4[(wid * MB + mb) * 64 + lane] = acc[mb];
  __syncthreads();

  auto epilogue = [&](int it, sk_f32x4 v) {
    const int ln = it & 63, m = (it >> 6) * 16 + (ln & 15), nb = n0 + 4 * (ln >> 4);
    if (m >= M) return;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = nb + r;
      if (n < N) out[(size_t)m * o_rs + n] = from_f<bf16>(v[r] + (bias ? bf2f(bias[n]) : 0.f));
    }
  };
  auto block_sum = [&](int it) {
    const int mb = it >> 6, ln = it & 63;
    return r4[mb * 64 + ln] + r4[(MB + mb) * 64 + ln] + r4[(2 * MB + mb) * 64 + ln] + r4[(3 * MB + mb) * 64 + ln];
  };
  if (splitk == 1) {
    for (int it = t; it < MB * 64; it += 256) epilogue(it, block_sum(it));
    return;
  }
  // split-K: slab of this (split, tile), then the counter hand-off (agent-scope release on the
  // writer, acquire on the last arriver; correct wherever the tile's splits ran)
  sk_f32x4* slab = reinterpret_cast<sk_f32x4*>(ws);
  for (int it = t; it < MB * 64; it += 256) slab[((size_t)split * ntiles + tile) * (MB * 64) + it] = block_sum(it);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* flag = reinterpret_cast<int*>(red + 4 * MB * 64 * 4);
  if (t == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int prev = __hip_atomic_fetch_add(&cnt[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = prev == splitk - 1;
  }
  __syncthreads();
  if (!*flag) return;
  if (t == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(&cnt[tile], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  for (int it = t; it < MB * 64; it += 256) {
    sk_f32x4 v = slab[(size_t)tile * (MB * 64) + it];
    for (int sp = 1; sp < splitk; ++sp) v += slab[((size_t)sp * ntiles + tile) * (MB * 64) + it];
    epilogue(it, v);
  }
}

// Gated-MLP decode projection with the activation in the epilogue:
//   out[M, I] = act(x · Wgᵀ) ⊙ (x · Wuᵀ),  gu = [Wg; Wu] ([2I, K], the packed gate|up weight).
// A workgroup owns 16 output columns n0.. and runs the skinny main loop on BOTH weight slices
// (gate rows n0 + r16 and up rows I + n0 + r16) with the same 4-way K split, group size and
// LDS reduction order as skinny_gemm_kernel at splitk 1; the epilogue rounds gate and up to bf16
// (the unfused GEMM's output) before act(g) · u, so the result is bit-identical to skinny_gemm
// followed by the packed gated-activation kernel — one launch and one [M, 2I] round trip fewer
// per block of the Gemma decode step.
template <int MB>
__global__ void __launch_bounds__(256) skinny_gated_kernel(const bf16* __restrict__ x, int64_t x_rs,
                                                           const bf16* __restrict__ gu, bf16* __restrict__ out,
                                                           int64_t o_rs, int M, int I, int K, int kind) {
  __shared__ __attribute__((aligned(16))) float red[2 * 4 * MB * 64 * 4];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int n0 = blockIdx.x * 16;
  const int steps = K / 32;
  const int s0 = steps * wid / 4, s1 = steps * (wid + 1) / 4;
  const int r16 = lane & 15, kq = 8 * (lane >> 4);
  const int nr = min(n0 + r16, I - 1);  // rows past I: clamped, never stored
  const bf16* wg = gu + (size_t)nr * K + kq;
  const bf16* wu = gu + (size_t)(I + nr) * K + kq;
  const bf16* xp[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int m = mb * 16 + r16;
    xp[mb] = x + (size_t)(m < M ? m : 0) * x_rs + kq;
  }
  sk_f32x4 ag[MB], au[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) ag[mb] = au[mb] = (sk_f32x4){0.f, 0.f, 0.f, 0.f};

  for (int s = s0; s < s1; s += kSkU) {
    sk_u32x4 ga[kSkU], ua[kSkU], xb[kSkU][MB];
#pragma unroll
    for (int u = 0; u < kSkU; ++u) {
      const size_t ko = (size_t)min(s + u, s1 - 1) * 32;
      ga[u] = *reinterpret_cast<const sk_u32x4*>(wg + ko);
      ua[u] = *reinterpret_cast<const sk_u32x4*>(wu + ko);
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) xb[u][mb] = *reinterpret_cast<const sk_u32x4*>(xp[mb] + ko);
    }
#pragma unroll
    for (int u = 0; u < kSkU; ++u) {
      if (s + u < s1) {
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) {
          ag[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(sk_bf16x8, ga[u]),
                                                           __builtin_bit_cast(sk_bf16x8, xb[u][mb]), ag[mb], 0, 0, 0);
          au[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(sk_bf16x8, ua[u]),
                                                           __builtin_bit_cast(sk_bf16x8, xb[u][mb]), au[mb], 0, 0, 0);
        }
      }
    }
  }

  sk_f32x4* r4 = reinterpret_cast<sk_f32x4*>(red);
  sk_f32x4* u4 = r4 + 4 * MB * 64;
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    r4[(wid * MB + mb) * 64 + lane] = ag[mb];
    u4[(wid * MB + mb) * 64 + lane] = au[mb];
  }
  __syncthreads();
  for (int it = t; it < MB * 64; it += 256) {
    const int mb = it >> 6, ln = it & 63;
    const sk_f32x4 g = r4[mb * 64 + ln] + r4[(MB + mb) * 64 + ln] + r4[(2 * MB + mb) * 64 + ln] +
                       r4[(3 * MB + mb) * 64 + ln];
    const sk_f32x4 v = u4[mb * 64 + ln] + u4[(MB + mb) * 64 + ln] + u4[(2 * MB + mb) * 64 + ln] +
                       u4[(3 * MB + mb) * 64 + ln];
    const int m = mb * 16 + (ln & 15), nb = n0 + 4 * (ln >> 4);
    if (m >= M) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = nb + r;
      if (n < I)
        out[(size_t)m * o_rs + n] =
            from_f<bf16>(act_f(bf2f(from_f<bf16>(g[r])), kind) * bf2f(from_f<bf16>(v[r])));
    }
  }
}

// Decode QKV projection with RoPE in the epilogue: out[M, (H + 2Hkv)·D] = rope(x · Wᵀ) for the
// first `nrot` heads (Q and K, rotate-half pairs (j, j + D/2) with one position's cos / sin [D/2]:
// every decode row sits at the same cache position), V columns passed through. A workgroup owns
// a PAIR of 16-column slices — columns j0.. and j0 + D/2.. of one head — so both halves of every
// rotated pair end in the same lanes; the main loop is the skinny one on two weight slices, with
// the split-K slab hand-off of skinny_gemm_kernel for the narrow grid (Gemma-3 1B: 48 pair tiles).
// Rounding: both halves are rounded to bf16 (the unfused GEMM's output) before the rotation, whose
// arithmetic is the RoPE kernel's (x1·c − x2·s, x2·c + x1·s). One launch and one [M, W] round trip
// per block fewer than GEMM → RoPE kernel.
template <int MB>
__global__ void __launch_bounds__(256) skinny_qkv_rope_kernel(const bf16* __restrict__ x, int64_t x_rs,
                                                              const bf16* __restrict__ w, bf16* __restrict__ out,
                                                              int64_t o_rs, int M, int K, int D, int nrot,
                                                              const float* __restrict__ cosv,
                                                              const float* __restrict__ sinv, int splitk,
                                                              float* __restrict__ ws, int* __restrict__ cnt) {
  __shared__ __attribute__((aligned(16))) float red[2 * 4 * MB * 64 * 4 + 4];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int ntiles = gridDim.x / splitk;
  const int tile = blockIdx.x / splitk, split = blockIdx.x % splitk;
  const int half = D / 2, ppt = half / 16;  // pair tiles per head
  const int head = tile / ppt, j0 = (tile - head * ppt) * 16;
  const int c1 = head * D + j0, c2 = c1 + half;
  const int steps = K / 32;
  const int sb0 = (int)((int64_t)steps * split / splitk), sb1 = (int)((int64_t)steps * (split + 1) / splitk);
  const int nsb = sb1 - sb0;
  const int s0 = sb0 + nsb * wid / 4, s1 = sb0 + nsb * (wid + 1) / 4;
  const int r16 = lane & 15, kq = 8 * (lane >> 4);
  const bf16* w1 = w + (size_t)(c1 + r16) * K + kq;
  const bf16* w2 = w + (size_t)(c2 + r16) * K + kq;
  const bf16* xp[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int m = mb * 16 + r16;
    xp[mb] = x + (size_t)(m < M ? m : 0) * x_rs + kq;
  }
  sk_f32x4 a1[MB], a2[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) a1[mb] = a2[mb] = (sk_f32x4){0.f, 0.f, 0.f, 0.f};

  for (int s = s0; s < s1; s += kSkU) {
    sk_u32x4 wa1[kSkU], wa2[kSkU], xb[kSkU][MB];
#pragma unroll
    for (int u = 0; u < kSkU; ++u) {
      const size_t ko = (size_t)min(s + u, s1 - 1) * 32;
      wa1[u] = *reinterpret_cast<const sk_u32x4*>(w1 + ko);
      wa2[u] = *reinterpret_cast<const sk_u32x4*>(w2 + ko);
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) xb[u][mb] = *reinterpret_cast<const sk_u32x4*>(xp[mb] + ko);
    }
#pragma unroll
    for (int u = 0; u < kSkU; ++u) {
      if (s + u < s1) {
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) {
          a1[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(sk_bf16x8, wa1[u]),
                                                           __builtin_bit_cast(sk_bf16x8, xb[u][mb]), a1[mb], 0, 0, 0);
          a2[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(sk_bf16x8, wa2[u]),
                                                           __builtin_bit_cast(sk_bf16x8, xb[u][mb]), a2[mb], 0, 0, 0);
        }
      }
    }
  }

  sk_f32x4* r4 = reinterpret_cast<sk_f32x4*>(red);  // [half 0 | half 1][wave][mb][lane]
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    r4[(wid * MB + mb) * 64 + lane] = a1[mb];
    r4[((4 + wid) * MB + mb) * 64 + lane] = a2[mb];
  }
  __syncthreads();
  auto block_sum = [&](int hf, int it) {
    const sk_f32x4* b = r4 + hf * 4 * MB * 64;
    const int mb = it >> 6, ln = it & 63;
    return b[mb * 64 + ln] + b[(MB + mb) * 64 + ln] + b[(2 * MB + mb) * 64 + ln] + b[(3 * MB + mb) * 64 + ln];
  };
  const bool rot = head < nrot;
  auto epilogue = [&](int it, sk_f32x4 v1, sk_f32x4 v2) {
    const int ln = it & 63, m = (it >> 6) * 16 + (ln & 15), nb = 4 * (ln >> 4);
    if (m >= M) return;
    bf16* o = out + (size_t)m * o_rs;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float x1 = bf2f(from_f<bf16>(v1[r])), x2 = bf2f(from_f<bf16>(v2[r]));
      float y1 = x1, y2 = x2;
      if (rot) {
        const float cs = cosv[j0 + nb + r], sn = sinv[j0 + nb + r];
        y1 = x1 * cs - x2 * sn;
        y2 = x2 * cs + x1 * sn;
      }
      o[c1 + nb + r] = from_f<bf16>(y1);
      o[c2 + nb + r] = from_f<bf16>(y2);
    }
  };
  if (splitk == 1) {
    for (int it = t; it < MB * 64; it += 256) epilogue(it, block_sum(0, it), block_sum(1, it));
    return;
  }
  // split-K: the pair's two partial slabs, then the counter hand-off of skinny_gemm_kernel
  sk_f32x4* slab = reinterpret_cast<sk_f32x4*>(ws);
  const size_t per = (size_t)2 * MB * 64;
  for (int it = t; it < MB * 64; it += 256) {
    slab[((size_t)split * ntiles + tile) * per + it] = block_sum(0, it);
    slab[((size_t)split * ntiles + tile) * per + MB * 64 + it] = block_sum(1, it);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* flag = reinterpret_cast<int*>(red + 2 * 4 * MB * 64 * 4);
  if (t == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int prev = __hip_atomic_fetch_add(&cnt[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = prev == splitk - 1;
  }
  __syncthreads();
  if (!*flag) return;
  if (t == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(&cnt[tile], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  for (int it = t; it < MB * 64; it += 256) {
    sk_f32x4 v1 = slab[(size_t)tile * per + it], v2 = slab[(size_t)tile * per + MB * 64 + it];
    for (int sp = 1; sp < splitk; ++sp) {
      v1 += slab[((size_t)sp * ntiles + tile) * per + it];
      v2 += slab[((size_t)sp * ntiles + tile) * per + MB * 64 + it];
    }
    epilogue(it, v1, v2);
  }
}

// Decode-step linear with the residual add + LayerNorm fused in front and an optional GELU
// behind: out = act(LN(resid_in + delta + dbias) · Wᵀ + bias), M ≤ 64 rows, K ≤ 1024. Every
// workgroup normalises all M rows itself (one wave per row, the add+LayerNorm kernel's math:
// fp32 two-pass statistics on the register copy) into a padded bf16 LDS image, then runs the
// skinny main loop with its x fragments read from LDS; workgroup 0 also writes resid_out (the
// fp32 residual stream after the add). It replaces add+LN → GEMM (→ GELU): 2-3 kernels of the
// graph-replayed decode step, whose fixed per-kernel cost (~4.5 µs at batch 64) exceeds what
// each of them computes. The redundant per-workgroup LayerNorm reads the rows from L2.
// act: 0 none, 1 GELU (erf), 2 GELU (tanh), applied to the bf16-rounded linear output (the
// rounding point of the unfused GEMM → GELU pair).
template <int MB>
__global__ void __launch_bounds__(256) decode_ln_linear_kernel(
    const float* __restrict__ rin, const bf16* __restrict__ delta, const float* __restrict__ dbias,
    float* __restrict__ rout, const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
    const bf16* __restrict__ w, const bf16* __restrict__ bias, bf16* __restrict__ out, int64_t o_rs, int M, int N,
    int K, int act) {
  extern __shared__ __attribute__((aligned(16))) char dsm[];  // [MB*16][K + 8] bf16 | partial tiles
  const int LDX = K + 8;  // +16 B per row: the 16 rows of a fragment read land on distinct banks
  bf16* xs = reinterpret_cast<bf16*>(dsm);
  float* red = reinterpret_cast<float*>(dsm + (size_t)MB * 16 * LDX * 2);
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const bool write_resid = rout != nullptr && blockIdx.x == 0;
  // rows wid, wid+4, ...: a compile-time trip count, so the loads of later rows can be issued
  // under the reductions of earlier ones (a runtime-bounded loop serialised one row's HBM/L2
  // latency after another)
#pragma unroll
  for (int i = 0; i < MB * 4; ++i) {
    const int m = wid + 4 * i;
    bf16* xr = xs + (size_t)m * LDX;
    if (m >= M) {
      for (int c = 8 * lane; c < K; c += 512) *reinterpret_cast<uint4*>(xr + c) = uint4{0u, 0u, 0u, 0u};
      continue;
    }
    const size_t base = (size_t)m * K;
    float v[4][4];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = 4 * (lane + 64 * j);
      if (c >= K) {
        v[j][0] = v[j][1] = v[j][2] = v[j][3] = 0.f;
        continue;
      }
      const float4_t r = *reinterpret_cast<const float4_t*>(rin + base + c);
      v[j][0] = r[0]; v[j][1] = r[1]; v[j][2] = r[2]; v[j][3] = r[3];
      if (delta) {
        const uint2 u = *reinterpret_cast<const uint2*>(delta + base + c);
        float d[4] = {__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                      __uint_as_float(u.y & 0xffff0000u)};
        if (dbias) {
          const float4_t e = *reinterpret_cast<const float4_t*>(dbias + c);
#pragma unroll
          for (int k = 0; k < 4; ++k) d[k] += e[k];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) v[j][k] += d[k];
        if (write_resid) *reinterpret_cast<float4_t*>(rout + base + c) = float4_t{v[j][0], v[j][1], v[j][2], v[j][3]};
      }
      s += v[j][0] + v[j][1] + v[j][2] + v[j][3];
    }
    const float mean = wave_sum(s) / K;
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float d = v[j][k] - mean;
        ss += 4 * (lane + 64 * j) < K ? d * d : 0.f;
      }
    const float rstd = rsqrtf(wave_sum(ss) / K + eps);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = 4 * (lane + 64 * j);
      if (c >= K) continue;
      const float4_t g = *reinterpret_cast<const float4_t*>(gamma + c);
      const float4_t b = *reinterpret_cast<const float4_t*>(beta + c);
      *reinterpret_cast<uint2*>(xr + c) =
          uint2{pack_bf16x2((v[j][0] - mean) * rstd * g[0] + b[0], (v[j][1] - mean) * rstd * g[1] + b[1]),
                pack_bf16x2((v[j][2] - mean) * rstd * g[2] + b[2], (v[j][3] - mean) * rstd * g[3] + b[3])};
    }
  }
  __syncthreads();

  const int n0 = blockIdx.x * 16;
  const int steps = K / 32;
  const int s0 = steps * wid / 4, s1 = steps * (wid + 1) / 4;
  const int r16 = lane & 15, kq = 8 * (lane >> 4);
  const bf16* wp = w + (size_t)min(n0 + r16, N - 1) * K + kq;  // rows past N: clamped, never stored
  const bf16* xl = xs + (size_t)r16 * LDX + kq;
  sk_f32x4 acc[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) acc[mb] = (sk_f32x4){0.f, 0.f, 0.f, 0.f};
  for (int s = s0; s < s1; s += kSkU) {
    sk_u32x4 wa[kSkU];
#pragma unroll
    for (int u = 0; u < kSkU; ++u) wa[u] = *reinterpret_cast<const sk_u32x4*>(wp + (size_t)min(s + u, s1 - 1) * 32);
#pragma unroll
    for (int u = 0; u < kSkU; ++u) {
      if (s + u < s1) {
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) {
          const sk_u32x4 xb = *reinterpret_cast<const sk_u32x4*>(xl + (size_t)mb * 16 * LDX + (s + u) * 32);
          acc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(sk_bf16x8, wa[u]),
                                                            __builtin_bit_cast(sk_bf16x8, xb), acc[mb], 0, 0, 0);
        }
      }
    }
  }
  sk_f32x4* r4 = reinterpret_cast<sk_f32x4*>(red);
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) r4[(wid * MB + mb) * 64 + lane] = acc[mb];
  __syncthreads();
  for (int it = t; it < MB * 64; it += 256) {
    const int mb = it >> 6, ln = it & 63;
    const sk_f32x4 v = r4[mb * 64 + ln] + r4[(MB + mb) * 64 + ln] + r4[(2 * MB + mb) * 64 + ln] +
                       r4[(3 * MB + mb) * 64 + ln];
    const int m = mb * 16 + (ln & 15), nb = n0 + 4 * (ln >> 4);
    if (m >= M) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = nb + r;
      if (n >= N) continue;
      float y = v[r] + (bias ? bf2f(bias[n]) : 0.f);
      if (act) y = gelu_f(bf2f(from_f<bf16>(y)), act - 1);
      out[(size_t)m * o_rs + n] = from_f<bf16>(y);
    }
  }
}

}  // namespace penroz

using namespace penroz;

// out = act(LN(resid_in + delta + dbias) · Wᵀ + bias); resid_out (optional) receives the sum.
void decode_ln_linear(torch::Tensor rin, c10::optional<torch::Tensor> delta, c10::optional<torch::Tensor> dbias,
                      c10::optional<torch::Tensor> rout, torch::Tensor gamma, torch::Tensor beta, double eps,
                      torch::Tensor w, c10::optional<torch::Tensor> bias, torch::Tensor out, int64_t act) {
  TORCH_CHECK(rin.is_cuda() && rin.scalar_type() == torch::kFloat32 && rin.dim() == 2 && rin.is_contiguous(),
              "decode_ln_linear: fp32 contiguous [M, K] residual");
  const int M = rin.size(0), K = rin.size(1), N = w.size(0);
  TORCH_CHECK(M >= 1 && M <= 64 && K % 32 == 0 && K <= 1024, "decode_ln_linear: M <= 64, K % 32 == 0, K <= 1024");
  TORCH_CHECK(w.scalar_type() == torch::kBFloat16 && w.is_contiguous() && w.size(1) == K &&
                  reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0, "decode_ln_linear: bf16 contiguous W [N, K]");
  TORCH_CHECK(out.scalar_type() == torch::kBFloat16 && out.dim() == 2 && out.size(0) == M && out.size(1) == N &&
                  out.stride(1) == 1, "decode_ln_linear: bf16 out [M, N]");
  TORCH_CHECK(gamma.scalar_type() == torch::kFloat32 && beta.scalar_type() == torch::kFloat32 && gamma.numel() == K &&
                  beta.numel() == K && gamma.is_contiguous() && beta.is_contiguous(), "decode_ln_linear: fp32 gamma/beta [K]");
  TORCH_CHECK(act >= 0 && act <= 2, "decode_ln_linear: act 0 (none), 1 (GELU erf), 2 (GELU tanh)");
  const bf16* dp = nullptr;
  const float* dbp = nullptr;
  float* rop = nullptr;
  const bf16* bp = nullptr;
  if (delta.has_value() && delta->defined()) {
    TORCH_CHECK(delta->scalar_type() == torch::kBFloat16 && delta->is_contiguous() && delta->numel() == (int64_t)M * K,
                "decode_ln_linear: bf16 contiguous delta [M, K]");
    dp = reinterpret_cast<const bf16*>(delta->data_ptr());
    TORCH_CHECK(rout.has_value() && rout->defined(), "decode_ln_linear: a residual add needs resid_out");
  }
  if (dbias.has_value() && dbias->defined()) {
    TORCH_CHECK(dp && dbias->scalar_type() == torch::kFloat32 && dbias->is_contiguous() && dbias->numel() == K,
                "decode_ln_linear: fp32 dbias [K] (with delta)");
    dbp = dbias->data_ptr<float>();
  }
  if (rout.has_value() && rout->defined()) {
    TORCH_CHECK(rout->scalar_type() == torch::kFloat32 && rout->is_contiguous() && rout->numel() == (int64_t)M * K &&
                    rout->data_ptr() != rin.data_ptr(), "decode_ln_linear: fp32 resid_out [M, K], not aliasing resid_in");
    rop = rout->data_ptr<float>();
  }
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->scalar_type() == torch::kBFloat16 && bias->is_contiguous() && bias->numel() == N,
                "decode_ln_linear: bf16 bias [N]");
    bp = reinterpret_cast<const bf16*>(bias->data_ptr());
  }
  const int MB = M <= 16 ? 1 : M <= 32 ? 2 : 4;
  const size_t lds = (size_t)MB * 16 * (K + 8) * 2 + (size_t)4 * MB * 64 * 16;
  static bool attr_set = false;
  if (!attr_set) {
    const int mx = 4 * 16 * (1024 + 8) * 2 + 4 * 4 * 64 * 16;
    hipFuncSetAttribute(reinterpret_cast<const void*>(decode_ln_linear_kernel<1>), hipFuncAttributeMaxDynamicSharedMemorySize, mx);
    hipFuncSetAttribute(reinterpret_cast<const void*>(decode_ln_linear_kernel<2>), hipFuncAttributeMaxDynamicSharedMemorySize, mx);
    hipFuncSetAttribute(reinterpret_cast<const void*>(decode_ln_linear_kernel<4>), hipFuncAttributeMaxDynamicSharedMemorySize, mx);
    attr_set = true;
  }
  auto stream = at::hip::getCurrentHIPStream();
  const dim3 grid((N + 15) / 16);
  const float* rp = rin.data_ptr<float>();
  const float* gp = gamma.data_ptr<float>();
  const float* bt = beta.data_ptr<float>();
  auto wp = reinterpret_cast<const bf16*>(w.data_ptr());
  auto op = reinterpret_cast<bf16*>(out.data_ptr());
#define PENROZ_DLL(MBV)                                                                                             \
  hipLaunchKernelGGL(decode_ln_linear_kernel<MBV>, grid, dim3(256), lds, stream, rp, dp, dbp, rop, gp, bt, (float)eps, \
                     wp, bp, op, (int64_t)out.stride(0), M, N, K, (int)act)
  if (MB == 1) PENROZ_DLL(1);
  else if (MB == 2) PENROZ_DLL(2);
  else PENROZ_DLL(4);
#undef PENROZ_DLL
}

// splitk <= 0: chosen here (workgroups ~ 192 when the 16-column slices alone are too few).
// ws: fp32 workspace (>= splitk * ceil(N/16) * MB * 256 floats when splitk > 1); cnt: int32
// counters (>= ceil(N/16)), zero on entry — every launch leaves them zero again.
int64_t skinny_gemm(torch::Tensor x, torch::Tensor w, c10::optional<torch::Tensor> bias, torch::Tensor out,
                    torch::Tensor ws, torch::Tensor cnt, int64_t splitk) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == torch::kBFloat16 && w.scalar_type() == torch::kBFloat16 &&
                  out.scalar_type() == torch::kBFloat16, "skinny_gemm: bf16 x / w / out");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2, "skinny_gemm: 2-D operands");
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(M >= 1 && M <= 64 && w.size(1) == K && K % 32 == 0, "skinny_gemm: M <= 64, K % 32 == 0");
  TORCH_CHECK(x.stride(1) == 1 && x.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "skinny_gemm: x rows 16-B aligned");
  TORCH_CHECK(w.is_contiguous() && reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0, "skinny_gemm: w contiguous");
  TORCH_CHECK(out.size(0) == M && out.size(1) == N && out.stride(1) == 1, "skinny_gemm: out [M, N]");
  const bf16* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->scalar_type() == torch::kBFloat16 && bias->is_contiguous() && bias->numel() == N,
                "skinny_gemm: bf16 bias [N]");
    bp = reinterpret_cast<const bf16*>(bias->data_ptr());
  }
  const int ntiles = (N + 15) / 16, steps = K / 32;
  const int MB = M <= 16 ? 1 : M <= 32 ? 2 : 4;
  if (splitk <= 0) {
    splitk = 1;
    if (ntiles < 128) splitk = std::max(1, std::min({(192 + ntiles - 1) / ntiles, steps / 4, 16}));
  }
  TORCH_CHECK(splitk >= 1 && splitk <= steps, "skinny_gemm: bad split");
  if (splitk > 1) {
    TORCH_CHECK(ws.is_cuda() && ws.scalar_type() == torch::kFloat32 &&
                    ws.numel() >= (int64_t)splitk * ntiles * MB * 256, "skinny_gemm: workspace too small");
    TORCH_CHECK(cnt.is_cuda() && cnt.scalar_type() == torch::kInt32 && cnt.numel() >= ntiles,
                "skinny_gemm: counters too small");
  }
  auto stream = at::hip::getCurrentHIPStream();
  const dim3 grid(ntiles * splitk);
  auto xp = reinterpret_cast<const bf16*>(x.data_ptr());
  auto wp = reinterpret_cast<const bf16*>(w.data_ptr());
  auto op = reinterpret_cast<bf16*>(out.data_ptr());
  float* wsp = splitk > 1 ? ws.data_ptr<float>() : nullptr;
  int* cp = splitk > 1 ? cnt.data_ptr<int>() : nullptr;
#define PENROZ_SKINNY(MBV)                                                                                       \
  hipLaunchKernelGGL(skinny_gemm_kernel<MBV>, grid, dim3(256), 0, stream, xp, (int64_t)x.stride(0), wp, bp, op, \
                     (int64_t)out.stride(0), M, N, K, (int)splitk, wsp, cp)
  if (MB == 1) PENROZ_SKINNY(1);
  else if (MB == 2) PENROZ_SKINNY(2);
  else PENROZ_SKINNY(4);
#undef PENROZ_SKINNY
  return splitk;
}

// out[M, I] = act(x · gu[:I]ᵀ) ⊙ (x · gu[I:]ᵀ) for M <= 64 decode rows (kind: 0 gelu, 1 gelu_tanh,
// 2 silu); bit-identical to skinny_gemm(x, gu) followed by gated_act_packed.
void skinny_gated(torch::Tensor x, torch::Tensor gu, torch::Tensor out, int64_t kind) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == torch::kBFloat16 && gu.scalar_type() == torch::kBFloat16 &&
                  out.scalar_type() == torch::kBFloat16, "skinny_gated: bf16 x / gu / out");
  TORCH_CHECK(x.dim() == 2 && gu.dim() == 2 && out.dim() == 2, "skinny_gated: 2-D operands");
  const int M = x.size(0), K = x.size(1);
  TORCH_CHECK(gu.size(0) % 2 == 0, "skinny_gated: packed [gate; up] weight [2I, K]");
  const int I = gu.size(0) / 2;
  TORCH_CHECK(M >= 1 && M <= 64 && I >= 1 && gu.size(1) == K && K % 32 == 0, "skinny_gated: M <= 64, K % 32 == 0");
  TORCH_CHECK(x.stride(1) == 1 && x.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "skinny_gated: x rows 16-B aligned");
  TORCH_CHECK(gu.is_contiguous() && reinterpret_cast<uintptr_t>(gu.data_ptr()) % 16 == 0, "skinny_gated: gu contiguous");
  TORCH_CHECK(out.size(0) == M && out.size(1) == I && out.stride(1) == 1, "skinny_gated: out [M, I]");
  TORCH_CHECK(kind >= 0 && kind <= 2, "skinny_gated: kind 0 (gelu), 1 (gelu_tanh), 2 (silu)");
  const int MB = M <= 16 ? 1 : M <= 32 ? 2 : 4;
  auto stream = at::hip::getCurrentHIPStream();
  const dim3 grid((I + 15) / 16);
  auto xp = reinterpret_cast<const bf16*>(x.data_ptr());
  auto wp = reinterpret_cast<const bf16*>(gu.data_ptr());
  auto op = reinterpret_cast<bf16*>(out.data_ptr());
#define PENROZ_SKG(MBV)                                                                                              \
  hipLaunchKernelGGL(skinny_gated_kernel<MBV>, grid, dim3(256), 0, stream, xp, (int64_t)x.stride(0), wp, op,        \
                     (int64_t)out.stride(0), M, I, K, (int)kind)
  if (MB == 1) PENROZ_SKG(1);
  else if (MB == 2) PENROZ_SKG(2);
  else PENROZ_SKG(4);
#undef PENROZ_SKG
}

// The fused QKV + RoPE kernel's automatic split-K (workgroups ~ 192 when the 32-column tiles alone
// are too few) and the fp32 workspace it then needs: ONE rule, used by the launcher below and
// exported (skinny_qkv_rope_plan) for the Python-side admission check (ops/gemm.py
// skinny_qkv_rope_ok), which must refuse a shape before a graph capture rather than let this
// launcher's workspace check throw inside it.
static int qkv_rope_auto_split(int N, int K) {
  const int ntiles = N / 32, steps = K / 32;
  return ntiles >= 128 ? 1 : std::max(1, std::min({(192 + ntiles - 1) / ntiles, steps / 4, 16}));
}
static int64_t qkv_rope_ws_floats(int M, int N, int splitk) {
  const int MB = M <= 16 ? 1 : M <= 32 ? 2 : 4;
  return splitk > 1 ? (int64_t)splitk * (N / 32) * MB * 512 : 0;
}

// (split-K, fp32 workspace floats, counters) of skinny_qkv_rope at M rows, N = heads·D, K
std::vector<int64_t> skinny_qkv_rope_plan(int64_t M, int64_t N, int64_t K) {
  const int split = qkv_rope_auto_split((int)N, (int)K);
  return {split, qkv_rope_ws_floats((int)M, (int)N, split), split > 1 ? N / 32 : 0};
}

// out[M, (H + 2Hkv)·D] = x · wᵀ with RoPE (cos / sin [D/2] of the one decode position) applied to
// the first nrot = H + Hkv heads; M <= 64, D % 32 == 0. Returns the split-K factor used.
int64_t skinny_qkv_rope(torch::Tensor x, torch::Tensor w, torch::Tensor cosv, torch::Tensor sinv, int64_t D,
                        int64_t nrot, torch::Tensor out, torch::Tensor ws, torch::Tensor cnt, int64_t splitk) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == torch::kBFloat16 && w.scalar_type() == torch::kBFloat16 &&
                  out.scalar_type() == torch::kBFloat16, "skinny_qkv_rope: bf16 x / w / out");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2, "skinny_qkv_rope: 2-D operands");
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(M >= 1 && M <= 64 && w.size(1) == K && K % 32 == 0, "skinny_qkv_rope: M <= 64, K % 32 == 0");
  TORCH_CHECK(D >= 32 && D % 32 == 0 && N % D == 0 && nrot >= 0 && nrot <= N / D,
              "skinny_qkv_rope: D % 32 == 0, whole heads, nrot <= heads");
  TORCH_CHECK(x.stride(1) == 1 && x.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "skinny_qkv_rope: x rows 16-B aligned");
  TORCH_CHECK(w.is_contiguous() && reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0, "skinny_qkv_rope: w contiguous");
  TORCH_CHECK(out.size(0) == M && out.size(1) == N && out.stride(1) == 1, "skinny_qkv_rope: out [M, N]");
  TORCH_CHECK(cosv.scalar_type() == torch::kFloat32 && sinv.scalar_type() == torch::kFloat32 && cosv.is_contiguous() &&
                  sinv.is_contiguous() && cosv.numel() == D / 2 && sinv.numel() == D / 2,
              "skinny_qkv_rope: fp32 cos / sin [D/2]");
  const int ntiles = N / 32, steps = K / 32;
  const int MB = M <= 16 ? 1 : M <= 32 ? 2 : 4;
  if (splitk <= 0) splitk = qkv_rope_auto_split(N, K);
  TORCH_CHECK(splitk >= 1 && splitk <= steps, "skinny_qkv_rope: bad split");
  if (splitk > 1) {
    TORCH_CHECK(ws.is_cuda() && ws.scalar_type() == torch::kFloat32 && ws.numel() >= qkv_rope_ws_floats(M, N, (int)splitk),
                "skinny_qkv_rope: workspace too small");
    TORCH_CHECK(cnt.is_cuda() && cnt.scalar_type() == torch::kInt32 && cnt.numel() >= ntiles,
                "skinny_qkv_rope: counters too small");
  }
  auto stream = at::hip::getCurrentHIPStream();
  const dim3 grid(ntiles * splitk);
  auto xp = reinterpret_cast<const bf16*>(x.data_ptr());
  auto wp = reinterpret_cast<const bf16*>(w.data_ptr());
  auto op = reinterpret_cast<bf16*>(out.data_ptr());
  float* wsp = splitk > 1 ? ws.data_ptr<float>() : nullptr;
  int* cp = splitk > 1 ? cnt.data_ptr<int>() : nullptr;
#define PENROZ_SQR(MBV)                                                                                              \
  hipLaunchKernelGGL(skinny_qkv_rope_kernel<MBV>, grid, dim3(256), 0, stream, xp, (int64_t)x.stride(0), wp, op,     \
                     (int64_t)out.stride(0), M, K, (int)D, (int)nrot, cosv.data_ptr<float>(), sinv.data_ptr<float>(), \
                     (int)splitk, wsp, cp)
  if (MB == 1) PENROZ_SQR(1);
  else if (MB == 2) PENROZ_SQR(2);
  else PENROZ_SQR(4);
#undef PENROZ_SQR
  return splitk;
}
