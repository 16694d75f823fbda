// Batched decode linears (M = decode rows, 16..64 typical): the two kernels of a GPT block's
// decode step besides attention, shaped so that a block costs 5 launches instead of 8.
//
//   decode_ln_gemm : out = act(LN(resid) · Wᵀ + bias)          (QKV; fc + GELU)
//   decode_gemm_acc: resid += x · Wᵀ + bias                     (proj; fc2)
//
// The residual stream stays fp32 and is updated IN PLACE by decode_gemm_acc's epilogue, so
// the separate "residual add + LayerNorm" kernel between the GEMMs disappears: the next
// decode_ln_gemm normalises the rows it needs itself. Two choices keep that redundant
// normalisation cheap (the round-2 fused kernel normalised all 64 rows in every 16-column
// workgroup and lost at 64 rows, profiles/decode_fused_rows_r2.log):
//   * a decode_ln_gemm workgroup owns 16 ROWS × 64 columns (4 waves × one 16x16x32 MFMA column
//     block over the full K), so it normalises only its 16 rows (4 per wave) — 16× less
//     prologue work per workgroup than 64 rows × 16 columns, for the same 144-192 workgroups;
//   * the weight fragments of the whole K range (K ≤ 1024: ≤ 32 × 16 B per lane) are issued
//     BEFORE the prologue, so their HBM latency hides under the normalisation.
// decode_gemm_acc owns 16 rows × 16 columns (N = 768 → 48 column blocks × 4 row blocks = 192
// workgroups without split-K), its 4 waves split K and reduce through LDS; the epilogue is a
// deterministic float4 read-modify-write of the residual (one owner per element, no atomics).
// Row blocks of one column tile are placed on one XCD (blockIdx % 8 picks the XCD), so the
// 4 row blocks' weight reads after the first hit that XCD's L2.
//
// MFMA: v_mfma_f32_16x16x32_bf16 with A = 16 weight rows (output columns n), B = 16 x rows
// (decode rows m): lane holds D[n = 4(lane>>4) + r][m = lane & 15], r = 0..3 — four
// consecutive outputs of one row, stored as 8 B (bf16) or RMW'd as 16 B (fp32).
#include "common.h"
#include <type_traits>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

namespace penroz {

typedef short dl_bf16x8 __attribute__((ext_vector_type(8)));
typedef float dl_f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t dl_u32x4 __attribute__((ext_vector_type(4)));

constexpr int kDlMaxSteps = 32;  // decode_ln_gemm: K <= 1024 (32 k-steps of 32)
constexpr int kDlGroup = 32;     // decode_gemm_acc: k-steps per wave whose loads are issued together

// (row block, column tile) of a workgroup: the nrb row blocks of column tile ct share
// blockIdx % 8 (one XCD) for the full groups of 8 tiles; the tail is row-block-major.
__device__ __forceinline__ void dl_tile(int id, int nrb, int nct, int& rb, int& ct) {
  const int full = (nct / 8) * 8 * nrb;
  if (id < full) {
    const int g = 8 * nrb;
    ct = (id / g) * 8 + (id & 7);
    rb = (id % g) >> 3;
  } else {
    const int r = id - full;
    ct = (nct / 8) * 8 + r / nrb;
    rb = r % nrb;
  }
}

// grid = ceil(M/16) * ceil(N/(64/KS)), block 256. LDS: 16 normalised rows [16][K + 8] bf16.
// KS = 2: 32-column tiles, the two waves of a column block split K in halves and meet in LDS —
// twice the workgroups (qkv at 64 rows: 288 instead of 144 on 256 CUs), half the weight bytes per
// workgroup.
template <int KS>
__global__ void __launch_bounds__(256) decode_ln_gemm_kernel(const float* __restrict__ resid,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, float eps,
                                                             const bf16* __restrict__ w, const bf16* __restrict__ bias,
                                                             bf16* __restrict__ out, int64_t o_rs, int M, int N, int K,
                                                             int act, int flags) {
  __shared__ __attribute__((aligned(16))) bf16 xs[16 * (1024 + 8)];
  __shared__ __attribute__((aligned(16))) dl_f32x4 kred[KS > 1 ? (KS - 1) * (4 / KS) * 64 : 1];
  constexpr int TW = 64 / KS, NCB = 4 / KS, MS = kDlMaxSteps / KS;
  const int LDX = K + 8;  // +16 B per row: a fragment's 16 row reads spread over the banks
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int cb = wid % NCB, kh = wid / NCB;  // column block, K part (KS = 2: halves)
  int rb, ct;
  dl_tile(blockIdx.x, (M + 15) / 16, (N + TW - 1) / TW, rb, ct);
  const int steps = K / 32 / KS, s0 = kh * steps;  // this wave's k-steps: s0 .. s0 + steps
  const int r16 = lane & 15, kq = 8 * (lane >> 4);
  const int n0 = ct * TW + cb * 16;  // this wave's column block
  const bool live = n0 < N;

  // 1. the wave's weight fragments for its K range, in flight during the prologue
  dl_u32x4 wa[MS];
  {
    const bf16* wp = w + (size_t)min(n0 + r16, N - 1) * K + kq + s0 * 32;
#pragma unroll
    for (int s = 0; s < MS; ++s)
      if (s < steps && live && !(flags & 2)) wa[s] = *reinterpret_cast<const dl_u32x4*>(wp + s * 32);
  }

  // the epilogue's bias terms, fetched now (not a memory round trip after the MFMAs)
  const int m = rb * 16 + r16, n = n0 + 4 * (lane >> 4);
  float bv[4] = {0.f, 0.f, 0.f, 0.f};
  if (bias && live) {
    const uint2 u = *reinterpret_cast<const uint2*>(bias + n);
    bv[0] = __uint_as_float(u.x << 16); bv[1] = __uint_as_float(u.x & 0xffff0000u);
    bv[2] = __uint_as_float(u.y << 16); bv[3] = __uint_as_float(u.y & 0xffff0000u);
  }

  // 2. LayerNorm of rows rb*16 + wid + 4i (fp32 two-pass on the register copy) -> bf16 LDS
  float v[4][4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = rb * 16 + wid + 4 * i;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = 4 * (lane + 64 * j);
      if (m < M && c < K && !(flags & 1)) {
        const float4_t r = *reinterpret_cast<const float4_t*>(resid + (size_t)m * K + c);
        v[i][j][0] = r[0]; v[i][j][1] = r[1]; v[i][j][2] = r[2]; v[i][j][3] = r[3];
      } else {
        v[i][j][0] = v[i][j][1] = v[i][j][2] = v[i][j][3] = 0.f;
      }
    }
  }
  float4_t g[4], b[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = 4 * (lane + 64 * j);
    if (c < K) {
      g[j] = *reinterpret_cast<const float4_t*>(gamma + c);
      b[j] = *reinterpret_cast<const float4_t*>(beta + c);
    }
  }
  const float inv_k = 1.f / (float)K;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (flags & 8) break;
    const int lr = wid + 4 * i;  // local row
    bf16* xr = xs + lr * LDX;
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) s += (v[i][j][0] + v[i][j][1]) + (v[i][j][2] + v[i][j][3]);
    const float mean = wave_sum(s) * inv_k;
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (4 * (lane + 64 * j) < K)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float d = v[i][j][k] - mean;
          ss += d * d;
        }
    const float rstd = rsqrtf(wave_sum(ss) * inv_k + eps);
    const bool row_ok = rb * 16 + lr < M;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = 4 * (lane + 64 * j);
      if (c >= K) continue;
      uint2 pk{0u, 0u};
      if (row_ok)
        pk = uint2{pack_bf16x2((v[i][j][0] - mean) * rstd * g[j][0] + b[j][0], (v[i][j][1] - mean) * rstd * g[j][1] + b[j][1]),
                   pack_bf16x2((v[i][j][2] - mean) * rstd * g[j][2] + b[j][2], (v[i][j][3] - mean) * rstd * g[j][3] + b[j][3])};
      *reinterpret_cast<uint2*>(xr + c) = pk;
    }
  }
  __syncthreads();
  if (KS == 1 && !live) return;
  if (flags & 2) {
#pragma unroll
    for (int s = 0; s < MS; ++s) wa[s] = dl_u32x4{0u, 0u, 0u, 0u};
  }

  // 3. MFMA over the wave's K range, x fragments from LDS
  dl_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const bf16* xl = xs + r16 * LDX + kq + s0 * 32;
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    if (s < steps && live && !(flags & 16)) {
      const dl_u32x4 xb = *reinterpret_cast<const dl_u32x4*>(xl + s * 32);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(dl_bf16x8, wa[s]),
                                                    __builtin_bit_cast(dl_bf16x8, xb), acc, 0, 0, 0);
    }
  }
  if constexpr (KS > 1) {  // the K parts of a column block meet in LDS (every wave reaches the barrier)
    if (kh > 0) kred[((kh - 1) * NCB + cb) * 64 + lane] = acc;
    __syncthreads();
    if (kh > 0 || !live) return;
#pragma unroll
    for (int p = 0; p < KS - 1; ++p) acc += kred[(p * NCB + cb) * 64 + lane];
  }

  // 4. bias (+ GELU on the bf16-rounded linear output, the unfused pair's rounding point)
  if (m >= M || (flags & 4)) return;
  float y[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    y[r] = acc[r] + bv[r];
    if (act) y[r] = gelu_f(bf2f(from_f<bf16>(y[r])), act - 1);
  }
  *reinterpret_cast<uint2*>(out + (size_t)m * o_rs + n) = uint2{pack_bf16x2(y[0], y[1]), pack_bf16x2(y[2], y[3])};
}

// grid = ceil(M/16) * (N/16), block 256; waves split K, partial tiles reduced through LDS.
__global__ void __launch_bounds__(256) decode_gemm_acc_kernel(const bf16* __restrict__ x, int64_t x_rs,
                                                              const bf16* __restrict__ w, const bf16* __restrict__ bias,
                                                              float* __restrict__ resid, int M, int N, int K, int flags) {
  __shared__ __attribute__((aligned(16))) dl_f32x4 red[3 * 64];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  int rb, ct;
  dl_tile(blockIdx.x, (M + 15) / 16, N / 16, rb, ct);
  const int steps = K / 32;
  const int s0 = steps * wid / 4, s1 = steps * (wid + 1) / 4;
  const int r16 = lane & 15, kq = 8 * (lane >> 4);
  const int n0 = ct * 16;
  const bf16* wp = w + (size_t)(n0 + r16) * K + kq;
  const int mx = rb * 16 + r16;
  const bf16* xp = x + (size_t)(mx < M ? mx : 0) * x_rs + kq;  // rows past M feed unstored outputs
  // the epilogue's operands (this lane's 4 residual values and bias terms, wave 0 only) are
  // fetched now, so the tail is LDS reduce + one store instead of two more memory round trips
  const int m = rb * 16 + r16, n = n0 + 4 * (lane >> 4);
  const bool owner = wid == 0 && m < M && !(flags & 4);
  float4_t cur = {0.f, 0.f, 0.f, 0.f}, bv = {0.f, 0.f, 0.f, 0.f};
  if (owner) {
    cur = *reinterpret_cast<const float4_t*>(resid + (size_t)m * N + n);
    if (bias) {
      const uint2 u = *reinterpret_cast<const uint2*>(bias + n);
      bv = float4_t{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                    __uint_as_float(u.y & 0xffff0000u)};
    }
  }
  dl_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int s = s0; s < s1; s += kDlGroup) {  // one pass for K <= 4096: every load in flight at once
    dl_u32x4 wa[kDlGroup], xb[kDlGroup];
#pragma unroll
    for (int u = 0; u < kDlGroup; ++u) {
      if (s + u < s1) {
        const size_t ko = (size_t)(s + u) * 32;
        wa[u] = (flags & 2) ? dl_u32x4{0u, 0u, 0u, 0u} : *reinterpret_cast<const dl_u32x4*>(wp + ko);
        xb[u] = (flags & 1) ? dl_u32x4{0u, 0u, 0u, 0u} : *reinterpret_cast<const dl_u32x4*>(xp + ko);
      }
    }
#pragma unroll
    for (int u = 0; u < kDlGroup; ++u)
      if (s + u < s1)
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(dl_bf16x8, wa[u]),
                                                      __builtin_bit_cast(dl_bf16x8, xb[u]), acc, 0, 0, 0);
  }
  if (wid) red[(wid - 1) * 64 + lane] = acc;
  __syncthreads();
  if (!owner) return;
  acc += red[lane] + red[64 + lane] + red[128 + lane];
  float4_t* rp = reinterpret_cast<float4_t*>(resid + (size_t)m * N + n);
#pragma unroll
  for (int r = 0; r < 4; ++r) cur[r] += acc[r] + bv[r];
  *rp = cur;
}

// out[M, N] = x · Wᵀ (bf16) — decode_gemm_acc's tiling (16 rows × 16 columns per workgroup, the 4
// waves split K, partial tiles reduced through LDS; every load of a wave's k-range in flight at
// once) with a plain store, or with GATED the packed [gate; up] weight [2I, K]: a workgroup takes
// gate columns n0..n0+15 and the matching up columns I + n0.., out[m, n] = bf16(act(bf16(g)) ·
// bf16(u)) — the rounding of GEMM -> gated_act_packed. For the Gemma decode program's 17-64-row
// steps, where hipBLASLt's picks for these skinny shapes ran 36-216 workgroups (gate|up at 64
// rows: 72 workgroups, 1.6 TB/s of weights; profiles/notes_r6.md).
// RB row blocks of 16 per workgroup share each weight fragment (RB = 4 at 33-64 rows and wide N:
// the weights are read once instead of once per row block).
template <bool GATED, int RB>
__global__ void __launch_bounds__(256) decode_gemm_kernel(const bf16* __restrict__ x, int64_t x_rs,
                                                          const bf16* __restrict__ w, bf16* __restrict__ out,
                                                          int64_t o_rs, int M, int N, int K, int kind) {
  constexpr int GROUP = (GATED ? 16 : kDlGroup) / RB;
  __shared__ __attribute__((aligned(16))) dl_f32x4 red[2][RB][3 * 64];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  int rbg, ct;
  dl_tile(blockIdx.x, (M + 16 * RB - 1) / (16 * RB), N / 16, rbg, ct);
  const int steps = K / 32;
  const int s0 = steps * wid / 4, s1 = steps * (wid + 1) / 4;
  const int r16 = lane & 15, kq = 8 * (lane >> 4);
  const int n0 = ct * 16;
  const bf16* wp = w + (size_t)(n0 + r16) * K + kq;
  const bf16* up = wp + (size_t)N * K;  // GATED: the up row of the same column
  const bf16* xp[RB];
#pragma unroll
  for (int r = 0; r < RB; ++r) {
    const int mx = (rbg * RB + r) * 16 + r16;
    xp[r] = x + (size_t)(mx < M ? mx : 0) * x_rs + kq;  // rows past M feed unstored outputs
  }
  dl_f32x4 acc0[RB], acc1[RB];
#pragma unroll
  for (int r = 0; r < RB; ++r) acc0[r] = acc1[r] = dl_f32x4{0.f, 0.f, 0.f, 0.f};
  for (int s = s0; s < s1; s += GROUP) {
    dl_u32x4 wg[GROUP], wu[GROUP], xb[RB * GROUP];  // (flat: a 2-D array of these miscompiled)
#pragma unroll
    for (int u = 0; u < GROUP; ++u) {
      if (s + u < s1) {
        const size_t ko = (size_t)(s + u) * 32;
        wg[u] = *reinterpret_cast<const dl_u32x4*>(wp + ko);
        if constexpr (GATED) wu[u] = *reinterpret_cast<const dl_u32x4*>(up + ko);
#pragma unroll
        for (int r = 0; r < RB; ++r) xb[r * GROUP + u] = *reinterpret_cast<const dl_u32x4*>(xp[r] + ko);
      }
    }
#pragma unroll
    for (int u = 0; u < GROUP; ++u) {
      if (s + u < s1) {
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          acc0[r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(dl_bf16x8, wg[u]),
                                                            __builtin_bit_cast(dl_bf16x8, xb[r * GROUP + u]), acc0[r], 0, 0, 0);
          if constexpr (GATED)
            acc1[r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(dl_bf16x8, wu[u]),
                                                              __builtin_bit_cast(dl_bf16x8, xb[r * GROUP + u]), acc1[r], 0, 0, 0);
        }
      }
    }
  }
  if (wid) {
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      red[0][r][(wid - 1) * 64 + lane] = acc0[r];
      if constexpr (GATED) red[1][r][(wid - 1) * 64 + lane] = acc1[r];
    }
  }
  __syncthreads();
  if (wid) return;
  const int n = n0 + 4 * (lane >> 4);
#pragma unroll
  for (int r = 0; r < RB; ++r) {
    const int m = (rbg * RB + r) * 16 + r16;
    if (m >= M) continue;
    dl_f32x4 a0 = acc0[r] + red[0][r][lane] + red[0][r][64 + lane] + red[0][r][128 + lane];
    dl_f32x4 a1 = acc1[r];
    if constexpr (GATED) a1 += red[1][r][lane] + red[1][r][64 + lane] + red[1][r][128 + lane];
    float y[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (GATED)
        y[i] = act_f(bf2f(from_f<bf16>(a0[i])), kind) * bf2f(from_f<bf16>(a1[i]));
      else
        y[i] = a0[i];
    }
    *reinterpret_cast<uint2*>(out + (size_t)m * o_rs + n) = uint2{pack_bf16x2(y[0], y[1]), pack_bf16x2(y[2], y[3])};
  }
}

// ------------------------------------------------------------------------------------------
// Decode GEMV for M <= 4 rows (batch-1..4 decode): out[M, N] = act(x · Wᵀ + bias), x either a
// bf16 matrix or — LN mode — LayerNorm(resid_in + delta + dbias) computed in the kernel (the
// residual sum also written to resid_out by workgroup 0). At these shapes a kernel's time is its
// fixed costs: launch, one memory round trip, reductions. So:
//   * one wave per workgroup, no LDS, no barrier: a half-wave (32 lanes) owns one weight row, a
//     wave 2·RP rows; lane l reads 16-B chunks l, l+32, ... of its row (512 contiguous bytes per
//     half-wave instruction) and the matching chunks of x;
//   * every load of the wave — all its weight chunks, its x (or residual / delta / bias / γ / β)
//     chunks — is issued before the first use: one round trip;
//   * LN mode normalises each row within the half-wave (fp32 two-pass on the register copy, the
//     add+LayerNorm kernel's math), rounds to bf16 (the GEMM operand's precision);
//   * products by v_dot2c_f32_bf16 (bf16 pairs into fp32), one 5-step half-wave reduction per
//     (row, x row), stores from lane 0 of each half.
// No MFMA: at M <= 4 a 16x16 MFMA tile would waste ≥ 3/4 of itself, and the VALU work is small.
typedef __bf16 dv_bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float dot8_bf16(const uint4& a, const uint4& b, float c) {
  c = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(dv_bf16x2, a.x), __builtin_bit_cast(dv_bf16x2, b.x), c, false);
  c = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(dv_bf16x2, a.y), __builtin_bit_cast(dv_bf16x2, b.y), c, false);
  c = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(dv_bf16x2, a.z), __builtin_bit_cast(dv_bf16x2, b.z), c, false);
  c = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(dv_bf16x2, a.w), __builtin_bit_cast(dv_bf16x2, b.w), c, false);
  return c;
}

__device__ __forceinline__ float half_sum(float v) {  // sum over the 32 lanes of this half-wave
#pragma unroll
  for (int o = 1; o < 32; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// EPI (the two half-waves' rows as a pair): 0 — independent rows, act(y + bias); 1 — gated MLP
// on the packed [gate; up] weight (N = 2I rows): half 0 takes gate row n, half 1 up row I + n,
// out[n] = act_f(bf16(g), kind) · bf16(u) (skinny_gated's rounding); 2 — RoPE QKV: pair p of head
// p / (D/2), j = p % (D/2): half 0 row head·D + j, half 1 row + D/2, both rounded to bf16, then
// rotated by one position's cos / sin [D/2] for the first nrot heads (skinny_qkv_rope's math).
// In modes 1 / 2 a wave owns RP output pairs.
// PRO: 0 — x is the bf16 operand; 1 — LN mode (GPT: fp32 residual + delta + dbias, LayerNorm)
template <int M, int PRO, int RP, int CPL, int EPI = 0>
__global__ void __launch_bounds__(64) decode_gemv_kernel(
    const float* __restrict__ rin, const bf16* __restrict__ delta, const float* __restrict__ dbias,
    float* __restrict__ rout, const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
    const bf16* __restrict__ x, int64_t x_rs, const bf16* __restrict__ w, const bf16* __restrict__ bias,
    bf16* __restrict__ out, int64_t o_rs, int N, int K, int act, int D = 0, int nrot = 0,
    const float* __restrict__ cosv = nullptr, const float* __restrict__ sinv = nullptr,
    const int64_t* __restrict__ eidx = nullptr, const bf16* __restrict__ ewte = nullptr,
    const bf16* __restrict__ ewpe = nullptr, const int64_t* __restrict__ epos = nullptr, int eV = 0, int eP = 0) {
  constexpr bool LN = PRO == 1;
  // EPI 3 (PRO 0 only): the whole wave on each of its RP rows — lane l reads chunks l, l + 64, …
  // — twice the workgroups of the half-wave form for the same rows per wave
  constexpr bool WR = EPI == 3;
  constexpr int CS = WR ? 64 : 32;  // lanes striding over a row's chunks
  static_assert(!WR || PRO == 0, "wave-per-row mode reads a bf16 x");
  const int lane = threadIdx.x, h = lane >> 5, l32 = lane & 31;
  const int cl = WR ? lane : l32;
  const int nc = K / 8;  // 16-B chunks per row
  const int n0 = blockIdx.x * (EPI == 0 ? 2 * RP : RP);
  const int npair = N / 2;  // modes 1 / 2: output pairs
  auto row_of = [&](int rp) -> int {  // this half's weight row for its rp-th row (pair)
    if constexpr (WR) {
      return min(n0 + rp, N - 1);
    } else if constexpr (EPI == 0) {
      return min(n0 + 2 * rp + h, N - 1);
    } else if constexpr (EPI == 1) {
      return min(n0 + rp, npair - 1) + h * npair;
    } else {
      const int p = min(n0 + rp, npair - 1), hd = D / 2, head = p / hd;
      return head * D + (p - head * hd) + h * hd;
    }
  };
  // 1. every load first: weight chunks of this half's rows
  uint4 wv[RP][CPL];
#pragma unroll
  for (int rp = 0; rp < RP; ++rp) {
    const bf16* wr = w + (size_t)row_of(rp) * K;
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c = cl + CS * i;
      wv[rp][i] = c < nc ? *reinterpret_cast<const uint4*>(wr + 8 * c) : uint4{0u, 0u, 0u, 0u};
    }
  }
  uint4 xb[M][CPL];
  if constexpr (PRO == 0) {
#pragma unroll
    for (int m = 0; m < M; ++m)
#pragma unroll
      for (int i = 0; i < CPL; ++i) {
        const int c = cl + CS * i;
        xb[m][i] = c < nc ? *reinterpret_cast<const uint4*>(x + (size_t)m * x_rs + 8 * c) : uint4{0u, 0u, 0u, 0u};
      }
  } else {
    float v[M][CPL][8];
    // embedding mode (ewte): the residual row is wte[token] + wpe[position] (the first block of a
    // decode step, embed_fwd_kernel's arithmetic: clamped token, position min(*epos, P - 1))
    const int epos_v = ewte ? min((int)*epos, eP - 1) : 0;
#pragma unroll
    for (int m = 0; m < M; ++m)
#pragma unroll
      for (int i = 0; i < CPL; ++i) {
        const int c = l32 + 32 * i;
        if (c < nc && ewte) {
          int64_t tok = eidx[m];
          tok = tok < 0 ? 0 : (tok >= eV ? eV - 1 : tok);
          float a[8], b[8];
          Vec8<bf16>::load(ewte + (size_t)tok * K + 8 * c, a);
          Vec8<bf16>::load(ewpe + (size_t)epos_v * K + 8 * c, b);
#pragma unroll
          for (int k = 0; k < 8; ++k) v[m][i][k] = a[k] + b[k];
        } else if (c < nc) {
          const float4_t* rp = reinterpret_cast<const float4_t*>(rin + (size_t)m * K + 8 * c);
          const float4_t a = rp[0], b = rp[1];
          v[m][i][0] = a[0]; v[m][i][1] = a[1]; v[m][i][2] = a[2]; v[m][i][3] = a[3];
          v[m][i][4] = b[0]; v[m][i][5] = b[1]; v[m][i][6] = b[2]; v[m][i][7] = b[3];
          if (delta) {
            float d[8];
            Vec8<bf16>::load(delta + (size_t)m * K + 8 * c, d);
            if (dbias) {
              const float4_t* e = reinterpret_cast<const float4_t*>(dbias + 8 * c);
              const float4_t e0 = e[0], e1 = e[1];
              d[0] += e0[0]; d[1] += e0[1]; d[2] += e0[2]; d[3] += e0[3];
              d[4] += e1[0]; d[5] += e1[1]; d[6] += e1[2]; d[7] += e1[3];
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) v[m][i][k] += d[k];
          }
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) v[m][i][k] = 0.f;
        }
      }
    if ((delta || ewte) && rout && blockIdx.x == 0 && h == 0) {
#pragma unroll
      for (int m = 0; m < M; ++m)
#pragma unroll
        for (int i = 0; i < CPL; ++i) {
          const int c = l32 + 32 * i;
          if (c < nc) {
            float4_t* op = reinterpret_cast<float4_t*>(rout + (size_t)m * K + 8 * c);
            op[0] = float4_t{v[m][i][0], v[m][i][1], v[m][i][2], v[m][i][3]};
            op[1] = float4_t{v[m][i][4], v[m][i][5], v[m][i][6], v[m][i][7]};
          }
        }
    }
    const float inv_k = 1.f / (float)K;
    float mean[M], rstd[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < CPL; ++i)
#pragma unroll
        for (int k = 0; k < 8; ++k) s += v[m][i][k];
      mean[m] = half_sum(s) * inv_k;
    }
#pragma unroll
    for (int m = 0; m < M; ++m) {
      float ss = 0.f;
#pragma unroll
      for (int i = 0; i < CPL; ++i) {
        const bool ok = l32 + 32 * i < nc;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float d = v[m][i][k] - mean[m];
          ss += ok ? d * d : 0.f;
        }
      }
      rstd[m] = rsqrtf(half_sum(ss) * inv_k + eps);
    }
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c = l32 + 32 * i;
      float g[8] = {}, bt[8] = {};
      if (c < nc) {
        const float4_t* gp = reinterpret_cast<const float4_t*>(gamma + 8 * c);
        const float4_t* bp = reinterpret_cast<const float4_t*>(beta + 8 * c);
        const float4_t g0 = gp[0], g1 = gp[1], b0 = bp[0], b1 = bp[1];
        g[0] = g0[0]; g[1] = g0[1]; g[2] = g0[2]; g[3] = g0[3]; g[4] = g1[0]; g[5] = g1[1]; g[6] = g1[2]; g[7] = g1[3];
        bt[0] = b0[0]; bt[1] = b0[1]; bt[2] = b0[2]; bt[3] = b0[3]; bt[4] = b1[0]; bt[5] = b1[1]; bt[6] = b1[2]; bt[7] = b1[3];
      }
#pragma unroll
      for (int m = 0; m < M; ++m) {
        float y[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) y[k] = (v[m][i][k] - mean[m]) * rstd[m] * g[k] + bt[k];
        xb[m][i] = uint4{pack_bf16x2(y[0], y[1]), pack_bf16x2(y[2], y[3]), pack_bf16x2(y[4], y[5]),
                         pack_bf16x2(y[6], y[7])};
      }
    }
  }
  // 2. products and the half-wave reductions
  float acc[RP][M];
#pragma unroll
  for (int rp = 0; rp < RP; ++rp)
#pragma unroll
    for (int m = 0; m < M; ++m) {
      float a = 0.f;
#pragma unroll
      for (int i = 0; i < CPL; ++i) a = dot8_bf16(wv[rp][i], xb[m][i], a);
      a = half_sum(a);
      if constexpr (WR) a += __shfl_xor(a, 32, 64);
      acc[rp][m] = a;
    }
  // 3. epilogue: lane 0 of each half stores its rows
  if constexpr (WR) {
    if (lane != 0) return;
#pragma unroll
    for (int rp = 0; rp < RP; ++rp) {
      const int n = n0 + rp;
      if (n >= N) continue;
      const float bv = bias ? bf2f(bias[n]) : 0.f;
#pragma unroll
      for (int m = 0; m < M; ++m) {
        float y = acc[rp][m] + bv;
        if (act) y = gelu_f(bf2f(from_f<bf16>(y)), act - 1);
        out[(size_t)m * o_rs + n] = from_f<bf16>(y);
      }
    }
    return;
  } else if constexpr (EPI != 0) {
    float other[RP][M];  // the partner half's sums (lane 0 <-> lane 32)
#pragma unroll
    for (int rp = 0; rp < RP; ++rp)
#pragma unroll
      for (int m = 0; m < M; ++m) other[rp][m] = __shfl_xor(acc[rp][m], 32, 64);
    if (l32 != 0) return;
#pragma unroll
    for (int rp = 0; rp < RP; ++rp) {
      const int p = n0 + rp;
      if (p >= npair) continue;
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const float mine = bf2f(from_f<bf16>(acc[rp][m])), theirs = bf2f(from_f<bf16>(other[rp][m]));
        if constexpr (EPI == 1) {
          if (h == 0) out[(size_t)m * o_rs + p] = from_f<bf16>(act_f(mine, act) * theirs);
        } else {
          const int hd = D / 2, head = p / hd, j = p - head * hd;
          float y = mine;
          if (head < nrot) {
            const float cs = cosv[j], sn = sinv[j];
            y = h == 0 ? mine * cs - theirs * sn : mine * cs + theirs * sn;
          }
          out[(size_t)m * o_rs + head * D + j + h * hd] = from_f<bf16>(y);
        }
      }
    }
    return;
  }
  if (l32 != 0) return;
#pragma unroll
  for (int rp = 0; rp < RP; ++rp) {
    const int n = n0 + 2 * rp + h;
    if (n >= N) continue;
    const float bv = bias ? bf2f(bias[n]) : 0.f;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      float y = acc[rp][m] + bv;
      if (act) y = gelu_f(bf2f(from_f<bf16>(y)), act - 1);
      out[(size_t)m * o_rs + n] = from_f<bf16>(y);
    }
  }
}

}  // namespace penroz

using namespace penroz;

static void dl_check_w(const torch::Tensor& w, int K, const char* who) {
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == torch::kBFloat16 && w.dim() == 2 && w.is_contiguous() &&
                  w.size(1) == K && w.size(0) % 16 == 0 && reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0,
              who, ": bf16 contiguous 16-B aligned W [N, K], N % 16 == 0");
}

static const bf16* dl_bias(const c10::optional<torch::Tensor>& bias, int N, const char* who) {
  if (!bias.has_value() || !bias->defined()) return nullptr;
  TORCH_CHECK(bias->scalar_type() == torch::kBFloat16 && bias->is_contiguous() && bias->numel() == N &&
                  reinterpret_cast<uintptr_t>(bias->data_ptr()) % 8 == 0,
              who, ": bf16 bias [N], 8-B aligned");
  return reinterpret_cast<const bf16*>(bias->data_ptr());
}

// out[M, N] = act(LayerNorm(resid) · wᵀ + bias); act 0 none, 1 GELU (erf), 2 GELU (tanh).
// flags (timing ablations only, outputs wrong when set): 1 no residual reads, 2 no weight reads,
// 4 no stores, 8 no LayerNorm (LDS image unwritten), 16 no MFMA
void decode_ln_gemm(torch::Tensor resid, torch::Tensor gamma, torch::Tensor beta, double eps, torch::Tensor w,
                    c10::optional<torch::Tensor> bias, torch::Tensor out, int64_t act, int64_t flags) {
  TORCH_CHECK(resid.is_cuda() && resid.scalar_type() == torch::kFloat32 && resid.dim() == 2 && resid.is_contiguous(),
              "decode_ln_gemm: fp32 contiguous resid [M, K]");
  const int M = resid.size(0), K = resid.size(1);
  TORCH_CHECK(M >= 1 && K % 32 == 0 && K <= 32 * kDlMaxSteps, "decode_ln_gemm: K % 32 == 0, K <= 1024");
  dl_check_w(w, K, "decode_ln_gemm");
  const int N = w.size(0);
  TORCH_CHECK(gamma.scalar_type() == torch::kFloat32 && beta.scalar_type() == torch::kFloat32 && gamma.numel() == K &&
                  beta.numel() == K && gamma.is_contiguous() && beta.is_contiguous(),
              "decode_ln_gemm: fp32 gamma / beta [K]");
  TORCH_CHECK(out.scalar_type() == torch::kBFloat16 && out.dim() == 2 && out.size(0) == M && out.size(1) == N &&
                  out.stride(1) == 1 && out.stride(0) % 4 == 0 && reinterpret_cast<uintptr_t>(out.data_ptr()) % 8 == 0,
              "decode_ln_gemm: bf16 out [M, N], rows 8-B aligned");
  TORCH_CHECK(act >= 0 && act <= 2, "decode_ln_gemm: act 0 (none), 1 (GELU erf), 2 (GELU tanh)");
  const bf16* bp = dl_bias(bias, N, "decode_ln_gemm");
  // K halves (KS = 2) by default: GPT-2 decode B = 16 / 32 / 64 0.567 / 0.584 / 0.636 -> 0.532 /
  // 0.550 / 0.620 ms/step; quarters (KS = 4) lost: 0.55 / 0.74 / 0.96 — every workgroup repeats the
  // LayerNorm of its 16 rows (profiles/decode_r5.md). PENROZ_DECODE_LN_KSPLIT=1: 64-column tiles.
  static const int ks_env = [] {
    const char* e = std::getenv("PENROZ_DECODE_LN_KSPLIT");
    return e && e[0] == '1' ? 1 : 2;
  }();
  const int ks = ks_env == 2 && (K / 32) % 2 == 0 ? 2 : 1;
  const int tw = 64 / ks;
  const int grid = ((M + 15) / 16) * ((N + tw - 1) / tw);
  hipLaunchKernelGGL(ks == 2 ? decode_ln_gemm_kernel<2> : decode_ln_gemm_kernel<1>,
                     dim3(grid), dim3(256), 0, at::hip::getCurrentHIPStream(), resid.data_ptr<float>(), gamma.data_ptr<float>(),
                     beta.data_ptr<float>(), (float)eps, reinterpret_cast<const bf16*>(w.data_ptr()), bp,
                     reinterpret_cast<bf16*>(out.data_ptr()), (int64_t)out.stride(0), M, N, K, (int)act, (int)flags);
}

// resid[M, N] += x · wᵀ + bias (fp32 residual, in place). flags: timing ablations (1 no x reads,
// 2 no weight reads, 4 no stores)
void decode_gemm_acc(torch::Tensor x, torch::Tensor w, c10::optional<torch::Tensor> bias, torch::Tensor resid,
                     int64_t flags) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == torch::kBFloat16 && x.dim() == 2 && x.stride(1) == 1 &&
                  x.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "decode_gemm_acc: bf16 x [M, K], rows 16-B aligned");
  const int M = x.size(0), K = x.size(1);
  TORCH_CHECK(M >= 1 && K % 32 == 0, "decode_gemm_acc: K % 32 == 0");
  dl_check_w(w, K, "decode_gemm_acc");
  const int N = w.size(0);
  TORCH_CHECK(resid.scalar_type() == torch::kFloat32 && resid.is_contiguous() && resid.dim() == 2 &&
                  resid.size(0) == M && resid.size(1) == N,
              "decode_gemm_acc: fp32 contiguous resid [M, N]");
  const bf16* bp = dl_bias(bias, N, "decode_gemm_acc");
  const int grid = ((M + 15) / 16) * (N / 16);
  hipLaunchKernelGGL(decode_gemm_acc_kernel, dim3(grid), dim3(256), 0, at::hip::getCurrentHIPStream(),
                     reinterpret_cast<const bf16*>(x.data_ptr()), (int64_t)x.stride(0),
                     reinterpret_cast<const bf16*>(w.data_ptr()), bp, resid.data_ptr<float>(), M, N, K, (int)flags);
}

// out[M, N] = x · Wᵀ (kind < 0), or with the packed [gate; up] weight [2I, K] out[M, I] =
// act(x·Wgᵀ) ⊙ (x·Wuᵀ) (kind 0 gelu, 1 gelu_tanh, 2 silu) — decode_gemm_kernel
void decode_gemm(torch::Tensor x, torch::Tensor w, torch::Tensor out, int64_t kind) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == torch::kBFloat16 && x.dim() == 2 && x.stride(1) == 1 &&
                  x.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "decode_gemm: bf16 x [M, K], rows 16-B aligned");
  const int M = x.size(0), K = x.size(1);
  TORCH_CHECK(M >= 1 && K % 32 == 0, "decode_gemm: K % 32 == 0");
  dl_check_w(w, K, "decode_gemm");
  const bool gated = kind >= 0;
  TORCH_CHECK(kind <= 2, "decode_gemm: kind -1 (plain), 0 gelu, 1 gelu_tanh, 2 silu");
  const int N = gated ? w.size(0) / 2 : w.size(0);
  TORCH_CHECK(N % 16 == 0 && (!gated || w.size(0) == 2 * N), "decode_gemm: N (gated: I) % 16 == 0");
  TORCH_CHECK(out.scalar_type() == torch::kBFloat16 && out.dim() == 2 && out.size(0) == M && out.size(1) == N &&
                  out.stride(1) == 1 && out.stride(0) % 4 == 0 && reinterpret_cast<uintptr_t>(out.data_ptr()) % 8 == 0,
              "decode_gemm: bf16 out [M, N], rows 8-B aligned");
  // 4 row blocks per workgroup once there are more than two and the columns alone give >= 256
  // workgroups (weights read once); otherwise one row block per workgroup (more workgroups)
  const int rb = (M > 32 && N / 16 >= 256) ? 4 : 1;
  const int grid = ((M + 16 * rb - 1) / (16 * rb)) * (N / 16);
  auto kern = gated ? (rb == 4 ? decode_gemm_kernel<true, 4> : decode_gemm_kernel<true, 1>)
                    : (rb == 4 ? decode_gemm_kernel<false, 4> : decode_gemm_kernel<false, 1>);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, at::hip::getCurrentHIPStream(),
                     reinterpret_cast<const bf16*>(x.data_ptr()), (int64_t)x.stride(0),
                     reinterpret_cast<const bf16*>(w.data_ptr()), reinterpret_cast<bf16*>(out.data_ptr()),
                     (int64_t)out.stride(0), M, N, K, (int)(gated ? kind : 0));
}

// out[M, N] = act(x · Wᵀ + bias) for M <= 4 decode rows (decode_gemv_kernel). LN mode (x
// undefined): x = LayerNorm(resid_in + delta + dbias) with γ / β, resid_out receives the sum.
// act 0 none, 1 GELU (erf), 2 GELU (tanh). rows_per_wave 2, 4 or 8 (0: by N).
void decode_gemv(c10::optional<torch::Tensor> x, c10::optional<torch::Tensor> rin, c10::optional<torch::Tensor> delta,
                 c10::optional<torch::Tensor> dbias, c10::optional<torch::Tensor> rout,
                 c10::optional<torch::Tensor> gamma, c10::optional<torch::Tensor> beta, double eps, torch::Tensor w,
                 c10::optional<torch::Tensor> bias, torch::Tensor out, int64_t act, int64_t rows_per_wave,
                 c10::optional<torch::Tensor> emb_idx, c10::optional<torch::Tensor> emb_wte,
                 c10::optional<torch::Tensor> emb_wpe, c10::optional<torch::Tensor> emb_pos) {
  const bool ln = !(x.has_value() && x->defined());
  const bool emb = emb_wte.has_value() && emb_wte->defined();
  const int64_t* eip = nullptr;
  const bf16 *ewp = nullptr, *epp = nullptr;
  const int64_t* eps_p = nullptr;
  int eV = 0, eP = 0;
  const int N = w.size(0), K = w.size(1);
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == torch::kBFloat16 && w.dim() == 2 && w.is_contiguous() &&
                  reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0 && K % 8 == 0,
              "decode_gemv: bf16 contiguous 16-B aligned W [N, K], K % 8 == 0");
  TORCH_CHECK(K <= 256 * 32, "decode_gemv: K <= 8192");
  TORCH_CHECK(act >= 0 && act <= 2, "decode_gemv: act 0 (none), 1 (GELU erf), 2 (GELU tanh)");
  int M;
  const bf16* xp = nullptr;
  int64_t x_rs = 0;
  const float *rp = nullptr, *dbp = nullptr, *gp = nullptr, *bt = nullptr;
  const bf16* dp = nullptr;
  float* rop = nullptr;
  if (!ln) {
    TORCH_CHECK(x->scalar_type() == torch::kBFloat16 && x->dim() == 2 && x->size(1) == K && x->stride(1) == 1 &&
                    x->stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(x->data_ptr()) % 16 == 0,
                "decode_gemv: bf16 x [M, K], rows 16-B aligned");
    M = x->size(0);
    xp = reinterpret_cast<const bf16*>(x->data_ptr());
    x_rs = x->stride(0);
  } else if (emb) {  // LN mode on the step's embedding rows; resid_out receives them
    TORCH_CHECK(emb_idx.has_value() && emb_wpe.has_value() && emb_pos.has_value(), "decode_gemv: embedding mode needs idx / wpe / pos");
    TORCH_CHECK(emb_idx->is_cuda() && emb_idx->scalar_type() == torch::kInt64 && emb_idx->is_contiguous(),
                "decode_gemv: int64 token ids");
    for (const torch::Tensor* t : {&*emb_wte, &*emb_wpe})
      TORCH_CHECK(t->scalar_type() == torch::kBFloat16 && t->dim() == 2 && t->is_contiguous() && t->size(1) == K &&
                      reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "decode_gemv: bf16 contiguous wte / wpe [*, K]");
    TORCH_CHECK(emb_pos->is_cuda() && emb_pos->scalar_type() == torch::kInt64 && emb_pos->numel() == 1, "decode_gemv: int64 pos [1]");
    TORCH_CHECK(K <= 1024, "decode_gemv: LN mode needs K <= 1024");
    TORCH_CHECK(gamma.has_value() && beta.has_value() && gamma->scalar_type() == torch::kFloat32 &&
                    beta->scalar_type() == torch::kFloat32 && gamma->numel() == K && beta->numel() == K &&
                    gamma->is_contiguous() && beta->is_contiguous(), "decode_gemv: fp32 gamma / beta [K]");
    M = emb_idx->numel();
    TORCH_CHECK(rout.has_value() && rout->defined() && rout->scalar_type() == torch::kFloat32 && rout->is_contiguous() &&
                    rout->numel() == (int64_t)M * K, "decode_gemv: fp32 resid_out [M, K] for the embedding rows");
    rop = rout->data_ptr<float>();
    gp = gamma->data_ptr<float>();
    bt = beta->data_ptr<float>();
    eip = emb_idx->data_ptr<int64_t>();
    ewp = reinterpret_cast<const bf16*>(emb_wte->data_ptr());
    epp = reinterpret_cast<const bf16*>(emb_wpe->data_ptr());
    eps_p = emb_pos->data_ptr<int64_t>();
    eV = (int)emb_wte->size(0);
    eP = (int)emb_wpe->size(0);
  } else {
    TORCH_CHECK(rin.has_value() && rin->defined() && rin->scalar_type() == torch::kFloat32 && rin->dim() == 2 &&
                    rin->is_contiguous() && rin->size(1) == K, "decode_gemv: fp32 contiguous resid_in [M, K]");
    TORCH_CHECK(K <= 1024, "decode_gemv: LN mode needs K <= 1024");
    TORCH_CHECK(gamma.has_value() && beta.has_value() && gamma->scalar_type() == torch::kFloat32 &&
                    beta->scalar_type() == torch::kFloat32 && gamma->numel() == K && beta->numel() == K &&
                    gamma->is_contiguous() && beta->is_contiguous(), "decode_gemv: fp32 gamma / beta [K]");
    M = rin->size(0);
    rp = rin->data_ptr<float>();
    gp = gamma->data_ptr<float>();
    bt = beta->data_ptr<float>();
    if (delta.has_value() && delta->defined()) {
      TORCH_CHECK(delta->scalar_type() == torch::kBFloat16 && delta->is_contiguous() && delta->numel() == (int64_t)M * K,
                  "decode_gemv: bf16 contiguous delta [M, K]");
      TORCH_CHECK(rout.has_value() && rout->defined() && rout->scalar_type() == torch::kFloat32 &&
                      rout->is_contiguous() && rout->numel() == (int64_t)M * K && rout->data_ptr() != rin->data_ptr(),
                  "decode_gemv: fp32 resid_out [M, K] (not aliasing resid_in) with a delta");
      dp = reinterpret_cast<const bf16*>(delta->data_ptr());
      rop = rout->data_ptr<float>();
      if (dbias.has_value() && dbias->defined()) {
        TORCH_CHECK(dbias->scalar_type() == torch::kFloat32 && dbias->is_contiguous() && dbias->numel() == K,
                    "decode_gemv: fp32 dbias [K]");
        dbp = dbias->data_ptr<float>();
      }
    }
  }
  TORCH_CHECK(M >= 1 && M <= 4, "decode_gemv: 1..4 rows");
  TORCH_CHECK(out.scalar_type() == torch::kBFloat16 && out.dim() == 2 && out.size(0) == M && out.size(1) == N &&
                  out.stride(1) == 1, "decode_gemv: bf16 out [M, N]");
  const bf16* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->scalar_type() == torch::kBFloat16 && bias->is_contiguous() && bias->numel() == N,
                "decode_gemv: bf16 bias [N]");
    bp = reinterpret_cast<const bf16*>(bias->data_ptr());
  }
  const int cpl = (K / 8 + 31) / 32;
  int rpw = (int)rows_per_wave;
  // by shape: the vocabulary projection wants fewer, longer-lived waves (8 rows); everything else
  // 2 rows per wave — the most workgroups in flight. In the replayed step that beat 4 rows for the
  // wider QKV / fc outputs, which the isolated microbench preferred (GPT-2 B = 1 0.3594 / 0.3608 ->
  // 0.3563 / 0.3547 ms, Gemma-3 1B neutral; profiles/decode_r5.md). PENROZ_DECODE_GEMV_RPW forces 2 /
  // 4 / 8 below 16k rows (A/B).
  static const int rpw_env = [] {
    const char* e = std::getenv("PENROZ_DECODE_GEMV_RPW");
    return e ? std::atoi(e) : 0;
  }();
  if (rpw <= 0 && rpw_env > 0 && N < 16384) rpw = rpw_env;
  if (rpw <= 0) rpw = N >= 16384 ? 8 : 2;
  TORCH_CHECK(rpw == 2 || rpw == 4 || rpw == 8, "decode_gemv: rows_per_wave 2, 4 or 8");
  const int RPv = rpw / 2;
  // wave-per-row form for the bf16-x GEMVs (proj, fc2, Gemma o / down): one row per wave, the
  // whole wave striding over K — twice the workgroups. Same box: Gemma-3 1B B = 1 1.2626 / 1.2621 ->
  // 1.2577 / 1.2555 ms, GPT-2 B = 4 0.549 / 0.544 -> 0.544 / 0.542, GPT-2 B = 1 even
  // (profiles/decode_r5.md). PENROZ_DECODE_GEMV_WAVE_ROW=0: the half-wave form.
  static const bool wave_row_env = [] {
    const char* e = std::getenv("PENROZ_DECODE_GEMV_WAVE_ROW");
    return !(e && e[0] == '0');
  }();
  const bool wave_row = wave_row_env && !ln && rows_per_wave <= 0 && N < 16384;
  const int cpl64 = (K / 8 + 63) / 64;
  const dim3 grid(wave_row ? N : (N + rpw - 1) / rpw);
  auto stream = at::hip::getCurrentHIPStream();
  auto wp = reinterpret_cast<const bf16*>(w.data_ptr());
  auto op = reinterpret_cast<bf16*>(out.data_ptr());
  const int64_t o_rs = out.stride(0);
  auto launch = [&](auto mt, auto lnt, auto rpt, auto cplt) {
    constexpr int MM = decltype(mt)::value, RR = decltype(rpt)::value, CC = decltype(cplt)::value;
    constexpr int LL = decltype(lnt)::value ? 1 : 0;
    hipLaunchKernelGGL((decode_gemv_kernel<MM, LL, RR, CC>), grid, dim3(64), 0, stream, rp, dp, dbp, rop, gp, bt,
                       (float)eps, xp, x_rs, wp, bp, op, o_rs, N, K, (int)act, 0, 0, (const float*)nullptr,
                       (const float*)nullptr, eip, ewp, epp, eps_p, eV, eP);
  };
  auto by_cpl = [&](auto mt, auto lnt, auto rpt) {
    using I = std::integral_constant<int, 0>;
    (void)sizeof(I);
    if (cpl <= 1) launch(mt, lnt, rpt, std::integral_constant<int, 1>{});
    else if (cpl <= 2) launch(mt, lnt, rpt, std::integral_constant<int, 2>{});
    else if (cpl <= 3) launch(mt, lnt, rpt, std::integral_constant<int, 3>{});
    else if (cpl <= 4) launch(mt, lnt, rpt, std::integral_constant<int, 4>{});
    else if (cpl <= 5) launch(mt, lnt, rpt, std::integral_constant<int, 5>{});
    else if (cpl <= 7) launch(mt, lnt, rpt, std::integral_constant<int, 7>{});
    else if (cpl <= 12) launch(mt, lnt, rpt, std::integral_constant<int, 12>{});
    else if (cpl <= 16) launch(mt, lnt, rpt, std::integral_constant<int, 16>{});
    else if (cpl <= 25) launch(mt, lnt, rpt, std::integral_constant<int, 25>{});
    else launch(mt, lnt, rpt, std::integral_constant<int, 32>{});
  };
  auto by_rp = [&](auto mt, auto lnt) {
    if (RPv == 1) by_cpl(mt, lnt, std::integral_constant<int, 1>{});
    else if (RPv == 2) by_cpl(mt, lnt, std::integral_constant<int, 2>{});
    else by_cpl(mt, lnt, std::integral_constant<int, 4>{});
  };
  auto by_ln = [&](auto mt) {
    if (wave_row) {  // one row per wave (RP = 1), chunks per lane over 64 lanes
      auto go = [&](auto cplt) {
        constexpr int MM = decltype(mt)::value, CC = decltype(cplt)::value;
        hipLaunchKernelGGL((decode_gemv_kernel<MM, 0, 1, CC, 3>), grid, dim3(64), 0, stream, rp, dp, dbp, rop, gp, bt,
                           (float)eps, xp, x_rs, wp, bp, op, o_rs, N, K, (int)act);
      };
      if (cpl64 <= 2) go(std::integral_constant<int, 2>{});
      else if (cpl64 <= 4) go(std::integral_constant<int, 4>{});
      else if (cpl64 <= 7) go(std::integral_constant<int, 7>{});
      else if (cpl64 <= 16) go(std::integral_constant<int, 16>{});
      else go(std::integral_constant<int, 16>{});  // K <= 8192 (checked above)
      return;
    }
    if (ln) {
      TORCH_CHECK(cpl <= 4, "decode_gemv: LN mode needs K <= 1024");
      // LN mode instantiates only the small chunk counts (K <= 1024)
      if (RPv == 1) {
        if (cpl <= 3) launch(mt, std::true_type{}, std::integral_constant<int, 1>{}, std::integral_constant<int, 3>{});
        else launch(mt, std::true_type{}, std::integral_constant<int, 1>{}, std::integral_constant<int, 4>{});
      } else if (RPv == 2) {
        if (cpl <= 3) launch(mt, std::true_type{}, std::integral_constant<int, 2>{}, std::integral_constant<int, 3>{});
        else launch(mt, std::true_type{}, std::integral_constant<int, 2>{}, std::integral_constant<int, 4>{});
      } else {
        if (cpl <= 3) launch(mt, std::true_type{}, std::integral_constant<int, 4>{}, std::integral_constant<int, 3>{});
        else launch(mt, std::true_type{}, std::integral_constant<int, 4>{}, std::integral_constant<int, 4>{});
      }
    } else {
      by_rp(mt, std::false_type{});
    }
  };
  switch (M) {
    case 1: by_ln(std::integral_constant<int, 1>{}); break;
    case 2: by_ln(std::integral_constant<int, 2>{}); break;
    case 3: by_ln(std::integral_constant<int, 3>{}); break;
    default: by_ln(std::integral_constant<int, 4>{});
  }
}

// Paired-row decode GEMV for 1..4 rows on a bf16 x (decode_gemv_kernel modes 1 / 2):
//   mode 1 (gated): out[M, I] = act_f(x·Wgᵀ, kind) ⊙ (x·Wuᵀ), w = [Wg; Wu] [2I, K];
//   mode 2 (RoPE QKV): out[M, (H + 2Hkv)·D] = rope(x · Wᵀ) for the first nrot heads, cos / sin [D/2].
void decode_gemv_pair(torch::Tensor x, torch::Tensor w, torch::Tensor out, int64_t mode, int64_t kind, int64_t D,
                      int64_t nrot, c10::optional<torch::Tensor> cosv, c10::optional<torch::Tensor> sinv,
                      int64_t pairs_per_wave) {
  const int N = w.size(0), K = w.size(1);
  TORCH_CHECK(mode == 1 || mode == 2, "decode_gemv_pair: mode 1 (gated) or 2 (RoPE)");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == torch::kBFloat16 && w.dim() == 2 && w.is_contiguous() &&
                  reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0 && K % 8 == 0 && N % 2 == 0,
              "decode_gemv_pair: bf16 contiguous 16-B aligned W [N, K], K % 8 == 0, N even");
  TORCH_CHECK(x.scalar_type() == torch::kBFloat16 && x.dim() == 2 && x.size(1) == K && x.stride(1) == 1 &&
                  x.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "decode_gemv_pair: bf16 x [M, K], rows 16-B aligned");
  const int M = x.size(0);
  TORCH_CHECK(M >= 1 && M <= 4, "decode_gemv_pair: 1..4 rows");
  const int cpl = (K / 8 + 31) / 32;
  TORCH_CHECK(cpl <= 7, "decode_gemv_pair: K <= 1792");
  const int Nout = mode == 1 ? N / 2 : N;
  TORCH_CHECK(out.scalar_type() == torch::kBFloat16 && out.dim() == 2 && out.size(0) == M && out.size(1) == Nout &&
                  out.stride(1) == 1, "decode_gemv_pair: bf16 out [M, N/2] (gated) or [M, N] (RoPE)");
  const float *cp = nullptr, *sp = nullptr;
  if (mode == 1) {
    TORCH_CHECK(kind >= 0 && kind <= 2, "decode_gemv_pair: kind 0 gelu, 1 gelu_tanh, 2 silu");
  } else if (mode == 2) {
    TORCH_CHECK(D >= 2 && D % 2 == 0 && N % D == 0 && nrot >= 0 && nrot <= N / D, "decode_gemv_pair: RoPE geometry");
    TORCH_CHECK(cosv.has_value() && sinv.has_value() && cosv->is_cuda() && sinv->is_cuda() &&
                    cosv->scalar_type() == torch::kFloat32 && sinv->scalar_type() == torch::kFloat32 &&
                    cosv->numel() >= D / 2 && sinv->numel() >= D / 2 && cosv->is_contiguous() && sinv->is_contiguous(),
                "decode_gemv_pair: fp32 cos / sin [D/2]");
    cp = cosv->data_ptr<float>();
    sp = sinv->data_ptr<float>();
  }
  int ppw = (int)pairs_per_wave;
  if (ppw <= 0) ppw = N / 2 >= 16384 ? 4 : N / 2 <= 1024 ? 1 : 2;
  TORCH_CHECK(ppw == 1 || ppw == 2 || ppw == 4, "decode_gemv_pair: pairs_per_wave 1, 2 or 4");
  const dim3 grid((N / 2 + ppw - 1) / ppw);
  auto stream = at::hip::getCurrentHIPStream();
  auto xp = reinterpret_cast<const bf16*>(x.data_ptr());
  auto wp = reinterpret_cast<const bf16*>(w.data_ptr());
  auto op = reinterpret_cast<bf16*>(out.data_ptr());
  const int64_t x_rs = x.stride(0), o_rs = out.stride(0);
  auto launch = [&](auto mt, auto rpt, auto cplt, auto et) {
    constexpr int MM = decltype(mt)::value, RR = decltype(rpt)::value, CC = decltype(cplt)::value;
    constexpr int EE = decltype(et)::value;
    hipLaunchKernelGGL((decode_gemv_kernel<MM, 0, RR, CC, EE>), grid, dim3(64), 0, stream, nullptr, nullptr,
                       nullptr, nullptr, nullptr, nullptr, 0.f, xp, x_rs, wp, nullptr, op, o_rs, N, K,
                       EE == 1 ? (int)kind : 0, (int)D, (int)nrot, cp, sp);
  };
  auto by_cpl = [&](auto mt, auto rpt, auto et) {
    if (cpl <= 3) launch(mt, rpt, std::integral_constant<int, 3>{}, et);
    else if (cpl <= 4) launch(mt, rpt, std::integral_constant<int, 4>{}, et);
    else if (cpl <= 5) launch(mt, rpt, std::integral_constant<int, 5>{}, et);
    else launch(mt, rpt, std::integral_constant<int, 7>{}, et);
  };
  auto by_rp = [&](auto mt, auto et) {
    if (ppw == 1) by_cpl(mt, std::integral_constant<int, 1>{}, et);
    else if (ppw == 2) by_cpl(mt, std::integral_constant<int, 2>{}, et);
    else by_cpl(mt, std::integral_constant<int, 4>{}, et);
  };
  auto by_mode = [&](auto mt) {
    if (mode == 1) by_rp(mt, std::integral_constant<int, 1>{});
    else by_rp(mt, std::integral_constant<int, 2>{});
  };
  switch (M) {
    case 1: by_mode(std::integral_constant<int, 1>{}); break;
    case 2: by_mode(std::integral_constant<int, 2>{}); break;
    case 3: by_mode(std::integral_constant<int, 3>{}); break;
    default: by_mode(std::integral_constant<int, 4>{});
  }
}
