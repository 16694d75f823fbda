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

// grid = ceil(M/16) * ceil(N/64), block 256. LDS: 16 normalised rows [16][K + 8] bf16.
__global__ void __launch_bounds__(256) decode_ln_gemm_kernel(const float* __restrict__ resid,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, float eps,
                                                             const bf16* __restrict__ w, const bf16* __restrict__ bias,
                                                             bf16* __restrict__ out, int64_t o_rs, int M, int N, int K,
                                                             int act, int flags) {
  __shared__ __attribute__((aligned(16))) bf16 xs[16 * (1024 + 8)];
  const int LDX = K + 8;  // +16 B per row: a fragment's 16 row reads spread over the banks
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  int rb, ct;
  dl_tile(blockIdx.x, (M + 15) / 16, (N + 63) / 64, rb, ct);
  const int steps = K / 32;
  const int r16 = lane & 15, kq = 8 * (lane >> 4);
  const int n0 = ct * 64 + wid * 16;  // this wave's column block
  const bool live = n0 < N;

  // 1. the wave's weight fragments for the whole K range, in flight during the prologue
  dl_u32x4 wa[kDlMaxSteps];
  {
    const bf16* wp = w + (size_t)min(n0 + r16, N - 1) * K + kq;
#pragma unroll
    for (int s = 0; s < kDlMaxSteps; ++s)
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
  if (!live) return;
  if (flags & 2) {
#pragma unroll
    for (int s = 0; s < kDlMaxSteps; ++s) wa[s] = dl_u32x4{0u, 0u, 0u, 0u};
  }

  // 3. MFMA over the full K, x fragments from LDS
  dl_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const bf16* xl = xs + r16 * LDX + kq;
#pragma unroll
  for (int s = 0; s < kDlMaxSteps; ++s) {
    if (s < steps && !(flags & 16)) {
      const dl_u32x4 xb = *reinterpret_cast<const dl_u32x4*>(xl + s * 32);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(dl_bf16x8, wa[s]),
                                                    __builtin_bit_cast(dl_bf16x8, xb), acc, 0, 0, 0);
    }
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
  const int grid = ((M + 15) / 16) * ((N + 63) / 64);
  hipLaunchKernelGGL(decode_ln_gemm_kernel, dim3(grid), dim3(256), 0, at::hip::getCurrentHIPStream(),
                     resid.data_ptr<float>(), gamma.data_ptr<float>(), beta.data_ptr<float>(), (float)eps,
                     reinterpret_cast<const bf16*>(w.data_ptr()), bp, reinterpret_cast<bf16*>(out.data_ptr()),
                     (int64_t)out.stride(0), M, N, K, (int)act, (int)flags);
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
