// LayerNorm forward / fused residual-add + LayerNorm forward / fused LayerNorm backward.
//
// Layout: one 64-lane wave per row, 4 rows per 256-thread workgroup. Each lane owns NCH
// chunks of 4 contiguous elements (chunk j of lane l starts at 4*(l + 64*j)), so every
// global access is a 16-B (fp32) or 8-B (bf16) per-lane vector and a wave instruction
// covers 1 KiB / 512 B contiguous. The row stays in registers between the statistics and
// the output pass (one HBM read, one write). Statistics are fp32 (two-pass mean/variance
// on the register copy — no E[x²]−E[x]² cancellation).
//
// Backward: dx = rstd·(w·dy − mean(w·dy) − x̂·mean(w·dy·x̂)); the residual gradient is
// accumulated in place (fp32), optionally mirrored as bf16 for the next dgrad GEMM, and the
// per-column partial sums dγ = Σ dy·x̂, dβ = Σ dy and (optionally) Σ dresid — the bias
// gradient of the linear that fed this residual — are reduced per workgroup in LDS and
// finished by a small column-reduction kernel (deterministic, no atomics).
//
// Residual dropout (HF GPT-2 resid_pdrop): the fused forward adds drop(delta) =
// delta·mask/(1-p) to the stream; the backward keeps the fp32 residual gradient unmasked and
// applies the regenerated mask to the branch gradient it hands on (the bf16 copy for the
// producing linear's dgrad and that linear's bias-gradient column sum).
#include "common.h"
#include "deferred.h"
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

namespace penroz {

template <typename T> struct V4;
template <> struct V4<float> {
  __device__ __forceinline__ static void ld(const float* p, float (&v)[4]) {
    float4_t a = *reinterpret_cast<const float4_t*>(p);
    v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
  }
  __device__ __forceinline__ static void st(float* p, const float (&v)[4]) {
    *reinterpret_cast<float4_t*>(p) = float4_t{v[0], v[1], v[2], v[3]};
  }
};
template <> struct V4<bf16> {
  __device__ __forceinline__ static void ld(const bf16* p, float (&v)[4]) {
    uint2 u = *reinterpret_cast<const uint2*>(p);
    v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
    v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
  }
  __device__ __forceinline__ static void st(bf16* p, const float (&v)[4]) {
    uint2 u;
    u.x = pack_bf16x2(v[0], v[1]);
    u.y = pack_bf16x2(v[2], v[3]);
    *reinterpret_cast<uint2*>(p) = u;
  }
};
template <> struct V4<__half> {
  __device__ __forceinline__ static void ld(const __half* p, float (&v)[4]) {
    uint2 u = *reinterpret_cast<const uint2*>(p);
    const __half2* h = reinterpret_cast<const __half2*>(&u);
    float2 a = __half22float2(h[0]), b = __half22float2(h[1]);
    v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
  }
  __device__ __forceinline__ static void st(__half* p, const float (&v)[4]) {
    uint2 u;
    __half2* h = reinterpret_cast<__half2*>(&u);
    h[0] = __floats2half2_rn(v[0], v[1]);
    h[1] = __floats2half2_rn(v[2], v[3]);
    *reinterpret_cast<uint2*>(p) = u;
  }
};

constexpr int kRowsPerBlock = 4;

// ------------------------------------------------------------------------------------------
// forward: y = LN(x [+ delta]); optional resid_out = x + delta (fp32)
template <int NCH, typename TX, typename TD, typename TY, bool ADD>
__global__ void __launch_bounds__(256) ln_fwd_kernel(const TX* __restrict__ x, const TD* __restrict__ delta, const float* __restrict__ dbias,
                                                     float* __restrict__ resid_out, const float* __restrict__ w,
                                                     const float* __restrict__ b, TY* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int N, int C, float eps, uint64_t dseed, float dp) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= N) return;
  const size_t base = (size_t)row * C;
  const float dinv = dp > 0.f ? 1.f / (1.f - dp) : 1.f;
  float v[NCH][4];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int c = 4 * (lane + 64 * j);
    if (c >= C) { v[j][0] = v[j][1] = v[j][2] = v[j][3] = 0.f; continue; }
    V4<TX>::ld(x + base + c, v[j]);
    if constexpr (ADD) {
      float d[4];
      V4<TD>::ld(delta + base + c, d);
      if (dbias) {  // the producing linear's bias, folded in here (decode program)
        float e[4];
        V4<float>::ld(dbias + c, e);
#pragma unroll
        for (int k = 0; k < 4; ++k) d[k] += e[k];
      }
      if (dp > 0.f) {
#pragma unroll
        for (int k = 0; k < 4; ++k) d[k] *= dropout_mult(dseed, base + c + k, dp, dinv);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) v[j][k] += d[k];
      V4<float>::st(resid_out + base + c, v[j]);
    }
    s += v[j][0] + v[j][1] + v[j][2] + v[j][3];
  }
  const float mean = wave_sum(s) / C;
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < NCH; ++j)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float d = v[j][k] - mean;
      ss += 4 * (lane + 64 * j) < C ? d * d : 0.f;
    }
  const float rstd = rsqrtf(wave_sum(ss) / C + eps);
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int c = 4 * (lane + 64 * j);
    if (c >= C) continue;
    float wv[4], bv[4], o[4];
    V4<float>::ld(w + c, wv);
    V4<float>::ld(b + c, bv);
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = (v[j][k] - mean) * rstd * wv[k] + bv[k];
    V4<TY>::st(y + base + c, o);
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// Generic-width fallback (C % 4 == 0): loops over the row twice through L2.
template <typename TX, typename TD, typename TY, bool ADD>
__global__ void __launch_bounds__(256) ln_fwd_loop_kernel(const TX* __restrict__ x, const TD* __restrict__ delta, const float* __restrict__ dbias,
                                                          float* __restrict__ resid_out, const float* __restrict__ w,
                                                          const float* __restrict__ b, TY* __restrict__ y,
                                                          float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                          int N, int C, float eps, uint64_t dseed, float dp) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= N) return;
  const size_t base = (size_t)row * C;
  const float dinv = dp > 0.f ? 1.f / (1.f - dp) : 1.f;
  float s = 0.f;
  for (int c = 4 * lane; c < C; c += 256) {
    float v[4];
    V4<TX>::ld(x + base + c, v);
    if constexpr (ADD) {
      float d[4];
      V4<TD>::ld(delta + base + c, d);
      if (dbias) {
        float e[4];
        V4<float>::ld(dbias + c, e);
#pragma unroll
        for (int k = 0; k < 4; ++k) d[k] += e[k];
      }
      if (dp > 0.f) {
#pragma unroll
        for (int k = 0; k < 4; ++k) d[k] *= dropout_mult(dseed, base + c + k, dp, dinv);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] += d[k];
      V4<float>::st(resid_out + base + c, v);
    }
    s += v[0] + v[1] + v[2] + v[3];
  }
  const float mean = wave_sum(s) / C;
  float ss = 0.f;
  for (int c = 4 * lane; c < C; c += 256) {
    float v[4];
    if constexpr (ADD) V4<float>::ld(resid_out + base + c, v); else V4<TX>::ld(x + base + c, v);
#pragma unroll
    for (int k = 0; k < 4; ++k) ss += (v[k] - mean) * (v[k] - mean);
  }
  const float rstd = rsqrtf(wave_sum(ss) / C + eps);
  for (int c = 4 * lane; c < C; c += 256) {
    float v[4], wv[4], bv[4], o[4];
    if constexpr (ADD) V4<float>::ld(resid_out + base + c, v); else V4<TX>::ld(x + base + c, v);
    V4<float>::ld(w + c, wv);
    V4<float>::ld(b + c, bv);
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = (v[k] - mean) * rstd * wv[k] + bv[k];
    V4<TY>::st(y + base + c, o);
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// ------------------------------------------------------------------------------------------
// backward
template <int NCH, typename TDY, typename TX>
__global__ void __launch_bounds__(256) ln_bwd_kernel(const TDY* __restrict__ dy, const TX* __restrict__ x,
                                                     const float* __restrict__ mean_in,
                                                     const float* __restrict__ rstd_in,
                                                     const float* __restrict__ w, float* __restrict__ dresid,
                                                     bf16* __restrict__ dresid_bf, float* __restrict__ part,
                                                     int N, int C, int accumulate, int want_bias, uint64_t dseed,
                                                     float dp) {
  const float dinv = dp > 0.f ? 1.f / (1.f - dp) : 1.f;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  float pw[NCH][4], pb[NCH][4], pz[NCH][4];
  float wv[NCH][4];
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    if (4 * (lane + 64 * j) < C) V4<float>::ld(w + 4 * (lane + 64 * j), wv[j]);
    else wv[j][0] = wv[j][1] = wv[j][2] = wv[j][3] = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) pw[j][k] = pb[j][k] = pz[j][k] = 0.f;
  }
  const int nwaves = gridDim.x * kRowsPerBlock;
  for (int row = blockIdx.x * kRowsPerBlock + wid; row < N; row += nwaves) {
    const size_t base = (size_t)row * C;
    const float mean = mean_in[row], rstd = rstd_in[row];
    float g[NCH][4], xh[NCH][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const int c = 4 * (lane + 64 * j);
      float xv[4];
      if (c < C) {
        V4<TDY>::ld(dy + base + c, g[j]);
        V4<TX>::ld(x + base + c, xv);
      } else {
        g[j][0] = g[j][1] = g[j][2] = g[j][3] = 0.f;
        xv[0] = xv[1] = xv[2] = xv[3] = mean;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        xh[j][k] = (xv[k] - mean) * rstd;
        const float wdy = g[j][k] * wv[j][k];
        s1 += wdy;
        s2 += wdy * xh[j][k];
        pw[j][k] += g[j][k] * xh[j][k];
        pb[j][k] += g[j][k];
      }
    }
    const float c1 = wave_sum(s1) / C, c2 = wave_sum(s2) / C;
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const int c = 4 * (lane + 64 * j);
      if (c >= C) continue;
      float r[4];
      if (accumulate) V4<float>::ld(dresid + base + c, r);
      else r[0] = r[1] = r[2] = r[3] = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) r[k] += (g[j][k] * wv[j][k] - c1 - xh[j][k] * c2) * rstd;
      V4<float>::st(dresid + base + c, r);
      if (dp > 0.f) {  // branch gradient = mask ⊙ residual gradient / (1-p)
#pragma unroll
        for (int k = 0; k < 4; ++k) r[k] *= dropout_mult(dseed, base + c + k, dp, dinv);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) pz[j][k] += r[k];
      if (dresid_bf != nullptr) V4<bf16>::st(dresid_bf + base + c, r);
    }
  }
  // block-level reduction of the three partial vectors through LDS, one array at a time
  const int nparts = want_bias ? 3 : 2;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    if (a >= nparts) break;
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const int c = 4 * (lane + 64 * j);
      if (c < C) V4<float>::st(lds + wid * C + c, a == 0 ? pw[j] : (a == 1 ? pb[j] : pz[j]));
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      float t = lds[c] + lds[C + c] + lds[2 * C + c] + lds[3 * C + c];
      part[((size_t)a * gridDim.x + blockIdx.x) * C + c] = t;
    }
    __syncthreads();
  }
}

}  // namespace penroz

// ============================================================================ host side
using namespace penroz;

#define DISPATCH_NCH(C, ...)                                   \
  switch (nch_pick(C)) {                                       \
    case 1: { constexpr int NCH = 1; __VA_ARGS__; break; }     \
    case 2: { constexpr int NCH = 2; __VA_ARGS__; break; }     \
    case 3: { constexpr int NCH = 3; __VA_ARGS__; break; }     \
    case 4: { constexpr int NCH = 4; __VA_ARGS__; break; }     \
    case 5: { constexpr int NCH = 5; __VA_ARGS__; break; }     \
    case 6: { constexpr int NCH = 6; __VA_ARGS__; break; }     \
    case 7: { constexpr int NCH = 7; __VA_ARGS__; break; }     \
    case 8: { constexpr int NCH = 8; __VA_ARGS__; break; }     \
    case 10: { constexpr int NCH = 10; __VA_ARGS__; break; }   \
    case 12: { constexpr int NCH = 12; __VA_ARGS__; break; }   \
    case 16: { constexpr int NCH = 16; __VA_ARGS__; break; }   \
    default: TORCH_CHECK(false, "unsupported width ", C);      \
  }

// register-resident row widths: ceil(C/256) chunks per lane rounded up to {1..8, 10, 12, 16}
static int nch_pick(int C) {
  if (C % 4 || C <= 0) return 0;
  int n = (C + 255) / 256;
  if (n <= 8) return n;
  if (n <= 10) return 10;
  if (n <= 12) return 12;
  if (n <= 16) return 16;
  return 0;
}
static bool nch_ok(int C) { return nch_pick(C) != 0; }

template <typename TX, typename TD, typename TY, bool ADD>
static void launch_fwd(const torch::Tensor& x, const torch::Tensor* delta, torch::Tensor* resid_out,
                       const torch::Tensor& w, const torch::Tensor& b, torch::Tensor& y, torch::Tensor& mean,
                       torch::Tensor& rstd, double eps, const float* dbias = nullptr, uint64_t dseed = 0,
                       float drop_p = 0.f) {
  const int N = x.size(0), C = x.size(1);
  if (N == 0) return;
  dim3 grid((N + kRowsPerBlock - 1) / kRowsPerBlock), block(256);
  auto stream = at::hip::getCurrentHIPStream();
  const TX* xp = reinterpret_cast<const TX*>(x.data_ptr());
  const TD* dp = delta ? reinterpret_cast<const TD*>(delta->data_ptr()) : nullptr;
  float* rp = resid_out ? resid_out->data_ptr<float>() : nullptr;
  TY* yp = reinterpret_cast<TY*>(y.data_ptr());
  if (nch_ok(C)) {
    DISPATCH_NCH(C, hipLaunchKernelGGL((ln_fwd_kernel<NCH, TX, TD, TY, ADD>), grid, block, 0, stream, xp, dp, dbias, rp,
                                       w.data_ptr<float>(), b.data_ptr<float>(), yp, mean.data_ptr<float>(),
                                       rstd.data_ptr<float>(), N, C, (float)eps, dseed, drop_p));
  } else {
    hipLaunchKernelGGL((ln_fwd_loop_kernel<TX, TD, TY, ADD>), grid, block, 0, stream, xp, dp, dbias, rp, w.data_ptr<float>(),
                       b.data_ptr<float>(), yp, mean.data_ptr<float>(), rstd.data_ptr<float>(), N, C, (float)eps,
                       dseed, drop_p);
  }
}

#define FOR_FLOAT_TYPES(t, NAME, ...)                                               \
  if ((t) == torch::kFloat32) { using NAME = float; __VA_ARGS__; }                  \
  else if ((t) == torch::kBFloat16) { using NAME = bf16; __VA_ARGS__; }             \
  else if ((t) == torch::kFloat16) { using NAME = __half; __VA_ARGS__; }            \
  else TORCH_CHECK(false, "unsupported dtype");

static void check_rows(const torch::Tensor& t, int64_t N, int64_t C, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), name, " must be a contiguous GPU tensor");
  TORCH_CHECK(t.dim() == 2 && t.size(0) == N && t.size(1) == C, name, " shape mismatch");
}

void layernorm_fwd(torch::Tensor x, torch::Tensor w, torch::Tensor b, double eps, torch::Tensor y,
                   torch::Tensor mean, torch::Tensor rstd) {
  const int64_t N = x.size(0), C = x.size(1);
  check_rows(x, N, C, "x");
  check_rows(y, N, C, "y");
  TORCH_CHECK(C % 4 == 0, "LayerNorm width must be a multiple of 4");
  TORCH_CHECK(w.scalar_type() == torch::kFloat32 && b.scalar_type() == torch::kFloat32 && w.numel() == C && b.numel() == C);
  TORCH_CHECK(mean.numel() == N && rstd.numel() == N);
  FOR_FLOAT_TYPES(x.scalar_type(), TX,
    FOR_FLOAT_TYPES(y.scalar_type(), TY, launch_fwd<TX, float, TY, false>(x, nullptr, nullptr, w, b, y, mean, rstd, eps)))
}

void add_layernorm_fwd(torch::Tensor resid_in, torch::Tensor delta, torch::Tensor resid_out, torch::Tensor w,
                       torch::Tensor b, double eps, torch::Tensor y, torch::Tensor mean, torch::Tensor rstd,
                       c10::optional<torch::Tensor> delta_bias, double dropout_p, int64_t dropout_seed) {
  TORCH_CHECK(dropout_p >= 0.0 && dropout_p < 1.0, "dropout p must be in [0, 1)");
  const int64_t N = resid_in.size(0), C = resid_in.size(1);
  check_rows(resid_in, N, C, "resid_in");
  check_rows(delta, N, C, "delta");
  check_rows(resid_out, N, C, "resid_out");
  check_rows(y, N, C, "y");
  TORCH_CHECK(resid_out.scalar_type() == torch::kFloat32, "residual stream must be fp32");
  TORCH_CHECK(w.numel() == C && b.numel() == C && mean.numel() == N && rstd.numel() == N);
  const float* dbp = nullptr;
  if (delta_bias.has_value() && delta_bias->defined()) {  // resid_out = resid_in + delta + delta_bias
    TORCH_CHECK(delta_bias->scalar_type() == torch::kFloat32 && delta_bias->is_contiguous() && delta_bias->numel() == C,
                "delta_bias must be fp32 [C]");
    dbp = delta_bias->data_ptr<float>();
  }
  FOR_FLOAT_TYPES(resid_in.scalar_type(), TX,
    FOR_FLOAT_TYPES(delta.scalar_type(), TD,
      FOR_FLOAT_TYPES(y.scalar_type(), TY,
        launch_fwd<TX, TD, TY, true>(resid_in, &delta, &resid_out, w, b, y, mean, rstd, eps, dbp,
                                     (uint64_t)dropout_seed, (float)dropout_p))))
}

void layernorm_bwd(torch::Tensor dy, torch::Tensor x, torch::Tensor mean, torch::Tensor rstd, torch::Tensor w,
                   torch::Tensor dresid, bool accumulate, c10::optional<torch::Tensor> dresid_bf,
                   torch::Tensor dw, torch::Tensor db, c10::optional<torch::Tensor> dbias_prev, double dropout_p,
                   int64_t dropout_seed) {
  TORCH_CHECK(dropout_p >= 0.0 && dropout_p < 1.0, "dropout p must be in [0, 1)");
  const int64_t N = x.size(0), C = x.size(1);
  check_rows(dy, N, C, "dy");
  check_rows(x, N, C, "x");
  check_rows(dresid, N, C, "dresid");
  TORCH_CHECK(dresid.scalar_type() == torch::kFloat32 && w.scalar_type() == torch::kFloat32);
  TORCH_CHECK(dw.scalar_type() == torch::kFloat32 && db.scalar_type() == torch::kFloat32 && dw.numel() == C && db.numel() == C);
  TORCH_CHECK(nch_ok(C), "LayerNorm backward supports widths %4 == 0 up to 4096 (ceil(C/256) in {1..8,10,12,16}), got ", C);
  bf16* dbf = nullptr;
  if (dresid_bf.has_value() && dresid_bf->defined()) {
    check_rows(*dresid_bf, N, C, "dresid_bf");
    TORCH_CHECK(dresid_bf->scalar_type() == torch::kBFloat16);
    dbf = reinterpret_cast<bf16*>(dresid_bf->data_ptr());
  }
  const bool want_bias = dbias_prev.has_value() && dbias_prev->defined();
  if (N == 0) return;
  int grid = (int)std::min<int64_t>((N + kRowsPerBlock - 1) / kRowsPerBlock, 1024);
  auto part = torch::empty({3, grid, C}, x.options().dtype(torch::kFloat32));
  auto stream = at::hip::getCurrentHIPStream();
  const size_t lds = sizeof(float) * kRowsPerBlock * C;
  FOR_FLOAT_TYPES(dy.scalar_type(), TDY,
    FOR_FLOAT_TYPES(x.scalar_type(), TX,
      DISPATCH_NCH(C, hipLaunchKernelGGL((ln_bwd_kernel<NCH, TDY, TX>), dim3(grid), dim3(256), lds, stream,
                                         reinterpret_cast<const TDY*>(dy.data_ptr()),
                                         reinterpret_cast<const TX*>(x.data_ptr()), mean.data_ptr<float>(),
                                         rstd.data_ptr<float>(), w.data_ptr<float>(), dresid.data_ptr<float>(), dbf,
                                         part.data_ptr<float>(), (int)N, (int)C, accumulate ? 1 : 0,
                                         want_bias ? 1 : 0, (uint64_t)dropout_seed, (float)dropout_p))))
  const int A = want_bias ? 3 : 2;
  float* outs[3] = {dw.data_ptr<float>(), db.data_ptr<float>(), want_bias ? dbias_prev->data_ptr<float>() : nullptr};
  reduce_partials_auto(part, A, grid, (int)C, outs, stream);
}
