// RMSNorm forward/backward (Gemma path).  y = round_x((x·rstd)) · w, rstd = rsqrt(mean(x²)+eps)
// in fp32 — the reference's exact rounding order (``neural_net_layers.py:151-155``); output
// dtype = promote(x, w). One wave per row (any width % 4), 4 rows per workgroup; dγ partials
// accumulate per workgroup in LDS and are finished by a column reduction (no global atomics).
#include "common.h"
#include "reduce.h"
#include <type_traits>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

namespace penroz {

constexpr int RMS_BWD_MAX_C = 10240;  // rms_bwd_wide_kernel: 4 waves x C fp32 partials in LDS (160 KiB)

template <typename TX, typename TW, typename TY>
__global__ void __launch_bounds__(256) rms_fwd_kernel(const TX* __restrict__ x, const TW* __restrict__ w,
                                                      TY* __restrict__ y, float* __restrict__ rstd_out, int N, int C,
                                                      float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= N) return;
  const TX* xr = x + (size_t)row * C;
  float ss = 0.f;
  for (int c = lane; c < C; c += 64) {
    const float v = to_f(xr[c]);
    ss += v * v;
  }
  const float r = rsqrtf(wave_sum(ss) / C + eps);
  for (int c = lane; c < C; c += 64) {
    const float n = to_f(from_f<TX>(to_f(xr[c]) * r));  // (x*norm).to(x.dtype)
    y[(size_t)row * C + c] = from_f<TY>(n * to_f(w[c]));
  }
  if (lane == 0) rstd_out[row] = r;
}

// One wave per row; lane l owns columns l + 64·k (k < NPL), so each row's x / dy stay in registers
// between the two passes and the dγ partial sums accumulate in registers across the wave's rows
// (no LDS atomics); the 4 waves' partials are combined through LDS into one row of `part`.
template <int NPL, typename TX, typename TW, typename TDY>
__global__ void __launch_bounds__(256) rms_bwd_kernel(const TDY* __restrict__ dy, const TX* __restrict__ x,
                                                      const TW* __restrict__ w, const float* __restrict__ rstd,
                                                      TX* __restrict__ dx, float* __restrict__ part, int N, int C) {
  extern __shared__ __attribute__((aligned(16))) float dwl[];  // [4 waves][C]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float wv[NPL], dwa[NPL];
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    const int c = lane + 64 * k;
    wv[k] = c < C ? to_f(w[c]) : 0.f;
    dwa[k] = 0.f;
  }
  for (int row = blockIdx.x * 4 + wid; row < N; row += gridDim.x * 4) {
    const size_t base = (size_t)row * C;
    const float r = rstd[row];
    float xv[NPL], gv[NPL];
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int c = lane + 64 * k;
      xv[k] = c < C ? to_f(x[base + c]) : 0.f;
      gv[k] = c < C ? to_f(dy[base + c]) : 0.f;
    }
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      dot += gv[k] * wv[k] * xv[k];
      dwa[k] += gv[k] * to_f(from_f<TX>(xv[k] * r));
    }
    dot = wave_sum(dot) / C;
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int c = lane + 64 * k;
      if (c < C) dx[base + c] = from_f<TX>(r * gv[k] * wv[k] - xv[k] * r * r * r * dot);
    }
  }
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    const int c = lane + 64 * k;
    if (c < C) dwl[wid * C + c] = dwa[k];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x)
    part[(size_t)blockIdx.x * C + c] = dwl[c] + dwl[C + c] + dwl[2 * C + c] + dwl[3 * C + c];
}

// Widths past the register-resident kernel (C > 2048: Gemma-3 4B 2560, 12B 3840, 27B 5376): one
// wave per row in two lane-strided (coalesced) passes over the row (dot, then dx); each wave's dγ partials live in its own LDS row [C] (no atomics), combined per
// workgroup exactly like rms_bwd_kernel. LDS = 16·C bytes, so C ≤ 10240.
template <typename TX, typename TW, typename TDY>
__global__ void __launch_bounds__(256) rms_bwd_wide_kernel(const TDY* __restrict__ dy, const TX* __restrict__ x,
                                                           const TW* __restrict__ w, const float* __restrict__ rstd,
                                                           TX* __restrict__ dx, float* __restrict__ part, int N, int C) {
  extern __shared__ __attribute__((aligned(16))) float dwl[];  // [4 waves][C]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float* my = dwl + wid * C;
  for (int c = lane; c < C; c += 64) my[c] = 0.f;
  for (int row = blockIdx.x * 4 + wid; row < N; row += gridDim.x * 4) {
    const size_t base = (size_t)row * C;
    const float r = rstd[row];
    float dot = 0.f;
    for (int c = lane; c < C; c += 64) dot += to_f(dy[base + c]) * to_f(w[c]) * to_f(x[base + c]);
    dot = wave_sum(dot) / C;
    for (int c = lane; c < C; c += 64) {
      const float xv = to_f(x[base + c]), gv = to_f(dy[base + c]);
      my[c] += gv * to_f(from_f<TX>(xv * r));  // each lane owns its columns: no race
      dx[base + c] = from_f<TX>(r * gv * to_f(w[c]) - xv * r * r * r * dot);
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x)
    part[(size_t)blockIdx.x * C + c] = dwl[c] + dwl[C + c] + dwl[2 * C + c] + dwl[3 * C + c];
}



// Decode-step fusion for Gemma blocks: residual add + post-norm + the next norm in one pass.
// The row lives in registers (one wave per row, NV 8-value vectors per lane). Every intermediate is
// rounded to T where the module path rounds (torch adds / RMSNorm output), so the result equals
// the module sequence  h = post(x, a); y = rms(h) * w2:
//   mode 0: h = rms(x + a) * w1        (Gemma 3+: post norm on the residual sum)
//   mode 1: h = x + rms(a) * w1        (Gemma 2: post norm on the branch output)
//   mode 2: h = x + a                  (Gemma 1: no post norms)
// y is skipped when w2 is null (h alone: the last block feeds the final norm separately).
template <int NV, typename T>
__global__ void __launch_bounds__(256) rms_residual_kernel(const T* __restrict__ x, const T* __restrict__ a,
                                                           const T* __restrict__ w1, const T* __restrict__ w2,
                                                           T* __restrict__ h, T* __restrict__ y, int N, int C,
                                                           int mode, float eps1, float eps2) {
  // lane owns 8-value vectors j = lane + 64 i (i < NV). Every load is issued before any use
  // (out-of-range vectors re-read the row's last one and are masked), so a row costs one memory
  // round trip instead of one per element.
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= N) return;
  const int nvec = C / 8;
  const T* xr = x + (size_t)row * C;
  const T* ar = a + (size_t)row * C;
  float xv[NV][8], v[NV][8];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int j = min(lane + 64 * i, nvec - 1);
    Vec8<T>::load(ar + 8 * j, v[i]);
    Vec8<T>::load(xr + 8 * j, xv[i]);
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const bool ok = lane + 64 * i < nvec;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (mode == 0) v[i][e] = to_f(from_f<T>(xv[i][e] + v[i][e]));  // torch's rounded add
      else if (mode == 2) v[i][e] = to_f(from_f<T>(xv[i][e] + v[i][e]));
      if (mode != 2 && ok) ss += v[i][e] * v[i][e];
    }
  }
  if (mode != 2) {
    const float r = rsqrtf(wave_sum(ss) / C + eps1);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      float wv[8];
      Vec8<T>::load(w1 + 8 * min(lane + 64 * i, nvec - 1), wv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float n = to_f(from_f<T>(to_f(from_f<T>(v[i][e] * r)) * wv[e]));
        v[i][e] = mode == 0 ? n : to_f(from_f<T>(xv[i][e] + n));
      }
    }
  }
  ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int j = lane + 64 * i;
    if (j < nvec) {
      Vec8<T>::store(h + (size_t)row * C + 8 * j, v[i]);
#pragma unroll
      for (int e = 0; e < 8; ++e) ss += v[i][e] * v[i][e];
    }
  }
  if (w2 == nullptr) return;
  const float r2 = rsqrtf(wave_sum(ss) / C + eps2);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int j = lane + 64 * i;
    float wv[8];
    Vec8<T>::load(w2 + 8 * min(j, nvec - 1), wv);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[i][e] = to_f(from_f<T>(v[i][e] * r2)) * wv[e];
    if (j < nvec) Vec8<T>::store(y + (size_t)row * C + 8 * j, v[i]);
  }
}

}  // namespace penroz

using namespace penroz;

#define RMS_TYPES(t, NAME, ...)                                                     \
  if ((t) == torch::kFloat32) { using NAME = float; __VA_ARGS__; }                  \
  else if ((t) == torch::kBFloat16) { using NAME = bf16; __VA_ARGS__; }             \
  else if ((t) == torch::kFloat16) { using NAME = __half; __VA_ARGS__; }            \
  else TORCH_CHECK(false, "unsupported dtype");

std::vector<torch::Tensor> rmsnorm_fwd(torch::Tensor x, torch::Tensor w, double eps) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.dim() == 2 && w.numel() == x.size(1));
  const int N = x.size(0), C = x.size(1);
  auto out_t = at::promote_types(x.scalar_type(), w.scalar_type());
  auto y = torch::empty({N, C}, x.options().dtype(out_t));
  auto rstd = torch::empty({N}, x.options().dtype(torch::kFloat32));
  if (N == 0) return {y, rstd};
  auto wc = w.contiguous();
  auto stream = at::hip::getCurrentHIPStream();
  RMS_TYPES(x.scalar_type(), TX, RMS_TYPES(w.scalar_type(), TW, RMS_TYPES(out_t, TY,
    hipLaunchKernelGGL((rms_fwd_kernel<TX, TW, TY>), dim3((N + 3) / 4), dim3(256), 0, stream,
                       reinterpret_cast<const TX*>(x.data_ptr()), reinterpret_cast<const TW*>(wc.data_ptr()),
                       reinterpret_cast<TY*>(y.data_ptr()), rstd.data_ptr<float>(), N, C, (float)eps))))
  return {y, rstd};
}

std::vector<torch::Tensor> rmsnorm_bwd(torch::Tensor dy, torch::Tensor x, torch::Tensor w, torch::Tensor rstd) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && dy.is_contiguous() && dy.numel() == x.numel());
  const int N = x.size(0), C = x.size(1);
  TORCH_CHECK(C <= RMS_BWD_MAX_C, "RMSNorm backward: width <= ", RMS_BWD_MAX_C);
  auto dx = torch::empty_like(x);
  const int G = std::max(1, std::min((N + 3) / 4, 2048));
  auto part = torch::empty({G, C}, x.options().dtype(torch::kFloat32));
  auto dw = torch::zeros({C}, x.options().dtype(torch::kFloat32));
  auto wc = w.contiguous();
  auto stream = at::hip::getCurrentHIPStream();
  if (N == 0) return {dx, dw};
  auto launch = [&](auto npl) {
    constexpr int NPL = decltype(npl)::value;
    RMS_TYPES(x.scalar_type(), TX, RMS_TYPES(w.scalar_type(), TW, RMS_TYPES(dy.scalar_type(), TDY,
      hipLaunchKernelGGL((rms_bwd_kernel<NPL, TX, TW, TDY>), dim3(G), dim3(256), 4 * C * sizeof(float), stream,
                         reinterpret_cast<const TDY*>(dy.data_ptr()), reinterpret_cast<const TX*>(x.data_ptr()),
                         reinterpret_cast<const TW*>(wc.data_ptr()), rstd.data_ptr<float>(),
                         reinterpret_cast<TX*>(dx.data_ptr()), part.data_ptr<float>(), N, C))))
  };
  const int npl = (C + 63) / 64;
  if (npl <= 4) launch(std::integral_constant<int, 4>{});
  else if (npl <= 8) launch(std::integral_constant<int, 8>{});
  else if (npl <= 18) launch(std::integral_constant<int, 18>{});
  else if (npl <= 32) launch(std::integral_constant<int, 32>{});
  else {
    RMS_TYPES(x.scalar_type(), TX, RMS_TYPES(w.scalar_type(), TW, RMS_TYPES(dy.scalar_type(), TDY,
      auto kern = rms_bwd_wide_kernel<TX, TW, TDY>;
      hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                          4 * C * (int)sizeof(float));
      hipLaunchKernelGGL(kern, dim3(G), dim3(256), 4 * C * sizeof(float), stream,
                         reinterpret_cast<const TDY*>(dy.data_ptr()), reinterpret_cast<const TX*>(x.data_ptr()),
                         reinterpret_cast<const TW*>(wc.data_ptr()), rstd.data_ptr<float>(),
                         reinterpret_cast<TX*>(dx.data_ptr()), part.data_ptr<float>(), N, C))))
  }
  // dγ = Σ of the G partial rows: the sliced two-stage column reduction (reduce.h), on the CURRENT
  // stream — dw goes straight back to autograd, so it must not be finished on the executor's
  // deferred side stream (nothing would order the caller's reads after it)
  const int S = reduce_slices(G);
  auto mid = torch::empty({1, S, C}, part.options());
  float* outs[1] = {dw.data_ptr<float>()};
  reduce_partials_add(part.data_ptr<float>(), 1, G, C, outs, mid.data_ptr<float>(), S, stream);
  return {dx, dw};
}

// x, a: [N, C] (same dtype as w1 / w2); returns {h, y} (y undefined when w2 is absent)
std::vector<torch::Tensor> rms_residual(torch::Tensor x, torch::Tensor a, c10::optional<torch::Tensor> w1,
                                        c10::optional<torch::Tensor> w2, int64_t mode, double eps1, double eps2) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && a.is_contiguous() && x.dim() == 2 && a.sizes() == x.sizes() &&
              a.scalar_type() == x.scalar_type(), "x, a: [N, C] contiguous, same dtype");
  TORCH_CHECK(mode >= 0 && mode <= 2 && (mode == 2 || (w1.has_value() && w1->defined())), "rms_residual mode");
  const int N = x.size(0), C = x.size(1);
  for (auto* w : {&w1, &w2})
    if (w->has_value() && (*w)->defined())
      TORCH_CHECK((*w)->is_contiguous() && (*w)->numel() == C && (*w)->scalar_type() == x.scalar_type(), "norm weight");
  TORCH_CHECK(C % 8 == 0 && C <= 64 * 8 * 12, "rms_residual: width % 8 == 0, <= 6144");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0,
              "rms_residual: 16-B aligned rows");
  auto h = torch::empty_like(x);
  const bool has_y = w2.has_value() && w2->defined();
  torch::Tensor y = has_y ? torch::empty_like(x) : torch::Tensor();
  if (N == 0) return {h, y};
  auto stream = at::hip::getCurrentHIPStream();
  const int nv = (C / 8 + 63) / 64;  // 8-value vectors per lane
  auto launch = [&](auto tag) {
    using T = decltype(tag);
    const T* w1p = mode != 2 ? reinterpret_cast<const T*>(w1->data_ptr()) : nullptr;
    const T* w2p = has_y ? reinterpret_cast<const T*>(w2->data_ptr()) : nullptr;
    T* yp = has_y ? reinterpret_cast<T*>(y.data_ptr()) : nullptr;
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3((N + 3) / 4), dim3(256), 0, stream, reinterpret_cast<const T*>(x.data_ptr()),
                         reinterpret_cast<const T*>(a.data_ptr()), w1p, w2p, reinterpret_cast<T*>(h.data_ptr()), yp, N,
                         C, (int)mode, (float)eps1, (float)eps2);
    };
    if (nv <= 1) go(rms_residual_kernel<1, T>);
    else if (nv <= 2) go(rms_residual_kernel<2, T>);
    else if (nv <= 3) go(rms_residual_kernel<3, T>);
    else if (nv <= 4) go(rms_residual_kernel<4, T>);
    else if (nv <= 6) go(rms_residual_kernel<6, T>);
    else if (nv <= 8) go(rms_residual_kernel<8, T>);
    else go(rms_residual_kernel<12, T>);
  };
  RMS_TYPES(x.scalar_type(), T, launch(T{}))
  return {h, y};
}
