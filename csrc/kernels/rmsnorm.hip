// RMSNorm forward/backward (Gemma path).  y = round_x((x·rstd)) · w, rstd = rsqrt(mean(x²)+eps)
// in fp32 — the reference's exact rounding order (``neural_net_layers.py:151-155``); output
// dtype = promote(x, w). One wave per row (any width % 4), 4 rows per workgroup; dγ partials
// accumulate per workgroup in LDS and are finished by a column reduction (no global atomics).
#include "common.h"
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

namespace penroz {

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

template <typename TX, typename TW, typename TDY>
__global__ void __launch_bounds__(256) rms_bwd_kernel(const TDY* __restrict__ dy, const TX* __restrict__ x,
                                                      const TW* __restrict__ w, const float* __restrict__ rstd,
                                                      TX* __restrict__ dx, float* __restrict__ part, int N, int C) {
  extern __shared__ __attribute__((aligned(16))) float dwl[];
  for (int c = threadIdx.x; c < C; c += blockDim.x) dwl[c] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int row = blockIdx.x * 4 + wid; row < N; row += gridDim.x * 4) {
    const size_t base = (size_t)row * C;
    const float r = rstd[row];
    float dot = 0.f;
    for (int c = lane; c < C; c += 64) {
      const float xv = to_f(x[base + c]);
      const float g = to_f(dy[base + c]);
      dot += g * to_f(w[c]) * xv;
      atomicAdd(&dwl[c], g * to_f(from_f<TX>(xv * r)));
    }
    dot = wave_sum(dot) / C;
    for (int c = lane; c < C; c += 64) {
      const float xv = to_f(x[base + c]);
      const float g = to_f(dy[base + c]) * to_f(w[c]);
      dx[base + c] = from_f<TX>(r * g - xv * r * r * r * dot);
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) part[(size_t)blockIdx.x * C + c] = dwl[c];
}

__global__ void __launch_bounds__(256) rms_finish_kernel(const float* __restrict__ part, int G, int C,
                                                         float* __restrict__ out) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int g = 0; g < G; ++g) s += part[(size_t)g * C + c];
  out[c] = s;
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
  TORCH_CHECK((size_t)C * 4 <= 160 * 1024, "RMSNorm width too large for the LDS dγ accumulator");
  auto dx = torch::empty_like(x);
  const int G = std::max(1, std::min((N + 3) / 4, 512));
  auto part = torch::empty({G, C}, x.options().dtype(torch::kFloat32));
  auto dw = torch::empty({C}, x.options().dtype(torch::kFloat32));
  auto wc = w.contiguous();
  auto stream = at::hip::getCurrentHIPStream();
  if (N == 0) return {dx, dw.zero_()};
  RMS_TYPES(x.scalar_type(), TX, RMS_TYPES(w.scalar_type(), TW, RMS_TYPES(dy.scalar_type(), TDY,
    hipLaunchKernelGGL((rms_bwd_kernel<TX, TW, TDY>), dim3(G), dim3(256), C * sizeof(float), stream,
                       reinterpret_cast<const TDY*>(dy.data_ptr()), reinterpret_cast<const TX*>(x.data_ptr()),
                       reinterpret_cast<const TW*>(wc.data_ptr()), rstd.data_ptr<float>(),
                       reinterpret_cast<TX*>(dx.data_ptr()), part.data_ptr<float>(), N, C))))
  hipLaunchKernelGGL(rms_finish_kernel, dim3((C + 255) / 256), dim3(256), 0, stream, part.data_ptr<float>(), G, C,
                     dw.data_ptr<float>());
  return {dx, dw};
}
