// Next-token selection, one 1024-thread workgroup per row of logits [B, V]:
//   temperature == 0  -> argmax (first index on ties, like torch.argmax);
//   top_k > 0         -> radix-select the k-th largest (4 × 8-bit passes, LDS histograms) and
//                        keep logits >= it;
//   then softmax of (logit / T) over the kept set and an inverse-CDF draw with the row's
//   uniform u: thread-major order (thread t owns elements t, t+1024, …), one block scan of
//   the per-thread sums finds the owning thread, which walks its own elements.
// The whole decision stays on the device (no sort, no host round trip per token).
#include "common.h"
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

namespace penroz {

constexpr int kST = 1024;

__device__ __forceinline__ uint32_t order_key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

template <typename T>
__global__ void __launch_bounds__(kST) sample_kernel(const T* __restrict__ logits, const float* __restrict__ uni,
                                                     int64_t* __restrict__ out, int V, float temperature, int top_k) {
  __shared__ float fred[kST / 64];
  __shared__ int ired[kST / 64];
  __shared__ uint32_t hist[256];
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
    if (t == 0) out[row] = result;
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
      for (int i = t; i < V; i += kST) {
        const uint32_t k = order_key(to_f(lp[i]));
        if ((k & msk) == pre) atomicAdd(&hist[(k >> shift) & 255u], 1u);
      }
      __syncthreads();
      if (t == 0) {
        int kk = sel_k;
        int d = 255;
        for (; d > 0; --d) {
          if ((int)hist[d] >= kk) break;
          kk -= hist[d];
        }
        sel_k = kk;
        sel_prefix = pre | ((uint32_t)d << shift);
        sel_mask = msk | (255u << shift);
      }
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
  const float target = uni[row] * total;
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
  if (t == 0) out[row] = result;
}

}  // namespace penroz

using namespace penroz;

torch::Tensor sample_tokens(torch::Tensor logits, c10::optional<torch::Tensor> uniform, double temperature,
                            int64_t top_k) {
  TORCH_CHECK(logits.is_cuda() && logits.is_contiguous() && logits.dim() == 2);
  const int B = logits.size(0), V = logits.size(1);
  auto out = torch::empty({B, 1}, logits.options().dtype(torch::kInt64));
  torch::Tensor u;
  if (uniform.has_value() && uniform->defined()) u = uniform->to(torch::kFloat32).contiguous();
  else u = torch::zeros({B}, logits.options().dtype(torch::kFloat32));
  TORCH_CHECK(u.numel() == B && u.is_cuda());
  auto stream = at::hip::getCurrentHIPStream();
  if (logits.scalar_type() == torch::kBFloat16)
    hipLaunchKernelGGL(sample_kernel<bf16>, dim3(B), dim3(kST), 0, stream,
                       reinterpret_cast<const bf16*>(logits.data_ptr()), u.data_ptr<float>(), out.data_ptr<int64_t>(),
                       V, (float)temperature, (int)top_k);
  else if (logits.scalar_type() == torch::kFloat32)
    hipLaunchKernelGGL(sample_kernel<float>, dim3(B), dim3(kST), 0, stream, logits.data_ptr<float>(),
                       u.data_ptr<float>(), out.data_ptr<int64_t>(), V, (float)temperature, (int)top_k);
  else if (logits.scalar_type() == torch::kFloat16)
    hipLaunchKernelGGL(sample_kernel<__half>, dim3(B), dim3(kST), 0, stream,
                       reinterpret_cast<const __half*>(logits.data_ptr()), u.data_ptr<float>(),
                       out.data_ptr<int64_t>(), V, (float)temperature, (int)top_k);
  else TORCH_CHECK(false, "unsupported logits dtype");
  return out;
}
