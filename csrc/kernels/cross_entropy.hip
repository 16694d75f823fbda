// Fused cross-entropy forward + backward over bf16 logits, gradient written in place.
//
// One 1024-thread workgroup (16 waves) per row. The row (V bf16, e.g. 50304 × 2 B = 98 KiB)
// is read ONCE into registers — 8 elements (16 B) per chunk, CPT chunks per thread, chunk k of
// thread t covers elements 8·(t + 1024·k) — i.e. 56 fp32 VGPRs per lane at GPT-2's
// vocabulary. The register file (512 KiB/CU) holds two rows per CU at once, more than LDS
// (160 KiB) could. max → Σexp → log-sum-exp are block reductions; the loss needs only the
// target logit; the gradient (softmax − onehot)·scale is rounded to bf16 and stored over the
// logits, so the lm_head backward GEMM reads it directly: one HBM read + one write per row,
// no fp32 logits (the reference's autocast CE materialises fp32 log-softmax of [B·T, V]).
// Rows with target == ignore_index contribute 0 loss and 0 gradient.
// Any V: rows live at a row stride ld (a multiple of 8, ≥ V rounded up to 8 — the executor pads
// the logits buffer, e.g. HF GPT-2's V = 50257 → ld 50264), so every 16-B chunk stays inside its
// row's allocation; elements at or past V count as −∞ logits and get a zero gradient.
#include "common.h"
#include <type_traits>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <cstdlib>

namespace penroz {

constexpr int kCEThreads = 1024;

__device__ __forceinline__ float block_reduce(float v, float* sh, bool is_max) {
  v = is_max ? wave_max(v) : wave_sum(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  float r = lane < (kCEThreads / 64) ? sh[lane] : (is_max ? -INFINITY : 0.f);
  r = is_max ? wave_max(r) : wave_sum(r);
  return r;
}

// NT: non-temporal row loads and gradient stores (PENROZ_CE_NT, see cross_entropy_fwd_bwd)
template <int CPT, typename T, bool NT = false>
__global__ void __launch_bounds__(kCEThreads) ce_kernel(T* __restrict__ logits, const int64_t* __restrict__ targets,
                                                        float* __restrict__ loss, int V, int ld, float scale,
                                                        int64_t ignore_index, T* __restrict__ gout) {
  __shared__ float sh[16];
  const int row = blockIdx.x;
  T* rp = logits + (size_t)row * ld;
  T* gp = gout ? gout + (size_t)row * ld : rp;  // gradient destination (in place by default)
  const int64_t tgt = targets[row];
  PZ_DEVICE_CHECK(tgt == ignore_index || (tgt >= 0 && tgt < V));
  const int t = threadIdx.x;
  if constexpr (std::is_same<T, bf16>::value) {
    // bf16 rows stay PACKED in registers (CPT × 4 VGPRs instead of CPT × 8 fp32): at GPT-2's
    // vocabulary (CPT = 7) the fp32 copy took the kernel to 76 VGPRs — 6 waves per SIMD, ONE
    // 16-wave workgroup (one row) per CU, so each row's load, two block reductions and store ran
    // back to back with the CU's memory pipe idle in between. Packed, two rows share a CU. The
    // exponentials are recomputed in the gradient pass (VALU is idle in this HBM-bound kernel).
    uint4 u[CPT];
    float m = -INFINITY;
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int c = 8 * (t + kCEThreads * k);
      u[k] = uint4{0xff80ff80u, 0xff80ff80u, 0xff80ff80u, 0xff80ff80u};  // bf16 -inf pairs
      if (c < V) {
        if constexpr (NT) {
          const u32x4_t r = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(rp + c));
          u[k] = uint4{r.x, r.y, r.z, r.w};
        } else {
          u[k] = *reinterpret_cast<const uint4*>(rp + c);
        }
        if (c + 8 > V) {  // the row's last, partial chunk: elements past V become -inf
          uint32_t w[4] = {u[k].x, u[k].y, u[k].z, u[k].w};
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (c + j >= V) w[j >> 1] = (j & 1) ? (w[j >> 1] & 0x0000ffffu) | 0xff800000u : (w[j >> 1] & 0xffff0000u) | 0xff80u;
          u[k] = uint4{w[0], w[1], w[2], w[3]};
        }
      }
      const uint32_t w[4] = {u[k].x, u[k].y, u[k].z, u[k].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) m = fmaxf(m, fmaxf(__uint_as_float(w[q] << 16), __uint_as_float(w[q] & 0xffff0000u)));
    }
    // the packed words are made opaque before each later pass: left alone, hipcc keeps the unpacked
    // fp32 values of the max pass alive for the other two (common subexpressions) — 78 VGPRs again
    auto opaque = [&]() {
#pragma unroll
      for (int k = 0; k < CPT; ++k) asm volatile("" : "+v"(u[k].x), "+v"(u[k].y), "+v"(u[k].z), "+v"(u[k].w));
    };
    m = block_reduce(m, sh, true);
    opaque();
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const uint32_t w[4] = {u[k].x, u[k].y, u[k].z, u[k].w};
#pragma unroll
      for (int q = 0; q < 4; ++q)
        s += __expf(__uint_as_float(w[q] << 16) - m) + __expf(__uint_as_float(w[q] & 0xffff0000u) - m);
    }
    s = block_reduce(s, sh, false);
    const float lse = m + __logf(s);
    const bool valid = tgt != ignore_index && tgt >= 0 && tgt < V;
    if (t == 0) loss[row] = valid ? lse - to_f(rp[tgt]) : 0.f;
    if (scale == 0.f) return;
    const float sc = valid ? scale : 0.f;
    const float ps = sc / s;
    __syncthreads();  // the target logit is read before any thread overwrites it
    opaque();
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int c = 8 * (t + kCEThreads * k);
      if (c < V) {
        const uint32_t w[4] = {u[k].x, u[k].y, u[k].z, u[k].w};
        float g[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          g[2 * q] = fmaf(__expf(__uint_as_float(w[q] << 16) - m), ps, c + 2 * q == tgt ? -sc : 0.f);
          g[2 * q + 1] = fmaf(__expf(__uint_as_float(w[q] & 0xffff0000u) - m), ps, c + 2 * q + 1 == tgt ? -sc : 0.f);
        }
        store8<NT>(gp + c, g);
      }
    }
    return;
  }
  float v[CPT][8];
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    const int c = 8 * (t + kCEThreads * k);
    if (c < V) {
      load8<NT>(rp + c, v[k]);
      if (c + 8 > V) {  // the row's last, partial chunk
#pragma unroll
        for (int j = 0; j < 8; ++j) v[k][j] = c + j < V ? v[k][j] : -INFINITY;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) m = fmaxf(m, v[k][j]);
    }
  }
  m = block_reduce(m, sh, true);
  // v becomes exp(v - m) in the sum pass, so the gradient pass needs no second exponential:
  // softmax = exp(v - m) / Σ
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    const int c = 8 * (t + kCEThreads * k);
    if (c < V) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[k][j] = __expf(v[k][j] - m);
        s += v[k][j];
      }
    }
  }
  s = block_reduce(s, sh, false);
  const float lse = m + __logf(s);
  const bool valid = tgt != ignore_index && tgt >= 0 && tgt < V;
  if (t == 0) loss[row] = valid ? lse - to_f(rp[tgt]) : 0.f;
  if (scale == 0.f) return;
  const float sc = valid ? scale : 0.f;
  const float ps = sc / s;
  __syncthreads();  // the target logit is read before any thread overwrites it
#pragma unroll
  for (int k = 0; k < CPT; ++k) {
    const int c = 8 * (t + kCEThreads * k);
    if (c < V) {
      float g[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = fmaf(v[k][j], ps, c + j == tgt ? -sc : 0.f);
      store8<NT>(gp + c, g);
    }
  }
}

// Wide-V fallback (more than 8 chunks per thread): three streamed passes through L2.
template <typename T, bool NT = false>
__global__ void __launch_bounds__(kCEThreads) ce_loop_kernel(T* __restrict__ logits,
                                                             const int64_t* __restrict__ targets,
                                                             float* __restrict__ loss, int V, int ld, float scale,
                                                             int64_t ignore_index, T* __restrict__ gout) {
  __shared__ float sh[16];
  const int row = blockIdx.x;
  T* rp = logits + (size_t)row * ld;
  T* gp = gout ? gout + (size_t)row * ld : rp;
  const int64_t tgt = targets[row];
  PZ_DEVICE_CHECK(tgt == ignore_index || (tgt >= 0 && tgt < V));
  // one pass for max and sum (online: the running sum is rescaled when the running max grows),
  // so the row is read twice in all (here and for the gradient) instead of three times —
  // Gemma's 262k-token rows are 512 KB each, beyond what the L2 keeps between passes
  float m = -INFINITY, s = 0.f;
  for (int c = 8 * threadIdx.x; c < V; c += 8 * kCEThreads) {
    float v[8];
    Vec8<T>::load(rp + c, v);
    float cm = -INFINITY;
#pragma unroll
    for (int j = 0; j < 8; ++j) cm = fmaxf(cm, c + j < V ? v[j] : -INFINITY);
    if (cm > m) {
      s *= __expf(m - cm);  // m = -inf: s is 0 and stays 0
      m = cm;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += c + j < V ? __expf(v[j] - m) : 0.f;
  }
  const float mb = block_reduce(m, sh, true);
  s = block_reduce(m == -INFINITY ? 0.f : s * __expf(m - mb), sh, false);
  m = mb;
  const float lse = m + __logf(s);
  const bool valid = tgt != ignore_index && tgt >= 0 && tgt < V;
  if (threadIdx.x == 0) loss[row] = valid ? lse - to_f(rp[tgt]) : 0.f;
  if (scale == 0.f) return;
  const float sc = valid ? scale : 0.f;
  __syncthreads();
  for (int c = 8 * threadIdx.x; c < V; c += 8 * kCEThreads) {
    float v[8];
    Vec8<T>::load(rp + c, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = c + j < V ? (__expf(v[j] - lse) - (c + j == tgt ? 1.f : 0.f)) * sc : 0.f;
    store8<NT>(gp + c, v);  // (the first pass keeps plain loads: the second reads the row again)
  }
}

}  // namespace penroz

using namespace penroz;

// grad_out (optional, same shape / row stride / dtype as logits): the gradient goes there and the
// logits stay intact (autograd callers); default: in place over the logits.
torch::Tensor cross_entropy_fwd_bwd(torch::Tensor logits, torch::Tensor targets, double scale, int64_t ignore_index,
                                    c10::optional<torch::Tensor> grad_out) {
  TORCH_CHECK(logits.is_cuda() && logits.dim() == 2 && logits.stride(1) == 1, "logits: [N, V] with unit column stride");
  TORCH_CHECK(targets.scalar_type() == torch::kInt64 && targets.numel() == logits.size(0));
  const int N = logits.size(0), V = logits.size(1);
  const int ld = N > 1 ? (int)logits.stride(0) : ((V + 7) & ~7);
  TORCH_CHECK(ld % 8 == 0 && ld >= ((V + 7) & ~7) && reinterpret_cast<uintptr_t>(logits.data_ptr()) % 16 == 0,
              "logits rows must start 16-B aligned with a row stride that is a multiple of 8 and >= V rounded up to "
              "8 (pad the buffer: [N, ld][:, :V])");
  // every row's 16-B chunks (the last one padded up to 8 elements) must be allocated — N == 1
  // included, where the row stride says nothing about the padding
  TORCH_CHECK(logits.storage().nbytes() >= (size_t)(logits.storage_offset() + (int64_t)(N > 0 ? N - 1 : 0) * ld +
                                                    ((V + 7) & ~7)) * logits.element_size(),
              "logits: the last row's padding must be allocated (pad the buffer: [N, ld][:, :V])");
  auto loss = torch::empty({N}, logits.options().dtype(torch::kFloat32));
  if (N == 0) return loss;
  auto tg = targets.contiguous();
  void* gptr = nullptr;
  if (grad_out.has_value() && grad_out->defined()) {
    TORCH_CHECK(grad_out->is_cuda() && grad_out->scalar_type() == logits.scalar_type() &&
                    grad_out->sizes() == logits.sizes() && grad_out->strides() == logits.strides() &&
                    reinterpret_cast<uintptr_t>(grad_out->data_ptr()) % 16 == 0,
                "grad_out must match the logits' shape, strides and dtype (16-B aligned)");
    gptr = grad_out->data_ptr();
  }
  auto stream = at::hip::getCurrentHIPStream();
  const int chunks = ((V + 7) / 8 + kCEThreads - 1) / kCEThreads;
  const char* ne = std::getenv("PENROZ_CE_NT");
  const bool nt = ne && *ne ? std::atoi(ne) != 0 : true;  // default on: GPT-2 64.52 / 64.82 -> 64.44 / 64.51 ms, Gemma neutral (profiles/ew_ab_r4.log)
  auto launch = [&](auto tag) {
    using T = decltype(tag);
    T* lp = reinterpret_cast<T*>(logits.data_ptr());
    const int64_t* tp = tg.data_ptr<int64_t>();
    float* op = loss.data_ptr<float>();
    const float sc = (float)scale;
    T* gp = reinterpret_cast<T*>(gptr);
    auto go = [&](auto nt_tag) {
      constexpr bool NT = decltype(nt_tag)::value;
      switch (chunks) {
#define PZ_CE_CASE(K) \
        case K: hipLaunchKernelGGL((ce_kernel<K, T, NT>), dim3(N), dim3(kCEThreads), 0, stream, lp, tp, op, V, ld, sc, ignore_index, gp); break;
        PZ_CE_CASE(1) PZ_CE_CASE(2) PZ_CE_CASE(3) PZ_CE_CASE(4) PZ_CE_CASE(5) PZ_CE_CASE(6) PZ_CE_CASE(7) PZ_CE_CASE(8)
#undef PZ_CE_CASE
        default: hipLaunchKernelGGL((ce_loop_kernel<T, NT>), dim3(N), dim3(kCEThreads), 0, stream, lp, tp, op, V, ld, sc, ignore_index, gp);
      }
    };
    if (nt) go(std::true_type{});
    else go(std::false_type{});
  };
  if (logits.scalar_type() == torch::kBFloat16) launch(bf16{});
  else if (logits.scalar_type() == torch::kFloat32) launch(float{});
  else if (logits.scalar_type() == torch::kFloat16) launch(__half{});
  else TORCH_CHECK(false, "unsupported logits dtype");
  return loss;
}
