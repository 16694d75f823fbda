// Fused Adam / AdamW steps.
//
// flat: one grid-stride launch over contiguous fp32 (param, grad, exp_avg, exp_avg_sq) buffers
//       with 16-B vectors; optionally rewrites the bf16 shadow copy the GEMMs read, so the
//       master update and the low-precision refresh cost one pass (≈30 B/param of traffic).
// multi-tensor: one launch over a device chunk table (tensor, offset) for parameter lists
//       that are not flat (generic models); fp32, or bf16 parameters with bf16 state (what
//       torch.optim keeps for them) updated in fp32 registers.
// Math = torch.optim.AdamW / Adam single-tensor path: decoupled decay p *= 1 − lr·wd (AdamW)
// or g += wd·p (Adam); m = lerp(m, g, 1 − β1); v = β2·v + (1 − β2)·g²;
// p −= (lr / bc1) · m / (sqrt(v) / sqrt(bc2) + eps). Bias corrections come from the host in
// double precision. ``grad_scale`` multiplies the gradient first (micro-step averaging).
#include "common.h"
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <cstdlib>

namespace penroz {

struct AdamHyper {
  float lr, b1, b2, eps, wd, step_size, inv_bc2_sqrt, grad_scale;
  int maximize, decoupled;
};

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, const AdamHyper& h) {
  g *= h.grad_scale;
  if (h.maximize) g = -g;
  if (h.decoupled) p *= 1.f - h.lr * h.wd;
  else g += h.wd * p;
  m += (g - m) * (1.f - h.b1);
  v = h.b2 * v + (1.f - h.b2) * g * g;
  const float denom = sqrtf(v) * h.inv_bc2_sqrt + h.eps;
  p -= h.step_size * m / denom;
}

// NT: 0 plain, 1 non-temporal loads and stores (default), 2 non-temporal stores only; every
// operand is streamed once per step (PENROZ_ADAM_NT picks, see flat_step)
template <int NT>
__device__ __forceinline__ float4_t ld4(const float4_t* a) {
  if constexpr (NT == 1) return __builtin_nontemporal_load(a);
  else return *a;
}
template <int NT, typename V>
__device__ __forceinline__ void st(V* a, V x) {
  if constexpr (NT != 0) __builtin_nontemporal_store(x, a);
  else *a = x;
}

template <int NT>
__global__ void __launch_bounds__(256) adam_flat_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v,
                                                        bf16* __restrict__ shadow, int64_t n, AdamHyper h) {
  const int64_t n4 = n / 4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4_t pv = ld4<NT>(reinterpret_cast<float4_t*>(p) + i);
    const float4_t gv = ld4<NT>(reinterpret_cast<const float4_t*>(g) + i);
    float4_t mv = ld4<NT>(reinterpret_cast<float4_t*>(m) + i);
    float4_t vv = ld4<NT>(reinterpret_cast<float4_t*>(v) + i);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float pk = pv[k], mk = mv[k], vk = vv[k];
      adam_elem(pk, gv[k], mk, vk, h);
      pv[k] = pk; mv[k] = mk; vv[k] = vk;
    }
    st<NT>(reinterpret_cast<float4_t*>(p) + i, pv);
    st<NT>(reinterpret_cast<float4_t*>(m) + i, mv);
    st<NT>(reinterpret_cast<float4_t*>(v) + i, vv);
    if (shadow) {
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
      const u32x2 u = {pack_bf16x2(pv[0], pv[1]), pack_bf16x2(pv[2], pv[3])};
      st<NT>(reinterpret_cast<u32x2*>(shadow) + i, u);
    }
  }
  // scalar tail
  for (int64_t i = 4 * n4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float pk = p[i], mk = m[i], vk = v[i];
    adam_elem(pk, g[i], mk, vk, h);
    p[i] = pk; m[i] = mk; v[i] = vk;
    if (shadow) shadow[i] = __float2bfloat16(pk);
  }
}

// Row-split step of an embedding table [R, C] inside the flat buffers (C % 4 == 0). A step's
// gradient is zero on every row its tokens did not touch, and those rows' update (moment decay,
// weight decay) does not depend on the backward: MODE 0 updates the rows with mask[row] == 0 as
// for g = 0 (no gradient read), any time during the step; MODE 1 then updates the touched rows —
// one workgroup per token, the first of a row's tokens claims it (mask 1 -> 2, vector
// compare-and-swap) — and clears their gradient, so the table's gradient is all zero again and
// zero_grad can skip it. Bitwise the same result as the dense step (adam_elem with g = 0.0f).
template <int MODE>
__global__ void __launch_bounds__(256) adam_rows_kernel(float* __restrict__ p, float* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v,
                                                        bf16* __restrict__ shadow, int64_t R, int C,
                                                        int* __restrict__ mask, const int64_t* __restrict__ rows,
                                                        int64_t nrows, AdamHyper h) {
  const int c4 = C / 4;
  auto row_update = [&](int64_t row, int64_t j) {  // float4 j of row
    const int64_t i = row * c4 + j;
    float4_t pv = reinterpret_cast<float4_t*>(p)[i];
    float4_t mv = reinterpret_cast<float4_t*>(m)[i];
    float4_t vv = reinterpret_cast<float4_t*>(v)[i];
    float4_t gv = {0.f, 0.f, 0.f, 0.f};
    if constexpr (MODE == 1) {
      gv = reinterpret_cast<float4_t*>(g)[i];
      reinterpret_cast<float4_t*>(g)[i] = float4_t{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float pk = pv[k], mk = mv[k], vk = vv[k];
      adam_elem(pk, gv[k], mk, vk, h);
      pv[k] = pk; mv[k] = mk; vv[k] = vk;
    }
    reinterpret_cast<float4_t*>(p)[i] = pv;
    reinterpret_cast<float4_t*>(m)[i] = mv;
    reinterpret_cast<float4_t*>(v)[i] = vv;
    if (shadow) {
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
      reinterpret_cast<u32x2*>(shadow)[i] = u32x2{pack_bf16x2(pv[0], pv[1]), pack_bf16x2(pv[2], pv[3])};
    }
  };
  if constexpr (MODE == 0) {
    const int64_t n4 = R * c4;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
      const int64_t row = i / c4;
      if (mask[row] == 0) row_update(row, i - row * c4);
    }
  } else {
    __shared__ int claimed;
    for (int64_t t = blockIdx.x; t < nrows; t += gridDim.x) {
      const int64_t row = rows[t];
      if (threadIdx.x == 0) claimed = (row >= 0 && row < R) ? atomicCAS(mask + row, 1, 2) == 1 : 0;
      __syncthreads();
      if (claimed)
        for (int j = threadIdx.x; j < c4; j += blockDim.x) row_update(row, j);
      __syncthreads();
    }
  }
}

struct TensorEntry {
  void* p;
  const void* g;
  void* m;
  void* v;
  int64_t n;
};

constexpr int kChunk = 8192;

// T = float, or bf16 for bf16 parameters (torch keeps their exp_avg / exp_avg_sq in bf16 too):
// the update is computed in fp32 and each of p / m / v is rounded once on store (torch's foreach
// path rounds after every elementwise op)
template <typename T>
__global__ void __launch_bounds__(256) adam_multi_kernel(const TensorEntry* __restrict__ tab,
                                                         const int32_t* __restrict__ chunk_tensor,
                                                         const int32_t* __restrict__ chunk_index, AdamHyper h) {
  const TensorEntry e = tab[chunk_tensor[blockIdx.x]];
  T* P = static_cast<T*>(e.p);
  const T* Gp = static_cast<const T*>(e.g);
  T* M = static_cast<T*>(e.m);
  T* V = static_cast<T*>(e.v);
  const int64_t start = (int64_t)chunk_index[blockIdx.x] * kChunk;
  const int64_t end = min(e.n, start + kChunk);
  for (int64_t i = start + threadIdx.x; i < end; i += blockDim.x) {
    float pk = to_f(P[i]), mk = to_f(M[i]), vk = to_f(V[i]);
    adam_elem(pk, to_f(Gp[i]), mk, vk, h);
    P[i] = from_f<T>(pk); M[i] = from_f<T>(mk); V[i] = from_f<T>(vk);
  }
}

}  // namespace penroz

using namespace penroz;

static AdamHyper make_hyper(double lr, double b1, double b2, double eps, double wd, int64_t step, double grad_scale,
                            bool maximize, bool decoupled) {
  AdamHyper h;
  const double bc1 = 1.0 - std::pow(b1, (double)step);
  const double bc2 = 1.0 - std::pow(b2, (double)step);
  h.lr = (float)lr; h.b1 = (float)b1; h.b2 = (float)b2; h.eps = (float)eps; h.wd = (float)wd;
  h.step_size = (float)(lr / bc1);
  h.inv_bc2_sqrt = (float)(1.0 / std::sqrt(bc2));
  h.grad_scale = (float)grad_scale;
  h.maximize = maximize ? 1 : 0;
  h.decoupled = decoupled ? 1 : 0;
  return h;
}

static void flat_step(torch::Tensor p, torch::Tensor g, torch::Tensor m, torch::Tensor v,
                      c10::optional<torch::Tensor> shadow, const AdamHyper& h) {
  for (auto* t : {&p, &g, &m, &v}) {
    TORCH_CHECK(t->is_cuda() && t->is_contiguous() && t->scalar_type() == torch::kFloat32, "flat buffers must be fp32");
    TORCH_CHECK(t->numel() == p.numel(), "flat buffer sizes differ");
  }
  bf16* sp = nullptr;
  if (shadow.has_value() && shadow->defined()) {
    TORCH_CHECK(shadow->scalar_type() == torch::kBFloat16 && shadow->numel() == p.numel());
    sp = reinterpret_cast<bf16*>(shadow->data_ptr());
  }
  const int64_t n = p.numel();
  const char* ge = std::getenv("PENROZ_ADAM_GRID");
  // one float4 per thread, non-temporal loads and stores by default: 1.36x (GPT-2 124M flat size)
  // and 1.17x (Gemma-3 1B) over a 4096-workgroup grid-stride loop (profiles/ew_ab_r4.log)
  const int64_t gmax = ge && *ge ? std::max(1, std::atoi(ge)) : (int64_t)1 << 30;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((n / 4 + 255) / 256, gmax));
  const char* ne = std::getenv("PENROZ_ADAM_NT");
  const int nt = ne && *ne ? std::atoi(ne) : 1;
  auto kern = nt == 1 ? adam_flat_kernel<1> : (nt == 2 ? adam_flat_kernel<2> : adam_flat_kernel<0>);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, at::hip::getCurrentHIPStream(), p.data_ptr<float>(),
                     g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), sp, n, h);
}

void adamw_step(torch::Tensor p, torch::Tensor g, torch::Tensor m, torch::Tensor v, c10::optional<torch::Tensor> shadow,
                double lr, double b1, double b2, double eps, double wd, int64_t step, double grad_scale, bool maximize) {
  flat_step(p, g, m, v, shadow, make_hyper(lr, b1, b2, eps, wd, step, grad_scale, maximize, true));
}

void adam_step(torch::Tensor p, torch::Tensor g, torch::Tensor m, torch::Tensor v, c10::optional<torch::Tensor> shadow,
               double lr, double b1, double b2, double eps, double wd, int64_t step, double grad_scale, bool maximize) {
  flat_step(p, g, m, v, shadow, make_hyper(lr, b1, b2, eps, wd, step, grad_scale, maximize, false));
}

// mode 0: rows with mask == 0 as for a zero gradient; mode 1: the rows of `rows` whose mask is 1
// (claimed once each, mask -> 2), with their gradient, which is then cleared
void adam_rows_step(torch::Tensor p, torch::Tensor g, torch::Tensor m, torch::Tensor v, c10::optional<torch::Tensor> shadow,
                    int64_t C, torch::Tensor mask, c10::optional<torch::Tensor> rows, int64_t mode, double lr, double b1,
                    double b2, double eps, double wd, int64_t step, double grad_scale, bool maximize, bool decoupled) {
  for (auto* t : {&p, &g, &m, &v}) {
    TORCH_CHECK(t->is_cuda() && t->is_contiguous() && t->scalar_type() == torch::kFloat32, "row buffers must be fp32");
    TORCH_CHECK(t->numel() == p.numel(), "row buffer sizes differ");
  }
  TORCH_CHECK(C > 0 && C % 4 == 0 && p.numel() % C == 0, "row width must divide the range and be a multiple of 4");
  const int64_t R = p.numel() / C;
  TORCH_CHECK(mask.is_cuda() && mask.scalar_type() == torch::kInt32 && mask.numel() == R, "mask: int32 [rows]");
  bf16* sp = nullptr;
  if (shadow.has_value() && shadow->defined()) {
    TORCH_CHECK(shadow->scalar_type() == torch::kBFloat16 && shadow->numel() == p.numel());
    sp = reinterpret_cast<bf16*>(shadow->data_ptr());
  }
  for (auto* t : {&p, &g, &m, &v})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "row buffers must be 16-B aligned");
  const AdamHyper h = make_hyper(lr, b1, b2, eps, wd, step, grad_scale, maximize, decoupled);
  auto stream = at::hip::getCurrentHIPStream();
  if (mode == 0) {
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((R * (C / 4) + 255) / 256, 1 << 20));
    hipLaunchKernelGGL(adam_rows_kernel<0>, dim3(grid), dim3(256), 0, stream, p.data_ptr<float>(), g.data_ptr<float>(),
                       m.data_ptr<float>(), v.data_ptr<float>(), sp, R, (int)C, mask.data_ptr<int>(),
                       (const int64_t*)nullptr, (int64_t)0, h);
  } else {
    TORCH_CHECK(rows.has_value() && rows->is_cuda() && rows->scalar_type() == torch::kInt64 && rows->is_contiguous(),
                "mode 1 needs the token rows (int64)");
    const int64_t n = rows->numel();
    if (n == 0) return;
    const int grid = (int)std::min<int64_t>(n, 65536);
    hipLaunchKernelGGL(adam_rows_kernel<1>, dim3(grid), dim3(256), 0, stream, p.data_ptr<float>(), g.data_ptr<float>(),
                       m.data_ptr<float>(), v.data_ptr<float>(), sp, R, (int)C, mask.data_ptr<int>(),
                       rows->data_ptr<int64_t>(), n, h);
  }
}

void multi_tensor_adam(std::vector<torch::Tensor> ps, std::vector<torch::Tensor> gs, std::vector<torch::Tensor> ms,
                       std::vector<torch::Tensor> vs, double lr, double b1, double b2, double eps, double wd,
                       int64_t step, double grad_scale, bool maximize, bool decoupled) {
  const size_t nt = ps.size();
  TORCH_CHECK(gs.size() == nt && ms.size() == nt && vs.size() == nt);
  if (nt == 0) return;
  const auto dt = ps[0].scalar_type();
  TORCH_CHECK(dt == torch::kFloat32 || dt == torch::kBFloat16, "multi-tensor Adam: fp32 or bf16 tensors");
  std::vector<TensorEntry> tab(nt);
  std::vector<int32_t> ct, ci;
  for (size_t i = 0; i < nt; ++i) {
    for (auto* t : {&ps[i], &gs[i], &ms[i], &vs[i]})
      TORCH_CHECK(t->is_cuda() && t->is_contiguous() && t->scalar_type() == dt && t->numel() == ps[i].numel(),
                  "multi-tensor Adam needs contiguous tensors of one dtype (fp32 or bf16) and equal size");
    tab[i] = {ps[i].data_ptr(), gs[i].data_ptr(), ms[i].data_ptr(), vs[i].data_ptr(), ps[i].numel()};
    const int64_t chunks = (ps[i].numel() + kChunk - 1) / kChunk;
    for (int64_t c = 0; c < chunks; ++c) {
      ct.push_back((int32_t)i);
      ci.push_back((int32_t)c);
    }
  }
  if (ct.empty()) return;
  // one host->device copy of the table (pinned staging, stream ordered)
  const int64_t tab_bytes = nt * sizeof(TensorEntry);
  const int64_t nchunks = ct.size();
  auto host = torch::empty({tab_bytes + 8 * nchunks}, torch::TensorOptions().dtype(torch::kUInt8).pinned_memory(true));
  std::memcpy(host.data_ptr(), tab.data(), tab_bytes);
  std::memcpy(host.data_ptr<uint8_t>() + tab_bytes, ct.data(), 4 * nchunks);
  std::memcpy(host.data_ptr<uint8_t>() + tab_bytes + 4 * nchunks, ci.data(), 4 * nchunks);
  auto dev = host.to(ps[0].device(), /*non_blocking=*/true);
  const uint8_t* base = dev.data_ptr<uint8_t>();
  AdamHyper h = make_hyper(lr, b1, b2, eps, wd, step, grad_scale, maximize, decoupled);
  auto launch = [&](auto kernel) {
    hipLaunchKernelGGL(kernel, dim3(nchunks), dim3(256), 0, at::hip::getCurrentHIPStream(),
                       reinterpret_cast<const TensorEntry*>(base), reinterpret_cast<const int32_t*>(base + tab_bytes),
                       reinterpret_cast<const int32_t*>(base + tab_bytes + 4 * nchunks), h);
  };
  if (dt == torch::kBFloat16) launch(adam_multi_kernel<bf16>);
  else launch(adam_multi_kernel<float>);
}

// ---- weight-update diagnostics ------------------------------------------------------------------
// Per-epoch weight-update ratios of the training loop (reference neural_net_model.py:684-703:
// std(w − w_prev) / std(w) per weight matrix): one launch over a chunk table of every (w, prev)
// pair computing fp64 partial sums (Σd, Σd², Σw, Σw²) per chunk, then one launch folding each
// tensor's chunks in chunk order (deterministic) into the two unbiased standard deviations. The
// per-tensor torch formulation (sub, cast, two std reductions and a stack per weight: ~300 small
// kernels) cost ≈ 8 ms of GPU time per epoch at GPT-2 124M (profiles/notes_r6.md).
namespace penroz {
namespace {
struct MomEntry {
  const void* w;
  const void* p;
  int64_t n;
};

template <typename T>
__global__ void __launch_bounds__(256) moments_chunk_kernel(const MomEntry* __restrict__ tab,
                                                            const int32_t* __restrict__ chunk_tensor,
                                                            const int32_t* __restrict__ chunk_index,
                                                            double* __restrict__ part) {
  const MomEntry e = tab[chunk_tensor[blockIdx.x]];
  const T* W = static_cast<const T*>(e.w);
  const T* P = static_cast<const T*>(e.p);
  const int64_t start = (int64_t)chunk_index[blockIdx.x] * kChunk;
  const int64_t end = min(e.n, start + kChunk);
  float sd = 0.f, sdd = 0.f, sw = 0.f, sww = 0.f;
  for (int64_t i = start + threadIdx.x; i < end; i += blockDim.x) {
    const float w = to_f(W[i]), d = w - to_f(P[i]);
    sd += d; sdd += d * d; sw += w; sww += w * w;
  }
  __shared__ double red[4][4];
  double v[4] = {sd, sdd, sw, sww};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    // wave sum in fp64 via two fp32 halves would lose the point; reduce the fp32 lane sums in fp64
    double x = v[k];
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    v[k] = x;
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < 4; ++k) red[wv][k] = v[k];
  __syncthreads();
  if (threadIdx.x < 4) {
    const int k = threadIdx.x;
    part[(size_t)blockIdx.x * 4 + k] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
  }
}

// out[t] = (std(w − prev), std(w)) of tensor t, chunks [first[t], first[t + 1])
__global__ void __launch_bounds__(64) moments_fold_kernel(const double* __restrict__ part,
                                                          const int32_t* __restrict__ first,
                                                          const int64_t* __restrict__ numel, float* __restrict__ out,
                                                          int nt) {
  const int t = blockIdx.x * 64 + threadIdx.x;
  if (t >= nt) return;
  double s[4] = {0.0, 0.0, 0.0, 0.0};
  for (int c = first[t]; c < first[t + 1]; ++c)
#pragma unroll
    for (int k = 0; k < 4; ++k) s[k] += part[(size_t)c * 4 + k];
  const double n = (double)numel[t];
  auto sdev = [&](double a, double aa) { return n > 1.0 ? sqrt(fmax(aa - a * a / n, 0.0) / (n - 1.0)) : 0.0; };
  out[2 * t] = (float)sdev(s[0], s[1]);
  out[2 * t + 1] = (float)sdev(s[2], s[3]);
}
}  // namespace
}  // namespace penroz

// [n, 2] fp32: (std(w − prev), std(w)) for every pair (same shape and dtype, fp32 or bf16)
torch::Tensor update_moments(std::vector<torch::Tensor> ws, std::vector<torch::Tensor> ps) {
  const size_t nt = ws.size();
  TORCH_CHECK(ps.size() == nt && nt > 0, "update_moments: one prev per weight");
  const auto dt = ws[0].scalar_type();
  TORCH_CHECK(dt == torch::kFloat32 || dt == torch::kBFloat16, "update_moments: fp32 or bf16");
  std::vector<MomEntry> tab(nt);
  std::vector<int32_t> ct, ci, first(nt + 1);
  std::vector<int64_t> numel(nt);
  for (size_t i = 0; i < nt; ++i) {
    TORCH_CHECK(ws[i].is_cuda() && ps[i].is_cuda() && ws[i].is_contiguous() && ps[i].is_contiguous() &&
                    ws[i].scalar_type() == dt && ps[i].scalar_type() == dt && ws[i].numel() == ps[i].numel(),
                "update_moments: contiguous GPU tensors of one dtype, prev shaped like its weight");
    tab[i] = {ws[i].data_ptr(), ps[i].data_ptr(), ws[i].numel()};
    numel[i] = ws[i].numel();
    first[i] = (int32_t)ct.size();
    const int64_t chunks = (ws[i].numel() + kChunk - 1) / kChunk;
    for (int64_t c = 0; c < chunks; ++c) {
      ct.push_back((int32_t)i);
      ci.push_back((int32_t)c);
    }
  }
  first[nt] = (int32_t)ct.size();
  const int64_t nchunks = ct.size();
  auto opt = ws[0].options();
  auto out = torch::zeros({(int64_t)nt, 2}, opt.dtype(torch::kFloat32));
  if (nchunks == 0) return out;
  const int64_t tab_bytes = nt * sizeof(MomEntry);
  const int64_t bytes = tab_bytes + 8 * nchunks + 4 * (nt + 1) + 8 * nt + 8;
  auto host = torch::empty({bytes}, torch::TensorOptions().dtype(torch::kUInt8).pinned_memory(true));
  uint8_t* hp = host.data_ptr<uint8_t>();
  std::memcpy(hp, tab.data(), tab_bytes);
  std::memcpy(hp + tab_bytes, ct.data(), 4 * nchunks);
  std::memcpy(hp + tab_bytes + 4 * nchunks, ci.data(), 4 * nchunks);
  const int64_t off_first = tab_bytes + 8 * nchunks;
  std::memcpy(hp + off_first, first.data(), 4 * (nt + 1));
  const int64_t off_numel = (off_first + 4 * (nt + 1) + 7) / 8 * 8;
  std::memcpy(hp + off_numel, numel.data(), 8 * nt);
  auto dev = host.to(ws[0].device(), /*non_blocking=*/true);
  const uint8_t* base = dev.data_ptr<uint8_t>();
  auto part = torch::empty({nchunks * 4}, opt.dtype(torch::kFloat64));
  auto stream = at::hip::getCurrentHIPStream();
  auto k1 = dt == torch::kBFloat16 ? moments_chunk_kernel<bf16> : moments_chunk_kernel<float>;
  hipLaunchKernelGGL(k1, dim3((unsigned)nchunks), dim3(256), 0, stream, reinterpret_cast<const MomEntry*>(base),
                     reinterpret_cast<const int32_t*>(base + tab_bytes),
                     reinterpret_cast<const int32_t*>(base + tab_bytes + 4 * nchunks), part.data_ptr<double>());
  hipLaunchKernelGGL(moments_fold_kernel, dim3((unsigned)((nt + 63) / 64)), dim3(64), 0, stream,
                     part.data_ptr<double>(), reinterpret_cast<const int32_t*>(base + off_first),
                     reinterpret_cast<const int64_t*>(base + off_numel), out.data_ptr<float>(), (int)nt);
  return out;
}
