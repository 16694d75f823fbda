// KV-cache attention for incremental decoding (memory-bound: every cached K/V byte is read
// once per step).
//
// Work item = (batch b, KV head g, query row tq, split s). One 256-thread workgroup owns all
// H/Hkv query heads that share KV head g (GQA by index math — the cache is never expanded),
// so each K/V row is loaded once for the whole group. The keys of a split are dealt to the
// 4 waves in 64-key blocks:
//   scores : lane j holds key (blk + j); its K row is read as 16-B vectors and dotted with the
//            group's query vectors (staged in LDS, fp32);
//   softmax: running (m, l) per query head, wave-wide max/sum, causal mask by absolute
//            position (query tq sits at q_offset + tq);
//   PV     : lane d owns output column d (and d+64 for D=128); V row j is read coalesced and
//            p_j is broadcast with a lane shuffle.
// int8 caches (TurboQuant) carry per-token fp32 scales that are folded into the score and
// the P·V weight, so the int8 cache is never dequantised to memory.
// The 4 waves merge through LDS; with several splits the partial (m, l, O) go to a workspace
// and a second kernel combines them. Enough splits are used to put ≥ 512 workgroups in
// flight (256 CUs) even at batch 1.
#include "common.h"
#include <type_traits>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

namespace penroz {

constexpr int kMaxGroup = 16;

template <typename TK> struct KRow;
template <> struct KRow<bf16> {
  __device__ __forceinline__ static float at(const bf16* p, int d) { return bf2f(p[d]); }
};
template <> struct KRow<__half> {
  __device__ __forceinline__ static float at(const __half* p, int d) { return __half2float(p[d]); }
};
template <> struct KRow<float> {
  __device__ __forceinline__ static float at(const float* p, int d) { return p[d]; }
};
template <> struct KRow<int8_t> {
  __device__ __forceinline__ static float at(const int8_t* p, int d) { return (float)p[d]; }
};

// 8 consecutive cache elements -> fp32 (one 16-B load for bf16/fp16, 8 B for int8, 32 B for fp32)
template <typename TK> struct Row8;
template <> struct Row8<bf16> {
  __device__ __forceinline__ static void load(const bf16* p, float (&v)[8]) { Vec8<bf16>::load(p, v); }
};
template <> struct Row8<__half> {
  __device__ __forceinline__ static void load(const __half* p, float (&v)[8]) { Vec8<__half>::load(p, v); }
};
template <> struct Row8<float> {
  __device__ __forceinline__ static void load(const float* p, float (&v)[8]) { Vec8<float>::load(p, v); }
};
template <> struct Row8<int8_t> {
  __device__ __forceinline__ static void load(const int8_t* p, float (&v)[8]) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = (float)(int8_t)((u.x >> (8 * i)) & 0xff);
      v[4 + i] = (float)(int8_t)((u.y >> (8 * i)) & 0xff);
    }
  }
};

template <int D, typename TQ, typename TK>
__global__ void __launch_bounds__(256) decode_kernel(const TQ* __restrict__ q, const TK* __restrict__ kc,
                                                     const TK* __restrict__ vc, const float* __restrict__ ks,
                                                     const float* __restrict__ vs, TQ* __restrict__ out,
                                                     float* __restrict__ ws_o, float* __restrict__ ws_ml, int B,
                                                     int Tq, int H, int Hkv, int cap, int S, int q_offset,
                                                     int splits, float scale, const int64_t* __restrict__ S_dev,
                                                     int64_t q_rs) {
  if (S_dev != nullptr) {  // graph-replayed decode: the cache length lives on the device
    S = (int)min<int64_t>(*S_dev, (int64_t)cap);
    q_offset = S - Tq;
  }
  constexpr int DL = D / 64;  // output columns per lane
  const int G = H / Hkv;
  int wid_lin = blockIdx.x;
  const int split = wid_lin % splits;
  wid_lin /= splits;
  const int tq = wid_lin % Tq;
  wid_lin /= Tq;
  const int g = wid_lin % Hkv;
  const int b = wid_lin / Hkv;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;

  __shared__ float qs[kMaxGroup][D];
  __shared__ float red_m[4][kMaxGroup], red_l[4][kMaxGroup];
  __shared__ float red_o[4][kMaxGroup][D];

  for (int i = threadIdx.x; i < G * D; i += 256) {
    const int h = g * G + i / D, d = i % D;
    qs[i / D][d] = to_f(q[((size_t)b * Tq + tq) * q_rs + (size_t)h * D + d]) * scale;
  }
  __syncthreads();

  const int kend_causal = min(S, q_offset + tq + 1);
  const int per_split = (kend_causal + splits - 1) / splits;
  const int k0 = split * per_split, k1 = min(kend_causal, k0 + per_split);
  const size_t head_base = ((size_t)b * Hkv + g) * cap;

  float m[kMaxGroup], l[kMaxGroup], o[kMaxGroup][DL];
#pragma unroll
  for (int i = 0; i < kMaxGroup; ++i) {
    m[i] = -INFINITY;
    l[i] = 0.f;
#pragma unroll
    for (int j = 0; j < DL; ++j) o[i][j] = 0.f;
  }

  for (int blk = k0 + 64 * wid; blk < k1; blk += 256) {
    const int key = blk + lane;
    const bool valid = key < k1;
    float kv[D];
    const TK* krow = kc + (head_base + (valid ? key : k0)) * D;
#pragma unroll
    for (int c = 0; c < D / 8; ++c) {  // whole K row in flight: D/8 vector loads
      float t[8];
      Row8<TK>::load(krow + 8 * c, t);
#pragma unroll
      for (int e = 0; e < 8; ++e) kv[8 * c + e] = t[e];
    }
    const float kscale = ks ? ks[head_base + (valid ? key : k0)] : 1.f;
    float p[kMaxGroup];
#pragma unroll
    for (int i = 0; i < kMaxGroup; ++i) {
      if (i >= G) break;
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < D; ++d) s += qs[i][d] * kv[d];
      s = valid ? s * kscale : -INFINITY;
      const float mn = fmaxf(m[i], wave_max(s));
      const float alpha = __expf(m[i] - mn);
      p[i] = valid ? __expf(s - mn) : 0.f;
      l[i] = l[i] * alpha + wave_sum(p[i]);
      m[i] = mn;
#pragma unroll
      for (int j = 0; j < DL; ++j) o[i][j] *= alpha;
    }
    // P·V: lane d owns output column(s) d; V rows are read coalesced, 16 rows in flight per
    // batch (a one-row-at-a-time loop serialises on the load latency: ~70 µs per call at S=128)
    const int nk = min(64, k1 - blk);
    for (int j0 = 0; j0 < nk; j0 += 16) {
      float vv[16][DL];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j = min(j0 + r, nk - 1);
        const TK* vrow = vc + (head_base + blk + j) * D;
        const float vsc = vs ? vs[head_base + blk + j] : 1.f;
#pragma unroll
        for (int jj = 0; jj < DL; ++jj) vv[r][jj] = KRow<TK>::at(vrow, lane + 64 * jj) * vsc;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (j0 + r >= nk) break;
#pragma unroll
        for (int i = 0; i < kMaxGroup; ++i) {
          if (i >= G) break;
          const float pj = __shfl(p[i], j0 + r, 64);
#pragma unroll
          for (int jj = 0; jj < DL; ++jj) o[i][jj] += pj * vv[r][jj];
        }
      }
    }
  }
  // merge the 4 waves
  for (int i = 0; i < G; ++i) {
    if (lane == 0) { red_m[wid][i] = m[i]; red_l[wid][i] = l[i]; }
#pragma unroll
    for (int jj = 0; jj < DL; ++jj) red_o[wid][i][lane + 64 * jj] = o[i][jj];
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < G * D; idx += 256) {
    const int i = idx / D, d = idx % D;
    float M = -INFINITY;
    for (int w = 0; w < 4; ++w) M = fmaxf(M, red_m[w][i]);
    float L = 0.f, O = 0.f;
    for (int w = 0; w < 4; ++w) {
      const float f = red_m[w][i] == -INFINITY ? 0.f : __expf(red_m[w][i] - M);
      L += red_l[w][i] * f;
      O += red_o[w][i][d] * f;
    }
    const int h = g * G + i;
    if (splits == 1) {
      out[(((size_t)b * Tq + tq) * H + h) * D + d] = from_f<TQ>(L > 0.f ? O / L : 0.f);
    } else {
      const size_t r = (((size_t)split * B + b) * Tq + tq) * H + h;
      ws_o[r * D + d] = O;
      if (d == 0) {
        ws_ml[2 * r] = M;
        ws_ml[2 * r + 1] = L;
      }
    }
  }
}

template <typename TQ>
__global__ void __launch_bounds__(256) decode_combine_kernel(const float* __restrict__ ws_o,
                                                             const float* __restrict__ ws_ml, TQ* __restrict__ out,
                                                             int rows, int D, int splits) {
  const int64_t total = (int64_t)rows * D;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / D;
    const int d = (int)(i - r * D);
    float M = -INFINITY;
    for (int s = 0; s < splits; ++s) M = fmaxf(M, ws_ml[2 * ((int64_t)s * rows + r)]);
    float L = 0.f, O = 0.f;
    for (int s = 0; s < splits; ++s) {
      const int64_t rr = (int64_t)s * rows + r;
      const float ms = ws_ml[2 * rr];
      const float f = ms == -INFINITY ? 0.f : __expf(ms - M);
      L += ws_ml[2 * rr + 1] * f;
      O += ws_o[rr * D + d] * f;
    }
    out[i] = from_f<TQ>(L > 0.f ? O / L : 0.f);
  }
}

// Append one token's K and V rows (read straight from the fused QKV projection) into the cache
// slot `pos` — taken from device memory when pos_dev is given (graph-replayed decode). One wave
// per (batch, KV head, K|V) row; int8 caches quantise per token (absmax / 127, round to nearest
// even) exactly like kv_quant_kernel.
template <typename T, typename TK>
__global__ void __launch_bounds__(256) kv_append_kernel(const T* __restrict__ k, const T* __restrict__ v,
                                                        int64_t k_rs, int64_t v_rs, TK* __restrict__ kc,
                                                        TK* __restrict__ vc, float* __restrict__ ks,
                                                        float* __restrict__ vs, int B, int Hkv, int D, int cap,
                                                        const int64_t* __restrict__ pos_dev, int pos_host) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);  // over B*Hkv*2
  if (row >= B * Hkv * 2) return;
  const int which = row & 1, bg = row >> 1;
  const int g = bg % Hkv, b = bg / Hkv;
  const T* src = (which ? v + (size_t)b * v_rs : k + (size_t)b * k_rs) + (size_t)g * D;
  const int pos = pos_dev ? (int)*pos_dev : pos_host;
  const size_t slot = ((size_t)b * Hkv + g) * cap + pos;
  TK* dst = (which ? vc : kc) + slot * D;
  if constexpr (std::is_same<TK, int8_t>::value) {
    float m = 0.f;
    for (int d = lane; d < D; d += 64) m = fmaxf(m, fabsf(to_f(src[d])));
    m = wave_max(m);
    float sc = m / 127.f;
    if (sc == 0.f) sc = 1.f;
    for (int d = lane; d < D; d += 64) {
      float x = rintf(to_f(src[d]) / sc);
      dst[d] = (int8_t)fminf(fmaxf(x, -128.f), 127.f);
    }
    if (lane == 0) (which ? vs : ks)[slot] = sc;
  } else {
    for (int d = lane; d < D; d += 64) dst[d] = src[d];
  }
}

}  // namespace penroz

using namespace penroz;

// seq_len_dev (optional int64 [1] on the device): the cache length is read by the kernel at run
// time (S / q_offset are then only upper bounds used to size the launch) — lets a captured HIP
// graph replay the same decode step at every position.
torch::Tensor decode_attn(torch::Tensor q, torch::Tensor kc, torch::Tensor vc, c10::optional<torch::Tensor> k_scale,
                          c10::optional<torch::Tensor> v_scale, int64_t S, int64_t q_offset, double scale,
                          c10::optional<torch::Tensor> seq_len_dev) {
  TORCH_CHECK(q.is_cuda() && q.dim() == 4, "q must be [B, Tq, H, D]");
  // q may be a view into the fused QKV rows: unit dim stride, packed heads, uniform row stride
  TORCH_CHECK(q.stride(3) == 1 && q.stride(2) == q.size(3) && q.stride(0) == q.size(1) * q.stride(1),
              "q must have packed heads and a uniform row stride");
  TORCH_CHECK(kc.is_contiguous() && vc.is_contiguous() && kc.dim() == 4 && kc.sizes() == vc.sizes());
  const int B = q.size(0), Tq = q.size(1), H = q.size(2), D = q.size(3);
  const int Hkv = kc.size(1), cap = kc.size(2);
  TORCH_CHECK(kc.size(0) == B && kc.size(3) == D && H % Hkv == 0 && H / Hkv <= kMaxGroup);
  TORCH_CHECK(S <= cap && q_offset >= 0 && q_offset + Tq <= S, "bad cache extent");
  TORCH_CHECK(D == 64 || D == 128, "decode attention supports head_dim 64/128");
  const bool quant = kc.scalar_type() == torch::kInt8;
  TORCH_CHECK(!quant || (k_scale.has_value() && v_scale.has_value()), "int8 cache needs scales");
  TORCH_CHECK(quant || kc.scalar_type() == q.scalar_type(), "cache dtype must match q");
  auto out = torch::empty({B, Tq, H * D}, q.options());
  const int64_t q_rs = q.stride(1);
  const int items = B * Hkv * Tq;
  int splits = std::max(1, std::min<int>((512 + items - 1) / items, (int)((S + 255) / 256)));
  torch::Tensor ws_o, ws_ml;
  float* wo = nullptr;
  float* wm = nullptr;
  if (splits > 1) {
    ws_o = torch::empty({(int64_t)splits * B * Tq * H * D}, q.options().dtype(torch::kFloat32));
    ws_ml = torch::empty({(int64_t)splits * B * Tq * H * 2}, q.options().dtype(torch::kFloat32));
    wo = ws_o.data_ptr<float>();
    wm = ws_ml.data_ptr<float>();
  }
  const int64_t* sdev = nullptr;
  if (seq_len_dev.has_value() && seq_len_dev->defined()) {
    TORCH_CHECK(seq_len_dev->is_cuda() && seq_len_dev->scalar_type() == torch::kInt64 && seq_len_dev->numel() == 1,
                "seq_len_dev must be a device int64 [1]");
    sdev = seq_len_dev->data_ptr<int64_t>();
  }
  const float* ksp = quant ? k_scale->data_ptr<float>() : nullptr;
  const float* vsp = quant ? v_scale->data_ptr<float>() : nullptr;
  auto stream = at::hip::getCurrentHIPStream();
  dim3 grid(items * splits);
  auto launch = [&](auto qtag, auto ktag) {
    using TQ = decltype(qtag);
    using TK = decltype(ktag);
    const TQ* qp = reinterpret_cast<const TQ*>(q.data_ptr());
    const TK* kp = reinterpret_cast<const TK*>(kc.data_ptr());
    const TK* vp = reinterpret_cast<const TK*>(vc.data_ptr());
    TQ* op = reinterpret_cast<TQ*>(out.data_ptr());
    if (D == 64)
      hipLaunchKernelGGL((decode_kernel<64, TQ, TK>), grid, dim3(256), 0, stream, qp, kp, vp, ksp, vsp, op, wo, wm, B,
                         Tq, H, Hkv, cap, (int)S, (int)q_offset, splits, (float)scale, sdev, q_rs);
    else
      hipLaunchKernelGGL((decode_kernel<128, TQ, TK>), grid, dim3(256), 0, stream, qp, kp, vp, ksp, vsp, op, wo, wm, B,
                         Tq, H, Hkv, cap, (int)S, (int)q_offset, splits, (float)scale, sdev, q_rs);
    if (splits > 1) {
      const int rows = B * Tq * H;
      hipLaunchKernelGGL(decode_combine_kernel<TQ>, dim3(std::min(2048, (rows * D + 255) / 256)), dim3(256), 0, stream,
                         wo, wm, op, rows, D, splits);
    }
  };
  auto with_k = [&](auto qtag) {
    if (quant) launch(qtag, int8_t{});
    else launch(qtag, qtag);
  };
  if (q.scalar_type() == torch::kBFloat16) with_k(bf16{});
  else if (q.scalar_type() == torch::kFloat32) with_k(float{});
  else if (q.scalar_type() == torch::kFloat16) with_k(__half{});
  else TORCH_CHECK(false, "unsupported q dtype");
  return out;
}

// k, v: [B, 1, Hkv, D] (views into the fused QKV rows allowed); caches [B, Hkv, cap, D]
void kv_append(torch::Tensor k, torch::Tensor v, torch::Tensor kc, torch::Tensor vc, c10::optional<torch::Tensor> ks,
               c10::optional<torch::Tensor> vs, c10::optional<torch::Tensor> pos_dev, int64_t pos) {
  TORCH_CHECK(k.is_cuda() && k.dim() == 4 && k.sizes() == v.sizes() && k.size(1) == 1, "k/v must be [B, 1, Hkv, D]");
  TORCH_CHECK(k.stride(3) == 1 && k.stride(2) == k.size(3) && v.stride(3) == 1 && v.stride(2) == v.size(3),
              "k/v rows must be packed");
  const int B = k.size(0), Hkv = k.size(2), D = k.size(3);
  TORCH_CHECK(kc.is_contiguous() && vc.is_contiguous() && kc.sizes() == vc.sizes() && kc.size(0) == B &&
              kc.size(1) == Hkv && kc.size(3) == D, "cache shape");
  const int cap = kc.size(2);
  const int64_t* pd = nullptr;
  if (pos_dev.has_value() && pos_dev->defined()) {
    TORCH_CHECK(pos_dev->is_cuda() && pos_dev->scalar_type() == torch::kInt64 && pos_dev->numel() == 1);
    pd = pos_dev->data_ptr<int64_t>();
  } else {
    TORCH_CHECK(pos >= 0 && pos < cap, "cache overflow");
  }
  const bool quant = kc.scalar_type() == torch::kInt8;
  TORCH_CHECK(!quant || (ks.has_value() && vs.has_value()), "int8 cache needs scales");
  TORCH_CHECK(quant || kc.scalar_type() == k.scalar_type(), "cache dtype must match k/v");
  const int rows = B * Hkv * 2;
  auto stream = at::hip::getCurrentHIPStream();
  auto launch = [&](auto ttag, auto ktag) {
    using T = decltype(ttag);
    using TK = decltype(ktag);
    hipLaunchKernelGGL((kv_append_kernel<T, TK>), dim3((rows + 3) / 4), dim3(256), 0, stream,
                       reinterpret_cast<const T*>(k.data_ptr()), reinterpret_cast<const T*>(v.data_ptr()), k.stride(0),
                       v.stride(0), reinterpret_cast<TK*>(kc.data_ptr()), reinterpret_cast<TK*>(vc.data_ptr()),
                       quant ? ks->data_ptr<float>() : nullptr, quant ? vs->data_ptr<float>() : nullptr, B, Hkv, D,
                       cap, pd, (int)pos);
  };
  auto with_k = [&](auto ttag) {
    if (quant) launch(ttag, int8_t{});
    else launch(ttag, ttag);
  };
  if (k.scalar_type() == torch::kBFloat16) with_k(bf16{});
  else if (k.scalar_type() == torch::kFloat32) with_k(float{});
  else if (k.scalar_type() == torch::kFloat16) with_k(__half{});
  else TORCH_CHECK(false, "unsupported k dtype");
}
