// Memory-bound kernels: GELU fwd/bwd (+ fused bias-gradient column sum), gated-MLP
// activation, column sums, token+position embedding fwd/bwd, RoPE on fused QKV, int8 KV
// quantisation, and on-device tensor statistics (moments, min/max, density histogram).
//
// All streams use 16-B per-lane vectors (8 bf16 or 4 fp32), grid-stride loops capped at
// 8192 workgroups for the large passes (2048 elsewhere; CDNA HIP guide, Guideline 11/13). Column-sum fusions keep each thread's
// 8 columns fixed while it walks rows, so the partial sums live in registers; a workgroup
// reduces its 4 waves in LDS and writes one partial row, finished by a tiny reduction.
#include "common.h"
#include "deferred.h"
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <cstdlib>

namespace penroz {

__device__ __forceinline__ float act_grad_f(float x, int kind) {
  if (kind == 2) {
    const float s = 1.f / (1.f + __expf(-x));
    return s * (1.f + x * (1.f - s));
  }
  return gelu_grad_f(x, kind);
}

template <typename T, bool NT = false>
__global__ void __launch_bounds__(256) gelu_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t n8,
                                                       int approx) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    float v[8];
    load8<NT>(x + 8 * i, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = gelu_f(v[k], approx);
    store8<NT>(y + 8 * i, v);
  }
}

template <typename T, bool NT = false>
__global__ void __launch_bounds__(256) gelu_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                       T* __restrict__ dx, int64_t n8, int approx) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    float g[8], v[8];
    load8<NT>(dy + 8 * i, g);
    load8<NT>(x + 8 * i, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) g[k] *= gelu_grad_f(v[k], approx);
    store8<NT>(dx + 8 * i, g);
  }
}

// MODE 0: colsum of x.  MODE 1: dx = dy*gelu'(x) written to out, colsum of dx.
// grid = (F/512 column tiles, R row splits); block 256 = 4 waves; lane -> 8 columns.
template <int MODE, typename T, bool NT = false>
__global__ void __launch_bounds__(256) rows_colsum_kernel(const T* __restrict__ a, const T* __restrict__ x,
                                                          T* __restrict__ out, float* __restrict__ part, int N, int F,
                                                          int approx) {
  __shared__ float red[4][512];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int col = blockIdx.x * 512 + 8 * lane;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bool active = col < F;
  const int R = gridDim.y;
  const int rows_per = (N + R - 1) / R;
  const int r0 = blockIdx.y * rows_per, r1 = min(N, r0 + rows_per);
  if (active) {
    for (int r = r0 + wid; r < r1; r += 4) {
      const size_t off = (size_t)r * F + col;
      float v[8];
      load8<NT>(a + off, v);
      if constexpr (MODE == 1) {
        float xv[8];
        load8<NT>(x + off, xv);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = to_f(from_f<T>(v[k] * gelu_grad_f(xv[k], approx)));
        // v now holds the *rounded* values: dbias matches the bf16 gradient the GEMMs see
        store8<NT>(out + off, v);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += v[k];
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[wid][8 * lane + k] = acc[k];
  __syncthreads();
  for (int c = threadIdx.x; c < 512; c += 256) {
    const int gc = blockIdx.x * 512 + c;
    if (gc < F) part[(size_t)blockIdx.y * F + gc] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
  }
}

// ------------------------------------------------------------------------------ gated MLP act
template <typename T, bool NT = false>
__global__ void __launch_bounds__(256) gated_fwd_kernel(const T* __restrict__ g, const T* __restrict__ u,
                                                        T* __restrict__ y, int64_t n8, int kind) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    float gv[8], uv[8];
    load8<NT>(g + 8 * i, gv);
    load8<NT>(u + 8 * i, uv);
#pragma unroll
    for (int k = 0; k < 8; ++k) gv[k] = act_f(gv[k], kind) * uv[k];
    store8<NT>(y + 8 * i, gv);
  }
}

// decode: gate and up halves of one fused [N, 2I] projection -> act(gate) * up [N, I]
template <typename T, bool NT = false>
__global__ void __launch_bounds__(256) gated_packed_kernel(const T* __restrict__ gu, T* __restrict__ y, int64_t n8,
                                                           int I8, int kind) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / I8, c = i - r * I8;
    float gv[8], uv[8];
    load8<NT>(gu + 8 * (r * 2 * I8 + c), gv);
    load8<NT>(gu + 8 * (r * 2 * I8 + I8 + c), uv);
#pragma unroll
    for (int k = 0; k < 8; ++k) gv[k] = act_f(gv[k], kind) * uv[k];
    store8<NT>(y + 8 * i, gv);
  }
}

template <typename T, bool NT = false>
__global__ void __launch_bounds__(256) gated_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ g,
                                                        const T* __restrict__ u, T* __restrict__ dg,
                                                        T* __restrict__ du, int64_t n8, int kind) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    float d[8], gv[8], uv[8], o1[8], o2[8];
    load8<NT>(dy + 8 * i, d);
    load8<NT>(g + 8 * i, gv);
    load8<NT>(u + 8 * i, uv);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      o1[k] = d[k] * uv[k] * act_grad_f(gv[k], kind);
      o2[k] = d[k] * act_f(gv[k], kind);
    }
    store8<NT>(dg + 8 * i, o1);
    store8<NT>(du + 8 * i, o2);
  }
}

// packed form of the backward: gu = [gate | up] per row (I8 chunks of 8 each), dgu likewise —
// the layout one GEMM over the concatenated [gate; up] weight consumes (fused Gemma executor)
template <typename T, bool NT = false>
__global__ void __launch_bounds__(256) gated_bwd_packed_kernel(const T* __restrict__ dy, const T* __restrict__ gu,
                                                               T* __restrict__ dgu, int64_t n8, int I8, int kind) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / I8, c = i - r * I8;
    const int64_t go = 8 * (r * 2 * I8 + c), uo = go + 8 * (int64_t)I8;
    float d[8], gv[8], uv[8], o1[8], o2[8];
    load8<NT>(dy + 8 * i, d);
    load8<NT>(gu + go, gv);
    load8<NT>(gu + uo, uv);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      o1[k] = d[k] * uv[k] * act_grad_f(gv[k], kind);
      o2[k] = d[k] * act_f(gv[k], kind);
    }
    store8<NT>(dgu + go, o1);
    store8<NT>(dgu + uo, o2);
  }
}

// ------------------------------------------------------------------------------ embedding
// out[n, :] = wte[idx[n], :] + wpe[off + n % T, :]   (one wave per token row, 16-B lanes)
template <typename TW>
__global__ void __launch_bounds__(256) embed_fwd_kernel(const int64_t* __restrict__ idx, const TW* __restrict__ wte,
                                                        const TW* __restrict__ wpe, float* __restrict__ out, int N,
                                                        int T, int C, int off, int V, const int64_t* __restrict__ off_dev,
                                                        int P, uint64_t dseed, float dp) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= N) return;
  int64_t tok = idx[row];
  PZ_DEVICE_CHECK(tok >= 0 && tok < V);
  tok = tok < 0 ? 0 : (tok >= V ? V - 1 : tok);
  if (off_dev != nullptr) off = (int)*off_dev;  // graph-replayed decode: position on the device
  const int pos = min(off + row % T, P - 1);
  for (int c = 8 * lane; c < C; c += 512) {
    float a[8], b[8];
    Vec8<TW>::load(wte + (size_t)tok * C + c, a);
    Vec8<TW>::load(wpe + (size_t)pos * C + c, b);
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] += b[k];
    if (dp > 0.f) {  // embedding dropout (HF GPT-2 embd_pdrop); the backward regenerates the mask
      const float inv = 1.f / (1.f - dp);
#pragma unroll
      for (int k = 0; k < 8; ++k) a[k] *= dropout_mult(dseed, (size_t)row * C + c + k, dp, inv);
    }
    Vec8<float>::store(out + (size_t)row * C + c, a);
  }
}

// out [C][R] = in [R][C]ᵀ, bf16, 64×64 tiles through LDS (16-B global loads and stores). Used
// for the weight copies of the data-gradient GEMMs (dx = dy·W runs ~12-22 % faster on
// hipBLASLt with W stored transposed: both operands then reduction-contiguous, the forward's
// layout — profiles/dgrad_layout_r1.log).
__global__ void __launch_bounds__(256) transpose_bf16_kernel(const uint16_t* __restrict__ in,
                                                             uint16_t* __restrict__ out, int R, int C) {
  __shared__ uint16_t tile[64][66];
  const int tiles_c = C / 64;
  const int r0 = (blockIdx.x / tiles_c) * 64, c0 = (blockIdx.x % tiles_c) * 64;
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int v = t + 256 * i, row = v >> 3, ch = v & 7;
    const uint4 u = *reinterpret_cast<const uint4*>(in + (size_t)(r0 + row) * C + c0 + 8 * ch);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      tile[row][8 * ch + 2 * j] = (uint16_t)(w[j] & 0xffff);
      tile[row][8 * ch + 2 * j + 1] = (uint16_t)(w[j] >> 16);
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int v = t + 256 * i, orow = v >> 3, ch = v & 7;  // output row = input column c0 + orow
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      w[j] = (uint32_t)tile[8 * ch + 2 * j][orow] | ((uint32_t)tile[8 * ch + 2 * j + 1][orow] << 16);
    *reinterpret_cast<uint4*>(out + (size_t)(c0 + orow) * R + r0 + 8 * ch) = uint4{w[0], w[1], w[2], w[3]};
  }
}

// dwte[idx[n]] += dout[n]  (fp32 atomics; each wave instruction = 256 contiguous bytes)
__global__ void __launch_bounds__(256) embed_bwd_tok_kernel(const float* __restrict__ dout,
                                                            const int64_t* __restrict__ idx,
                                                            float* __restrict__ dwte, int N, int C, int V,
                                                            uint64_t dseed, float dp) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= N) return;
  const int64_t tok = idx[row];
  PZ_DEVICE_CHECK(tok >= 0 && tok < V);
  if (tok < 0 || tok >= V) return;
  float* dst = dwte + (size_t)tok * C;
  const float* src = dout + (size_t)row * C;
  if (dp > 0.f) {
    const float inv = 1.f / (1.f - dp);
    for (int c = lane; c < C; c += 64)
      atomicAdd(dst + c, src[c] * dropout_mult(dseed, (size_t)row * C + c, dp, inv));
  } else {
    for (int c = lane; c < C; c += 64) atomicAdd(dst + c, src[c]);
  }
}

// dwpe[off + t] += Σ_b dout[b*T + t]   (one workgroup per position, no atomics)
__global__ void __launch_bounds__(256) embed_bwd_pos_kernel(const float* __restrict__ dout, float* __restrict__ dwpe,
                                                            int B, int T, int C, int off, uint64_t dseed, float dp) {
  const int t = blockIdx.x;
  const float inv = dp > 0.f ? 1.f / (1.f - dp) : 1.f;
  for (int c = threadIdx.x * 4; c < C; c += 1024) {
    float4_t s = {0.f, 0.f, 0.f, 0.f};
    for (int b = 0; b < B; ++b) {
      const size_t e = ((size_t)b * T + t) * C + c;
      float4_t g = *reinterpret_cast<const float4_t*>(dout + e);
      if (dp > 0.f) {
#pragma unroll
        for (int k = 0; k < 4; ++k) g[k] *= dropout_mult(dseed, e + k, dp, inv);
      }
      s += g;
    }
    float4_t* d = reinterpret_cast<float4_t*>(dwpe + (size_t)(off + t) * C + c);
    *d = *d + s;
  }
}

// ------------------------------------------------------------------------------ RoPE
// qkv [B*T, (H+2Hkv)*D]; rotate the first H+Hkv heads (Q and K); V copied. cos/sin [T, D/2].
template <typename T>
__global__ void __launch_bounds__(256) rope_kernel(const T* __restrict__ in, T* __restrict__ out,
                                                   const float* __restrict__ cosv, const float* __restrict__ sinv,
                                                   int64_t rows, int Tlen, int H, int Hkv, int D, int inverse) {
  const int W = (H + 2 * Hkv) * D;
  const int half = D / 2;
  const int64_t total = rows * (int64_t)W;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / W;
    const int c = (int)(i - r * W);
    const int head = c / D;
    const int d = c - head * D;
    if (head >= H + Hkv) {
      out[i] = in[i];
      continue;
    }
    const int t = (int)(r % Tlen);
    const int j = d < half ? d : d - half;
    const float cs = cosv[(size_t)t * half + j];
    float sn = sinv[(size_t)t * half + j];
    if (inverse) sn = -sn;
    const int64_t hb = r * W + (int64_t)head * D;
    const float x1 = to_f(in[hb + j]), x2 = to_f(in[hb + j + half]);
    const float o = d < half ? (x1 * cs - x2 * sn) : (x2 * cs + x1 * sn);
    out[i] = from_f<T>(o);
  }
}

// Vectorised form (D % 16 == 0, contiguous fp32 cos / sin tables): one work item = 8 rotated pairs
// (16-B loads of both halves and of cos / sin) or one 16-B chunk of the V columns copied through;
// the scalar kernel above did a 64-bit division, two gathered 2-B loads and a 2-B store per element
// (≈ 0.6 TB/s at Gemma-3 1B shapes).
template <typename T>
__global__ void __launch_bounds__(256) rope_vec_kernel(const T* __restrict__ in, T* __restrict__ out,
                                                       const float* __restrict__ cosv,
                                                       const float* __restrict__ sinv, int64_t rows, int Tlen,
                                                       int H, int Hkv, int D, int inverse) {
  const int W = (H + 2 * Hkv) * D, half = D / 2, h8 = half / 8;
  const int nrot = (H + Hkv) * h8, per = nrot + Hkv * D / 8;
  const int64_t total = rows * (int64_t)per;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / per;
    const int k = (int)(i - r * per);
    if (k < nrot) {
      const int head = k / h8, j0 = 8 * (k - head * h8);
      const int t = (int)(r % Tlen);
      const int64_t base = r * W + (int64_t)head * D;
      float x1[8], x2[8];
      Vec8<T>::load(in + base + j0, x1);
      Vec8<T>::load(in + base + half + j0, x2);
      const float* cp = cosv + (size_t)t * half + j0;
      const float* sp = sinv + (size_t)t * half + j0;
      const float4 c0 = *reinterpret_cast<const float4*>(cp), c1 = *reinterpret_cast<const float4*>(cp + 4);
      const float4 s0 = *reinterpret_cast<const float4*>(sp), s1 = *reinterpret_cast<const float4*>(sp + 4);
      const float cs[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
      float sn[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
      float o1[8], o2[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (inverse) sn[e] = -sn[e];
        o1[e] = x1[e] * cs[e] - x2[e] * sn[e];
        o2[e] = x2[e] * cs[e] + x1[e] * sn[e];
      }
      Vec8<T>::store(out + base + j0, o1);
      Vec8<T>::store(out + base + half + j0, o2);
    } else {
      const int64_t off = r * W + (int64_t)(H + Hkv) * D + 8 * (k - nrot);
      float v[8];
      Vec8<T>::load(in + off, v);
      Vec8<T>::store(out + off, v);
    }
  }
}

// ------------------------------------------------------------------------------ int8 KV quant
// x [B, T, Hkv, D] -> q [B, Hkv, cap, D] int8 at pos.., scale [B, Hkv, cap] f32 (absmax/127)
template <typename T>
__global__ void __launch_bounds__(256) kv_quant_kernel(const T* __restrict__ x, int8_t* __restrict__ q,
                                                       float* __restrict__ scale, int Bn, int Tn, int Hkv, int D,
                                                       int cap, int pos) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);  // over B*T*Hkv
  if (row >= Bn * Tn * Hkv) return;
  const int h = row % Hkv;
  const int t = (row / Hkv) % Tn;
  const int b = row / (Hkv * Tn);
  const T* src = x + (size_t)row * D;
  float m = 0.f;
  for (int d = lane; d < D; d += 64) m = fmaxf(m, fabsf(to_f(src[d])));
  m = wave_max(m);
  float s = m / 127.f;
  if (s == 0.f) s = 1.f;
  const size_t slot = ((size_t)b * Hkv + h) * cap + pos + t;
  for (int d = lane; d < D; d += 64) {
    float v = rintf(to_f(src[d]) / s);
    v = fminf(fmaxf(v, -128.f), 127.f);
    q[slot * D + d] = (int8_t)v;
  }
  if (lane == 0) scale[slot] = s;
}

// ------------------------------------------------------------------------------ stats
// pass 1: per-block (sum, min, max); pass 2: per-block Σ(x-mean)^2 + LDS histogram.
template <typename T>
__global__ void __launch_bounds__(256) stats_pass1_kernel(const T* __restrict__ x, int64_t n,
                                                          float* __restrict__ part) {
  __shared__ float red[3][4];
  float s = 0.f, mn = INFINITY, mx = -INFINITY;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = to_f(x[i]);
    s += v;
    mn = fminf(mn, v);
    mx = fmaxf(mx, v);
  }
  s = wave_sum(s);
  mn = wave_min(mn);
  mx = wave_max(mx);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[0][w] = s; red[1][w] = mn; red[2][w] = mx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[blockIdx.x * 3 + 0] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    part[blockIdx.x * 3 + 1] = fminf(fminf(red[1][0], red[1][1]), fminf(red[1][2], red[1][3]));
    part[blockIdx.x * 3 + 2] = fmaxf(fmaxf(red[2][0], red[2][1]), fmaxf(red[2][2], red[2][3]));
  }
}

template <typename T>
__global__ void __launch_bounds__(256) stats_pass2_kernel(const T* __restrict__ x, int64_t n,
                                                          const float* __restrict__ mmm,  // mean, lo, hi
                                                          float* __restrict__ part, float* __restrict__ hist,
                                                          int bins) {
  extern __shared__ __attribute__((aligned(16))) float lh[];
  __shared__ float red[4];
  for (int b = threadIdx.x; b < bins; b += blockDim.x) lh[b] = 0.f;
  __syncthreads();
  const float mean = mmm[0], lo = mmm[1], hi = mmm[2];
  const float inv = bins / (hi - lo);
  float ss = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = to_f(x[i]);
    ss += (v - mean) * (v - mean);
    int b = (int)((v - lo) * inv);
    b = b < 0 ? 0 : (b >= bins ? bins - 1 : b);
    atomicAdd(&lh[b], 1.f);
  }
  ss = wave_sum(ss);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
  for (int b = threadIdx.x; b < bins; b += blockDim.x)
    if (lh[b] != 0.f) atomicAdd(&hist[b], lh[b]);
}

}  // namespace penroz

// ============================================================================ host side
using namespace penroz;

#define FOR_FLOAT_TYPES(t, NAME, ...)                                               \
  if ((t) == torch::kFloat32) { using NAME = float; __VA_ARGS__; }                  \
  else if ((t) == torch::kBFloat16) { using NAME = bf16; __VA_ARGS__; }             \
  else if ((t) == torch::kFloat16) { using NAME = __half; __VA_ARGS__; }            \
  else TORCH_CHECK(false, "unsupported dtype");

// PENROZ_EW_NT (non-temporal loads / stores, default on) and PENROZ_EW_GRID (workgroup cap of the
// grid-stride launches, default 8192) for the large streaming passes: GELU, gated activation,
// GELU backward + bias columns. Against the old plain / 2048 setting (profiles/ew_ab_r4.log):
// gelu_fwd 180-198 -> 146-152 us, GELU backward + columns 292 -> 246 us (GPT-2 shapes), gated
// forward 68 -> 58 us, gated backward 129 -> 109 us (Gemma-3 1B shapes).
static bool ew_nt() {
  const char* e = std::getenv("PENROZ_EW_NT");
  return e && *e ? std::atoi(e) != 0 : true;
}
static int ew_cap() {
  const char* e = std::getenv("PENROZ_EW_GRID");
  return e && *e ? std::max(1, std::atoi(e)) : 8192;
}

static inline int grid_for(int64_t work, int block = 256, int cap = 2048) {
  int64_t g = (work + block - 1) / block;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, cap));
}

static void check_vec8(const torch::Tensor& t) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "expected a contiguous GPU tensor");
  TORCH_CHECK(t.numel() % 8 == 0, "element count must be a multiple of 8");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "tensor must be 16-byte aligned");
}

void gelu_fwd(torch::Tensor x, int64_t approx, torch::Tensor y) {
  check_vec8(x);
  check_vec8(y);
  TORCH_CHECK(x.scalar_type() == y.scalar_type() && x.numel() == y.numel());
  const int64_t n8 = x.numel() / 8;
  auto stream = at::hip::getCurrentHIPStream();
  FOR_FLOAT_TYPES(x.scalar_type(), T,
    hipLaunchKernelGGL((ew_nt() ? gelu_fwd_kernel<T, true> : gelu_fwd_kernel<T, false>), dim3(grid_for(n8, 256, ew_cap())), dim3(256), 0, stream,
                       reinterpret_cast<const T*>(x.data_ptr()), reinterpret_cast<T*>(y.data_ptr()), n8, (int)approx))
}

static void colsum_impl(const torch::Tensor& a, const torch::Tensor* x, torch::Tensor* out, torch::Tensor& dst,
                        int approx, int mode) {
  const int N = a.size(0), F = a.size(1);
  TORCH_CHECK(F % 8 == 0, "column count must be a multiple of 8");
  TORCH_CHECK(dst.scalar_type() == torch::kFloat32 && dst.numel() == F && dst.is_contiguous());
  if (N == 0) return;
  const int ctiles = (F + 511) / 512;
  int R = std::max(1, std::min(N / 16, ew_cap() / ctiles));
  const bool nt = ew_nt();
  auto part = torch::empty({R, F}, a.options().dtype(torch::kFloat32));
  auto stream = at::hip::getCurrentHIPStream();
  FOR_FLOAT_TYPES(a.scalar_type(), T, {
    const T* ap = reinterpret_cast<const T*>(a.data_ptr());
    const T* xp = x ? reinterpret_cast<const T*>(x->data_ptr()) : nullptr;
    T* op = out ? reinterpret_cast<T*>(out->data_ptr()) : nullptr;
    if (mode == 0)
      hipLaunchKernelGGL((nt ? rows_colsum_kernel<0, T, true> : rows_colsum_kernel<0, T, false>), dim3(ctiles, R), dim3(256), 0, stream, ap, xp, op,
                         part.data_ptr<float>(), N, F, approx);
    else
      hipLaunchKernelGGL((nt ? rows_colsum_kernel<1, T, true> : rows_colsum_kernel<1, T, false>), dim3(ctiles, R), dim3(256), 0, stream, ap, xp, op,
                         part.data_ptr<float>(), N, F, approx);
  })
  float* outs[1] = {dst.data_ptr<float>()};
  reduce_partials_auto(part, 1, R, F, outs, stream);
}

void gelu_bwd(torch::Tensor dy, torch::Tensor x, int64_t approx, c10::optional<torch::Tensor> dbias,
              torch::Tensor out) {
  check_vec8(dy);
  check_vec8(x);
  check_vec8(out);
  TORCH_CHECK(dy.scalar_type() == x.scalar_type() && out.scalar_type() == x.scalar_type());
  TORCH_CHECK(dy.numel() == x.numel() && out.numel() == x.numel());
  auto stream = at::hip::getCurrentHIPStream();
  if (dbias.has_value() && dbias->defined()) {
    TORCH_CHECK(x.dim() == 2, "fused bias gradient needs a 2-D input");
    colsum_impl(dy, &x, &out, *dbias, (int)approx, 1);
    return;
  }
  const int64_t n8 = x.numel() / 8;
  FOR_FLOAT_TYPES(x.scalar_type(), T,
    hipLaunchKernelGGL((ew_nt() ? gelu_bwd_kernel<T, true> : gelu_bwd_kernel<T, false>), dim3(grid_for(n8, 256, ew_cap())), dim3(256), 0, stream,
                       reinterpret_cast<const T*>(dy.data_ptr()), reinterpret_cast<const T*>(x.data_ptr()),
                       reinterpret_cast<T*>(out.data_ptr()), n8, (int)approx))
}

void colsum(torch::Tensor x, torch::Tensor out) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.dim() == 2);
  colsum_impl(x, nullptr, nullptr, out, 0, 0);
}

torch::Tensor gated_act_fwd(torch::Tensor g, torch::Tensor u, int64_t kind) {
  check_vec8(g);
  check_vec8(u);
  auto y = torch::empty_like(g);
  const int64_t n8 = g.numel() / 8;
  auto stream = at::hip::getCurrentHIPStream();
  FOR_FLOAT_TYPES(g.scalar_type(), T,
    hipLaunchKernelGGL((ew_nt() ? gated_fwd_kernel<T, true> : gated_fwd_kernel<T, false>), dim3(grid_for(n8, 256, ew_cap())), dim3(256), 0, stream,
                       reinterpret_cast<const T*>(g.data_ptr()), reinterpret_cast<const T*>(u.data_ptr()),
                       reinterpret_cast<T*>(y.data_ptr()), n8, (int)kind))
  return y;
}

torch::Tensor gated_act_packed(torch::Tensor gu, int64_t kind, c10::optional<torch::Tensor> out) {
  TORCH_CHECK(gu.is_cuda() && gu.is_contiguous() && gu.dim() == 2 && gu.size(1) % 16 == 0, "gu: [N, 2I], I % 8 == 0");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(gu.data_ptr()) % 16 == 0);
  const int64_t N = gu.size(0), I = gu.size(1) / 2;
  torch::Tensor y;
  if (out.has_value() && out->defined()) {
    y = *out;
    TORCH_CHECK(y.is_contiguous() && y.numel() == N * I && y.scalar_type() == gu.scalar_type() &&
                    reinterpret_cast<uintptr_t>(y.data_ptr()) % 16 == 0,
                "gated_act_packed: out must be a contiguous 16-B aligned [N, I] tensor of gu's dtype");
  } else {
    y = torch::empty({N, I}, gu.options());
  }
  const int64_t n8 = N * I / 8;
  if (n8 == 0) return y;
  auto stream = at::hip::getCurrentHIPStream();
  FOR_FLOAT_TYPES(gu.scalar_type(), T,
    hipLaunchKernelGGL((ew_nt() ? gated_packed_kernel<T, true> : gated_packed_kernel<T, false>), dim3(grid_for(n8, 256, ew_cap())), dim3(256), 0, stream,
                       reinterpret_cast<const T*>(gu.data_ptr()), reinterpret_cast<T*>(y.data_ptr()), n8, (int)(I / 8),
                       (int)kind))
  return y;
}

std::vector<torch::Tensor> gated_act_bwd(torch::Tensor dy, torch::Tensor g, torch::Tensor u, int64_t kind) {
  check_vec8(dy);
  check_vec8(g);
  check_vec8(u);
  auto dg = torch::empty_like(g), du = torch::empty_like(u);
  const int64_t n8 = g.numel() / 8;
  auto stream = at::hip::getCurrentHIPStream();
  FOR_FLOAT_TYPES(g.scalar_type(), T,
    hipLaunchKernelGGL((ew_nt() ? gated_bwd_kernel<T, true> : gated_bwd_kernel<T, false>), dim3(grid_for(n8, 256, ew_cap())), dim3(256), 0, stream,
                       reinterpret_cast<const T*>(dy.data_ptr()), reinterpret_cast<const T*>(g.data_ptr()),
                       reinterpret_cast<const T*>(u.data_ptr()), reinterpret_cast<T*>(dg.data_ptr()),
                       reinterpret_cast<T*>(du.data_ptr()), n8, (int)kind))
  return {dg, du};
}

// dgu [N, 2I] (packed [d gate | d up]) from dy [N, I] and the packed forward input gu [N, 2I]
void gated_act_bwd_packed(torch::Tensor dy, torch::Tensor gu, torch::Tensor dgu, int64_t kind) {
  check_vec8(dy);
  check_vec8(gu);
  check_vec8(dgu);
  TORCH_CHECK(gu.dim() == 2 && gu.size(1) % 16 == 0 && dy.dim() == 2 && dy.size(0) == gu.size(0) &&
                  2 * dy.size(1) == gu.size(1) && dgu.sizes() == gu.sizes() && dy.scalar_type() == gu.scalar_type() &&
                  dgu.scalar_type() == gu.scalar_type(),
              "gated_act_bwd_packed: dy [N, I], gu / dgu [N, 2I], I % 8 == 0, one dtype");
  const int64_t I = dy.size(1), n8 = dy.numel() / 8;
  auto stream = at::hip::getCurrentHIPStream();
  FOR_FLOAT_TYPES(gu.scalar_type(), T,
    hipLaunchKernelGGL((ew_nt() ? gated_bwd_packed_kernel<T, true> : gated_bwd_packed_kernel<T, false>), dim3(grid_for(n8, 256, ew_cap())), dim3(256), 0, stream,
                       reinterpret_cast<const T*>(dy.data_ptr()), reinterpret_cast<const T*>(gu.data_ptr()),
                       reinterpret_cast<T*>(dgu.data_ptr()), n8, (int)(I / 8), (int)kind))
}

void embedding_fwd(torch::Tensor idx, torch::Tensor wte, torch::Tensor wpe, int64_t off, torch::Tensor out,
                   c10::optional<torch::Tensor> off_dev, double dropout_p, int64_t dropout_seed) {
  TORCH_CHECK(dropout_p >= 0.0 && dropout_p < 1.0, "dropout p must be in [0, 1)");
  TORCH_CHECK(idx.is_cuda() && idx.scalar_type() == torch::kInt64 && idx.dim() == 2);
  const int B = idx.size(0), T = idx.size(1), C = wte.size(1), V = wte.size(0);
  TORCH_CHECK(C % 8 == 0 && wpe.size(1) == C && wte.scalar_type() == wpe.scalar_type());
  const int64_t* od = nullptr;
  if (off_dev.has_value() && off_dev->defined()) {  // device offset: the caller bounds it (clamped here)
    TORCH_CHECK(off_dev->is_cuda() && off_dev->scalar_type() == torch::kInt64 && off_dev->numel() == 1);
    od = off_dev->data_ptr<int64_t>();
  } else {
    TORCH_CHECK(off + T <= wpe.size(0), "positions exceed the position table");
  }
  TORCH_CHECK(out.scalar_type() == torch::kFloat32 && out.numel() == (int64_t)B * T * C && out.is_contiguous());
  auto idxc = idx.contiguous();
  const int N = B * T;
  auto stream = at::hip::getCurrentHIPStream();
  FOR_FLOAT_TYPES(wte.scalar_type(), TW,
    hipLaunchKernelGGL(embed_fwd_kernel<TW>, dim3((N + 3) / 4), dim3(256), 0, stream, idxc.data_ptr<int64_t>(),
                       reinterpret_cast<const TW*>(wte.data_ptr()), reinterpret_cast<const TW*>(wpe.data_ptr()),
                       out.data_ptr<float>(), N, T, C, (int)off, V, od, (int)wpe.size(0), (uint64_t)dropout_seed,
                       (float)dropout_p))
}

void transpose_bf16(torch::Tensor in, torch::Tensor out) {
  TORCH_CHECK(in.is_cuda() && in.scalar_type() == torch::kBFloat16 && out.scalar_type() == torch::kBFloat16 &&
                  in.dim() == 2 && out.dim() == 2, "transpose_bf16: 2-D bf16");
  const int R = in.size(0), C = in.size(1);
  TORCH_CHECK(in.is_contiguous() && out.is_contiguous() && out.size(0) == C && out.size(1) == R,
              "transpose_bf16: out must be the contiguous [C, R]");
  TORCH_CHECK(R % 64 == 0 && C % 64 == 0, "transpose_bf16: dims must be multiples of 64");
  if (R == 0 || C == 0) return;
  auto stream = at::hip::getCurrentHIPStream();
  hipLaunchKernelGGL(transpose_bf16_kernel, dim3((R / 64) * (C / 64)), dim3(256), 0, stream,
                     reinterpret_cast<const uint16_t*>(in.data_ptr()), reinterpret_cast<uint16_t*>(out.data_ptr()), R, C);
}

void embedding_bwd(torch::Tensor dout, torch::Tensor idx, torch::Tensor dwte, torch::Tensor dwpe, int64_t off,
                   double dropout_p, int64_t dropout_seed) {
  TORCH_CHECK(dropout_p >= 0.0 && dropout_p < 1.0, "dropout p must be in [0, 1)");
  const int B = idx.size(0), T = idx.size(1), C = dwte.size(1), V = dwte.size(0);
  TORCH_CHECK(dout.scalar_type() == torch::kFloat32 && dwte.scalar_type() == torch::kFloat32 &&
              dwpe.scalar_type() == torch::kFloat32 && C % 4 == 0);
  TORCH_CHECK(off + T <= dwpe.size(0));
  auto idxc = idx.contiguous();
  const int N = B * T;
  auto stream = at::hip::getCurrentHIPStream();
  hipLaunchKernelGGL(embed_bwd_tok_kernel, dim3((N + 3) / 4), dim3(256), 0, stream, dout.data_ptr<float>(),
                     idxc.data_ptr<int64_t>(), dwte.data_ptr<float>(), N, C, V, (uint64_t)dropout_seed,
                     (float)dropout_p);
  hipLaunchKernelGGL(embed_bwd_pos_kernel, dim3(T), dim3(256), 0, stream, dout.data_ptr<float>(), dwpe.data_ptr<float>(),
                     B, T, C, (int)off, (uint64_t)dropout_seed, (float)dropout_p);
}

// out (optional): a preallocated contiguous tensor of qkv's shape and dtype (not aliasing qkv)
torch::Tensor rope_qkv(torch::Tensor qkv, torch::Tensor cosv, torch::Tensor sinv, int64_t H, int64_t Hkv, int64_t D,
                       bool inverse, c10::optional<torch::Tensor> out_opt) {
  TORCH_CHECK(qkv.is_cuda() && qkv.is_contiguous() && qkv.dim() == 3);
  const int64_t B = qkv.size(0), T = qkv.size(1);
  TORCH_CHECK(qkv.size(2) == (H + 2 * Hkv) * D && cosv.size(0) == T && cosv.size(1) == D / 2);
  torch::Tensor out;
  if (out_opt.has_value() && out_opt->defined()) {
    out = *out_opt;
    TORCH_CHECK(out.is_contiguous() && out.numel() == qkv.numel() && out.scalar_type() == qkv.scalar_type() &&
                    out.data_ptr() != qkv.data_ptr() && reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
                "rope_qkv: out must be a contiguous 16-B aligned tensor like qkv, not aliasing it");
    out = out.view(qkv.sizes());
  } else {
    out = torch::empty_like(qkv);
  }
  const int64_t rows = B * T;
  auto stream = at::hip::getCurrentHIPStream();
  const bool vec = D % 16 == 0 && cosv.is_contiguous() && sinv.is_contiguous() &&
                   cosv.scalar_type() == torch::kFloat32 && sinv.scalar_type() == torch::kFloat32 &&
                   reinterpret_cast<uintptr_t>(cosv.data_ptr()) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(sinv.data_ptr()) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(qkv.data_ptr()) % 16 == 0;
  if (vec) {
    const int64_t per = (H + Hkv) * (D / 16) + Hkv * D / 8;
    FOR_FLOAT_TYPES(qkv.scalar_type(), TT,
      hipLaunchKernelGGL(rope_vec_kernel<TT>, dim3(grid_for(rows * per)), dim3(256), 0, stream,
                         reinterpret_cast<const TT*>(qkv.data_ptr()), reinterpret_cast<TT*>(out.data_ptr()),
                         cosv.data_ptr<float>(), sinv.data_ptr<float>(), rows, (int)T, (int)H, (int)Hkv, (int)D,
                         inverse ? 1 : 0))
    return out;
  }
  FOR_FLOAT_TYPES(qkv.scalar_type(), TT,
    hipLaunchKernelGGL(rope_kernel<TT>, dim3(grid_for(rows * qkv.size(2))), dim3(256), 0, stream,
                       reinterpret_cast<const TT*>(qkv.data_ptr()), reinterpret_cast<TT*>(out.data_ptr()),
                       cosv.data_ptr<float>(), sinv.data_ptr<float>(), rows, (int)T, (int)H, (int)Hkv, (int)D,
                       inverse ? 1 : 0))
  return out;
}

void kv_quantize(torch::Tensor x, torch::Tensor q, torch::Tensor scale, int64_t pos) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.dim() == 4);
  const int B = x.size(0), T = x.size(1), Hkv = x.size(2), D = x.size(3);
  TORCH_CHECK(q.scalar_type() == torch::kInt8 && q.size(0) == B && q.size(1) == Hkv && q.size(3) == D);
  const int cap = q.size(2);
  TORCH_CHECK(pos + T <= cap, "cache overflow");
  const int rows = B * T * Hkv;
  auto stream = at::hip::getCurrentHIPStream();
  FOR_FLOAT_TYPES(x.scalar_type(), TT,
    hipLaunchKernelGGL(kv_quant_kernel<TT>, dim3((rows + 3) / 4), dim3(256), 0, stream,
                       reinterpret_cast<const TT*>(x.data_ptr()), q.data_ptr<int8_t>(), scale.data_ptr<float>(), B,
                       T, Hkv, D, cap, (int)pos))
}

std::vector<torch::Tensor> tensor_stats(torch::Tensor x, int64_t bins) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous());
  const int64_t n = x.numel();
  auto fopt = x.options().dtype(torch::kFloat32);
  if (n == 0) {
    auto z = torch::zeros({}, fopt);
    return {z, z, z, z, torch::zeros({bins}, fopt), torch::zeros({bins + 1}, fopt)};
  }
  const int G = grid_for(n, 256, 1024);
  auto p1 = torch::empty({G, 3}, fopt);
  auto stream = at::hip::getCurrentHIPStream();
  FOR_FLOAT_TYPES(x.scalar_type(), T,
    hipLaunchKernelGGL(stats_pass1_kernel<T>, dim3(G), dim3(256), 0, stream, reinterpret_cast<const T*>(x.data_ptr()),
                       n, p1.data_ptr<float>()))
  auto sum = p1.select(1, 0).to(torch::kFloat64).sum();
  auto mean = (sum / (double)n).to(torch::kFloat32);
  auto mn = p1.select(1, 1).min();
  auto mx = p1.select(1, 2).max();
  // torch.histogram widens an empty range by +-0.5 around a constant input
  auto same = mn.eq(mx);
  auto lo = torch::where(same, mn - 0.5f, mn);
  auto hi = torch::where(same, mx + 0.5f, mx);
  auto mmm = torch::stack({mean, lo, hi}).contiguous();
  auto p2 = torch::empty({G}, fopt);
  auto hist = torch::zeros({bins}, fopt);
  FOR_FLOAT_TYPES(x.scalar_type(), T,
    hipLaunchKernelGGL(stats_pass2_kernel<T>, dim3(G), dim3(256), bins * sizeof(float), stream,
                       reinterpret_cast<const T*>(x.data_ptr()), n, mmm.data_ptr<float>(), p2.data_ptr<float>(),
                       hist.data_ptr<float>(), (int)bins))
  auto var = p2.to(torch::kFloat64).sum() / (double)std::max<int64_t>(1, n - 1);
  auto stdv = var.sqrt().to(torch::kFloat32);
  auto edges = torch::linspace(0.0, 1.0, bins + 1, fopt) * (hi - lo) + lo;
  auto width = (hi - lo) / (double)bins;
  auto density = hist / ((double)n * width);
  return {mean, stdv, mn, mx, density, edges};
}

namespace penroz {
DeferredReduce& deferred_reduce() {
  static DeferredReduce d;
  return d;
}
}  // namespace penroz

// stream = 0: finish column reductions on the current stream (default)
void set_deferred_reduce_stream(int64_t stream, int64_t device) {
  penroz::deferred_reduce().stream = reinterpret_cast<hipStream_t>(stream);
  penroz::deferred_reduce().device = (int)device;
}
