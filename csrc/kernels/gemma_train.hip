// Residual combine + RMSNorm kernels of the fused Gemma training executor
// (models/gemma_executor.py). A Gemma block (reference neural_net_layers.py:188-225) joins each
// branch output `a` (attention O-projection or MLP down-projection, bf16) to the fp32 residual
// stream `x` and normalises the result for the next GEMM, with the family's post-norm variants:
//
//   mode 0 (Gemma 3+, post-norm on the residual): s = x + a;  h = RMS(s)·w1;  y = RMS(h)·w2
//   mode 1 (Gemma 2, post-norm on the branch):    h = x + RMS(a)·w1;          y = RMS(h)·w2
//   mode 2 (Gemma 1, no post-norms):              h = x + a;                  y = RMS(h)·w2
//   mode 3 (the first block's input norm):        h = x;                      y = RMS(x)·w2
//
// RMS(v)·w = v · rsqrt(mean(v²) + eps) · w in fp32 (HF Gemma's (1 + weight) is folded into w at
// import). h is the new residual (fp32), y the bf16 input of the next GEMM (the attention
// block's QKV, the MLP's gate|up, or — after the last block — the lm_head); w2 is the NEXT
// norm (pre-MLP, the next block's input norm, or the final norm), so one pass replaces the
// module path's residual add, one or two RMSNorms and their dtype glue.
//
// The backward of one combine takes dy (bf16, from the next GEMM's dgrad) and dh_in (fp32: the
// gradient of h through the residual path, from the LATER combine; absent for the last one) and
// produces dx (fp32 gradient of x, in place over dh_in allowed), da (bf16 gradient of the
// branch output, the input of the branch's dgrad GEMM) and per-wave partial rows of dw1, dw2
// (finished by the deterministic two-stage column reduction, on the deferred stream):
//   dh  = r2·w2·dy − h·r2³·mean(h·w2·dy) + dh_in            dw2 += dy·h·r2
//   mode 0: ds = r1·w1·dh − s·r1³·mean(s·w1·dh)  -> dx = da = ds,   dw1 += dh·s·r1
//   mode 1: dx = dh;  da = r1·w1·dh − a·r1³·mean(a·w1·dh),          dw1 += dh·a·r1
//   mode 2: dx = da = dh;   mode 3: dx = dh
// One wave per token row (lane l owns columns 4(l + 64j)); statistics are wave reductions.
#include "common.h"
#include "deferred.h"
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <cstdlib>

namespace penroz {

namespace {

template <int NCH>
struct RowF {  // one row's fp32 values owned by a lane: columns 4(lane + 64j) .. +3
  float v[NCH][4];
};

// NT: non-temporal row loads / stores (rows are streamed once; the weight loads stay plain)
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
template <bool NT, typename V>
__device__ __forceinline__ V ldv(const V* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT, typename V>
__device__ __forceinline__ void stv(V* p, V x) {
  if constexpr (NT) __builtin_nontemporal_store(x, p);
  else *p = x;
}

template <int NCH, bool NT = false>
__device__ __forceinline__ void ld_f32(RowF<NCH>& r, const float* p, int lane, int C) {
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int c = 4 * (lane + 64 * j);
    if (c < C) {
      const float4_t t = ldv<NT>(reinterpret_cast<const float4_t*>(p + c));
      r.v[j][0] = t[0]; r.v[j][1] = t[1]; r.v[j][2] = t[2]; r.v[j][3] = t[3];
    } else {
      r.v[j][0] = r.v[j][1] = r.v[j][2] = r.v[j][3] = 0.f;
    }
  }
}

template <int NCH, bool NT = false>
__device__ __forceinline__ void ld_bf16(RowF<NCH>& r, const bf16* p, int lane, int C) {
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int c = 4 * (lane + 64 * j);
    if (c < C) {
      const u32x2_t u = ldv<NT>(reinterpret_cast<const u32x2_t*>(p + c));
      r.v[j][0] = __uint_as_float(u.x << 16); r.v[j][1] = __uint_as_float(u.x & 0xffff0000u);
      r.v[j][2] = __uint_as_float(u.y << 16); r.v[j][3] = __uint_as_float(u.y & 0xffff0000u);
    } else {
      r.v[j][0] = r.v[j][1] = r.v[j][2] = r.v[j][3] = 0.f;
    }
  }
}

template <int NCH, bool NT = false>
__device__ __forceinline__ void st_f32(float* p, const RowF<NCH>& r, int lane, int C) {
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int c = 4 * (lane + 64 * j);
    if (c < C) stv<NT>(reinterpret_cast<float4_t*>(p + c), float4_t{r.v[j][0], r.v[j][1], r.v[j][2], r.v[j][3]});
  }
}

template <int NCH, bool NT = false>
__device__ __forceinline__ void st_bf16(bf16* p, const RowF<NCH>& r, int lane, int C) {
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int c = 4 * (lane + 64 * j);
    if (c < C)
      stv<NT>(reinterpret_cast<u32x2_t*>(p + c),
              u32x2_t{pack_bf16x2(r.v[j][0], r.v[j][1]), pack_bf16x2(r.v[j][2], r.v[j][3])});
  }
}

template <int NCH>
__device__ __forceinline__ float sumsq(const RowF<NCH>& r) {
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NCH; ++j)
#pragma unroll
    for (int k = 0; k < 4; ++k) s += r.v[j][k] * r.v[j][k];
  return wave_sum(s);
}

// w (fp32 [C]) at this lane's columns
template <int NCH>
__device__ __forceinline__ void ld_w(RowF<NCH>& r, const float* w, int lane, int C) {
  ld_f32<NCH>(r, w, lane, C);
}

}  // namespace

template <int NCH, bool NT = false>
__global__ void __launch_bounds__(256) gm_combine_fwd_kernel(int mode, const float* __restrict__ x,
                                                             const bf16* __restrict__ a, const float* __restrict__ w1,
                                                             const float* __restrict__ w2, float eps1, float eps2,
                                                             float* __restrict__ h_out, bf16* __restrict__ y_out,
                                                             float* __restrict__ s_save, float* __restrict__ r1_out,
                                                             float* __restrict__ r2_out, int N, int C) {
  const int lane = threadIdx.x & 63;
  const float inv_c = 1.f / (float)C;
  for (int row = blockIdx.x * 4 + (threadIdx.x >> 6); row < N; row += gridDim.x * 4) {
    const size_t base = (size_t)row * C;
    RowF<NCH> h;
    ld_f32<NCH, NT>(h, x + base, lane, C);
    if (mode != 3) {
      RowF<NCH> av, wv;
      ld_bf16<NCH, NT>(av, a + base, lane, C);
      if (mode == 1) {  // h = x + RMS(a)·w1
        ld_w<NCH>(wv, w1, lane, C);
        const float r1 = rsqrtf(sumsq<NCH>(av) * inv_c + eps1);
        if (lane == 0) r1_out[row] = r1;
#pragma unroll
        for (int j = 0; j < NCH; ++j)
#pragma unroll
          for (int k = 0; k < 4; ++k) h.v[j][k] += av.v[j][k] * r1 * wv.v[j][k];
      } else {
#pragma unroll
        for (int j = 0; j < NCH; ++j)
#pragma unroll
          for (int k = 0; k < 4; ++k) h.v[j][k] += av.v[j][k];
        if (mode == 0) {  // s = x + a (kept for the backward); h = RMS(s)·w1
          st_f32<NCH, NT>(s_save + base, h, lane, C);
          ld_w<NCH>(wv, w1, lane, C);
          const float r1 = rsqrtf(sumsq<NCH>(h) * inv_c + eps1);
          if (lane == 0) r1_out[row] = r1;
#pragma unroll
          for (int j = 0; j < NCH; ++j)
#pragma unroll
            for (int k = 0; k < 4; ++k) h.v[j][k] *= r1 * wv.v[j][k];
        }
      }
      st_f32<NCH, NT>(h_out + base, h, lane, C);
    }
    RowF<NCH> wv2;
    ld_w<NCH>(wv2, w2, lane, C);
    const float r2 = rsqrtf(sumsq<NCH>(h) * inv_c + eps2);
    if (lane == 0) r2_out[row] = r2;
#pragma unroll
    for (int j = 0; j < NCH; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k) h.v[j][k] *= r2 * wv2.v[j][k];
    st_bf16<NCH, NT>(y_out + base, h, lane, C);
  }
}

// part: fp32 [2][gridDim.x][C] — this workgroup's dw1 (row block 0) and dw2 (row block 1) sums
template <int NCH, bool NT = false>
__global__ void __launch_bounds__(256) gm_combine_bwd_kernel(int mode, const bf16* __restrict__ dy,
                                                             const float* __restrict__ dh_in,
                                                             const float* __restrict__ h_save,
                                                             const float* __restrict__ s_save,
                                                             const bf16* __restrict__ a_save,
                                                             const float* __restrict__ r1_in,
                                                             const float* __restrict__ r2_in,
                                                             const float* __restrict__ w1, const float* __restrict__ w2,
                                                             float* __restrict__ dx, bf16* __restrict__ da,
                                                             float* __restrict__ dh_save, float* __restrict__ part,
                                                             int N, int C) {
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
  const float inv_c = 1.f / (float)C;
  RowF<NCH> p1, p2;
#pragma unroll
  for (int j = 0; j < NCH; ++j)
#pragma unroll
    for (int k = 0; k < 4; ++k) p1.v[j][k] = p2.v[j][k] = 0.f;
  for (int row = gw; row < N; row += nw) {
    const size_t base = (size_t)row * C;
    RowF<NCH> g, hv, wv;
    ld_bf16<NCH, NT>(g, dy + base, lane, C);
    ld_f32<NCH, NT>(hv, h_save + base, lane, C);
    ld_w<NCH>(wv, w2, lane, C);
    const float r2 = r2_in[row];
    float dot = 0.f;
#pragma unroll
    for (int j = 0; j < NCH; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float gw2 = g.v[j][k] * wv.v[j][k];
        dot += gw2 * hv.v[j][k];
        p2.v[j][k] += g.v[j][k] * hv.v[j][k] * r2;
        g.v[j][k] = gw2;  // g now holds dy·w2
      }
    const float c2 = wave_sum(dot) * inv_c * r2 * r2 * r2;
    RowF<NCH> dh;
    if (dh_in != nullptr) ld_f32<NCH, NT>(dh, dh_in + base, lane, C);
    else {
#pragma unroll
      for (int j = 0; j < NCH; ++j)
#pragma unroll
        for (int k = 0; k < 4; ++k) dh.v[j][k] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < NCH; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k) dh.v[j][k] += r2 * g.v[j][k] - hv.v[j][k] * c2;
    if (dh_save != nullptr) st_f32<NCH, NT>(dh_save + base, dh, lane, C);  // diagnostics: dL/dh
    if (mode == 0 || mode == 1) {
      RowF<NCH> sv;  // the post-norm's input: s (mode 0) or a (mode 1)
      if (mode == 0) ld_f32<NCH, NT>(sv, s_save + base, lane, C);
      else ld_bf16<NCH, NT>(sv, a_save + base, lane, C);
      ld_w<NCH>(wv, w1, lane, C);
      const float r1 = r1_in[row];
      float dot1 = 0.f;
#pragma unroll
      for (int j = 0; j < NCH; ++j)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          dot1 += dh.v[j][k] * wv.v[j][k] * sv.v[j][k];
          p1.v[j][k] += dh.v[j][k] * sv.v[j][k] * r1;
        }
      const float c1 = wave_sum(dot1) * inv_c * r1 * r1 * r1;
      RowF<NCH> dn;  // gradient of the post-norm's input
#pragma unroll
      for (int j = 0; j < NCH; ++j)
#pragma unroll
        for (int k = 0; k < 4; ++k) dn.v[j][k] = r1 * wv.v[j][k] * dh.v[j][k] - sv.v[j][k] * c1;
      if (mode == 0) {
        st_f32<NCH, NT>(dx + base, dn, lane, C);
        st_bf16<NCH, NT>(da + base, dn, lane, C);
      } else {
        st_f32<NCH, NT>(dx + base, dh, lane, C);
        st_bf16<NCH, NT>(da + base, dn, lane, C);
      }
    } else {
      st_f32<NCH, NT>(dx + base, dh, lane, C);
      if (mode == 2) st_bf16<NCH, NT>(da + base, dh, lane, C);
    }
  }
  // the workgroup's 4 wave partials summed through LDS in wave order (deterministic): one partial
  // row per workgroup and weight
  extern __shared__ __attribute__((aligned(16))) float red[];  // [4][C]
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    st_f32<NCH>(red + (size_t)w * C, pass == 0 ? p1 : p2, lane, C);
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256)
      part[((size_t)pass * gridDim.x + blockIdx.x) * C + c] = (red[c] + red[C + c]) + (red[2 * C + c] + red[3 * C + c]);
    __syncthreads();
  }
}

}  // namespace penroz

using namespace penroz;

#define PENROZ_GM_NCH(C, ...)                                   \
  [&] {                                                         \
    const int need = (int)((C + 255) / 256);                    \
    if (need <= 2) { constexpr int NCH = 2; __VA_ARGS__; }      \
    else if (need <= 3) { constexpr int NCH = 3; __VA_ARGS__; } \
    else if (need <= 5) { constexpr int NCH = 5; __VA_ARGS__; } \
    else if (need <= 8) { constexpr int NCH = 8; __VA_ARGS__; } \
    else if (need <= 10) { constexpr int NCH = 10; __VA_ARGS__; } \
    else if (need <= 12) { constexpr int NCH = 12; __VA_ARGS__; } \
    else if (need <= 16) { constexpr int NCH = 16; __VA_ARGS__; } \
    else { constexpr int NCH = 24; __VA_ARGS__; }               \
  }()

static void gm_check_rows(const torch::Tensor& t, int64_t N, int64_t C, c10::ScalarType dt, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.numel() == N * C && t.scalar_type() == dt &&
                  reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              "gemma combine: ", what, " must be a contiguous 16-B aligned [N, C] tensor of the expected dtype");
}

static void gm_check_vec(const c10::optional<torch::Tensor>& t, int64_t n, const char* what) {
  TORCH_CHECK(t.has_value() && t->defined() && t->is_cuda() && t->is_contiguous() && t->numel() == n &&
                  t->scalar_type() == torch::kFloat32,
              "gemma combine: ", what, " must be a contiguous fp32 vector of ", n, " elements");
}

// 4 rows in flight per workgroup, up to 4 workgroups per CU: enough waves to overlap each row's
// memory latency (a one-workgroup-per-CU grid ran the backward 2.4x off its HBM roofline)
static int gm_grid(int64_t N) {
  const char* e = std::getenv("PENROZ_GM_GRID");
  const int64_t cap = e && *e ? std::max(1, std::atoi(e)) : 1024;
  return (int)std::min<int64_t>((N + 3) / 4, cap);
}

// PENROZ_GM_NT: non-temporal row loads / stores in the combine kernels (default on: Gemma-3 1B B=8
// 68.65 / 68.57 -> 68.24 / 68.33 ms; a 2048-workgroup cap was slower either way, ew_ab_r4.log)
static bool gm_nt() {
  const char* e = std::getenv("PENROZ_GM_NT");
  return e && *e ? std::atoi(e) != 0 : true;
}

// see the file header; x fp32 [N, C]; a bf16 [N, C] (modes 0-2); h_out fp32 (modes 0-2);
// y_out bf16; s_save fp32 (mode 0); r1 fp32 [N] (modes 0, 1); r2 fp32 [N]
void gemma_combine_fwd(int64_t mode, torch::Tensor x, c10::optional<torch::Tensor> a, c10::optional<torch::Tensor> w1,
                       torch::Tensor w2, double eps1, double eps2, c10::optional<torch::Tensor> h_out, torch::Tensor y_out,
                       c10::optional<torch::Tensor> s_save, c10::optional<torch::Tensor> r1, torch::Tensor r2) {
  TORCH_CHECK(mode >= 0 && mode <= 3, "gemma combine: mode 0..3");
  const int64_t N = x.size(0), C = x.size(1);
  TORCH_CHECK(x.dim() == 2 && C % 4 == 0 && C <= 6144, "gemma combine: C % 4 == 0, C <= 6144");
  gm_check_rows(x, N, C, torch::kFloat32, "x");
  gm_check_rows(y_out, N, C, torch::kBFloat16, "y");
  TORCH_CHECK(w2.is_contiguous() && w2.numel() == C && w2.scalar_type() == torch::kFloat32, "gemma combine: w2");
  TORCH_CHECK(r2.numel() == N && r2.scalar_type() == torch::kFloat32, "gemma combine: r2");
  if (mode != 3) {
    TORCH_CHECK(a.has_value() && h_out.has_value(), "gemma combine: a and h_out needed");
    gm_check_rows(*a, N, C, torch::kBFloat16, "a");
    gm_check_rows(*h_out, N, C, torch::kFloat32, "h_out");
  }
  if (mode == 0 || mode == 1) {
    gm_check_vec(w1, C, "w1");
    gm_check_vec(r1, N, "r1");
  }
  if (mode == 0) gm_check_rows(*s_save, N, C, torch::kFloat32, "s_save");
  if (N == 0) return;
  auto stream = at::hip::getCurrentHIPStream();
  PENROZ_GM_NCH(C, hipLaunchKernelGGL((gm_nt() ? gm_combine_fwd_kernel<NCH, true> : gm_combine_fwd_kernel<NCH, false>), dim3(gm_grid(N)), dim3(256), 0, stream, (int)mode,
                                      x.data_ptr<float>(),
                                      mode != 3 ? reinterpret_cast<const bf16*>(a->data_ptr()) : nullptr,
                                      (mode == 0 || mode == 1) ? w1->data_ptr<float>() : nullptr, w2.data_ptr<float>(),
                                      (float)eps1, (float)eps2, mode != 3 ? h_out->data_ptr<float>() : nullptr,
                                      reinterpret_cast<bf16*>(y_out.data_ptr()),
                                      mode == 0 ? s_save->data_ptr<float>() : nullptr,
                                      (mode == 0 || mode == 1) ? r1->data_ptr<float>() : nullptr, r2.data_ptr<float>(),
                                      (int)N, (int)C));
}

// dy bf16 [N, C]; dh_in fp32 (optional; may alias dx); h fp32 (mode 3: x); s fp32 (mode 0);
// a bf16 (mode 1); dx fp32 out; da bf16 out (modes 0-2); dw1 (modes 0, 1) / dw2 fp32 [C]
// accumulated (+=) through the two-stage column reduction; dh_save (optional): dL/dh
void gemma_combine_bwd(int64_t mode, torch::Tensor dy, c10::optional<torch::Tensor> dh_in, torch::Tensor h,
                       c10::optional<torch::Tensor> s_save, c10::optional<torch::Tensor> a_save,
                       c10::optional<torch::Tensor> r1, torch::Tensor r2, c10::optional<torch::Tensor> w1,
                       torch::Tensor w2, torch::Tensor dx, c10::optional<torch::Tensor> da,
                       c10::optional<torch::Tensor> dw1, torch::Tensor dw2, c10::optional<torch::Tensor> dh_save) {
  TORCH_CHECK(mode >= 0 && mode <= 3, "gemma combine: mode 0..3");
  const int64_t N = h.size(0), C = h.size(1);
  TORCH_CHECK(h.dim() == 2 && C % 4 == 0 && C <= 6144, "gemma combine: C % 4 == 0, C <= 6144");
  gm_check_rows(dy, N, C, torch::kBFloat16, "dy");
  gm_check_rows(h, N, C, torch::kFloat32, "h");
  gm_check_rows(dx, N, C, torch::kFloat32, "dx");
  const float* dhp = nullptr;
  if (dh_in.has_value() && dh_in->defined()) {
    gm_check_rows(*dh_in, N, C, torch::kFloat32, "dh_in");
    dhp = dh_in->data_ptr<float>();
  }
  TORCH_CHECK(w2.numel() == C && w2.scalar_type() == torch::kFloat32 && dw2.numel() == C &&
                  dw2.scalar_type() == torch::kFloat32 && r2.numel() == N,
              "gemma combine: w2 / dw2 [C], r2 [N] fp32");
  const bool post = mode == 0 || mode == 1;
  if (post) {
    gm_check_vec(w1, C, "w1");
    gm_check_vec(dw1, C, "dw1");
    gm_check_vec(r1, N, "r1");
  }
  if (mode == 0) gm_check_rows(*s_save, N, C, torch::kFloat32, "s_save");
  if (mode == 1) gm_check_rows(*a_save, N, C, torch::kBFloat16, "a_save");
  if (mode != 3) {
    TORCH_CHECK(da.has_value() && da->defined(), "gemma combine: da needed");
    gm_check_rows(*da, N, C, torch::kBFloat16, "da");
  }
  float* dhs = nullptr;
  if (dh_save.has_value() && dh_save->defined()) {
    gm_check_rows(*dh_save, N, C, torch::kFloat32, "dh_save");
    dhs = dh_save->data_ptr<float>();
  }
  if (N == 0) return;
  const int grid = gm_grid(N), G = grid;
  auto part = torch::empty({2, G, C}, h.options());
  auto stream = at::hip::getCurrentHIPStream();
  PENROZ_GM_NCH(C, hipLaunchKernelGGL((gm_nt() ? gm_combine_bwd_kernel<NCH, true> : gm_combine_bwd_kernel<NCH, false>), dim3(grid), dim3(256), 4 * C * sizeof(float),
                                      stream, (int)mode,
                                      reinterpret_cast<const bf16*>(dy.data_ptr()), dhp, h.data_ptr<float>(),
                                      mode == 0 ? s_save->data_ptr<float>() : nullptr,
                                      mode == 1 ? reinterpret_cast<const bf16*>(a_save->data_ptr()) : nullptr,
                                      post ? r1->data_ptr<float>() : nullptr, r2.data_ptr<float>(),
                                      post ? w1->data_ptr<float>() : nullptr, w2.data_ptr<float>(), dx.data_ptr<float>(),
                                      mode != 3 ? reinterpret_cast<bf16*>(da->data_ptr()) : nullptr, dhs,
                                      part.data_ptr<float>(), (int)N, (int)C));
  // partial rows: [0] dw1 (zeros unless a post-norm), [1] dw2
  if (post) {
    float* outs[2] = {dw1->data_ptr<float>(), dw2.data_ptr<float>()};
    reduce_partials_auto(part, 2, G, (int)C, outs, stream);
  } else {
    float* outs[1] = {dw2.data_ptr<float>()};
    reduce_partials_auto(part.narrow(0, 1, 1), 1, G, (int)C, outs, stream);
  }
}
