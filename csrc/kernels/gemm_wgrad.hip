// Weight-gradient GEMM for MI355X:  G[M][N] (+)= Σ_k A[k][M] · B[k][N]   (bf16 in, fp32 out)
//
// For a linear y = x·Wᵀ: A = dY [tokens, out], B = X [tokens, in], G = dW [out, in]. Both
// operands are row-major in the reduction dimension k (tokens), which is what makes this GEMM
// awkward for library kernels at GPT-2 shapes (hipBLASLt measured 280–670 TF here: tiny M×N,
// K = 65 536).  Design:
//   * 128×128 output tile per 256-thread workgroup (4 waves, 2×2 of 64×64 = 2×2 MFMA
//     32x32x16 tiles each), k-step 64;
//   * both operand tiles are staged row-major [64 k][128] in LDS (16-B global loads, issued one
//     k-step ahead into registers, written after the MFMAs — T14) and consumed column-wise
//     with ds_read_b64_tr_b16, so no transposes in memory; 256-B rows use the XOR swizzle
//     ch ^ ((row&3)<<2 | (row>>2)&3), which makes the 4-row × 4-chunk transposed half-wave
//     reads bank-conflict-free;
//   * split-K over tokens to put ≥ 512 workgroups on 256 CUs; each split writes an fp32
//     slab and a deterministic column-ordered reduction adds the slabs into the gradient
//     buffer (fused accumulate, bitwise reproducible); one split => direct read-add-write;
//   * XCD-aware bijective block remap: a contiguous chunk of (split, tile) pairs per XCD so
//     workgroups sharing a k-range and an operand panel share that XCD's L2.
#include "common.h"
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

namespace penroz {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int BM = 128, BN = 128, BK = 64;

__device__ __forceinline__ f32x16 mfma32(uint4 a, uint4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                 0, 0, 0);
}

__device__ __forceinline__ int off256(int row, int ch) {
  return row * 256 + ((ch ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4);
}

__device__ __forceinline__ uint2 tr_read(const char* tile, int row, int col) {
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(tile + off256(row, col >> 3) + ((col & 4) << 1)));
  return __builtin_bit_cast(uint2, v);
}

// element j = tile[rbase + 8(j>>2) + 4hh + (j&3)][cbase + (lane&31)]
__device__ __forceinline__ uint4 tr_frag(const char* tile, int rbase, int cbase, int lane) {
  const int hh = lane >> 5, q = (lane & 15) >> 2, p = lane & 3;
  const int col = cbase + 16 * ((lane >> 4) & 1) + 4 * p;
  const uint2 a = tr_read(tile, rbase + 4 * hh + q, col);
  const uint2 b = tr_read(tile, rbase + 8 + 4 * hh + q, col);
  return uint4{a.x, a.y, b.x, b.y};
}

__global__ void __launch_bounds__(256, 2) wgrad_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                       float* __restrict__ out, int M, int N, int K, int lda, int ldb,
                                                       int klen, int tiles_m, int tiles_n, int direct) {
  __shared__ __attribute__((aligned(16))) char smem[2][2][BK * 256];
  // XCD-aware bijective remap (blocks b and b+8 share an XCD under round-robin dispatch)
  const int nwg = gridDim.x, wg = blockIdx.x;
  const int xcd = wg & 7, qd = nwg >> 3, rd = nwg & 7;
  const int id = (xcd < rd ? xcd * (qd + 1) : rd * (qd + 1) + (xcd - rd) * qd) + (wg >> 3);
  const int ntiles = tiles_m * tiles_n;
  const int split = id / ntiles, tile = id - split * ntiles;
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int k0 = split * klen, k1 = min(K, k0 + klen);
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), hh = lane >> 5;
  const int wm = w >> 1, wn = w & 1;

  // staging: thread t -> row r = t>>2 of the k-tile, chunks 4(t&3)..+3 (8 bf16 each)
  const int sr = threadIdx.x >> 2, sc = 4 * (threadIdx.x & 3);
  uint4 ast[4], bst[4];
  auto gload = [&](int kk) {
    const int k = kk + sr;
    const bool kok = k < k1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int mc = m0 + 8 * (sc + i), nc = n0 + 8 * (sc + i);
      ast[i] = (kok && mc < M) ? *reinterpret_cast<const uint4*>(A + (size_t)k * lda + mc) : uint4{0, 0, 0, 0};
      bst[i] = (kok && nc < N) ? *reinterpret_cast<const uint4*>(B + (size_t)k * ldb + nc) : uint4{0, 0, 0, 0};
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      *reinterpret_cast<uint4*>(smem[buf][0] + off256(sr, sc + i)) = ast[i];
      *reinterpret_cast<uint4*>(smem[buf][1] + off256(sr, sc + i)) = bst[i];
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nsteps = (k1 - k0 + BK - 1) / BK;
  if (nsteps > 0) {
    gload(k0);
    lstore(0);
  }
  __syncthreads();
  for (int st = 0; st < nsteps; ++st) {
    if (st + 1 < nsteps) gload(k0 + (st + 1) * BK);
    const char* At = smem[st & 1][0];
    const char* Bt = smem[st & 1][1];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      uint4 af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = tr_frag(At, 16 * s, 64 * wm + 32 * i, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[j] = tr_frag(Bt, 16 * s, 64 * wn + 32 * j, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(af[i], bf[j], acc[i][j]);
    }
    if (st + 1 < nsteps) lstore((st + 1) & 1);
    __syncthreads();
  }
  // epilogue: row m = m0 + 64wm + 32i + acc_row(r), col n = n0 + 64wn + 32j + (lane&31)
  float* o = direct ? out : out + (size_t)split * M * N;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + 64 * wn + 32 * j + (lane & 31);
      if (n >= N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + 64 * wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hh;
        if (m < M) {
          float* p = o + (size_t)m * N + n;
          if (direct) *p += acc[i][j][r];
          else *p = acc[i][j][r];
        }
      }
    }
}

// G[e] += Σ_s slab[s][e]  (vectorised, fixed order)
__global__ void __launch_bounds__(256) slab_reduce_kernel(const float* __restrict__ slab, float* __restrict__ g,
                                                          int64_t n4, int splits, int64_t stride4) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4_t acc = reinterpret_cast<float4_t*>(g)[i];
    for (int s = 0; s < splits; ++s) acc += reinterpret_cast<const float4_t*>(slab)[s * stride4 + i];
    reinterpret_cast<float4_t*>(g)[i] = acc;
  }
}

}  // namespace
}  // namespace penroz

using namespace penroz;

// grad[M][N] += dyᵀ·x with dy [K, M], x [K, N] (bf16, row-major, contiguous rows)
void wgrad_gemm(torch::Tensor dy, torch::Tensor x, torch::Tensor grad) {
  TORCH_CHECK(dy.is_cuda() && x.is_cuda() && grad.is_cuda());
  TORCH_CHECK(dy.scalar_type() == torch::kBFloat16 && x.scalar_type() == torch::kBFloat16 &&
              grad.scalar_type() == torch::kFloat32, "wgrad: bf16 operands, fp32 gradient");
  TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && dy.size(0) == x.size(0), "wgrad: [K, M] x [K, N]");
  TORCH_CHECK(dy.stride(1) == 1 && x.stride(1) == 1 && grad.is_contiguous());
  const int K = dy.size(0), M = dy.size(1), N = x.size(1);
  TORCH_CHECK(grad.size(0) == M && grad.size(1) == N, "wgrad: gradient shape mismatch");
  TORCH_CHECK(M % 8 == 0 && N % 8 == 0 && dy.stride(0) % 8 == 0 && x.stride(0) % 8 == 0,
              "wgrad: widths and row strides must be multiples of 8");
  if (K == 0) return;
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int ntiles = tiles_m * tiles_n;
  int splits = std::max(1, std::min((512 + ntiles - 1) / ntiles, K / 512));
  int klen = ((K + splits - 1) / splits + BK - 1) / BK * BK;
  splits = (K + klen - 1) / klen;
  auto stream = at::hip::getCurrentHIPStream();
  const int nwg = ntiles * splits;
  const bf16* a = reinterpret_cast<const bf16*>(dy.data_ptr());
  const bf16* b = reinterpret_cast<const bf16*>(x.data_ptr());
  if (splits == 1) {
    hipLaunchKernelGGL(wgrad_kernel, dim3(nwg), dim3(256), 0, stream, a, b, grad.data_ptr<float>(), M, N, K,
                       (int)dy.stride(0), (int)x.stride(0), klen, tiles_m, tiles_n, 1);
    return;
  }
  auto slab = torch::empty({(int64_t)splits * M * N}, grad.options());
  hipLaunchKernelGGL(wgrad_kernel, dim3(nwg), dim3(256), 0, stream, a, b, slab.data_ptr<float>(), M, N, K,
                     (int)dy.stride(0), (int)x.stride(0), klen, tiles_m, tiles_n, 0);
  const int64_t n4 = (int64_t)M * N / 4;
  hipLaunchKernelGGL(slab_reduce_kernel, dim3((int)std::min<int64_t>((n4 + 255) / 256, 2048)), dim3(256), 0, stream,
                     slab.data_ptr<float>(), grad.data_ptr<float>(), n4, splits, n4);
}
