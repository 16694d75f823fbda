// Weight-gradient GEMM for MI355X:  G[M][N] (+)= Σ_k A[k][M] · B[k][N]   (bf16 in, fp32 out)
//
// For a linear y = x·Wᵀ: A = dY [tokens, out], B = X [tokens, in], G = dW [out, in]. Both
// operands are row-major in the reduction dimension k (tokens), which is what makes this GEMM
// awkward for library kernels at GPT-2 shapes (hipBLASLt measured 270–980 TF here, 410–1000 TF
// tuned: profiles/wgrad_native_vs_hipblaslt_r2.log).  Design (default path =
// wgrad256_ring16o_kernel<32, 4, true>, variant 8):
//   * 256×256 output tile per 512-thread workgroup (8 waves as 2×4, each 128×64 = 8×4 MFMA
//     16x16x32 tiles), one workgroup per CU (128 KiB LDS);
//   * operand tiles arrive by LDS-DMA (global_load_lds_dwordx4, issued in inline asm so the
//     compiler does not serialise it against ds_reads) into a 4-stage ring of [32 k][256]
//     tiles; three stages are in flight and the end-of-step wait is a counted vmcnt; DMA
//     sources are a scalar row base plus a per-lane offset fixed for the kernel;
//   * tiles are consumed column-wise with ds_read_b64_tr_b16 (no transposes in memory); the
//     512-B rows use an XOR swizzle of the 16-B chunk (swz16), applied on the DMA SOURCE
//     address because the DMA destination is lane-linear; per-lane fragment offsets are
//     computed once;
//   * split-K over tokens chosen by a wave-quantisation cost model; each split writes an fp32
//     slab and a deterministic fixed-order reduction adds the slabs into the gradient buffer
//     (bitwise reproducible); one split => direct read-add-write;
//   * XCD-aware bijective block remap: a contiguous chunk of (split, tile) pairs per XCD so
//     workgroups sharing a k-range and an operand panel share that XCD's L2.
// wgrad_kernel (128×128, 4 waves, register staging; tile=128) and wgrad256_ring16_kernel
// (variant 4, the round-1 default) stay selectable for A/B measurement.
#include "common.h"
#include "host_plan.h"
#include <cstdlib>
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

  // staging: consecutive lanes take consecutive 16-B chunks of a row (coalesced global
  // loads; every 8-lane ds_write_b128 group covers 8 distinct chunks = all 32 banks):
  // thread t -> chunk t&15 of rows (t>>4) + 16i, i = 0..3
  const int sr = threadIdx.x >> 4, sc = threadIdx.x & 15;
  uint4 ast[4], bst[4];
  auto gload = [&](int kk) {
    const int mc = m0 + 8 * sc, nc = n0 + 8 * sc;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = kk + sr + 16 * i;
      const bool kok = k < k1;
      ast[i] = (kok && mc < M) ? *reinterpret_cast<const uint4*>(A + (size_t)k * lda + mc) : uint4{0, 0, 0, 0};
      bst[i] = (kok && nc < N) ? *reinterpret_cast<const uint4*>(B + (size_t)k * ldb + nc) : uint4{0, 0, 0, 0};
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      *reinterpret_cast<uint4*>(smem[buf][0] + off256(sr + 16 * i, sc)) = ast[i];
      *reinterpret_cast<uint4*>(smem[buf][1] + off256(sr + 16 * i, sc)) = bst[i];
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


// ---------------------------------------------------------------------------------------
// 256×256 tile, 8 waves (2 along M × 4 along N, each wave 128×64). Per 32-deep k-step: 32 KiB
// of operands for 2·256·256·32 FLOP = 128 FLOP/B (the 128² tile's 64 FLOP/B left it
// L2-bandwidth-bound at 320–500 TF). LDS rows are 512 B. (The 32x32x16 and register-staged
// 256-tile variants of round 1 measured slower and were removed.)
constexpr int BM2 = 256, BN2 = 256, BK2 = 32;

// ---- 16x16x32 MFMA variant ---------------------------------------------------------------
// LDS-DMA ring: NBUF stages of BKT k-rows; tile t+NBUF-1 is issued while tile t is consumed,
// and the end-of-step wait is a counted vmcnt that leaves NBUF-2 tiles in flight across the
// barrier (tiles beyond the split's range DMA the zero page, so the count is uniform).
// Each wave's 128×64 output is 8×4 tiles of v_mfma_f32_16x16x32_bf16 (the
// 16x16 shape holds a higher clock than 32x32x16 on random data at equal cycles per FLOP).
// Operand fragment (A or B, from a [k][256] tile): lane l holds k = 8·(l>>4) + j, j = 0..7, of
// column c0 + (l&15) — two ds_read_b64_tr_b16 (rows 8g..8g+3 and 8g+4..8g+7 of its 16-lane
// group g). One 32-lane read group then covers rows {0-3, 8-11} (or {4-7, 12-15}) × two 16-B
// chunks; the swizzle ch ^ ((row&3)<<2 | ((row>>3)&1)<<1) puts those 16 pieces on 16 distinct
// bank slots.
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma16(uint4 a, uint4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                 0, 0, 0);
}

__device__ __forceinline__ int swz16(int row) { return ((row & 3) << 2) | (((row >> 3) & 1) << 1); }

__device__ __forceinline__ int off512b(int row, int ch) { return row * 512 + ((ch ^ swz16(row)) << 4); }

// element j = tile[kbase + 8·(lane>>4) + j][c0 + (lane&15)]
__device__ __forceinline__ uint4 tr_frag16(const char* tile, int kbase, int c0, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int col = c0 + 4 * p;
  const int r0 = kbase + 8 * g + q;
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4*)(tile + off512b(r0, col >> 3) + ((col & 4) << 1)));
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4*)(tile + off512b(r0 + 4, col >> 3) + ((col & 4) << 1)));
  const uint2 ua = __builtin_bit_cast(uint2, a), ub = __builtin_bit_cast(uint2, b);
  return uint4{ua.x, ua.y, ub.x, ub.y};
}

template <int BKT, int NBUF>
__global__ void __launch_bounds__(512, 1) wgrad256_ring16_kernel(const bf16* __restrict__ A,
                                                                 const bf16* __restrict__ B, float* __restrict__ out,
                                                                 int M, int N, int K, int lda, int ldb, int klen,
                                                                 int tiles_m, int tiles_n, int direct) {
  extern __shared__ __attribute__((aligned(16))) char smem2[];  // [NBUF][A|B][BKT * 512]
  constexpr int TILE = BKT * 512;
  constexpr int PIECES = BKT / 16;
  constexpr int G = 2 * PIECES;
  static_assert(BKT % 32 == 0 && NBUF >= 3 && (NBUF - 2) * G <= 63, "ring geometry");
  const int nwg = gridDim.x, wg = blockIdx.x;
  const int xcd = wg & 7, qd = nwg >> 3, rd = nwg & 7;
  const int id = (xcd < rd ? xcd * (qd + 1) : rd * (qd + 1) + (xcd - rd) * qd) + (wg >> 3);
  const int ntiles = tiles_m * tiles_n;
  const int split = id / ntiles, tile = id - split * ntiles;
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int m0 = tm * BM2, n0 = tn * BN2;
  const int k0 = split * klen, k1 = min(K, k0 + klen);
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w >> 2, wn = w & 3;

  const int rl = lane >> 5, pc = lane & 31;
  const bf16* asrc[PIECES];
  const bf16* bsrc[PIECES];
  int krow[PIECES];
#pragma unroll
  for (int i = 0; i < PIECES; ++i) {
    const int row = 2 * (PIECES * w + i) + rl;
    const int ch = pc ^ swz16(row);
    const int mc = m0 + 8 * ch, nc = n0 + 8 * ch;
    krow[i] = k0 + row;
    asrc[i] = mc < M ? A + (size_t)krow[i] * lda + mc : nullptr;
    bsrc[i] = nc < N ? B + (size_t)krow[i] * ldb + nc : nullptr;
  }
  const unsigned lds_base = (unsigned)(size_t)(lds_void_t*)smem2;
  const void* zero = (const void*)g_zero16;
  auto dma = [&](int st) {
    const int dk = st * BKT, buf = st % NBUF;
#pragma unroll
    for (int i = 0; i < PIECES; ++i) {
      const bool kok = krow[i] + dk < k1;
      const void* ga = (kok && asrc[i]) ? (const void*)(asrc[i] + (size_t)dk * lda) : zero;
      const void* gb = (kok && bsrc[i]) ? (const void*)(bsrc[i] + (size_t)dk * ldb) : zero;
      const unsigned la = __builtin_amdgcn_readfirstlane(lds_base + buf * 2 * TILE + (PIECES * w + i) * 1024);
      glds16(ga, la);
      glds16(gb, la + TILE);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nsteps = (k1 - k0 + BKT - 1) / BKT;
#pragma unroll
  for (int t = 0; t < NBUF - 1; ++t) dma(t);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NBUF - 2) * G) : "memory");
  __syncthreads();
  for (int st = 0; st < nsteps; ++st) {
    dma(st + NBUF - 1);
    const char* At = smem2 + (st % NBUF) * 2 * TILE;
    const char* Bt = At + TILE;
#pragma unroll
    for (int s = 0; s < BKT / 32; ++s) {
      uint4 bf[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = tr_frag16(Bt, 32 * s, 64 * wn + 16 * j, lane);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint4 af = tr_frag16(At, 32 * s, 128 * wm + 16 * i, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af, bf[j], acc[i][j]);
      }
    }
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NBUF - 2) * G) : "memory");
    __syncthreads();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  float* o = direct ? out : out + (size_t)split * M * N;
  const int g = lane >> 4;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + 64 * wn + 16 * j + (lane & 15);
      if (n >= N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + 128 * wm + 16 * i + 4 * g + r;
        if (m < M) {
          float* p = o + (size_t)m * N + n;
          if (direct) *p += acc[i][j][r];
          else *p = acc[i][j][r];
        }
      }
    }
}

// ---- ring16 with scalar-base DMA and precomputed fragment offsets (variant 6; + PF: 8, default) --
// The ring16 pipeline with the per-step address work moved off the vector ALUs: each DMA piece
// is global_load_lds with a wave-uniform SGPR row base (A + k·lda, advanced by scalar adds) and
// a per-lane 32-bit offset fixed for the whole kernel; tile columns past M / N are clamped to
// the last valid 16-B chunk (their products only reach output rows / columns that are never
// stored), so only a ragged K tail takes the per-lane zero-page path. Fragment reads use
// per-lane LDS offsets computed once (off512b is periodic in 16 rows, so the k slice and the
// second half-read are immediates) and the loop is unrolled by the ring depth, making every
// stage base a constant. (s_setprio around the MFMA clusters measured 4 % slower.)
template <int I, int N, typename F>
__device__ __forceinline__ void unroll_steps(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    unroll_steps<I + 1, N>(f);
  }
}

template <int BKT, int NBUF, bool PF = false>
__global__ void __launch_bounds__(512, 1) wgrad256_ring16o_kernel(const bf16* __restrict__ A,
                                                                  const bf16* __restrict__ B,
                                                                  float* __restrict__ grad, float* __restrict__ slab,
                                                                  int M, int N, int K, int lda, int ldb, int tiles_m,
                                                                  int tiles_n, WgradPlan plan, int acc_in) {
  extern __shared__ __attribute__((aligned(16))) char smem2[];  // [NBUF][A|B][BKT * 512]
  constexpr int TILE = BKT * 512;
  constexpr int PIECES = BKT / 16;
  constexpr int G = 2 * PIECES;
  static_assert(BKT % 32 == 0 && NBUF == 4 && (NBUF - 2) * G <= 63, "ring geometry");
  static_assert(!PF || (BKT == 32 && NBUF == 4), "fragment prefetch: 32-deep stages, 4-stage ring");
  const int nwg = gridDim.x, wg = blockIdx.x;
  const int ntiles = tiles_m * tiles_n;
  // (plan_wgrad, host_plan.h) ids [0, main_tiles·main_splits): the main tiles, split-major; then
  // the tail tiles [main_tiles, ntiles) split-major, each split into its own per-tile slab. The
  // XCD remap is applied within each range, so the main range is dispatched first and the tail's
  // short workgroups fill the last round (a remap over the whole grid sent tail ids to the first
  // round of some XCDs and long main tiles to their last).
  const int n_main = plan.main_tiles * plan.main_splits;
  const bool in_tail = wg >= n_main;
  const int rbase = in_tail ? n_main : 0, rcnt = in_tail ? nwg - n_main : n_main, rwg = wg - rbase;
  const int xcd = rwg & 7, qd = rcnt >> 3, rd = rcnt & 7;
  const int id = rbase + (xcd < rd ? xcd * (qd + 1) : rd * (qd + 1) + (xcd - rd) * qd) + (rwg >> 3);
  const int nt = ntiles - plan.main_tiles;
  const int jt = id - n_main;
  const int split = in_tail ? jt / nt : id / plan.main_tiles;
  const int tail_i = in_tail ? jt - split * nt : 0;
  const int tile = in_tail ? plan.main_tiles + tail_i : id - split * plan.main_tiles;
  const int klen = in_tail ? plan.tail_klen : plan.main_klen;
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int m0 = tm * BM2, n0 = tn * BN2;
  const int k0 = split * klen, k1 = min(K, k0 + klen);
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // Half tiles (the last tile column of N = 1152 = 4.5 × 256, or the last tile row of M = 1152):
  // the 8 waves are re-laid out over the 256 × 128 (4 × 2 waves) or 128 × 256 (2 × 4) part that
  // exists, 64 × 64 outputs each, so every wave does useful MFMAs and the tile takes about half
  // the time (with the full-tile layout half of the waves multiply clamped columns).
  const int half = N - n0 <= 128 ? 1 : (M - m0 <= 128 ? 2 : 0);
  const int wm = half == 1 ? w >> 1 : w >> 2, wn = half == 1 ? w & 1 : w & 3;
  const int rspan = half ? 64 : 128;  // output rows per wave

  // DMA: piece i of wave w = tile rows 2(PIECES·w + i) + (lane>>5), 16-B chunk (lane&31) ^ swz
  const int rl = lane >> 5, pc = lane & 31;
  const int mlast = ((M + 7) & ~7) - 8, nlast = N - 8;
  unsigned aoff[PIECES], boff[PIECES];
#pragma unroll
  for (int i = 0; i < PIECES; ++i) {
    const int row = 2 * (PIECES * w + i) + rl;
    const int ch = pc ^ swz16(row);
    aoff[i] = (unsigned)(row * lda + min(m0 + 8 * ch, mlast)) * 2u;
    boff[i] = (unsigned)(row * ldb + min(n0 + 8 * ch, nlast)) * 2u;
  }
  const unsigned lds_base = (unsigned)(size_t)(lds_void_t*)smem2;
  const char* zero = reinterpret_cast<const char*>(g_zero16);
  auto dma = [&](int st) {
    const int kr = k0 + st * BKT;
    const unsigned la = __builtin_amdgcn_readfirstlane(lds_base + (st % NBUF) * 2 * TILE + PIECES * w * 1024);
    const char* sa = reinterpret_cast<const char*>(A + (size_t)kr * lda);
    const char* sb = reinterpret_cast<const char*>(B + (size_t)kr * ldb);
    if (kr + BKT <= k1) {
#pragma unroll
      for (int i = 0; i < PIECES; ++i) {
        glds16_s(sa, aoff[i], la + i * 1024);
        glds16_s(sb, boff[i], la + TILE + i * 1024);
      }
    } else {  // ragged K tail or a prefetch past the end: rows >= k1 read the zero page
#pragma unroll
      for (int i = 0; i < PIECES; ++i) {
        const bool ok = kr + 2 * (PIECES * w + i) + rl < k1;
        glds16(ok ? sa + aoff[i] : zero, la + i * 1024);
        glds16(ok ? sb + boff[i] : zero, la + TILE + i * 1024);
      }
    }
  };

  // fragment reads: lane holds k = 8·(lane>>4) + j of column c0 + (lane&15); rows r and r + 4
  const int g = lane >> 4, q = (lane & 15) >> 2, p4 = 4 * (lane & 3);
  unsigned fa[8], fb[4];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int col = rspan * wm + 16 * i + p4;
    fa[i] = (unsigned)(off512b(8 * g + q, col >> 3) + ((col & 4) << 1));
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = 64 * wn + 16 * j + p4;
    fb[j] = (unsigned)(off512b(8 * g + q, col >> 3) + ((col & 4) << 1));
  }
  auto frag = [&](const char* t, unsigned off) -> uint4 {
    const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(t + off));
    const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(t + off + 4 * 512));
    const uint2 ua = __builtin_bit_cast(uint2, a), ub = __builtin_bit_cast(uint2, b);
    return uint4{ua.x, ua.y, ub.x, ub.y};
  };

  auto run = [&](auto ni_c) {  // NI = 16-row fragment blocks per wave: 8 (full tile) or 4 (half)
    constexpr int NI = decltype(ni_c)::value;
    f32x4 acc[8][4];
  #pragma unroll
    for (int i = 0; i < NI; ++i)
  #pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nsteps = (k1 - k0 + BKT - 1) / BKT;
    // PF (fragment prefetch): each step's MFMAs run on fragments read during the PREVIOUS step, so
    // no wave starts a step waiting on LDS reads after the barrier; the barrier at the end of step
    // st must then publish stage st+2 (read during step st+1), leaving one stage in flight
    constexpr int WAITN = PF ? (NBUF - 3) * G : (NBUF - 2) * G;
  #pragma unroll
    for (int t = 0; t < NBUF - 1; ++t) dma(t);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WAITN) : "memory");
    __syncthreads();
    constexpr int PFA = 2;  // A fragments read one step ahead
    uint4 ca[PFA], cb[4];  // PF: the current step's prefetched fragments
    if constexpr (PF) {
  #pragma unroll
      for (int j = 0; j < 4; ++j) cb[j] = frag(smem2 + TILE, fb[j]);
  #pragma unroll
      for (int i = 0; i < PFA; ++i) ca[i] = frag(smem2, fa[i]);
    }
    auto step = [&](int st, auto stage_tag) {
      constexpr int ST = decltype(stage_tag)::value;
      dma(st + NBUF - 1);  // into the stage consumed at step st-1 (freed by its barrier)
      const char* At = smem2 + ST * 2 * TILE;
      const char* Bt = At + TILE;
      if constexpr (PF) {
        // the B fragments and the first PFA A fragments come from the previous step; the other A
        // fragments of this stage are read under those MFMAs, then next stage's prefetch is read
        // under the rest (all 8 A fragments ahead would need 48 more VGPRs: 31 spilled)
        const char* An = smem2 + ((ST + 1) % NBUF) * 2 * TILE;  // published by the previous barrier
        uint4 la[NI - PFA];
  #pragma unroll
        for (int i = PFA; i < NI; ++i) la[i - PFA] = frag(At, fa[i]);
  #pragma unroll
        for (int i = 0; i < PFA; ++i)
  #pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(ca[i], cb[j], acc[i][j]);
        uint4 nb[4], na[PFA];
  #pragma unroll
        for (int i = PFA; i < NI; ++i) {
  #pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(la[i - PFA], cb[j], acc[i][j]);
          if (i == PFA) {
  #pragma unroll
            for (int q = 0; q < PFA; ++q) na[q] = frag(An, fa[q]);
          }
        }
  #pragma unroll
        for (int j = 0; j < 4; ++j) nb[j] = frag(An + TILE, fb[j]);
  #pragma unroll
        for (int i = 0; i < PFA; ++i) ca[i] = na[i];
  #pragma unroll
        for (int j = 0; j < 4; ++j) cb[j] = nb[j];
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WAITN) : "memory");  // stage st+2 landed
        __syncthreads();
        return;
      }
  #pragma unroll
      for (int s = 0; s < BKT / 32; ++s) {
        uint4 bf[4];
  #pragma unroll
        for (int j = 0; j < 4; ++j) bf[j] = frag(Bt + s * 32 * 512, fb[j]);
  #pragma unroll
        for (int i = 0; i < NI; ++i) {
          const uint4 af = frag(At + s * 32 * 512, fa[i]);
  #pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af, bf[j], acc[i][j]);
        }
      }
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NBUF - 2) * G) : "memory");  // stage st+1 landed
      __syncthreads();
    };
    int st = 0;
    for (; st + NBUF <= nsteps; st += NBUF)  // unrolled by the ring depth: stage bases are immediates
      unroll_steps<0, NBUF>([&](auto ic) { step(st + decltype(ic)::value, ic); });
    unroll_steps<0, NBUF - 1>([&](auto ic) {
      if (st + decltype(ic)::value < nsteps) step(st + decltype(ic)::value, ic);
    });
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the zero-page prefetches
    // main tiles: direct read-add-write (one split) or a full-size slab per split; tail tiles: a
    // packed [256][256] slab per (split, tail tile), added by tile_slab_reduce_kernel
    const bool direct = !in_tail && plan.main_splits == 1;
    float* const obase = direct ? grad : slab;
    const int64_t ld = in_tail ? BN2 : N;  // element (m, n) sits at obase[ob + m·ld + n]
    const int64_t ob = direct ? 0
                       : in_tail ? ((int64_t)split * nt + tail_i) * (BM2 * BN2) - (int64_t)m0 * BN2 - n0
                                 : (int64_t)split * M * N;
    if (direct) {
      // read-add-write in groups of 16 values: every read of a group is issued before its writes
      // (written element by element, the compiler must assume each write may alias the next read
      // and serialises 128 memory round trips per lane: 1.0 ms of a 4.0 ms lm_head wgrad)
  #pragma unroll
      for (int i0 = 0; i0 < NI; ++i0) {
        float cur[1][4][4];
  #pragma unroll
        for (int ii = 0; ii < 1; ++ii)
  #pragma unroll
          for (int j = 0; j < 4; ++j)
  #pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int n = n0 + 64 * wn + 16 * j + (lane & 15);
              const int m = m0 + rspan * wm + 16 * (i0 + ii) + 4 * g + r;
              cur[ii][j][r] = (acc_in && m < M && n < N) ? grad[(int64_t)m * N + n] : 0.f;
            }
  #pragma unroll
        for (int ii = 0; ii < 1; ++ii)
  #pragma unroll
          for (int j = 0; j < 4; ++j)
  #pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int n = n0 + 64 * wn + 16 * j + (lane & 15);
              const int m = m0 + rspan * wm + 16 * (i0 + ii) + 4 * g + r;
              if (m < M && n < N) grad[(int64_t)m * N + n] = cur[ii][j][r] + acc[i0 + ii][j][r];
            }
      }
      return;
    }
  #pragma unroll
    for (int i = 0; i < NI; ++i)
  #pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + 64 * wn + 16 * j + (lane & 15);
        if (n >= N) continue;
  #pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + rspan * wm + 16 * i + 4 * g + r;
          if (m < M) obase[ob + (int64_t)m * ld + n] = acc[i][j][r];
        }
      }
  };
  if (half) run(std::integral_constant<int, 4>{});
  else run(std::integral_constant<int, 8>{});
}

// G[e] += Σ_s slab[s][e]  (vectorised, fixed order)
__global__ void __launch_bounds__(256) slab_reduce_kernel(const float* __restrict__ slab, float* __restrict__ g,
                                                          int64_t n4, int splits, int64_t stride4, int acc_in) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4_t acc = acc_in ? reinterpret_cast<float4_t*>(g)[i] : float4_t{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < splits; ++s) acc += reinterpret_cast<const float4_t*>(slab)[s * stride4 + i];
    reinterpret_cast<float4_t*>(g)[i] = acc;
  }
}

// G[tile t of the tail] += Σ_s slab[s][t] for the tail tiles of a split-tail plan (packed
// [256][256] fp32 per (split, tile); fixed order, so the result is bitwise reproducible)
__global__ void __launch_bounds__(256) tile_slab_reduce_kernel(const float* __restrict__ slab, float* __restrict__ g,
                                                               int M, int N, int tiles_n, int first_tile, int nt,
                                                               int splits, int acc_in) {
  constexpr int T4 = BM2 * BN2 / 4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < (int64_t)nt * T4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int ti = (int)(i / T4), e = (int)(i - (int64_t)ti * T4);
    const int r = e / (BN2 / 4), c = 4 * (e - r * (BN2 / 4));
    const int tile = first_tile + ti, tm = tile / tiles_n, tn = tile - tm * tiles_n;
    const int m = tm * BM2 + r, n = tn * BN2 + c;
    if (m >= M || n >= N) continue;  // N % 8 == 0: n < N covers n + 3
    float4_t* gp = reinterpret_cast<float4_t*>(g + (size_t)m * N + n);
    float4_t acc = acc_in ? *gp : float4_t{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < splits; ++s)
      acc += reinterpret_cast<const float4_t*>(slab + ((size_t)s * nt + ti) * (BM2 * BN2))[e];
    *gp = acc;
  }
}

}  // namespace
}  // namespace penroz

using namespace penroz;

// grad[M][N] += dyᵀ·x with dy [K, M], x [K, N] (bf16, row-major, contiguous rows).
// tile = 256 (default, 8 waves) or 128 (4 waves); variant selects the 256-tile pipeline (see below).
void wgrad_gemm(torch::Tensor dy, torch::Tensor x, torch::Tensor grad, int64_t tile, int64_t variant, bool accumulate) {
  TORCH_CHECK(dy.is_cuda() && x.is_cuda() && grad.is_cuda());
  TORCH_CHECK(dy.scalar_type() == torch::kBFloat16 && x.scalar_type() == torch::kBFloat16 &&
              grad.scalar_type() == torch::kFloat32, "wgrad: bf16 operands, fp32 gradient");
  TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && dy.size(0) == x.size(0), "wgrad: [K, M] x [K, N]");
  TORCH_CHECK(dy.stride(1) == 1 && x.stride(1) == 1 && grad.is_contiguous());
  const int K = dy.size(0), M = dy.size(1), N = x.size(1);
  TORCH_CHECK(grad.size(0) == M && grad.size(1) == N, "wgrad: gradient shape mismatch");
  // the kernels load 8-column (16-B) chunks: a width that is not a multiple of 8 is fine when
  // the rows are padded (row stride >= the width rounded up to 8, e.g. the executor's logits
  // rows for V = 50257), the tail chunk then reads pad columns of the same row (their products
  // only reach output rows >= M, which are never stored)
  const int Mp = (M + 7) & ~7;
  TORCH_CHECK(N % 8 == 0 && dy.stride(0) % 8 == 0 && x.stride(0) % 8 == 0 && (M % 8 == 0 || dy.stride(0) >= Mp),
              "wgrad: N and row strides must be multiples of 8, and M too unless dy's rows are padded to it");
  TORCH_CHECK(M % 8 == 0 || dy.storage().nbytes() >= (size_t)(dy.storage_offset() + (int64_t)(K - 1) * dy.stride(0) +
                                                             Mp) * 2,
              "wgrad: dy's last row padding must be allocated");
  TORCH_CHECK(tile == 128 || tile == 256, "wgrad: tile must be 128 or 256");
  if (K == 0) {
    if (!accumulate) grad.zero_();
    return;
  }
  const int T = (int)tile;
  const int tiles_m = (M + T - 1) / T, tiles_n = (N + T - 1) / T;
  const int ntiles = tiles_m * tiles_n;
  static int n_cu = 0;
  if (n_cu == 0) {
    hipDeviceProp_t prop;
    n_cu = hipGetDeviceProperties(&prop, grad.get_device()) == hipSuccess ? prop.multiProcessorCount : 256;
  }
  // split-K from the wave-quantisation cost model (host_plan.h, sanitizer-tested on the host);
  // the ring16o variants (6, 8) may also take a split-tail plan (plan_wgrad)
  const SplitK uplan = plan_wgrad_splits(M, N, K, T, n_cu, T == 256 ? BK2 : BK);
  static const bool tail_ok = [] {  // PENROZ_WGRAD_TAIL=0: uniform plans only (A/B)
    const char* e = std::getenv("PENROZ_WGRAD_TAIL");
    return !(e && e[0] == '0');
  }();
  const bool ring16o = T == 256 && (variant == 6 || variant == 8) && tail_ok;
  const WgradPlan wp = ring16o ? plan_wgrad(M, N, K, T, n_cu, BK2) : WgradPlan{ntiles, uplan.splits, uplan.klen, 0, 0};
  const int splits = wp.main_splits, klen = wp.main_klen;
  const int tail_tiles = ntiles - wp.main_tiles;
  auto stream = at::hip::getCurrentHIPStream();
  const int nwg = wp.main_tiles * splits + tail_tiles * wp.tail_splits;
  const bf16* a = reinterpret_cast<const bf16*>(dy.data_ptr());
  const bf16* b = reinterpret_cast<const bf16*>(x.data_ptr());
  torch::Tensor slab;
  float* dst = grad.data_ptr<float>();
  if (splits > 1) {
    slab = torch::empty({(int64_t)splits * M * N}, grad.options());
    dst = slab.data_ptr<float>();
  } else if (wp.tail_splits > 0) {
    slab = torch::empty({(int64_t)wp.tail_splits * tail_tiles * T * T}, grad.options());
  }
  const int direct = splits == 1 ? 1 : 0;
  // overwrite (accumulate = false: the first micro-step after a zero-free zero_grad): the ring16o
  // variants and the slab reductions write instead of read-add-write; the others zero first
  if (!accumulate && !ring16o) grad.zero_();
  const int acc_in = accumulate || !ring16o ? 1 : 0;
  if (T == 256) {
    // variant 6: ring16o; 4: ring16 (per-lane 64-bit DMA addresses and fragment
    // address math in the loop; kept for A/B). v4 / v6 (TF): qkv 879/959, proj 822/914,
    // fc 1006/1089, fc2 1020/1058, lm_head 1128/1255 (bench/wgrad_variants.py,
    // profiles/wgrad_variants_r2.log; s_setprio around the MFMA clusters: 909/850/1067/1045/1162).
    // 8 (default): ring16o with the B and first A fragments read one step ahead (PF): 14.54 vs
    // 14.68 ms/step of wgrad (profiles/wgrad_variants_r2b.log; a 64-deep 2-stage ring measured
    // 16.23: the per-step barrier is not what bounds this kernel)
    TORCH_CHECK(variant == 4 || variant == 6 || variant == 8, "wgrad: variant must be 4, 6 or 8");
    constexpr int lds = 4 * 2 * BK2 * 512;
    static bool attr_set = false;
    if (!attr_set) {
      hipFuncSetAttribute(reinterpret_cast<const void*>(wgrad256_ring16_kernel<BK2, 4>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, lds);
      hipFuncSetAttribute(reinterpret_cast<const void*>(wgrad256_ring16o_kernel<BK2, 4>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, lds);
      hipFuncSetAttribute(reinterpret_cast<const void*>(wgrad256_ring16o_kernel<BK2, 4, true>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, lds);
      attr_set = true;
    }
    const int lda = (int)dy.stride(0), ldb = (int)x.stride(0);
    if (variant == 4)
      hipLaunchKernelGGL((wgrad256_ring16_kernel<BK2, 4>), dim3(nwg), dim3(512), lds, stream, a, b, dst, M, N, K,
                         lda, ldb, klen, tiles_m, tiles_n, direct);
    else if (variant == 8)
      hipLaunchKernelGGL((wgrad256_ring16o_kernel<BK2, 4, true>), dim3(nwg), dim3(512), lds, stream, a, b,
                         grad.data_ptr<float>(), slab.defined() ? slab.data_ptr<float>() : nullptr, M, N, K, lda, ldb,
                         tiles_m, tiles_n, wp, acc_in);
    else
      hipLaunchKernelGGL((wgrad256_ring16o_kernel<BK2, 4>), dim3(nwg), dim3(512), lds, stream, a, b,
                         grad.data_ptr<float>(), slab.defined() ? slab.data_ptr<float>() : nullptr, M, N, K, lda, ldb,
                         tiles_m, tiles_n, wp, acc_in);
  } else {
    hipLaunchKernelGGL(wgrad_kernel, dim3(nwg), dim3(256), 0, stream, a, b, dst, M, N, K, (int)dy.stride(0),
                       (int)x.stride(0), klen, tiles_m, tiles_n, direct);
  }
  if (wp.tail_splits > 0) {
    const int64_t n4 = (int64_t)tail_tiles * T * T / 4;
    hipLaunchKernelGGL(tile_slab_reduce_kernel, dim3((int)std::min<int64_t>((n4 + 255) / 256, 2048)), dim3(256), 0,
                       stream, slab.data_ptr<float>(), grad.data_ptr<float>(), M, N, tiles_n, wp.main_tiles, tail_tiles,
                       wp.tail_splits, acc_in);
    return;
  }
  if (splits == 1) return;
  const int64_t n4 = (int64_t)M * N / 4;
  hipLaunchKernelGGL(slab_reduce_kernel, dim3((int)std::min<int64_t>((n4 + 255) / 256, 2048)), dim3(256), 0, stream,
                     slab.data_ptr<float>(), grad.data_ptr<float>(), n4, splits, n4, acc_in);
}
