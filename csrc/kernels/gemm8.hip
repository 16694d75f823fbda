// Forward / data-gradient GEMM for MI355X on the 8-phase ping-pong schedule:
//
//   C[M][N] = A[M][K] · B[N][K]ᵀ (+ bias[N]) (→ GELU),   bf16 operands, fp32 accumulation, bf16 out
//
// Both operands are K-contiguous ("TN"): a linear layer's forward y = x·Wᵀ (B = W [out, in]) and,
// with the executor's transposed weight copy Wᵀ [in, out], its data gradient dx = dy·W. Replaces
// hipBLASLt for the GPT-2 forward / dgrad GEMMs (reference: every ``nn.Linear`` of
// /root/reference/main.py:63-82 through cuBLAS) so that bias and GELU (pre-activation AND
// activation written by one pass) live in the epilogue instead of separate memory-bound kernels.
//
// Structure (cdna_hip_programming.md §5 "The 256² 8-phase template", rebuilt here):
//   * 256×256 output tiles, one persistent 512-thread workgroup per CU (131 KiB LDS) walking its
//     tiles with the DMA stream running straight on into the next tile (no per-tile pipeline fill);
//     8 waves as 2 (M) × 4
//     (N), each wave 128×64 = 2×2 C-quadrants of 64×32 (4×2 v_mfma_f32_16x16x32_bf16 tiles);
//   * a k-tile is 64 deep and is consumed in 4 PHASES, one C-quadrant each (16 MFMAs), in the order
//     (ma,nb) = (0,0) (0,1) (1,1) (1,0), so each phase reloads at most one operand subtile
//     (A: 8 ds_read_b128, B: 4) and the operand registers are 32 (A) + 2×16 (B) VGPRs;
//   * operands arrive by LDS-DMA (global_load_lds_dwordx4 from a wave-uniform SGPR base + a per-lane
//     32-bit offset fixed for the tile) in UNITS of 16 KiB = 128 rows × 64 k: A rows of quadrant row
//     ma of both wave rows, or B rows of quadrant column nb of all four wave columns. Every phase
//     issues exactly one unit (2 DMA pieces per wave) — unit u in global phase u − 5 — so the
//     in-flight count is uniform and ONE counted `s_waitcnt vmcnt(8)` per phase (before its first
//     barrier) retires the unit issued four phases earlier: each unit lands ≥ 1 phase before the
//     phase that reads it, and is overwritten ≥ 2 phases after its last read (two k-tile buffers);
//     the DMA is buffer_load ... lds through buffer resources over the tile's 256-row panels (rows past
//     the matrix edge read 0; past the last tile the resources are empty, so the tail keeps the count);
//   * ping-pong: wave row 1 runs one raw s_barrier behind wave row 0, so on every SIMD one wave
//     issues its 16 MFMAs (s_setprio 1, fenced by sched_barriers) while its partner issues the
//     next phase's ds_reads and DMA;
//   * [rows][64] images with 128-B rows: 16-B chunk c of row r sits in slot c ^ ((r>>1)&7) (the
//     swizzle is applied on the DMA SOURCE address; the destination is lane-linear) — every
//     16-lane ds_read_b128 group hits 16 distinct bank slots;
//   * MFMA operands swapped (D = B·Aᵀ) so each lane holds 4 consecutive output columns of one row;
//     a v_permlane16_swap widens that to 8 columns: 16-B stores;
//   * XCD-aware bijective tile order in groups of 8 row panels (an XCD's A and B panels stay in
//     its L2).
#include "common.h"
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

namespace penroz {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;

constexpr int TILE = 256, KT = 64, GM = 8;
constexpr int UNIT = 16384;                // 128 rows x 64 k bf16
constexpr int KBUF = 4 * UNIT;             // one k-tile: [A_ma0 | B_nb0 | B_nb1 | A_ma1]
constexpr int BIAS_OFF = 2 * KBUF;         // epilogue bias, [tile parity][256] bf16
constexpr int BIAS_SINK = BIAS_OFF + 1024;  // the bias piece of waves 2-7 (uniform VMEM count)
constexpr int LDS_BYTES = BIAS_SINK + 2048;  // 131 KiB

enum Epi8 { E8_NONE = 0, E8_BIAS = 1, E8_BIAS_GELU = 2 };

__device__ __forceinline__ f32x4 mfma16(uint4 a, uint4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                 0, 0, 0);
}

__device__ __forceinline__ int rswz(int r) { return (r >> 1) & 7; }

typedef __amdgpu_buffer_rsrc_t rsrc_t;

// A raw buffer resource over [p, p + bytes): loads past it return 0, stores past it are dropped.
__device__ __forceinline__ rsrc_t make_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, bytes, 0x00020000);
}

// The two 1-KiB LDS-DMA pieces of one wave for one unit (buffer_load_dwordx4 ... lds): LDS
// [lds0, +2 KiB), per-lane byte offsets v0 / v1 (range-checked against the resource: rows past
// the matrix edge read 0), k offset in soffset. M0 is saved and restored around the statement;
// only s_mov touches it (an s_add would clobber SCC, which the compiler may hold live across the
// statement: that corrupted results whenever the surrounding code kept a compare in SCC).
// `s_nop 4`: the descriptor / soffset SGPRs may have just been written.
__device__ __forceinline__ void bdma2(rsrc_t r, unsigned v0, unsigned v1, unsigned soff, unsigned lds0) {
  unsigned keep;
  const unsigned lds1 = lds0 + 1024u;
  asm volatile(
      "s_nop 4\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %5\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %3, %4 offen lds\n\t"
      "s_mov_b32 m0, %6\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %2, %3, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(v0), "v"(v1), "s"(r), "s"(soff), "s"(lds0), "s"(lds1)
      : "memory");
}

// one 256-B LDS-DMA piece (buffer_load_dword ... lds): 64 lanes x 4 B to LDS [lds0, +256 B)
__device__ __forceinline__ void bdma1(rsrc_t r, unsigned v0, unsigned lds0) {
  unsigned keep;
  asm volatile(
      "s_nop 4\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "buffer_load_dword %1, %2, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(v0), "s"(r), "s"(lds0)
      : "memory");
}

__device__ __forceinline__ void tile_coords8(int t, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int per_group = GM * tiles_n;
  const int group = t / per_group;
  const int first_m = group * GM;
  const int gsz = min(tiles_m - first_m, GM);
  const int r = t - group * per_group;
  tm = first_m + r % gsz;
  tn = r / gsz;
}

__device__ __forceinline__ float bflo(uint32_t u) { return __uint_as_float(u << 16); }

// erf-GELU with erf from Abramowitz & Stegun 7.1.26 (|error| < 1.5e-7, far below a bf16 ulp):
// one rcp + one exp2 + 9 VALU, no branches (ocml's erff takes a polynomial / exp-rational branch pair)
__device__ __forceinline__ float gelu_erf_fast(float x) {
  const float z = fabsf(x) * 0.7071067811865476f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float e = 1.f - p * t * __builtin_amdgcn_exp2f(-z * z * 1.4426950408889634f);  // erf(z)
  return 0.5f * x * (1.f + copysignf(e, x));
}
__device__ __forceinline__ float bfhi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }

// 16-B buffer store with a cache policy chosen at run time (ablation: 0 plain, 1 sc0, 2 nt, 3 sc0 nt)
__device__ __forceinline__ void store_pol(u32x4 v, rsrc_t r, unsigned off, int pol) {
  if (pol == 0) __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)off, 0, 0);
  else if (pol == 1) __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)off, 0, 1);
  else if (pol == 2) __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)off, 0, 2);
  else __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)off, 0, 3);
}

#define PZ_BARRIER()                  \
  do {                                \
    asm volatile("" ::: "memory");    \
    __builtin_amdgcn_s_barrier();     \
    asm volatile("" ::: "memory");    \
  } while (0)

template <int I, int N, typename F>
__device__ __forceinline__ void unroll8(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    unroll8<I + 1, N>(f);
  }
}

template <int EPI>
__global__ void __launch_bounds__(512, 1) gemm8_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                       const bf16* __restrict__ bias, bf16* __restrict__ C,
                                                       bf16* __restrict__ C2, int M, int N, int K, int lda, int ldb,
                                                       int ldc, int tiles_m, int tiles_n, int approx, int ablate) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int EXTRA = EPI != E8_NONE ? 1 : 0;        // the bias piece rides with every A_ma0 unit
  constexpr int VM = 8 + EXTRA;                         // VMEM ops of four consecutive phases
  constexpr int S = EPI == E8_BIAS_GELU ? 32 : 16;      // epilogue stores per wave
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 2, wc = w & 3;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, qd = nwg >> 3, rd = nwg & 7;
  const int u = (xcd < rd ? xcd * (qd + 1) : rd * (qd + 1) + (xcd - rd) * qd) + (bid >> 3);
  const int ntiles = tiles_m * tiles_n;
  const int my_tiles = (ntiles - u + nwg - 1) / nwg;  // tiles u, u + nwg, ... of this workgroup
  const int nk = K / KT, nh = nk / 2;                 // k-tiles per tile, 8-phase iterations per tile
  const int g = lane >> 4;
  const unsigned lds_base = (unsigned)(size_t)(lds_void_t*)smem;

  // ---- DMA state (all wave-uniform: SGPRs): tile dti (local index), k-tile dkt, and buffer
  // resources over the tile's 256-row panels of A and B (rows past the matrix edge read 0) and its
  // bias slice. The per-lane offsets of this wave's two pieces of each unit do not depend on the
  // tile: they are computed once.
  // (plain pointers and sizes here; the descriptors are built at each use, so everything stays in
  // SGPRs — a descriptor variable assigned inside the loop was kept in scratch memory)
  int dti = 0, dkt = 0;
  const bf16* pa = A;
  const bf16* pb = B;
  const bf16* pbias = bias;
  unsigned na = 0, nbb = 0, nbias = 0;
  auto set_dma_tile = [&](int t) {
    int tm, tn;
    tile_coords8(u + min(t, my_tiles - 1) * nwg, tiles_m, tiles_n, tm, tn);
    const int m0 = tm * TILE, n0 = tn * TILE;
    const bool live = t < my_tiles;  // past the last tile: empty resources (the tail keeps its count)
    pa = A + (size_t)m0 * lda;
    pb = B + (size_t)n0 * ldb;
    na = live ? (unsigned)(min(M - m0, TILE) * lda * 2) : 0u;
    nbb = live ? (unsigned)(min(N - n0, TILE) * ldb * 2) : 0u;
    if constexpr (EXTRA) {
      pbias = bias + n0;
      nbias = live ? (unsigned)(min(N - n0, TILE) * 2) : 0u;
    }
  };
  // (the second unit of each operand, A_ma1 / B_nb1, is the first one shifted by 64 / 32 rows:
  // that goes into the scalar soffset, so only these four offsets occupy VGPRs)
  unsigned va[2], vb[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int lr = 16 * w + 8 * i + (lane >> 3);  // row of the unit image
    const int c = (lane & 7) ^ rswz(lr);          // logical 16-B chunk held by this lane's slot
    va[i] = (unsigned)((lr + (lr >= 64 ? 64 : 0)) * lda + 8 * c) * 2u;
    vb[i] = (unsigned)(((lr >> 5) * 64 + (lr & 31)) * ldb + 8 * c) * 2u;
  }
  const unsigned vbias = (unsigned)(128 * (w & 1) + 2 * lane) * 2u;
  auto advance = [&]() {  // next k-tile of the DMA stream (crossing into the next tile)
    if (++dkt == nk) {
      dkt = 0;
      set_dma_tile(++dti);
    }
  };
  // unit KIND (0 A_ma0, 1 B_nb0, 2 B_nb1, 3 A_ma1) of the current DMA k-tile into k-buffer DB; past
  // the last tile the zero-size resources make it a DMA of zeros into the same (already retired)
  // slot, so every phase issues the same VMEM count
  auto issue = [&](auto kind_c, auto db_c) {
    constexpr int KIND = decltype(kind_c)::value, DB = decltype(db_c)::value;
    constexpr bool IS_A = KIND == 0 || KIND == 3;
    constexpr int H = (KIND == 0 || KIND == 1) ? 0 : 1;
    const unsigned soff = (unsigned)(dkt * KT * 2) + (H ? (unsigned)((IS_A ? 64 * lda : 32 * ldb) * 2) : 0u);
    if constexpr (EXTRA && KIND == 0)
      bdma1(make_rsrc(pbias, nbias), vbias, __builtin_amdgcn_readfirstlane(w < 2 ? lds_base + BIAS_OFF + (dti & 1) * 512 + (w & 1) * 256
                                                               : lds_base + BIAS_SINK + (w - 2) * 256));
    bdma2(IS_A ? make_rsrc(pa, na) : make_rsrc(pb, nbb), IS_A ? va[0] : vb[0], IS_A ? va[1] : vb[1], soff,
          __builtin_amdgcn_readfirstlane(lds_base + DB * KBUF + KIND * UNIT + w * 2048));
  };

  // ---- fragment reads: the swizzled chunk of row r depends only on r's bits 1-3 = lane bits 1-3
  const unsigned lpart0 = (unsigned)((lane & 15) * 128 + (((lane >> 4) ^ ((lane >> 1) & 7)) << 4));
  const unsigned lpart1 = (unsigned)((lane & 15) * 128 + (((4 + (lane >> 4)) ^ ((lane >> 1) & 7)) << 4));
  const unsigned aoff = (unsigned)(wr * 64 * 128), boff = (unsigned)(wc * 32 * 128);
  auto rd128 = [&](unsigned off) -> uint4 { return __builtin_bit_cast(uint4, *(const lds_u32x4*)(smem + off)); };

  f32x4 acc[2][4][2][2];
  auto zero_acc = [&]() {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[a][i][b][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  zero_acc();
  uint4 af[4][2], bfr[2][2][2];  // A: [m-frag][k-step]; B: [nb][n-frag][k-step]

  // ablation (ablate >> 8): odd workgroups start that many s_sleep 127 late (de-synchronised epilogues)
  if ((ablate >> 8) && (u & 1))
    for (int i = 0; i < (ablate >> 8); ++i) __builtin_amdgcn_s_sleep(127);
  // ---- prologue: units 0-5 (k-tile 0 whole, k-tile 1's A_ma0 / B_nb0); the first two landed
  set_dma_tile(0);
  issue(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
  issue(std::integral_constant<int, 1>{}, std::integral_constant<int, 0>{});
  issue(std::integral_constant<int, 2>{}, std::integral_constant<int, 0>{});
  issue(std::integral_constant<int, 3>{}, std::integral_constant<int, 0>{});
  advance();
  issue(std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{});
  issue(std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{});
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM) : "memory");
  PZ_BARRIER();
  if (wr == 1) PZ_BARRIER();  // stagger: wave row 1 runs one barrier behind
  __builtin_amdgcn_s_waitcnt(0xC07F);  // compiler-visible lgkmcnt(0): no scalar load pending in the loop

  // one phase: this quadrant's operand reads, one DMA unit, the counted wait, 16 MFMAs. After an
  // epilogue (AE) the wave's S stores sit between the units in flight: count them in phases 1-4.
  auto phase = [&](auto ph_c, bool ae) {
    constexpr int PH = decltype(ph_c)::value + 1;  // 1..8
    constexpr int DB = (PH - 1) / 4;               // this iteration's k-tile 2it + DB is in k-buffer DB
    constexpr int QP = (PH - 1) % 4;
    constexpr int MA = QP < 2 ? 0 : 1;
    constexpr int NB = (QP == 1 || QP == 2) ? 1 : 0;
    constexpr unsigned KB = DB * KBUF;
    if constexpr (QP == 0 || QP == 2) {  // A subtile of quadrant row MA
      constexpr unsigned UA = KB + (MA == 0 ? 0 : 3) * UNIT;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        af[i][0] = rd128(UA + aoff + lpart0 + 2048 * i);
        af[i][1] = rd128(UA + aoff + lpart1 + 2048 * i);
      }
    }
    if constexpr (QP == 0 || QP == 1) {  // B subtile of quadrant column NB
      constexpr unsigned UB = KB + (NB == 0 ? 1 : 2) * UNIT;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        bfr[NB][j][0] = rd128(UB + boff + lpart0 + 2048 * j);
        bfr[NB][j][1] = rd128(UB + boff + lpart1 + 2048 * j);
      }
    }
    constexpr int U = PH + 5;  // the unit of this phase: kind U%4 of k-tile 2it + U/4
    if constexpr (U % 4 == 0) advance();
    issue(std::integral_constant<int, U % 4>{}, std::integral_constant<int, (U / 4) & 1>{});
    if (PH <= 4 && ae) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM + S) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM) : "memory");
    PZ_BARRIER();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int s = 0; s < 2; ++s) acc[MA][i][NB][j] = mfma16(bfr[NB][j][s], af[i][s], acc[MA][i][NB][j]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    PZ_BARRIER();
  };

  // ---- epilogue of local tile ct: lane (row lane&15 of its 16-row frag, g) holds columns
  // 4g..4g+3 of each n-frag; a permlane16 swap of the pair (j = 0, 1) gives 8 consecutive columns:
  // one 16-B buffer store each. EVERY lane stores (rows / columns past the edge get an offset past
  // the buffer: dropped by the range check), so the store count S is exact for the counted waits.
  auto epilogue = [&](int ct) {
    // lane-derived addresses are recomputed here from an opaque lane id: hoisted out of the tile
    // loop they would be spilled around it (their reloads' waits would drain the in-flight DMA)
    const int lane = opaque_lane_id();
    const int g = lane >> 4;
    int tm, tn;
    tile_coords8(u + ct * nwg, tiles_m, tiles_n, tm, tn);
    const int m0 = tm * TILE, n0 = tn * TILE;
    const unsigned nrec = (unsigned)(TILE * ldc * 2);
    const rsrc_t rc = make_rsrc(C + (size_t)m0 * ldc, nrec);
    rsrc_t rc2 = rc;
    if constexpr (EPI == E8_BIAS_GELU) rc2 = make_rsrc(C2 + (size_t)m0 * ldc, nrec);
    uint2 bq[2][2];
    if constexpr (EXTRA) {
      const char* bl = smem + BIAS_OFF + (ct & 1) * 512;
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bq[nb][j] = *reinterpret_cast<const uint2*>(bl + 2 * (wc * 64 + nb * 32 + 16 * j + 4 * g));
    }
#pragma unroll
    for (int ma = 0; ma < 2; ++ma)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ml = wr * 128 + ma * 64 + 16 * i + (lane & 15);
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
          uint32_t px[2][2];
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            float bb[4] = {0.f, 0.f, 0.f, 0.f};
            if constexpr (EXTRA) {
              bb[0] = bflo(bq[nb][j].x); bb[1] = bfhi(bq[nb][j].x); bb[2] = bflo(bq[nb][j].y); bb[3] = bfhi(bq[nb][j].y);
            }
            const f32x4 v = acc[ma][i][nb][j];
            px[j][0] = pack_bf16x2(v[0] + bb[0], v[1] + bb[1]);
            px[j][1] = pack_bf16x2(v[2] + bb[2], v[3] + bb[3]);
          }
          const auto sx = __builtin_amdgcn_permlane16_swap(px[0][0], px[1][0], false, false);
          const auto sy = __builtin_amdgcn_permlane16_swap(px[0][1], px[1][1], false, false);
          const uint4 o = uint4{sx[0], sy[0], sx[1], sy[1]};
          const int n = n0 + wc * 64 + nb * 32 + 16 * (g & 1) + 8 * (g >> 1);
          const unsigned off = (m0 + ml < M && n < N) ? (unsigned)(ml * ldc + n) * 2u : 0xFFFFFFF0u;
          if (ablate & 1) {
            asm volatile("" ::"v"(o.x), "v"(o.y), "v"(o.z), "v"(o.w));
          } else {
            store_pol(__builtin_bit_cast(u32x4, o), rc, off, (ablate >> 4) & 3);
          }
          if constexpr (EPI == E8_BIAS_GELU) {
            auto gl = [&](float v) { return (!approx && (ablate & 8)) ? gelu_erf_fast(v) : gelu_f(v, approx); };
            const uint4 q = uint4{pack_bf16x2(gl(bflo(o.x)), gl(bfhi(o.x))), pack_bf16x2(gl(bflo(o.y)), gl(bfhi(o.y))),
                                  pack_bf16x2(gl(bflo(o.z)), gl(bfhi(o.z))), pack_bf16x2(gl(bflo(o.w)), gl(bfhi(o.w)))};
            if (ablate & 1) asm volatile("" ::"v"(q.x), "v"(q.y), "v"(q.z), "v"(q.w));
            else store_pol(__builtin_bit_cast(u32x4, q), rc2, off, (ablate >> 4) & 3);
          }
        }
      }
  };

  for (int ct = 0; ct < my_tiles; ++ct) {
    for (int j = 0; j < nh; ++j) {
      const bool ae = j == 0 && ct > 0;  // the previous tile's epilogue stores are in flight
      unroll8<0, 8>([&](auto ph) { phase(ph, ae); });
    }
    epilogue(ct);
    zero_acc();
  }
  if (wr == 0) PZ_BARRIER();  // balance the stagger
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tail's DMA of zeros
}

}  // namespace
}  // namespace penroz

using namespace penroz;

// out[M][N] = a[M][K] · b[N][K]ᵀ (+ bias[N]); with act: out = pre-activation, act = GELU(out).
// bf16, unit column stride, K % 128 == 0, N % 8 == 0, row strides % 8 == 0, 16-B aligned.
void gemm8_bf16(torch::Tensor a, torch::Tensor b, c10::optional<torch::Tensor> bias, torch::Tensor out,
                c10::optional<torch::Tensor> act, int64_t gelu_approx, int64_t ablate) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && out.is_cuda(), "gemm8: GPU tensors");
  TORCH_CHECK(a.scalar_type() == torch::kBFloat16 && b.scalar_type() == torch::kBFloat16 &&
              out.scalar_type() == torch::kBFloat16, "gemm8: bf16 operands");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && out.dim() == 2, "gemm8: 2-D operands");
  TORCH_CHECK(a.stride(1) == 1 && b.stride(1) == 1 && out.stride(1) == 1, "gemm8: unit column stride");
  const int M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(b.size(1) == K, "gemm8: inner dimensions differ");
  TORCH_CHECK(out.size(0) == M && out.size(1) == N, "gemm8: output shape");
  TORCH_CHECK(K % 128 == 0 && K >= 128 && N % 8 == 0, "gemm8: K % 128 == 0 and N % 8 == 0 required");
  TORCH_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0 && out.stride(0) % 8 == 0, "gemm8: row strides % 8");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(b.data_ptr()) % 16 == 0 &&
              reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0, "gemm8: 16-B alignment");
  // the per-lane DMA offset is 32-bit: a 256-row panel of either operand must span < 4 GiB
  TORCH_CHECK((int64_t)256 * std::max({a.stride(0), b.stride(0), out.stride(0)}) * 2 < (int64_t)1 << 31,
              "gemm8: row stride too large (256-row panels are addressed with 32-bit offsets)");
  const bool has_bias = bias.has_value() && bias->defined();
  const bool gelu = act.has_value() && act->defined();
  if (has_bias)
    TORCH_CHECK(bias->scalar_type() == torch::kBFloat16 && bias->numel() == N && bias->is_contiguous() &&
                reinterpret_cast<uintptr_t>(bias->data_ptr()) % 8 == 0, "gemm8: bias [N] bf16");
  if (gelu)
    TORCH_CHECK(has_bias && act->scalar_type() == torch::kBFloat16 && act->sizes() == out.sizes() &&
                act->strides() == out.strides() && reinterpret_cast<uintptr_t>(act->data_ptr()) % 16 == 0,
                "gemm8: the GELU epilogue needs a bias and an act tensor shaped like out");
  if (M == 0 || N == 0) return;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(gemm8_kernel<E8_NONE>), hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    hipFuncSetAttribute(reinterpret_cast<const void*>(gemm8_kernel<E8_BIAS>), hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    hipFuncSetAttribute(reinterpret_cast<const void*>(gemm8_kernel<E8_BIAS_GELU>), hipFuncAttributeMaxDynamicSharedMemorySize,
                        LDS_BYTES);
    attr_set = true;
  }
  static int n_cu = 0;
  if (n_cu == 0) {
    hipDeviceProp_t prop;
    n_cu = hipGetDeviceProperties(&prop, out.get_device()) == hipSuccess ? prop.multiProcessorCount : 256;
  }
  const int tiles_m = (M + TILE - 1) / TILE, tiles_n = (N + TILE - 1) / TILE;
  // persistent: one workgroup per CU (ablate & 4: one workgroup per tile, dispatched as CUs free up)
  const int grid = (ablate & 4) ? tiles_m * tiles_n : std::min(tiles_m * tiles_n, n_cu);
  auto stream = at::hip::getCurrentHIPStream();
  const bf16* ap = reinterpret_cast<const bf16*>(a.data_ptr());
  const bf16* bp = reinterpret_cast<const bf16*>(b.data_ptr());
  const bf16* biasp = has_bias ? reinterpret_cast<const bf16*>(bias->data_ptr()) : nullptr;
  bf16* cp = reinterpret_cast<bf16*>(out.data_ptr());
  bf16* c2 = gelu ? reinterpret_cast<bf16*>(act->data_ptr()) : nullptr;
  const int lda = a.stride(0), ldb = b.stride(0), ldc = out.stride(0);
#define PZ_G8(EPIV)                                                                                             \
  hipLaunchKernelGGL((gemm8_kernel<EPIV>), dim3(grid), dim3(512), LDS_BYTES, stream, ap, bp, biasp, cp, c2, M, N, K, \
                     lda, ldb, ldc, tiles_m, tiles_n, (int)gelu_approx, (int)ablate)
  if (gelu) PZ_G8(E8_BIAS_GELU);
  else if (has_bias) PZ_G8(E8_BIAS);
  else PZ_G8(E8_NONE);
#undef PZ_G8
}

// Diagnostic: one wave DMAs 2 KiB (two bdma2 pieces) from src into LDS at byte offset `lds_off`
// through the same buffer-resource path as the GEMM, then copies that LDS window to out.
namespace penroz {
namespace {
__global__ void __launch_bounds__(64) gemm8_dma_probe_kernel(const bf16* src, unsigned bytes, int lds_off, int soff,
                                                             uint4* out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x;
  for (int i = lane; i < 2048 / 16; i += 64) reinterpret_cast<uint4*>(smem + lds_off)[i] = uint4{7u, 7u, 7u, 7u};
  __syncthreads();
  const unsigned lds_base = (unsigned)(size_t)(lds_void_t*)smem;
  bdma2(make_rsrc(src, bytes), (unsigned)lane * 16u, 1024u + (unsigned)lane * 16u, (unsigned)soff,
        __builtin_amdgcn_readfirstlane(lds_base + lds_off));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = lane; i < 2048 / 16; i += 64) out[i] = reinterpret_cast<const uint4*>(smem + lds_off)[i];
}
}  // namespace
}  // namespace penroz

torch::Tensor gemm8_dma_probe(torch::Tensor src, int64_t bytes, int64_t lds_off, int64_t soff) {
  auto out = torch::empty({128, 4}, src.options().dtype(torch::kInt32));
  hipFuncSetAttribute(reinterpret_cast<const void*>(gemm8_dma_probe_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                      160 * 1024);
  hipLaunchKernelGGL(gemm8_dma_probe_kernel, dim3(1), dim3(64), 160 * 1024, at::hip::getCurrentHIPStream(),
                     reinterpret_cast<const bf16*>(src.data_ptr()), (unsigned)bytes, (int)lds_off, (int)soff,
                     reinterpret_cast<uint4*>(out.data_ptr()));
  return out;
}
