// Forward GEMM with a DEFERRED epilogue, for the linears whose output is followed by an
// elementwise pass (MI355X, gfx950):
//
//   C[M][N] = A[M][K] · B[N][K]ᵀ (+ bias[N]),  bf16 operands, fp32 accumulation, bf16 out
//   EG_GELU:  C = pre-activation, C2 = GELU(C)   (the fc linear of a GPT-2 MLP and its activation)
//
// Why a second GEMM structure (beside hipBLASLt and csrc/kernels/gemm8.hip): the fc linear's output
// goes through a memory-bound GELU kernel (1.8 ms / step at the GPT-2 headline shape) that only a
// GEMM epilogue can remove, and in a persistent kernel whose workgroups run identical tiles the
// epilogue is a chip-wide lock-step burst: every CU stores its 128 KiB tile at the same moment
// (33.5 MB at HBM write speed, ≈ 6 µs) and, because stores and the LDS-DMA of the next tile share
// one in-order VMEM counter per wave, the next tile's MFMA work waits behind it. gemm8 measured the
// burst at ≈ 45 µs of a 221 µs GEMM and a GELU epilogue at ≈ +420 µs of exposed VALU
// (profiles/gemm8_ablate_r4.log) — slower fused than library GEMM + standalone GELU.
//
// Here the epilogue of tile t runs INSIDE tile t+1's main loop:
//   * 4 waves (256 threads), one workgroup per CU, persistent over 256 × 256 tiles; each wave owns a
//     128 × 128 quarter = 4 × 4 v_mfma_f32_32x32x16_bf16 accumulators (256 registers: the AGPR half
//     of the 512-entry register file a single wave per SIMD gets);
//   * at the end of a tile the accumulators (+ bias) are packed to bf16 into 32 "deferred units" of
//     16 B per lane (128 VGPRs: the T21 permlane32 swap makes each unit one 16-B store of 8
//     consecutive columns); during the next tile's first 8 k-tiles, one unit per k-step is stored
//     (EG_GELU: the unit, and GELU of it to C2 — the activation's VALU interleaves with the MFMAs of
//     the same wave), so the output traffic is a steady stream over the tile instead of a burst;
//   * operands by LDS-DMA (buffer_load … lds through buffer resources over the tile's 256-row
//     panels: rows past the edge read 0), two 64-KiB k-tile buffers, ONE barrier per 64-deep k-tile:
//     before it every wave waits (counted vmcnt: the stores issued after the DMA are not waited for)
//     for the next k-tile's DMA, after it the k-tile after that is issued into the buffer just
//     released; fragments of k-step s+1 are read (ds_read_b128, XOR-swizzled [rows][64] image,
//     attn_common.h tile_off) while the MFMAs of k-step s run;
//   * MFMA operands swapped (D = B·Aᵀ): a lane holds 4 consecutive output columns of one row;
//   * XCD-aware bijective tile order, groups of 8 row panels (as gemm8).
// Requirements: K % 128 == 0 and K ≥ 640 (≥ 10 k-tiles: the 32 units drain in k-tiles 0-7, and the
// k-tile buffer parity is compile-time), N % 8 == 0, 16-B aligned rows.
#include "attn_common.h"
#include <type_traits>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

namespace penroz {
namespace {

typedef unsigned u32x4e __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4e lds_u32x4e;
typedef __amdgpu_buffer_rsrc_t rsrc_e;

enum EpiG { EG_NONE = 0, EG_BIAS = 1, EG_GELU = 2, EG_GELU_TANH = 3 };

constexpr int TILE = 256, KT = 64, GM = 8, NUNIT = 32;
constexpr int A_OFF = 0;                // A k-tile buffers: [2][256 rows][128 B]
constexpr int B_OFF = 65536;            // B k-tile buffers
constexpr int KBUF = 32768;             // one operand's k-tile
constexpr int BIAS_OFF = 131072;        // [tile parity][256] bf16
constexpr int BIAS_SINK = BIAS_OFF + 1024;  // waves 2-3's bias piece (uniform VMEM counts)
constexpr int LDS_BYTES = BIAS_SINK + 512;

__device__ __forceinline__ rsrc_e rsrc_of(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, bytes, 0x00020000);
}

// two 1-KiB LDS-DMA pieces (buffer_load_dwordx4 … lds): LDS [lds0, +2 KiB), per-lane byte offsets
// v0 / v1, row / k offset in soffset. M0 saved / restored, only s_mov touches it (an s_add would
// clobber SCC the compiler may keep live across the statement). `s_nop 4`: descriptor / soffset
// SGPRs may have just been written.
__device__ __forceinline__ void dma2(rsrc_e r, unsigned v0, unsigned v1, unsigned soff, unsigned lds0) {
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

// one 256-B piece (buffer_load_dword … lds): 64 lanes × 4 B
__device__ __forceinline__ void dma1(rsrc_e r, unsigned v0, unsigned lds0) {
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

__device__ __forceinline__ void tile_coords(int t, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int per_group = GM * tiles_n;
  const int group = t / per_group;
  const int first_m = group * GM;
  const int gsz = min(tiles_m - first_m, GM);
  const int r = t - group * per_group;
  tm = first_m + r % gsz;
  tn = r / gsz;
}

// erf-GELU, erf from Abramowitz & Stegun 7.1.26 (|error| < 1.5e-7, far below a bf16 ulp of the
// output): one rcp + one exp2 + ~10 VALU, no branches
__device__ __forceinline__ float gelu_erf(float x) {
  const float z = fabsf(x) * 0.7071067811865476f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float e = 1.f - p * t * __builtin_amdgcn_exp2f(-z * z * 1.4426950408889634f);
  return 0.5f * x * (1.f + copysignf(e, x));
}

// tanh-GELU (HF gelu_new), tanh(u) = 1 − 2 / (exp(2u) + 1): one exp2 + one rcp
__device__ __forceinline__ float gelu_tanh(float x) {
  const float u = 0.7978845608028654f * fmaf(0.044715f * x, x * x, x);
  const float e = __builtin_amdgcn_exp2f(fminf(2.f * u * 1.4426950408889634f, 64.f));
  const float th = 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);
  return 0.5f * x * (1.f + th);
}

template <bool TANH>
__device__ __forceinline__ uint32_t gelu_pair(uint32_t u) {
  const float lo = __uint_as_float(u << 16), hi = __uint_as_float(u & 0xffff0000u);
  if constexpr (TANH) return pack_bf16x2(gelu_tanh(lo), gelu_tanh(hi));
  else return pack_bf16x2(gelu_erf(lo), gelu_erf(hi));
}


template <int I, int N, typename F>
__device__ __forceinline__ void unroll(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    unroll<I + 1, N>(f);
  }
}

#define PE_BARRIER()                  \
  do {                                \
    asm volatile("" ::: "memory");    \
    __builtin_amdgcn_s_barrier();     \
    asm volatile("" ::: "memory");    \
  } while (0)

template <int EPI>
__global__ void __launch_bounds__(256, 1) gemm_epi_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                          const bf16* __restrict__ bias, bf16* __restrict__ C,
                                                          bf16* __restrict__ C2, int M, int N, int K, int lda, int ldb,
                                                          int ldc, int tiles_m, int tiles_n, int approx, int flags) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr bool HAS_BIAS = EPI != EG_NONE;
  constexpr bool GELU = EPI == EG_GELU || EPI == EG_GELU_TANH;
  constexpr int SPU = GELU ? 2 : 1;  // stores per deferred unit
  const int lane = threadIdx.x & 63, hh = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, qd = nwg >> 3, rd = nwg & 7;
  const int u0 = (xcd < rd ? xcd * (qd + 1) : rd * (qd + 1) + (xcd - rd) * qd) + (bid >> 3);
  const int ntiles = tiles_m * tiles_n;
  const int my_tiles = (ntiles - u0 + nwg - 1) / nwg;
  const int nk = K / KT;
  const unsigned lds_base = (unsigned)(size_t)(lds_void_t*)smem;
  const bool no_stores = (flags & 1) != 0;

  // ---- DMA stream (wave-uniform state): local tile dti, k-tile dkt; panel pointers / sizes
  int dti = 0, dkt = 0;
  const bf16* pa = A;
  const bf16* pb = B;
  const bf16* pbias = bias;
  unsigned na = 0, nbb = 0, nbias = 0;
  auto set_dma_tile = [&](int t) {
    int tm, tn;
    tile_coords(u0 + min(t, max(my_tiles - 1, 0)) * nwg, tiles_m, tiles_n, tm, tn);
    const int m0 = tm * TILE, n0 = tn * TILE;
    const bool live = t < my_tiles;  // past the last tile: empty resources (the tail keeps its counts)
    pa = A + (size_t)m0 * lda;
    pb = B + (size_t)n0 * ldb;
    na = live ? (unsigned)(min(M - m0, TILE) * lda * 2) : 0u;
    nbb = live ? (unsigned)(min(N - n0, TILE) * ldb * 2) : 0u;
    if constexpr (HAS_BIAS) {
      pbias = bias + n0;
      nbias = live ? (unsigned)(min(N - n0, TILE) * 2) : 0u;
    }
  };
  // per-lane source offsets of a piece (8 rows × 128 B): lane -> row r8 = lane >> 3 of the piece,
  // LDS slot lane & 7, which holds logical chunk slot ^ swz(row) (attn_common.h tile_off). A pair's
  // second piece is 8 rows further: row bit 3 enters the swizzle, so it has its own offsets.
  // (recomputed at each use from an opaque lane id: kept live across the loop they were spilled)
  auto swz_row = [](int r) { return (((r >> 1) & 1) << 2) | ((r >> 2) & 3); };
  // wave-uniform bases of this wave's DMA rows (64w ..): LDS byte address and the panel byte
  // offsets of the first row in A / B, and the stride of 16 rows. They are passed through an empty
  // asm at every use so the compiler recomputes the per-piece sums (a few SALU adds) instead of
  // hoisting 16+ precomputed SGPRs out of the loop (which spilled SGPRs into VGPR lanes)
  const unsigned lds_w0 = __builtin_amdgcn_readfirstlane(lds_base + (unsigned)(64 * w * 128));
  const unsigned sa_w0 = (unsigned)(64 * w * lda * 2), sb_w0 = (unsigned)(64 * w * ldb * 2);
  const unsigned sa16_0 = (unsigned)(16 * lda * 2), sb16_0 = (unsigned)(16 * ldb * 2);
  // k-tile dkt of the stream into buffer PAR: this wave's 64 rows of A and of B (4 piece pairs each)
  auto issue_dma = [&](auto par_c) {
    constexpr int PAR = decltype(par_c)::value;
    unsigned lw = lds_w0, sa = sa_w0, sb = sb_w0, sa16 = sa16_0, sb16 = sb16_0;
    asm volatile("" : "+s"(lw), "+s"(sa), "+s"(sb), "+s"(sa16), "+s"(sb16));
    if constexpr (HAS_BIAS) {
      if (dkt == 0)  // the tile's bias slice rides with its first k-tile (every wave issues one piece)
        dma1(rsrc_of(pbias, nbias), (unsigned)(128 * (w & 1) + 2 * opaque_lane_id()) * 2u,
             __builtin_amdgcn_readfirstlane(w < 2 ? lds_base + BIAS_OFF + (dti & 1) * 512 + (w & 1) * 256
                                                  : lds_base + BIAS_SINK + (w - 2) * 128));
    }
    const int ln = opaque_lane_id(), r8 = ln >> 3;
    const int ch0 = (ln & 7) ^ swz_row(r8), ch1 = (ln & 7) ^ swz_row(8 + r8);
    const unsigned va0 = (unsigned)(r8 * lda + 8 * ch0) * 2u, va1 = (unsigned)((8 + r8) * lda + 8 * ch1) * 2u;
    const unsigned vb0 = (unsigned)(r8 * ldb + 8 * ch0) * 2u, vb1 = (unsigned)((8 + r8) * ldb + 8 * ch1) * 2u;
    const rsrc_e ra = rsrc_of(pa, na), rb = rsrc_of(pb, nbb);
    const unsigned kof = (unsigned)(dkt * KT * 2);
    sa += kof;
    sb += kof;
#pragma unroll
    for (int pp = 0; pp < 4; ++pp) {
      dma2(ra, va0, va1, sa, lw + (unsigned)(A_OFF + PAR * KBUF + pp * 16 * 128));
      dma2(rb, vb0, vb1, sb, lw + (unsigned)(B_OFF + PAR * KBUF + pp * 16 * 128));
      sa += sa16;
      sb += sb16;
    }
    if (++dkt == nk) {
      dkt = 0;
      set_dma_tile(++dti);
    }
  };

  // ---- fragment reads: row 32·f + (lane & 31) of the wave's 128-row half, chunk 2s + hh
  const int rl = lane & 31;
  const int swl = (((rl >> 1) & 1) << 2) | ((rl >> 2) & 3);
  // per-lane fragment base per k-step s (the wave's half of A / B included): every fragment read
  // is then base + an immediate (buffer parity, fragment row block) of at most 45 056 bytes
  unsigned ab[4], bb[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const unsigned fo = (unsigned)(rl * 128 + (((2 * s + hh) ^ swl) << 4));
    ab[s] = (unsigned)(A_OFF + wr * 128 * 128) + fo;
    bb[s] = (unsigned)(B_OFF + wc * 128 * 128) + fo;
    asm volatile("" : "+v"(ab[s]), "+v"(bb[s]));
  }
  auto lds16 = [&](unsigned off) -> uint4 { return __builtin_bit_cast(uint4, *(const lds_u32x4e*)(smem + off)); };

  f32x16 acc[4][4];
  auto zero_acc = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  };
  zero_acc();
  uint4 fa[2][4], fb[2][4];
  auto load_a = [&](auto par_c, auto s_c, auto slot_c, int f) {
    constexpr int PAR = decltype(par_c)::value, S = decltype(s_c)::value, SL = decltype(slot_c)::value;
    fa[SL][f] = lds16(ab[S] + PAR * KBUF + f * 32 * 128);
  };
  auto load_b = [&](auto par_c, auto s_c, auto slot_c) {
    constexpr int PAR = decltype(par_c)::value, S = decltype(s_c)::value, SL = decltype(slot_c)::value;
#pragma unroll
    for (int f = 0; f < 4; ++f) fb[SL][f] = lds16(bb[S] + PAR * KBUF + f * 32 * 128);
  };
  auto load_frags = [&](auto par_c, auto s_c, auto slot_c) {
    load_b(par_c, s_c, slot_c);
#pragma unroll
    for (int f = 0; f < 4; ++f) load_a(par_c, s_c, slot_c, f);
  };

  // ---- deferred output of the previous tile: unit U = (im, jn, kp) -> 8 columns of one row
  // store addressing: the tile's C / C2 panel resources cover its live rows only (rows past M are
  // dropped by the range check); per lane one row offset and one column, per unit an immediate
  // column offset and the row block IM·32 rows in soffset; columns past N get an offset past the
  // resource. Every lane stores, so the per-k-step store count is exact for the counted waits.
  uint4 dout[NUNIT];
  const bf16* cpan = C;
  const bf16* c2pan = C2;
  unsigned crec = 0;      // resource size: 0 before the first tile (its units are dropped)
  int ncols = 0;          // live columns of the deferred tile
  unsigned vrow = (unsigned)(((wr * 128 + rl) * ldc + wc * 128 + 8 * hh) * 2);
  int vcol = wc * 128 + 8 * hh;
  asm volatile("" : "+v"(vrow), "+v"(vcol));
  const unsigned ld32_0 = (unsigned)(32 * ldc * 2);
  auto store_unit = [&](auto u_c) {
    constexpr int U = decltype(u_c)::value;
    constexpr int IM = U >> 3, JN = (U >> 1) & 3, KP = U & 1;
    constexpr int CO = JN * 32 + KP * 16;
    // opaque copies: the 32 units' offsets are recomputed at each store instead of being hoisted
    // to the top of the tile (32 live VGPRs beside the deferred units spilled)
    unsigned ld32 = ld32_0, vr = vrow;
    int vc = vcol, nc = ncols;
    asm volatile("" : "+s"(ld32), "+v"(vr), "+v"(vc), "+s"(nc));
    const unsigned off = vc + CO < nc ? vr + (unsigned)(CO * 2) : 0x80000000u;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4e, dout[U]), rsrc_of(cpan, crec), (int)off,
                                           (int)(IM * ld32), 0);
    if constexpr (GELU) {
      constexpr bool TH = EPI == EG_GELU_TANH;
      const uint4 d = dout[U];
      const uint4 q = uint4{gelu_pair<TH>(d.x), gelu_pair<TH>(d.y), gelu_pair<TH>(d.z), gelu_pair<TH>(d.w)};
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4e, q), rsrc_of(c2pan, crec), (int)off,
                                             (int)(IM * ld32), 0);
    }
  };

  // ---- one 64-deep k-tile (buffer PAR): 4 k-steps of 16 MFMAs; unit 4·KTU + s after k-step s
  // (KTU < 8), the barrier after k-step 2 (waits for the next k-tile: VMC stores issued since its
  // DMA), then the DMA of the k-tile after next, and the next k-tile's first fragments during
  // k-step 3
  auto ktile = [&](auto par_c, auto ktu_c, auto vmc_c) {
    constexpr int PAR = decltype(par_c)::value, KTU = decltype(ktu_c)::value, VMC = decltype(vmc_c)::value;
    unroll<0, 4>([&](auto s_c) {
      constexpr int S = decltype(s_c)::value;
      // the next k-step's operands: in this k-tile's buffer for k-steps 1-3, the next k-tile's
      // (released by the barrier of k-step 2) for k-step 0. B fragments first (all four rows of
      // MFMAs read them); A fragment i as soon as MFMA row i has consumed the current one, so the
      // two operand sets overlap in 52 registers rather than 64
      constexpr int NP = S < 3 ? PAR : (PAR ^ 1), NS = S < 3 ? S + 1 : 0, NSL = (S + 1) & 1;
      using NPc = std::integral_constant<int, NP>;
      using NSc = std::integral_constant<int, NS>;
      using NSLc = std::integral_constant<int, NSL>;
      load_b(NPc{}, NSc{}, NSLc{});
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma32(fb[S & 1][j], fa[S & 1][i], acc[i][j]);
        load_a(NPc{}, NSc{}, NSLc{}, i);
      }
      __builtin_amdgcn_s_setprio(0);
      if constexpr (KTU < 8) store_unit(std::integral_constant<int, 4 * KTU + S>{});
      if constexpr (S == 2) {
        // the k-step-3 fragments (read above) are in registers before the buffer is released
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VMC * SPU) : "memory");
        PE_BARRIER();
        issue_dma(std::integral_constant<int, PAR>{});
      }
    });
  };
  // vmcnt after k-tile KTU's barrier: units of k-step 3 of the previous k-tile and k-steps 0-2 of
  // this one (in units; the previous tile's last k-tile carries none)
#define PE_KT(P, KTU, VMC) ktile(std::integral_constant<int, P>{}, std::integral_constant<int, KTU>{}, \
                                 std::integral_constant<int, VMC>{})

  // ---- prologue: k-tiles 0 and 1 of the first tile in flight, the first landed
  set_dma_tile(0);
  issue_dma(std::integral_constant<int, 0>{});
  issue_dma(std::integral_constant<int, 1>{});
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  PE_BARRIER();
  load_frags(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});

  for (int ct = 0; ct < my_tiles; ++ct) {
    PE_KT(0, 0, 3); PE_KT(1, 1, 4); PE_KT(0, 2, 4); PE_KT(1, 3, 4);
    PE_KT(0, 4, 4); PE_KT(1, 5, 4); PE_KT(0, 6, 4); PE_KT(1, 7, 4);
    PE_KT(0, 8, 1); PE_KT(1, 9, 0);
    for (int kt = 10; kt < nk; kt += 2) {
      PE_KT(0, 8 + 2, 0);
      PE_KT(1, 8 + 2, 0);
    }
    // ---- tile end: accumulators (+ bias) -> the deferred units of this tile
    int tm, tn;
    tile_coords(u0 + ct * nwg, tiles_m, tiles_n, tm, tn);
    const int pm0 = tm * TILE, pn0 = tn * TILE;
    cpan = C + (size_t)pm0 * ldc;
    if constexpr (GELU) c2pan = C2 + (size_t)pm0 * ldc;
    crec = no_stores ? 0u : (unsigned)(min(M - pm0, TILE) * ldc * 2);
    ncols = N - pn0;
    const char* bl = smem + BIAS_OFF + (ct & 1) * 512;
#pragma unroll
    for (int jn = 0; jn < 4; ++jn) {
      float bv[4][4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if constexpr (HAS_BIAS) {
          const uint2 q = *reinterpret_cast<const uint2*>(bl + 2 * (wc * 128 + jn * 32 + 8 * k + 4 * hh));
          bv[k][0] = __uint_as_float(q.x << 16); bv[k][1] = __uint_as_float(q.x & 0xffff0000u);
          bv[k][2] = __uint_as_float(q.y << 16); bv[k][3] = __uint_as_float(q.y & 0xffff0000u);
        } else {
          bv[k][0] = bv[k][1] = bv[k][2] = bv[k][3] = 0.f;
        }
      }
#pragma unroll
      for (int im = 0; im < 4; ++im)
#pragma unroll
        for (int kp = 0; kp < 2; ++kp) {
          const f32x16& v = acc[im][jn];
          const int ka = 2 * kp, kb = 2 * kp + 1;
          uint32_t ax = pack_bf16x2(v[4 * ka] + bv[ka][0], v[4 * ka + 1] + bv[ka][1]);
          uint32_t ay = pack_bf16x2(v[4 * ka + 2] + bv[ka][2], v[4 * ka + 3] + bv[ka][3]);
          uint32_t bx = pack_bf16x2(v[4 * kb] + bv[kb][0], v[4 * kb + 1] + bv[kb][1]);
          uint32_t by = pack_bf16x2(v[4 * kb + 2] + bv[kb][2], v[4 * kb + 3] + bv[kb][3]);
          const auto sx = __builtin_amdgcn_permlane32_swap(ax, bx, false, false);
          const auto sy = __builtin_amdgcn_permlane32_swap(ay, by, false, false);
          dout[im * 8 + jn * 2 + kp] = uint4{sx[0], sy[0], sx[1], sy[1]};
        }
    }
    zero_acc();
  }
#undef PE_KT
  // the last tile's units
  unroll<0, NUNIT>([&](auto u_c) { store_unit(u_c); });
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tail's DMA of zeros, the last stores
}

}  // namespace
}  // namespace penroz

using namespace penroz;

// out[M][N] = a[M][K] · b[N][K]ᵀ (+ bias[N]); with act: out = pre-activation, act = GELU(out).
// bf16, unit column stride, K % 128 == 0, K >= 640, N % 8 == 0, row strides % 8 == 0, 16-B aligned.
// flags (timing ablation): 1 no stores (outputs wrong)
bool gemm_epi_supported(int64_t M, int64_t N, int64_t K) { return K % 128 == 0 && K >= 640 && N % 8 == 0 && M > 0; }

void gemm_epi_bf16(torch::Tensor a, torch::Tensor b, c10::optional<torch::Tensor> bias, torch::Tensor out,
                   c10::optional<torch::Tensor> act, int64_t gelu_approx, int64_t flags) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && out.is_cuda(), "gemm_epi: GPU tensors");
  TORCH_CHECK(a.scalar_type() == torch::kBFloat16 && b.scalar_type() == torch::kBFloat16 &&
                  out.scalar_type() == torch::kBFloat16, "gemm_epi: bf16 operands");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && out.dim() == 2, "gemm_epi: 2-D operands");
  TORCH_CHECK(a.stride(1) == 1 && b.stride(1) == 1 && out.stride(1) == 1, "gemm_epi: unit column stride");
  const int M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(b.size(1) == K, "gemm_epi: inner dimensions differ");
  TORCH_CHECK(out.size(0) == M && out.size(1) == N, "gemm_epi: output shape");
  TORCH_CHECK(gemm_epi_supported(M, N, K), "gemm_epi: K % 128 == 0, K >= 640 and N % 8 == 0 required");
  TORCH_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0 && out.stride(0) % 8 == 0, "gemm_epi: row strides % 8");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(b.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0, "gemm_epi: 16-B alignment");
  TORCH_CHECK((int64_t)256 * std::max({a.stride(0), b.stride(0), out.stride(0)}) * 2 < (int64_t)1 << 31,
              "gemm_epi: row stride too large (256-row panels are addressed with 32-bit offsets)");
  const bool has_bias = bias.has_value() && bias->defined();
  const bool gelu = act.has_value() && act->defined();
  if (has_bias)
    TORCH_CHECK(bias->scalar_type() == torch::kBFloat16 && bias->numel() == N && bias->is_contiguous() &&
                    reinterpret_cast<uintptr_t>(bias->data_ptr()) % 4 == 0, "gemm_epi: bias [N] bf16");
  if (gelu)
    TORCH_CHECK(has_bias && act->scalar_type() == torch::kBFloat16 && act->sizes() == out.sizes() &&
                    act->strides() == out.strides() && reinterpret_cast<uintptr_t>(act->data_ptr()) % 16 == 0,
                "gemm_epi: the GELU epilogue needs a bias and an act tensor shaped like out");
  if (M == 0 || N == 0) return;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_epi_kernel<EG_NONE>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_epi_kernel<EG_BIAS>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_epi_kernel<EG_GELU>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_epi_kernel<EG_GELU_TANH>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    attr_set = true;
  }
  static int n_cu = 0;
  if (n_cu == 0) {
    hipDeviceProp_t prop;
    n_cu = hipGetDeviceProperties(&prop, out.get_device()) == hipSuccess ? prop.multiProcessorCount : 256;
  }
  const int tiles_m = (M + TILE - 1) / TILE, tiles_n = (N + TILE - 1) / TILE;
  const int grid = std::min(tiles_m * tiles_n, n_cu);
  auto stream = at::hip::getCurrentHIPStream();
  const bf16* ap = reinterpret_cast<const bf16*>(a.data_ptr());
  const bf16* bp = reinterpret_cast<const bf16*>(b.data_ptr());
  const bf16* biasp = has_bias ? reinterpret_cast<const bf16*>(bias->data_ptr()) : nullptr;
  bf16* cp = reinterpret_cast<bf16*>(out.data_ptr());
  bf16* c2 = gelu ? reinterpret_cast<bf16*>(act->data_ptr()) : nullptr;
  const int lda = a.stride(0), ldb = b.stride(0), ldc = out.stride(0);
#define PE_LAUNCH(EPIV)                                                                                         \
  hipLaunchKernelGGL((gemm_epi_kernel<EPIV>), dim3(grid), dim3(256), LDS_BYTES, stream, ap, bp, biasp, cp, c2, M, N, \
                     K, lda, ldb, ldc, tiles_m, tiles_n, (int)gelu_approx, (int)flags)
  if (gelu && gelu_approx) PE_LAUNCH(EG_GELU_TANH);
  else if (gelu) PE_LAUNCH(EG_GELU);
  else if (has_bias) PE_LAUNCH(EG_BIAS);
  else PE_LAUNCH(EG_NONE);
#undef PE_LAUNCH
}
