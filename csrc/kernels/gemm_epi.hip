// Forward GEMM with a DEFERRED epilogue, for the linears whose output is followed by an
// elementwise pass (MI355X, gfx950):
//
//   C[M][N] = A[M][K] · B[N][K]ᵀ (+ bias[N]),  bf16 operands, fp32 accumulation, bf16 out
//   EG_GELU:  C = pre-activation, C2 = GELU(C)   (the fc linear of a GPT-2 MLP and its activation)
//   EG_DGELU: C = bf16(A·Bᵀ) · GELU'(P), and the column sums of C (the fc bias gradient) as
//             per-128-row partial rows   (fc2's data gradient and the GELU backward, one kernel)
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
#include "deferred.h"
#include <type_traits>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

namespace penroz {
namespace {

typedef unsigned u32x4e __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4e lds_u32x4e;
typedef __amdgpu_buffer_rsrc_t rsrc_e;

enum EpiG { EG_NONE = 0, EG_BIAS = 1, EG_GELU = 2, EG_GELU_TANH = 3, EG_DGELU = 4, EG_DGELU_TANH = 5 };

constexpr int TILE = 256, KT = 64, GM = 8, NUNIT = 32;
constexpr int A_OFF = 0;                // A k-tile buffers: [2][256 rows][128 B]
constexpr int B_OFF = 65536;            // B k-tile buffers
constexpr int KBUF = 32768;             // one operand's k-tile
constexpr int BIAS_OFF = 131072;        // [tile parity][256] bf16
constexpr int BIAS_SINK = BIAS_OFF + 1024;  // waves 2-3's bias piece (uniform VMEM counts)
// non-DGELU: per-wave staging of 4 deferred units (32 rows x 64 columns bf16), read back as
// full 128-B row segments for the stores
constexpr int STAGE_OFF = BIAS_SINK + 512;
constexpr int LDS_BYTES = STAGE_OFF + 4 * 4096;
// EG_DGELU (no bias): the P chunks of the deferred units ride with the k-tile stream into
// [k-tile parity][unit step][wave][64 lanes × 16 B] after the operand buffers (exactly 160 KiB)
constexpr int P_OFF = 131072;
constexpr int LDS_BYTES_DG = P_OFF + 2 * 4 * 4 * 1024;

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

// one 1-KiB piece (buffer_load_dwordx4 … lds) with a scalar offset: 64 lanes × 16 B
__device__ __forceinline__ void dmaP(rsrc_e r, unsigned v0, unsigned soff, unsigned lds0) {
  unsigned keep;
  asm volatile(
      "s_nop 4\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %4\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %3 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(v0), "s"(r), "s"(soff), "s"(lds0)
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

// GELU'(x): erf form cdf + x·pdf with the A&S erf sharing its exp(−x²/2) with the pdf; tanh form
// as elementwise.hip gelu_grad_f
template <bool TANH>
__device__ __forceinline__ float gelu_grad(float x) {
  if constexpr (TANH) {
    const float k = 0.7978845608028654f, x2 = x * x;
    const float u = k * fmaf(0.044715f * x, x2, x);
    const float e = __builtin_amdgcn_exp2f(fminf(2.f * u * 1.4426950408889634f, 64.f));
    const float t = 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);
    return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k * (1.f + 3.f * 0.044715f * x2);
  } else {
    const float z = fabsf(x) * 0.7071067811865476f;
    const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.f));
    float p = fmaf(1.061405429f, t, -1.453152027f);
    p = fmaf(p, t, 1.421413741f);
    p = fmaf(p, t, -0.284496736f);
    p = fmaf(p, t, 0.254829592f);
    const float e = __builtin_amdgcn_exp2f(-z * z * 1.4426950408889634f);  // exp(−x²/2)
    const float erfz = 1.f - p * t * e;
    return 0.5f * (1.f + copysignf(erfz, x)) + x * 0.3989422804014327f * e;
  }
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
                                                          bf16* __restrict__ C2, const bf16* __restrict__ P,
                                                          float* __restrict__ colpart, int M, int N, int K, int lda,
                                                          int ldb, int ldc, int tiles_m, int tiles_n, int flags) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr bool GELU = EPI == EG_GELU || EPI == EG_GELU_TANH;
  constexpr bool DGELU = EPI == EG_DGELU || EPI == EG_DGELU_TANH;
  constexpr bool TANH = EPI == EG_GELU_TANH || EPI == EG_DGELU_TANH;
  constexpr bool HAS_BIAS = EPI == EG_BIAS || GELU;
  // VMEM operations per unit step (every one issued on every unit step, dummies included, so the
  // counted waits are compile-time constants): GELU stores C and C2; DGELU stores C and two 16-B
  // column-sum pieces (its P chunks arrive by LDS-DMA with the k-tile stream)
  constexpr int OPS = GELU ? 2 : (DGELU ? 3 : 1);
  constexpr int PPC = DGELU ? 4 : 0;  // P pieces in the DMA of k-tiles 0-7
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
  const unsigned ld32_0 = (unsigned)(32 * ldc * 2);  // 32 output rows in bytes
  // DGELU: the P panel of the stream's PREVIOUS tile (its units are stored during this one)
  const bf16* ppan_s = P;
  unsigned prec_s = 0;
  int pncols_s = 0, pn0_s = 0;
  int cur_m0 = 0, cur_n0 = 0;
  auto set_dma_tile = [&](int t) {
    if constexpr (DGELU) {
      ppan_s = P + (size_t)cur_m0 * ldc;
      prec_s = t > 0 ? (unsigned)(min(M - cur_m0, TILE) * ldc * 2) : 0u;
      pncols_s = N - cur_n0;
      pn0_s = cur_n0;
    }
    int tm, tn;
    tile_coords(u0 + min(t, max(my_tiles - 1, 0)) * nwg, tiles_m, tiles_n, tm, tn);
    const int m0 = tm * TILE, n0 = tn * TILE;
    cur_m0 = m0;
    cur_n0 = n0;
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
    if constexpr (DGELU) {
      // the P chunks of unit steps 0-3 of k-tile dkt (units 4·dkt + s: row block s, columns 16·dkt)
      // of the deferred tile, one 1-KiB piece per wave and step, lane-linear like the stores
      if (dkt < 8) {
        const int l2 = opaque_lane_id();
        const int vc = wc * 128 + 8 * (l2 >> 5) + 16 * dkt;  // column within the tile
        const unsigned vr = (unsigned)(((wr * 128 + (l2 & 31)) * ldc + vc) * 2);
        const unsigned pcol2_s = (unsigned)(pn0_s * 2);
        const unsigned voff = vc < pncols_s ? vr : 0x80000000u;
        unsigned ld32 = ld32_0;
        asm volatile("" : "+s"(ld32));
        const rsrc_e rp = rsrc_of(ppan_s, prec_s);
#pragma unroll
        for (int st = 0; st < 4; ++st)
          dmaP(rp, voff, st * ld32 + pcol2_s, lw - (unsigned)(64 * w * 128) + (unsigned)(P_OFF + (PAR * 4 + st) * 4096 + w * 1024));
      }
    }
    if (++dkt == nk) {
      dkt = 0;
      set_dma_tile(++dti);
    }
  };

  // ---- fragment reads: row 32·f + (lane & 31) of the wave's 128-row half, chunk 2s + hh
  const int rl = lane & 31;
  const int swl = (((rl >> 1) & 1) << 2) | ((rl >> 2) & 3);
  // per-lane fragment bases of k-step 0 (the wave's half of A / B included); k-step s reads chunk
  // 2s + hh ^ swz = that of k-step 0 XOR 2s, i.e. base XOR (s << 5) (the added constants have
  // bits 5-6 clear). Every fragment read is then base + an immediate (buffer parity, fragment row
  // block) of at most 45 056 bytes. The XOR is redone per k-step on an opaque copy: 2 live
  // registers instead of 8 precomputed bases (the tile-end peak is 12 registers short)
  unsigned ab0 = (unsigned)(A_OFF + wr * 128 * 128 + rl * 128 + ((hh ^ swl) << 4));
  unsigned bb0 = (unsigned)(B_OFF + wc * 128 * 128 + rl * 128 + ((hh ^ swl) << 4));
  asm volatile("" : "+v"(ab0), "+v"(bb0));
  auto abase = [&](int S) { unsigned x = ab0; asm volatile("" : "+v"(x)); return S ? x ^ (unsigned)(S << 5) : x; };
  auto bbase = [&](int S) { unsigned x = bb0; asm volatile("" : "+v"(x)); return S ? x ^ (unsigned)(S << 5) : x; };
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
    fa[SL][f] = lds16(abase(S) + PAR * KBUF + f * 32 * 128);
  };
  auto load_b = [&](auto par_c, auto s_c, auto slot_c) {
    constexpr int PAR = decltype(par_c)::value, S = decltype(s_c)::value, SL = decltype(slot_c)::value;
    const unsigned b0 = bbase(S);
#pragma unroll
    for (int f = 0; f < 4; ++f) fb[SL][f] = lds16(b0 + PAR * KBUF + f * 32 * 128);
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
  uint4 pr3 = uint4{0u, 0u, 0u, 0u};  // DGELU: unit step 3's P chunk, read before its slot is released
  float cs[8];            // DGELU: this lane's running column sums of the current 8 columns
#pragma unroll
  for (int e = 0; e < 8; ++e) cs[e] = 0.f;
  const bf16* ppan = P;
  int cprow = 0, pn0c = 0;  // DGELU: partial-row index of the wave's 128 rows, tile's first column
  const unsigned cprec = DGELU ? (unsigned)(tiles_m * 2 * N * 4) : 0u;
  const bf16* cpan = C;
  const bf16* c2pan = C2;
  unsigned crec = 0;      // resource size: 0 before the first tile (its units are dropped)
  int ncols = 0;          // live columns of the deferred tile
  // DGELU stores a unit per lane pair and row (16 B at column 8·hh); the others store 4 staged
  // units as 8 rows x 128 B per instruction (lane -> row lane >> 3, 8 columns at 8·(lane & 7))
  unsigned vrow = DGELU ? (unsigned)(((wr * 128 + rl) * ldc + wc * 128 + 8 * hh) * 2)
                        : (unsigned)(((wr * 128 + (lane >> 3)) * ldc + wc * 128 + 8 * (lane & 7)) * 2);
  int vcol = DGELU ? wc * 128 + 8 * hh : wc * 128 + 8 * (lane & 7);
  asm volatile("" : "+v"(vrow), "+v"(vcol));
  int pcol2 = 0;  // byte offset of the deferred tile's first column (its panel starts at column 0)
  // unit U: C[row block IM, 8 columns at CO + 8·hh] of the deferred tile. DGELU: `pr` is the unit's
  // P chunk (from LDS in the loop, from global memory in the final flush)
  auto store_unit = [&](auto u_c, uint4 pr) {
    constexpr int U = decltype(u_c)::value;
    constexpr int IM = U & 3, KP = (U >> 2) & 1, JN = U >> 3;  // the 4 row blocks of 8 columns in a row
    constexpr int CO = JN * 32 + KP * 16;
    // opaque copies: the 32 units' offsets are recomputed at each store instead of being hoisted
    // to the top of the tile (32 live VGPRs beside the deferred units spilled)
    unsigned ld32 = ld32_0, vr = vrow;
    int vc = vcol, nc = ncols, pc2 = pcol2;
    asm volatile("" : "+s"(ld32), "+v"(vr), "+v"(vc), "+s"(nc), "+s"(pc2));
    const unsigned off = vc + CO < nc ? vr + (unsigned)(CO * 2) : 0x80000000u;
    const int soff = (int)(IM * ld32) + pc2;
    if constexpr (DGELU) {
      // dC = bf16(acc) · GELU'(P) and its column sums
      const uint4 d = dout[U];
      const uint32_t dw[4] = {d.x, d.y, d.z, d.w}, pw[4] = {pr.x, pr.y, pr.z, pr.w};
      uint32_t ow[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float g0 = __uint_as_float(dw[e] << 16) * gelu_grad<TANH>(__uint_as_float(pw[e] << 16));
        const float g1 = __uint_as_float(dw[e] & 0xffff0000u) * gelu_grad<TANH>(__uint_as_float(pw[e] & 0xffff0000u));
        ow[e] = pack_bf16x2(g0, g1);
        // the column sums add the ROUNDED gradient (what the fc dgrad / wgrad GEMMs read), as the
        // unfused GELU-backward kernel does
        cs[2 * e] += __uint_as_float(ow[e] << 16);
        cs[2 * e + 1] += __uint_as_float(ow[e] & 0xffff0000u);
      }
      __builtin_amdgcn_raw_buffer_store_b128(u32x4e{ow[0], ow[1], ow[2], ow[3]}, rsrc_of(cpan, crec), (int)off, soff, 0);
      // after the 4th row block of these 8 columns: sum over the 32 rows of the lane half
      // (lanes rl = 0..31 hold the same columns), lane rl == 0 writes 8 partial sums; the two
      // 16-B stores are issued at every unit step (dropped unless they carry sums): exact counts
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = cs[e];
      if constexpr (IM == 3) {
#pragma unroll
        for (int m = 1; m < 32; m <<= 1)
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += __shfl_xor(v[e], m, 64);
#pragma unroll
        for (int e = 0; e < 8; ++e) cs[e] = 0.f;
      }
      const bool writer = IM == 3 && (opaque_lane_id() & 31) == 0 && vc + CO < nc;
      const unsigned co = writer ? (unsigned)((cprow * N + (pn0c + vc + CO)) * 4) : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b128(u32x4e{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                                                    __float_as_uint(v[3])}, rsrc_of(colpart, cprec), (int)co, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(u32x4e{__float_as_uint(v[4]), __float_as_uint(v[5]), __float_as_uint(v[6]),
                                                    __float_as_uint(v[7])}, rsrc_of(colpart, cprec),
                                             (int)(writer ? co + 16u : 0x80000000u), 0, 0);
    } else {
      // unit U = (IM, column pair JP, G = 2·jn-in-pair + kp): stage it as columns 16·G + 8·hh of a
      // [32 rows][64 columns] image (16-B chunks XOR-swizzled by row); after the 4th unit of the
      // group the wave reads the image back 8 rows at a time and stores full 128-B row segments
      // (the lane-pair layout of the MFMA output would store 32-B segments: a quarter of a line)
      (void)off;
      (void)soff;
      constexpr int G = U & 3, JP = (U >> 2) & 1, IMS = U >> 3;
      const int ln = opaque_lane_id(), r = ln & 31, h = ln >> 5;
      const unsigned sw = (unsigned)(STAGE_OFF + w * 4096 + r * 128 + (((2 * G + h) ^ (r & 7)) << 4));
      *(lds_u32x4e*)(smem + sw) = __builtin_bit_cast(u32x4e, dout[U]);
      if constexpr (G == 3) {
        const unsigned rd0 = (unsigned)(STAGE_OFF + w * 4096 + (ln >> 3) * 128 + (((ln & 7) ^ (ln >> 3)) << 4));
        const unsigned soff0 = (unsigned)(IMS * ld32 + pc2);
        const unsigned off2 = vc + 64 * JP < nc ? vr + (unsigned)(128 * JP) : 0x80000000u;
        // one 8-row piece at a time (sched barriers: hoisting the 4 reads costs 16 registers the
        // deferred units do not leave)
#pragma unroll
        for (int q8 = 0; q8 < 4; ++q8) {
          __builtin_amdgcn_sched_barrier(0);
          const uint4 d = lds16(rd0 + q8 * 1024);
          const int so = (int)(soff0 + q8 * (ld32 >> 2));
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4e, d), rsrc_of(cpan, crec), (int)off2, so, 0);
          if constexpr (GELU) {
            constexpr bool TH = EPI == EG_GELU_TANH;
            const uint4 q = uint4{gelu_pair<TH>(d.x), gelu_pair<TH>(d.y), gelu_pair<TH>(d.z), gelu_pair<TH>(d.w)};
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4e, q), rsrc_of(c2pan, crec), (int)off2, so, 0);
          }
        }
      }
    }
  };
  // DGELU: this lane's P chunk of unit step S of k-tile parity PAR (LDS, staged by the DMA stream)
  const unsigned plds = (unsigned)(P_OFF + w * 1024 + lane * 16);
  auto p_lds = [&](auto par_c, auto s_c) -> uint4 {
    constexpr int PAR = decltype(par_c)::value, S = decltype(s_c)::value;
    return lds16(plds + (unsigned)((PAR * 4 + S) * 4096));
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
      if constexpr (KTU < 8) {
        uint4 pr = uint4{0u, 0u, 0u, 0u};
        if constexpr (DGELU) {
          if constexpr (S < 3) pr = p_lds(std::integral_constant<int, PAR>{}, std::integral_constant<int, S>{});
          else pr = pr3;
        }
        store_unit(std::integral_constant<int, 4 * KTU + S>{}, pr);
      }
      if constexpr (S == 2) {
        if constexpr (DGELU && KTU < 8)  // the DMA issued after this barrier overwrites the slot
          pr3 = p_lds(std::integral_constant<int, PAR>{}, std::integral_constant<int, 3>{});
        // the k-step-3 fragments (read above) are in registers before the buffer is released
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VMC) : "memory");
        PE_BARRIER();
        issue_dma(std::integral_constant<int, PAR>{});
      }
    });
  };
  // vmcnt at k-tile KTU's barrier: the VMEM ops issued after the DMA it waits for — the unit steps
  // of k-step 3 of the previous k-tile and k-steps 0-2 of this one (the previous tile's last k-tile
  // carries none; at KTU 0 the tile-end ops of the previous tile come first)
#define PE_KT(P, KTU, VMC) ktile(std::integral_constant<int, P>{}, std::integral_constant<int, KTU>{}, \
                                 std::integral_constant<int, VMC>{})

  // ---- prologue: k-tiles 0 and 1 of the first tile in flight, the first landed
  set_dma_tile(0);
  issue_dma(std::integral_constant<int, 0>{});
  issue_dma(std::integral_constant<int, 1>{});
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(16 + PPC) : "memory");  // k-tile 0 landed
  PE_BARRIER();
  load_frags(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});

  for (int ct = 0; ct < my_tiles; ++ct) {
    // (non-DGELU: a k-tile's 4·OPS stores all issue at its k-step 3)
    PE_KT(0, 0, DGELU ? 3 * OPS : 0); PE_KT(1, 1, 4 * OPS); PE_KT(0, 2, 4 * OPS); PE_KT(1, 3, 4 * OPS);
    PE_KT(0, 4, 4 * OPS); PE_KT(1, 5, 4 * OPS); PE_KT(0, 6, 4 * OPS); PE_KT(1, 7, 4 * OPS);
    PE_KT(0, 8, DGELU ? OPS : 4 * OPS); PE_KT(1, 9, 0);
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
    pcol2 = pn0 * 2;
    if constexpr (DGELU) {
      ppan = P + (size_t)pm0 * ldc;
      cprow = tm * 2 + wr;
      pn0c = pn0;
    }
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
          dout[DGELU ? jn * 8 + kp * 4 + im : im * 8 + (jn >> 1) * 4 + (jn & 1) * 2 + kp] =
              uint4{sx[0], sy[0], sx[1], sy[1]};
          // accumulator by accumulator: left free, the scheduler hoists the AGPR reads of many
          // accumulators ahead of their packing and spills deferred units
          __builtin_amdgcn_sched_barrier(0);
        }
    }
    zero_acc();
  }
#undef PE_KT
  // the last tile's units
  unroll<0, NUNIT>([&](auto u_c) {
    constexpr int U = decltype(u_c)::value;
    uint4 pr = uint4{0u, 0u, 0u, 0u};
    if constexpr (DGELU) {  // the stream has stopped: this tile's P chunks from global memory
      constexpr int IM = U & 3, CO = (U >> 3) * 32 + ((U >> 2) & 1) * 16;
      const unsigned off = vcol + CO < ncols ? vrow + (unsigned)(CO * 2) : 0x80000000u;
      pr = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsrc_of(ppan, crec), (int)off,
                                                                           (int)(IM * ld32_0) + pcol2, 0));
    }
    store_unit(u_c, pr);
  });
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tail's DMA of zeros, the last stores
}

}  // namespace
}  // namespace penroz

using namespace penroz;

// out[M][N] = a[M][K] · b[N][K]ᵀ (+ bias[N]); with act: out = pre-activation, act = GELU(out).
// bf16, unit column stride, K % 128 == 0, K >= 640, N % 8 == 0, row strides % 8 == 0, 16-B aligned.
// flags (timing ablation): 1 no stores (outputs wrong)
bool gemm_epi_supported(int64_t M, int64_t N, int64_t K) { return K % 128 == 0 && K >= 640 && N % 8 == 0 && M > 0; }

static void pe_check_operands(const torch::Tensor& a, const torch::Tensor& b, const torch::Tensor& out) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && out.is_cuda(), "gemm_epi: GPU tensors");
  TORCH_CHECK(a.scalar_type() == torch::kBFloat16 && b.scalar_type() == torch::kBFloat16 &&
                  out.scalar_type() == torch::kBFloat16, "gemm_epi: bf16 operands");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && out.dim() == 2, "gemm_epi: 2-D operands");
  TORCH_CHECK(a.stride(1) == 1 && b.stride(1) == 1 && out.stride(1) == 1, "gemm_epi: unit column stride");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(b.size(1) == K, "gemm_epi: inner dimensions differ");
  TORCH_CHECK(out.size(0) == M && out.size(1) == N, "gemm_epi: output shape");
  TORCH_CHECK(gemm_epi_supported(M, N, K), "gemm_epi: K % 128 == 0, K >= 640 and N % 8 == 0 required");
  TORCH_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0 && out.stride(0) % 8 == 0, "gemm_epi: row strides % 8");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(b.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0, "gemm_epi: 16-B alignment");
  TORCH_CHECK((int64_t)256 * std::max({a.stride(0), b.stride(0), out.stride(0)}) * 2 < (int64_t)1 << 31,
              "gemm_epi: row stride too large (256-row panels are addressed with 32-bit offsets)");
}

static int pe_grid(const torch::Tensor& out, int tiles) {
  static bool attr_set = false;
  if (!attr_set) {
    for (const void* f : {reinterpret_cast<const void*>(gemm_epi_kernel<EG_NONE>),
                          reinterpret_cast<const void*>(gemm_epi_kernel<EG_BIAS>),
                          reinterpret_cast<const void*>(gemm_epi_kernel<EG_GELU>),
                          reinterpret_cast<const void*>(gemm_epi_kernel<EG_GELU_TANH>)})
      (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    for (const void* f : {reinterpret_cast<const void*>(gemm_epi_kernel<EG_DGELU>),
                          reinterpret_cast<const void*>(gemm_epi_kernel<EG_DGELU_TANH>)})
      (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES_DG);
    attr_set = true;
  }
  static int n_cu = 0;
  if (n_cu == 0) {
    hipDeviceProp_t prop;
    n_cu = hipGetDeviceProperties(&prop, out.get_device()) == hipSuccess ? prop.multiProcessorCount : 256;
  }
  return std::min(tiles, n_cu);
}

#define PE_LAUNCH(EPIV, PP, CP)                                                                                 \
  hipLaunchKernelGGL((gemm_epi_kernel<EPIV>), dim3(grid), dim3(256), (EPIV == EG_DGELU || EPIV == EG_DGELU_TANH) ? LDS_BYTES_DG : LDS_BYTES, stream, ap, bp, biasp, cp, c2, PP, CP, \
                     M, N, K, lda, ldb, ldc, tiles_m, tiles_n, (int)flags)

void gemm_epi_bf16(torch::Tensor a, torch::Tensor b, c10::optional<torch::Tensor> bias, torch::Tensor out,
                   c10::optional<torch::Tensor> act, int64_t gelu_approx, int64_t flags) {
  pe_check_operands(a, b, out);
  const int M = a.size(0), K = a.size(1), N = b.size(0);
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
  const int tiles_m = (M + TILE - 1) / TILE, tiles_n = (N + TILE - 1) / TILE;
  const int grid = pe_grid(out, tiles_m * tiles_n);
  auto stream = at::hip::getCurrentHIPStream();
  const bf16* ap = reinterpret_cast<const bf16*>(a.data_ptr());
  const bf16* bp = reinterpret_cast<const bf16*>(b.data_ptr());
  const bf16* biasp = has_bias ? reinterpret_cast<const bf16*>(bias->data_ptr()) : nullptr;
  bf16* cp = reinterpret_cast<bf16*>(out.data_ptr());
  bf16* c2 = gelu ? reinterpret_cast<bf16*>(act->data_ptr()) : nullptr;
  const int lda = a.stride(0), ldb = b.stride(0), ldc = out.stride(0);
  if (gelu && gelu_approx) PE_LAUNCH(EG_GELU_TANH, nullptr, nullptr);
  else if (gelu) PE_LAUNCH(EG_GELU, nullptr, nullptr);
  else if (has_bias) PE_LAUNCH(EG_BIAS, nullptr, nullptr);
  else PE_LAUNCH(EG_NONE, nullptr, nullptr);
}

// Data gradient through a GELU: out = bf16(dy · wtᵀ) · GELU'(pre) (the unfused pair's rounding
// points), and dbias (fp32 [N], accumulated: +=) += the column sums of out — the fc bias gradient,
// from per-128-row partial rows reduced deterministically (on the deferred-reduction stream when
// one is set, like every bias / norm-weight reduction of the executors). pre is shaped and strided
// like out. `out` may not alias `pre`.
void gemm_epi_dgelu(torch::Tensor dy, torch::Tensor wt, torch::Tensor pre, torch::Tensor out,
                    c10::optional<torch::Tensor> dbias, int64_t gelu_approx, int64_t flags) {
  pe_check_operands(dy, wt, out);
  TORCH_CHECK(pre.scalar_type() == torch::kBFloat16 && pre.sizes() == out.sizes() && pre.strides() == out.strides() &&
                  reinterpret_cast<uintptr_t>(pre.data_ptr()) % 16 == 0 && pre.data_ptr() != out.data_ptr(),
              "gemm_epi_dgelu: pre shaped and strided like out, not aliasing it");
  const int M = dy.size(0), K = dy.size(1), N = wt.size(0);
  const bool has_db = dbias.has_value() && dbias->defined();
  if (has_db)
    TORCH_CHECK(dbias->scalar_type() == torch::kFloat32 && dbias->numel() == N && dbias->is_contiguous(),
                "gemm_epi_dgelu: dbias fp32 [N]");
  if (M == 0 || N == 0) return;
  const int tiles_m = (M + TILE - 1) / TILE, tiles_n = (N + TILE - 1) / TILE;
  const int grid = pe_grid(out, tiles_m * tiles_n);
  auto stream = at::hip::getCurrentHIPStream();
  auto part = torch::empty({(int64_t)tiles_m * 2, N}, out.options().dtype(torch::kFloat32));
  const bf16* ap = reinterpret_cast<const bf16*>(dy.data_ptr());
  const bf16* bp = reinterpret_cast<const bf16*>(wt.data_ptr());
  const bf16* biasp = nullptr;
  bf16* cp = reinterpret_cast<bf16*>(out.data_ptr());
  bf16* c2 = nullptr;
  const bf16* pp = reinterpret_cast<const bf16*>(pre.data_ptr());
  float* cpart = part.data_ptr<float>();
  const int lda = dy.stride(0), ldb = wt.stride(0), ldc = out.stride(0);
  if (gelu_approx) PE_LAUNCH(EG_DGELU_TANH, pp, cpart);
  else PE_LAUNCH(EG_DGELU, pp, cpart);
  if (has_db) {
    float* outs[1] = {dbias->data_ptr<float>()};
    reduce_partials_auto(part, 1, tiles_m * 2, N, outs, stream);
  }
}
#undef PE_LAUNCH
