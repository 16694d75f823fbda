// Shared device helpers of the flash-attention kernels (flash_attn.hip: head_dim 64, tuned;
// flash_attn_gen.hip: head_dim 128 / 256). v_mfma_f32_32x32x16_bf16 operand / accumulator
// maps, the XOR-swizzled LDS tile image, softmax lane exchanges, dropout hash, XCD mapping.
#pragma once
#include "common.h"

namespace penroz {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

__device__ __forceinline__ f32x16 mfma32(uint4 a, uint4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                 0, 0, 0);
}

__device__ __forceinline__ int tile_off(int row, int ch) {
  return row * 128 + ((ch ^ ((((row >> 1) & 1) << 2) | ((row >> 2) & 3))) << 4);
}

// element j = tile[rbase + (lane&31)][16s + 8·hh + j]
__device__ __forceinline__ uint4 row_frag(const char* tile, int rbase, int s, int lane) {
  return *reinterpret_cast<const uint4*>(tile + tile_off(rbase + (lane & 31), 2 * s + (lane >> 5)));
}

__device__ __forceinline__ uint2 tr_read(const char* tile, int row, int col) {
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4*)(tile + tile_off(row, col >> 3) + ((col & 4) << 1)));
  return __builtin_bit_cast(uint2, v);
}

// element j = tile[rbase + 8(j>>2) + 4·hh + (j&3)][cbase + (lane&31)]  (transposed read)
__device__ __forceinline__ uint4 tr_frag(const char* tile, int rbase, int cbase, int lane) {
  const int hh = lane >> 5, q = (lane & 15) >> 2, p = lane & 3;
  const int col = cbase + 16 * ((lane >> 4) & 1) + 4 * p;
  const uint2 a = tr_read(tile, rbase + 4 * hh + q, col);
  const uint2 b = tr_read(tile, rbase + 8 + 4 * hh + q, col);
  return uint4{a.x, a.y, b.x, b.y};
}

// accumulator registers 8ss..8ss+7 -> bf16x8 operand
__device__ __forceinline__ uint4 acc_frag(const f32x16& a, int ss) {
  const int o = 8 * ss;
  return uint4{pack_bf16x2(a[o], a[o + 1]), pack_bf16x2(a[o + 2], a[o + 3]), pack_bf16x2(a[o + 4], a[o + 5]),
               pack_bf16x2(a[o + 6], a[o + 7])};
}

__device__ __forceinline__ int acc_row(int i, int lane) { return (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5); }

// Attention-dropout mask, regenerated identically by every forward / backward kernel.
// Element (q, k) of head row-block bh (= b·H + h) is kept iff the 16-bit half (k & 1) of
// H = fmix32(rowkey(seed, bh·T + q) ^ (k >> 1)·0x85EBCA6B) is ≥ p·65536 (p quantised to 2⁻¹⁶).
// 32-bit arithmetic only (two v_mul_lo_u32 per hash) and one hash per key PAIR: the
// kernels that hold consecutive keys of one query row in consecutive registers (forward, dQ)
// get both halves from one hash; the dK/dV kernel (key on the lane) pays one per element.
__device__ __forceinline__ uint32_t fmix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x;
}

// The same hash in pieces, for kernels that walk consecutive rows / key pairs: row·kDropRowMul and
// (k>>1)·kDropKeyMul distribute over addition (mod 2³²), so a caller keeps one product per tile
// and adds compile-time multiples of the constant instead of multiplying per element (v_mul_lo_u32
// is a quarter-rate instruction; it dominated the dropout kernels' VALU time).
constexpr uint32_t kDropRowMul = 0x9E3779B1u, kDropKeyMul = 0x85EBCA6Bu;
__device__ __forceinline__ uint32_t dropout_seedmix(uint64_t seed) {
  return (uint32_t)seed ^ ((uint32_t)(seed >> 32) * 0x27D4EB2Fu);
}
__device__ __forceinline__ uint32_t dropout_thr(float p) { return (uint32_t)(p * 65536.f); }
// hashed input = seedmix ^ row·kDropRowMul ^ (k>>1)·kDropKeyMul (row = (b·H + h)·T + q), given as two
// XOR terms so a kernel pre-combines the seed mix with whichever term is constant per lane
// (x ^ y: one operand per lane, the other per element); odd = k & 1 picks the 16-bit half
__device__ __forceinline__ bool dropout_keep_mixed(uint32_t x, uint32_t y, bool odd, uint32_t thr) {
  const uint32_t hsh = fmix32(x ^ y);
  const uint32_t u16 = odd ? (hsh >> 16) : (hsh & 0xFFFFu);
  return u16 >= thr;
}

__device__ __forceinline__ bool dropout_keep(uint64_t seed, int b, int h, int H, int T, int q, int k, float p) {
  return dropout_keep_mixed(dropout_seedmix(seed) ^ ((uint32_t)((b * H + h) * T + q) * kDropRowMul),
                            (uint32_t)(k >> 1) * kDropKeyMul, (k & 1) != 0, dropout_thr(p));
}

__device__ __forceinline__ uint4 zero4() { return uint4{0u, 0u, 0u, 0u}; }

// 8 bf16 values × c, rounded back to bf16: the backward kernels prescale the operand of
// S = Q·Kᵀ that they keep in registers by c = scale·log2(e) once, and start the S accumulator
// at the row's −LSE·log2(e), so P = exp2(S) costs one instruction per score instead of an FMA
// and an exponential (the same one extra bf16 rounding of that operand a Triton flash kernel
// applies to q; the forward's statistics stay exact)
__device__ __forceinline__ uint4 scale_bf16x8(uint4 u, float c) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
  uint32_t o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    o[i] = pack_bf16x2(__uint_as_float(w[i] << 16) * c, __uint_as_float(w[i] & 0xffff0000u) * c);
  return uint4{o[0], o[1], o[2], o[3]};
}

// raw v_exp_f32 (no denormal range fix-up: softmax weights that small are 0 anyway)
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// wave index, provably wave-uniform for the compiler (keeps causal-mask branches scalar)
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// Combine a value across the two 32-lane halves (lane l and l^32) with one
// v_permlane32_swap instead of a ds_bpermute round trip. The swap of (v, v) returns
// {[lo|lo], [hi|hi]}, so op(r0, r1) is the full-row result in every lane.
__device__ __forceinline__ float halves_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float halves_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// defer-rescale threshold (log2 units): the running max is only raised when some row's max
// grows by more than 2^8, so most tiles skip the O rescale (P then stays <= 256: bf16-safe)
constexpr float kRescaleThr = 8.0f;

// stores 4 consecutive bf16 (8 bytes)
__device__ __forceinline__ void store4(bf16* p, float a, float b, float c, float d) {
  *reinterpret_cast<uint2*>(p) = uint2{pack_bf16x2(a, b), pack_bf16x2(c, d)};
}

// XCD-aware block mapping. Workgroups are dealt to the 8 XCDs round-robin in dispatch order
// (x fastest), so the plain grid would scatter one head's blocks over all eight L2s. Remap so
// the gridDim.x blocks of a head share an XCD with heads dealt to XCDs round-robin, and within
// an XCD dispatch block-major: block 0 (the heaviest) of every head, then block 1, ... — a
// head-major order ended every launch on the last heads' whole block sequences (GPT-2 B=64:
// forward -3.5 %, backward -5.5 %, headline -0.6 ms vs head-major, profiles/attn_ab_pmc_r4.log).
// A head's K/V (256 KB at D = 64) then stay in the 256 MB infinity cache rather than in one L2.
// Bijective; a tail of heads that is not a multiple of 8 keeps the plain order.
__device__ __forceinline__ void xcd_head_block(int& blk, int& head) {
  const int nblk = gridDim.x, nheads = gridDim.y;
  const int id = blockIdx.x + nblk * blockIdx.y;
  const int hp = nheads >> 3, full = hp * nblk;  // slots per XCD in the full head groups
  const int xcd = id & 7, slot = id >> 3;
  if (slot < full) {  // block-major within the XCD: every head's heaviest block first
    blk = slot / hp;
    head = (slot - blk * hp) * 8 + xcd;
  } else {
    const int r = id - 8 * full;
    head = (nheads & ~7) + r / nblk;
    blk = r - (r / nblk) * nblk;
  }
}

// Bias-gradient partial of one wave's 32 rows (on lanes lane&31) of a 64-column head slice held in
// MFMA accumulators: acc[dh][i] is column 32·dh + 8·(i>>2) + 4·(lane>>5) + (i&3). Each value is
// scaled by `mul` and rounded to bf16 exactly as the kernel stores it (so the sums equal the
// column sums of the stored gradient); invalid rows count 0. A transpose-reduce over the five
// lane bits (xor 16 … 1, each step halving the registers in play: 31 shuffles, no LDS, no
// barrier) leaves lane L holding the sum of register 16·dh + i = L&31, stored to part[column].
// one transpose-reduce step over lane bit N (registers v[0 .. 2N) in play -> v[0 .. N)); the
// register count is a template constant so every index stays static (no dynamic register indexing)
template <int N>
__device__ __forceinline__ void transpose_reduce_step(float (&v)[32], int lane) {
  const bool up = (lane & N) != 0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const float send = up ? v[i] : v[i + N];
    const float keep = up ? v[i + N] : v[i];
    v[i] = keep + __shfl_xor(send, N, 64);
  }
  if constexpr (N > 1) transpose_reduce_step<N / 2>(v, lane);
}

__device__ __forceinline__ void colsum32_wave(const f32x16 (&acc)[2], float mul, bool valid, float* __restrict__ part) {
  const int lane = threadIdx.x & 63;
  float v[32];
#pragma unroll
  for (int dh = 0; dh < 2; ++dh)
#pragma unroll
    for (int i = 0; i < 16; ++i) v[16 * dh + i] = valid ? __bfloat162float(__float2bfloat16(acc[dh][i] * mul)) : 0.f;
  transpose_reduce_step<16>(v, lane);
  const int r = lane & 31, dh = r >> 4, i = r & 15;
  part[32 * dh + 8 * (i >> 2) + 4 * (lane >> 5) + (i & 3)] = v[0];
}


}  // namespace penroz
