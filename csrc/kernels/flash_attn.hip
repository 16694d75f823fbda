// Causal flash attention for CDNA4 (gfx950), head_dim 64, bf16 in/out, fp32 accumulate.
//
// Operates directly on the fused QKV projection [B, T, (H + 2·Hkv)·D] (no split / transpose
// copies) and writes O head-merged [B, T, H·D] — the layout the following projection GEMM
// reads. GQA: kv head = q head / (H/Hkv), never expanded.
//
// MFMA: v_mfma_f32_32x32x16_bf16 throughout. C/D layout: col = lane&31,
// row = (i&3) + 8(i>>2) + 4(lane>>5) for accumulator register i.
//
// forward (one 256-thread workgroup = 4 waves × 32 query rows = 128 rows of one (b, h)):
//   Sᵀ = K·Qᵀ — K (A operand) from an XOR-swizzled LDS tile, Q (B operand) resident in 16
//   VGPRs — so each lane owns ONE query row: the row max needs one cross-half exchange, the
//   row sum stays lane-local until the epilogue;
//   Oᵀ += Vᵀ·Pᵀ — P goes from the accumulator straight into the B operand (pairs of
//   registers → bf16), Vᵀ (A operand) comes from the row-major V tile through
//   ds_read_b64_tr_b16 (hardware transposed read), and the per-row rescale of Oᵀ is
//   lane-local too;
//   K/V tiles of 64 keys are double-buffered in LDS and staged through registers (the global
//   loads of tile j+1 are issued before tile j's MFMAs, written to LDS after them);
//   heaviest (latest) query blocks launch first; fully-masked tiles are skipped per wave.
// backward (deterministic, no atomics; the S = Q·Kᵀ operand each kernel keeps in registers is
// prescaled by scale·log2(e) and S starts from the row's −LSE·log2(e), so P = exp2(S) — one VALU
// instruction per score fewer than exp2(fma(S, c, −LSE·log2 e)); attn_common.h scale_bf16x8):
//   dK/dV kernel — a wave keeps 32 keys' K, V fragments and dKᵀ, dVᵀ accumulators in
//   registers while sweeping 32-row query slices staged in LDS (all query heads of its KV
//   group): S = Q·Kᵀ and dP = dO·Vᵀ put the key on the lane, so P and dS feed dVᵀ = dOᵀ·P and
//   dKᵀ = Qᵀ·dS from registers (Qᵀ, dOᵀ by transposed LDS reads);
//   dQ kernel — forward-shaped: a wave keeps 32 query rows' Q, dO, LSE, δ and dQᵀ in
//   registers while sweeping K/V tiles; dQᵀ = Kᵀ·dSᵀ.
//
// LDS tiles are [rows][64 bf16] = 128-B rows; 16-B chunk ch of row r lives at chunk
// ch ^ f(r), f(r) = ((r>>1)&1)<<2 | ((r>>2)&3). This single swizzle makes both the
// ds_read_b128 row reads (16 lanes on 16 distinct rows, same chunk) and the
// ds_read_b64_tr_b16 transposed reads (4 consecutive rows × 4 chunks per half-wave)
// bank-conflict-free.
//
// Dropout (attn_pdrop) uses a counter-based hash of (b, h, q, k): the backward regenerates
// the identical mask; the softmax normaliser uses the undropped probabilities (SDPA
// semantics).
#include "attn_common.h"
#include <cstdlib>
#include "deferred.h"
#include <type_traits>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

namespace penroz {

constexpr int kD = 64;

// ------------------------------------------------------------------------------------------
// forward
template <bool DROPOUT>
__global__ void __launch_bounds__(256, 2) fa_fwd_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ out,
                                                     float* __restrict__ lse, int T, int H, int Hkv, float scale,
                                                     float p_drop, uint64_t seed) {
  constexpr int BM = 128, BN = 64;
  __shared__ __attribute__((aligned(16))) char smem[2][2][BN * 128];
  const int nqb = (T + BM - 1) / BM;
  int qi, bh;
  xcd_head_block(qi, bh);
  const int qb = nqb - 1 - qi;
  const int b = bh / H, h = bh % H, hk = h / (H / Hkv);
  const int lane = threadIdx.x & 63, w = wave_id(), hh = lane >> 5;
  const size_t RS = (size_t)(H + 2 * Hkv) * kD;
  const bf16* qbase = qkv + (size_t)b * T * RS + (size_t)h * kD;
  const bf16* kbase = qkv + (size_t)b * T * RS + (size_t)(H + hk) * kD;
  const bf16* vbase = qkv + (size_t)b * T * RS + (size_t)(H + Hkv + hk) * kD;
  const int q0 = qb * BM + 32 * w;
  const int qrow = q0 + (lane & 31);
  // dropout hash pieces (attn_common.h): per-lane seed mix ^ row product, 16-bit threshold
  const uint32_t drow = DROPOUT ? dropout_seedmix(seed) ^ ((uint32_t)((b * H + h) * T + qrow) * kDropRowMul) : 0u;
  const uint32_t dthr = dropout_thr(p_drop);
  const float c = scale * kLog2e;
  const float inv_keep = DROPOUT ? 1.f / (1.f - p_drop) : 1.f;

  uint4 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s)
    qf[s] = qrow < T ? *reinterpret_cast<const uint4*>(qbase + (size_t)qrow * RS + 16 * s + 8 * hh) : zero4();

  // staging: thread t -> chunk t&7 of rows (t>>3) + 32i (8 lanes cover one 128-B row:
  // coalesced, conflict-free ds_write_b128 groups)
  const int sr = threadIdx.x >> 3, sc = threadIdx.x & 7;
  uint4 kst[2], vst[2];
  auto gload = [&](int kt0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int key = kt0 + sr + 32 * i;
      kst[i] = key < T ? *reinterpret_cast<const uint4*>(kbase + (size_t)key * RS + 8 * sc) : zero4();
      vst[i] = key < T ? *reinterpret_cast<const uint4*>(vbase + (size_t)key * RS + 8 * sc) : zero4();
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      *reinterpret_cast<uint4*>(smem[buf][0] + tile_off(sr + 32 * i, sc)) = kst[i];
      *reinterpret_cast<uint4*>(smem[buf][1] + tile_off(sr + 32 * i, sc)) = vst[i];
    }
  };

  const int kend = min(T, qb * BM + BM);
  const int ntiles = (kend + BN - 1) / BN;
  f32x16 o[2];
#pragma unroll
  for (int dh = 0; dh < 2; ++dh)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[dh][i] = 0.f;
  float m = -1e30f, l = 0.f;

  gload(0);
  lstore(0);
  __syncthreads();
  for (int j = 0; j < ntiles; ++j) {
    const int kt0 = j * BN;
    const uint32_t kpair0 = DROPOUT ? (uint32_t)((kt0 + 4 * hh) >> 1) * kDropKeyMul : 0u;
    if (j + 1 < ntiles) gload(kt0 + BN);
    const char* Kt = smem[j & 1][0];
    const char* Vt = smem[j & 1][1];
    if (kt0 <= q0 + 31) {
      f32x16 s[2];
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
#pragma unroll
        for (int i = 0; i < 16; ++i) s[kh][i] = 0.f;
#pragma unroll
        for (int st = 0; st < 4; ++st) s[kh] = mfma32(row_frag(Kt, 32 * kh, st, lane), qf[st], s[kh]);
      }
      // softmax on raw scores: max first (scaling commutes with max, c > 0), then
      // p = 2^(s·c − m) as one fma + exp. The mask variant is a separate code path so the
      // common (off-diagonal) tile has no per-element select or branch.
      auto softmax = [&](auto mask_tag) {
        constexpr bool MASK = decltype(mask_tag)::value;
        float tmax = -INFINITY;
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            if constexpr (MASK) {
              const int key = kt0 + 32 * kh + acc_row(i, lane);
              s[kh][i] = (key > qrow || key >= T) ? -INFINITY : s[kh][i];
            }
            tmax = fmaxf(tmax, s[kh][i]);
          }
        tmax = halves_max(tmax) * c;
        if (!__all(tmax <= m + kRescaleThr)) {  // wave-uniform: rare after the first tiles
          const float mnew = fmaxf(m, tmax);
          const float alpha = fexp2(m - mnew);
          m = mnew;
          l *= alpha;
#pragma unroll
          for (int dh = 0; dh < 2; ++dh)
#pragma unroll
            for (int i = 0; i < 16; ++i) o[dh][i] *= alpha;
        }
        const float negm = -m;
        float2_t lsum = {0.f, 0.f};
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
          for (int i = 0; i < 16; i += 2) {
            float2_t p = {fexp2(fmaf(s[kh][i], c, negm)), fexp2(fmaf(s[kh][i + 1], c, negm))};
            lsum += p;
            if constexpr (DROPOUT) {  // keys (and key + 1) kt0 + 32kh + 4hh + (i&3) + 8(i>>2): one hash
              const uint32_t km = kpair0 + (uint32_t)(16 * kh + 4 * (i >> 2) + ((i & 3) >> 1)) * kDropKeyMul;
              p[0] = dropout_keep_mixed(drow, km, false, dthr) ? p[0] * inv_keep : 0.f;
              p[1] = dropout_keep_mixed(drow, km, true, dthr) ? p[1] * inv_keep : 0.f;
            }
            s[kh][i] = p[0];
            s[kh][i + 1] = p[1];
          }
        l += lsum[0] + lsum[1];
      };
      const bool need_mask = (kt0 + BN - 1 > q0) || (kt0 + BN > T);
      if (need_mask)
        softmax(std::true_type{});
      else
        softmax(std::false_type{});
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          const uint4 pf = acc_frag(s[kh], ss);
#pragma unroll
          for (int dh = 0; dh < 2; ++dh) o[dh] = mfma32(tr_frag(Vt, 32 * kh + 16 * ss, 32 * dh, lane), pf, o[dh]);
        }
    }
    if (j + 1 < ntiles) lstore((j + 1) & 1);
    __syncthreads();
  }
  l = halves_sum(l);
  const float inv = l > 0.f ? 1.f / l : 0.f;
  if (qrow < T) {
    bf16* orow = out + ((size_t)b * T + qrow) * H * kD + (size_t)h * kD;
#pragma unroll
    for (int dh = 0; dh < 2; ++dh)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        store4(orow + 32 * dh + 8 * g + 4 * hh, o[dh][4 * g] * inv, o[dh][4 * g + 1] * inv, o[dh][4 * g + 2] * inv,
               o[dh][4 * g + 3] * inv);
    if (hh == 0) lse[((size_t)b * H + h) * T + qrow] = (m + log2f(l)) * kLn2;
  }
}

// ------------------------------------------------------------------------------------------
// forward, two query blocks per wave (default): a 128-thread workgroup = 2 waves × 64 query
// rows; each wave holds two independent 32-row blocks A and B. Per 64-key tile the K
// fragments (row reads) and V fragments (transposed reads) are read from LDS ONCE per wave
// and used by both blocks, halving LDS traffic per MFMA, and the two blocks' dependency
// chains interleave: S_B's MFMAs run under softmax_A, P_A·V's under softmax_B. Query blocks
// of 64 rows are aligned to key tiles, so a wave's only masked tile is its diagonal one.
template <bool DROPOUT>  // instantiated without dropout only (see flash_attn_fwd)
__global__ void __launch_bounds__(128, 2) fa_fwd3_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ out,
                                                      float* __restrict__ lse, int T, int H, int Hkv, float scale,
                                                      float p_drop, uint64_t seed) {
  constexpr int BM = 128, BN = 64;
  __shared__ __attribute__((aligned(16))) char smem[2][2][BN * 128];
  const int nqb = (T + BM - 1) / BM;
  int qi, bh;
  xcd_head_block(qi, bh);
  const int qb = nqb - 1 - qi;
  const int b = bh / H, h = bh % H, hk = h / (H / Hkv);
  const int lane = threadIdx.x & 63, w = wave_id(), hh = lane >> 5;
  const size_t RS = (size_t)(H + 2 * Hkv) * kD;
  const bf16* qbase = qkv + (size_t)b * T * RS + (size_t)h * kD;
  const bf16* kbase = qkv + (size_t)b * T * RS + (size_t)(H + hk) * kD;
  const bf16* vbase = qkv + (size_t)b * T * RS + (size_t)(H + Hkv + hk) * kD;
  const int q0 = qb * BM + 64 * w;  // block A rows q0..q0+31, block B rows q0+32..q0+63
  const float c = scale * kLog2e;
  const float inv_keep = DROPOUT ? 1.f / (1.f - p_drop) : 1.f;
  int qrow[2];
  qrow[0] = q0 + (lane & 31);
  qrow[1] = q0 + 32 + (lane & 31);

  uint4 qf[2][4];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int s = 0; s < 4; ++s)
      qf[a][s] = qrow[a] < T ? *reinterpret_cast<const uint4*>(qbase + (size_t)qrow[a] * RS + 16 * s + 8 * hh) : zero4();
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int s = 0; s < 4; ++s) launder(qf[a][s]);  // no compiler-tracked load left for the loop

  // LDS-DMA staging (no staging registers). K image is chunk-major [8 chunks][64 keys][16 B]:
  // row-fragment reads (16 lanes on 16 consecutive keys, one chunk) are conflict-free and all
  // fragment addresses differ by immediates; one DMA piece = one chunk column, so wave 0's
  // eight pieces share ONE per-lane source pointer. V keeps the swizzled row-major image
  // (tile_off) for the transposed reads; wave 1 fills it, piece p = keys 8p..8p+7. Keys past
  // T are clamped to T-1: finite data that the mask (K) or P = 0 (V) cancels.
  // fast path (whole tile inside T): SGPR base per piece, per-lane byte offsets fixed
  const unsigned RSB = (unsigned)RS * 2;  // row stride in bytes
  const unsigned k_voff = (unsigned)lane * RSB;
  unsigned v_voff[2];
#pragma unroll
  for (int par = 0; par < 2; ++par) {
    const int row = 8 * par + (lane >> 3);  // rows 8p + (lane>>3): the swizzle depends on p&1 only
    const int ch = (lane & 7) ^ ((((row >> 1) & 1) << 2) | ((row >> 2) & 3));
    v_voff[par] = (unsigned)(lane >> 3) * RSB + 16u * ch;
  }
  // per-lane byte offsets of the two transposed reads of a V fragment (tile_off is periodic in
  // 16 rows, so the key offset 32kh + 16ss becomes an immediate)
  unsigned vto[2][2];
#pragma unroll
  for (int dh = 0; dh < 2; ++dh)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int col = 32 * dh + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
      vto[dh][jj] = (unsigned)(tile_off(4 * hh + ((lane & 15) >> 2) + 8 * jj, col >> 3) + ((col & 4) << 1));
    }
  auto vfrag = [&](const char* t, int dh) -> uint4 {
    const s16x4 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(t + vto[dh][0]));
    const s16x4 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(t + vto[dh][1]));
    const uint2 ux = __builtin_bit_cast(uint2, x), uy = __builtin_bit_cast(uint2, y);
    return uint4{ux.x, ux.y, uy.x, uy.y};
  };
  auto dma = [&](int kt0, int buf) {
    const unsigned dst = __builtin_amdgcn_readfirstlane(lds_addr_of(smem[buf][w]));
    if (kt0 + BN <= T) {
      if (w == 0) {
        const char* sb = reinterpret_cast<const char*>(kbase + (size_t)kt0 * RS);
        // (the chunk offset goes on the SGPR base: an instruction offset would shift the LDS
        // destination too)
#pragma unroll
        for (int p = 0; p < 8; ++p) glds16_s(sb + 16 * p, k_voff, dst + p * 1024);
      } else {
#pragma unroll
        for (int p = 0; p < 8; ++p)
          glds16_s(reinterpret_cast<const char*>(vbase + (size_t)(kt0 + 8 * p) * RS), v_voff[p & 1],
                      dst + p * 1024);
      }
    } else if (w == 0) {  // ragged last tile: clamp keys to T-1 per lane
      const bf16* g = kbase + (size_t)min(kt0 + lane, T - 1) * RS;
#pragma unroll
      for (int p = 0; p < 8; ++p) glds16(g + 8 * p, dst + p * 1024);
    } else {
      const int prow = lane >> 3, pch = lane & 7;
#pragma unroll
      for (int p = 0; p < 8; ++p) {
        const int row = 8 * p + prow;
        const int ch = pch ^ ((((row >> 1) & 1) << 2) | ((row >> 2) & 3));
        glds16(vbase + (size_t)min(kt0 + row, T - 1) * RS + 8 * ch, dst + p * 1024);
      }
    }
  };

  const int kend = min(T, qb * BM + BM);
  const int ntiles = (kend + BN - 1) / BN;
  const int jlast = min(ntiles - 1, q0 / BN);  // the wave's diagonal tile
  f32x16 o[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int dh = 0; dh < 2; ++dh)
#pragma unroll
      for (int i = 0; i < 16; ++i) o[a][dh][i] = 0.f;
  float m[2] = {-1e30f, -1e30f}, l[2] = {0.f, 0.f};

  auto softmax = [&](auto mask_tag, int a, int kt0, f32x16 (&sa)[2]) {
    constexpr bool MASK = decltype(mask_tag)::value;
    float tmax = -INFINITY;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if constexpr (MASK) {
          const int key = kt0 + 32 * kh + acc_row(i, lane);
          sa[kh][i] = (key > qrow[a] || key >= T) ? -INFINITY : sa[kh][i];
        }
        tmax = fmaxf(tmax, sa[kh][i]);
      }
    tmax = halves_max(tmax) * c;
    if (!__all(tmax <= m[a] + kRescaleThr)) {
      const float mnew = fmaxf(m[a], tmax);
      const float alpha = fexp2(m[a] - mnew);
      m[a] = mnew;
      l[a] *= alpha;
#pragma unroll
      for (int dh = 0; dh < 2; ++dh)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[a][dh][i] *= alpha;
    }
    const float negm = -m[a];
    const float2_t c2 = {c, c}, negm2 = {negm, negm};
    float2_t lsum = {0.f, 0.f};
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        // s·c − m for a register pair in one v_pk_fma_f32 (half the VALU issues of two fmas)
        const float2_t e = __builtin_elementwise_fma((float2_t){sa[kh][i], sa[kh][i + 1]}, c2, negm2);
        float2_t p = {fexp2(e[0]), fexp2(e[1])};
        lsum += p;
        if constexpr (DROPOUT) {
          const int key = kt0 + 32 * kh + acc_row(i, lane);
          p[0] = dropout_keep(seed, b, h, H, T, qrow[a], key, p_drop) ? p[0] * inv_keep : 0.f;
          p[1] = dropout_keep(seed, b, h, H, T, qrow[a], key + 1, p_drop) ? p[1] * inv_keep : 0.f;
        }
        sa[kh][i] = p[0];
        sa[kh][i + 1] = p[1];
      }
    l[a] += lsum[0] + lsum[1];
  };

  // one tile for both blocks; MASK only on the diagonal tile
  auto tile = [&](auto mask_tag, int j) {
    const int kt0 = j * BN;
    const char* Kt = smem[j & 1][0];
    const char* Vt = smem[j & 1][1];
    f32x16 sA[2], sB[2];
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {  // K fragments of one 32-key half at a time (16 VGPRs)
      uint4 kfr[4];
#pragma unroll
      for (int st = 0; st < 4; ++st)  // element j = K[32kh + (lane&31)][16st + 8hh + j]
        kfr[st] = *reinterpret_cast<const uint4*>(Kt + (2 * st + hh) * 1024 + (32 * kh + (lane & 31)) * 16);
#pragma unroll
      for (int i = 0; i < 16; ++i) sA[kh][i] = sB[kh][i] = 0.f;
#pragma unroll
      for (int st = 0; st < 4; ++st) sA[kh] = mfma32(kfr[st], qf[0][st], sA[kh]);
#pragma unroll
      for (int st = 0; st < 4; ++st) sB[kh] = mfma32(kfr[st], qf[1][st], sB[kh]);
    }
    uint4 vfr[2][2][2];
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss)
#pragma unroll
        for (int dh = 0; dh < 2; ++dh) vfr[kh][ss][dh] = vfrag(Vt + (32 * kh + 16 * ss) * 128, dh);
    softmax(mask_tag, 0, kt0, sA);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const uint4 pf = acc_frag(sA[kh], ss);
#pragma unroll
        for (int dh = 0; dh < 2; ++dh) o[0][dh] = mfma32(vfr[kh][ss][dh], pf, o[0][dh]);
      }
    softmax(mask_tag, 1, kt0, sB);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const uint4 pf = acc_frag(sB[kh], ss);
#pragma unroll
        for (int dh = 0; dh < 2; ++dh) o[1][dh] = mfma32(vfr[kh][ss][dh], pf, o[1][dh]);
      }
  };

  dma(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // unmasked tiles, then the peeled diagonal tile (kept out of the loop so its mask
  // predicates are not hoisted as loop invariants), then barrier-only steps while the other
  // wave finishes; every wave passes the same ntiles barriers and issues its DMA share
  int j = 0;
  for (; j < jlast; ++j) {
    dma((j + 1) * BN, (j + 1) & 1);  // j < jlast <= ntiles-1: buffer freed by the last barrier
    tile(std::false_type{}, j);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (j + 1 < ntiles) dma((j + 1) * BN, (j + 1) & 1);
  tile(std::true_type{}, j);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (++j; j < ntiles; ++j) {
    if (j + 1 < ntiles) dma((j + 1) * BN, (j + 1) & 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const float ls = halves_sum(l[a]);
    const float inv = ls > 0.f ? 1.f / ls : 0.f;
    if (qrow[a] < T) {
      bf16* orow = out + ((size_t)b * T + qrow[a]) * H * kD + (size_t)h * kD;
#pragma unroll
      for (int dh = 0; dh < 2; ++dh)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          store4(orow + 32 * dh + 8 * g + 4 * hh, o[a][dh][4 * g] * inv, o[a][dh][4 * g + 1] * inv,
                 o[a][dh][4 * g + 2] * inv, o[a][dh][4 * g + 3] * inv);
      if (hh == 0) lse[((size_t)b * H + h) * T + qrow[a]] = (m[a] + log2f(ls)) * kLn2;
    }
  }
}

// ------------------------------------------------------------------------------------------
// backward preprocessing: delta[b, h, q] = Σ_d dO·O  (8 lanes per row, 16-B loads)
__global__ void __launch_bounds__(256) fa_bwd_pre_kernel(const bf16* __restrict__ dout, const bf16* __restrict__ out,
                                                         float* __restrict__ delta, int B, int T, int H) {
  const int gid = blockIdx.x * 256 + threadIdx.x;
  const int row = gid >> 3, part = gid & 7;  // row over B*T*H in [b][t][h] order
  const bool ok = row < B * T * H;
  float s = 0.f;
  if (ok) {
    float a[8], o[8];
    Vec8<bf16>::load(dout + (size_t)row * kD + 8 * part, a);
    Vec8<bf16>::load(out + (size_t)row * kD + 8 * part, o);
#pragma unroll
    for (int k = 0; k < 8; ++k) s += a[k] * o[k];
  }
  s += __shfl_xor(s, 1, 64);
  s += __shfl_xor(s, 2, 64);
  s += __shfl_xor(s, 4, 64);
  if (ok && part == 0) {
    const int h = row % H, t = (row / H) % T, b = row / (H * T);
    delta[((size_t)b * H + h) * T + t] = s;
  }
}

// ------------------------------------------------------------------------------------------
// dK / dV: grid (ceil(T/128) key blocks, B*Hkv); wave w owns keys kb*128 + 32w + (lane&31); P / dS
// are computed in place in the S / dP accumulators. The Q / dO slices (64 rows) and their LSE / δ
// rows arrive by LDS-DMA into an NST-stage ring, NST - 1 slices ahead, so global latency hides
// behind iterations of MFMA work; K / V fragments are laundered so no compiler-tracked load is
// outstanding inside the loop. Per iteration waves 0-1 fetch the Q slice (4 pieces each), waves
// 2-3 the dO slice, waves 0 / 1 also the LSE / δ rows (one 4-byte DMA each). Every LDS fragment
// address is precomputed per lane (4 row-read + 4 transposed-read offsets; the 32-row half, the
// 16-row sub-block and — the loop unrolled by the ring stages — the stage base become
// immediates), removing ~140 swizzle-address VALU instructions per iteration.
// NST = ring depth (3: variant 3, default; 4: variant 4). Dropout (hashed mask regenerated per
// score) spills 9 VGPRs outside the hot loop and still beats the former rolled-ring kernel
// (975 vs 987 µs at the GPT-2 shape, p = 0.1; profiles/attn_bench_r2_dropout_ring.log).
template <int NST>
struct RingWait {  // s_waitcnt that leaves the newest NST - 2 stages' DMAs in flight
  template <int PER>  // DMA instructions per stage and wave (4 pieces, +1 LSE / δ row)
  static __device__ __forceinline__ void wait() {
    static_assert(NST >= 3 && NST <= 4 && (PER == 4 || PER == 5), "ring depth / pieces");
    if constexpr (NST == 3) {
      if constexpr (PER == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    } else {
      if constexpr (PER == 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    }
  }
};

// f(base + S, integral_constant<S>) for every S of the sequence (the ring stage is compile-time)
template <typename F, int... S>
__device__ __forceinline__ void ring_unroll(F&& f, int base, std::integer_sequence<int, S...>) {
  (f(base + S, std::integral_constant<int, S>{}), ...);
}
template <typename F, int... S>
__device__ __forceinline__ void ring_tail(F&& f, int base, int total, std::integer_sequence<int, S...>) {
  ((base + S < total ? f(base + S, std::integral_constant<int, S>{}) : void()), ...);
}

// GC: the query-group size H/Hkv when known at compile time (1: multi-head attention — the
// slice counter then maps to (head, slice) without the per-iteration division), 0 = any
// x as two bf16 (hi = bf16(x), lo = bf16(x − hi)) packed in the low / high halves of a word: the
// k = 0 / 1 elements of a fold operand — an MFMA against a "ones" operand adds hi + lo = x to within
// 2^-16 relative, exactly in its fp32 accumulator
__device__ __forceinline__ uint32_t bf16_hilo(float x) {
  const float hi = __bfloat162float(__float2bfloat16(x));
  return pack_bf16x2(hi, x - hi);
}

// STAMP (diagnostic build only, flash_bwd_stamps): s_memtime brackets around the phases of every
// ring iteration, summed per wave and added into stamps[0..5] (DMA issue, S/dP MFMA issue, softmax-
// gradient + dV/dK, DMA wait, barrier, iterations); sched_barrier(0) pins each bracket, so the
// instrumented schedule differs slightly from the production one
template <bool DROPOUT, int NST, int GC, bool STAMP = false>
__global__ void __launch_bounds__(256, 2) fa_bwd_dkdv3_kernel(const bf16* __restrict__ qkv,
                                                              const bf16* __restrict__ dout,
                                                              const float* __restrict__ lse,
                                                              const float* __restrict__ delta,
                                                              bf16* __restrict__ dqkv, float* __restrict__ cpart, int T, int H, int Hkv,
                                                              float scale, float p_drop, uint64_t seed,
                                                              unsigned long long* __restrict__ stamps = nullptr,
                                                              int diag = 0) {
  unsigned long long st_acc[5] = {0, 0, 0, 0, 0}, st_n = 0, st_t = 0;
  auto stamp = [&](int seg) {
    if constexpr (STAMP) {
      __builtin_amdgcn_sched_barrier(0);
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      if (seg >= 0) st_acc[seg] += now - st_t;
      st_t = now;
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  constexpr int BK = 128, QS = 64;
  constexpr int TILE = QS * 128;              // one 64-row slice, 128-B rows
  constexpr int STAGE = 2 * TILE + 512;       // Q | dO | LSE[64] | δ[64]
  __shared__ __attribute__((aligned(16))) char smem[NST * STAGE];
  int kb, bh;
  xcd_head_block(kb, bh);
  const int b = bh / Hkv, hk = bh % Hkv;
  const int G = GC ? GC : H / Hkv;
  const int lane = threadIdx.x & 63, w = wave_id(), hh = lane >> 5;
  const size_t RS = (size_t)(H + 2 * Hkv) * kD;
  const size_t ORS = (size_t)H * kD;
  const int kw0 = kb * BK + 32 * w;
  const int key = kw0 + (lane & 31);
  // dropout hash pieces (attn_common.h): seed mix ^ this lane's key-pair product, threshold
  const uint32_t dkey = DROPOUT ? dropout_seedmix(seed) ^ ((uint32_t)(key >> 1) * kDropKeyMul) : 0u;
  const uint32_t dthr = dropout_thr(p_drop);
  const float c = scale * kLog2e;
  const float inv_keep = DROPOUT ? 1.f / (1.f - p_drop) : 1.f;

  const bf16* kbase = qkv + (size_t)b * T * RS + (size_t)(H + hk) * kD;
  const bf16* vbase = qkv + (size_t)b * T * RS + (size_t)(H + Hkv + hk) * kD;
  uint4 kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = key < T ? *reinterpret_cast<const uint4*>(kbase + (size_t)key * RS + 16 * s + 8 * hh) : zero4();
    vf[s] = key < T ? *reinterpret_cast<const uint4*>(vbase + (size_t)key * RS + 16 * s + 8 * hh) : zero4();
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = scale_bf16x8(kf[s], c);  // S = Q·(cK)ᵀ (see scale_bf16x8); dK uses Q, not K
    launder(kf[s]);
    launder(vf[s]);
  }
  f32x16 dk[2], dv[2];
#pragma unroll
  for (int dh = 0; dh < 2; ++dh)
#pragma unroll
    for (int i = 0; i < 16; ++i) dk[dh][i] = dv[dh][i] = 0.f;
  // fold operands (k = 0 / 1 live in the first half-wave's lanes only): ones = 1.0 at k = 0 and 1
  const uint32_t lo_lane = hh == 0 ? 0xFFFFFFFFu : 0u;
  const uint4 onesf = uint4{0x3F803F80u & lo_lane, 0u, 0u, 0u};
  const f32x16 zacc = {};

  // per-lane LDS byte offsets: row reads (row lane&31, chunk 2s+hh) and transposed reads (rows
  // 4hh+q and 8+4hh+q, columns 32dh + 16((lane>>4)&1) + 4p); tile_off(r0 + x, ch) = 128·r0 +
  // tile_off(x, ch) for r0 % 16 == 0, so the row bases below are immediates
  unsigned ro[4], to[2][2];
#pragma unroll
  for (int s = 0; s < 4; ++s) ro[s] = (unsigned)tile_off(lane & 31, 2 * s + hh);
#pragma unroll
  for (int dh = 0; dh < 2; ++dh)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = 32 * dh + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
      to[dh][j] = (unsigned)(tile_off(4 * hh + ((lane & 15) >> 2) + 8 * j, col >> 3) + ((col & 4) << 1));
    }
  auto rowf = [&](const char* t, int s) -> uint4 { return *reinterpret_cast<const uint4*>(t + ro[s]); };
  auto trf = [&](const char* t, int dh) -> uint4 {
    const s16x4 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(t + to[dh][0]));
    const s16x4 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(t + to[dh][1]));
    const uint2 ux = __builtin_bit_cast(uint2, x), uy = __builtin_bit_cast(uint2, y);
    return uint4{ux.x, ux.y, uy.x, uy.y};
  };

  const int s_first = (kb * BK) / QS;
  const int nslices = (T + QS - 1) / QS;
  const int per_head = nslices - s_first;
  const int total = G * per_head;

  // DMA roles: w0/w1 -> Q rows 32w'..32w'+31 (pieces 4w'..4w'+3), w2/w3 -> dO likewise
  const int is_do = w >> 1, half_sel = w & 1;
  const unsigned rsb = (unsigned)(is_do ? ORS : RS) * 2;  // row stride in bytes
  unsigned voff[2];
#pragma unroll
  for (int par = 0; par < 2; ++par) {
    const int row = 8 * par + (lane >> 3);
    const int ch = (lane & 7) ^ ((((row >> 1) & 1) << 2) | ((row >> 2) & 3));
    voff[par] = (unsigned)(lane >> 3) * rsb + 16u * ch;
  }
  auto dma = [&](int it) {
    // (STAMP diagnostics, wrong results: diag 2 = no DMA at all, diag 1 = every DMA refetches the
    // first slice — cache-hot sources)
    if (STAMP && diag == 2) return;
    const int itc = (STAMP && diag == 1) ? 0 : min(it, total - 1);  // beyond the end: refetch the last slice
    const int hq = GC == 1 ? hk : hk * G + itc / per_head;
    const int qs0 = (s_first + (GC == 1 ? itc : itc % per_head)) * QS;
    const unsigned st = __builtin_amdgcn_readfirstlane(lds_addr_of(smem + (it % NST) * STAGE));
    const bf16* src = is_do ? dout + (size_t)b * T * ORS + (size_t)hq * kD : qkv + (size_t)b * T * RS + (size_t)hq * kD;
    const size_t rs = is_do ? ORS : RS;
    const unsigned dst = st + is_do * TILE + half_sel * 4096;
    if (qs0 + QS <= T) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int p = 4 * half_sel + i;
        glds16_s(reinterpret_cast<const char*>(src + (size_t)(qs0 + 8 * p) * rs), voff[p & 1], dst + i * 1024);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int p = 4 * half_sel + i;
        const int row = 8 * p + (lane >> 3);
        const int ch = (lane & 7) ^ ((((row >> 1) & 1) << 2) | ((row >> 2) & 3));
        glds16(src + (size_t)min(qs0 + row, T - 1) * rs + 8 * ch, dst + i * 1024);
      }
    }
    if (w < 2) {  // LSE (w0) / δ (w1) rows, clamped to T-1 (those rows are masked anyway)
      const float* sp = (w == 0 ? lse : delta) + ((size_t)b * H + hq) * T + min(qs0 + lane, T - 1);
      glds4(sp, st + 2 * TILE + 256 * w);
    }
  };
  auto wait_next = [&]() {  // this wave's DMAs for the next stage done; the later ones in flight
    if (w < 2)
      RingWait<NST>::template wait<5>();
    else
      RingWait<NST>::template wait<4>();
  };
  if (total > 0) {
#pragma unroll
    for (int i = 0; i < NST - 1; ++i) dma(i);
    wait_next();
  }
  __syncthreads();
  auto iter = [&](int it, auto stage_tag) {
    constexpr int ST = decltype(stage_tag)::value;
    stamp(-1);
    dma(it + NST - 1);  // into the stage consumed at it-1 (freed by its barrier)
    stamp(0);
    const char* stg = smem + ST * STAGE;
    const float* lse_s = reinterpret_cast<const float*>(stg + 2 * TILE);
    const float* del_s = lse_s + QS;
    const int hq = GC == 1 ? hk : hk * G + it / per_head;
    const int qs0 = (s_first + (GC == 1 ? it : it % per_head)) * QS;
    bool act[2];
    f32x16 sp[2], dp[2];
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int qh0 = qs0 + 32 * half;
      act[half] = qh0 + 31 >= kw0 && kw0 < T && qh0 < T;
      if (act[half]) {
        const char* Qt = stg + half * 32 * 128;
        const char* Dt = stg + TILE + half * 32 * 128;
        // all 8 operand fragments requested first, then the MFMAs: one LDS latency per half
        // instead of one per MFMA pair
        uint4 qa[4], da[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          qa[s] = rowf(Qt, s);
          da[s] = rowf(Dt, s);
        }
        // row constants folded into the chains: S starts at −LSE·log2(e) (P = exp2(S)) and dP at −δ
        // of each query row — one MFMA each against the ones operand (this lane's row = lane&31
        // supplies k = 0 / 1 as a bf16 hi + lo pair) instead of 32 per-register moves
        const int r = 32 * half + (lane & 31);
        const uint4 lfold = uint4{bf16_hilo(-lse_s[r] * kLog2e) & lo_lane, 0u, 0u, 0u};
        sp[half] = mfma32(lfold, onesf, zacc);
        if constexpr (DROPOUT) {
#pragma unroll
          for (int i = 0; i < 16; ++i) dp[half][i] = 0.f;
        } else {
          const uint4 dfold = uint4{bf16_hilo(-del_s[r]) & lo_lane, 0u, 0u, 0u};
          dp[half] = mfma32(dfold, onesf, zacc);
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          sp[half] = mfma32(qa[s], kf[s], sp[half]);
          dp[half] = mfma32(da[s], vf[s], dp[half]);
        }
      }
    }
    stamp(1);
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int qh0 = qs0 + 32 * half;
      if (act[half]) {
        const char* Qt = stg + half * 32 * 128;
        const char* Dt = stg + TILE + half * 32 * 128;
        const bool need_mask = (kw0 + 31 > qh0) || (qh0 + 32 > T) || (kw0 + 32 > T);
        const uint32_t drow0 = DROPOUT ? (uint32_t)((b * H + hq) * T + qh0 + 4 * hh) * kDropRowMul : 0u;
        // the dV / dK operand fragments (transposed reads) go out before the softmax-gradient VALU
        // (not with dropout: its hash registers leave no room — 42 spilled — so it reads at use)
        constexpr bool HOIST = !DROPOUT;
        uint4 tdo[2][2], tqq[2][2];
        if constexpr (HOIST) {
#pragma unroll
          for (int ss = 0; ss < 2; ++ss)
#pragma unroll
            for (int dh = 0; dh < 2; ++dh) {
              tdo[ss][dh] = trf(Dt + 16 * ss * 128, dh);
              tqq[ss][dh] = trf(Qt + 16 * ss * 128, dh);
            }
        }
        auto grads = [&](auto mask_tag) {
          constexpr bool MASK = decltype(mask_tag)::value;
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int r0 = 8 * g + 4 * hh;
            float4_t dl = {0.f, 0.f, 0.f, 0.f};
            if constexpr (DROPOUT) dl = *reinterpret_cast<const float4_t*>(&del_s[32 * half + r0]);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const int i = 4 * g + k;
              const int q = qh0 + r0 + k;
              float p = fexp2(sp[half][i]);
              if constexpr (MASK) p = (key > q || q >= T || key >= T) ? 0.f : p;
              if constexpr (DROPOUT) {  // row q = qh0 + 4hh + 8g + k: row product by addition
                const bool keep = dropout_keep_mixed(drow0 + (uint32_t)(8 * g + k) * kDropRowMul, dkey, key & 1, dthr);
                sp[half][i] = keep ? p * inv_keep : 0.f;
                dp[half][i] = p * ((keep ? dp[half][i] * inv_keep : 0.f) - dl[k]);
              } else {
                sp[half][i] = p;
                dp[half][i] = p * dp[half][i];
              }
            }
          }
        };
        if (need_mask)
          grads(std::true_type{});
        else
          grads(std::false_type{});
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          const uint4 pf = acc_frag(sp[half], ss), sf = acc_frag(dp[half], ss);
#pragma unroll
          for (int dh = 0; dh < 2; ++dh) {
            dv[dh] = mfma32(HOIST ? tdo[ss][dh] : trf(Dt + 16 * ss * 128, dh), pf, dv[dh]);
            dk[dh] = mfma32(HOIST ? tqq[ss][dh] : trf(Qt + 16 * ss * 128, dh), sf, dk[dh]);
          }
        }
      }
    }
    stamp(2);
    wait_next();
    stamp(3);
    __syncthreads();
    stamp(4);
    if constexpr (STAMP) ++st_n;
  };
  int it = 0;
  for (; it + NST <= total; it += NST) ring_unroll(iter, it, std::make_integer_sequence<int, NST>{});
  ring_tail(iter, it, total, std::make_integer_sequence<int, NST - 1>{});
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (STAMP) {
    if (lane == 0) {
#pragma unroll
      for (int i = 0; i < 5; ++i) atomicAdd(stamps + i, st_acc[i]);
      atomicAdd(stamps + 5, st_n);
    }
  }
  if (cpart != nullptr) {  // qkv-bias gradient: this wave's dK / dV column sums (one partial row)
    float* prow = cpart + (((size_t)b * gridDim.x + kb) * 4 + w) * RS;
    colsum32_wave(dk, scale, key < T, prow + (size_t)(H + hk) * kD);
    colsum32_wave(dv, 1.f, key < T, prow + (size_t)(H + Hkv + hk) * kD);
  }
  if (key < T) {
    bf16* dkrow = dqkv + ((size_t)b * T + key) * RS + (size_t)(H + hk) * kD;
    bf16* dvrow = dqkv + ((size_t)b * T + key) * RS + (size_t)(H + Hkv + hk) * kD;
#pragma unroll
    for (int dh = 0; dh < 2; ++dh)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = 32 * dh + 8 * g + 4 * hh;
        store4(dkrow + d, dk[dh][4 * g] * scale, dk[dh][4 * g + 1] * scale, dk[dh][4 * g + 2] * scale,
               dk[dh][4 * g + 3] * scale);
        store4(dvrow + d, dv[dh][4 * g], dv[dh][4 * g + 1], dv[dh][4 * g + 2], dv[dh][4 * g + 3]);
      }
  }
}

// dQ: grid (ceil(T/128) query blocks, heaviest first, B*H); forward-shaped — a wave keeps 32 query
// rows' Q, dO, LSE, δ and dQᵀ in registers while K / V tiles of 64 keys arrive by LDS-DMA into an
// NST-stage ring; per-lane precomputed LDS fragment offsets and the ring loop unrolled by its
// stages (stage bases and row bases become immediates), as in the dK/dV kernel.
template <bool DROPOUT, int NST>
__global__ void __launch_bounds__(256, 2) fa_bwd_dq4_kernel(const bf16* __restrict__ qkv, const bf16* __restrict__ dout,
                                                        const float* __restrict__ lse,
                                                        float* __restrict__ delta, bf16* __restrict__ dqkv, float* __restrict__ cpart,
                                                        int T, int H, int Hkv, float scale, float p_drop,
                                                        uint64_t seed, const bf16* __restrict__ out) {
  constexpr int BM = 128, BN = 64;
  __shared__ __attribute__((aligned(16))) char smem[NST][2][BN * 128];
  const int nqb = (T + BM - 1) / BM;
  int qi, bh;
  xcd_head_block(qi, bh);
  const int qb = nqb - 1 - qi;
  const int b = bh / H, h = bh % H, hk = h / (H / Hkv);
  const int lane = threadIdx.x & 63, w = wave_id(), hh = lane >> 5;
  const size_t RS = (size_t)(H + 2 * Hkv) * kD;
  const size_t ORS = (size_t)H * kD;
  const bf16* kbase = qkv + (size_t)b * T * RS + (size_t)(H + hk) * kD;
  const bf16* vbase = qkv + (size_t)b * T * RS + (size_t)(H + Hkv + hk) * kD;
  const int q0 = qb * BM + 32 * w;
  const int qrow = q0 + (lane & 31);
  // dropout hash pieces (attn_common.h): per-lane seed mix ^ row product, threshold
  const uint32_t drow = DROPOUT ? dropout_seedmix(seed) ^ ((uint32_t)((b * H + h) * T + qrow) * kDropRowMul) : 0u;
  const uint32_t dthr = dropout_thr(p_drop);
  const float c = scale * kLog2e;
  const float inv_keep = DROPOUT ? 1.f / (1.f - p_drop) : 1.f;

  uint4 qf[4], dof[4];
  const bool qok = qrow < T;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = qok ? *reinterpret_cast<const uint4*>(qkv + (size_t)b * T * RS + (size_t)h * kD + (size_t)qrow * RS + 16 * s +
                                                  8 * hh)
                : zero4();
    dof[s] = qok ? *reinterpret_cast<const uint4*>(dout + (size_t)b * T * ORS + (size_t)h * kD + (size_t)qrow * ORS +
                                                   16 * s + 8 * hh)
                 : zero4();
  }
  const size_t rr = ((size_t)b * H + h) * T + qrow;
  float l2 = qok ? lse[rr] * kLog2e : 0.f;
  float dl;
  if (out != nullptr) {
    // δ = Σ_d dO·O of this row, from the dO fragments already in registers and the matching O
    // fragments (lanes l and l + 32 hold the two halves of a row); written for the dK/dV kernel,
    // which runs after this one — no separate pre-pass over dO and O
    float sum = 0.f;
    if (qok) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const uint4 o4 = *reinterpret_cast<const uint4*>(out + (size_t)b * T * ORS + (size_t)h * kD +
                                                         (size_t)qrow * ORS + 16 * s + 8 * hh);
        const uint32_t ow[4] = {o4.x, o4.y, o4.z, o4.w}, dw[4] = {dof[s].x, dof[s].y, dof[s].z, dof[s].w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
          sum += __uint_as_float(ow[k] << 16) * __uint_as_float(dw[k] << 16) +
                 __uint_as_float(ow[k] & 0xffff0000u) * __uint_as_float(dw[k] & 0xffff0000u);
      }
    }
    sum += __shfl_xor(sum, 32, 64);
    dl = sum;
    if (qok && hh == 0) delta[rr] = sum;
  } else {
    dl = qok ? delta[rr] : 0.f;
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = scale_bf16x8(qf[s], c);  // S = (cQ)·Kᵀ (see scale_bf16x8); dQ uses K, not Q
    launder(qf[s]);
    launder(dof[s]);
  }
  asm volatile("" : "+v"(l2), "+v"(dl));
  // the S / dP accumulator starts (−LSE·log2 e and −δ of this lane's query row) as loop-invariant
  // register blocks: each chain's first MFMA reads its C operand from them, so no per-tile moves
  f32x16 s_init, dp_init;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    s_init[i] = -l2;
    dp_init[i] = DROPOUT ? 0.f : -dl;
  }

  // LDS-DMA ring (3 stages, two tiles ahead): waves 0-1 fetch the K tile, waves 2-3 the V
  // tile, 4 pieces (8 keys x 128 B each) per wave, tile_off image
  const int is_v = w >> 1, half_sel = w & 1;
  const unsigned RSB = (unsigned)RS * 2;
  unsigned voff[2];
#pragma unroll
  for (int par = 0; par < 2; ++par) {
    const int row = 8 * par + (lane >> 3);
    const int ch = (lane & 7) ^ ((((row >> 1) & 1) << 2) | ((row >> 2) & 3));
    voff[par] = (unsigned)(lane >> 3) * RSB + 16u * ch;
  }
  const bf16* dsrc = is_v ? vbase : kbase;
  const int kend = min(T, qb * BM + BM);
  const int ntiles = (kend + BN - 1) / BN;
  f32x16 dq[2];
#pragma unroll
  for (int dh = 0; dh < 2; ++dh)
#pragma unroll
    for (int i = 0; i < 16; ++i) dq[dh][i] = 0.f;

  unsigned ro[4], to[2][2];
#pragma unroll
  for (int s = 0; s < 4; ++s) ro[s] = (unsigned)tile_off(lane & 31, 2 * s + hh);
#pragma unroll
  for (int dh = 0; dh < 2; ++dh)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = 32 * dh + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
      to[dh][j] = (unsigned)(tile_off(4 * hh + ((lane & 15) >> 2) + 8 * j, col >> 3) + ((col & 4) << 1));
    }
  auto rowf = [&](const char* t, int s) -> uint4 { return *reinterpret_cast<const uint4*>(t + ro[s]); };
  auto trf = [&](const char* t, int dh) -> uint4 {
    const s16x4 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(t + to[dh][0]));
    const s16x4 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(t + to[dh][1]));
    const uint2 ux = __builtin_bit_cast(uint2, x), uy = __builtin_bit_cast(uint2, y);
    return uint4{ux.x, ux.y, uy.x, uy.y};
  };
  auto dma = [&](int jt) {
    const int kt0 = min(jt, ntiles - 1) * BN;  // beyond the end: refetch the last tile (uniform counts)
    const unsigned dst = __builtin_amdgcn_readfirstlane(lds_addr_of(smem[jt % NST][is_v])) + half_sel * 4096;
    if (kt0 + BN <= T) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int p = 4 * half_sel + i;
        glds16_s(reinterpret_cast<const char*>(dsrc + (size_t)(kt0 + 8 * p) * RS), voff[p & 1], dst + i * 1024);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int p = 4 * half_sel + i;
        const int row = 8 * p + (lane >> 3);
        const int ch = (lane & 7) ^ ((((row >> 1) & 1) << 2) | ((row >> 2) & 3));
        glds16(dsrc + (size_t)min(kt0 + row, T - 1) * RS + 8 * ch, dst + i * 1024);
      }
    }
  };
#pragma unroll
  for (int i = 0; i < NST - 1; ++i) dma(i);
  RingWait<NST>::template wait<4>();
  __syncthreads();
  auto iter = [&](int j, auto stage_tag) {
    constexpr int ST = decltype(stage_tag)::value;
    const int kt0 = j * BN;
    dma(j + NST - 1);  // into the stage consumed at j-1 (freed by its barrier)
    const char* Kt = smem[ST][0];
    const char* Vt = smem[ST][1];
    if (kt0 <= q0 + 31) {
      // dP starts from -δ (row constant = this lane's query row); per 32-key half the dS math
      // is followed by its dQ MFMAs so the second half's VALU overlaps the first half's MFMAs
      f32x16 s[2], dp[2];
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        uint4 ka[4], va[4];  // fragments first, then the MFMAs (one LDS latency per 32 keys)
#pragma unroll
        for (int st = 0; st < 4; ++st) {
          ka[st] = rowf(Kt + 32 * kh * 128, st);
          va[st] = rowf(Vt + 32 * kh * 128, st);
        }
        // S accumulates onto −LSE·log2(e) of this lane's query row (P = exp2(S)), dP onto −δ
        s[kh] = mfma32(ka[0], qf[0], s_init);
        dp[kh] = mfma32(va[0], dof[0], dp_init);
#pragma unroll
        for (int st = 1; st < 4; ++st) {
          s[kh] = mfma32(ka[st], qf[st], s[kh]);
          dp[kh] = mfma32(va[st], dof[st], dp[kh]);
        }
      }
      const bool need_mask = (kt0 + BN - 1 > q0) || (kt0 + BN > T) || (q0 + 32 > T);
      const uint32_t kpair0 = DROPOUT ? (uint32_t)((kt0 + 4 * hh) >> 1) * kDropKeyMul : 0u;
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        uint4 tk[2][2];  // the dQ operand fragments (transposed K reads) before the VALU
#pragma unroll
        for (int ss = 0; ss < 2; ++ss)
#pragma unroll
          for (int dh = 0; dh < 2; ++dh) tk[ss][dh] = trf(Kt + (32 * kh + 16 * ss) * 128, dh);
        auto grads = [&](auto mask_tag) {
          constexpr bool MASK = decltype(mask_tag)::value;
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int k = kt0 + 32 * kh + acc_row(i, lane);
            float p = fexp2(s[kh][i]);
            if constexpr (MASK) p = (k > qrow || k >= T || !qok) ? 0.f : p;
            if constexpr (DROPOUT) {  // key k = kt0 + 32kh + 4hh + (i&3) + 8(i>>2); pairs share a hash
              const uint32_t km = kpair0 + (uint32_t)(16 * kh + 4 * (i >> 2) + ((i & 3) >> 1)) * kDropKeyMul;
              const bool keep = dropout_keep_mixed(drow, km, (i & 1) != 0, dthr);
              s[kh][i] = p * ((keep ? dp[kh][i] * inv_keep : 0.f) - dl);
            } else {
              s[kh][i] = p * dp[kh][i];
            }
          }
        };
        if (need_mask)
          grads(std::true_type{});
        else
          grads(std::false_type{});
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          const uint4 sf = acc_frag(s[kh], ss);
#pragma unroll
          for (int dh = 0; dh < 2; ++dh) dq[dh] = mfma32(tk[ss][dh], sf, dq[dh]);
        }
      }
    }
    RingWait<NST>::template wait<4>();  // tile j+1 landed, the later ones in flight
    __syncthreads();
  };
  int j = 0;
  for (; j + NST <= ntiles; j += NST) ring_unroll(iter, j, std::make_integer_sequence<int, NST>{});
  ring_tail(iter, j, ntiles, std::make_integer_sequence<int, NST - 1>{});
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (cpart != nullptr)  // qkv-bias gradient: this wave's dQ column sums (one partial row)
    colsum32_wave(dq, scale, qok, cpart + (((size_t)b * nqb + qb) * 4 + w) * RS + (size_t)h * kD);
  if (qok) {
    bf16* dqrow = dqkv + ((size_t)b * T + qrow) * RS + (size_t)h * kD;
#pragma unroll
    for (int dh = 0; dh < 2; ++dh)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        store4(dqrow + 32 * dh + 8 * g + 4 * hh, dq[dh][4 * g] * scale, dq[dh][4 * g + 1] * scale,
               dq[dh][4 * g + 2] * scale, dq[dh][4 * g + 3] * scale);
  }
}

}  // namespace penroz

// ============================================================================ host side
using namespace penroz;

static void check_qkv(const torch::Tensor& qkv, int64_t H, int64_t Hkv, int64_t D) {
  TORCH_CHECK(qkv.is_cuda() && qkv.is_contiguous() && qkv.dim() == 3, "qkv must be a contiguous [B, T, W] GPU tensor");
  TORCH_CHECK(qkv.scalar_type() == torch::kBFloat16, "flash attention expects bf16");
  TORCH_CHECK(D == kD, "flash attention kernel is built for head_dim 64");
  TORCH_CHECK(H % Hkv == 0 && qkv.size(2) == (H + 2 * Hkv) * D, "qkv width must be (H + 2*Hkv)*D");
}

static int g_fa_fwd_variant = 3;

void flash_attn_fwd(torch::Tensor qkv, torch::Tensor out, torch::Tensor lse, int64_t H, int64_t Hkv, int64_t D,
                    double scale, double p_drop, int64_t seed) {
  check_qkv(qkv, H, Hkv, D);
  const int B = qkv.size(0), T = qkv.size(1);
  TORCH_CHECK(out.is_contiguous() && out.scalar_type() == torch::kBFloat16 && out.numel() == (int64_t)B * T * H * D);
  TORCH_CHECK(lse.is_contiguous() && lse.scalar_type() == torch::kFloat32 && lse.numel() == (int64_t)B * H * T);
  if (B == 0 || T == 0) return;
  dim3 grid((T + 127) / 128, B * H);
  auto stream = at::hip::getCurrentHIPStream();
  const bf16* q = reinterpret_cast<const bf16*>(qkv.data_ptr());
  bf16* o = reinterpret_cast<bf16*>(out.data_ptr());
  // dropout takes the single-stage kernel: the two-block kernel spills with the mask hashing of
  // both query blocks live (159 VGPRs to scratch)
  if (p_drop > 0.0)
    hipLaunchKernelGGL(fa_fwd_kernel<true>, grid, dim3(256), 0, stream, q, o, lse.data_ptr<float>(), T, (int)H,
                       (int)Hkv, (float)scale, (float)p_drop, (uint64_t)seed);
  else if (g_fa_fwd_variant == 1)
    hipLaunchKernelGGL(fa_fwd_kernel<false>, grid, dim3(256), 0, stream, q, o, lse.data_ptr<float>(), T, (int)H,
                       (int)Hkv, (float)scale, 0.f, (uint64_t)seed);
  else
    hipLaunchKernelGGL(fa_fwd3_kernel<false>, grid, dim3(128), 0, stream, q, o, lse.data_ptr<float>(), T, (int)H,
                       (int)Hkv, (float)scale, 0.f, (uint64_t)seed);
}

// forward: 1 = single-stage (fa_fwd_kernel; also the dropout path), 3 = two query blocks per
// wave (fa_fwd3_kernel, default). backward:
// 3-stage LDS-DMA rings throughout the backward (4 stages measured neutral in the training step:
// 65.47 / 65.51 vs 65.52 / 65.35 ms, so the knob is gone)
int64_t flash_fwd_variant(int64_t v) {
  const int64_t prev = g_fa_fwd_variant;
  if (v > 0) g_fa_fwd_variant = (int)v;
  return prev;
}

// dbias (optional, fp32 [(H + 2·Hkv)·D]): += the column sums of dqkv over all B·T rows (the fused
// QKV projection's bias gradient), produced in the dK/dV and dQ epilogues (one fp32 partial row
// per 32-row wave slice, finished by the deferred reduction).
// diagnostic: when set (uint64 [6] on the GPU), the MHA no-dropout dK/dV launch runs the STAMP build
static unsigned long long* g_fa_stamps = nullptr;
void flash_bwd_stamps(c10::optional<torch::Tensor> buf) {
  if (buf.has_value() && buf->defined()) {
    TORCH_CHECK(buf->is_cuda() && buf->scalar_type() == torch::kInt64 && buf->numel() >= 6 && buf->is_contiguous());
    g_fa_stamps = reinterpret_cast<unsigned long long*>(buf->data_ptr());
  } else {
    g_fa_stamps = nullptr;
  }
}

void flash_attn_bwd(torch::Tensor dout, torch::Tensor qkv, torch::Tensor out, torch::Tensor lse, torch::Tensor dqkv,
                    int64_t H, int64_t Hkv, int64_t D, double scale, double p_drop, int64_t seed,
                    c10::optional<torch::Tensor> dbias) {
  check_qkv(qkv, H, Hkv, D);
  const int B = qkv.size(0), T = qkv.size(1);
  TORCH_CHECK(dout.is_contiguous() && dout.scalar_type() == torch::kBFloat16 && dout.numel() == (int64_t)B * T * H * D);
  TORCH_CHECK(out.is_contiguous() && out.numel() == dout.numel());
  TORCH_CHECK(dqkv.is_contiguous() && dqkv.scalar_type() == torch::kBFloat16 && dqkv.numel() == qkv.numel());
  if (B == 0 || T == 0) return;
  auto delta = torch::empty({B, H, T}, qkv.options().dtype(torch::kFloat32));
  auto stream = at::hip::getCurrentHIPStream();
  // δ = rowsum(dO·O) is computed by the dQ kernel from the dO fragments it loads anyway and written
  // for the dK/dV kernel, so dQ runs first (PENROZ_FA_DELTA_PREPASS=1: the separate pre-pass)
  static const bool prepass = [] {
    const char* e = std::getenv("PENROZ_FA_DELTA_PREPASS");
    return e && e[0] == '1';
  }();
  if (prepass) {
    const int rows = B * T * H;
    hipLaunchKernelGGL(fa_bwd_pre_kernel, dim3((rows * 8 + 255) / 256), dim3(256), 0, stream,
                       reinterpret_cast<const bf16*>(dout.data_ptr()), reinterpret_cast<const bf16*>(out.data_ptr()),
                       delta.data_ptr<float>(), B, T, (int)H);
  }
  const bf16* q = reinterpret_cast<const bf16*>(qkv.data_ptr());
  const bf16* d = reinterpret_cast<const bf16*>(dout.data_ptr());
  bf16* g = reinterpret_cast<bf16*>(dqkv.data_ptr());
  dim3 gkv((T + 127) / 128, B * Hkv), gq((T + 127) / 128, B * H);
  using BwdKernel = void (*)(const bf16*, const bf16*, const float*, const float*, bf16*, float*, int, int, int, float, float,
                            uint64_t, unsigned long long*, int);
  using DqKernel = void (*)(const bf16*, const bf16*, const float*, float*, bf16*, float*, int, int, int, float, float,
                            uint64_t, const bf16*);
  const bool drop = p_drop > 0.0;
  BwdKernel kv;
  DqKernel dq;
  if (H == Hkv && !drop && g_fa_stamps)
    kv = fa_bwd_dkdv3_kernel<false, 3, 1, true>;
  else if (H == Hkv)
    kv = drop ? fa_bwd_dkdv3_kernel<true, 3, 1> : fa_bwd_dkdv3_kernel<false, 3, 1>;
  else
    kv = drop ? fa_bwd_dkdv3_kernel<true, 3, 0> : fa_bwd_dkdv3_kernel<false, 3, 0>;
  dq = drop ? fa_bwd_dq4_kernel<true, 3> : fa_bwd_dq4_kernel<false, 3>;
  const float pd = drop ? (float)p_drop : 0.f;
  // (STAMP diagnostics only: PENROZ_FA_STAMP_DIAG=1 cache-hot DMA sources, 2 no DMA)
  static const int kv_diag = [] {
    const char* e = std::getenv("PENROZ_FA_STAMP_DIAG");
    return e ? std::atoi(e) : 0;
  }();
  const bool want_bias = dbias.has_value() && dbias->defined();
  const int W = (int)((H + 2 * Hkv) * D), nblk = (T + 127) / 128;
  if (want_bias)
    TORCH_CHECK(dbias->is_cuda() && dbias->scalar_type() == torch::kFloat32 && dbias->is_contiguous() &&
                    dbias->numel() == W, "dbias must be a contiguous fp32 [(H + 2*Hkv)*D] GPU tensor");
  torch::Tensor part;
  if (want_bias) part = torch::empty({(int64_t)B * nblk * 4, W}, qkv.options().dtype(torch::kFloat32));
  float* pp = want_bias ? part.data_ptr<float>() : nullptr;
  hipLaunchKernelGGL(dq, gq, dim3(256), 0, stream, q, d, lse.data_ptr<float>(), delta.data_ptr<float>(), g, pp, T,
                     (int)H, (int)Hkv, (float)scale, pd, (uint64_t)seed,
                     prepass ? nullptr : reinterpret_cast<const bf16*>(out.data_ptr()));
  hipLaunchKernelGGL(kv, gkv, dim3(256), 0, stream, q, d, lse.data_ptr<float>(), delta.data_ptr<float>(), g, pp, T,
                     (int)H, (int)Hkv, (float)scale, pd, (uint64_t)seed, g_fa_stamps, kv_diag);
  if (want_bias) {
    float* outs[1] = {dbias->data_ptr<float>()};
    reduce_partials_auto(part, 1, B * nblk * 4, W, outs, stream);
  }
}
