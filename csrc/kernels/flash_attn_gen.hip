// Causal flash attention for head_dim 128, 256 and 512 (Gemma-family training / prefill; the tuned
// head_dim-64 kernels live in flash_attn.hip). bf16 in/out, fp32 accumulate, GQA by index math.
//
// Same algebra and operand maps as the head_dim-64 kernels (v_mfma_f32_32x32x16_bf16 with the
// key on the MFMA lane or row so softmax rows never cross LDS; see flash_attn.hip), generalised
// over D by storing every LDS tile as D/64 "panels" of 64 columns: panel p holds columns
// 64p..64p+63 of all the tile's rows in the head_dim-64 image (128-B rows, XOR-swizzled chunk
// order tile_off), so the bank-conflict-free row reads (ds_read_b128) and transposed reads
// (ds_read_b64_tr_b16) carry over unchanged. Tiles arrive by LDS-DMA (global_load_lds_dwordx4,
// swizzle applied on the per-lane SOURCE address, the LDS image stays lane-linear), double
// buffered: tile j+1 is in flight while tile j computes.
//
//   forward   — 32-key tiles; Sᵀ = K·Qᵀ (Q in registers), online softmax per lane (one query row
//               per lane), Oᵀ += Vᵀ·Pᵀ; heaviest query blocks first; writes O head-merged and the
//               row log-sum-exp (natural log), like the head_dim-64 kernel. D = 128: 2 waves ×
//               32 rows. D = 256 / 512: 8 waves, the head dimension split over 2 / 4 waves that
//               share 32 query rows — each holds its part of Q, computes the partial S over it and
//               owns that part of the Oᵀ columns; the partials are summed through LDS in part order
//               (bitwise the same S in every wave of the group), ≤ 256 registers: 2 waves / SIMD.
//   backward  — δ = rowsum(dO·O); dK/dV kernel (fa_roles_bwd_dkdv_kernel): per 32 keys an S-wave
//               (cK in registers, dVᵀ accumulators) and a dP-wave (V, dKᵀ) sweep the 32-row query
//               slices of every query head of the KV group, P handed over through LDS (no
//               cross-workgroup sum, deterministic); dQ kernel: forward-shaped, Q, dO and dQᵀ in
//               registers (D = 256 / 512: split over 2 / 4 waves, partial S and dP exchanged).
// D = 512 (Gemma-4 full-attention layers, global_head_dim) splits dVᵀ / dKᵀ over two workgroups.
#include "attn_common.h"
#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <queue>
#include <tuple>
#include <type_traits>
#include <vector>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

namespace penroz {

// At D = 256 hipcc would hoist every LDS fragment read of a fully unrolled MFMA chain ahead of
// the chain (~128 extra VGPRs beside 128–256 accumulators) and spill; a scheduling fence per
// group keeps at most a few fragments in flight.
template <int D>
__device__ __forceinline__ void d_fence() {
  if constexpr (D >= 256) __builtin_amdgcn_sched_barrier(0);
}

// panel p of an LDS tile with R rows (R·128 bytes per panel)
__device__ __forceinline__ const char* panel(const char* tile, int R, int p) { return tile + p * R * 128; }

// swizzle of the LDS image for row r (depends on r & 15): physical chunk = logical ^ swz(r)
__device__ __forceinline__ int swz(int r) { return (((r >> 1) & 1) << 2) | ((r >> 2) & 3); }

// DMA R rows × D columns of a row-major bf16 matrix (row stride RS elements) into the paneled
// tile image (PR rows per panel) at LDS byte address `dst`: NP·R/8 pieces (8 rows × 128 B each)
// issued by this wave. Rows past T are clamped to T-1 (finite data the mask / P = 0 cancels).
template <int NP, int R = 32, int PR = R>
__device__ __forceinline__ void dma_rows(const bf16* base, size_t RS, int r0, int T, unsigned dst, int lane) {
  const int rr = lane >> 3;
#pragma unroll
  for (int p = 0; p < NP; ++p)
#pragma unroll
    for (int r8 = 0; r8 < R / 8; ++r8) {
      const int lc = (lane & 7) ^ swz(8 * (r8 & 1) + rr);  // the image row is 8·r8 + rr (PR, R % 16 == 0)
      const int row = min(r0 + 8 * r8 + rr, T - 1);
      glds16(base + (size_t)row * RS + 64 * p + 8 * lc, dst + (p * PR + 8 * r8) * 128);
    }
}

// D-split exchange (D = 512): the ZS waves of row group rg each hold a partial accumulator over
// their part of D; after this every one of them holds the sum, added in part order (so the ZS
// copies are bitwise identical). x4 = this lane's slot of an LDS [wave][4][64] float4 image
// (conflict-free b128 rows); `act` is uniform over the row group. Ends with the readers done
// only if the caller adds a barrier before reusing the image.
template <int ZS>
__device__ __forceinline__ void dsplit_sum(f32x16& v, float4_t* x4, int w, int rg, bool act) {
  if (act)
#pragma unroll
    for (int i4 = 0; i4 < 4; ++i4) x4[(w * 4 + i4) * 64] = float4_t{v[4 * i4], v[4 * i4 + 1], v[4 * i4 + 2], v[4 * i4 + 3]};
  __syncthreads();
  if (act) {
    const float4_t* r4 = x4 + rg * ZS * 4 * 64;
#pragma unroll
    for (int i4 = 0; i4 < 4; ++i4) {
      float4_t a = r4[i4 * 64];
#pragma unroll
      for (int z = 1; z < ZS; ++z) a += r4[(z * 4 + i4) * 64];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[4 * i4 + k] = a[k];
    }
  }
}

// ------------------------------------------------------------------------------------------
// forward
// D = 256 runs 4 waves per workgroup (128 query rows): its LDS (K/V double buffer + the Q image,
// 128 KB) admits one workgroup per CU, and 4 waves then occupy all four SIMDs.
template <int D> constexpr int fwd_waves() { return D >= 256 ? 8 : 2; }
// column parts of the backward kernels (folded into the 1-D grid as virtual heads, see
// item_head): dK / dV and dQ accumulators per part
// D = 512 splits the head dimension across the waves of ONE workgroup instead (no recomputation):
//   forward: 8 waves, a group of four shares 32 query rows; each wave holds a quarter of Q in
//   registers, computes the partial S over its quarter of D and owns a quarter of the Oᵀ columns;
//   the partials meet in LDS (one exchange per tile, summed in quarter order: bitwise the same S
//   in all four waves). ≤ 256 registers per wave: two waves per SIMD, no spills (the 4-wave halves
//   version spilled ~90 B per lane and ran fwd at 195 TF);
//   dQ: the same (8 waves, quarters of Q, dO; partial S, then partial dP exchanged);
//   dK / dV: fa_roles_bwd_dkdv_kernel below (S-wave / dP-wave roles, every D).
// (The round-4 design recomputed S over the full D in every column part — forward 2×, dQ 2×,
// dK / dV 4× — and still spilled 350-560 B per lane: 106 / 64 TF fwd / bwd, slower than SDPA.)
template <int D> constexpr int fwd_dsplit() { return D >= 512 ? 4 : (D >= 256 ? 2 : 1); }
template <int D> constexpr int dq_dsplit() { return D >= 512 ? 4 : (D >= 256 ? 2 : 1); }

// ---- work lists (causal balance) ---------------------------------------------------------
// A causal query block's cost grows with its index, so a grid that fits in ONE round of
// workgroups (Gemma-3 1B at B = 8: 256 forward workgroups on 256 CUs) runs as long as its
// heaviest block — about 1.8× the mean. The forward and dQ kernels therefore take a per-head
// work list, heaviest item first: block qb whole, or (qb >= split0) one of the two halves of its
// key-tile range, each half writing fp32 partials that fa_gen_combine merges (forward: the
// online-softmax (m, l) merge; dQ: a plain sum). The host picks split0 by simulating the
// workgroup dispatch (attn_plan below). Launch order is item-major across the heads of an XCD, so
// every XCD runs its heaviest items first (a head-major order dealt a whole second plane of
// workgroups to CUs in head order rather than by size).
constexpr int kMaxItems = 480;
struct WorkList {
  int n;       // items per head
  int split0;  // first split block (>= number of blocks: nothing split, item i = block n-1-i)
  int it[kMaxItems];  // block | part << 16 (part 0 whole, 1 first half, 2 second half)
};

// blockIdx.x over n_items × (zp·heads) workgroups -> (item, virtual head vh = z·heads + head):
// virtual heads are dealt to the 8 XCDs round-robin (a head's z parts share an XCD when heads is
// a multiple of 8), items outermost within an XCD
__device__ __forceinline__ void item_head(int nitems, int& item, int& vh) {
  const int nvh = gridDim.x / nitems, id = blockIdx.x;
  const int hp = nvh >> 3, full = hp * nitems;
  const int xcd = id & 7, slot = id >> 3;
  if (slot < full) {
    item = slot / hp;
    vh = (slot - item * hp) * 8 + xcd;
  } else {
    const int r = id - 8 * full, nt = nvh & 7;
    item = r / nt;
    vh = (nvh & ~7) + (r - item * nt);
  }
}

// item -> (block, part); the part's key tiles: [0, n) whole, [0, n/2) first, [n/2, n) second half
__device__ __forceinline__ void item_block(const WorkList& wl, int nblk, int item, int& blk, int& part) {
  if (wl.split0 >= nblk) {
    blk = nblk - 1 - item;
    part = 0;
  } else {
    const int e = wl.it[item];
    blk = e & 0xffff;
    part = e >> 16;
  }
}

__device__ __forceinline__ void part_tiles(int part, int n, int& j0, int& j1) {
  j0 = part == 2 ? n / 2 : 0;
  j1 = part == 1 ? n / 2 : n;
}

template <int D, bool DROPOUT>
__global__ void __launch_bounds__(64 * fwd_waves<D>(), (D >= 256 ? 1 : 2))
    fa_gen_fwd_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ out, float* __restrict__ lse, int T, int H,
                      int Hkv, float scale, float p_drop, uint64_t seed, const WorkList wl, float* __restrict__ ws) {
  constexpr int NP = D / 64, NS = D / 16, ND = D / 32, NW = fwd_waves<D>(), ZS = fwd_dsplit<D>();
  constexpr int BM = 32 * NW / ZS, BN = 32, TILE = BN * 128 * NP;
  // D = 256: the 32 Q fragments would not fit beside Oᵀ (128 accumulators) in registers; the
  // workgroup's query rows sit in LDS instead (read as B-operand row fragments per tile).
  // D = 512: the K / V double buffer alone is 128 KB; a wave keeps its quarter of Q (32 VGPRs) in
  // registers and accumulates its quarter of Oᵀ (fwd_dsplit)
  constexpr bool QLDS = D == 256 && ZS == 1;
  constexpr int NDO = ND / ZS, NSH = NS / ZS;
  constexpr int QTILE = QLDS ? BM * 128 * NP : (ZS > 1 ? 0 : 16);
  constexpr int XB = ZS > 1 ? NW * 16 * 64 * 4 : 16;  // partial-S exchange: [wave][4][64 lanes] float4
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE + QTILE + XB];
  const int nqb = (T + BM - 1) / BM;
  int item, vh, qb, part;
  item_head(wl.n, item, vh);
  item_block(wl, nqb, item, qb, part);
  const int nbh = gridDim.x / wl.n;
  const int bh = vh;
  const int b = bh / H, h = bh % H, hk = h / (H / Hkv);
  const int lane = threadIdx.x & 63, w = wave_id(), hh = lane >> 5;
  const int rg = w / ZS, dz = w % ZS;  // row group (32 query rows), part of D (ZS = 4: a quarter)
  const int do0 = dz * NDO, sq0 = dz * NSH;
  const size_t RS = (size_t)(H + 2 * Hkv) * D;
  const bf16* qbase = qkv + (size_t)b * T * RS + (size_t)h * D;
  const bf16* kbase = qkv + (size_t)b * T * RS + (size_t)(H + hk) * D;
  const bf16* vbase = qkv + (size_t)b * T * RS + (size_t)(H + Hkv + hk) * D;
  const int q0 = qb * BM + 32 * rg;
  const int qrow = q0 + (lane & 31);
  const float c = scale * kLog2e;
  const float inv_keep = DROPOUT ? 1.f / (1.f - p_drop) : 1.f;
  const char* Qs = smem + 4 * TILE;
  float* xb = reinterpret_cast<float*>(smem + 4 * TILE + QTILE);

  uint4 qf[QLDS ? 1 : NSH];
  if constexpr (QLDS) {
    // both waves' rows, 32 per wave, into one 64-row paneled image
    dma_rows<NP, 32, BM>(qbase, RS, qb * BM + 32 * w, T,
                         __builtin_amdgcn_readfirstlane(lds_addr_of(smem + 4 * TILE)) + w * 32 * 128, lane);
  } else {
#pragma unroll
    for (int s = 0; s < NSH; ++s)
      qf[s] = qrow < T ? *reinterpret_cast<const uint4*>(qbase + (size_t)qrow * RS + 16 * (sq0 + s) + 8 * hh) : zero4();
#pragma unroll
    for (int s = 0; s < NSH; ++s) launder(qf[s]);
  }
  // B fragment s (of this wave's NSH) of Qᵀ: element j = Q[qrow][16(sq0 + s) + 8hh + j]
  auto qfrag = [&](int s) -> uint4 {
    if constexpr (QLDS) return row_frag(panel(Qs, BM, s >> 2), 32 * w, s & 3, lane);
    else return qf[s];
  };

  const int kend = min(T, qb * BM + BM);
  int j0, j1;
  part_tiles(part, (kend + BN - 1) / BN, j0, j1);
  f32x16 o[NDO];
#pragma unroll
  for (int dh = 0; dh < NDO; ++dh)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[dh][i] = 0.f;
  float m = -1e30f, l = 0.f;

  auto dma = [&](int j, int ln) {  // even waves: K tile, odd waves: V tile (NW = 4: half the panels each)
    constexpr int NPW = NP * 2 / NW;
    const int p0 = (w >> 1) * NPW;
    const unsigned dst = __builtin_amdgcn_readfirstlane(lds_addr_of(smem + ((j & 1) * 2 + (w & 1)) * TILE)) +
                         p0 * BN * 128;
    dma_rows<NPW>(((w & 1) == 0 ? kbase : vbase) + 64 * p0, RS, j * BN, T, dst, ln);
  };

  if (j0 < j1) dma(j0, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int j = j0; j < j1; ++j) {
    const int kt0 = j * BN;
    const int ln = lane;
    if (j + 1 < j1) dma(j + 1, ln);  // buffer (j+1)&1 was released by the previous barrier
    const char* Kt = smem + (j & 1) * 2 * TILE;
    const char* Vt = Kt + TILE;
    const bool act = kt0 <= q0 + 31 && q0 < T;  // uniform over a wave pair (same rows)
    f32x16 st;
#pragma unroll
    for (int i = 0; i < 16; ++i) st[i] = 0.f;
    if (act) {
      const char* Kh = Kt + (sq0 >> 2) * BN * 128;  // this wave's half of D (compile-time offsets below)
#pragma unroll
      for (int s = 0; s < NSH; ++s) {
        st = mfma32(row_frag(panel(Kh, BN, s >> 2), 0, s & 3, ln), qfrag(s), st);
        if ((s & 3) == 3) d_fence<D>();
      }
    }
    if constexpr (ZS > 1) dsplit_sum<ZS>(st, reinterpret_cast<float4_t*>(xb) + ln, w, rg, act);
    if (act) {
      auto softmax = [&](auto mask_tag) {
        constexpr bool MASK = decltype(mask_tag)::value;
        float tmax = -INFINITY;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          if constexpr (MASK) {
            const int key = kt0 + acc_row(i, lane);
            st[i] = (key > qrow || key >= T) ? -INFINITY : st[i];
          }
          tmax = fmaxf(tmax, st[i]);
        }
        tmax = halves_max(tmax) * c;
        if (!__all(tmax <= m + kRescaleThr)) {
          const float mnew = fmaxf(m, tmax);
          const float alpha = fexp2(m - mnew);
          m = mnew;
          l *= alpha;
#pragma unroll
          for (int dh = 0; dh < NDO; ++dh)
#pragma unroll
            for (int i = 0; i < 16; ++i) o[dh][i] *= alpha;
        }
        const float negm = -m;
        float lsum = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float p = fexp2(fmaf(st[i], c, negm));
          lsum += p;
          if constexpr (DROPOUT) {
            const int key = kt0 + acc_row(i, lane);
            p = dropout_keep(seed, b, h, H, T, qrow, key, p_drop) ? p * inv_keep : 0.f;
          }
          st[i] = p;
        }
        l += lsum;
      };
      if (kt0 + BN - 1 > q0 || kt0 + BN > T)
        softmax(std::true_type{});
      else
        softmax(std::false_type{});
      const char* Vh = Vt + (do0 >> 1) * BN * 128;  // do0 even
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const uint4 pf = acc_frag(st, ss);
#pragma unroll
        for (int j = 0; j < NDO; ++j) {
          o[j] = mfma32(tr_frag(panel(Vh, BN, j >> 1), 16 * ss, 32 * (j & 1), ln), pf, o[j]);
          if (j & 1) d_fence<D>();
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  l = halves_sum(l);
  if (part != 0) {  // half of a split block: raw Oᵀ, m, l (fp32) for fa_gen_combine
    if (qrow < T) {
      const size_t nsr = (size_t)(nqb - wl.split0) * BM;  // split rows per head
      const size_t r = ((size_t)(part - 1) * nbh + bh) * nsr + (qrow - wl.split0 * BM);
      float* orow = ws + r * D;
#pragma unroll
      for (int j = 0; j < NDO; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<float4*>(orow + 32 * (do0 + j) + 8 * g + 4 * hh) =
              float4{o[j][4 * g], o[j][4 * g + 1], o[j][4 * g + 2], o[j][4 * g + 3]};
      if (hh == 0 && do0 == 0)
        *reinterpret_cast<float2*>(ws + 2 * nbh * nsr * D + 2 * r) = float2{m, l};
    }
    return;
  }
  const float inv = l > 0.f ? 1.f / l : 0.f;
  if (qrow < T) {
    bf16* orow = out + ((size_t)b * T + qrow) * H * D + (size_t)h * D;
#pragma unroll
    for (int j = 0; j < NDO; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        store4(orow + 32 * (do0 + j) + 8 * g + 4 * hh, o[j][4 * g] * inv, o[j][4 * g + 1] * inv,
               o[j][4 * g + 2] * inv, o[j][4 * g + 3] * inv);
    if (hh == 0 && do0 == 0) lse[((size_t)b * H + h) * T + qrow] = (m + log2f(l)) * kLn2;
  }
}

// ------------------------------------------------------------------------------------------
// backward preprocessing: delta[b, h, q] = Σ_d dO·O  (D/8 lanes per row, 16-B loads)
template <int D>
__global__ void __launch_bounds__(256) fa_gen_bwd_pre_kernel(const bf16* __restrict__ dout,
                                                             const bf16* __restrict__ out, float* __restrict__ delta,
                                                             int B, int T, int H) {
  constexpr int LPR = D / 8;  // lanes per row (16 or 32; divides 64)
  const int gid = blockIdx.x * 256 + threadIdx.x;
  const int row = gid / LPR, part = gid % LPR;  // row over B*T*H in [b][t][h] order
  const bool ok = row < B * T * H;
  float s = 0.f;
  if (ok) {
    float a[8], o[8];
    Vec8<bf16>::load(dout + (size_t)row * D + 8 * part, a);
    Vec8<bf16>::load(out + (size_t)row * D + 8 * part, o);
#pragma unroll
    for (int k = 0; k < 8; ++k) s += a[k] * o[k];
  }
#pragma unroll
  for (int off = 1; off < LPR; off <<= 1) s += __shfl_xor(s, off, 64);
  if (ok && part == 0) {
    const int h = row % H, t = (row / H) % T, b = row / (H * T);
    delta[((size_t)b * H + h) * T + t] = s;
  }
}

// ------------------------------------------------------------------------------------------
// dK / dV: 1-D grid over (key block of 64, KV head [, query head: split], column part); heaviest
// key block first. 4 waves = 2 key groups (32 keys each) × 2 roles, sweeping the 32-row query
// slices (Q | dO | LSE | δ, double-buffered by LDS-DMA) of every query head of the KV group. The S-wave holds
// cK (32 fragments, full D) and accumulates dVᵀ over all of D; the dP-wave holds V and accumulates
// dKᵀ. Per 32-row query slice the S-wave computes S and P and hands P (fp32) to its dP-wave through
// LDS; the dP-wave forms dS = P ⊙ (dP − δ). Each wave then runs 32 MFMAs of S or dP and 32 of dV or
// dK. D = 128 / 256: 32 / 64 operand + 64 / 128 accumulator registers, 3 / 2 waves per SIMD, no
// recomputation (the round-4 kernel held K and V in every wave and computed both S and dP —
// at D = 256 in both column halves of two workgroups: D = 128 bwd 1855 -> 1502 µs, D = 256
// 227 -> 177 µs). D = 512: the dVᵀ / dKᵀ columns are split over kv_role_parts = 2 workgroups
// (virtual heads) — a wave's 256 accumulators for all of D beside its 128 operand registers
// spilled ~800 B — so S and dP are computed twice (the round-4 kernel: four times).
// Query-head split (part != nullptr): each workgroup sweeps ONE query head of its group and writes
// fp32 partial dK / dV ([G][B·T][K | V][Hkv·D]) that fa_gen_kv_reduce sums (Gemma-3 1B: Hkv = 1).
template <int D> constexpr int kv_role_parts() { return D >= 512 ? 2 : 1; }

template <int D, bool DROPOUT>
__global__ void __launch_bounds__(256, (D >= 512 ? 1 : 2))
    fa_roles_bwd_dkdv_kernel(const bf16* __restrict__ qkv, const bf16* __restrict__ dout, const float* __restrict__ lse,
                          const float* __restrict__ delta, bf16* __restrict__ dqkv, float* __restrict__ part, int T,
                          int H, int Hkv, float scale, float p_drop, uint64_t seed) {
  constexpr int NP = D / 64, NS = D / 16, ND = D / 32, NDW = ND / kv_role_parts<D>();
  constexpr int BK = 64, QS = 32;
  constexpr int TILE = QS * 128 * NP;          // one 32-row slice of Q (or dO)
  constexpr int STAGE = 2 * TILE + 2 * 256;    // Q | dO | LSE[64] | δ[64]
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE + 2 * 16 * 64 * 4];
  float* xp = reinterpret_cast<float*>(smem + 2 * STAGE);  // P hand-over: [key group][16][64]
  int kb, vh;
  item_head((T + BK - 1) / BK, kb, vh);
  const int nbhx = gridDim.x / (((T + BK - 1) / BK) * kv_role_parts<D>());
  const int zc = vh / nbhx, bhx = vh - zc * nbhx;
  const int dh0 = zc * NDW;  // this workgroup's dVᵀ / dKᵀ column blocks
  const int G = H / Hkv;
  const int GS = part != nullptr ? G : 1;
  const int gi = bhx % GS, bh = bhx / GS;
  const int b = bh / Hkv, hk = bh % Hkv;
  const int lane = threadIdx.x & 63, w = wave_id(), hh = lane >> 5;
  const int kg = w >> 1, role = w & 1;  // role 0: S, P, dV; role 1: dP, dS, dK
  const size_t RS = (size_t)(H + 2 * Hkv) * D;
  const size_t ORS = (size_t)H * D;
  const int kw0 = kb * BK + 32 * kg;
  const int key = kw0 + (lane & 31);
  const float c = scale * kLog2e;
  const float inv_keep = DROPOUT ? 1.f / (1.f - p_drop) : 1.f;

  const bf16* kbase = qkv + (size_t)b * T * RS + (size_t)(H + hk) * D;
  const bf16* vbase = qkv + (size_t)b * T * RS + (size_t)(H + Hkv + hk) * D;
  const bf16* obase = role == 0 ? kbase : vbase;
  uint4 of[NS];  // role 0: cK, role 1: V (B fragments of Kᵀ / Vᵀ: element j = X[key][16s + 8hh + j])
#pragma unroll
  for (int s = 0; s < NS; ++s)
    of[s] = key < T ? *reinterpret_cast<const uint4*>(obase + (size_t)key * RS + 16 * s + 8 * hh) : zero4();
  if (role == 0)
#pragma unroll
    for (int s = 0; s < NS; ++s) of[s] = scale_bf16x8(of[s], c);  // S = Q·(cK)ᵀ (attn_common.h)
#pragma unroll
  for (int s = 0; s < NS; ++s) launder(of[s]);
  f32x16 acc[NDW];  // role 0: dVᵀ, role 1: dKᵀ (column block dh: columns 32(dh0 + dh) ..)
#pragma unroll
  for (int dh = 0; dh < NDW; ++dh)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[dh][i] = 0.f;

  const int s_first = (kb * BK) / QS;
  const int nslices = (T + QS - 1) / QS;
  const int per_head = nslices - s_first;
  const int total = (GS == 1 ? G : 1) * per_head;
  auto head_of = [&](int it) { return hk * G + (GS == 1 ? it / per_head : gi); };

  auto dma = [&](int it) {  // role 0: Q slice (+ LSE), role 1: dO slice (+ δ); key groups take half the panels
    const int hq = head_of(it);
    const int qs0 = (s_first + it % per_head) * QS;
    const unsigned st = __builtin_amdgcn_readfirstlane(lds_addr_of(smem + (it & 1) * STAGE));
    constexpr int NPW = NP / 2;
    const int p0 = kg * NPW;
    if (role == 0)
      dma_rows<NPW>(qkv + (size_t)b * T * RS + (size_t)hq * D + 64 * p0, RS, qs0, T, st + p0 * QS * 128, lane);
    else
      dma_rows<NPW>(dout + (size_t)b * T * ORS + (size_t)hq * D + 64 * p0, ORS, qs0, T, st + TILE + p0 * QS * 128,
                    lane);
    if (kg == 0) {
      const float* sp = (role == 0 ? lse : delta) + ((size_t)b * H + hq) * T + min(qs0 + lane, T - 1);
      glds4(sp, st + 2 * TILE + 256 * role);
    }
  };

  if (total > 0) dma(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int it = 0; it < total; ++it) {
    if (it + 1 < total) dma(it + 1);
    const char* stg = smem + (it & 1) * STAGE;
    const char* Qt = stg;
    const char* Dt = stg + TILE;
    const float* lse_s = reinterpret_cast<const float*>(stg + 2 * TILE);
    const float* del_s = lse_s + 64;
    const int hq = head_of(it);
    const int qs0 = (s_first + it % per_head) * QS;
    const bool act = qs0 + QS - 1 >= kw0 && kw0 < T && qs0 < T;  // uniform over the key group
    const bool mask = kw0 + 31 > qs0 || qs0 + QS > T || kw0 + 32 > T;
    f32x16 sc;  // role 0: S (onto −LSE·log2 e), role 1: dP (onto −δ)
    if (act) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4_t cs = role == 0 ? *reinterpret_cast<const float4_t*>(&lse_s[8 * g + 4 * hh]) * (-kLog2e)
                                      : (DROPOUT ? float4_t{0.f, 0.f, 0.f, 0.f}
                                                 : -*reinterpret_cast<const float4_t*>(&del_s[8 * g + 4 * hh]));
#pragma unroll
        for (int k = 0; k < 4; ++k) sc[4 * g + k] = cs[k];
      }
      const char* At = role == 0 ? Qt : Dt;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        sc = mfma32(row_frag(panel(At, QS, s >> 2), 0, s & 3, lane), of[s], sc);
        if ((s & 3) == 3) __builtin_amdgcn_sched_barrier(0);
      }
      if (role == 0) {  // P (masked, before dropout) to the dP-wave; P with dropout for dV
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int i = 4 * g + k, q = qs0 + 8 * g + 4 * hh + k;
            float p = fexp2(sc[i]);
            if (mask) p = (key > q || q >= T || key >= T) ? 0.f : p;
            xp[(kg * 16 + i) * 64 + lane] = p;
            if constexpr (DROPOUT) p = dropout_keep(seed, b, hq, H, T, q, key, p_drop) ? p * inv_keep : 0.f;
            sc[i] = p;
          }
      }
    }
    __syncthreads();
    if (act) {
      if (role == 1) {  // dS = P ⊙ (dP − δ)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          float4_t dl = {0.f, 0.f, 0.f, 0.f};
          if constexpr (DROPOUT) dl = *reinterpret_cast<const float4_t*>(&del_s[8 * g + 4 * hh]);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int i = 4 * g + k;
            const float p = xp[(kg * 16 + i) * 64 + lane];
            if constexpr (DROPOUT) {
              const int q = qs0 + 8 * g + 4 * hh + k;
              const bool keep = dropout_keep(seed, b, hq, H, T, q, key, p_drop);
              sc[i] = p * ((keep ? sc[i] * inv_keep : 0.f) - dl[k]);
            } else {
              sc[i] = p * sc[i];
            }
          }
        }
      }
      // role 0: dVᵀ += dOᵀ·P, role 1: dKᵀ += Qᵀ·dS
      const char* Bt = (role == 0 ? Dt : Qt) + (dh0 >> 1) * QS * 128;
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const uint4 pf = acc_frag(sc, ss);
#pragma unroll
        for (int dh = 0; dh < NDW; ++dh) {
          acc[dh] = mfma32(tr_frag(panel(Bt, QS, dh >> 1), 16 * ss, 32 * (dh & 1), lane), pf, acc[dh]);
          if (dh & 1) __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  const float mul = role == 0 ? 1.f : scale;
  if (key < T && part != nullptr) {  // fp32 partials of this query head: [gi][b·T + key][K | V][hk·D + d]
    const int Bn = nbhx / (Hkv * GS);
    float* prow = part + ((size_t)gi * Bn * T + (size_t)b * T + key) * (2 * Hkv * D) + (size_t)hk * D +
                  (role == 0 ? (size_t)Hkv * D : 0);
#pragma unroll
    for (int dh = 0; dh < NDW; ++dh)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<float4*>(prow + 32 * (dh0 + dh) + 8 * g + 4 * hh) =
            float4{acc[dh][4 * g] * mul, acc[dh][4 * g + 1] * mul, acc[dh][4 * g + 2] * mul, acc[dh][4 * g + 3] * mul};
  } else if (key < T) {
    bf16* row = dqkv + ((size_t)b * T + key) * RS + (size_t)(role == 0 ? H + Hkv + hk : H + hk) * D;
#pragma unroll
    for (int dh = 0; dh < NDW; ++dh)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        store4(row + 32 * (dh0 + dh) + 8 * g + 4 * hh, acc[dh][4 * g] * mul, acc[dh][4 * g + 1] * mul,
               acc[dh][4 * g + 2] * mul, acc[dh][4 * g + 3] * mul);
  }
}

// Σ over the G query-head partials -> the K | V columns of dqkv (bf16). One thread per 8 columns.
__global__ void __launch_bounds__(256) fa_gen_kv_reduce(const float* __restrict__ part, bf16* __restrict__ dqkv,
                                                        int64_t rows, int W2, int G, int64_t RS, int64_t col0) {
  const int64_t n8 = rows * (W2 / 8);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / (W2 / 8), c = 8 * (i - r * (W2 / 8));
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int g = 0; g < G; ++g) {
      const float* src = part + ((size_t)g * rows + r) * W2 + c;
      const float4 a = *reinterpret_cast<const float4*>(src), bq = *reinterpret_cast<const float4*>(src + 4);
      acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
      acc[4] += bq.x; acc[5] += bq.y; acc[6] += bq.z; acc[7] += bq.w;
    }
    bf16* dst = dqkv + r * RS + col0 + c;
    store4(dst, acc[0], acc[1], acc[2], acc[3]);
    store4(dst + 4, acc[4], acc[5], acc[6], acc[7]);
  }
}

// Split-block partials -> the final rows. FWD: O = Σ_p o_p·2^(m_p − m) / Σ_p l_p·2^(m_p − m)
// (bf16, head-merged) and the LSE; otherwise dQ = Σ_p dQ_p (bf16, the Q columns of dqkv).
// ws: [2][nbh][nsr][D] fp32 (+ FWD: [2][nbh][nsr] (m, l)); split row rr of head bh is query
// row r0 + rr. One thread per 8 columns.
template <bool FWD>
__global__ void __launch_bounds__(256) fa_gen_combine(const float* __restrict__ ws, bf16* __restrict__ dst,
                                                      float* __restrict__ lse, int nbh, int nsr, int r0, int T, int H,
                                                      int D, int64_t RS) {
  const int c8 = D / 8;
  const int64_t n8 = (int64_t)nbh * nsr * c8, plane = (int64_t)nbh * nsr;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / c8;
    const int c = 8 * (int)(i - row * c8);
    const int bh = (int)(row / nsr), rr = (int)(row - (int64_t)bh * nsr), q = r0 + rr;
    if (q >= T) continue;
    const int b = bh / H, h = bh - b * H;
    const float* p0 = ws + row * D + c;
    const float* p1 = p0 + plane * D;
    const float4 a0 = *reinterpret_cast<const float4*>(p0), a1 = *reinterpret_cast<const float4*>(p0 + 4);
    const float4 b0 = *reinterpret_cast<const float4*>(p1), b1 = *reinterpret_cast<const float4*>(p1 + 4);
    float w0 = 1.f, w1 = 1.f;
    bf16* o;
    if constexpr (FWD) {
      const float2 ml0 = reinterpret_cast<const float2*>(ws + 2 * plane * D)[row];
      const float2 ml1 = reinterpret_cast<const float2*>(ws + 2 * plane * D)[plane + row];
      const float m = fmaxf(ml0.x, ml1.x);
      const float e0 = fexp2(ml0.x - m), e1 = fexp2(ml1.x - m);
      const float l = ml0.y * e0 + ml1.y * e1;
      const float inv = l > 0.f ? 1.f / l : 0.f;
      w0 = e0 * inv;
      w1 = e1 * inv;
      if (c == 0) lse[(size_t)bh * T + q] = (m + log2f(l)) * kLn2;
      o = dst + (((size_t)b * T + q) * H + h) * D + c;
    } else {
      o = dst + ((size_t)b * T + q) * RS + (size_t)h * D + c;
    }
    store4(o, a0.x * w0 + b0.x * w1, a0.y * w0 + b0.y * w1, a0.z * w0 + b0.z * w1, a0.w * w0 + b0.w * w1);
    store4(o + 4, a1.x * w0 + b1.x * w1, a1.y * w0 + b1.y * w1, a1.z * w0 + b1.z * w1, a1.w * w0 + b1.w * w1);
  }
}

// ------------------------------------------------------------------------------------------
// dQ: grid (ceil(T/64) query blocks, heaviest first, B*H); forward-shaped: a wave keeps 32
// query rows' Q, dO, LSE, δ and dQᵀ in registers while sweeping 32-key K/V tiles.
template <int D> constexpr int dq_waves() { return 2 * dq_dsplit<D>(); }

template <int D, bool DROPOUT>
__global__ void __launch_bounds__(64 * dq_waves<D>(), (D >= 512 ? 1 : 2))
    fa_gen_bwd_dq_kernel(const bf16* __restrict__ qkv, const bf16* __restrict__ dout, const float* __restrict__ lse,
                         const float* __restrict__ delta, bf16* __restrict__ dqkv, int T, int H, int Hkv, float scale,
                         float p_drop, uint64_t seed, const WorkList wl, float* __restrict__ ws) {
  constexpr int NP = D / 64, NS = D / 16, ND = D / 32, ZS = dq_dsplit<D>(), NWQ = dq_waves<D>();
  constexpr int BM = 64, BN = 32, TILE = BN * 128 * NP;
  constexpr int NSH = NS / ZS;
  // [stage][K | V] tiles, then (ZS > 1) the partial S / dP exchange image [wave][4][64] float4 —
  // 160 KB at D = 512 (S and dP go through it one after the other)
  constexpr int XB = ZS > 1 ? NWQ * 16 * 64 * 4 : 16;
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE + XB];
  float* xb = reinterpret_cast<float*>(smem + 4 * TILE);
  const int nqb = (T + BM - 1) / BM;
  int item, vh, qb, part;
  item_head(wl.n, item, vh);
  item_block(wl, nqb, item, qb, part);
  const int nbh = gridDim.x / wl.n;
  const int bh = vh;
  const int b = bh / H, h = bh % H, hk = h / (H / Hkv);
  const int lane = threadIdx.x & 63, w = wave_id(), hh = lane >> 5;
  const int rg = w / ZS, dz = w % ZS;  // row group (32 query rows), part of D (ZS = 4: a quarter)
  const int sq0 = dz * NSH;
  const size_t RS = (size_t)(H + 2 * Hkv) * D;
  const size_t ORS = (size_t)H * D;
  const bf16* kbase = qkv + (size_t)b * T * RS + (size_t)(H + hk) * D;
  const bf16* vbase = qkv + (size_t)b * T * RS + (size_t)(H + Hkv + hk) * D;
  const int q0 = qb * BM + 32 * rg;
  const int qrow = q0 + (lane & 31);
  const bool qok = qrow < T;
  const float c = scale * kLog2e;
  const float inv_keep = DROPOUT ? 1.f / (1.f - p_drop) : 1.f;

  constexpr int NDQ = ND / ZS;  // dQᵀ column blocks of 32 owned here (D = 512: a quarter)
  const int dq0 = dz * NDQ;
  uint4 qf[NSH], dof[NSH];
#pragma unroll
  for (int s = 0; s < NSH; ++s) {
    qf[s] = qok ? *reinterpret_cast<const uint4*>(qkv + (size_t)b * T * RS + (size_t)h * D + (size_t)qrow * RS +
                                                  16 * (sq0 + s) + 8 * hh)
                : zero4();
    dof[s] = qok ? *reinterpret_cast<const uint4*>(dout + (size_t)b * T * ORS + (size_t)h * D + (size_t)qrow * ORS +
                                                   16 * (sq0 + s) + 8 * hh)
                 : zero4();
  }
  const size_t rr = ((size_t)b * H + h) * T + qrow;
  float l2 = qok ? lse[rr] * kLog2e : 0.f;
  float dl = qok ? delta[rr] : 0.f;
#pragma unroll
  for (int s = 0; s < NSH; ++s) {
    qf[s] = scale_bf16x8(qf[s], c);  // S = (cQ)·Kᵀ (attn_common.h); dQ uses K, not Q
    launder(qf[s]);
    launder(dof[s]);
  }
  asm volatile("" : "+v"(l2), "+v"(dl));

  const int kend = min(T, qb * BM + BM);
  int j0, j1;
  part_tiles(part, (kend + BN - 1) / BN, j0, j1);
  f32x16 dq[NDQ];
#pragma unroll
  for (int dh = 0; dh < NDQ; ++dh)
#pragma unroll
    for (int i = 0; i < 16; ++i) dq[dh][i] = 0.f;

  auto dma = [&](int j) {  // even waves: K tile, odd waves: V tile (NWQ = 8: a quarter of the panels each)
    constexpr int NPW = NP * 2 / NWQ;
    const int role = w & 1, p0 = (w >> 1) * NPW;
    const unsigned dst = __builtin_amdgcn_readfirstlane(lds_addr_of(smem + ((j & 1) * 2 + role) * TILE)) +
                         p0 * BN * 128;
    dma_rows<NPW>((role == 0 ? kbase : vbase) + 64 * p0, RS, j * BN, T, dst, lane);
  };
  if (j0 < j1) dma(j0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int j = j0; j < j1; ++j) {
    const int kt0 = j * BN;
    if (j + 1 < j1) dma(j + 1);
    const char* Kt = smem + (j & 1) * 2 * TILE;
    const char* Vt = Kt + TILE;
    const bool act = kt0 <= q0 + 31 && q0 < T;  // uniform over a wave pair (same rows)
    f32x16 st, dp;
#pragma unroll
    for (int i = 0; i < 16; ++i) {  // (ZS > 1: the row constants are added after the exchange)
      st[i] = ZS > 1 ? 0.f : -l2;  // S accumulates onto −LSE·log2(e): P = exp2(S)
      dp[i] = DROPOUT || ZS > 1 ? 0.f : -dl;
    }
    if (act) {
      const char* Kh = Kt + (sq0 >> 2) * BN * 128;  // this wave's half of D (compile-time offsets below)
      const char* Vh = Vt + (sq0 >> 2) * BN * 128;
#pragma unroll
      for (int s = 0; s < NSH; ++s) {
        st = mfma32(row_frag(panel(Kh, BN, s >> 2), 0, s & 3, lane), qf[s], st);
        dp = mfma32(row_frag(panel(Vh, BN, s >> 2), 0, s & 3, lane), dof[s], dp);
        if (s & 1) d_fence<D>();
      }
    }
    if constexpr (ZS > 1) {  // full S, then full dP (Σ of the row group's parts, in part order)
      float4_t* x4 = reinterpret_cast<float4_t*>(xb) + lane;
      dsplit_sum<ZS>(st, x4, w, rg, act);
      __syncthreads();  // every S read done before the image takes dP
      dsplit_sum<ZS>(dp, x4, w, rg, act);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        st[i] -= l2;
        if constexpr (!DROPOUT) dp[i] -= dl;
      }
    }
    if (act) {
      auto grads = [&](auto mask_tag) {
        constexpr bool MASK = decltype(mask_tag)::value;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int k = kt0 + acc_row(i, lane);
          float p = fexp2(st[i]);
          if constexpr (MASK) p = (k > qrow || k >= T || !qok) ? 0.f : p;
          if constexpr (DROPOUT) {
            const bool keep = dropout_keep(seed, b, h, H, T, qrow, k, p_drop);
            st[i] = p * ((keep ? dp[i] * inv_keep : 0.f) - dl);
          } else {
            st[i] = p * dp[i];
          }
        }
      };
      if (kt0 + BN - 1 > q0 || kt0 + BN > T || q0 + 32 > T)
        grads(std::true_type{});
      else
        grads(std::false_type{});
      const char* Kq = Kt + (dq0 >> 1) * BN * 128;  // dq0 even (or 0)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const uint4 sf = acc_frag(st, ss);
#pragma unroll
        for (int j = 0; j < NDQ; ++j) {
          dq[j] = mfma32(tr_frag(panel(Kq, BN, j >> 1), 16 * ss, 32 * (j & 1), lane), sf, dq[j]);
          if (j & 1) d_fence<D>();
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (qok && part != 0) {  // half of a split block: fp32 partial dQ for fa_gen_combine
    const size_t nsr = (size_t)(nqb - wl.split0) * BM;
    float* prow = ws + (((size_t)(part - 1) * nbh + bh) * nsr + (qrow - wl.split0 * BM)) * D;
#pragma unroll
    for (int j = 0; j < NDQ; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<float4*>(prow + 32 * (dq0 + j) + 8 * g + 4 * hh) =
            float4{dq[j][4 * g] * scale, dq[j][4 * g + 1] * scale, dq[j][4 * g + 2] * scale,
                   dq[j][4 * g + 3] * scale};
  } else if (qok) {
    bf16* dqrow = dqkv + ((size_t)b * T + qrow) * RS + (size_t)h * D;
#pragma unroll
    for (int j = 0; j < NDQ; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        store4(dqrow + 32 * (dq0 + j) + 8 * g + 4 * hh, dq[j][4 * g] * scale, dq[j][4 * g + 1] * scale,
               dq[j][4 * g + 2] * scale, dq[j][4 * g + 3] * scale);
  }
}

}  // namespace penroz

// ============================================================================ host side
using namespace penroz;

#define FA_GEN_DISPATCH(D, DROP, ...)                                                         \
  if ((D) == 128 && (DROP)) { constexpr int DD = 128; constexpr bool DR = true; __VA_ARGS__; }   \
  else if ((D) == 128) { constexpr int DD = 128; constexpr bool DR = false; __VA_ARGS__; }       \
  else if ((D) == 256 && (DROP)) { constexpr int DD = 256; constexpr bool DR = true; __VA_ARGS__; } \
  else if ((D) == 256) { constexpr int DD = 256; constexpr bool DR = false; __VA_ARGS__; }       \
  else if ((D) == 512 && (DROP)) { constexpr int DD = 512; constexpr bool DR = true; __VA_ARGS__; } \
  else if ((D) == 512) { constexpr int DD = 512; constexpr bool DR = false; __VA_ARGS__; }       \
  else TORCH_CHECK(false, "generic flash attention supports head_dim 128, 256 and 512, got ", (D));

namespace {

// resident workgroups of `kernel` on the whole chip (CUs × occupancy), cached per kernel
int chip_slots(const void* kernel, int block) {
  static std::mutex mu;
  static std::map<const void*, int> cache;
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(kernel);
  if (it != cache.end()) return it->second;
  int dev = 0, ncu = 256, nb = 1;
  hipDeviceProp_t prop;
  if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess) ncu = prop.multiProcessorCount;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, block, 0) != hipSuccess || nb < 1) nb = 1;
  return cache[kernel] = nb * ncu;
}

// PENROZ_ATTN_KV_SPLIT: 0 = never split, 2 = split every block but the first (tests), else auto
int split_mode() {
  const char* e = std::getenv("PENROZ_ATTN_KV_SPLIT");
  return e && *e ? std::atoi(e) : 1;
}

// Work list for nblk causal blocks of BM query rows swept in BN-key tiles, over nvh virtual heads
// on `slots` resident workgroups. Auto: list-schedule the sorted items per XCD (each XCD runs its
// ceil(nvh / 8) heads on slots / 8 workgroup slots, a freed slot takes the next item) for every
// split0, and keep the one whose makespan·tile_us plus the combine pass (its fp32 traffic at
// ~4.5 TB/s plus a launch) is smallest.
WorkList attn_plan(int nblk, int nvh, int slots, int BM, int BN, int T, int D, double tile_us) {
  const int mode = split_mode();
  using Key = std::tuple<int, int, int, int, int, int, int, int, long long>;
  static std::mutex mu;
  static std::map<Key, WorkList> cache;
  const Key key{nblk, nvh, slots, BM, BN, T, D, mode, (long long)(tile_us * 1e3)};
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  auto ntiles = [&](int qb) { return (std::min(T, (qb + 1) * BM) + BN - 1) / BN; };
  auto build = [&](int s0, WorkList* wl) -> double {  // returns the makespan in tiles
    std::vector<std::pair<int, int>> items;  // (tiles, entry)
    for (int qb = nblk - 1; qb >= 0; --qb) {
      const int n = ntiles(qb);
      if (qb >= s0) {
        items.push_back({n - n / 2, qb | 2 << 16});
        items.push_back({n / 2, qb | 1 << 16});
      } else {
        items.push_back({n, qb});
      }
    }
    std::stable_sort(items.begin(), items.end(), [](auto& a, auto& b) { return a.first > b.first; });
    if (wl) {
      wl->n = (int)items.size();
      wl->split0 = s0;
      for (size_t i = 0; i < items.size(); ++i) wl->it[i] = items[i].second;
    }
    const int hx = (nvh + 7) / 8, sx = std::max(1, slots / 8);
    std::priority_queue<long long, std::vector<long long>, std::greater<long long>> free_at;
    for (int i = 0; i < sx; ++i) free_at.push(0);
    long long span = 0;
    for (auto& [n, e] : items)
      for (int hh = 0; hh < hx; ++hh) {
        const long long t = free_at.top() + n;
        free_at.pop();
        free_at.push(t);
        span = std::max(span, t);
      }
    return (double)span;
  };
  WorkList wl;
  wl.n = nblk;
  wl.split0 = nblk;
  const bool can_split = mode != 0 && nblk >= 2 && 2 * nblk - 1 <= kMaxItems;
  if (can_split && mode == 2) {
    build(1, &wl);
  } else if (can_split && (long long)nblk * nvh <= 2LL * slots) {
    double best = build(nblk, nullptr) * tile_us;
    int best_s = nblk;
    for (int s0 = nblk - 1; s0 >= 1; --s0) {
      const double rows = (double)(nblk - s0) * BM * nvh;
      const double comb_us = rows * D * 4.0 * 4.0 / 4.5e6 + 4.0;
      const double c = build(s0, nullptr) * tile_us + comb_us;
      if (c < best) best = c, best_s = s0;
    }
    if (best_s < nblk) build(best_s, &wl);
  }
  return cache[key] = wl;
}

void launch_combine(bool fwd, const float* ws, bf16* dst, float* lse, int nbh, int nsr, int r0, int T, int H, int D,
                    int64_t RS, hipStream_t stream) {
  const int64_t n8 = (int64_t)nbh * nsr * (D / 8);
  const dim3 g((unsigned)std::min<int64_t>((n8 + 255) / 256, 8192));
  if (fwd)
    hipLaunchKernelGGL(fa_gen_combine<true>, g, dim3(256), 0, stream, ws, dst, lse, nbh, nsr, r0, T, H, D, RS);
  else
    hipLaunchKernelGGL(fa_gen_combine<false>, g, dim3(256), 0, stream, ws, dst, lse, nbh, nsr, r0, T, H, D, RS);
}

}  // namespace

// the causal work list attn_plan builds (host only, for tests): {items, split0, entries...}
std::vector<int64_t> attn_work_plan(int64_t nblk, int64_t nvh, int64_t slots, int64_t BM, int64_t BN, int64_t T,
                                    int64_t D, double tile_us) {
  const WorkList wl = attn_plan((int)nblk, (int)nvh, (int)slots, (int)BM, (int)BN, (int)T, (int)D, tile_us);
  std::vector<int64_t> r{wl.n, wl.split0};
  if (wl.split0 < nblk)
    for (int i = 0; i < wl.n; ++i) r.push_back(wl.it[i]);
  return r;
}

void flash_attn_gen_fwd(torch::Tensor qkv, torch::Tensor out, torch::Tensor lse, int64_t H, int64_t Hkv, int64_t D,
                        double scale, double p_drop, int64_t seed) {
  TORCH_CHECK(qkv.is_cuda() && qkv.is_contiguous() && qkv.dim() == 3 && qkv.scalar_type() == torch::kBFloat16,
              "qkv must be a contiguous bf16 [B, T, W] GPU tensor");
  TORCH_CHECK(H > 0 && Hkv > 0 && H % Hkv == 0 && qkv.size(2) == (H + 2 * Hkv) * D, "qkv width must be (H+2Hkv)*D");
  const int B = qkv.size(0), T = qkv.size(1);
  TORCH_CHECK(out.is_contiguous() && out.scalar_type() == torch::kBFloat16 && out.numel() == (int64_t)B * T * H * D);
  TORCH_CHECK(lse.is_contiguous() && lse.scalar_type() == torch::kFloat32 && lse.numel() == (int64_t)B * H * T);
  if (B == 0 || T == 0) return;
  auto stream = at::hip::getCurrentHIPStream();
  const bf16* q = reinterpret_cast<const bf16*>(qkv.data_ptr());
  bf16* o = reinterpret_cast<bf16*>(out.data_ptr());
  FA_GEN_DISPATCH(D, p_drop > 0.0, {
    constexpr int NW = fwd_waves<DD>(), BM = 32 * NW / fwd_dsplit<DD>();
    const int nqb = (T + BM - 1) / BM, nvh = B * (int)H;
    // measured: ~2.7 µs per 32-key tile for a 128-row, D = 256 block (Gemma-3 1B step)
    const double tile_us = 2.7 * (BM / 128.0) * DD / 256.0;
    const auto kern = fa_gen_fwd_kernel<DD, DR>;
    const WorkList wl = attn_plan(nqb, nvh, chip_slots((const void*)kern, 64 * NW), BM, 32, T, DD, tile_us);
    torch::Tensor ws;
    const int nsr = (nqb - wl.split0) * BM;
    if (wl.split0 < nqb) ws = torch::empty({2 * (int64_t)B * H * nsr * (DD + 2)}, lse.options());
    float* wsp = wl.split0 < nqb ? ws.data_ptr<float>() : nullptr;
    hipLaunchKernelGGL(kern, dim3(wl.n * nvh), dim3(64 * NW), 0, stream, q, o, lse.data_ptr<float>(), T, (int)H,
                       (int)Hkv, (float)scale, (float)p_drop, (uint64_t)seed, wl, wsp);
    if (wsp)
      launch_combine(true, wsp, o, lse.data_ptr<float>(), B * (int)H, nsr, wl.split0 * BM, T, (int)H, DD, 0, stream);
  })
}

void flash_attn_gen_bwd(torch::Tensor dout, torch::Tensor qkv, torch::Tensor out, torch::Tensor lse,
                        torch::Tensor dqkv, int64_t H, int64_t Hkv, int64_t D, double scale, double p_drop,
                        int64_t seed) {
  TORCH_CHECK(qkv.is_cuda() && qkv.is_contiguous() && qkv.dim() == 3 && qkv.scalar_type() == torch::kBFloat16);
  TORCH_CHECK(H > 0 && Hkv > 0 && H % Hkv == 0 && qkv.size(2) == (H + 2 * Hkv) * D, "qkv width must be (H+2Hkv)*D");
  const int B = qkv.size(0), T = qkv.size(1);
  TORCH_CHECK(dout.is_contiguous() && dout.scalar_type() == torch::kBFloat16 && dout.numel() == (int64_t)B * T * H * D);
  TORCH_CHECK(out.is_contiguous() && out.numel() == dout.numel() && lse.numel() == (int64_t)B * H * T);
  TORCH_CHECK(dqkv.is_contiguous() && dqkv.scalar_type() == torch::kBFloat16 && dqkv.numel() == qkv.numel());
  if (B == 0 || T == 0) return;
  auto delta = torch::empty({B, H, T}, qkv.options().dtype(torch::kFloat32));
  auto stream = at::hip::getCurrentHIPStream();
  const int rows = B * T * H;
  const bf16* q = reinterpret_cast<const bf16*>(qkv.data_ptr());
  const bf16* d = reinterpret_cast<const bf16*>(dout.data_ptr());
  bf16* g = reinterpret_cast<bf16*>(dqkv.data_ptr());
  // GQA with few KV workgroups: split the dK / dV sweep over the query heads of each group
  // (fp32 partials + one reduction pass) so the grid covers the chip
  const int G = (int)(H / Hkv), nkb = (T + 63) / 64;
  const bool split = G > 1 && (int64_t)B * Hkv * nkb < 1024;
  torch::Tensor part;
  if (split) part = torch::empty({(int64_t)G * B * T, 2 * Hkv * D}, qkv.options().dtype(torch::kFloat32));
  // 1-D grids: items (key / query blocks) × the column parts of D (dK / dV: 2 at D = 256, 4 at
  // 512; dQ: 2 at 512) × heads
  const int64_t nkv = (int64_t)nkb * B * Hkv * (split ? G : 1) * (D == 512 ? 2 : 1);  // kv_role_parts

  FA_GEN_DISPATCH(D, p_drop > 0.0, {
    hipLaunchKernelGGL((fa_gen_bwd_pre_kernel<DD>), dim3(((int64_t)rows * (DD / 8) + 255) / 256), dim3(256), 0,
                       stream, d, reinterpret_cast<const bf16*>(out.data_ptr()), delta.data_ptr<float>(), B, T,
                       (int)H);
    hipLaunchKernelGGL((fa_roles_bwd_dkdv_kernel<DD, DR>), dim3((unsigned)nkv), dim3(256), 0, stream, q, d,
                       lse.data_ptr<float>(), delta.data_ptr<float>(), g, split ? part.data_ptr<float>() : nullptr, T,
                       (int)H, (int)Hkv, (float)scale, (float)p_drop, (uint64_t)seed);
    if (split) {
      const int64_t n8 = (int64_t)B * T * (2 * Hkv * DD / 8);
      hipLaunchKernelGGL(fa_gen_kv_reduce, dim3((unsigned)std::min<int64_t>((n8 + 255) / 256, 4096)), dim3(256), 0,
                         stream, part.data_ptr<float>(), g, (int64_t)B * T, (int)(2 * Hkv * DD), G,
                         (int64_t)(H + 2 * Hkv) * DD, (int64_t)H * DD);
    }
    constexpr int NWQ = dq_waves<DD>();
    const int nqb = (T + 63) / 64, nvh = B * (int)H;
    // measured: ~2.9 µs per 32-key tile for a 64-row, D = 256 block (Gemma-3 1B step)
    const double tile_us = 2.9 * DD / 256.0;
    const auto kq = fa_gen_bwd_dq_kernel<DD, DR>;
    const WorkList wl = attn_plan(nqb, nvh, chip_slots((const void*)kq, 64 * NWQ), 64, 32, T, DD, tile_us);
    torch::Tensor ws;
    const int nsr = (nqb - wl.split0) * 64;
    if (wl.split0 < nqb) ws = torch::empty({2 * (int64_t)B * H * nsr * DD}, lse.options());
    float* wsp = wl.split0 < nqb ? ws.data_ptr<float>() : nullptr;
    hipLaunchKernelGGL(kq, dim3(wl.n * nvh), dim3(64 * NWQ), 0, stream, q, d, lse.data_ptr<float>(),
                       delta.data_ptr<float>(), g, T, (int)H, (int)Hkv, (float)scale, (float)p_drop, (uint64_t)seed,
                       wl, wsp);
    if (wsp)
      launch_combine(false, wsp, g, nullptr, B * (int)H, nsr, wl.split0 * 64, T, (int)H, DD,
                     (int64_t)(H + 2 * Hkv) * DD, stream);
  })
}
