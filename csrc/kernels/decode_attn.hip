// KV-cache attention for incremental decoding (memory-bound: every cached K/V byte is read
// once per step).
//
// Work item = (batch b, KV head g, query row tq, split s). One 256-thread workgroup owns all
// H/Hkv query heads that share KV head g (GQA by index math — the cache is never expanded),
// so each K/V row is loaded once for the whole group. Keys go in chunks of up to 256 (one key
// per thread, or 1/2, 1/4 of one for wide rows), so a whole chunk's K and V reads are in
// flight together — a decode step's cache is short (S ~ 100s) and the kernel is latency-bound:
//   scores : thread = key; its K row is read as 16-B vectors and dotted with the group's query
//            vectors (LDS, fp32); V row pieces go raw to an XOR-swizzled LDS tile;
//   softmax: online (m, l) per query head across chunks, block max/sum through LDS, causal
//            mask by absolute position (query tq sits at q_offset + tq);
//   PV     : thread = 2 output columns × every NG-th key of the chunk, from LDS.
// int8 caches (TurboQuant) carry per-token fp32 scales that are folded into the score and
// the P·V weight, so the int8 cache is never dequantised to memory.
// The key groups merge through LDS; with several splits the partial (m, l, O) go to a workspace
// and the last split workgroup of the item to arrive combines them (or, without arrival
// counters, a second kernel). Enough splits are used to put ≥ 512 workgroups in
// flight (256 CUs) even at batch 1.
#include "common.h"
#include <cstdlib>
#include <type_traits>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

namespace penroz {

constexpr int kMaxGroup = 16;
constexpr int kMaxMergeSplits = 16;
constexpr int64_t kMergeMaxKeys = 8192;

template <typename TK> struct KRow;
template <> struct KRow<bf16> {
  __device__ __forceinline__ static float at(const bf16* p, int d) { return bf2f(p[d]); }
};
template <> struct KRow<__half> {
  __device__ __forceinline__ static float at(const __half* p, int d) { return __half2float(p[d]); }
};
template <> struct KRow<float> {
  __device__ __forceinline__ static float at(const float* p, int d) { return p[d]; }
};
template <> struct KRow<int8_t> {
  __device__ __forceinline__ static float at(const int8_t* p, int d) { return (float)p[d]; }
};

// 8 consecutive cache elements -> fp32 (one 16-B load for bf16/fp16, 8 B for int8, 32 B for fp32)
template <typename TK> struct Row8;
template <> struct Row8<bf16> {
  __device__ __forceinline__ static void load(const bf16* p, float (&v)[8]) { Vec8<bf16>::load(p, v); }
};
template <> struct Row8<__half> {
  __device__ __forceinline__ static void load(const __half* p, float (&v)[8]) { Vec8<__half>::load(p, v); }
};
template <> struct Row8<float> {
  __device__ __forceinline__ static void load(const float* p, float (&v)[8]) { Vec8<float>::load(p, v); }
};
template <> struct Row8<int8_t> {
  __device__ __forceinline__ static void load(const int8_t* p, float (&v)[8]) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = (float)(int8_t)((u.x >> (8 * i)) & 0xff);
      v[4 + i] = (float)(int8_t)((u.y >> (8 * i)) & 0xff);
    }
  }
};

// raw 16-B pieces live in ext-vector registers (HIP's uint4 struct defeats register promotion
// of an array that is carried across the chunk loop: it went to scratch)
typedef uint32_t dec_u32x4 __attribute__((ext_vector_type(4)));

// 16 raw cache bytes -> fp32 (8 bf16/fp16, 4 fp32 or 16 int8 values)
template <typename TK> struct Piece {
  static constexpr int N = 16 / (int)sizeof(TK);
  __device__ __forceinline__ static void cvt(const dec_u32x4 u, float (&v)[N]) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (std::is_same<TK, bf16>::value) {
        v[2 * i] = __uint_as_float(w[i] << 16);
        v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
      } else if constexpr (std::is_same<TK, __half>::value) {
        v[2 * i] = __half2float(__ushort_as_half((unsigned short)(w[i] & 0xffff)));
        v[2 * i + 1] = __half2float(__ushort_as_half((unsigned short)(w[i] >> 16)));
      } else if constexpr (std::is_same<TK, float>::value) {
        v[i] = __uint_as_float(w[i]);
      } else {
#pragma unroll
        for (int b = 0; b < 4; ++b) v[4 * i + b] = (float)(int8_t)((w[i] >> (8 * b)) & 0xff);
      }
    }
  }
};

// GC: the exact query-group size H/Hkv (1, 4, 8: branch-free loops), or 0 = any size <= 16
template <int D, int GC, typename TQ, typename TK>
__global__ void __launch_bounds__(256) decode_kernel(const TQ* __restrict__ q, const TK* __restrict__ kc,
                                                     const TK* __restrict__ vc, const float* __restrict__ ks,
                                                     const float* __restrict__ vs, TQ* __restrict__ out,
                                                     float* __restrict__ ws_o, float* __restrict__ ws_ml, int B,
                                                     int Tq, int H, int Hkv, int cap, int S, int q_offset,
                                                     int splits, float scale, const int64_t* __restrict__ S_dev,
                                                     int64_t q_rs, const TQ* __restrict__ k_new,
                                                     const TQ* __restrict__ v_new, int64_t kv_rs,
                                                     int* __restrict__ cnt, int min_keys) {
  constexpr int GMAX = GC ? GC : kMaxGroup;
  constexpr int RB = D * (int)sizeof(TK);                 // cache row bytes
  constexpr int KC = RB * 256 <= 32768 ? 256 : 32768 / RB;  // keys per chunk (V chunk <= 32 KB of LDS)
  constexpr int TPK = 256 / KC;                           // threads per key in the score phase
  constexpr int CR = RB / 16;                             // 16-B pieces per row
  constexpr int CPT = CR / TPK;                           // 16-B pieces of K (and of V) per thread
  constexpr int PN = Piece<TK>::N;                        // values per piece
  constexpr int SW = (CR < 8 ? CR : 8) - 1;               // LDS row swizzle mask (pieces)
  constexpr int NP = D / 2, NG = 256 / NP;                // P·V: column pairs × key groups
  constexpr int VBUF = KC * RB > NG * GMAX * D * 4 ? KC * RB : NG * GMAX * D * 4;
  constexpr int QPT = (GMAX * D + 255) / 256;             // query values staged per thread
  static_assert(CPT >= 1 && NG * NP == 256, "decode tiling");

  const int G = GC ? GC : H / Hkv;
  int wid_lin = blockIdx.x;
  const int split = wid_lin % splits;
  wid_lin /= splits;
  const int tq = wid_lin % Tq;
  wid_lin /= Tq;
  const int g = wid_lin % Hkv;
  const int b = wid_lin / Hkv;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;

  __shared__ __attribute__((aligned(16))) char vbuf[VBUF];  // V chunk, later the P·V partials
  __shared__ float qs[GMAX][D];
  __shared__ float pl[GMAX][KC];
  __shared__ float red_m[4][GMAX], red_l[4][GMAX];
  __shared__ float fin[GMAX][2];

  // the query group's reads go out first (the LDS write below then waits for them only)
  float qv[QPT];
#pragma unroll
  for (int r = 0; r < QPT; ++r) {
    const int i = t + 256 * r;
    qv[r] = i < G * D ? to_f(q[((size_t)b * Tq + tq) * q_rs + (size_t)(g * G + i / D) * D + i % D]) : 0.f;
  }
  if (S_dev != nullptr) {  // graph-replayed decode: the cache length lives on the device
    S = (int)min<int64_t>(*S_dev, (int64_t)cap);
    q_offset = S - Tq;
  }
  const int kend_causal = min(S, q_offset + tq + 1);
  // With the in-launch merge (cnt) the grid is sized for the capacity, but only the splits the
  // actual context needs (>= min_keys keys each) run: a short context is one workgroup writing the
  // output directly, the other split workgroups of the item leave at once (every workgroup of the
  // item derives the same count from the device-side length).
  const int nsplit = cnt != nullptr ? max(1, min(splits, (kend_causal + min_keys - 1) / min_keys)) : splits;
  if (split >= nsplit) return;
  const int per_split = (kend_causal + nsplit - 1) / nsplit;
  const int k0 = split * per_split, k1 = min(kend_causal, k0 + per_split);
  const size_t head_base = ((size_t)b * Hkv + g) * cap;
  const int kk = t / TPK, part = t % TPK;     // score phase: key kk of the chunk, pieces part*CPT..
  const int kg = t / NP, d0 = 2 * (t % NP);   // P·V phase: columns d0, d0+1 over keys kg, kg+NG, ..

  // one key (or 1/TPK of it) per thread: a whole chunk's K and V reads are in flight at once
  // (kept raw in registers, converted at use), and the next chunk's are issued before this
  // chunk's P·V. V goes raw to LDS (16-B pieces XOR-swizzled by row: conflict-free both ways).
  dec_u32x4 kr[CPT], vr[CPT];
  float ksc = 1.f, vsc = 1.f;
  // Fused append (k_new given, Tq == 1): the newest key S-1 is read from this step's QKV rows
  // instead of the cache, and the thread(s) holding it write it into cache slot S-1 (int8 caches:
  // quantised per token exactly like kv_append) — one kernel less per layer and step.
  constexpr bool SAME = std::is_same<TQ, TK>::value;
  const size_t new_off = (size_t)b * kv_rs + (size_t)g * D;
  auto load_chunk = [&](int c0) {
    const int key = c0 + kk;
    const size_t row = head_base + (key < k1 ? key : c0);
    const bool fresh = SAME && k_new != nullptr && key == S - 1;  // pointer select, no branch
    const char* ksrc = reinterpret_cast<const char*>(fresh ? reinterpret_cast<const TK*>(k_new) + new_off : kc + row * D) +
                       part * CPT * 16;
    const char* vsrc = reinterpret_cast<const char*>(fresh ? reinterpret_cast<const TK*>(v_new) + new_off : vc + row * D) +
                       part * CPT * 16;
#pragma unroll
    for (int c = 0; c < CPT; ++c) kr[c] = *reinterpret_cast<const dec_u32x4*>(ksrc + 16 * c);
#pragma unroll
    for (int c = 0; c < CPT; ++c) vr[c] = *reinterpret_cast<const dec_u32x4*>(vsrc + 16 * c);
    if (ks) ksc = ks[row];
    if (vs) vsc = vs[row];
  };
  if (k0 < k1) load_chunk(k0);
#pragma unroll
  for (int r = 0; r < QPT; ++r) {
    const int i = t + 256 * r;
    if (i < G * D) qs[i / D][i % D] = qv[r] * scale;
  }
  __syncthreads();

  float M[GMAX], L[GMAX], o[GMAX][2], s[GMAX];
#pragma unroll
  for (int i = 0; i < GMAX; ++i) {
    M[i] = -INFINITY;
    L[i] = 0.f;
    o[i][0] = o[i][1] = 0.f;
  }

  for (int c0 = k0; c0 < k1; c0 += KC) {
    const bool valid = c0 + kk < k1;
    if (k_new != nullptr && c0 + kk == S - 1) {
      const size_t row = head_base + (S - 1);
      if constexpr (std::is_same<TK, int8_t>::value) {
        static_assert(!std::is_same<TK, int8_t>::value || TPK * CPT * 16 == D, "int8 row split over TPK threads");
        // quantise the new K and V rows: every thread of the key takes the whole row's absmax
        // (identical result), then quantises and stores its own 16-B pieces
        auto quant = [&](const TQ* src, dec_u32x4 (&raw)[CPT], float& sc_out, float* sc_dst, TK* dst) {
          float m = 0.f;
          for (int d = 0; d < D; ++d) m = fmaxf(m, fabsf(to_f(src[d])));
          float sc = m / 127.f;
          if (sc == 0.f) sc = 1.f;
#pragma unroll
          for (int c = 0; c < CPT; ++c) {
            uint32_t w[4];
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
              uint32_t acc = 0;
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const float x = fminf(fmaxf(rintf(to_f(src[16 * (part * CPT + c) + 4 * q4 + e]) / sc), -128.f), 127.f);
                acc |= ((uint32_t)(uint8_t)(int8_t)x) << (8 * e);
              }
              w[q4] = acc;
            }
            raw[c] = (dec_u32x4){w[0], w[1], w[2], w[3]};
            *reinterpret_cast<dec_u32x4*>(dst + row * D + 16 * (part * CPT + c)) = raw[c];
          }
          sc_out = sc;
          if (part == 0) sc_dst[row] = sc;
        };
        quant(k_new + new_off, kr, ksc, const_cast<float*>(ks), const_cast<TK*>(kc));
        quant(v_new + new_off, vr, vsc, const_cast<float*>(vs), const_cast<TK*>(vc));
      } else {
#pragma unroll
        for (int c = 0; c < CPT; ++c) {
          *reinterpret_cast<dec_u32x4*>(reinterpret_cast<char*>(const_cast<TK*>(kc) + row * D) + part * CPT * 16 + 16 * c) = kr[c];
          *reinterpret_cast<dec_u32x4*>(reinterpret_cast<char*>(const_cast<TK*>(vc) + row * D) + part * CPT * 16 + 16 * c) = vr[c];
        }
      }
    }
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int pc = part * CPT + c;
      *reinterpret_cast<dec_u32x4*>(vbuf + kk * RB + ((pc ^ (kk & SW)) << 4)) = vr[c];
    }
    // scores and the chunk max per query head
#pragma unroll
    for (int i = 0; i < GMAX; ++i) {
      if (!GC && i >= G) break;
      float a = 0.f;
#pragma unroll
      for (int c = 0; c < CPT; ++c) {
        float kv[PN];
        Piece<TK>::cvt(kr[c], kv);
#pragma unroll
        for (int e = 0; e < PN; ++e) a += qs[i][(part * CPT + c) * PN + e] * kv[e];
      }
#pragma unroll
      for (int x = 1; x < TPK; x <<= 1) a += __shfl_xor(a, x, 64);
      s[i] = valid ? a * ksc : -INFINITY;
      const float wm = wave_max(s[i]);
      if (lane == 0) red_m[wid][i] = wm;
    }
    const float vsc_c = vsc;
    __syncthreads();
    // online softmax: p (with the V scale folded in) to LDS, chunk sums
#pragma unroll
    for (int i = 0; i < GMAX; ++i) {
      if (!GC && i >= G) break;
      const float cm = fmaxf(fmaxf(red_m[0][i], red_m[1][i]), fmaxf(red_m[2][i], red_m[3][i]));
      const float mn = fmaxf(M[i], cm);
      const float alpha = M[i] == -INFINITY ? 0.f : __expf(M[i] - mn);
      const float p = valid ? __expf(s[i] - mn) : 0.f;
      if (part == 0) pl[i][kk] = p * vsc_c;
      const float ws = wave_sum(part == 0 ? p : 0.f);
      if (lane == 0) red_l[wid][i] = ws;
      M[i] = mn;
      s[i] = alpha;
    }
    if (c0 + KC < k1) load_chunk(c0 + KC);  // prefetch: lands while this chunk's P·V runs
    __syncthreads();
    const int nv = min(KC, k1 - c0);
#pragma unroll
    for (int i = 0; i < GMAX; ++i) {
      if (!GC && i >= G) break;
      L[i] = L[i] * s[i] + (red_l[0][i] + red_l[1][i]) + (red_l[2][i] + red_l[3][i]);
      o[i][0] *= s[i];
      o[i][1] *= s[i];
    }
    // P·V from LDS: thread owns columns d0, d0+1 and keys kg, kg+NG, ...
    constexpr int ES = (int)sizeof(TK);
    const int bo = d0 * ES;
#pragma unroll 8
    for (int j = kg; j < nv; j += NG) {
      const char* vp = vbuf + j * RB + ((((bo >> 4) ^ (j & SW))) << 4) + (bo & 15);
      float v0, v1;
      if constexpr (std::is_same<TK, bf16>::value) {
        const uint32_t w = *reinterpret_cast<const uint32_t*>(vp);
        v0 = __uint_as_float(w << 16);
        v1 = __uint_as_float(w & 0xffff0000u);
      } else if constexpr (std::is_same<TK, __half>::value) {
        const __half2 h2 = *reinterpret_cast<const __half2*>(vp);
        v0 = __low2float(h2);
        v1 = __high2float(h2);
      } else if constexpr (std::is_same<TK, float>::value) {
        const float2 f2 = *reinterpret_cast<const float2*>(vp);
        v0 = f2.x;
        v1 = f2.y;
      } else {
        const uint16_t w = *reinterpret_cast<const uint16_t*>(vp);
        v0 = (float)(int8_t)(w & 0xff);
        v1 = (float)(int8_t)(w >> 8);
      }
#pragma unroll
      for (int i = 0; i < GMAX; ++i) {
        if (!GC && i >= G) break;
        const float pw = pl[i][j];
        o[i][0] += pw * v0;
        o[i][1] += pw * v1;
      }
    }
    __syncthreads();
  }
  // merge the NG key groups (partials reuse the V buffer)
  float* ro = reinterpret_cast<float*>(vbuf);
#pragma unroll
  for (int i = 0; i < GMAX; ++i) {
    if (!GC && i >= G) break;
    *reinterpret_cast<float2*>(ro + (kg * GMAX + i) * D + d0) = make_float2(o[i][0], o[i][1]);
    if (t == 0) {
      fin[i][0] = M[i];
      fin[i][1] = L[i];
    }
  }
  __syncthreads();
  for (int idx = t; idx < G * D; idx += 256) {
    const int i = idx / D, d = idx % D;
    float O = 0.f;
#pragma unroll
    for (int x = 0; x < NG; ++x) O += ro[(x * GMAX + i) * D + d];
    const float Mi = fin[i][0], Li = fin[i][1];
    const int h = g * G + i;
    if (nsplit == 1) {
      out[(((size_t)b * Tq + tq) * H + h) * D + d] = from_f<TQ>(Li > 0.f ? O / Li : 0.f);
    } else {
      const size_t r = (((size_t)split * B + b) * Tq + tq) * H + h;
      ws_o[r * D + d] = O;
      if (d == 0) {
        ws_ml[2 * r] = Mi;
        ws_ml[2 * r + 1] = Li;
      }
    }
  }
  if (nsplit == 1 || cnt == nullptr) return;
  // In-launch merge: the last of the item's split workgroups to arrive combines all splits' (m, l, O)
  // in split order — the same arithmetic, in the same order, as decode_combine_kernel (so the
  // result does not depend on which workgroup arrives last), without a second launch. The counter
  // is left at zero for the next launch (a replayed graph reuses it).
  __syncthreads();
  __shared__ int last;
  const int item = blockIdx.x / splits;
  if (t == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int prev = __hip_atomic_fetch_add(&cnt[item], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = prev == nsplit - 1;
  }
  __syncthreads();
  if (!last) return;
  if (t == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(&cnt[item], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const int64_t rows = (int64_t)B * Tq * H;
  for (int idx = t; idx < G * D; idx += 256) {
    const int i = idx / D, d = idx % D;
    const int64_t r = ((int64_t)b * Tq + tq) * H + g * G + i;
    // every split's (m, l, o) loads issue together (one memory round trip, not 3 per split: the
    // serial form cost ~0.1 ms per layer at 16 splits)
    float mv[kMaxMergeSplits], lv[kMaxMergeSplits], ov[kMaxMergeSplits];
#pragma unroll
    for (int sp = 0; sp < kMaxMergeSplits; ++sp) {
      const int64_t rr = sp * rows + r;
      const bool on = sp < nsplit;
      mv[sp] = on ? ws_ml[2 * rr] : -INFINITY;
      lv[sp] = on ? ws_ml[2 * rr + 1] : 0.f;
      ov[sp] = on ? ws_o[rr * D + d] : 0.f;
    }
    float Mx = -INFINITY;
#pragma unroll
    for (int sp = 0; sp < kMaxMergeSplits; ++sp) Mx = fmaxf(Mx, mv[sp]);
    float Lx = 0.f, Ox = 0.f;
#pragma unroll
    for (int sp = 0; sp < kMaxMergeSplits; ++sp) {
      if (sp >= nsplit) break;
      const float f = mv[sp] == -INFINITY ? 0.f : __expf(mv[sp] - Mx);
      Lx += lv[sp] * f;
      Ox += ov[sp] * f;
    }
    out[r * D + d] = from_f<TQ>(Lx > 0.f ? Ox / Lx : 0.f);
  }
}

// Small-batch decode attention (bf16 cache, one query row, query group G <= 16): one workgroup
// per (batch, KV head), its 4 waves each own a contiguous quarter of the keys — no split-K launch,
// no barrier inside the key loop. Per 16-key block a wave computes the scores of all G heads with
// v_mfma_f32_16x16x32_bf16 (A = 16 K rows straight from global memory, B = the group's queries,
// held in registers), runs the online softmax per head with two cross-lane exchanges, parks P in
// its own LDS slice and accumulates P·V on the VALU with lane = D/64 output columns (the V rows
// read whole and coalesced). The next block's K and V rows are issued before this block's math.
// The 4 waves' (m, l, O) merge through LDS at the end. Made for the batch-1 GQA shapes where the
// general kernel's thread-per-key loop is serial (Gemma-3 1B: G = 4, D = 256 — 19 µs per layer).
// Fused append as in decode_kernel: key S-1 comes from k_new / v_new and is written to the cache.
// rc / rs (optional, fp32 [D/2]: this step's RoPE cos / sin): the query and the new key arrive
// unrotated and are rotated here (rotate-half pairs d, d + D/2, rope_vec_kernel's arithmetic), so the
// decode step needs no separate RoPE pass. Column chunk s2 of a lane pairs with chunk s2 + KS/2 of
// the same lane, so the rotation stays in registers.
// ROPE is a template flag so the default instantiations compile exactly as without it (as a run-time
// branch it cost the D = 512 kernels 320 B/lane of scratch).
template <int D, int GMAX, bool ROPE = false>  // GMAX: the exact query-group size H / Hkv
__global__ void __launch_bounds__(256) decode_small_kernel(const bf16* __restrict__ q, bf16* __restrict__ kc,
                                                           bf16* __restrict__ vc, bf16* __restrict__ out, int H,
                                                           int Hkv, int cap, int S, float scale,
                                                           const int64_t* __restrict__ S_dev, int64_t q_rs,
                                                           const bf16* __restrict__ k_new,
                                                           const bf16* __restrict__ v_new, int64_t kv_rs,
                                                           const float* __restrict__ rc,
                                                           const float* __restrict__ rs) {
  constexpr int KS = D / 32;   // MFMA k-steps per score block
  constexpr int EPL = D / 64;  // P·V output columns per lane
  static_assert(EPL >= 1 && (EPL & (EPL - 1)) == 0 && GMAX <= 16, "decode_small geometry");
  typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
  typedef float f32x4_t __attribute__((ext_vector_type(4)));
  constexpr int G = GMAX;
  const int g = blockIdx.x % Hkv, b = blockIdx.x / Hkv;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int r16 = lane & 15, qd = lane >> 4;
  __shared__ float pl[4][16][16];           // a wave's P block [key][head]
  __shared__ float wm[4][GMAX], wl[4][GMAX];
  __shared__ float wo[4][GMAX][D];

  if (S_dev != nullptr) S = (int)min<int64_t>(*S_dev, (int64_t)cap);
  const size_t head_base = ((size_t)b * Hkv + g) * cap;
  const size_t new_off = (size_t)b * kv_rs + (size_t)g * D;
  const float c = scale * 1.4426950408889634f;

  // this lane's query column (head r16 of the group), d-chunks 8qd + 32s
  uint4 qf[KS];
  {
    const bool ok = r16 < G;
    const bf16* qp = q + (size_t)b * q_rs + (size_t)(g * G + (ok ? r16 : 0)) * D + 8 * qd;
#pragma unroll
    for (int s2 = 0; s2 < KS; ++s2) qf[s2] = ok ? *reinterpret_cast<const uint4*>(qp + 32 * s2) : uint4{0u, 0u, 0u, 0u};
  }
  // rotate a lane's KS chunks (columns 32 s2 + 8 qd .. +8) of one head row in place
  auto rotate = [&](uint4* f) {
#pragma unroll
    for (int s2 = 0; s2 < KS / 2; ++s2) {
      const int j0 = 32 * s2 + 8 * qd;
      const float4 c0 = *reinterpret_cast<const float4*>(rc + j0), c1 = *reinterpret_cast<const float4*>(rc + j0 + 4);
      const float4 n0 = *reinterpret_cast<const float4*>(rs + j0), n1 = *reinterpret_cast<const float4*>(rs + j0 + 4);
      const float cs[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
      const float sn[8] = {n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, n1.z, n1.w};
      const uint32_t a[4] = {f[s2].x, f[s2].y, f[s2].z, f[s2].w};
      const uint32_t bb[4] = {f[s2 + KS / 2].x, f[s2 + KS / 2].y, f[s2 + KS / 2].z, f[s2 + KS / 2].w};
      uint32_t o1[4], o2[4];
#pragma unroll
      for (int e2 = 0; e2 < 4; ++e2) {
        const float x1l = __uint_as_float(a[e2] << 16), x1h = __uint_as_float(a[e2] & 0xffff0000u);
        const float x2l = __uint_as_float(bb[e2] << 16), x2h = __uint_as_float(bb[e2] & 0xffff0000u);
        const int e = 2 * e2;
        const float y1l = x1l * cs[e] - x2l * sn[e], y1h = x1h * cs[e + 1] - x2h * sn[e + 1];
        const float y2l = x2l * cs[e] + x1l * sn[e], y2h = x2h * cs[e + 1] + x1h * sn[e + 1];
        o1[e2] = pack_bf16x2(y1l, y1h);
        o2[e2] = pack_bf16x2(y2l, y2h);
      }
      f[s2] = uint4{o1[0], o1[1], o1[2], o1[3]};
      f[s2 + KS / 2] = uint4{o2[0], o2[1], o2[2], o2[3]};
    }
  };
  if constexpr (ROPE) rotate(qf);
  // keys of this wave
  const int per = ((S + 63) / 64) * 16;  // 16-key blocks, a quarter each
  const int k0 = w * per, k1 = min(S, k0 + per);
  float m = -INFINITY, l = 0.f;  // for head r16 (replicated over qd)
  float o[GMAX][EPL];
#pragma unroll
  for (int i = 0; i < GMAX; ++i)
#pragma unroll
    for (int e = 0; e < EPL; ++e) o[i][e] = 0.f;

  uint4 kf[KS];
  uint32_t vraw[16][(EPL + 1) / 2];  // this lane's EPL bf16 of 16 V rows
  auto load_block = [&](int kb) {
    const int key = min(kb + r16, S - 1);
    const bool fresh = k_new != nullptr && key == S - 1;
    const bf16* kr = fresh ? k_new + new_off : kc + (head_base + key) * D;
#pragma unroll
    for (int s2 = 0; s2 < KS; ++s2) kf[s2] = *reinterpret_cast<const uint4*>(kr + 32 * s2 + 8 * qd);
    if constexpr (ROPE) {
      if (fresh) rotate(kf);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int kj = min(kb + j, S - 1);
      const bool fr = v_new != nullptr && kj == S - 1;
      const bf16* vr = (fr ? v_new + new_off : vc + (head_base + kj) * D) + EPL * lane;
      if constexpr (EPL == 1) vraw[j][0] = *reinterpret_cast<const uint16_t*>(vr);
      else if constexpr (EPL == 2) vraw[j][0] = *reinterpret_cast<const uint32_t*>(vr);
      else if constexpr (EPL == 4) {
        const uint2 u = *reinterpret_cast<const uint2*>(vr);
        vraw[j][0] = u.x;
        vraw[j][1] = u.y;
      } else {
        const uint4 u = *reinterpret_cast<const uint4*>(vr);
        vraw[j][0] = u.x; vraw[j][1] = u.y; vraw[j][2] = u.z; vraw[j][3] = u.w;
      }
    }
  };
  // fused append: the wave holding key S-1 writes this step's K / V row into the cache
  if (k_new != nullptr && k0 < k1 && S - 1 >= k0 && S - 1 < k1) {
    const bf16* ks = k_new + new_off;
    const bf16* vs = v_new + new_off;
    bf16* kd = kc + (head_base + S - 1) * D;
    bf16* vd = vc + (head_base + S - 1) * D;
    for (int d = 8 * lane; d < D; d += 512) {
      if constexpr (ROPE) {
        constexpr int half = D / 2;
        const int j0 = d < half ? d : d - half;
        float x1[8], x2[8], y[8];
        Vec8<bf16>::load(ks + j0, x1);
        Vec8<bf16>::load(ks + j0 + half, x2);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          y[e] = d < half ? x1[e] * rc[j0 + e] - x2[e] * rs[j0 + e] : x2[e] * rc[j0 + e] + x1[e] * rs[j0 + e];
        Vec8<bf16>::store(kd + d, y);
      } else {
        *reinterpret_cast<uint4*>(kd + d) = *reinterpret_cast<const uint4*>(ks + d);
      }
      *reinterpret_cast<uint4*>(vd + d) = *reinterpret_cast<const uint4*>(vs + d);
    }
  }
  if (k0 < k1) load_block(k0);
  for (int kb = k0; kb < k1; kb += 16) {
    f32x4_t sacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s2 = 0; s2 < KS; ++s2)
      sacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, kf[s2]),
                                                     __builtin_bit_cast(bf16x8_t, qf[s2]), sacc, 0, 0, 0);
    float vf[16][EPL];  // this block's V values (fp32), taken before the next block's loads land
#pragma unroll
    for (int j = 0; j < 16; ++j)
#pragma unroll
      for (int e = 0; e < EPL; ++e) {
        const uint32_t word = vraw[j][e >> 1];
        vf[j][e] = EPL == 1 ? __uint_as_float(word << 16)
                            : ((e & 1) ? __uint_as_float(word & 0xffff0000u) : __uint_as_float(word << 16));
      }
    const int nk = min(16, k1 - kb);
    if (kb + 16 < k1) load_block(kb + 16);
    // scores of keys kb + 4qd + r for head r16 (masked past the wave's range)
    float sc[4], bmax = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      sc[r] = (4 * qd + r < nk) ? sacc[r] * c : -INFINITY;
      bmax = fmaxf(bmax, sc[r]);
    }
    bmax = fmaxf(bmax, __shfl_xor(bmax, 16, 64));
    bmax = fmaxf(bmax, __shfl_xor(bmax, 32, 64));
    const float mn = fmaxf(m, bmax);
    const float alpha = m == -INFINITY ? 0.f : exp2f(m - mn);
    float ps = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float pv = exp2f(sc[r] - mn);
      ps += pv;
      pl[w][4 * qd + r][r16] = pv;
    }
    ps += __shfl_xor(ps, 16, 64);
    ps += __shfl_xor(ps, 32, 64);
    l = l * alpha + ps;
    m = mn;
    // every lane needs alpha of every head: head i's value lives in lane i
    float al[GMAX];
#pragma unroll
    for (int i = 0; i < GMAX; ++i) al[i] = __shfl(alpha, i, 64);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's P writes visible to its reads
#pragma unroll
    for (int i = 0; i < G; ++i)
#pragma unroll
      for (int e = 0; e < EPL; ++e) o[i][e] *= al[i];
    // keys past the range have p = 0 (their scores are -inf): all 16 rows, no branch
#pragma unroll
    for (int j = 0; j < 16; ++j)
#pragma unroll
      for (int i = 0; i < G; ++i) {
        const float pw = pl[w][j][i];
#pragma unroll
        for (int e = 0; e < EPL; ++e) o[i][e] += pw * vf[j][e];
      }
  }
  // merge the 4 waves
  if (qd == 0 && r16 < G) {
    wm[w][r16] = m;
    wl[w][r16] = l;
  }
#pragma unroll
  for (int i = 0; i < G; ++i)
#pragma unroll
    for (int e = 0; e < EPL; ++e) wo[w][i][EPL * lane + e] = o[i][e];
  __syncthreads();
  for (int idx = t; idx < G * D; idx += 256) {
    const int i = idx / D, d = idx - i * D;
    const float M = fmaxf(fmaxf(wm[0][i], wm[1][i]), fmaxf(wm[2][i], wm[3][i]));
    float O = 0.f, L = 0.f;
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const float e = wm[x][i] == -INFINITY ? 0.f : exp2f(wm[x][i] - M);
      O += e * wo[x][i][d];
      L += e * wl[x][i];
    }
    out[((size_t)b * H + g * G + i) * D + d] = from_f<bf16>(L > 0.f ? O / L : 0.f);
  }
}

template <typename TQ>
__global__ void __launch_bounds__(256) decode_combine_kernel(const float* __restrict__ ws_o,
                                                             const float* __restrict__ ws_ml, TQ* __restrict__ out,
                                                             int rows, int D, int splits) {
  const int64_t total = (int64_t)rows * D;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / D;
    const int d = (int)(i - r * D);
    float M = -INFINITY;
    for (int s = 0; s < splits; ++s) M = fmaxf(M, ws_ml[2 * ((int64_t)s * rows + r)]);
    float L = 0.f, O = 0.f;
    for (int s = 0; s < splits; ++s) {
      const int64_t rr = (int64_t)s * rows + r;
      const float ms = ws_ml[2 * rr];
      const float f = ms == -INFINITY ? 0.f : __expf(ms - M);
      L += ws_ml[2 * rr + 1] * f;
      O += ws_o[rr * D + d] * f;
    }
    out[i] = from_f<TQ>(L > 0.f ? O / L : 0.f);
  }
}

// Append one token's K and V rows (read straight from the fused QKV projection) into the cache
// slot `pos` — taken from device memory when pos_dev is given (graph-replayed decode). One wave
// per (batch, KV head, K|V) row; int8 caches quantise per token (absmax / 127, round to nearest
// even) exactly like kv_quant_kernel.
template <typename T, typename TK>
__global__ void __launch_bounds__(256) kv_append_kernel(const T* __restrict__ k, const T* __restrict__ v,
                                                        int64_t k_rs, int64_t v_rs, TK* __restrict__ kc,
                                                        TK* __restrict__ vc, float* __restrict__ ks,
                                                        float* __restrict__ vs, int B, int Hkv, int D, int cap,
                                                        const int64_t* __restrict__ pos_dev, int pos_host) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);  // over B*Hkv*2
  if (row >= B * Hkv * 2) return;
  const int which = row & 1, bg = row >> 1;
  const int g = bg % Hkv, b = bg / Hkv;
  const T* src = (which ? v + (size_t)b * v_rs : k + (size_t)b * k_rs) + (size_t)g * D;
  const int pos = pos_dev ? (int)*pos_dev : pos_host;
  const size_t slot = ((size_t)b * Hkv + g) * cap + pos;
  TK* dst = (which ? vc : kc) + slot * D;
  if constexpr (std::is_same<TK, int8_t>::value) {
    float m = 0.f;
    for (int d = lane; d < D; d += 64) m = fmaxf(m, fabsf(to_f(src[d])));
    m = wave_max(m);
    float sc = m / 127.f;
    if (sc == 0.f) sc = 1.f;
    for (int d = lane; d < D; d += 64) {
      float x = rintf(to_f(src[d]) / sc);
      dst[d] = (int8_t)fminf(fmaxf(x, -128.f), 127.f);
    }
    if (lane == 0) (which ? vs : ks)[slot] = sc;
  } else {
    for (int d = lane; d < D; d += 64) dst[d] = src[d];
  }
}

}  // namespace penroz

using namespace penroz;

// Whether decode_attn takes the one-workgroup-per-(batch, KV head) kernel (decode_small_kernel) for
// a bf16 cache of S slots (the capacity under graph capture). Callers fusing RoPE into the decode
// step ask this first: only that kernel rotates in place.
bool decode_small_applies(int64_t B, int64_t Tq, int64_t H, int64_t Hkv, int64_t D, int64_t S) {
  // PENROZ_DECODE_SMALL_ITEMS: the largest B·Hkv it takes (0 disables)
  static const int small_items = [] {
    const char* e = std::getenv("PENROZ_DECODE_SMALL_ITEMS");
    return e ? std::atoi(e) : 64;
  }();
  static const bool small_any = [] {  // (A/B switch: also MHA head_dim 64 — GPT-2)
    const char* e = std::getenv("PENROZ_DECODE_SMALL_ANY");
    return e && e[0] == '1';
  }();
  static const int split_keys_env = [] {
    const char* e = std::getenv("PENROZ_DECODE_SPLIT_KEYS");
    const int v = e ? std::atoi(e) : 0;
    return v >= 64 ? v : 0;
  }();
  if (Hkv <= 0 || H % Hkv) return false;
  const int64_t G0 = H / Hkv;
  // the one-workgroup-per-item kernel takes contexts up to 1024 keys (GQA batch 1: Gemma-3 1B
  // 1.57 -> 1.26 ms/token at a 1024-slot cache, profiles/decode_r5.md); GQA or wide heads only: at
  // G = 1, D = 64 (GPT-2 batch 1) the general kernel is ~1 µs faster per layer. It runs ONE
  // workgroup per (batch, KV head) over the whole cache, so longer contexts keep the key-split
  // grid
  const int64_t small_keys = split_keys_env ? split_keys_env : 1024;
  return Tq == 1 && B * Hkv <= small_items && S <= small_keys && (G0 >= 2 || D >= 128 || small_any) &&
         (G0 == 1 || G0 == 2 || G0 == 4 || G0 == 8 || G0 == 16) && (D == 64 || D == 128 || D == 256 || D == 512) &&
         G0 * D <= 4096;
}

// seq_len_dev (optional int64 [1] on the device): the cache length is read by the kernel at run
// time (S / q_offset are then only upper bounds used to size the launch) — lets a captured HIP
// graph replay the same decode step at every position.
// k_new / v_new (optional, Tq == 1): this step's K / V rows [B, 1, Hkv, D] (views into the fused
// QKV rows allowed): appended at slot S-1 by the kernel itself (see decode_kernel).
torch::Tensor decode_attn(torch::Tensor q, torch::Tensor kc, torch::Tensor vc, c10::optional<torch::Tensor> k_scale,
                          c10::optional<torch::Tensor> v_scale, int64_t S, int64_t q_offset, double scale,
                          c10::optional<torch::Tensor> seq_len_dev, c10::optional<torch::Tensor> k_new,
                          c10::optional<torch::Tensor> v_new, c10::optional<torch::Tensor> counters,
                          c10::optional<torch::Tensor> rope_cos, c10::optional<torch::Tensor> rope_sin) {
  TORCH_CHECK(q.is_cuda() && q.dim() == 4, "q must be [B, Tq, H, D]");
  // q may be a view into the fused QKV rows: unit dim stride, packed heads, uniform row stride
  // (a size-1 Tq dim may carry any stride: the row stride is then stride(0))
  TORCH_CHECK(q.stride(3) == 1 && q.stride(2) == q.size(3) && (q.size(1) == 1 || q.stride(0) == q.size(1) * q.stride(1)),
              "q must have packed heads and a uniform row stride");
  TORCH_CHECK(kc.is_contiguous() && vc.is_contiguous() && kc.dim() == 4 && kc.sizes() == vc.sizes());
  const int B = q.size(0), Tq = q.size(1), H = q.size(2), D = q.size(3);
  const int Hkv = kc.size(1), cap = kc.size(2);
  TORCH_CHECK(kc.size(0) == B && kc.size(3) == D && H % Hkv == 0 && H / Hkv <= kMaxGroup);
  TORCH_CHECK(S <= cap && q_offset >= 0 && q_offset + Tq <= S, "bad cache extent");
  TORCH_CHECK(D == 32 || D == 64 || D == 128 || D == 256 || D == 512,
              "decode attention supports head_dim 32/64/128/256/512");
  const bool quant = kc.scalar_type() == torch::kInt8;
  TORCH_CHECK(!quant || (k_scale.has_value() && v_scale.has_value()), "int8 cache needs scales");
  TORCH_CHECK(quant || kc.scalar_type() == q.scalar_type(), "cache dtype must match q");
  auto out = torch::empty({B, Tq, H * D}, q.options());
  const int64_t q_rs = Tq == 1 ? q.stride(0) : q.stride(1);
  const int items = B * Hkv * Tq;
  // keys per split (each workgroup sweeps its keys in chunks of 256; a graph captures S = the cache
  // capacity and the kernel stops at the device-side length). With zeroed arrival counters
  // (`counters`, int32 >= items) the last split workgroup of an item merges the partials itself,
  // so a split costs no second launch and contexts beyond 256 keys are split; without them a split
  // costs the combine launch (~4.6 µs in a replayed step) and only contexts beyond 1024 keys are.
  // GPT-2 B = 1 at a 1024-key context: 0.489 ms/token unsplit vs 0.418 split four ways
  // (profiles/decode_longctx_r6.log). PENROZ_DECODE_SPLIT_KEYS overrides both.
  static const int split_keys_env = [] {
    const char* e = std::getenv("PENROZ_DECODE_SPLIT_KEYS");
    const int v = e ? std::atoi(e) : 0;
    return v >= 64 ? v : 0;
  }();
  int* cnt = nullptr;
  if (counters.has_value() && counters->defined()) {
    TORCH_CHECK(counters->is_cuda() && counters->scalar_type() == torch::kInt32 && counters->is_contiguous(),
                "counters: contiguous int32 on the device");
    // beyond 8192 keys the combine launch wins again: every merging item costs its split
    // workgroups a device-scope release (Gemma-3 1B batch 1 at 16k keys, 16 splits either way:
    // 10.89-10.91 ms/token merged in launch vs 10.54-10.56 with the combine kernel)
    if (counters->numel() >= items && S <= kMergeMaxKeys) cnt = counters->data_ptr<int>();
  }
  const int split_keys = split_keys_env ? split_keys_env : (cnt ? 256 : 1024);
  int splits = std::max(1, std::min<int>((512 + items - 1) / items, (int)((S + split_keys - 1) / split_keys)));
  // the merging workgroup reads every split's partials: at most 16
  if (cnt) splits = std::min(splits, kMaxMergeSplits);
  const int64_t* sdev = nullptr;
  if (seq_len_dev.has_value() && seq_len_dev->defined()) {
    TORCH_CHECK(seq_len_dev->is_cuda() && seq_len_dev->scalar_type() == torch::kInt64 && seq_len_dev->numel() == 1,
                "seq_len_dev must be a device int64 [1]");
    sdev = seq_len_dev->data_ptr<int64_t>();
  }
  const bool fuse = k_new.has_value() && k_new->defined();
  int64_t kv_rs = 0;
  if (fuse) {
    TORCH_CHECK(v_new.has_value() && v_new->defined() && Tq == 1, "fused append: k_new and v_new, Tq == 1");
    for (const auto* t : {&*k_new, &*v_new}) {
      TORCH_CHECK(t->scalar_type() == q.scalar_type() && t->dim() == 4 && t->size(0) == B && t->size(1) == 1 &&
                      t->size(2) == Hkv && t->size(3) == D && t->stride(3) == 1 && t->stride(2) == D &&
                      reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0,
                  "k_new / v_new must be [B, 1, Hkv, D] with packed heads");
    }
    TORCH_CHECK(k_new->stride(0) == v_new->stride(0) && k_new->stride(0) % 8 == 0, "k_new / v_new row stride");
    kv_rs = k_new->stride(0);
  }
  const float* ksp = quant ? k_scale->data_ptr<float>() : nullptr;
  const float* vsp = quant ? v_scale->data_ptr<float>() : nullptr;
  auto stream = at::hip::getCurrentHIPStream();
  // small batches, bf16, one query row: the wave-parallel MFMA kernel (decode_small_kernel)
  const bool small = !quant && q.scalar_type() == torch::kBFloat16 && decode_small_applies(B, Tq, H, Hkv, D, S) &&
                     (!fuse || kv_rs % 8 == 0);
  const bool rope = rope_cos.has_value() && rope_cos->defined();
  if (rope) {
    TORCH_CHECK(small && fuse && D <= 256, "in-kernel RoPE: the small decode kernel with the fused append, "
                "head_dim <= 256 only (check decode_small_applies first)");
    for (const auto* t : {&*rope_cos, &*rope_sin})
      TORCH_CHECK(t->is_cuda() && t->scalar_type() == torch::kFloat32 && t->is_contiguous() && t->numel() == D / 2,
                  "rope cos / sin: contiguous fp32 [D/2] (one position)");
  }
  const float* rcp = rope ? rope_cos->data_ptr<float>() : nullptr;
  const float* rsp = rope ? rope_sin->data_ptr<float>() : nullptr;
  if (small) {
    const int G0 = H / Hkv;
    const bf16* qp = reinterpret_cast<const bf16*>(q.data_ptr());
    bf16* kp = reinterpret_cast<bf16*>(kc.data_ptr());
    bf16* vp = reinterpret_cast<bf16*>(vc.data_ptr());
    bf16* op = reinterpret_cast<bf16*>(out.data_ptr());
    const bf16* knp = fuse ? reinterpret_cast<const bf16*>(k_new->data_ptr()) : nullptr;
    const bf16* vnp = fuse ? reinterpret_cast<const bf16*>(v_new->data_ptr()) : nullptr;
#define PENROZ_DSMALL(DD, GG)                                                                                   \
  do {                                                                                                            \
  if (rope && DD <= 256)                                                                                          \
    hipLaunchKernelGGL((decode_small_kernel<DD, GG, true>), dim3(B * Hkv), dim3(256), 0, stream, qp, kp, vp, op, H, \
                       Hkv, cap, (int)S, (float)scale, sdev, q_rs, knp, vnp, kv_rs, rcp, rsp);                       \
  else                                                                                                            \
    hipLaunchKernelGGL((decode_small_kernel<DD, GG, false>), dim3(B * Hkv), dim3(256), 0, stream, qp, kp, vp, op, H, \
                       Hkv, cap, (int)S, (float)scale, sdev, q_rs, knp, vnp, kv_rs, nullptr, nullptr);                \
  } while (0)
#define PENROZ_DSMALL_G(DD)                      \
  switch (G0) {                                   \
    case 1: PENROZ_DSMALL(DD, 1); break;          \
    case 2: PENROZ_DSMALL(DD, 2); break;          \
    case 4: PENROZ_DSMALL(DD, 4); break;          \
    case 8: PENROZ_DSMALL(DD, 8); break;          \
    default: PENROZ_DSMALL(DD, 16);               \
  }
    if (D == 64) PENROZ_DSMALL_G(64)
    else if (D == 128) PENROZ_DSMALL_G(128)
    else if (D == 256) PENROZ_DSMALL_G(256)
    else if (G0 == 1) PENROZ_DSMALL(512, 1);
    else if (G0 == 2) PENROZ_DSMALL(512, 2);
    else if (G0 == 4) PENROZ_DSMALL(512, 4);
    else PENROZ_DSMALL(512, 8);
#undef PENROZ_DSMALL_G
#undef PENROZ_DSMALL
    return out;
  }
  torch::Tensor ws_o, ws_ml;
  float* wo = nullptr;
  float* wm = nullptr;
  if (splits > 1) {
    ws_o = torch::empty({(int64_t)splits * B * Tq * H * D}, q.options().dtype(torch::kFloat32));
    ws_ml = torch::empty({(int64_t)splits * B * Tq * H * 2}, q.options().dtype(torch::kFloat32));
    wo = ws_o.data_ptr<float>();
    wm = ws_ml.data_ptr<float>();
  }
  dim3 grid(items * splits);
  auto launch = [&](auto qtag, auto ktag) {
    using TQ = decltype(qtag);
    using TK = decltype(ktag);
    const TQ* qp = reinterpret_cast<const TQ*>(q.data_ptr());
    const TK* kp = reinterpret_cast<const TK*>(kc.data_ptr());
    const TK* vp = reinterpret_cast<const TK*>(vc.data_ptr());
    TQ* op = reinterpret_cast<TQ*>(out.data_ptr());
    const TQ* knp = fuse ? reinterpret_cast<const TQ*>(k_new->data_ptr()) : nullptr;
    const TQ* vnp = fuse ? reinterpret_cast<const TQ*>(v_new->data_ptr()) : nullptr;
    const int G = H / Hkv;
#define PENROZ_DECODE(DD, GC)                                                                                   \
  hipLaunchKernelGGL((decode_kernel<DD, GC, TQ, TK>), grid, dim3(256), 0, stream, qp, kp, vp, ksp, vsp, op, wo, wm, \
                     B, Tq, H, Hkv, cap, (int)S, (int)q_offset, splits, (float)scale, sdev, q_rs, knp, vnp, kv_rs, cnt, \
                     split_keys)
#define PENROZ_DECODE_G(DD)              \
  switch (G) {                           \
    case 1: PENROZ_DECODE(DD, 1); break; \
    case 4: PENROZ_DECODE(DD, 4); break; \
    case 8: PENROZ_DECODE(DD, 8); break; \
    default: PENROZ_DECODE(DD, 0);       \
  }
    if (D == 64) PENROZ_DECODE_G(64)
    else if (D == 128) PENROZ_DECODE_G(128)
    else if (D == 256) PENROZ_DECODE_G(256)  // Gemma
    else if (D == 32) PENROZ_DECODE(32, 0);  // small GPT-style models (any group size)
    else PENROZ_DECODE(512, 0);              // Gemma-4 full-attention layers (global_head_dim)
#undef PENROZ_DECODE_G
#undef PENROZ_DECODE
    if (splits > 1 && cnt == nullptr) {
      const int rows = B * Tq * H;
      hipLaunchKernelGGL(decode_combine_kernel<TQ>, dim3(std::min(2048, (rows * D + 255) / 256)), dim3(256), 0, stream,
                         wo, wm, op, rows, D, splits);
    }
  };
  auto with_k = [&](auto qtag) {
    if (quant) launch(qtag, int8_t{});
    else launch(qtag, qtag);
  };
  if (q.scalar_type() == torch::kBFloat16) with_k(bf16{});
  else if (q.scalar_type() == torch::kFloat32) with_k(float{});
  else if (q.scalar_type() == torch::kFloat16) with_k(__half{});
  else TORCH_CHECK(false, "unsupported q dtype");
  return out;
}

// k, v: [B, 1, Hkv, D] (views into the fused QKV rows allowed); caches [B, Hkv, cap, D]
void kv_append(torch::Tensor k, torch::Tensor v, torch::Tensor kc, torch::Tensor vc, c10::optional<torch::Tensor> ks,
               c10::optional<torch::Tensor> vs, c10::optional<torch::Tensor> pos_dev, int64_t pos) {
  TORCH_CHECK(k.is_cuda() && k.dim() == 4 && k.sizes() == v.sizes() && k.size(1) == 1, "k/v must be [B, 1, Hkv, D]");
  TORCH_CHECK(k.stride(3) == 1 && k.stride(2) == k.size(3) && v.stride(3) == 1 && v.stride(2) == v.size(3),
              "k/v rows must be packed");
  const int B = k.size(0), Hkv = k.size(2), D = k.size(3);
  TORCH_CHECK(kc.is_contiguous() && vc.is_contiguous() && kc.sizes() == vc.sizes() && kc.size(0) == B &&
              kc.size(1) == Hkv && kc.size(3) == D, "cache shape");
  const int cap = kc.size(2);
  const int64_t* pd = nullptr;
  if (pos_dev.has_value() && pos_dev->defined()) {
    TORCH_CHECK(pos_dev->is_cuda() && pos_dev->scalar_type() == torch::kInt64 && pos_dev->numel() == 1);
    pd = pos_dev->data_ptr<int64_t>();
  } else {
    TORCH_CHECK(pos >= 0 && pos < cap, "cache overflow");
  }
  const bool quant = kc.scalar_type() == torch::kInt8;
  TORCH_CHECK(!quant || (ks.has_value() && vs.has_value()), "int8 cache needs scales");
  TORCH_CHECK(quant || kc.scalar_type() == k.scalar_type(), "cache dtype must match k/v");
  const int rows = B * Hkv * 2;
  auto stream = at::hip::getCurrentHIPStream();
  auto launch = [&](auto ttag, auto ktag) {
    using T = decltype(ttag);
    using TK = decltype(ktag);
    hipLaunchKernelGGL((kv_append_kernel<T, TK>), dim3((rows + 3) / 4), dim3(256), 0, stream,
                       reinterpret_cast<const T*>(k.data_ptr()), reinterpret_cast<const T*>(v.data_ptr()), k.stride(0),
                       v.stride(0), reinterpret_cast<TK*>(kc.data_ptr()), reinterpret_cast<TK*>(vc.data_ptr()),
                       quant ? ks->data_ptr<float>() : nullptr, quant ? vs->data_ptr<float>() : nullptr, B, Hkv, D,
                       cap, pd, (int)pos);
  };
  auto with_k = [&](auto ttag) {
    if (quant) launch(ttag, int8_t{});
    else launch(ttag, ttag);
  };
  if (k.scalar_type() == torch::kBFloat16) with_k(bf16{});
  else if (k.scalar_type() == torch::kFloat32) with_k(float{});
  else if (k.scalar_type() == torch::kFloat16) with_k(__half{});
  else TORCH_CHECK(false, "unsupported k dtype");
}
