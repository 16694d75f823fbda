// Shared device helpers for the penroz CDNA4 (gfx950) kernels.
//
// Conventions: wave64 everywhere (lane = threadIdx.x & 63), 16-byte vector memory access for
// every bf16/fp32 stream (Guideline 13 of the CDNA HIP guide), fp32 math internally, bf16
// rounding to nearest-even via the compiler's native conversion (v_cvt_pk_bf16_f32 on gfx950).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

namespace penroz {

constexpr int kWave = 64;

using bf16 = __hip_bfloat16;
typedef float float4_t __attribute__((ext_vector_type(4)));
typedef short short8_t __attribute__((ext_vector_type(8)));
typedef short short4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(uint16_t u) { return __uint_as_float(((uint32_t)u) << 16); }
__device__ __forceinline__ float bf2f(bf16 v) { return __bfloat162float(v); }

// fp32 -> bf16 bits, round to nearest even (NaN stays NaN through the native cvt).
__device__ __forceinline__ uint16_t f2bf_bits(float f) {
  bf16 b = __float2bfloat16(f);
  return *reinterpret_cast<uint16_t*>(&b);
}

typedef float float2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

// two fp32 -> packed bf16x2 (RNE) in ONE v_cvt_pk_bf16_f32 (the scalar form costs 4 VALU ops)
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((float2_t){lo, hi}, bf16x2_t));
}

// Whole-wave reductions (all 64 lanes active; every lane gets the result). Within each 16-lane
// row the lanes combine through DPP (quad_perm [1,0,3,2], [2,3,0,1], then row_ror 4 and 8: no
// LDS traffic, a few cycles each), then the four row results are read into scalar registers
// (v_readlane) and combined in a fixed order. The former __shfl_xor butterfly issued six
// ds_bpermute round trips through the LDS crossbar per reduction (~100 cycles each, serially
// dependent): in the decode LayerNorm prologues that alone was microseconds per kernel.
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float lane_f32(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
template <typename Op>
__device__ __forceinline__ float wave_reduce(float v, Op op) {
  v = op(v, dpp_f32<0xB1>(v));   // quad_perm [1,0,3,2]
  v = op(v, dpp_f32<0x4E>(v));   // quad_perm [2,3,0,1]
  v = op(v, dpp_f32<0x124>(v));  // row_ror:4
  v = op(v, dpp_f32<0x128>(v));  // row_ror:8
  return op(op(lane_f32(v, 0), lane_f32(v, 16)), op(lane_f32(v, 32), lane_f32(v, 48)));
}

__device__ __forceinline__ float wave_sum(float v) {
  return wave_reduce(v, [](float a, float b) { return a + b; });
}

__device__ __forceinline__ float wave_max(float v) {
  return wave_reduce(v, [](float a, float b) { return fmaxf(a, b); });
}

__device__ __forceinline__ float wave_min(float v) {
  return wave_reduce(v, [](float a, float b) { return fminf(a, b); });
}

// Load 8 consecutive elements (16 B for bf16, 32 B for fp32) as floats.
template <typename T> struct Vec8;
template <> struct Vec8<float> {
  __device__ __forceinline__ static void load(const float* p, float (&v)[8]) {
    float4_t a = *reinterpret_cast<const float4_t*>(p);
    float4_t b = *reinterpret_cast<const float4_t*>(p + 4);
    v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
    v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
  }
  __device__ __forceinline__ static void store(float* p, const float (&v)[8]) {
    *reinterpret_cast<float4_t*>(p) = float4_t{v[0], v[1], v[2], v[3]};
    *reinterpret_cast<float4_t*>(p + 4) = float4_t{v[4], v[5], v[6], v[7]};
  }
};
template <> struct Vec8<bf16> {
  __device__ __forceinline__ static void load(const bf16* p, float (&v)[8]) {
    uint4 u = *reinterpret_cast<const uint4*>(p);
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  __device__ __forceinline__ static void store(bf16* p, const float (&v)[8]) {
    uint4 u;
    u.x = pack_bf16x2(v[0], v[1]);
    u.y = pack_bf16x2(v[2], v[3]);
    u.z = pack_bf16x2(v[4], v[5]);
    u.w = pack_bf16x2(v[6], v[7]);
    *reinterpret_cast<uint4*>(p) = u;
  }
};
template <> struct Vec8<__half> {
  __device__ __forceinline__ static void load(const __half* p, float (&v)[8]) {
    const __half2* h = reinterpret_cast<const __half2*>(p);
    uint4 u = *reinterpret_cast<const uint4*>(p);
    const __half2* hh = reinterpret_cast<const __half2*>(&u);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float2 f = __half22float2(hh[i]);
      v[2 * i] = f.x;
      v[2 * i + 1] = f.y;
    }
    (void)h;
  }
  __device__ __forceinline__ static void store(__half* p, const float (&v)[8]) {
    uint4 u;
    __half2* hh = reinterpret_cast<__half2*>(&u);
#pragma unroll
    for (int i = 0; i < 4; ++i) hh[i] = __floats2half2_rn(v[2 * i], v[2 * i + 1]);
    *reinterpret_cast<uint4*>(p) = u;
  }
};

// Vec8 load / store with an optional non-temporal hint (NT: the stream is touched once; measured
// faster for the large elementwise passes, see the PENROZ_EW_NT note in elementwise.hip)
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
template <bool NT, typename T>
__device__ __forceinline__ void load8(const T* p, float (&v)[8]) {
  if constexpr (!NT) {
    Vec8<T>::load(p, v);
  } else {
    constexpr int NB = (int)sizeof(T) / 2;  // 16-B pieces: 1 (16-bit types) or 2 (fp32)
    u32x4_t r[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) r[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p) + i);
    Vec8<T>::load(reinterpret_cast<const T*>(r), v);
  }
}
template <bool NT, typename T>
__device__ __forceinline__ void store8(T* p, const float (&v)[8]) {
  if constexpr (!NT) {
    Vec8<T>::store(p, v);
  } else {
    constexpr int NB = (int)sizeof(T) / 2;
    u32x4_t r[NB];
    Vec8<T>::store(reinterpret_cast<T*>(r), v);
#pragma unroll
    for (int i = 0; i < NB; ++i) __builtin_nontemporal_store(r[i], reinterpret_cast<u32x4_t*>(p) + i);
  }
}

template <typename T> __device__ __forceinline__ float to_f(T v);
template <> __device__ __forceinline__ float to_f<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f<bf16>(bf16 v) { return __bfloat162float(v); }
template <> __device__ __forceinline__ float to_f<__half>(__half v) { return __half2float(v); }

template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float v) { return __float2bfloat16(v); }
template <> __device__ __forceinline__ __half from_f<__half>(float v) { return __float2half(v); }

// GELU (erf, or tanh when approx) and its derivative, fp32; shared by the elementwise kernels
// and the GEMM epilogues.
__device__ __forceinline__ float gelu_f(float x, int approx) {
  if (approx) {
    const float k = 0.7978845608028654f;
    const float t = tanhf(k * (x + 0.044715f * x * x * x));
    return 0.5f * x * (1.f + t);
  }
  return 0.5f * x * (1.f + erff(x * 0.7071067811865476f));
}

// gated-MLP activations: 0 gelu (erf), 1 gelu (tanh), 2 silu
__device__ __forceinline__ float act_f(float x, int kind) {  // 0 gelu, 1 gelu_tanh, 2 silu
  if (kind == 2) return x / (1.f + __expf(-x));
  return gelu_f(x, kind);
}

__device__ __forceinline__ float gelu_grad_f(float x, int approx) {
  if (approx) {
    const float k = 0.7978845608028654f;
    const float x2 = x * x;
    const float t = tanhf(k * (x + 0.044715f * x2 * x));
    return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k * (1.f + 3.f * 0.044715f * x2);
  }
  const float cdf = 0.5f * (1.f + erff(x * 0.7071067811865476f));
  const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

// Counter-based RNG (splitmix/murmur finalizer) -> uniform in [0, 1).
__device__ __forceinline__ uint32_t hash_u32(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return (uint32_t)x;
}
__device__ __forceinline__ float uniform01(uint64_t seed, uint64_t counter) {
  return (hash_u32(seed * 0x9E3779B97F4A7C15ULL + counter) >> 8) * (1.0f / 16777216.0f);
}

// Element dropout multiplier for the residual-branch / embedding dropout of the fused GPT
// executor: 1/(1-p) when element `counter` of stream `seed` is kept, else 0. Forward and backward
// regenerate the same mask from (seed, row·C + col) — nothing is stored.
__device__ __forceinline__ float dropout_mult(uint64_t seed, uint64_t counter, float p, float inv_keep) {
  return uniform01(seed, counter) >= p ? inv_keep : 0.f;
}


// ---- LDS-DMA (global_load_lds_dwordx4) ----------------------------------------------------
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;
static __device__ uint4 g_zero16[1];  // zero-initialised: source of out-of-range LDS-DMA lanes

// one global_load_lds_dwordx4: 64 lanes x 16 B from per-lane `g` to LDS [lds_addr, +1 KiB)
// (lane-linear destination, wave-uniform base). Issued as inline asm so hipcc's waitcnt pass
// does not serialise it against ds_reads of other LDS buffers; completion is counted by hand
// (s_waitcnt vmcnt before the barrier that publishes the buffer).
__device__ __forceinline__ void glds16(const void* g, unsigned lds_addr) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(lds_addr)
               : "memory");
}



// 4-byte LDS-DMA (global_load_lds_dword): 64 lanes x 4 B to LDS [lds_addr, +256 B).
__device__ __forceinline__ void glds4(const void* g, unsigned lds_addr) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(lds_addr)
               : "memory");
}

// LDS-DMA with a wave-uniform 64-bit SGPR base and a per-lane 32-bit byte offset: per-piece
// address updates become scalar adds (no 64-bit VALU address math). No instruction offset:
// on an LDS-DMA load it would shift the LDS destination as well as the global address.
__device__ __forceinline__ void glds16_s(const void* sbase, unsigned voff, unsigned lds_addr) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(sbase), "s"(lds_addr)
               : "memory");
}

// Make the compiler treat a register value as freshly produced here: it waits for the load
// that produced it BEFORE this point, so no compiler-tracked load stays outstanding into a
// loop whose waits are counted by hand (LDS-DMA issued in inline asm is invisible to hipcc's
// waitcnt pass, and a wait for an old load would also drain the in-flight DMA).
__device__ __forceinline__ void launder(uint4& v) {
  asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
}


// Lane id the compiler cannot hoist (volatile v_mbcnt): address math derived from it is
// recomputed where used instead of being precomputed as loop invariants and spilled.
__device__ __forceinline__ int opaque_lane_id() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

__device__ __forceinline__ unsigned lds_addr_of(const void* p) { return (unsigned)(size_t)(lds_void_t*)p; }


// ---- debug build (PENROZ_DEBUG=1 python setup.py build_ext -> build_ext/debug) --------------
// Device-side checks of data-dependent indices (token ids, targets, cache positions). Release
// builds compile them out (and clamp / skip instead); debug builds print the failing
// condition with its location and trap, which surfaces as a HIP error on the next sync.
#ifdef PENROZ_DEBUG
#define PZ_DEVICE_CHECK(cond)                                                                  \
  do {                                                                                         \
    if (!(cond)) {                                                                             \
      printf("penroz device check failed: %s at %s:%d (block %d, thread %d)\n", #cond, __FILE__, \
             __LINE__, (int)blockIdx.x, (int)threadIdx.x);                                     \
      __builtin_trap();                                                                        \
    }                                                                                          \
  } while (0)
#else
#define PZ_DEVICE_CHECK(cond) ((void)0)
#endif

}  // namespace penroz
