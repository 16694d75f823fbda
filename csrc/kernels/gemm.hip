// Forward / data-gradient GEMM for MI355X with fused epilogues:
//
//   C[M][N] = A[M][K] · Bᵀ (+ bias[N]) (→ GELU),   bf16 operands, fp32 accumulation, bf16 out
//
// B is either [N][K] (TN: a linear layer's forward, y = x·Wᵀ with W [out, in]) or [K][N]
// (NN: its input gradient, dx = dy·W). Replaces hipBLASLt for the GPT-2 forward and dgrad
// GEMMs so that bias add, GELU (writing both the pre-activation and the activation) happen
// in the epilogue instead of in separate memory-bound passes.
//
// Design (gfx950):
//   * persistent: one 512-thread workgroup per CU walks a strided list of 256×256 output
//     tiles; the operand stream is ONE LDS-DMA ring over all (tile, k-step) pairs of the
//     workgroup, so the next tile's first k-steps are already in flight while the epilogue of
//     the current tile stores (no per-tile pipeline fill/drain at K = 768);
//   * ring of 4 stages × [A 256×32 | B 256×32] bf16 (128 KiB + 2 KiB epilogue bias), three stages in flight, filled
//     by global_load_lds_dwordx4 (inline asm, counted vmcnt, raw s_barrier: no hidden drains);
//   * 8 waves as 2 (M) × 4 (N), each 128×64 = 8×4 v_mfma_f32_16x16x32_bf16 tiles, issued with
//     the operands swapped (D = B·Aᵀ) so each lane ends up holding 4 consecutive output
//     COLUMNS of one row; a v_permlane16_swap of tile pairs widens that to 8 columns, so the
//     epilogue issues 16-B stores (16 per wave per tile), and the two ring waits after an
//     epilogue count those stores instead of waiting for them;
//   * [rows][32] operand images have 64-B rows; the 16-B chunk of row r is stored at slot
//     ch ^ ((-(r>>2)) & 3), which makes every 16-lane ds_read_b128 group conflict-free (the
//     DMA destination is lane-linear, so the swizzle is applied on the source address);
//     [32][256] images (NN B operand) use the wgrad kernel's 512-B-row XOR image and
//     ds_read_b64_tr_b16;
//   * XCD-aware tile order: workgroups of one XCD take consecutive tile indices, and tiles are
//     ordered in groups of 8 row panels so an XCD's working set (A and B panels) stays in its L2;
//   * the epilogue bias arrives by LDS-DMA too (issued BEFORE the tile's last-step DMA and
//     covered by that step's counted vmcnt), so no compiler-visible global load ever forces the
//     in-flight ring to drain (hipcc waits vmcnt(0) for its own loads).
#include "common.h"
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

namespace penroz {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) u32x2 lds_u32x2;

constexpr int TM = 256, TN = 256, KC = 64, GM = 8;
constexpr int A_IMG = TM * KC * 2;          // 32 KiB: A chunk [256][64]
constexpr int CHUNK = A_IMG + TN * KC * 2;  // 64 KiB: A + B chunk (two of them double-buffer)

enum Epi { EPI_NONE = 0, EPI_BIAS = 1, EPI_BIAS_GELU = 2 };

__device__ __forceinline__ f32x4 mfma16(uint4 a, uint4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                 0, 0, 0);
}

// [rows][64] bf16 image (128-B rows = whole cache lines per DMA row): 16-B chunk ch (0..7) of
// row r lives at slot ch ^ rswz(r); every 16-lane ds_read_b128 group of a 16-row fragment read
// then covers 16 distinct bank slots (conflict-free).
__device__ __forceinline__ int rswz(int row) { return (row >> 1) & 7; }

// fragment of 16 rows starting at a 16-aligned row, k-step `sub` (0/1) of the 64-deep chunk:
// lane l gets row r0 + (l&15), k = 32·sub + 8(l>>4) .. +7
__device__ __forceinline__ uint4 row_frag(const char* tile, int r0, int sub, int lane) {
  const int r = r0 + (lane & 15);
  const u32x4 v = *(const lds_u32x4*)(tile + r * 128 + ((((lane >> 4) + 4 * sub) ^ rswz(r)) << 4));
  return __builtin_bit_cast(uint4, v);
}

// [64][256] bf16 image (512-B rows) for the NN B operand (same image as gemm_wgrad.hip)
__device__ __forceinline__ int swz16(int row) { return ((row & 3) << 2) | (((row >> 3) & 1) << 1); }
__device__ __forceinline__ int off512b(int row, int ch) { return row * 512 + ((ch ^ swz16(row)) << 4); }

// element j = tile[kbase + 8·(lane>>4) + j][c0 + (lane&15)]
__device__ __forceinline__ uint4 tr_frag(const char* tile, int kbase, int c0, int lane) {
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

__device__ __forceinline__ void tile_coords(int t, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int per_group = GM * tiles_n;
  const int group = t / per_group;
  const int first_m = group * GM;
  const int gsz = min(tiles_m - first_m, GM);
  const int r = t - group * per_group;
  tm = first_m + r % gsz;
  tn = r / gsz;
}

__device__ __forceinline__ float bf_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }

// raw barrier between ring steps: this wave's LDS reads are done (lgkmcnt 0) and its DMAs up to
// the counted stage have landed; the asm statements keep the compiler from moving LDS accesses
// across the barrier.
#define RING_BARRIER()                \
  do {                                \
    asm volatile("" ::: "memory");    \
    if (!(ablate & 2)) __builtin_amdgcn_s_barrier(); \
    asm volatile("" ::: "memory");    \
  } while (0)

#define RING_SYNC_LGKM()                                    \
  do {                                                      \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");      \
    if (!(ablate & 2)) __builtin_amdgcn_s_barrier();        \
    asm volatile("" ::: "memory");                          \
  } while (0)

#define RING_SYNC(VMCNT)                                                                \
  do {                                                                                  \
    asm volatile("s_waitcnt vmcnt(" #VMCNT ")\n\ts_waitcnt lgkmcnt(0)" ::: "memory");   \
    if (!(ablate & 2)) __builtin_amdgcn_s_barrier();                                    \
    asm volatile("" ::: "memory");                                                      \
  } while (0)

template <bool B_KN, int EPI>
__global__ void __launch_bounds__(512, 1) gemm_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                      const bf16* __restrict__ bias, bf16* __restrict__ C,
                                                      bf16* __restrict__ C2, int M, int N, int K, int lda, int ldb,
                                                      int ldc, int tiles_m, int tiles_n, int approx, int ablate) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w >> 2, wn = w & 3;
  const int nwg = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, qd = nwg >> 3, rd = nwg & 7;
  const int u = (xcd < rd ? xcd * (qd + 1) : rd * (qd + 1) + (xcd - rd) * qd) + (b >> 3);
  const int ntiles = tiles_m * tiles_n;
  const int nc = K / KC;                // 64-deep chunks per tile
  const int my_tiles = (ntiles - u + nwg - 1) / nwg;
  const int total = my_tiles * nc * 2;  // 32-deep MFMA steps of this workgroup
  const unsigned lds_base = (unsigned)(size_t)(lds_void_t*)smem;
  const void* zero = (const void*)g_zero16;
  const unsigned bias_lds = lds_base + 2 * CHUNK;  // 8 waves x 256 B: epilogue bias

  // ---- LDS-DMA of whole 64-deep chunks (A and B: 4 + 4 global_load_lds_dwordx4 per wave), issued
  // strictly in order. One wave-uniform SGPR base per operand + per-lane 32-bit offsets that change
  // only at a new tile (rows / columns past the matrix edge are clamped to the last valid one: their
  // products land in output rows / columns that are never stored).
  int dj = 0, dk = 0, dc = 0, dm0 = 0, dn0 = 0;
  unsigned voa[4], vob[4];
  auto new_tile = [&](int t) {
    int tm, tn;
    tile_coords(t, tiles_m, tiles_n, tm, tn);
    dm0 = tm * TM, dn0 = tn * TN;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int piece = 4 * w + p;
      const int r = 8 * piece + (lane >> 3);
      const int c = (lane & 7) ^ rswz(r);
      voa[p] = (unsigned)((min(r, M - 1 - dm0) * lda + 8 * c) * 2);
      if constexpr (B_KN) {
        const int kr = 2 * piece + (lane >> 5);
        const int ch = (lane & 31) ^ swz16(kr);
        vob[p] = (unsigned)((kr * ldb + min(8 * ch, N - 8 - dn0)) * 2);
      } else {
        vob[p] = (unsigned)((min(r, N - 1 - dn0) * ldb + 8 * c) * 2);
      }
    }
  };
  new_tile(u);
  auto dma_next = [&]() {
    const int k = dk * KC;
    const unsigned buf = lds_base + (unsigned)((dc & 1) * CHUNK);
    const bf16* ba = A + (size_t)dm0 * lda + k;
    const bf16* bb = B_KN ? B + (size_t)k * ldb + dn0 : B + (size_t)dn0 * ldb + k;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int piece = 4 * w + p;
      glds16_s(ba, voa[p], __builtin_amdgcn_readfirstlane(buf + piece * 1024));
      glds16_s(bb, vob[p], __builtin_amdgcn_readfirstlane(buf + A_IMG + piece * 1024));
    }
    ++dc;
    if (++dk == nc) {
      dk = 0;
      ++dj;
      new_tile(u + dj * nwg);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int jn = 0; jn < 4; ++jn) acc[i][jn] = f32x4{0.f, 0.f, 0.f, 0.f};

  dma_next();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // ---- ping-pong main loop. Group 0 = waves 0-3, group 1 = waves 4-7 (one of each per SIMD).
  // Two barriers per 32-deep step, X and Y; between them one group runs its 32 MFMAs while the
  // other reads its fragments (and, on a chunk's first step, issues the next chunk's DMA), and the
  // roles swap at every barrier:
  //   group 0:  reads(st) [DMA]   X   MFMA(st) [epilogue]  wait  Y
  //   group 1:        X   reads(st) [DMA]  wait  Y   MFMA(st) [epilogue]
  // Chunk c is read in steps 2c, 2c+1; chunk c+1's DMA goes to the other buffer from step 2c
  // (after Y(2c-1), when both groups are done with chunk c-1) and every wave waits for it before
  // Y(2c+1). Group 1 waits lgkmcnt(0) before every Y, so its reads are done before the buffer it
  // read can be re-filled.
  const int grp = wm;
  int kk = 0, j = 0;  // kk: 32-deep step within the tile
  const int nk = 2 * nc;
  constexpr int ST_OPS = EPI == EPI_BIAS_GELU ? 32 : 16;  // 16-B stores per wave per epilogue
  const int g = lane >> 4;
  // a compiler-visible lgkmcnt(0) (vmcnt/expcnt untouched): no scalar load is pending at the loop
  // entry, so hipcc can count the LDS fragment reads inside the loop instead of waiting for 0
  __builtin_amdgcn_s_waitcnt(0xC07F);
  uint4 bf[4], af[8];

  auto issue = [&](int st, bool dma) {
    if constexpr (EPI != EPI_NONE) {
      if (kk == nk - 2) {  // the tile ends with the next step: its bias -> this wave's LDS slot
        int tm, tn;
        tile_coords(u + j * nwg, tiles_m, tiles_n, tm, tn);
        const int n = tn * TN + 64 * wn + 2 * lane;
        glds4(lane < 32 && n < N ? (const void*)(bias + n) : zero, __builtin_amdgcn_readfirstlane(bias_lds + w * 256));
      }
    }
    const int sub = st & 1;
    const char* At = smem + ((st >> 1) & 1) * CHUNK;
    const char* Bt = At + A_IMG;
#pragma unroll
    for (int jn = 0; jn < 4; ++jn)
      bf[jn] = B_KN ? tr_frag(Bt, 32 * sub, 64 * wn + 16 * jn, lane) : row_frag(Bt, 64 * wn + 16 * jn, sub, lane);
#pragma unroll
    for (int i = 0; i < 8; ++i) af[i] = row_frag(At, 128 * wm + 16 * i, sub, lane);
    if (dma && !(ablate & 1)) dma_next();
  };
  auto compute = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int jn = 0; jn < 4; ++jn) acc[i][jn] = mfma16(bf[jn], af[i], acc[i][jn]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  };
  auto epilogue = [&](int jt) {
    int tm, tn;
    tile_coords(u + jt * nwg, tiles_m, tiles_n, tm, tn);
    const int m0 = tm * TM + 128 * wm + (lane & 15);
    // lane (m, g) holds columns 16·jn + 4g + r of each (i, jn) tile; a permlane16 swap of the
    // packed pairs (jn, jn+1) gives even-g lanes 8 consecutive columns of tile jn and odd-g
    // lanes 8 of tile jn+1: one 16-B store per lane per pair
    const int ncol = tn * TN + 64 * wn + 16 * (g & 1) + 8 * (g >> 1);
    uint2 bq[4];
    if constexpr (EPI != EPI_NONE) {
#pragma unroll
      for (int jn = 0; jn < 4; ++jn)
        bq[jn] = __builtin_bit_cast(uint2, *(const lds_u32x2*)(smem + 2 * CHUNK + w * 256 + 2 * (16 * jn + 4 * g)));
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = m0 + 16 * i;
#pragma unroll
      for (int jp = 0; jp < 4; jp += 2) {
        uint32_t px[2][2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          float bb[4] = {0.f, 0.f, 0.f, 0.f};
          if constexpr (EPI != EPI_NONE) {
            bb[0] = bf_lo(bq[jp + h].x); bb[1] = bf_hi(bq[jp + h].x); bb[2] = bf_lo(bq[jp + h].y); bb[3] = bf_hi(bq[jp + h].y);
          }
          const f32x4 v = acc[i][jp + h];
          px[h][0] = pack_bf16x2(v[0] + bb[0], v[1] + bb[1]);
          px[h][1] = pack_bf16x2(v[2] + bb[2], v[3] + bb[3]);
          acc[i][jp + h] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        const auto sx = __builtin_amdgcn_permlane16_swap(px[0][0], px[1][0], false, false);
        const auto sy = __builtin_amdgcn_permlane16_swap(px[0][1], px[1][1], false, false);
        const uint4 o = uint4{sx[0], sy[0], sx[1], sy[1]};
        const int n = ncol + 16 * jp;
        if (ablate & 8) {  // timing ablation: epilogue math without the global stores
          asm volatile("" ::"v"(o.x), "v"(o.y), "v"(o.z), "v"(o.w));
        } else if (m < M && n < N) {
          if (ablate & 16) __builtin_nontemporal_store(__builtin_bit_cast(u32x4, o), reinterpret_cast<u32x4*>(C + (size_t)m * ldc + n));
          else *reinterpret_cast<uint4*>(C + (size_t)m * ldc + n) = o;
          if constexpr (EPI == EPI_BIAS_GELU) {
            const uint4 q = uint4{pack_bf16x2(gelu_f(bf_lo(o.x), approx), gelu_f(bf_hi(o.x), approx)),
                                  pack_bf16x2(gelu_f(bf_lo(o.y), approx), gelu_f(bf_hi(o.y), approx)),
                                  pack_bf16x2(gelu_f(bf_lo(o.z), approx), gelu_f(bf_hi(o.z), approx)),
                                  pack_bf16x2(gelu_f(bf_lo(o.w), approx), gelu_f(bf_hi(o.w), approx))};
            *reinterpret_cast<uint4*>(C2 + (size_t)m * ldc + n) = q;
          }
        }
      }
    }
  };

  // Epilogues run right after the barrier that starts the OTHER group's MFMA phase (group 0:
  // after Y, group 1: after X), so the stores and the bias/GELU math overlap the other group's
  // MFMAs instead of stalling both groups at a barrier.
  bool pending = false;  // this wave holds a finished tile (acc) whose epilogue has not run yet
  for (int st = 0; st < total; ++st) {
    const bool last_k = kk == nk - 1;
    const bool odd = st & 1;
    const bool dma = !odd && st + 2 < total;  // first step of a chunk that has a successor
    if (grp == 1) {
      RING_BARRIER();  // X (group 1)
      if (pending && !(ablate & 4)) epilogue(j - 1);
      pending = false;
    }
    issue(st, dma);
    if (grp == 0) {
      RING_BARRIER();  // X (group 0)
    } else {           // Y (group 1): next chunk landed before an odd step's Y (this also covers the bias)
      if (odd) RING_SYNC(0);
      else RING_SYNC_LGKM();
    }
    compute();
    if (grp == 0) {  // Y (group 0)
      if (odd) RING_SYNC(0);
      else RING_BARRIER();
      if (last_k && !(ablate & 4)) epilogue(j);
    }
    if (last_k) {
      pending = true;
      kk = 0;
      ++j;
    } else {
      ++kk;
    }
  }
  if (grp == 1 && pending && !(ablate & 4)) epilogue(j - 1);
}

}  // namespace
}  // namespace penroz

using namespace penroz;

// out[M][N] = a[M][K] · (b_kn ? b[K][N] : b[N][K]ᵀ) (+ bias) (GELU: out = pre-activation,
// act = GELU(pre)). bf16 tensors with unit column stride; K % 64 == 0, K >= 128, N % 8 == 0.
// `ablate` (timing experiments only, results are wrong): 1 = no DMA after the first chunk,
// 2 = no barriers, 4 = no epilogue.
void gemm_bf16(torch::Tensor a, torch::Tensor b, bool b_kn, c10::optional<torch::Tensor> bias, torch::Tensor out,
               c10::optional<torch::Tensor> act, int64_t gelu_approx, int64_t ablate) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && out.is_cuda(), "gemm: GPU tensors");
  TORCH_CHECK(a.scalar_type() == torch::kBFloat16 && b.scalar_type() == torch::kBFloat16 &&
              out.scalar_type() == torch::kBFloat16, "gemm: bf16 operands");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && out.dim() == 2, "gemm: 2-D operands");
  TORCH_CHECK(a.stride(1) == 1 && b.stride(1) == 1 && out.stride(1) == 1, "gemm: unit column stride");
  const int M = a.size(0), K = a.size(1);
  const int N = b_kn ? b.size(1) : b.size(0);
  TORCH_CHECK((b_kn ? b.size(0) : b.size(1)) == K, "gemm: inner dimensions differ");
  TORCH_CHECK(out.size(0) == M && out.size(1) == N, "gemm: output shape");
  TORCH_CHECK(K % KC == 0 && K >= 2 * KC && N % 8 == 0, "gemm: K % 64 == 0, K >= 128 and N % 8 == 0 required");
  TORCH_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0 && out.stride(0) % 8 == 0, "gemm: row strides");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(b.data_ptr()) % 16 == 0 &&
              reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0, "gemm: alignment");
  const bool has_bias = bias.has_value() && bias->defined();
  const bool gelu = act.has_value() && act->defined();
  if (has_bias) {
    TORCH_CHECK(bias->scalar_type() == torch::kBFloat16 && bias->numel() == N && bias->is_contiguous() &&
                reinterpret_cast<uintptr_t>(bias->data_ptr()) % 8 == 0, "gemm: bias [N] bf16");
  }
  if (gelu) {
    TORCH_CHECK(has_bias, "gemm: the GELU epilogue needs a bias");
    TORCH_CHECK(act->scalar_type() == torch::kBFloat16 && act->sizes() == out.sizes() && act->strides() == out.strides(),
                "gemm: act must match out");
  }
  if (M == 0 || N == 0) return;
  static int n_cu = 0;
  static bool attr_set = false;
  if (n_cu == 0) {
    hipDeviceProp_t prop;
    n_cu = hipGetDeviceProperties(&prop, out.get_device()) == hipSuccess ? prop.multiProcessorCount : 256;
  }
  constexpr int LDS = 2 * CHUNK + 8 * 256;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_kernel<false, EPI_NONE>), hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_kernel<false, EPI_BIAS>), hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_kernel<false, EPI_BIAS_GELU>), hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_kernel<true, EPI_NONE>), hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_kernel<true, EPI_BIAS>), hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr_set = true;
  }
  const int tiles_m = (M + TM - 1) / TM, tiles_n = (N + TN - 1) / TN;
  const int ntiles = tiles_m * tiles_n;
  const int grid = std::min(ntiles, n_cu);
  auto stream = at::hip::getCurrentHIPStream();
  const bf16* ap = reinterpret_cast<const bf16*>(a.data_ptr());
  const bf16* bp = reinterpret_cast<const bf16*>(b.data_ptr());
  const bf16* biasp = has_bias ? reinterpret_cast<const bf16*>(bias->data_ptr()) : nullptr;
  bf16* cp = reinterpret_cast<bf16*>(out.data_ptr());
  bf16* c2 = gelu ? reinterpret_cast<bf16*>(act->data_ptr()) : nullptr;
  const int lda = a.stride(0), ldb = b.stride(0), ldc = out.stride(0);
#define PZ_GEMM_LAUNCH(BKN, EPIV)                                                                          \
  hipLaunchKernelGGL((gemm_kernel<BKN, EPIV>), dim3(grid), dim3(512), LDS, stream, ap, bp, biasp, cp, c2, M, N, K, \
                     lda, ldb, ldc, tiles_m, tiles_n, (int)gelu_approx, (int)ablate)
  if (b_kn) {
    TORCH_CHECK(!gelu, "gemm: GELU epilogue is forward (TN) only");
    if (has_bias) PZ_GEMM_LAUNCH(true, EPI_BIAS);
    else PZ_GEMM_LAUNCH(true, EPI_NONE);
  } else if (gelu) {
    PZ_GEMM_LAUNCH(false, EPI_BIAS_GELU);
  } else if (has_bias) {
    PZ_GEMM_LAUNCH(false, EPI_BIAS);
  } else {
    PZ_GEMM_LAUNCH(false, EPI_NONE);
  }
#undef PZ_GEMM_LAUNCH
}
