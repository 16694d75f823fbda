// Forward / data-gradient GEMM for MI355X:  C[M][N] = A[M][K] · B[N][K]ᵀ (+ bias[N]) (→ GELU)
// (bf16 operands, fp32 accumulate, bf16 out). Both operands are reduction-contiguous: for a linear
// y = x·Wᵀ, A = x and B = W as stored; for its data gradient dx = dy·W, A = dy and B = the
// transposed weight copy the executors keep ([in, out], models/executor.py _init_transposed).
//
// Derived from the weight-gradient pipeline that wins in step (gemm_wgrad.hip, 1.28 PF): 256×256
// output tile per 512-thread workgroup, 8 waves as 2 (M) × 4 (N), each 128 × 64 = 8 × 4
// v_mfma_f32_16x16x32_bf16 tiles; operand stages of [256 rows][32 k] (64-B rows) arrive by LDS-DMA
// (global_load_lds_dwordx4 with a scalar row base and a per-lane offset fixed for the kernel) into
// a 4-stage ring, three stages in flight, one counted vmcnt + one barrier per 32-deep k-step.
// What is new for the NT layout and short reductions (K = 768: 24 k-steps per tile):
//   * fragments are plain ds_read_b128 of 8 consecutive k (no transposed reads); the 16-B chunk of
//     row r sits at chunk ^ (((r >> 3) & 1) << 1), which puts each 16-lane ds_read_b128 group on 16
//     distinct bank slots (the XOR is applied to the DMA SOURCE address: the destination is
//     lane-linear);
//   * the operand order is swapped in the MFMA (B fragment first), so a lane's accumulator holds
//     4 consecutive OUTPUT COLUMNS of one row: one v_permlane16_swap per dword pairs two 16-column
//     blocks into 16-B row segments (dwordx4 stores, a wave instruction covers 16 rows × 64 B);
//   * persistent: one workgroup per CU walks its tiles with the DMA ring running on into the next
//     tile, so a tile's first k-steps are in flight during the previous tile's last MFMAs;
//   * the epilogue stores are NOT waited for: vmcnt counts loads, LDS-DMA and stores in issue
//     order, so the stores are issued right after the k-step's DMA and the next three end-of-step
//     waits count them among the younger operations (vmcnt(2G + S)) — the stores get three
//     k-steps to drain before anything waits on them (the round-3/4 designs stalled the next
//     tile's DMA behind the store burst: profiles/native_gemm_r4.md);
//   * tile order: XCD-aware (the 32 workgroups of one XCD take 32 consecutive tiles per round)
//     and grouped along M (GROUP_M row tiles × the column tiles), so concurrently running tiles
//     share A row panels and B column panels in that XCD's L2;
//   * epilogues: bias (from an LDS copy made in the prologue), and GELU (erf or tanh) writing the
//     pre-activation and the activation from one accumulator pass (mode 1: fc + bias + GELU).
// Reference semantics: nn.Linear (+ nn.GELU), /root/reference/mappers.py:21, main.py:63-82.
#include "common.h"
#include <cstdlib>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

namespace penroz {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int NT_BM = 256, NT_BN = 256, NT_BK = 32, NT_NBUF = 4;
constexpr int NT_TILE = NT_BM * NT_BK * 2;     // 16 KiB: one operand, one stage
constexpr int NT_STAGE = 2 * NT_TILE;          // A | B
constexpr int NT_RING = NT_NBUF * NT_STAGE;    // 128 KiB
constexpr int NT_G = 4;                        // LDS-DMA instructions per wave per k-step
constexpr int NT_SCRATCH = 8 * 2048;          // epilogue: 2 KiB per wave
constexpr int NT_MAX_BIAS = 8192;              // bias columns kept in LDS (16 KiB)

__device__ __forceinline__ f32x4 mfma16(uint4 a, uint4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                 0, 0, 0);
}

// the 16-B chunk holding logical k-chunk c (0..3) of tile row r
__device__ __forceinline__ int nt_swz(int r) { return ((r >> 3) & 1) << 1; }

__device__ __forceinline__ void nt_tile_coords(int L, int tiles_m, int tiles_n, int gm, int& tm, int& tn) {
  const int per = gm * tiles_n;
  const int grp = L / per, first = grp * gm;
  const int gs = min(gm, tiles_m - first);
  const int r = L - grp * per;
  tm = first + r % gs;
  tn = r / gs;
}

template <int N_>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory");
}

__device__ __forceinline__ uint4 lds_read16(const char* base, unsigned off) {
  return *reinterpret_cast<const uint4*>(base + off);
}

__device__ __forceinline__ float nt_gelu(float x, int approx) { return gelu_f(x, approx); }

// GELU without library branches: erf by Abramowitz & Stegun 7.1.26 (|error| < 1.5e-7, far below
// a bf16 ulp of the result: one rcp, one exp2, 9 VALU) or, for the tanh form, the exact identity
// 0.5·x·(1 + tanh(u)) = x / (1 + exp(−2u)) (one exp2, one rcp)
__device__ __forceinline__ float gelu_fast(float x, int approx) {
  if (approx) {
    const float u = x * fmaf(0.0356774081f, x * x, 0.7978845608f);
    return x * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-2.8853900818f * u));
  }
  const float z = fabsf(x) * 0.7071067811865476f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float e = 1.f - p * t * __builtin_amdgcn_exp2f(-z * z * 1.4426950408889634f);  // erf(z)
  return 0.5f * x * (1.f + copysignf(e, x));
}

// MODE 0: C = A·Bᵀ; 1: C = A·Bᵀ + bias; 2: C = pre = A·Bᵀ + bias, C2 = GELU(bf16(pre)).
// RAGGED: N is not a multiple of 256 (the last column tile is partial; its stores are masked).
template <int MODE, bool RAGGED>
__global__ void __launch_bounds__(512, 1) gemm_nt_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                         const bf16* __restrict__ bias, bf16* __restrict__ C,
                                                         bf16* __restrict__ C2, int M, int N, int K, int lda, int ldb,
                                                         int ldc, int tiles_m, int tiles_n, int group_m, int approx,
                                                         int ablate) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // [ring 128 KiB][bias N × fp32... bf16]
  constexpr int S_ST = MODE == 2 ? 32 : 16;  // stores per wave per tile (dwordx4)
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w >> 2, wn = w & 3;
  const int G = gridDim.x;  // a multiple of 8 (host)
  const int my0 = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  const int ntiles = tiles_m * tiles_n;
  const int T = my0 < ntiles ? (ntiles - my0 + G - 1) / G : 0;
  if (T == 0) return;
  const int KS = K / NT_BK;

  // bias → LDS (once; nothing is in flight yet, so the barrier's waits cost nothing)
  bf16* sbias = reinterpret_cast<bf16*>(smem + NT_RING + NT_SCRATCH);
  if constexpr (MODE >= 1) {
    for (int c = threadIdx.x * 8; c < N; c += 512 * 8)
      *reinterpret_cast<uint4*>(sbias + c) = *reinterpret_cast<const uint4*>(bias + c);
  }
  __syncthreads();

  // LDS-DMA: piece i (0, 1) of wave w covers tile rows 16(2w + i) .. +15; lane -> row (lane >> 2),
  // physical 16-B chunk (lane & 3) holding logical chunk (lane & 3) ^ swz(row)
  unsigned aoff[2], boff[2];
  int prow[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 16 * (2 * w + i) + (lane >> 2);
    const int c = (lane & 3) ^ nt_swz(row);
    prow[i] = row;
    aoff[i] = (unsigned)row * (unsigned)lda * 2u + (unsigned)c * 16u;
    boff[i] = (unsigned)row * (unsigned)ldb * 2u + (unsigned)c * 16u;
  }
  const unsigned lds_base = (unsigned)(size_t)(lds_void_t*)smem;

  // DMA stream state (scalar): tile ordinal, its row bases, k offset
  int d_t = 0, d_k = 0, d_m0 = 0, d_n0 = 0;
  bool d_edge = false;
  auto d_tile = [&](int t) {
    int tm, tn;
    nt_tile_coords(t * G + my0, tiles_m, tiles_n, group_m, tm, tn);
    d_m0 = tm * NT_BM;
    d_n0 = tn * NT_BN;
    d_edge = RAGGED && d_n0 + NT_BN > N;
  };
  d_tile(0);
  auto dma = [&](int stage) {
    const unsigned la = __builtin_amdgcn_readfirstlane(lds_base + stage * NT_STAGE + 2 * w * 1024);
    const char* sa = reinterpret_cast<const char*>(A + (size_t)d_m0 * lda + d_k);
    const char* sb = reinterpret_cast<const char*>(B + (size_t)d_n0 * ldb + d_k);
    if (!d_edge) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        glds16_s(sa, aoff[i], la + i * 1024);
        glds16_s(sb, boff[i], la + NT_TILE + i * 1024);
      }
    } else {  // last column tile of a ragged N: rows past N re-read row N-1 (never stored)
      const int nmax = N - 1 - d_n0;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        glds16_s(sa, aoff[i], la + i * 1024);
        const int r = min(prow[i], nmax);
        const unsigned o = (unsigned)r * (unsigned)ldb * 2u + (boff[i] - (unsigned)prow[i] * (unsigned)ldb * 2u);
        glds16_s(sb, o, la + NT_TILE + i * 1024);
      }
    }
    // advance (the stream stops at the last tile's last k-step: later issues re-load it, which
    // keeps every wave's vmcnt arithmetic uniform; nobody reads those stages)
    if (d_k + NT_BK < K) {
      d_k += NT_BK;
    } else if (d_t + 1 < T) {
      d_k = 0;
      ++d_t;
      d_tile(d_t);
    }
  };

  // fragment reads: lane -> row (lane & 15), logical k-chunk (lane >> 4)
  const unsigned fl = (unsigned)((lane & 15) * 64 + (((lane >> 4) ^ nt_swz(lane & 15)) << 4));
  const unsigned fa = fl + (unsigned)(128 * wm) * 64u;
  const unsigned fb = NT_TILE + fl + (unsigned)(64 * wn) * 64u;
  const int g = lane >> 4;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: stages 0..2 in flight, wait for stage 0
  dma(0);
  dma(1);
  dma(2);
  vm_wait<2 * NT_G>();
  __builtin_amdgcn_s_barrier();

  if ((ablate & 2) && w >= 4) __builtin_amdgcn_s_setprio(1);  // the second-dispatched half
  // (A/B: stagger the workgroups' tile phases. ablate >> 8 = delay step in 10-ns ticks; bit 5: two
  // groups by (blockIdx >> 3) & 1, bit 6: four groups by (blockIdx >> 3) & 3)
  if (ablate & 96) {
    const int grp = (ablate & 64) ? ((blockIdx.x >> 3) & 3) : ((blockIdx.x >> 3) & 1);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const uint64_t until = t0 + (uint64_t)grp * (uint64_t)(ablate >> 8);
    while (__builtin_amdgcn_s_memrealtime() < until) __builtin_amdgcn_s_sleep(8);
  }
  int pending = 0;  // end-of-step waits that still count the last epilogue's stores
  int st = 0;       // global k-step (ring position)
  for (int t = 0; t < T; ++t) {
    int tm, tn;
    nt_tile_coords(t * G + my0, tiles_m, tiles_n, group_m, tm, tn);
    const int m0 = tm * NT_BM, n0 = tn * NT_BN;
    for (int ks = 0; ks < KS; ++ks, ++st) {
      dma((st + 3) & 3);
      const char* stg = smem + (st & 3) * NT_STAGE;
      uint4 bfr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = lds_read16(stg, fb + j * 1024);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint4 af = lds_read16(stg, fa + i * 1024);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(bfr[j], af, acc[i][j]);
      }
      if (ks == KS - 1) {
        // ---- epilogue. A lane holds rows m = 16 i + (lane & 15) and columns 16 j + 4 g + r of the
        // wave's 128 × 64 sub-tile; each 16-row slice goes through the wave's own 2-KiB LDS
        // scratch ([16 rows][128 B], 16-B chunk c of row r at c ^ ((r >> 1) & 7): conflict-free
        // 8-B writes and 16-B reads) and leaves as two stores of 8 rows × one whole 128-B line
        // (8 lanes per row). Stores of half lines (16 rows × 64 B per instruction, straight from
        // the accumulator layout) cost 125 µs of a 393 µs fc GEMM: profiles/gemm_nt_r6.md.
        const bool edge = RAGGED && n0 + NT_BN > N;
        char* scr = smem + NT_RING + w * 2048;
        float bv[4][4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) bv[j][r] = 0.f;
        if constexpr (MODE >= 1) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const uint2 bb = *reinterpret_cast<const uint2*>(sbias + min(n0 + 64 * wn + 16 * j + 4 * g, N - 4));
            bv[j][0] = __uint_as_float(bb.x << 16);
            bv[j][1] = __uint_as_float(bb.x & 0xffff0000u);
            bv[j][2] = __uint_as_float(bb.y << 16);
            bv[j][3] = __uint_as_float(bb.y & 0xffff0000u);
          }
        }
        const int wrow = lane & 15;
        const unsigned woff = (unsigned)(wrow * 128 + (g & 1) * 8);
        const int wsw = (wrow >> 1) & 7;
        const int rr = lane >> 3, rc = lane & 7;
        const unsigned roff0 = (unsigned)(rr * 128 + ((rc ^ ((rr >> 1) & 7)) << 4));
        const unsigned roff1 = (unsigned)((rr + 8) * 128 + ((rc ^ (((rr + 8) >> 1) & 7)) << 4));
        const int col = n0 + 64 * wn + 8 * rc;
        const bool col_ok = !RAGGED || !edge || col < N;
        const bool fast = (ablate & 8) != 0;
        const bool nt = (ablate & 16) != 0;
        auto put = [&](const uint2 (&p)[4], bf16* dst, int i) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            *reinterpret_cast<uint2*>(scr + woff + ((((2 * j + (g >> 1)) ^ wsw)) << 4)) = p[j];
          const uint4 v0 = *reinterpret_cast<const uint4*>(scr + roff0);
          const uint4 v1 = *reinterpret_cast<const uint4*>(scr + roff1);
          const int m = m0 + 128 * wm + 16 * i + rr;
          bf16* d0 = dst + (size_t)m * ldc + col;
          bf16* d1 = d0 + (size_t)8 * ldc;
          if (ablate & 1) {
            asm volatile("" ::"v"(v0.x), "v"(v0.y), "v"(v0.z), "v"(v0.w), "v"(v1.x), "v"(v1.y), "v"(v1.z), "v"(v1.w));
          } else if (col_ok) {
            if (nt) {
              __builtin_nontemporal_store(__builtin_bit_cast(u32x4_t, v0), reinterpret_cast<u32x4_t*>(d0));
              __builtin_nontemporal_store(__builtin_bit_cast(u32x4_t, v1), reinterpret_cast<u32x4_t*>(d1));
            } else {
              *reinterpret_cast<uint4*>(d0) = v0;
              *reinterpret_cast<uint4*>(d1) = v1;
            }
          }
        };
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          uint2 pv[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const f32x4 a = acc[i][j];
            pv[j] = uint2{pack_bf16x2(a[0] + bv[j][0], a[1] + bv[j][1]), pack_bf16x2(a[2] + bv[j][2], a[3] + bv[j][3])};
          }
          put(pv, C, i);
          if constexpr (MODE == 2) {
            uint2 qv[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float x0 = __uint_as_float(pv[j].x << 16), x1 = __uint_as_float(pv[j].x & 0xffff0000u);
              const float x2 = __uint_as_float(pv[j].y << 16), x3 = __uint_as_float(pv[j].y & 0xffff0000u);
              if (fast)
                qv[j] = uint2{pack_bf16x2(gelu_fast(x0, approx), gelu_fast(x1, approx)),
                              pack_bf16x2(gelu_fast(x2, approx), gelu_fast(x3, approx))};
              else
                qv[j] = uint2{pack_bf16x2(nt_gelu(x0, approx), nt_gelu(x1, approx)),
                              pack_bf16x2(nt_gelu(x2, approx), nt_gelu(x3, approx))};
            }
            put(qv, C2, i);
          }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (ablate & 1) {
          pending = 0;
        } else if (edge) {  // masked stores: their count is not uniform; drain them here
          vm_wait<0>();
          pending = 0;
        } else {
          pending = 3;
        }
      }
      if (pending > 0) {
        --pending;
        vm_wait<2 * NT_G + S_ST>();
      } else {
        vm_wait<2 * NT_G>();
      }
      __builtin_amdgcn_s_barrier();
    }
  }
  vm_wait<0>();
}

}  // namespace
}  // namespace penroz

using namespace penroz;

// out[M, N] (bf16, row stride ldc) = a[M, K] · b[N, K]ᵀ (+ bias[N]); mode 1 also writes
// act = GELU(out) (approx 0 erf, 1 tanh). Shapes: M % 256 == 0, N % 128 == 0, K % 32 == 0,
// K >= 160, row strides % 8 == 0.
bool gemm_nt_supported(int64_t M, int64_t N, int64_t K) {
  return M > 0 && M % 256 == 0 && N % 128 == 0 && N > 0 && K % 32 == 0 && K >= 5 * 32;
}

void gemm_nt(torch::Tensor a, torch::Tensor b, c10::optional<torch::Tensor> bias, torch::Tensor out,
             c10::optional<torch::Tensor> act, int64_t approx, int64_t group_m, int64_t grid, int64_t ablate) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && out.is_cuda(), "gemm_nt: CUDA tensors");
  TORCH_CHECK(a.scalar_type() == torch::kBFloat16 && b.scalar_type() == torch::kBFloat16 &&
                  out.scalar_type() == torch::kBFloat16, "gemm_nt: bf16 tensors");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && out.dim() == 2 && a.stride(1) == 1 && b.stride(1) == 1 &&
                  out.stride(1) == 1, "gemm_nt: 2-D row-major operands");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(b.size(1) == K && out.size(0) == M && out.size(1) == N, "gemm_nt: shape mismatch");
  TORCH_CHECK(gemm_nt_supported(M, N, K), "gemm_nt: needs M % 256 == 0, N % 128 == 0, K % 32 == 0, K >= 160");
  TORCH_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0 && out.stride(0) % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(b.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0, "gemm_nt: 16-B aligned rows");
  TORCH_CHECK((int64_t)a.stride(0) * 256 * 2 < (1ll << 32) && (int64_t)b.stride(0) * 256 * 2 < (1ll << 32),
              "gemm_nt: a 256-row panel must span < 4 GiB");
  const bf16* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->scalar_type() == torch::kBFloat16 && bias->is_contiguous() && bias->numel() == N &&
                    N <= NT_MAX_BIAS, "gemm_nt: bf16 bias [N], N <= 8192");
    bp = reinterpret_cast<const bf16*>(bias->data_ptr());
  }
  const bool gelu = act.has_value() && act->defined();
  if (gelu) {
    TORCH_CHECK(act->scalar_type() == torch::kBFloat16 && act->sizes() == out.sizes() &&
                    act->strides() == out.strides() && reinterpret_cast<uintptr_t>(act->data_ptr()) % 16 == 0,
                "gemm_nt: act like out");
    TORCH_CHECK(bp != nullptr, "gemm_nt: the GELU epilogue needs the bias");
  }
  const int tiles_m = (int)(M / 256), tiles_n = (int)((N + 255) / 256);
  const int ntiles = tiles_m * tiles_n;
  static int n_cu = 0;
  if (n_cu == 0) {
    hipDeviceProp_t prop;
    n_cu = hipGetDeviceProperties(&prop, out.get_device()) == hipSuccess ? prop.multiProcessorCount : 256;
  }
  int G = grid > 0 ? (int)grid : n_cu;
  G = std::max(8, std::min(G, (ntiles + 7) / 8 * 8)) / 8 * 8;
  const int gm = group_m > 0 ? (int)group_m : 8;
  const int lds = NT_RING + NT_SCRATCH + (bp ? (int)N * 2 : 0);
  auto stream = at::hip::getCurrentHIPStream();
  const bf16* ap = reinterpret_cast<const bf16*>(a.data_ptr());
  const bf16* bq = reinterpret_cast<const bf16*>(b.data_ptr());
  bf16* op = reinterpret_cast<bf16*>(out.data_ptr());
  bf16* actp = gelu ? reinterpret_cast<bf16*>(act->data_ptr()) : nullptr;
  const int mode = gelu ? 2 : (bp ? 1 : 0);
  const bool ragged = N % 256 != 0;
  auto launch = [&](auto kern) {
    static bool attr = false;  // one static per kernel instantiation (generic lambda)
    if (!attr) {
      hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                          NT_RING + NT_SCRATCH + NT_MAX_BIAS * 2);
      attr = true;
    }
    hipLaunchKernelGGL(kern, dim3(G), dim3(512), lds, stream, ap, bq, bp, op, actp, (int)M, (int)N, (int)K,
                       (int)a.stride(0), (int)b.stride(0), (int)out.stride(0), tiles_m, tiles_n, gm, (int)approx,
                       (int)ablate);
  };
#define PZ_NT(MD)                                          \
  if (ragged) launch(gemm_nt_kernel<MD, true>);            \
  else launch(gemm_nt_kernel<MD, false>);
  if (mode == 0) { PZ_NT(0) }
  else if (mode == 1) { PZ_NT(1) }
  else { PZ_NT(2) }
#undef PZ_NT
}
