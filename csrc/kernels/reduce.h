// Deterministic column reduction of per-workgroup partial rows: out[a][c] += Σ_g part[a][g][c].
//
// Stage 1 splits the G partial rows into S slices (grid C/256 × S × A, one column per thread,
// ≤ 16 rows each) so several hundred workgroups are in flight instead of C/64 (a single
// strided walk over 1024 partial rows ran 67–93 µs, latency-bound on 12 CUs); stage 2 adds the
// S slice sums in slice order. Fixed summation order => bitwise reproducible.
#pragma once
#include <hip/hip_runtime.h>
#include "host_plan.h"

namespace penroz {
namespace {  // internal linkage: every including translation unit gets its own copy

__global__ void __launch_bounds__(256) reduce_stage1_kernel(const float* __restrict__ part, int G, int C, int S,
                                                            float* __restrict__ mid) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int s = blockIdx.y, a = blockIdx.z;
  if (c >= C) return;
  const int per = (G + S - 1) / S;
  const int g0 = s * per, g1 = min(G, g0 + per);
  const float* p = part + (size_t)a * G * C + c;
  float acc = 0.f;
  for (int g = g0; g < g1; ++g) acc += p[(size_t)g * C];
  mid[((size_t)a * S + s) * C + c] = acc;
}

struct OutPtrs {
  float* p[3];
};

__global__ void __launch_bounds__(256) reduce_stage2_kernel(const float* __restrict__ mid, int C, int S, OutPtrs outs) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int a = blockIdx.y;
  if (c >= C) return;
  float acc = 0.f;
  for (int s = 0; s < S; ++s) acc += mid[((size_t)a * S + s) * C + c];
  outs.p[a][c] += acc;
}

// part: [A][G][C] fp32 (A <= 3); outs[a] fp32 [C] (accumulated into). `mid` needs A*S*C floats.
inline void reduce_partials_add(const float* part, int A, int G, int C, float* const* outs, float* mid, int S,
                                hipStream_t stream) {
  OutPtrs o{};
  for (int a = 0; a < A; ++a) o.p[a] = outs[a];
  dim3 g1((C + 255) / 256, S, A), g2((C + 255) / 256, A);
  hipLaunchKernelGGL(reduce_stage1_kernel, g1, dim3(256), 0, stream, part, G, C, S, mid);
  hipLaunchKernelGGL(reduce_stage2_kernel, g2, dim3(256), 0, stream, mid, C, S, o);
}

}  // namespace
}  // namespace penroz
