// Probe: cost of a device-wide barrier inside one persistent kernel (one workgroup per CU) vs a
// kernel boundary in a replayed HIP graph. Decides whether a persistent decode step (one launch,
// grid barriers between its phases) can beat ~64 graph-replayed kernels per step.
//   hipcc --offload-arch=gfx950 -O3 bench/probes/grid_barrier_probe.hip -o /tmp/gbp && /tmp/gbp
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

struct Bar { unsigned count; unsigned gen; unsigned err; unsigned pad; };

// sense-free generation barrier: the last arriver resets the count and bumps the generation
__device__ __forceinline__ void grid_sync(Bar* b, unsigned nwg) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned gen = __hip_atomic_load(&b->gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    if (__hip_atomic_fetch_add(&b->count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == nwg - 1) {
      __hip_atomic_store(&b->count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&b->gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      unsigned spins = 0;
      while (__hip_atomic_load(&b->gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == gen) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 24)) {  // ~1 s: give up (no hang), flag it
          __hip_atomic_fetch_add(&b->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
  }
  __syncthreads();
}

__global__ void __launch_bounds__(256) persistent(Bar* b, int nbar, float* sink) {
  float acc = threadIdx.x;
  for (int i = 0; i < nbar; ++i) {
    acc = acc * 1.0001f + 1.f;
    grid_sync(b, gridDim.x);
  }
  if (acc == 12345.f) sink[0] = acc;
}

__global__ void __launch_bounds__(256) tiny(float* sink, int i) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && i < 0) sink[0] = 1.f;
}

int main() {
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int ncu = prop.multiProcessorCount;
  int occ = 0;
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, persistent, 256, 0);
  printf("CUs %d, occupancy %d wg/CU\n", ncu, occ);
  Bar* b; float* sink;
  hipMalloc(&b, sizeof(Bar)); hipMemset(b, 0, sizeof(Bar));
  hipMalloc(&sink, 4);
  hipStream_t s; hipStreamCreate(&s);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int grid : {ncu / 2, ncu}) {
    for (int nbar : {0, 60, 600}) {
      hipLaunchKernelGGL(persistent, dim3(grid), dim3(256), 0, s, b, nbar, sink);
      hipStreamSynchronize(s);
      hipEventRecord(e0, s);
      for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(persistent, dim3(grid), dim3(256), 0, s, b, nbar, sink);
      hipEventRecord(e1, s);
      hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      Bar hb; hipMemcpy(&hb, b, sizeof(Bar), hipMemcpyDeviceToHost);
      printf("persistent grid %d: %d barriers: %.2f us per launch (err %u)\n", grid, nbar, ms * 1000 / 20, hb.err);
    }
  }
  // graph of 64 tiny kernels of 192 workgroups, replayed
  for (int wgs : {192, 768}) {
    hipGraph_t g; hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    for (int i = 0; i < 64; ++i) hipLaunchKernelGGL(tiny, dim3(wgs), dim3(256), 0, s, sink, i);
    hipStreamEndCapture(s, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    hipGraphLaunch(ge, s); hipStreamSynchronize(s);
    hipEventRecord(e0, s);
    for (int r = 0; r < 20; ++r) hipGraphLaunch(ge, s);
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("graph of 64 empty kernels x %d wgs: %.2f us per replay (%.2f us per kernel)\n", wgs, ms * 1000 / 20,
           ms * 1000 / 20 / 64);
  }
  return 0;
}
