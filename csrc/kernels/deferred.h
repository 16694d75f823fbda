// Deferred (side-stream) finishing of gradient column reductions.
//
// LayerNorm backward and the GELU-backward / column-sum kernels write per-workgroup partial
// rows and finish them with the two small reduce kernels of reduce.h. Those sums are PARAMETER
// gradients (dγ, dβ, biases): nothing later in the backward reads them, so while the fused
// executor's backward runs, the finishing kernels can go to its side stream (the one running the
// weight-gradient GEMMs) instead of sitting on the critical path: the side stream waits for the
// producer with an event, and the partial buffers are recorded on it for the caching allocator.
// set_deferred_reduce_stream(0) (the default) keeps everything on the current stream.
#pragma once
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPStream.h>
#include "reduce.h"

namespace penroz {

struct DeferredReduce {
  hipStream_t stream = nullptr;
  int device = 0;
};
DeferredReduce& deferred_reduce();  // defined in elementwise.hip

// out[a][c] += Σ_g part[a][g][c] for a < A (part fp32 [A][G][C]); on the deferred stream if set
inline void reduce_partials_auto(const torch::Tensor& part, int A, int G, int C, float* const* outs, hipStream_t cur) {
  const int S = reduce_slices(G);
  auto mid = torch::empty({A, S, C}, part.options());
  hipStream_t rs = cur;
  const DeferredReduce& d = deferred_reduce();
  if (d.stream != nullptr && d.stream != cur) {
    hipEvent_t e;
    TORCH_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess, "hipEventCreate failed");
    TORCH_CHECK(hipEventRecord(e, cur) == hipSuccess && hipStreamWaitEvent(d.stream, e, 0) == hipSuccess,
                "deferred reduce: event ordering failed");
    hipEventDestroy(e);  // released once the wait has been satisfied
    auto hs = c10::hip::getStreamFromExternal(d.stream, (c10::DeviceIndex)d.device);
    c10::hip::HIPCachingAllocator::recordStream(part.storage().data_ptr(), hs);
    c10::hip::HIPCachingAllocator::recordStream(mid.storage().data_ptr(), hs);
    rs = d.stream;
  }
  reduce_partials_add(part.data_ptr<float>(), A, G, C, outs, mid.data_ptr<float>(), S, rs);
}

}  // namespace penroz
