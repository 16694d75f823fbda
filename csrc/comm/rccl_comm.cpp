// Native RCCL communicator for gradient synchronisation over xGMI (module ``penroz_comm``).
//
// Owns an ncclComm_t (RCCL is ROCm's NCCL) created from a unique id that rank 0 publishes
// through the torch.distributed TCPStore, and a dedicated high-priority non-blocking HIP
// stream. all_reduce_avg_async() fences the comm stream behind the producer's current stream
// with an event (so a bucket's all-reduce starts as soon as the kernels that wrote it finish,
// while the compute stream runs on) and launches ncclAllReduce(ncclAvg) in place, then records a
// completion event and returns its handle: wait(handle) makes the compute stream wait for that
// one collective (the optimizer updates bucket i as soon as bucket i has landed), wait_all()
// for everything launched so far.
// This replaces the reference's implicit C++ DDP Reducer + ProcessGroupNCCL
// (``neural_net_model.py:609``) with an explicit, bucket-granular, stream-ordered design.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <stdexcept>
#include <string>
#include <vector>

#define HIP_OK(x)                                                                            \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) throw std::runtime_error(std::string("HIP: ") + hipGetErrorString(e_)); \
  } while (0)
#define NCCL_OK(x)                                                                           \
  do {                                                                                       \
    ncclResult_t r_ = (x);                                                                   \
    if (r_ != ncclSuccess) throw std::runtime_error(std::string("RCCL: ") + ncclGetErrorString(r_)); \
  } while (0)

static ncclDataType_t to_nccl(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kDouble: return ncclFloat64;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    default: throw std::runtime_error("unsupported dtype for RCCL");
  }
}

class RcclComm {
 public:
  // channels > 0: the communicator is built with exactly that many channels (RCCL CTAs:
  // ncclConfig_t minCTAs = maxCTAs), the per-communicator form of NCCL_MIN/MAX_NCHANNELS — the
  // environment variables are read once per process, so the first-contact sweep compares
  // channel counts with one communicator each
  RcclComm(const std::string& id_bytes, int rank, int world, int device, int channels = 0)
      : rank_(rank), world_(world), device_(device), channels_(channels) {
    if (id_bytes.size() != sizeof(ncclUniqueId)) throw std::runtime_error("bad RCCL unique id size");
    ncclUniqueId id;
    std::memcpy(&id, id_bytes.data(), sizeof(id));
    HIP_OK(hipSetDevice(device));
    int lo = 0, hi = 0;
    HIP_OK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIP_OK(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, hi));  // highest priority
    if (channels > 0) {
      ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
      cfg.minCTAs = channels;
      cfg.maxCTAs = channels;
      NCCL_OK(ncclCommInitRankConfig(&comm_, world, id, rank, &cfg));
    } else {
      NCCL_OK(ncclCommInitRank(&comm_, world, id, rank));
    }
  }

  ~RcclComm() {
    if (comm_) ncclCommDestroy(comm_);
    comm_ = nullptr;
    for (auto e : events_) hipEventDestroy(e);
    for (auto e : done_) hipEventDestroy(e);
    if (stream_) hipStreamDestroy(stream_);
  }

  static std::string unique_id() {
    ncclUniqueId id;
    NCCL_OK(ncclGetUniqueId(&id));
    return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
  }

  // in-place average of `t` across ranks, ordered after the current torch stream's work;
  // returns the handle of its completion event (valid until wait_all() / reset_handles())
  int64_t all_reduce_avg_async(torch::Tensor t) {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "RCCL all-reduce needs a contiguous GPU tensor");
    fence_from_current();
    NCCL_OK(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), ncclAvg, comm_, stream_));
    ++pending_;
    return record_done();
  }

  int64_t all_reduce_sum_async(torch::Tensor t) {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous());
    fence_from_current();
    NCCL_OK(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), ncclSum, comm_, stream_));
    ++pending_;
    return record_done();
  }

  // the current torch stream waits for the collective with this handle only
  void wait(int64_t handle) {
    TORCH_CHECK(handle >= 0 && handle < n_done_, "unknown collective handle ", handle);
    HIP_OK(hipStreamWaitEvent(at::hip::getCurrentHIPStream().stream(), done_[handle], 0));
  }

  // forget the handles (their events are re-recorded by later collectives)
  void reset_handles() { n_done_ = 0; }

  void broadcast(torch::Tensor t, int root) {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous());
    fence_from_current();
    NCCL_OK(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), root, comm_, stream_));
    ++pending_;
    wait_all();
  }

  // the current torch stream waits for every collective launched so far
  void wait_all() {
    if (pending_ == 0) return;
    hipEvent_t e = next_event();
    HIP_OK(hipEventRecord(e, stream_));
    HIP_OK(hipStreamWaitEvent(at::hip::getCurrentHIPStream().stream(), e, 0));
    pending_ = 0;
    n_done_ = 0;
  }

  void synchronize() { HIP_OK(hipStreamSynchronize(stream_)); }

  // tear the communicator down WITHOUT waiting for collectives in flight (a peer that never
  // enqueued its side would leave them hanging forever); the object is unusable afterwards
  void abort() {
    if (comm_) ncclCommAbort(comm_);
    comm_ = nullptr;
    pending_ = 0;
    n_done_ = 0;
  }
  int rank() const { return rank_; }
  int world() const { return world_; }
  int channels() const { return channels_; }
  // what RCCL itself says about the communicator (not what the caller passed in): the rank count
  // of the clique, this member's rank and the device it is bound to
  int nranks() const {
    int n = 0;
    NCCL_OK(ncclCommCount(comm_, &n));
    return n;
  }
  int comm_rank() const {
    int r = -1;
    NCCL_OK(ncclCommUserRank(comm_, &r));
    return r;
  }
  int comm_device() const {
    int d = -1;
    NCCL_OK(ncclCommCuDevice(comm_, &d));
    return d;
  }

 private:
  void fence_from_current() {
    hipEvent_t e = next_event();
    HIP_OK(hipEventRecord(e, at::hip::getCurrentHIPStream().stream()));
    HIP_OK(hipStreamWaitEvent(stream_, e, 0));
  }

  // one completion event per collective since the last reset (a bucket plan has tens)
  int64_t record_done() {
    if (n_done_ == (int64_t)done_.size()) {
      hipEvent_t e;
      HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      done_.push_back(e);
    }
    HIP_OK(hipEventRecord(done_[n_done_], stream_));
    return n_done_++;
  }

  hipEvent_t next_event() {
    // a small ring of events; an event may be re-recorded once its previous waits were issued
    if (events_.size() < 64) {
      hipEvent_t e;
      HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      events_.push_back(e);
      return e;
    }
    hipEvent_t e = events_[ring_++ % events_.size()];
    return e;
  }

  int rank_, world_, device_, channels_;
  ncclComm_t comm_ = nullptr;
  hipStream_t stream_ = nullptr;
  std::vector<hipEvent_t> events_;
  std::vector<hipEvent_t> done_;
  int64_t n_done_ = 0;
  size_t ring_ = 0;
  int pending_ = 0;
};

PYBIND11_MODULE(penroz_comm, m) {
  m.doc() = "penroz native RCCL communicator (xGMI gradient all-reduce on a dedicated HIP stream)";
  pybind11::class_<RcclComm>(m, "RcclComm")
      .def(pybind11::init<const std::string&, int, int, int, int>(), pybind11::arg("id"), pybind11::arg("rank"),
           pybind11::arg("world"), pybind11::arg("device"), pybind11::arg("channels") = 0)
      .def_static("unique_id", [] { return pybind11::bytes(RcclComm::unique_id()); })
      .def("all_reduce_avg_async", &RcclComm::all_reduce_avg_async)
      .def("all_reduce_sum_async", &RcclComm::all_reduce_sum_async)
      .def("broadcast", &RcclComm::broadcast)
      .def("wait", &RcclComm::wait)
      .def("reset_handles", &RcclComm::reset_handles)
      .def("wait_all", &RcclComm::wait_all)
      .def("synchronize", &RcclComm::synchronize)
      .def("abort", &RcclComm::abort)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("world", &RcclComm::world)
      .def_property_readonly("channels", &RcclComm::channels)
      .def_property_readonly("nranks", &RcclComm::nranks)
      .def_property_readonly("comm_rank", &RcclComm::comm_rank)
      .def_property_readonly("comm_device", &RcclComm::comm_device);
  m.def("version", [] {
    int v = 0;
    ncclGetVersion(&v);
    return v;
  });
}
