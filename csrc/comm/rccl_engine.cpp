// N1/N2: native RCCL communicator for data-parallel training on MI355X.
//
// One Engine per process (one process per GPU).  It owns
//   * an RCCL communicator built with ncclCommInitRank from a unique id that rank 0 generates and the
//     Python side ships through the c10d store (parallel/comm.py);
//   * a dedicated non-blocking HIP stream at the device's highest priority, so RCCL's kernels are
//     scheduled ahead of the backward GEMMs that share the CUs with them;
//   * a pool of HIP events.
// A collective is ordered after the work already queued on the caller's (torch current) stream by an
// event -> hipStreamWaitEvent, runs on the comm stream, and records a completion event.  wait(h) makes
// the caller's stream wait for that event on the device -- no host synchronisation anywhere on the
// gradient path, so bucket all-reduces overlap the rest of the backward pass.
//
// xGMI note: inside an MI355X node every GPU pair has its own link (7 x ~153 GB/s per GPU); RCCL's
// rings/trees stripe one collective over several channels, so fewer, larger buckets (tens of MB) keep
// all links busy -- bucket sizing lives in parallel/ddp.py, the bus-bandwidth sweep in
// tools/comm_bench.py (bench_all_reduce below).
#include <torch/extension.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace {

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error in ") + what + ": " + hipGetErrorString(e));
}

void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string("RCCL error in ") + what + ": " + ncclGetErrorString(r));
}

ncclDataType_t to_nccl(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kDouble: return ncclFloat64;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kByte: return ncclUint8;
    default: throw std::runtime_error("rccl engine: unsupported dtype");
  }
}

ncclRedOp_t to_op(const std::string& op) {
  if (op == "sum") return ncclSum;
  if (op == "max") return ncclMax;
  if (op == "min") return ncclMin;
  if (op == "prod") return ncclProd;
  if (op == "avg") return ncclAvg;
  throw std::runtime_error("rccl engine: unknown reduction " + op);
}

py::bytes unique_id() {
  ncclUniqueId id;
  nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  return py::bytes(id.internal, NCCL_UNIQUE_ID_BYTES);
}

class Engine {
 public:
  Engine(const std::string& uid, int rank, int world, int device) : rank_(rank), world_(world), device_(device) {
    if (uid.size() != NCCL_UNIQUE_ID_BYTES) throw std::runtime_error("rccl engine: bad unique id size");
    hip_check(hipSetDevice(device), "hipSetDevice");
    int least = 0, greatest = 0;
    hip_check(hipDeviceGetStreamPriorityRange(&least, &greatest), "hipDeviceGetStreamPriorityRange");
    hip_check(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, greatest), "hipStreamCreateWithPriority");
    ncclUniqueId id;
    std::memcpy(id.internal, uid.data(), NCCL_UNIQUE_ID_BYTES);
    nccl_check(ncclCommInitRank(&comm_, world, id, rank), "ncclCommInitRank");
  }

  // Nothing is torn down implicitly: the destructor may run during interpreter finalisation, after
  // the HIP runtime / RCCL proxies are gone.  The stream and events live as long as the process
  // because the caching allocator keeps recorded-stream references to blocks freed later.
  ~Engine() = default;

  void shutdown() {
    if (comm_) {
      hipStreamSynchronize(stream_);
      ncclCommDestroy(comm_);
      comm_ = nullptr;
    }
  }

  int rank() const { return rank_; }
  int world() const { return world_; }
  int64_t stream_ptr() const { return reinterpret_cast<int64_t>(stream_); }

  // out-of-place or in-place all-reduce; returns a completion handle
  int all_reduce(at::Tensor& t, const std::string& op) {
    check_tensor(t);
    begin(t);
    nccl_check(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), to_op(op), comm_,
                             stream_),
               "ncclAllReduce");
    return finish();
  }

  int broadcast(at::Tensor& t, int root) {
    check_tensor(t);
    begin(t);
    nccl_check(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), root, comm_, stream_),
               "ncclBroadcast");
    return finish();
  }

  // out [world * n] <- every rank's inp [n]
  int all_gather(at::Tensor& out, const at::Tensor& inp) {
    check_tensor(out);
    check_tensor(inp);
    TORCH_CHECK(out.numel() == inp.numel() * world_ && out.scalar_type() == inp.scalar_type(), "all_gather: shapes");
    begin(inp);
    record(out);
    nccl_check(ncclAllGather(inp.data_ptr(), out.data_ptr(), inp.numel(), to_nccl(inp.scalar_type()), comm_, stream_),
               "ncclAllGather");
    return finish();
  }

  // out [n] <- reduction over ranks of inp[rank * n : (rank + 1) * n]
  int reduce_scatter(at::Tensor& out, const at::Tensor& inp, const std::string& op) {
    check_tensor(out);
    check_tensor(inp);
    TORCH_CHECK(inp.numel() == out.numel() * world_ && out.scalar_type() == inp.scalar_type(), "reduce_scatter: shapes");
    begin(inp);
    record(out);
    nccl_check(ncclReduceScatter(inp.data_ptr(), out.data_ptr(), out.numel(), to_nccl(out.scalar_type()), to_op(op),
                                 comm_, stream_),
               "ncclReduceScatter");
    return finish();
  }

  // the caller's current stream waits (on the device) for collective h
  void wait(int h) {
    auto cur = c10::hip::getCurrentHIPStream(device_).stream();
    hip_check(hipStreamWaitEvent(cur, event(h), 0), "hipStreamWaitEvent");
  }

  void synchronize(int h) { hip_check(hipEventSynchronize(event(h)), "hipEventSynchronize"); }

  bool query(int h) {
    auto r = hipEventQuery(event(h));
    if (r == hipErrorNotReady) return false;
    hip_check(r, "hipEventQuery");
    return true;
  }

  // handles are recycled after reset(): call once per step after every wait()
  void reset() { next_ = 0; }

  // bus bandwidth probe on the comm stream (tools/comm_bench.py): seconds per all-reduce of n elements
  double bench_all_reduce(at::Tensor& t, int iters) {
    check_tensor(t);
    hip_check(hipStreamSynchronize(stream_), "sync");
    nccl_check(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), ncclSum, comm_, stream_),
               "warmup");
    hip_check(hipStreamSynchronize(stream_), "sync");
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; ++i)
      nccl_check(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), ncclSum, comm_,
                               stream_),
                 "ncclAllReduce");
    hip_check(hipStreamSynchronize(stream_), "sync");
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / iters;
  }

 private:
  void check_tensor(const at::Tensor& t) const {
    TORCH_CHECK(t.is_cuda() && t.get_device() == device_, "rccl engine: tensor must live on this rank's GPU");
    TORCH_CHECK(t.is_contiguous(), "rccl engine: tensor must be contiguous");
    TORCH_CHECK(comm_ != nullptr, "rccl engine: communicator is shut down");
  }

  hipEvent_t event(int h) {
    TORCH_CHECK(h >= 0 && h < (int)events_.size(), "rccl engine: bad handle");
    return events_[h];
  }

  hipEvent_t take() {
    if (next_ == (int)events_.size()) {
      hipEvent_t e;
      hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
      events_.push_back(e);
    }
    return events_[next_++];
  }

  // order the collective after the caller's queued work; keep the allocator from recycling the memory
  // while the comm stream may still touch it
  void begin(const at::Tensor& t) {
    auto cur = c10::hip::getCurrentHIPStream(device_).stream();
    hipEvent_t ready = take();
    hip_check(hipEventRecord(ready, cur), "hipEventRecord");
    hip_check(hipStreamWaitEvent(stream_, ready, 0), "hipStreamWaitEvent");
    record(t);
  }

  void record(const at::Tensor& t) {
    c10::hip::HIPCachingAllocator::recordStream(t.storage().data_ptr(),
                                                c10::hip::getStreamFromExternal(stream_, device_));
  }

  int finish() {
    const int h = next_;
    hip_check(hipEventRecord(take(), stream_), "hipEventRecord");
    return h;
  }

  int rank_, world_, device_;
  ncclComm_t comm_ = nullptr;
  hipStream_t stream_ = nullptr;
  std::vector<hipEvent_t> events_;
  int next_ = 0;
};

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "finetune_controller_amd native RCCL engine (dedicated high-priority comm stream, event ordering)";
  m.def("unique_id", &unique_id);
  m.def("version", [] {
    int v = 0;
    ncclGetVersion(&v);
    return v;
  });
  py::class_<Engine>(m, "Engine")
      .def(py::init<const std::string&, int, int, int>(), py::arg("uid"), py::arg("rank"), py::arg("world"),
           py::arg("device"))
      .def_property_readonly("rank", &Engine::rank)
      .def_property_readonly("world", &Engine::world)
      .def_property_readonly("stream_ptr", &Engine::stream_ptr)
      .def("all_reduce", &Engine::all_reduce, py::arg("t"), py::arg("op") = "sum")
      .def("broadcast", &Engine::broadcast, py::arg("t"), py::arg("root") = 0)
      .def("all_gather", &Engine::all_gather)
      .def("reduce_scatter", &Engine::reduce_scatter, py::arg("out"), py::arg("inp"), py::arg("op") = "sum")
      .def("wait", &Engine::wait)
      .def("synchronize", &Engine::synchronize)
      .def("query", &Engine::query)
      .def("reset", &Engine::reset)
      .def("bench_all_reduce", &Engine::bench_all_reduce)
      .def("shutdown", &Engine::shutdown);
}
