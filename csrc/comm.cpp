// Native collective layer over RCCL (xGMI inside an MI355X node): our own communicator on our own HIP
// stream, and a gradient bucketer in C++ -- the MI355X-native counterparts of c10d ProcessGroupNCCL and
// the DDP Reducer that the reference relies on.
//
//   * Communicator: one ncclComm_t per process (unique id exchanged through the launcher's TCP store),
//     a dedicated non-blocking comm stream, and event-based ordering: a collective is enqueued behind
//     everything already on the caller's (compute) stream, and wait() makes the compute stream wait for
//     the comm stream -- no host synchronisation anywhere.
//   * Bucketer: buckets are contiguous element ranges of the flat fp32 gradient buffer (grads are
//     bucket views, no copy-in/copy-out); ready(pid) counts a parameter's gradient as produced and
//     launches that bucket's all-reduce (in place, SUM; 1/world is folded into the SGD kernel) as soon as
//     its count reaches zero, so the reductions overlap the rest of backward; finish() launches leftover
//     buckets (unused parameters) and joins the comm stream into the compute stream.
//   * Failure handling: async_error() polls ncclCommGetAsyncError; abort() tears the communicator down
//     (ncclCommAbort) so a hung peer cannot wedge this process forever.
// RCCL is the copy PyTorch already loaded (same soname), so there is one RCCL instance per process.
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <torch/extension.h>

#include <cstring>
#include <memory>
#include <string>
#include <vector>

namespace pdt_comm {

namespace py = pybind11;
using at::Tensor;

#define PDT_NCCL_CHECK(expr)                                                                     \
  do {                                                                                           \
    ncclResult_t _r = (expr);                                                                    \
    TORCH_CHECK(_r == ncclSuccess, #expr " failed: ", ncclGetErrorString(_r));                   \
  } while (0)
#define PDT_HIP_OK(expr)                                                                         \
  do {                                                                                           \
    hipError_t _e = (expr);                                                                      \
    TORCH_CHECK(_e == hipSuccess, #expr " failed: ", hipGetErrorString(_e));                     \
  } while (0)

static ncclDataType_t nccl_type(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kDouble: return ncclFloat64;
    case at::kHalf: return ncclFloat16;
    case at::kBFloat16: return ncclBfloat16;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kByte: return ncclUint8;
    default: TORCH_CHECK(false, "rccl: unsupported dtype ", t.scalar_type());
  }
}

static ncclRedOp_t nccl_op(const std::string& op) {
  if (op == "sum") return ncclSum;
  if (op == "max") return ncclMax;
  if (op == "min") return ncclMin;
  if (op == "prod") return ncclProd;
  TORCH_CHECK(false, "rccl: unsupported reduction ", op);
}

py::bytes unique_id() {
  ncclUniqueId id;
  PDT_NCCL_CHECK(ncclGetUniqueId(&id));
  return py::bytes(id.internal, sizeof(id.internal));
}

class Communicator {
 public:
  Communicator(const std::string& id, int world, int rank, int device) : world_(world), rank_(rank), device_(device) {
    TORCH_CHECK(id.size() == sizeof(ncclUniqueId::internal), "rccl: unique id must be ", sizeof(ncclUniqueId::internal),
                " bytes");
    TORCH_CHECK(world >= 1 && rank >= 0 && rank < world, "rccl: bad rank / world");
    ncclUniqueId uid;
    std::memcpy(uid.internal, id.data(), sizeof(uid.internal));
    PDT_HIP_OK(hipSetDevice(device));
    PDT_HIP_OK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    PDT_HIP_OK(hipEventCreateWithFlags(&ev_in_, hipEventDisableTiming));
    PDT_HIP_OK(hipEventCreateWithFlags(&ev_out_, hipEventDisableTiming));
    PDT_NCCL_CHECK(ncclCommInitRank(&comm_, world, uid, rank));
  }
  ~Communicator() {
    if (comm_) ncclCommDestroy(comm_);
    if (ev_in_) (void)hipEventDestroy(ev_in_);
    if (ev_out_) (void)hipEventDestroy(ev_out_);
    if (stream_) (void)hipStreamDestroy(stream_);
  }
  Communicator(const Communicator&) = delete;
  Communicator& operator=(const Communicator&) = delete;

  int rank() const { return rank_; }
  int world() const { return world_; }
  hipStream_t stream() const { return stream_; }
  ncclComm_t comm() const {
    TORCH_CHECK(comm_ != nullptr, "rccl: communicator was aborted");
    return comm_;
  }

  // comm stream <- everything already enqueued on the caller's compute stream
  void join_compute() {
    hipStream_t cs = at::hip::getCurrentHIPStream().stream();
    PDT_HIP_OK(hipEventRecord(ev_in_, cs));
    PDT_HIP_OK(hipStreamWaitEvent(stream_, ev_in_, 0));
  }
  // compute stream <- every collective enqueued so far
  void wait() {
    hipStream_t cs = at::hip::getCurrentHIPStream().stream();
    PDT_HIP_OK(hipEventRecord(ev_out_, stream_));
    PDT_HIP_OK(hipStreamWaitEvent(cs, ev_out_, 0));
  }

  void all_reduce(Tensor& t, const std::string& op, bool async_op) {
    check(t);
    join_compute();
    PDT_NCCL_CHECK(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), nccl_type(t), nccl_op(op), comm(), stream_));
    if (!async_op) wait();
  }
  void broadcast(Tensor& t, int root, bool async_op) {
    check(t);
    join_compute();
    PDT_NCCL_CHECK(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), nccl_type(t), root, comm(), stream_));
    if (!async_op) wait();
  }
  void all_gather(const Tensor& in, Tensor& out, bool async_op) {
    check(in);
    check(out);
    TORCH_CHECK(out.numel() == in.numel() * world_ && out.scalar_type() == in.scalar_type(),
                "rccl all_gather: out must hold world x in");
    join_compute();
    PDT_NCCL_CHECK(ncclAllGather(in.data_ptr(), out.data_ptr(), in.numel(), nccl_type(in), comm(), stream_));
    if (!async_op) wait();
  }
  void barrier() {
    auto t = at::zeros({1}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, device_));
    all_reduce(t, "sum", false);
    PDT_HIP_OK(hipStreamSynchronize(at::hip::getCurrentHIPStream().stream()));
  }
  std::string async_error() {
    if (!comm_) return "aborted";
    ncclResult_t e = ncclSuccess;
    PDT_NCCL_CHECK(ncclCommGetAsyncError(comm_, &e));
    return e == ncclSuccess ? std::string() : std::string(ncclGetErrorString(e));
  }
  void abort() {
    if (comm_) {
      ncclCommAbort(comm_);
      comm_ = nullptr;
    }
  }

 private:
  void check(const Tensor& t) const {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "rccl: expected a contiguous GPU tensor");
    TORCH_CHECK(t.get_device() == device_, "rccl: tensor on device ", t.get_device(), ", communicator on ", device_);
  }
  int world_, rank_, device_;
  ncclComm_t comm_ = nullptr;
  hipStream_t stream_ = nullptr;
  hipEvent_t ev_in_ = nullptr, ev_out_ = nullptr;
};

class Bucketer {
 public:
  Bucketer(std::shared_ptr<Communicator> comm, Tensor flat_grad, std::vector<int64_t> lo, std::vector<int64_t> hi,
           std::vector<int64_t> param_bucket)
      : comm_(std::move(comm)), grad_(std::move(flat_grad)), lo_(std::move(lo)), hi_(std::move(hi)),
        param_bucket_(std::move(param_bucket)) {
    TORCH_CHECK(grad_.is_cuda() && grad_.scalar_type() == at::kFloat && grad_.is_contiguous(),
                "bucketer: flat gradient must be a contiguous fp32 GPU tensor");
    TORCH_CHECK(lo_.size() == hi_.size() && !lo_.empty(), "bucketer: bad bucket ranges");
    nparams_.assign(lo_.size(), 0);
    for (int64_t b : param_bucket_) {
      TORCH_CHECK(b >= 0 && b < (int64_t)lo_.size(), "bucketer: parameter bucket id out of range");
      ++nparams_[b];
    }
    for (size_t b = 0; b < lo_.size(); ++b)
      TORCH_CHECK(0 <= lo_[b] && lo_[b] < hi_[b] && hi_[b] <= grad_.numel(), "bucketer: bucket outside the buffer");
    reset();
  }
  void ready(int64_t pid) {
    TORCH_CHECK(pid >= 0 && pid < (int64_t)param_bucket_.size(), "bucketer: bad parameter id");
    const int64_t b = param_bucket_[pid];
    TORCH_CHECK(pending_[b] > 0, "bucketer: parameter ", pid, " reported ready twice in one step");
    if (--pending_[b] == 0) launch(b);
  }
  void finish() {
    for (size_t b = 0; b < lo_.size(); ++b)
      if (!launched_[b]) launch(b);  // buckets of unused parameters: reduce zeros, stay in lock-step
    comm_->wait();
    reset();
  }
  int64_t launched() const {
    int64_t n = 0;
    for (bool l : launched_) n += l;
    return n;
  }

 private:
  void launch(size_t b) {
    comm_->join_compute();
    float* p = grad_.data_ptr<float>() + lo_[b];
    PDT_NCCL_CHECK(ncclAllReduce(p, p, hi_[b] - lo_[b], ncclFloat32, ncclSum, comm_->comm(), comm_->stream()));
    launched_[b] = true;
  }
  void reset() {
    pending_ = nparams_;
    launched_.assign(lo_.size(), false);
  }
  std::shared_ptr<Communicator> comm_;
  Tensor grad_;
  std::vector<int64_t> lo_, hi_, param_bucket_, nparams_, pending_;
  std::vector<bool> launched_;
};

void register_comm(py::module& m) {
  m.def("rccl_unique_id", &unique_id);
  m.def("rccl_version", []() {
    int v = 0;
    PDT_NCCL_CHECK(ncclGetVersion(&v));
    return v;
  });
  py::class_<Communicator, std::shared_ptr<Communicator>>(m, "Communicator")
      .def(py::init<const std::string&, int, int, int>())
      .def_property_readonly("rank", &Communicator::rank)
      .def_property_readonly("world", &Communicator::world)
      .def("all_reduce", &Communicator::all_reduce, py::arg("t"), py::arg("op") = "sum", py::arg("async_op") = false)
      .def("broadcast", &Communicator::broadcast, py::arg("t"), py::arg("root") = 0, py::arg("async_op") = false)
      .def("all_gather", &Communicator::all_gather, py::arg("inp"), py::arg("out"), py::arg("async_op") = false)
      .def("barrier", &Communicator::barrier)
      .def("wait", &Communicator::wait)
      .def("async_error", &Communicator::async_error)
      .def("abort", &Communicator::abort);
  py::class_<Bucketer>(m, "Bucketer")
      .def(py::init<std::shared_ptr<Communicator>, Tensor, std::vector<int64_t>, std::vector<int64_t>,
                    std::vector<int64_t>>())
      .def("ready", &Bucketer::ready)
      .def("finish", &Bucketer::finish)
      .def("launched", &Bucketer::launched);
}

}  // namespace pdt_comm
