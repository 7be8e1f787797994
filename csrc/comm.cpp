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
//     Optional bf16 gradient compression (``compress``; upstream DDP's bf16_compress_hook, SURVEY §5 comm notes):
//     a bucket is cast to a bf16 scratch, all-reduced in bf16 (half the xGMI bytes) and widened back into the
//     fp32 gradient, all three on the comm stream.
//   * Failure handling (the reference has none; c10d's ProcessGroupNCCL watchdog is the model): every
//     collective records a completion event on the comm stream; a watchdog thread polls those events and
//     ncclCommGetAsyncError.  A collective still pending after ``timeout_s`` (the trainer's
//     --dist-timeout) or an asynchronous RCCL error aborts the communicator (ncclCommAbort, which also
//     unblocks a host thread stuck in RCCL) and ends the process with a non-zero status, so the launcher
//     tears the group down instead of every rank hanging in a ring that will never complete.
//     async_error()/abort() stay available for explicit polling.
//   * HIP graphs: every call only enqueues work and orders streams with events, so a training step that
//     issues its collectives through this class can be captured (the comm stream joins the capture through
//     join_compute's event and leaves it through wait()); captured collectives are not watchdog-tracked, so the
//     trainer records one tracked event on the compute stream after every graph replay (track_compute).
//   * Transports: the Communicator / Bucketer logic sits on a Transport interface with two implementations --
//     RcclTransport (ncclComm_t, the production path over xGMI) and HostTransport (csrc/shm_group.h: a POSIX
//     shared-memory group, fixed rank-order reductions).  The host transport runs the SAME multi-rank C++ code
//     where RCCL cannot: ranks sharing one GPU (RCCL refuses duplicate devices; the 1-GPU DDP rehearsals) and
//     CPU-only processes with host tensors (the CPU test suite, world 2 / 4).  Its collectives are synchronous
//     (device buffers are staged through host memory behind a stream synchronisation), so it is a correctness
//     transport, not a fast one.
// RCCL is the copy PyTorch already loaded (same soname), so there is one RCCL instance per process.
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <torch/extension.h>

#include "dtypes.h"
#include "kernels/optim.h"
#include "shm_group.h"

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
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

static pdt_shm::Dt shm_type(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return pdt_shm::Dt::F32;
    case at::kDouble: return pdt_shm::Dt::F64;
    case at::kHalf: return pdt_shm::Dt::F16;
    case at::kBFloat16: return pdt_shm::Dt::BF16;
    case at::kInt: return pdt_shm::Dt::I32;
    case at::kLong: return pdt_shm::Dt::I64;
    case at::kByte: return pdt_shm::Dt::U8;
    default: TORCH_CHECK(false, "host transport: unsupported dtype ", t.scalar_type());
  }
}

static pdt_shm::Op shm_op(const std::string& op) {
  if (op == "sum") return pdt_shm::Op::Sum;
  if (op == "max") return pdt_shm::Op::Max;
  if (op == "min") return pdt_shm::Op::Min;
  if (op == "prod") return pdt_shm::Op::Prod;
  TORCH_CHECK(false, "host transport: unsupported reduction ", op);
}

// A collective backend.  Buffers are raw pointers with their element type taken from a tensor of that type
// (``proto``), so both transports see the same call; ``s`` is the stream the collective is ordered on
// (ignored by a host-memory group).
class Transport {
 public:
  virtual ~Transport() = default;
  virtual const char* name() const = 0;
  virtual bool synchronous() const = 0;  // the call has completed when it returns (no watchdog tracking needed)
  virtual void all_reduce(void* buf, int64_t n, const Tensor& proto, const std::string& op, hipStream_t s) = 0;
  virtual void broadcast(void* buf, int64_t n, const Tensor& proto, int root, hipStream_t s) = 0;
  virtual void all_gather(const void* in, void* out, int64_t n, const Tensor& proto, hipStream_t s) = 0;
  virtual int count() = 0;
  virtual std::string async_error() = 0;
  virtual void abort() = 0;
  virtual void destroy(hipStream_t s) = 0;
};

class RcclTransport final : public Transport {
 public:
  RcclTransport(const std::string& id, int world, int rank) {
    TORCH_CHECK(id.size() == sizeof(ncclUniqueId::internal), "rccl: unique id must be ", sizeof(ncclUniqueId::internal),
                " bytes");
    ncclUniqueId uid;
    std::memcpy(uid.internal, id.data(), sizeof(uid.internal));
    PDT_NCCL_CHECK(ncclCommInitRank(&comm_, world, uid, rank));
  }
  ~RcclTransport() override {
    if (comm_ && !aborted_.load()) ncclCommDestroy(comm_);
  }
  const char* name() const override { return "rccl"; }
  bool synchronous() const override { return false; }
  ncclComm_t comm() const {
    TORCH_CHECK(comm_ != nullptr && !aborted_.load(), "rccl: communicator was aborted");
    return comm_;
  }
  void all_reduce(void* buf, int64_t n, const Tensor& proto, const std::string& op, hipStream_t s) override {
    PDT_NCCL_CHECK(ncclAllReduce(buf, buf, n, nccl_type(proto), nccl_op(op), comm(), s));
  }
  void broadcast(void* buf, int64_t n, const Tensor& proto, int root, hipStream_t s) override {
    PDT_NCCL_CHECK(ncclBroadcast(buf, buf, n, nccl_type(proto), root, comm(), s));
  }
  void all_gather(const void* in, void* out, int64_t n, const Tensor& proto, hipStream_t s) override {
    PDT_NCCL_CHECK(ncclAllGather(in, out, n, nccl_type(proto), comm(), s));
  }
  int count() override {
    int n = 0;
    PDT_NCCL_CHECK(ncclCommCount(comm(), &n));
    return n;
  }
  std::string async_error() override {
    if (!comm_ || aborted_.load()) return "aborted";
    ncclResult_t e = ncclSuccess;
    PDT_NCCL_CHECK(ncclCommGetAsyncError(comm_, &e));
    return (e == ncclSuccess || e == ncclInProgress) ? std::string() : std::string(ncclGetErrorString(e));
  }
  void abort() override {
    if (comm_ && !aborted_.exchange(true)) ncclCommAbort(comm_);
  }
  void destroy(hipStream_t s) override {
    if (comm_ && !aborted_.load()) {
      if (s) PDT_HIP_OK(hipStreamSynchronize(s));
      PDT_NCCL_CHECK(ncclCommDestroy(comm_));
    }
    comm_ = nullptr;
  }

 private:
  ncclComm_t comm_ = nullptr;
  std::atomic<bool> aborted_{false};
};

// Shared-memory group over host memory.  ``device >= 0``: buffers are device memory, staged through host memory
// (D2H on the collective's stream + synchronise, host collective, H2D + synchronise).
class HostTransport final : public Transport {
 public:
  HostTransport(const std::string& name, int world, int rank, bool create, int64_t slot_bytes, double timeout_s,
                int device)
      : grp_(name, world, rank, create, (size_t)slot_bytes, timeout_s > 0 ? timeout_s : 600.0), device_(device) {
    grp_.barrier();  // every rank has mapped the segment: its name can go (no leak if a rank dies later)
    if (rank == 0) grp_.unlink();
  }
  ~HostTransport() override {
    if (stage_) (void)hipHostFree(stage_);
  }
  const char* name() const override { return "host"; }
  bool synchronous() const override { return true; }
  void all_reduce(void* buf, int64_t n, const Tensor& proto, const std::string& op, hipStream_t s) override {
    const size_t bytes = (size_t)n * proto.element_size();
    void* h = stage_in(buf, bytes, s);
    run([&] { grp_.all_reduce(h, n, shm_type(proto), shm_op(op)); });
    stage_out(buf, h, bytes, s);
  }
  void broadcast(void* buf, int64_t n, const Tensor& proto, int root, hipStream_t s) override {
    const size_t bytes = (size_t)n * proto.element_size();
    void* h = stage_in(buf, bytes, s);
    run([&] { grp_.broadcast(h, n, shm_type(proto), root); });
    stage_out(buf, h, bytes, s);
  }
  void all_gather(const void* in, void* out, int64_t n, const Tensor& proto, hipStream_t s) override {
    const size_t bytes = (size_t)n * proto.element_size();
    if (device_ < 0) {
      run([&] { grp_.all_gather(in, out, n, shm_type(proto)); });
      return;
    }
    reserve(bytes * (1 + grp_.world()));
    uint8_t* hin = static_cast<uint8_t*>(stage_);
    uint8_t* hout = hin + bytes;
    PDT_HIP_OK(hipStreamSynchronize(s));
    PDT_HIP_OK(hipMemcpyAsync(hin, in, bytes, hipMemcpyDeviceToHost, s));
    PDT_HIP_OK(hipStreamSynchronize(s));
    run([&] { grp_.all_gather(hin, hout, n, shm_type(proto)); });
    PDT_HIP_OK(hipMemcpyAsync(out, hout, bytes * grp_.world(), hipMemcpyHostToDevice, s));
    PDT_HIP_OK(hipStreamSynchronize(s));
  }
  int count() override { return grp_.world(); }
  std::string async_error() override { return grp_.aborted() ? "host group aborted by a peer" : std::string(); }
  void abort() override { grp_.abort(); }
  void destroy(hipStream_t) override {}

 private:
  template <typename F>
  void run(F&& f) {
    try {
      f();
    } catch (const std::exception& e) {
      TORCH_CHECK(false, "host transport: ", e.what());
    }
  }
  // Device buffers cross through PINNED host staging.  The stream is drained BEFORE the device-to-host copy: a copy
  // into pageable memory was observed (tests/test_ddp_numerics_gpu.py, native-2) to read the gradient before the
  // kernels the stream had been made to wait for (join_compute's event) had written it -- stale bucket contents,
  // bit-identical on every rank, so only the single-process oracle caught it.
  void* stage_in(void* buf, size_t bytes, hipStream_t s) {
    if (device_ < 0) return buf;
    reserve(bytes);
    PDT_HIP_OK(hipStreamSynchronize(s));
    PDT_HIP_OK(hipMemcpyAsync(stage_, buf, bytes, hipMemcpyDeviceToHost, s));
    PDT_HIP_OK(hipStreamSynchronize(s));
    return stage_;
  }
  void stage_out(void* buf, void* h, size_t bytes, hipStream_t s) {
    if (device_ < 0) return;
    PDT_HIP_OK(hipMemcpyAsync(buf, h, bytes, hipMemcpyHostToDevice, s));
    PDT_HIP_OK(hipStreamSynchronize(s));  // the staging buffer is reused by the next collective
  }
  void reserve(size_t bytes) {
    if (bytes <= stage_bytes_) return;
    if (stage_) PDT_HIP_OK(hipHostFree(stage_));
    stage_ = nullptr;
    PDT_HIP_OK(hipHostMalloc(&stage_, bytes, hipHostMallocDefault));
    stage_bytes_ = bytes;
  }
  pdt_shm::ShmGroup grp_;
  int device_;
  void* stage_ = nullptr;  // pinned host staging for device buffers
  size_t stage_bytes_ = 0;
};

class Communicator {
 public:
  // RCCL over the devices of the job (one rank per GPU)
  Communicator(const std::string& id, int world, int rank, int device, double timeout_s = 0.0, int exit_code = 75)
      : world_(world), rank_(rank), device_(device), timeout_s_(timeout_s), exit_code_(exit_code) {
    TORCH_CHECK(world >= 1 && rank >= 0 && rank < world, "rccl: bad rank / world");
    TORCH_CHECK(device >= 0, "rccl: a device is required");
    make_streams();
    transport_ = std::make_unique<RcclTransport>(id, world, rank);
    if (timeout_s_ > 0) {
      live_watchdogs().fetch_add(1);
      watchdog_ = std::thread([this] { watch(); });
    }
  }
  // live watchdog threads in this process (teardown checks: tests/test_end_to_end_cpu.py)
  static std::atomic<int>& live_watchdogs() {
    static std::atomic<int> n{0};
    return n;
  }
  // Host shared-memory group (``device`` < 0: host tensors only; >= 0: device tensors staged through the host)
  Communicator(std::unique_ptr<Transport> t, int world, int rank, int device, double timeout_s)
      : world_(world), rank_(rank), device_(device), timeout_s_(timeout_s), exit_code_(75) {
    if (device_ >= 0) make_streams();
    transport_ = std::move(t);
  }
  ~Communicator() {
    stop_watchdog();
    transport_.reset();
    for (auto& p : pending_)
      if (p.ev) (void)hipEventDestroy(p.ev);
    for (hipEvent_t e : free_evs_) (void)hipEventDestroy(e);
    if (ev_in_) (void)hipEventDestroy(ev_in_);
    if (ev_out_) (void)hipEventDestroy(ev_out_);
    if (stream_) (void)hipStreamDestroy(stream_);
  }
  Communicator(const Communicator&) = delete;
  Communicator& operator=(const Communicator&) = delete;

  int rank() const { return rank_; }
  int world() const { return world_; }
  int device() const { return device_; }
  hipStream_t stream() const { return stream_; }
  Transport& transport() {
    TORCH_CHECK(transport_ != nullptr, "comm: communicator was destroyed");
    return *transport_;
  }
  std::string transport_name() const { return transport_ ? transport_->name() : "destroyed"; }
  int count() { return transport().count(); }
  double timeout_s() const { return timeout_s_; }

  // Watchdog bookkeeping: a completion event on the comm stream behind the collective just enqueued.
  // Not while the caller's stream is being captured into a HIP graph: the collective is then a graph node
  // (replayed later, possibly many times) and an event recorded now would never complete as a real event.
  // Synchronous transports have nothing in flight to watch.
  void track(const std::string& what, hipStream_t on = nullptr) {
    if (timeout_s_ <= 0 || device_ < 0 || transport().synchronous()) return;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(at::hip::getCurrentHIPStream().stream(), &cap) == hipSuccess &&
        cap != hipStreamCaptureStatusNone)
      return;
    if (on == nullptr) on = stream_;
    std::lock_guard<std::mutex> lk(mu_);
    hipEvent_t ev;
    if (!free_evs_.empty()) {
      ev = free_evs_.back();
      free_evs_.pop_back();
    } else {
      PDT_HIP_OK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    }
    PDT_HIP_OK(hipEventRecord(ev, on));
    pending_.push_back({ev, std::chrono::steady_clock::now(), what});
  }
  // After a HIP-graph replay whose captured collectives the watchdog cannot see: one tracked event on the
  // compute stream, completing when the replayed step (and its collectives) did.
  void track_compute(const std::string& what) {
    if (device_ < 0) return;
    track(what, at::hip::getCurrentHIPStream().stream());
  }
  // Test hook: a pending "collective" that never completes, enqueued ``age_s`` seconds ago.
  void inject_stall(double age_s) {
    std::lock_guard<std::mutex> lk(mu_);
    auto t = std::chrono::steady_clock::now() -
             std::chrono::duration_cast<std::chrono::steady_clock::duration>(std::chrono::duration<double>(age_s));
    pending_.push_back({nullptr, t, "injected stall"});
  }
  int64_t pending() {
    std::lock_guard<std::mutex> lk(mu_);
    return (int64_t)pending_.size();
  }
  // Collective log (ordering tests): "<kind>:<stream>:<elements>" per collective in issue order, where stream is
  // "comm" (this communicator's stream, queued behind every collective issued on it before) or "inline" (the
  // caller's compute stream).  Off by default; bounded.
  void set_log(bool on) {
    std::lock_guard<std::mutex> lk(mu_);
    log_on_ = on;
    log_.clear();
  }
  std::vector<std::string> log() {
    std::lock_guard<std::mutex> lk(mu_);
    return log_;
  }
  void note(const char* kind, bool inline_stream, int64_t n) {
    std::lock_guard<std::mutex> lk(mu_);
    if (log_on_ && log_.size() < 100000)
      log_.push_back(std::string(kind) + (inline_stream ? ":inline:" : ":comm:") + std::to_string(n));
  }

  // comm stream <- everything already enqueued on the caller's compute stream
  void join_compute() {
    if (device_ < 0) return;
    hipStream_t cs = at::hip::getCurrentHIPStream().stream();
    PDT_HIP_OK(hipEventRecord(ev_in_, cs));
    PDT_HIP_OK(hipStreamWaitEvent(stream_, ev_in_, 0));
  }
  // compute stream <- every collective enqueued so far
  void wait() {
    if (device_ < 0) return;
    hipStream_t cs = at::hip::getCurrentHIPStream().stream();
    PDT_HIP_OK(hipEventRecord(ev_out_, stream_));
    PDT_HIP_OK(hipStreamWaitEvent(cs, ev_out_, 0));
  }

  void all_reduce(Tensor& t, const std::string& op, bool async_op) {
    check(t);
    join_compute();
    transport().all_reduce(t.data_ptr(), t.numel(), t, op, stream_);
    note("all_reduce", false, t.numel());
    track("all_reduce");
    if (!async_op) wait();
  }
  // In-place all-reduce enqueued on the CALLER's (compute) stream: no event hop to the comm stream and back.
  // Only for collectives whose order relative to every comm-stream collective is fixed by the compute stream
  // itself -- e.g. SyncBN forward statistics, issued while no gradient bucket is in flight -- since RCCL needs
  // the same operation order on every rank.
  void all_reduce_inline(Tensor& t, const std::string& op) {
    check(t);
    hipStream_t cs = compute_stream();
    transport().all_reduce(t.data_ptr(), t.numel(), t, op, cs);
    note("all_reduce", true, t.numel());
    track("all_reduce (compute stream)", cs);
  }
  void broadcast_inline(Tensor& t, int root) {  // on the caller's stream; same ordering contract as above
    check(t);
    hipStream_t cs = compute_stream();
    transport().broadcast(t.data_ptr(), t.numel(), t, root, cs);
    note("broadcast", true, t.numel());
    track("broadcast (compute stream)", cs);
  }
  void broadcast(Tensor& t, int root, bool async_op) {
    check(t);
    join_compute();
    transport().broadcast(t.data_ptr(), t.numel(), t, root, stream_);
    note("broadcast", false, t.numel());
    track("broadcast");
    if (!async_op) wait();
  }
  void all_gather(const Tensor& in, Tensor& out, bool async_op) {
    check(in);
    check(out);
    TORCH_CHECK(out.numel() == in.numel() * world_ && out.scalar_type() == in.scalar_type(),
                "comm all_gather: out must hold world x in");
    join_compute();
    transport().all_gather(in.data_ptr(), out.data_ptr(), in.numel(), in, stream_);
    note("all_gather", false, in.numel());
    track("all_gather");
    if (!async_op) wait();
  }
  void barrier() {
    auto opts = at::TensorOptions().dtype(at::kFloat);
    auto t = device_ >= 0 ? at::zeros({1}, opts.device(at::kCUDA, device_)) : at::zeros({1}, opts);
    all_reduce(t, "sum", false);
    if (device_ >= 0) PDT_HIP_OK(hipStreamSynchronize(at::hip::getCurrentHIPStream().stream()));
  }
  std::string async_error() {
    if (!transport_) return "aborted";
    return transport_->async_error();
  }
  // Collective teardown: every rank calls it at the same point (after a barrier).
  void destroy() {
    stop_watchdog();
    if (transport_ && !aborted_.load()) transport_->destroy(stream_);
    transport_.reset();
  }
  void abort() {
    stop_watchdog();
    if (transport_ && !aborted_.exchange(true)) transport_->abort();
  }

 private:
  struct Pending {
    hipEvent_t ev;  // nullptr: injected stall (never completes)
    std::chrono::steady_clock::time_point t;
    std::string what;  // by value: the watchdog reads it, the caller's string may change or die
  };

  void make_streams() {
    PDT_HIP_OK(hipSetDevice(device_));
    PDT_HIP_OK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    PDT_HIP_OK(hipEventCreateWithFlags(&ev_in_, hipEventDisableTiming));
    PDT_HIP_OK(hipEventCreateWithFlags(&ev_out_, hipEventDisableTiming));
  }
  hipStream_t compute_stream() const {
    return device_ >= 0 ? at::hip::getCurrentHIPStream().stream() : nullptr;
  }

  void stop_watchdog() {
    if (!watchdog_.joinable()) return;
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (watchdog_.get_id() != std::this_thread::get_id()) {
      watchdog_.join();
      live_watchdogs().fetch_sub(1);
    }
  }

  [[noreturn]] void fail(const std::string& why) {
    std::fprintf(stderr, "[pdt comm watchdog] rank %d/%d: %s; aborting the communicator and exiting (%d)\n",
                 rank_, world_, why.c_str(), exit_code_);
    std::fflush(stderr);
    if (!aborted_.exchange(true) && transport_) transport_->abort();
    std::_Exit(exit_code_);
  }

  // Poll the oldest pending collective and the transport's async error every 50 ms.
  void watch() {
    (void)hipSetDevice(device_);
    const auto limit = std::chrono::duration<double>(timeout_s_);
    std::unique_lock<std::mutex> lk(mu_);
    while (!stop_) {
      cv_.wait_for(lk, std::chrono::milliseconds(50));
      if (stop_) break;
      while (!pending_.empty()) {
        Pending& p = pending_.front();
        hipError_t q = p.ev ? hipEventQuery(p.ev) : hipErrorNotReady;
        // another thread is capturing a HIP graph (the trainer captures in thread-local mode, but be safe): the
        // query is refused, not failed -- poll again later
        if (q == hipErrorStreamCaptureUnsupported || q == hipErrorStreamCaptureImplicit ||
            q == hipErrorStreamCaptureInvalidated || q == hipErrorCapturedEvent) {
          (void)hipGetLastError();
          break;
        }
        if (q == hipSuccess) {
          free_evs_.push_back(p.ev);
          pending_.pop_front();
          continue;
        }
        if (q != hipErrorNotReady) fail(std::string("comm stream error: ") + hipGetErrorString(q));
        if (std::chrono::steady_clock::now() - p.t > limit)
          fail(std::string(p.what) + " did not complete within " + std::to_string(timeout_s_) + " s");
        break;
      }
      if (transport_ && !aborted_) {
        const std::string e = transport_->async_error();
        if (!e.empty()) fail(std::string("asynchronous transport error: ") + e);
      }
    }
  }

  void check(const Tensor& t) const {
    TORCH_CHECK(t.is_contiguous(), "comm: expected a contiguous tensor");
    if (device_ < 0) {
      TORCH_CHECK(!t.is_cuda(), "comm: host communicator got a GPU tensor");
      return;
    }
    TORCH_CHECK(t.is_cuda(), "comm: expected a GPU tensor");
    TORCH_CHECK(t.get_device() == device_, "comm: tensor on device ", t.get_device(), ", communicator on ", device_);
  }
  int world_, rank_, device_;
  double timeout_s_;
  int exit_code_;
  std::unique_ptr<Transport> transport_;
  hipStream_t stream_ = nullptr;
  hipEvent_t ev_in_ = nullptr, ev_out_ = nullptr;
  std::atomic<bool> aborted_{false};
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false;
  std::deque<Pending> pending_;
  std::vector<hipEvent_t> free_evs_;
  bool log_on_ = false;
  std::vector<std::string> log_;
  std::thread watchdog_;
};

std::shared_ptr<Communicator> make_host_communicator(const std::string& name, int world, int rank, int device,
                                                     bool create, int64_t slot_bytes, double timeout_s) {
  TORCH_CHECK(slot_bytes >= 64 && slot_bytes % 64 == 0, "host transport: slot_bytes must be a multiple of 64");
  if (device >= 0) PDT_HIP_OK(hipSetDevice(device));
  std::unique_ptr<Transport> t;
  try {
    t = std::make_unique<HostTransport>(name, world, rank, create, slot_bytes, timeout_s, device);
  } catch (const c10::Error&) {
    throw;
  } catch (const std::exception& e) {
    TORCH_CHECK(false, "host transport: ", e.what());
  }
  return std::make_shared<Communicator>(std::move(t), world, rank, device, timeout_s);
}

class Bucketer {
 public:
  Bucketer(std::shared_ptr<Communicator> comm, Tensor flat_grad, std::vector<int64_t> lo, std::vector<int64_t> hi,
           std::vector<int64_t> param_bucket, int64_t compress = 0)
      : comm_(std::move(comm)), grad_(std::move(flat_grad)), lo_(std::move(lo)), hi_(std::move(hi)),
        param_bucket_(std::move(param_bucket)), compress_(compress) {
    TORCH_CHECK(compress_ == 0 || compress_ == 1, "bucketer: compress must be 0 (fp32) or 1 (bf16)");
    const bool on_dev = comm_->device() >= 0;
    TORCH_CHECK(grad_.scalar_type() == at::kFloat && grad_.is_contiguous() && grad_.is_cuda() == on_dev,
                "bucketer: flat gradient must be a contiguous fp32 tensor on the communicator's device");
    TORCH_CHECK(!compress_ || on_dev, "bucketer: bf16 compression needs a GPU communicator");
    if (compress_) scratch_ = at::empty({grad_.numel()}, grad_.options().dtype(at::kBFloat16));
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
    --pending_[b];
    // launch strictly in bucket-index order (upstream Reducer::mark_bucket_ready / next_bucket_): a rank whose local
    // gradient-ready order differs from another's still issues the same collective sequence
    while (next_ < lo_.size() && pending_[next_] == 0) launch(next_++);
  }
  void finish() {
    while (next_ < lo_.size()) launch(next_++);  // buckets of unused parameters: reduce zeros, stay in lock-step
    comm_->wait();
    reset();
  }
  int64_t launched() const {
    int64_t n = 0;
    for (bool l : launched_) n += l;
    return n;
  }
  // bucket ids in the order their all-reduces were launched this step (tests: production order, lock-step)
  std::vector<int64_t> launch_order() const { return order_; }

 private:
  void launch(size_t b) {
    comm_->join_compute();
    float* p = grad_.data_ptr<float>() + lo_[b];
    const int64_t n = hi_[b] - lo_[b];
    Transport& tr = comm_->transport();
    if (compress_) {
      uint16_t* h = reinterpret_cast<uint16_t*>(scratch_.data_ptr()) + lo_[b];
      pdt::cast16_launch(pdt::kBF16, p, h, n, comm_->stream());
      tr.all_reduce(h, n, scratch_, "sum", comm_->stream());
      pdt::widen16_launch(pdt::kBF16, h, p, n, comm_->stream());
    } else {
      tr.all_reduce(p, n, grad_, "sum", comm_->stream());
    }
    comm_->note("bucket", false, n);
    comm_->track("gradient bucket all_reduce");
    launched_[b] = true;
    order_.push_back((int64_t)b);
  }
  void reset() {
    pending_ = nparams_;
    launched_.assign(lo_.size(), false);
    next_ = 0;
    last_order_ = order_;
    order_.clear();
  }
  std::shared_ptr<Communicator> comm_;
  Tensor grad_;
  std::vector<int64_t> lo_, hi_, param_bucket_, nparams_, pending_;
  std::vector<bool> launched_;
  size_t next_ = 0;  // next bucket index to launch
  std::vector<int64_t> order_, last_order_;
  int64_t compress_ = 0;
  Tensor scratch_;  // bf16 image of the flat gradient (compress_)

 public:
  std::vector<int64_t> last_launch_order() const { return last_order_; }
};

void register_comm(py::module& m) {
  m.def("rccl_unique_id", &unique_id);
  m.def("rccl_version", []() {
    int v = 0;
    PDT_NCCL_CHECK(ncclGetVersion(&v));
    return v;
  });
  py::class_<Communicator, std::shared_ptr<Communicator>>(m, "Communicator")
      .def(py::init<const std::string&, int, int, int, double, int>(), py::arg("uid"), py::arg("world"),
           py::arg("rank"), py::arg("device"), py::arg("timeout_s") = 0.0, py::arg("exit_code") = 75)
      .def_property_readonly("rank", &Communicator::rank)
      .def_property_readonly("world", &Communicator::world)
      .def_property_readonly("device", &Communicator::device)
      .def_property_readonly("transport", &Communicator::transport_name)
      .def_property_readonly("timeout_s", &Communicator::timeout_s)
      .def("track_compute", &Communicator::track_compute, py::arg("what") = "graph replay")
      .def("count", &Communicator::count)
      .def("pending", &Communicator::pending)
      .def("set_log", &Communicator::set_log)
      .def("log", &Communicator::log)
      .def("inject_stall", &Communicator::inject_stall)
      .def("all_reduce", &Communicator::all_reduce, py::arg("t"), py::arg("op") = "sum", py::arg("async_op") = false)
      .def("all_reduce_inline", &Communicator::all_reduce_inline, py::arg("t"), py::arg("op") = "sum")
      .def("broadcast_inline", &Communicator::broadcast_inline, py::arg("t"), py::arg("root") = 0)
      .def("broadcast", &Communicator::broadcast, py::arg("t"), py::arg("root") = 0, py::arg("async_op") = false)
      .def("all_gather", &Communicator::all_gather, py::arg("inp"), py::arg("out"), py::arg("async_op") = false)
      .def("barrier", &Communicator::barrier)
      .def("wait", &Communicator::wait)
      .def("async_error", &Communicator::async_error)
      .def("abort", &Communicator::abort)
      .def("destroy", &Communicator::destroy)
      .def_static("live_watchdogs", []() { return Communicator::live_watchdogs().load(); });
  py::class_<Bucketer>(m, "Bucketer")
      .def(py::init<std::shared_ptr<Communicator>, Tensor, std::vector<int64_t>, std::vector<int64_t>,
                    std::vector<int64_t>, int64_t>(),
           py::arg("comm"), py::arg("flat_grad"), py::arg("lo"), py::arg("hi"), py::arg("param_bucket"),
           py::arg("compress") = 0)
      .def("ready", &Bucketer::ready)
      .def("finish", &Bucketer::finish)
      .def("launched", &Bucketer::launched)
      .def("launch_order", &Bucketer::launch_order)
      .def("last_launch_order", &Bucketer::last_launch_order);
  m.def("host_communicator", &make_host_communicator, py::arg("name"), py::arg("world"), py::arg("rank"),
        py::arg("device"), py::arg("create"), py::arg("slot_bytes") = 8 << 20, py::arg("timeout_s") = 600.0);
}

}  // namespace pdt_comm
