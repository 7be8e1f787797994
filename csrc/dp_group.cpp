// Single-process multi-GPU collectives for the DataParallel engine (reference C09, `dataparallel.py:119`;
// SURVEY §2.3 DP row, §2.7 "DP engine: ncclCommInitAll, per-device threads/streams").
//
// One process owns every visible MI355X: ncclCommInitAll builds one RCCL communicator per device in a
// single call (no rendezvous), and each collective is one ncclGroupStart/End over the devices, enqueued
// on each device's CURRENT HIP stream -- the stream its replica's kernels run on -- so replica compute,
// the parameter broadcast and the gradient reduction are ordered by the streams alone (no events, no
// host sync).  xGMI carries the transfers peer to peer.
//   broadcast(ts, root): ts[i] on device i; every ts[i] <- ts[root]        (per-forward replication)
//   reduce(ts, root):    ts[root] <- sum_i ts[i], in place on the root     (gradient reduce-add to GPU 0)
//   all_reduce(ts):      every ts[i] <- sum_i ts[i]
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <torch/extension.h>

#include <vector>

namespace pdt_dp {

namespace py = pybind11;
using at::Tensor;

#define PDT_NCCL_OK(expr)                                                                        \
  do {                                                                                           \
    ncclResult_t _r = (expr);                                                                    \
    TORCH_CHECK(_r == ncclSuccess, #expr " failed: ", ncclGetErrorString(_r));                   \
  } while (0)

static ncclDataType_t nccl_type(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kHalf: return ncclFloat16;
    case at::kBFloat16: return ncclBfloat16;
    case at::kDouble: return ncclFloat64;
    case at::kLong: return ncclInt64;
    case at::kInt: return ncclInt32;
    default: TORCH_CHECK(false, "dp group: unsupported dtype ", t.scalar_type());
  }
}

class DeviceGroup {
 public:
  explicit DeviceGroup(std::vector<int> devices) : devices_(std::move(devices)) {
    TORCH_CHECK(!devices_.empty(), "dp group: no devices");
    comms_.resize(devices_.size(), nullptr);
    PDT_NCCL_OK(ncclCommInitAll(comms_.data(), (int)devices_.size(), devices_.data()));
  }
  ~DeviceGroup() {
    for (auto c : comms_)
      if (c) ncclCommDestroy(c);
  }
  DeviceGroup(const DeviceGroup&) = delete;
  DeviceGroup& operator=(const DeviceGroup&) = delete;

  int size() const { return (int)devices_.size(); }

  void broadcast(const std::vector<Tensor>& ts, int root) {
    check(ts, root);
    PDT_NCCL_OK(ncclGroupStart());
    for (size_t i = 0; i < ts.size(); ++i)
      PDT_NCCL_OK(ncclBroadcast(ts[root].data_ptr(), ts[i].data_ptr(), ts[i].numel(), nccl_type(ts[i]), root,
                                comms_[i], stream(i)));
    PDT_NCCL_OK(ncclGroupEnd());
  }
  void reduce(const std::vector<Tensor>& ts, int root) {
    check(ts, root);
    PDT_NCCL_OK(ncclGroupStart());
    for (size_t i = 0; i < ts.size(); ++i)
      PDT_NCCL_OK(ncclReduce(ts[i].data_ptr(), ts[root].data_ptr(), ts[i].numel(), nccl_type(ts[i]), ncclSum, root,
                             comms_[i], stream(i)));
    PDT_NCCL_OK(ncclGroupEnd());
  }
  void all_reduce(const std::vector<Tensor>& ts) {
    check(ts, 0);
    PDT_NCCL_OK(ncclGroupStart());
    for (size_t i = 0; i < ts.size(); ++i)
      PDT_NCCL_OK(ncclAllReduce(ts[i].data_ptr(), ts[i].data_ptr(), ts[i].numel(), nccl_type(ts[i]), ncclSum,
                                comms_[i], stream(i)));
    PDT_NCCL_OK(ncclGroupEnd());
  }

 private:
  hipStream_t stream(size_t i) const { return at::hip::getCurrentHIPStream(devices_[i]).stream(); }
  void check(const std::vector<Tensor>& ts, int root) const {
    TORCH_CHECK(ts.size() == devices_.size(), "dp group: need one tensor per device");
    TORCH_CHECK(root >= 0 && root < (int)ts.size(), "dp group: bad root");
    for (size_t i = 0; i < ts.size(); ++i) {
      TORCH_CHECK(ts[i].is_cuda() && ts[i].is_contiguous(), "dp group: tensors must be contiguous GPU tensors");
      TORCH_CHECK(ts[i].get_device() == devices_[i], "dp group: tensor ", i, " is on device ", ts[i].get_device(),
                  ", expected ", devices_[i]);
      TORCH_CHECK(ts[i].numel() == ts[root].numel() && ts[i].scalar_type() == ts[root].scalar_type(),
                  "dp group: tensors differ in size or dtype");
    }
  }
  std::vector<int> devices_;
  std::vector<ncclComm_t> comms_;
};

void register_dp(py::module& m) {
  py::class_<DeviceGroup>(m, "DeviceGroup")
      .def(py::init<std::vector<int>>())
      .def_property_readonly("size", &DeviceGroup::size)
      .def("broadcast", &DeviceGroup::broadcast, py::arg("tensors"), py::arg("root") = 0)
      .def("reduce", &DeviceGroup::reduce, py::arg("tensors"), py::arg("root") = 0)
      .def("all_reduce", &DeviceGroup::all_reduce);
}

}  // namespace pdt_dp
