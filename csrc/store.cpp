// Native TCP rendezvous store: the MI355X-native counterpart of c10d's TCPStore that the reference's
// `dist.init_process_group(backend='nccl')` (env://) relies on (SURVEY §2.4, X1, §7.1 comm/tcp_store).
//
// Rank 0 (or the launcher) runs the server: one acceptor thread plus one thread per client connection,
// serving a key -> bytes map behind a mutex/condition variable.  Clients are thin synchronous sockets.
// Operations (all length-prefixed, little endian):
//   SET key value          store / overwrite, wakes waiters
//   GET key                block until the key exists (or the client timeout), return its value
//   ADD key delta          atomic int64 counter (created at 0), returns the new value
//   CHECK key              non-blocking existence test
//   DEL key                remove
// barrier(tag) is ADD on "<tag>/arrive" followed by a GET on "<tag>/done" that the last arriver SETs --
// no polling.  The RCCL unique id of csrc/comm.cpp travels through SET/GET.  Timeouts surface as
// exceptions in the waiting process instead of a silent hang (failure detection).
#include <memory>
#include <string>

#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "store_core.h"

namespace pdt_store {

namespace py = pybind11;

// Python face of StoreClient: bytes in / out, the GIL released around every blocking socket operation.
class Store {
 public:
  Store(const std::string& host, int port, bool is_server, double timeout_s)
      : c_(std::make_unique<StoreClient>(host, port, is_server, timeout_s)) {}
  int port() const { return c_->port(); }
  void set(const std::string& key, const py::bytes& value) {
    std::string v = value;
    py::gil_scoped_release nogil;
    c_->set(key, v);
  }
  py::bytes get(const std::string& key, double timeout_s) {
    std::string v;
    {
      py::gil_scoped_release nogil;
      v = c_->get(key, timeout_s);
    }
    return py::bytes(v);
  }
  int64_t add(const std::string& key, int64_t delta) {
    py::gil_scoped_release nogil;
    return c_->add(key, delta);
  }
  bool check(const std::string& key) {
    py::gil_scoped_release nogil;
    return c_->check(key);
  }
  void del(const std::string& key) {
    py::gil_scoped_release nogil;
    c_->del(key);
  }
  void barrier(const std::string& tag, int world) {
    py::gil_scoped_release nogil;
    c_->barrier(tag, world);
  }

 private:
  std::unique_ptr<StoreClient> c_;
};

void register_store(py::module& m) {
  py::class_<Store>(m, "TCPStore")
      .def(py::init<const std::string&, int, bool, double>(), py::arg("host"), py::arg("port"),
           py::arg("is_server"), py::arg("timeout_s") = 300.0)
      .def_property_readonly("port", &Store::port)
      .def("set", &Store::set)
      .def("get", &Store::get, py::arg("key"), py::arg("timeout_s") = -1.0)
      .def("add", &Store::add)
      .def("check", &Store::check)
      .def("delete_key", &Store::del)
      .def("barrier", &Store::barrier, py::arg("tag"), py::arg("world"));
}

}  // namespace pdt_store
