// pybind11 module `_rccl`: RCCL all-reduce over xGMI on a scheduler-chosen device subset.
//
//  * local_sweep(devs, sizes, ...)  — single process, ncclCommInitAll over `devs`.
//  * unique_id() / Comm(...)        — one process per GPU (torchrun / pod per rank): rank 0 creates
//                                     the ncclUniqueId, ships the 128 bytes through any store, every
//                                     rank builds a Comm on its chosen device (ncclCommInitRank).
// Comm.step() enqueues one out-of-place all-reduce on the Comm's stream and returns immediately so
// a Python-side timing loop (bench.py) brackets exactly K of them with barrier + synchronize.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "rccl_core.h"

namespace py = pybind11;
using namespace gtk;

namespace {

class Comm {
 public:
  // min_ctas / max_ctas > 0 go through ncclCommInitRankConfig (ncclConfig_t.minCTAs/maxCTAs =
  // the communicator's channel count bounds); bench.py tunes them per subset size on the node.
  Comm(py::bytes uid, int nranks, int rank, int device, int min_ctas, int max_ctas) {
    std::string s = uid;
    if (s.size() != sizeof(ncclUniqueId)) throw std::invalid_argument("unique id must be NCCL_UNIQUE_ID_BYTES long");
    ncclUniqueId id;
    std::memcpy(&id, s.data(), sizeof(id));
    st_.device = device;
    st_.rank = rank;
    st_.nranks = nranks;
    py::gil_scoped_release nogil;
    st_.set_device();
    if (min_ctas > 0 || max_ctas > 0) {
      ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
      if (min_ctas > 0) cfg.minCTAs = min_ctas;
      if (max_ctas > 0) cfg.maxCTAs = max_ctas;
      NCCL_CHECK(ncclCommInitRankConfig(&st_.comm, nranks, id, rank, &cfg));
    } else {
      NCCL_CHECK(ncclCommInitRank(&st_.comm, nranks, id, rank));
    }
    min_ctas_ = min_ctas;
    max_ctas_ = max_ctas;
    RCCL_HIP_CHECK(hipStreamCreateWithFlags(&st_.stream, hipStreamNonBlocking));
  }
  ~Comm() { st_.release(); }

  void prepare(size_t bytes, const std::string& dtype) {
    t_ = parse_dtype(dtype, &elem_);
    count_ = std::max<size_t>(1, bytes / elem_);
    st_.ensure(count_ * elem_);
    st_.fill(count_, t_);
    RCCL_HIP_CHECK(hipStreamSynchronize(st_.stream));
  }

  void step(bool inplace) {
    if (!count_) throw std::runtime_error("prepare() first");
    st_.set_device();
    st_.allreduce(count_, t_, inplace);
  }

  void synchronize() {
    st_.set_device();
    RCCL_HIP_CHECK(hipStreamSynchronize(st_.stream));
  }

  // Fresh fill + one all-reduce + exact check; returns the number of wrong elements on this rank.
  unsigned long long check(bool inplace) {
    if (!count_) throw std::runtime_error("prepare() first");
    st_.fill(count_, t_);
    st_.allreduce(count_, t_, inplace);
    return st_.check(count_, t_, inplace);
  }

  size_t bytes() const { return count_ * elem_; }
  int rank() const { return st_.rank; }
  int nranks() const { return st_.nranks; }
  int device() const { return st_.device; }
  int min_ctas() const { return min_ctas_; }
  int max_ctas() const { return max_ctas_; }
  void destroy() { st_.release(); }

 private:
  RankState st_;
  ncclDataType_t t_ = ncclBfloat16;
  size_t elem_ = 2, count_ = 0;
  int min_ctas_ = 0, max_ctas_ = 0;
};

py::bytes unique_id() {
  ncclUniqueId id;
  NCCL_CHECK(ncclGetUniqueId(&id));
  return py::bytes(reinterpret_cast<const char*>(&id), sizeof(id));
}

py::list local_sweep(const std::vector<int>& devs, const std::vector<size_t>& sizes, const std::string& dtype, int iters,
                     int warmup, bool inplace, bool check) {
  std::vector<SweepPoint> pts;
  {
    py::gil_scoped_release nogil;
    LocalGroup g(devs);
    for (size_t b : sizes) pts.push_back(g.run(b, dtype, iters, warmup, inplace, check));
  }
  py::list out;
  for (const auto& p : pts) {
    py::dict d;
    d["bytes"] = p.bytes;
    d["count"] = p.count;
    d["time_us"] = p.time_us;
    d["algbw_gbps"] = p.algbw;
    d["busbw_gbps"] = p.busbw;
    d["wrong"] = p.wrong;
    out.append(d);
  }
  return out;
}

int version() {
  int v = 0;
  NCCL_CHECK(ncclGetVersion(&v));
  return v;
}

}  // namespace

PYBIND11_MODULE(_rccl, m) {
  m.doc() = "RCCL all-reduce placement validator (xGMI)";
  m.def("version", &version);
  m.def("unique_id", &unique_id);
  m.def("bus_factor", &bus_factor, py::arg("k"));
  m.def("size_sweep", &size_sweep, py::arg("min_bytes"), py::arg("max_bytes"), py::arg("factor") = 2);
  m.def("local_sweep", &local_sweep, py::arg("devs"), py::arg("sizes"), py::arg("dtype") = "bf16", py::arg("iters") = 20,
        py::arg("warmup") = 5, py::arg("inplace") = false, py::arg("check") = true);
  py::class_<Comm>(m, "Comm")
      .def(py::init<py::bytes, int, int, int, int, int>(), py::arg("uid"), py::arg("nranks"), py::arg("rank"),
           py::arg("device"), py::arg("min_ctas") = 0, py::arg("max_ctas") = 0)
      .def("prepare", &Comm::prepare, py::arg("bytes"), py::arg("dtype") = "bf16",
           py::call_guard<py::gil_scoped_release>())
      .def("step", &Comm::step, py::arg("inplace") = false, py::call_guard<py::gil_scoped_release>())
      .def("synchronize", &Comm::synchronize, py::call_guard<py::gil_scoped_release>())
      .def("check", &Comm::check, py::arg("inplace") = false, py::call_guard<py::gil_scoped_release>())
      .def("destroy", &Comm::destroy, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("bytes", &Comm::bytes)
      .def_property_readonly("rank", &Comm::rank)
      .def_property_readonly("nranks", &Comm::nranks)
      .def_property_readonly("device", &Comm::device)
      .def_property_readonly("min_ctas", &Comm::min_ctas)
      .def_property_readonly("max_ctas", &Comm::max_ctas);
}
