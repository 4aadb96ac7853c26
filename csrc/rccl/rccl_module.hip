// pybind11 module `_rccl`: RCCL all-reduce over xGMI on a scheduler-chosen device subset.
//
//  * local_sweep(devs, sizes, ...)  — single process, ncclCommInitAll over `devs`.
//  * unique_id() / Comm(...)        — one process per GPU (torchrun / pod per rank): rank 0 creates
//                                     the ncclUniqueId, ships the 128 bytes through any store, every
//                                     rank builds a Comm on its chosen device (ncclCommInitRank).
// Comm.step() enqueues one out-of-place all-reduce on the Comm's stream and returns immediately so
// a Python-side timing loop (bench.py) brackets exactly K of them with barrier + synchronize.
// Comm.capture(n) records n back-to-back all-reduces into one hipGraph and Comm.replay() launches
// it: small messages are launch-bound (a few µs of host enqueue per call), and a graph replays the
// whole chain with one launch — the latency a graph-captured training step sees.
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
  ~Comm() {
    drop_graph();
    st_.release();
  }

  void prepare(size_t bytes, const std::string& dtype) {
    drop_graph();
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

  // Capture n all-reduces of the prepared buffer into one executable graph (every rank of the
  // communicator must capture the same n).  One eager call first so RCCL's lazy per-size setup
  // (channels, proxy buffers) happens outside the capture.
  void capture(int n, bool inplace) {
    if (!count_) throw std::runtime_error("prepare() first");
    if (n < 1) throw std::invalid_argument("capture needs n >= 1");
    drop_graph();
    st_.set_device();
    st_.allreduce(count_, t_, inplace);
    RCCL_HIP_CHECK(hipStreamSynchronize(st_.stream));
    hipGraph_t g = nullptr;
    RCCL_HIP_CHECK(hipStreamBeginCapture(st_.stream, hipStreamCaptureModeThreadLocal));
    try {
      for (int i = 0; i < n; ++i) st_.allreduce(count_, t_, inplace);
    } catch (...) {
      (void)hipStreamEndCapture(st_.stream, &g);
      if (g) (void)hipGraphDestroy(g);
      throw;
    }
    RCCL_HIP_CHECK(hipStreamEndCapture(st_.stream, &g));
    hipError_t e = hipGraphInstantiate(&exec_, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (e != hipSuccess) {
      exec_ = nullptr;
      throw std::runtime_error(std::string("hipGraphInstantiate failed: ") + hipGetErrorString(e));
    }
    graph_n_ = n;
  }

  void replay() {
    if (!exec_) throw std::runtime_error("capture() first");
    st_.set_device();
    RCCL_HIP_CHECK(hipGraphLaunch(exec_, st_.stream));
  }

  int graph_ops() const { return graph_n_; }

  // Exact check of the receive buffer as it stands (no new all-reduce): after out-of-place graph
  // replays of prepare()'s fill it must hold the same sums as one eager call.
  unsigned long long verify() {
    if (!count_) throw std::runtime_error("prepare() first");
    return st_.check(count_, t_, false);
  }

  size_t bytes() const { return count_ * elem_; }
  int rank() const { return st_.rank; }
  int nranks() const { return st_.nranks; }
  int device() const { return st_.device; }
  int min_ctas() const { return min_ctas_; }
  int max_ctas() const { return max_ctas_; }
  void destroy() {
    drop_graph();
    st_.release();
  }

 private:
  void drop_graph() {
    if (exec_) {
      (void)hipSetDevice(st_.device);
      (void)hipStreamSynchronize(st_.stream);
      (void)hipGraphExecDestroy(exec_);
    }
    exec_ = nullptr;
    graph_n_ = 0;
  }
  hipGraphExec_t exec_ = nullptr;
  int graph_n_ = 0;

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
      .def("capture", &Comm::capture, py::arg("n"), py::arg("inplace") = false, py::call_guard<py::gil_scoped_release>())
      .def("replay", &Comm::replay, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("graph_ops", &Comm::graph_ops)
      .def("verify", &Comm::verify, py::call_guard<py::gil_scoped_release>())
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
