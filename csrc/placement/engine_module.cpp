// pybind11 module `_placement`: native branch-and-bound placement engine (engine.h).
//
// Python side: gpu_topology_on_k8s_amd/placement/core.py builds a Problem (cost matrix, free mask,
// hierarchy levels, access costs) and calls `select` / `worst` / `evaluate`; results are plain
// dicts so the extender hot path (prioritize per node per pod) stays allocation-light.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <chrono>

#include "placement/engine.h"

namespace py = pybind11;
using namespace gtk;

namespace {

using DArray = py::array_t<double, py::array::c_style | py::array::forcecast>;

Problem make_problem(py::array_t<double, py::array::c_style | py::array::forcecast> cost,
                     py::array_t<bool, py::array::c_style | py::array::forcecast> free_mask,
                     const std::vector<std::vector<int>>& levels,
                     py::array_t<double, py::array::c_style | py::array::forcecast> access, DArray deficit = DArray()) {
  Problem p;
  auto c = cost.unchecked<2>();
  if (c.shape(0) != c.shape(1)) throw std::invalid_argument("cost must be square");
  p.n = (int)c.shape(0);
  p.cost.assign(cost.data(), cost.data() + (size_t)p.n * p.n);
  auto f = free_mask.unchecked<1>();
  if (f.shape(0) != p.n) throw std::invalid_argument("free mask length != n");
  p.free.resize(p.n);
  for (int i = 0; i < p.n; ++i) p.free[i] = f(i) ? 1 : 0;
  p.levels = levels;
  auto a = access.unchecked<1>();
  if (a.shape(0) != 0 && a.shape(0) != p.n) throw std::invalid_argument("access length != n");
  p.access.assign(access.data(), access.data() + a.shape(0));
  if (deficit.size() > 0) {
    if (deficit.ndim() != 2 || deficit.shape(0) != p.n || deficit.shape(1) != p.n) throw std::invalid_argument("deficit must be n x n");
    p.deficit.assign(deficit.data(), deficit.data() + (size_t)p.n * p.n);
  }
  return p;
}

py::dict to_dict(const Result& r, double us) {
  py::dict d;
  d["ids"] = r.ids;
  d["objective"] = r.objective;
  d["feasible"] = r.feasible;
  d["exact"] = r.exact;
  d["nodes"] = r.nodes;
  d["leaves"] = r.leaves;
  d["micros"] = us;
  py::dict t;
  t["comm"] = r.terms.comm;
  t["bottleneck"] = r.terms.bott;
  t["span"] = r.terms.span;
  t["frag"] = r.terms.frag;
  t["fit"] = r.terms.fit;
  t["access"] = r.terms.access;
  t["nic_deficit"] = r.terms.nicdef;
  t["link_deficit"] = r.terms.deficit;
  d["terms"] = t;
  return d;
}

Policy make_policy(double w_span, double w_frag, double w_fit, double w_access, double w_bottleneck, double w_nic = 1.0,
                   double w_link_deficit = 1.0) {
  if (!(w_bottleneck >= 0.0 && w_bottleneck <= 1.0)) throw std::invalid_argument("w_bottleneck must be in [0, 1]");
  Policy pol;
  pol.w_bottleneck = w_bottleneck;
  pol.w_nic = w_nic;
  pol.w_span = w_span;
  pol.w_frag = w_frag;
  pol.w_fit = w_fit;
  pol.w_access = w_access;
  pol.w_link_deficit = w_link_deficit;
  return pol;
}

}  // namespace

PYBIND11_MODULE(_placement, m) {
  m.doc() = "Exact branch-and-bound GPU/XCP subset placement engine";
  m.def(
      "select",
      [](py::array_t<double, py::array::c_style | py::array::forcecast> cost,
         py::array_t<bool, py::array::c_style | py::array::forcecast> free_mask, const std::vector<std::vector<int>>& levels,
         py::array_t<double, py::array::c_style | py::array::forcecast> access, int k, double w_span, double w_frag,
         double w_fit, double w_access, uint64_t node_limit, bool collect_ties, double w_bottleneck,
         const std::vector<int>& nic, double w_nic, DArray deficit, double w_link_deficit) {
        Problem p = make_problem(cost, free_mask, levels, access, deficit);
        p.nic = nic;
        Result r;
        double us = 0;
        {
          py::gil_scoped_release nogil;
          auto t0 = std::chrono::steady_clock::now();
          Engine e(p, make_policy(w_span, w_frag, w_fit, w_access, w_bottleneck, w_nic, w_link_deficit));
          r = e.select(k, node_limit, collect_ties);
          us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        }
        py::dict d = to_dict(r, us);
        if (collect_ties) d["ties"] = r.ties;
        return d;
      },
      py::arg("cost"), py::arg("free"), py::arg("levels"), py::arg("access"), py::arg("k"), py::arg("w_span") = 0.5,
      py::arg("w_frag") = 0.25, py::arg("w_fit") = 0.05, py::arg("w_access") = 0.1,
      py::arg("node_limit") = (uint64_t)2000000, py::arg("collect_ties") = false,
      py::arg("w_bottleneck") = 0.4, py::arg("nic") = std::vector<int>{}, py::arg("w_nic") = 1.0,
      py::arg("deficit") = DArray(), py::arg("w_link_deficit") = 1.0);
  m.def(
      "worst",
      [](py::array_t<double, py::array::c_style | py::array::forcecast> cost,
         py::array_t<bool, py::array::c_style | py::array::forcecast> free_mask, const std::vector<std::vector<int>>& levels,
         py::array_t<double, py::array::c_style | py::array::forcecast> access, int k, double w_span, double w_frag,
         double w_fit, double w_access, uint64_t node_limit, double w_bottleneck,
         const std::vector<int>& nic, double w_nic, DArray deficit, double w_link_deficit) {
        Problem p = make_problem(cost, free_mask, levels, access, deficit);
        p.nic = nic;
        Result r;
        double us = 0;
        {
          py::gil_scoped_release nogil;
          auto t0 = std::chrono::steady_clock::now();
          Engine e(p, make_policy(w_span, w_frag, w_fit, w_access, w_bottleneck, w_nic, w_link_deficit));
          r = e.worst(k, node_limit);
          us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        }
        return to_dict(r, us);
      },
      py::arg("cost"), py::arg("free"), py::arg("levels"), py::arg("access"), py::arg("k"), py::arg("w_span") = 0.5,
      py::arg("w_frag") = 0.25, py::arg("w_fit") = 0.05, py::arg("w_access") = 0.1,
      py::arg("node_limit") = (uint64_t)2000000, py::arg("w_bottleneck") = 0.4, py::arg("nic") = std::vector<int>{},
      py::arg("w_nic") = 1.0, py::arg("deficit") = DArray(), py::arg("w_link_deficit") = 1.0);
  m.def(
      "evaluate",
      [](py::array_t<double, py::array::c_style | py::array::forcecast> cost,
         py::array_t<bool, py::array::c_style | py::array::forcecast> free_mask, const std::vector<std::vector<int>>& levels,
         py::array_t<double, py::array::c_style | py::array::forcecast> access, const std::vector<int>& ids,
         double w_span, double w_frag, double w_fit, double w_access, double w_bottleneck,
         const std::vector<int>& nic, double w_nic, DArray deficit, double w_link_deficit) {
        Problem p = make_problem(cost, free_mask, levels, access, deficit);
        p.nic = nic;
        Engine e(p, make_policy(w_span, w_frag, w_fit, w_access, w_bottleneck, w_nic, w_link_deficit));
        Result r;
        r.ids = ids;
        r.objective = e.evaluate(ids, &r.terms);
        r.feasible = true;
        return to_dict(r, 0.0);
      },
      py::arg("cost"), py::arg("free"), py::arg("levels"), py::arg("access"), py::arg("ids"), py::arg("w_span") = 0.5,
      py::arg("w_frag") = 0.25, py::arg("w_fit") = 0.05, py::arg("w_access") = 0.1, py::arg("w_bottleneck") = 0.4,
      py::arg("nic") = std::vector<int>{}, py::arg("w_nic") = 1.0, py::arg("deficit") = DArray(),
      py::arg("w_link_deficit") = 1.0);
  m.attr("EPS") = kEps;
}
