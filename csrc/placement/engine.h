// Native placement engine: exact branch-and-bound search for the k-device subset minimising the
// placement objective of gpu_topology_on_k8s_amd/placement/core.py.
//
// Reference behaviour being replaced: design.md:162-190 grows a greedy/Prim set from the closest
// free pair and admits (design.md:188-190) that a tie on the seed pair can lock in a worse set; the
// Gaia Link policy (paper p.5 Alg. 4) searches a cost tree.  Both are heuristics.  On an 8-GPU
// MI355X node the exact search is at most C(8,4)=70 subsets, but in CPX mode a node exposes 64 XCP
// devices (C(64,8) ~ 4.4e9 subsets), which is why the engine is native and prunes with bounds.
//
// Objective (identical to core.evaluate):
//   J(S) = comm + w_bottleneck*(bott - comm) + w_span*span + w_frag*frag + w_fit*fit + w_access*acc
//   comm = mean unordered-pair cost of S (1.0 when |S| == 1)
//   bott = costliest pair of S (== comm when |S| <= 2 or every link is alike): a ring collective runs
//          at its slowest link, which the mean dilutes (one half-bandwidth link in a 4-set is +1/6)
//   span = sum_levels (#groups touched - #groups minimally needed for k free devices)
//   frag = sum_levels #pristine groups left partially used
//   fit  = sum_levels sum_touched free_after/size
//   acc  = mean access cost of S
//   + w_link_deficit * deficit: the largest Problem::deficit over the pairs of S (a link's shortfall
//     against the best link of its class on the node, beyond a dead band; empty = 0 everywhere)
//   + w_nic * nicdef (only with Problem::nic): NIC domains (device -> its nearest RDMA NIC) a
//     multi-node pod could use but S leaves out, min(k, domains with a free device) - domains touched
// Enumeration is lexicographic over free device ids and a candidate replaces the incumbent only if
// it is better by more than kEps, so the result equals itertools.combinations + first-minimum.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace gtk {

constexpr double kEps = 1e-9;

struct Policy {
  double w_span = 0.5, w_frag = 0.25, w_fit = 0.05, w_access = 0.1, w_bottleneck = 0.4;  // w_bottleneck in [0, 1]
  double w_nic = 1.0;
  double w_link_deficit = 1.0;
};

struct Problem {
  int n = 0;
  std::vector<double> cost;               // n*n row-major, symmetric
  std::vector<uint8_t> free;              // n
  std::vector<std::vector<int>> levels;   // per level: group id per device (any ints)
  std::vector<double> access;             // n
  std::vector<int> nic;                   // empty, or n: NIC domain per device (-1 = none)
  std::vector<double> deficit;            // empty (all 0), or n*n row-major, symmetric, >= 0
};

struct Terms {
  double comm = 0, bott = 0, span = 0, frag = 0, fit = 0, access = 0, nicdef = 0, deficit = 0;
};

struct Result {
  std::vector<int> ids;
  double objective = 0;
  Terms terms;
  bool exact = true;
  bool feasible = false;
  uint64_t nodes = 0;     // search-tree nodes expanded
  uint64_t leaves = 0;    // complete subsets evaluated
  // select(collect_ties=true): every subset within kEps of the optimum, in lexicographic order (what
  // a random tie-break draws from: Gaia Table I splits 1-GPU requests between equal cousins).
  std::vector<std::vector<int>> ties;
};

class Engine {
 public:
  Engine(const Problem& p, const Policy& pol);

  // Exact (branch and bound) unless more than `node_limit` nodes are needed, in which case the
  // best set found by greedy growth + 1-swap descent is returned with exact=false.
  // With `collect_ties` the bound prunes only strictly worse branches and the optima (at most
  // `max_ties`) come back in Result::ties.
  Result select(int k, uint64_t node_limit, bool collect_ties = false, size_t max_ties = 65536) const;
  // Highest-objective subset ("worst placement" baseline of BASELINE config 5): exhaustive when
  // C(free, k) <= node_limit, else greedy ascent + 1-swap (exact=false).
  Result worst(int k, uint64_t node_limit = 2000000) const;
  // Objective of an arbitrary set.
  double evaluate(const std::vector<int>& ids, Terms* terms) const;

 private:
  struct Level {
    std::vector<int> gid;      // dense group id per device
    std::vector<int> size;     // devices per group
    std::vector<int> free;     // free devices per group
    std::vector<int> sorted_free;  // `free`, descending (min_groups)
  };
  int min_groups(const Level& lv, int k) const;
  double nic_deficit(const int* ids, int k) const;  // ids: device ids
  // `cls` (optional, class id per device id, -1 = not free): interchangeable devices share a class, and
  // only the first not-yet-chosen member of each class is tried (identical objective otherwise).
  void greedy(int k, const std::vector<int>& free_ids, std::vector<int>* best, double* best_j, bool maximise,
              const std::vector<int>* cls = nullptr) const;

  Problem p_;
  Policy pol_;
  std::vector<Level> lv_;
  int nic_domains_free_ = 0;  // NIC domains with at least one free device
};

}  // namespace gtk
