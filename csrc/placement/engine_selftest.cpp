// Host-only self test of the placement engine, built with -fsanitize=address,undefined by
// `python -m gpu_topology_on_k8s_amd._native.build --only engine_selftest`.
// Checks branch-and-bound == exhaustive enumeration on random problems, including CPX-sized ones.
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "placement/engine.h"

using namespace gtk;

static double brute(const Engine& e, const std::vector<int>& F, int k, std::vector<int>* best, bool maximise = false) {
  const int m = (int)F.size();
  std::vector<int> idx(k);
  for (int i = 0; i < k; ++i) idx[i] = i;
  const double sgn = maximise ? -1.0 : 1.0;
  double bj = INFINITY;
  std::vector<int> cur(k);
  while (true) {
    for (int i = 0; i < k; ++i) cur[i] = F[idx[i]];
    double j = sgn * e.evaluate(cur, nullptr);
    if (j < bj - kEps) {
      bj = j;
      *best = cur;
    }
    int i = k - 1;
    while (i >= 0 && idx[i] == m - k + i) --i;
    if (i < 0) break;
    ++idx[i];
    for (int q = i + 1; q < k; ++q) idx[q] = idx[q - 1] + 1;
  }
  return sgn * bj;
}

int main() {
  std::mt19937 rng(1234);
  int failures = 0, cases = 0;
  for (int trial = 0; trial < 400; ++trial) {
    const int n = 2 + (int)(rng() % 15);
    Problem p;
    p.n = n;
    p.cost.assign((size_t)n * n, 0.0);
    std::uniform_real_distribution<double> u(0.25, 4.0);
    for (int i = 0; i < n; ++i)
      for (int j = i + 1; j < n; ++j) p.cost[(size_t)i * n + j] = p.cost[(size_t)j * n + i] = (rng() % 3 == 0) ? 1.0 : u(rng);
    p.free.resize(n);
    for (int i = 0; i < n; ++i) p.free[i] = (rng() % 4) != 0;
    const int per_pkg = 1 + (int)(rng() % 4);
    std::vector<int> pkg(n), numa(n);
    for (int i = 0; i < n; ++i) {
      pkg[i] = i / per_pkg;
      numa[i] = i < n / 2 ? 0 : 1;
    }
    if (per_pkg > 1) p.levels.push_back(pkg);
    p.levels.push_back(numa);
    p.access.resize(n);
    for (int i = 0; i < n; ++i) p.access[i] = (rng() % 2) ? 0.0 : u(rng);
    Engine e(p, Policy{});
    std::vector<int> F;
    for (int i = 0; i < n; ++i)
      if (p.free[i]) F.push_back(i);
    for (int k = 1; k <= (int)F.size(); ++k) {
      std::vector<int> bb;
      double bj = brute(e, F, k, &bb);
      Result r = e.select(k, 50000000ull);
      ++cases;
      if (!r.exact || r.ids != bb || std::fabs(r.objective - bj) > 1e-9) {
        ++failures;
        std::printf("MISMATCH n=%d k=%d bnb_j=%.12f brute_j=%.12f\n", n, k, r.objective, bj);
      }
      std::vector<int> wb;
      double wj = brute(e, F, k, &wb, /*maximise=*/true);
      Result w = e.worst(k, 50000000ull);
      ++cases;
      if (!w.exact || w.ids != wb || std::fabs(w.objective - wj) > 1e-9) {
        ++failures;
        std::printf("WORST MISMATCH n=%d k=%d worst_j=%.12f brute_j=%.12f\n", n, k, w.objective, wj);
      }
    }
  }
  // symmetric (CPX-like) problems: packages of interchangeable partitions, package-level costs, a
  // random used set — the exact symmetry breaking must return the brute-force first optimum
  for (int trial = 0; trial < 120; ++trial) {
    const int pk = 2 + (int)(rng() % 3), per = 2 + (int)(rng() % 3), n = pk * per;
    Problem p;
    p.n = n;
    p.cost.assign((size_t)n * n, 0.0);
    std::uniform_real_distribution<double> u(0.5, 3.0);
    std::vector<double> pc((size_t)pk * pk);
    for (int a = 0; a < pk; ++a)
      for (int b = a; b < pk; ++b) pc[(size_t)a * pk + b] = pc[(size_t)b * pk + a] = a == b ? 0.25 : ((rng() % 2) ? 1.0 : u(rng));
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j)
        if (i != j) p.cost[(size_t)i * n + j] = pc[(size_t)(i / per) * pk + j / per];
    p.free.resize(n);
    for (int i = 0; i < n; ++i) p.free[i] = (rng() % 5) != 0;
    std::vector<int> pkg(n), numa(n);
    for (int i = 0; i < n; ++i) {
      pkg[i] = i / per;
      numa[i] = (i / per) < pk / 2 ? 0 : 1;
    }
    p.levels.push_back(pkg);
    p.levels.push_back(numa);
    p.access.assign(n, 0.0);
    for (int i = 0; i < n; ++i) p.access[i] = (i / per) % 2 ? 0.5 : 0.0;
    Engine e(p, Policy{});
    std::vector<int> F;
    for (int i = 0; i < n; ++i)
      if (p.free[i]) F.push_back(i);
    for (int k = 1; k <= (int)F.size(); ++k) {
      std::vector<int> bb;
      double bj = brute(e, F, k, &bb);
      Result r = e.select(k, 50000000ull);
      ++cases;
      if (!r.exact || r.ids != bb || std::fabs(r.objective - bj) > 1e-9) {
        ++failures;
        std::printf("SYMMETRIC MISMATCH n=%d k=%d bnb_j=%.12f brute_j=%.12f\n", n, k, r.objective, bj);
      }
    }
  }
  std::printf("engine_selftest: %d cases, %d failures\n", cases, failures);
  return failures ? 1 : 0;
}
