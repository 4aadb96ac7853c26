// Branch-and-bound placement engine (see engine.h for the objective and the reference mapping).
#include "placement/engine.h"

#include <algorithm>
#include <cmath>
#include <functional>
#include <limits>
#include <map>
#include <numeric>
#include <stdexcept>

namespace gtk {

Engine::Engine(const Problem& p, const Policy& pol) : p_(p), pol_(pol) {
  if (p_.n < 0) throw std::invalid_argument("n < 0");
  const size_t n = (size_t)p_.n;
  if (p_.cost.size() != n * n) throw std::invalid_argument("cost must be n*n");
  if (p_.free.size() != n) throw std::invalid_argument("free must have n entries");
  if (p_.access.empty()) p_.access.assign(n, 0.0);
  if (p_.access.size() != n) throw std::invalid_argument("access must have n entries");
  if (!p_.deficit.empty() && p_.deficit.size() != n * n) throw std::invalid_argument("deficit must be empty or n*n");
  for (const auto& raw : p_.levels) {
    if (raw.size() != n) throw std::invalid_argument("every level needs n group ids");
    Level lv;
    std::map<int, int> dense;
    lv.gid.resize(n);
    for (size_t i = 0; i < n; ++i) {
      auto it = dense.find(raw[i]);
      if (it == dense.end()) it = dense.emplace(raw[i], (int)dense.size()).first;
      lv.gid[i] = it->second;
    }
    lv.size.assign(dense.size(), 0);
    lv.free.assign(dense.size(), 0);
    for (size_t i = 0; i < n; ++i) {
      lv.size[lv.gid[i]] += 1;
      lv.free[lv.gid[i]] += p_.free[i] ? 1 : 0;
    }
    lv.sorted_free = lv.free;
    std::sort(lv.sorted_free.begin(), lv.sorted_free.end(), std::greater<int>());

    lv_.push_back(std::move(lv));
  }
  if (!p_.nic.empty()) {
    if (p_.nic.size() != n) throw std::invalid_argument("nic must be empty or have n entries");
    std::vector<int> seen;
    for (size_t i = 0; i < n; ++i)
      if (p_.free[i] && p_.nic[i] >= 0 && std::find(seen.begin(), seen.end(), p_.nic[i]) == seen.end()) seen.push_back(p_.nic[i]);
    nic_domains_free_ = (int)seen.size();
  }
}

double Engine::nic_deficit(const int* ids, int k) const {
  if (p_.nic.empty() || pol_.w_nic == 0.0) return 0.0;
  int touched = 0;
  for (int a = 0; a < k; ++a) {
    const int d = p_.nic[ids[a]];
    if (d < 0) continue;
    bool first = true;
    for (int b = 0; b < a; ++b)
      if (p_.nic[ids[b]] == d) {
        first = false;
        break;
      }
    touched += first;
  }
  return (double)std::max(0, std::min(k, nic_domains_free_) - touched);
}

int Engine::min_groups(const Level& lv, int k) const {
  // lv.sorted_free: free counts in descending order (fixed for the problem)
  int s = 0;
  for (size_t i = 0; i < lv.sorted_free.size(); ++i) {
    s += lv.sorted_free[i];
    if (s >= k) return (int)i + 1;
  }
  return (int)lv.sorted_free.size();
}

double Engine::evaluate(const std::vector<int>& ids, Terms* terms) const {
  // Allocation-free: k is small, so groups are de-duplicated by an O(k^2) scan instead of a map
  // (the greedy / 1-swap searches of CPX-sized problems call this ~1e5 times per request).
  const int k = (int)ids.size();
  const int n = p_.n;
  Terms t;
  if (k >= 2) {
    double s = 0, mx = -std::numeric_limits<double>::infinity();
    for (int a = 0; a < k; ++a)
      for (int b = a + 1; b < k; ++b) {
        const double c = p_.cost[(size_t)ids[a] * n + ids[b]];
        s += c;
        mx = std::max(mx, c);
      }
    t.comm = 2.0 * s / ((double)k * (k - 1));
    t.bott = mx;
    if (!p_.deficit.empty())
      for (int a = 0; a < k; ++a)
        for (int b = a + 1; b < k; ++b) t.deficit = std::max(t.deficit, p_.deficit[(size_t)ids[a] * n + ids[b]]);
  } else {
    t.comm = t.bott = 1.0;
  }
  for (const auto& lv : lv_) {
    int touched = 0;
    for (int a = 0; a < k; ++a) {
      const int g = lv.gid[ids[a]];
      bool first = true;
      for (int b = 0; b < a; ++b)
        if (lv.gid[ids[b]] == g) {
          first = false;
          break;
        }
      if (!first) continue;
      int take = 1;
      for (int b = a + 1; b < k; ++b) take += lv.gid[ids[b]] == g;
      ++touched;
      const int after = lv.free[g] - take;
      if (lv.free[g] == lv.size[g] && after > 0) t.frag += 1;
      t.fit += (double)after / lv.size[g];
    }
    t.span += (double)touched - min_groups(lv, k);
  }
  double acc = 0;
  for (int i : ids) acc += p_.access[i];
  t.access = k ? acc / k : 0.0;
  t.nicdef = k ? nic_deficit(ids.data(), k) : 0.0;
  if (terms) *terms = t;
  return t.comm + pol_.w_nic * t.nicdef + pol_.w_bottleneck * (t.bott - t.comm) + pol_.w_span * t.span + pol_.w_frag * t.frag + pol_.w_fit * t.fit + pol_.w_access * t.access +
         pol_.w_link_deficit * t.deficit;
}

void Engine::greedy(int k, const std::vector<int>& F, std::vector<int>* best, double* best_j, bool maximise,
                    const std::vector<int>* cls) const {
  // Greedy growth from every seed, then first-improvement 1-swap descent (core._greedy_local).
  // `maximise` flips the direction (worst-placement search): sgn*J is minimised either way.
  const double sgn = maximise ? -1.0 : 1.0;
  // candidate filter under symmetry: a device is worth trying only if every lower-id member of its
  // class is already in the set (the others give the same objective as that member)
  auto skip = [&](const std::vector<int>& cur, int c) {
    if (std::find(cur.begin(), cur.end(), c) != cur.end()) return true;
    if (cls == nullptr) return false;
    const int cc = (*cls)[c];
    for (int d : F) {
      if (d >= c) break;
      if ((*cls)[d] == cc && std::find(cur.begin(), cur.end(), d) == cur.end()) return true;
    }
    return false;
  };
  for (int seed : F) {
    if (cls != nullptr && skip(std::vector<int>{}, seed)) continue;  // one seed per class
    std::vector<int> cur{seed};
    while ((int)cur.size() < k) {
      int cand = -1;
      double cj = std::numeric_limits<double>::infinity();
      for (int c : F) {
        if (skip(cur, c)) continue;
        cur.push_back(c);
        double j = sgn * evaluate(cur, nullptr);
        cur.pop_back();
        if (j < cj - kEps) {
          cj = j;
          cand = c;
        }
      }
      cur.push_back(cand);
    }
    double cur_j = sgn * evaluate(cur, nullptr);
    bool improved = true;
    while (improved) {
      improved = false;
      for (size_t a = 0; a < cur.size() && !improved; ++a) {
        for (int b : F) {
          if (skip(cur, b)) continue;
          std::vector<int> trial = cur;
          trial[a] = b;
          double tj = sgn * evaluate(trial, nullptr);
          if (tj < cur_j - kEps) {
            cur = trial;
            cur_j = tj;
            improved = true;
            break;
          }
        }
      }
    }
    std::sort(cur.begin(), cur.end());
    // best_j is kept in the caller's sign convention (a real objective value)
    const double bj = sgn * *best_j;
    if (cur_j < bj - kEps || (std::fabs(cur_j - bj) <= kEps && (best->empty() || cur < *best))) {
      *best = cur;
      *best_j = sgn * cur_j;
    }
  }
}

Result Engine::select(int k, uint64_t node_limit, bool collect_ties, size_t max_ties) const {
  Result res;
  if (k <= 0) throw std::invalid_argument("k must be >= 1");
  const int n = p_.n;
  std::vector<int> F;
  for (int i = 0; i < n; ++i)
    if (p_.free[i]) F.push_back(i);
  const int m = (int)F.size();
  if (m < k) return res;  // infeasible

  // ---- global bounds helpers
  // suffix-sorted access: amin_suffix[s][r] would be O(m^2); a global minimum is enough here.
  double amin = std::numeric_limits<double>::infinity();
  for (int i : F) amin = std::min(amin, p_.access[i]);
  // pre[c][t] = sum of the t cheapest links from F[c] to other free devices: every device of a
  // completion R (|R| = r) pays at least half of its r-1 cheapest links inside R.
  std::vector<std::vector<double>> pre(m, std::vector<double>(m, 0.0));
  {
    std::vector<double> row;
    for (int a = 0; a < m; ++a) {
      row.clear();
      for (int b = 0; b < m; ++b)
        if (b != a) row.push_back(p_.cost[(size_t)F[a] * n + F[b]]);
      std::sort(row.begin(), row.end());
      for (size_t t = 0; t < row.size(); ++t) pre[a][t + 1] = pre[a][t] + row[t];
    }
  }
  std::vector<int> mg(lv_.size());
  for (size_t l = 0; l < lv_.size(); ++l) mg[l] = min_groups(lv_[l], k);
  // suf[l][start * G + g]: free devices of group g (level l) at positions >= start of F
  std::vector<std::vector<int>> suf(lv_.size());
  size_t gmax = 1;
  for (size_t l = 0; l < lv_.size(); ++l) {
    const int G = (int)lv_[l].free.size();
    gmax = std::max(gmax, (size_t)G);
    suf[l].assign((size_t)(m + 1) * G, 0);
    for (int a = m - 1; a >= 0; --a) {
      for (int g = 0; g < G; ++g) suf[l][(size_t)a * G + g] = suf[l][(size_t)(a + 1) * G + g];
      suf[l][(size_t)a * G + lv_[l].gid[F[a]]] += 1;
    }
  }
  std::vector<int> ucap(gmax);
  const double pairs_k = k >= 2 ? 0.5 * k * (k - 1) : 1.0;

  // ---- exact symmetry breaking.  Free devices a and b are interchangeable when they sit in the same
  // group at every level, have the same access cost and the same link cost to every other free
  // device: swapping them maps any set onto one with the same objective.  The XCPs of one package on
  // a CPX node (64 devices, 8 classes of 8) are the case that matters: without this, C(64,16) sets.
  // Only canonical sets are searched — within a class, the chosen members are a prefix of the class
  // in id order — which keeps the first (lexicographically smallest) optimum of the full enumeration.
  // Off when collecting ties: a random tie-break must see every optimal set (Gaia Table I).
  std::vector<int> prev_same(m, -1);
  if (!collect_ties) {
    auto same = [&](int a, int b) {  // positions into F
      const int i = F[a], j = F[b];
      for (const auto& lv : lv_)
        if (lv.gid[i] != lv.gid[j]) return false;
      if (std::fabs(p_.access[i] - p_.access[j]) > 1e-12 * std::max(1.0, std::fabs(p_.access[i]))) return false;
      if (!p_.nic.empty() && p_.nic[i] != p_.nic[j]) return false;
      const double* ri = &p_.cost[(size_t)i * n];
      const double* rj = &p_.cost[(size_t)j * n];
      const double* di = p_.deficit.empty() ? nullptr : &p_.deficit[(size_t)i * n];
      const double* dj = p_.deficit.empty() ? nullptr : &p_.deficit[(size_t)j * n];
      for (int c = 0; c < m; ++c) {
        const int x = F[c];
        if (x == i || x == j) continue;
        if (std::fabs(ri[x] - rj[x]) > 1e-12 * std::max(1.0, std::fabs(ri[x]))) return false;
        if (di && std::fabs(di[x] - dj[x]) > 1e-12 * std::max(1.0, std::fabs(di[x]))) return false;
      }
      return true;
    };
    for (int a = 1; a < m; ++a)
      for (int b = a - 1; b >= 0; --b)
        if (same(b, a)) {  // exact equality is transitive: the nearest equal one is the class predecessor
          prev_same[a] = b;
          break;
        }
  }
  std::vector<char> inset(m, 0);

  // ---- DFS state
  std::vector<int> chosen;  // positions into F
  chosen.reserve(k);
  std::vector<std::vector<int>> take(lv_.size());
  std::vector<int> touched(lv_.size(), 0);
  for (size_t l = 0; l < lv_.size(); ++l) take[l].assign(lv_[l].size.size(), 0);
  std::vector<std::vector<double>> cross(k + 1, std::vector<double>(m, 0.0));  // cross[d][c] = sum cost(F[c], P_d)
  std::vector<std::vector<double>> xmax(k + 1, std::vector<double>(m, 0.0));   // xmax[d][c] = max cost(F[c], P_d)
  const bool has_def = !p_.deficit.empty();
  std::vector<std::vector<double>> dmax(has_def ? k + 1 : 0, std::vector<double>(m, 0.0));  // dmax[d][c] = max deficit(F[c], P_d)
  std::vector<double> scratch(m);

  double best_j = std::numeric_limits<double>::infinity();
  std::vector<int> best_pos;
  std::vector<std::vector<int>> tie_pos;
  uint64_t nodes = 0, leaves = 0;
  bool aborted = false;

  // Leaf objective from the incremental state.
  const double wb = pol_.w_bottleneck;
  auto leaf_objective = [&](double pairsum, double pairmax, double accsum, double defmax) {
    double comm = k >= 2 ? pairsum / pairs_k : 1.0;
    double bott = k >= 2 ? pairmax : 1.0;
    double span = 0, frag = 0, fit = 0;
    for (size_t l = 0; l < lv_.size(); ++l) {
      span += touched[l] - mg[l];
      const auto& lv = lv_[l];
      // walk the touched groups once: use the chosen devices' groups, dedup by marking
      for (size_t ci = 0; ci < chosen.size(); ++ci) {
        int g = lv.gid[F[chosen[ci]]];
        bool first = true;
        for (size_t cj = 0; cj < ci; ++cj)
          if (lv.gid[F[chosen[cj]]] == g) {
            first = false;
            break;
          }
        if (!first) continue;
        int after = lv.free[g] - take[l][g];
        if (lv.free[g] == lv.size[g] && after > 0) frag += 1;
        fit += (double)after / lv.size[g];
      }
    }
    double nicdef = 0.0;
    if (!p_.nic.empty()) {
      int small[64];
      std::vector<int> big;
      int* ids = small;
      if (k > 64) {
        big.resize(k);
        ids = big.data();
      }
      for (int i = 0; i < k; ++i) ids[i] = F[chosen[i]];
      nicdef = nic_deficit(ids, k);
    }
    return comm + wb * (bott - comm) + pol_.w_span * span + pol_.w_frag * frag + pol_.w_fit * fit +
           pol_.w_access * (accsum / k) + pol_.w_nic * nicdef + pol_.w_link_deficit * (k >= 2 ? defmax : 0.0);
  };

  // Large search spaces: seed the incumbent with greedy + 1-swap so pruning bites from the start.
  // (Ties then resolve to the greedy set rather than the lexicographically first optimum.)  The size
  // that matters is the number of CANONICAL k-sets: count vectors over the symmetry classes.
  double log_space;
  {
    std::vector<int> class_size;
    for (int a = 0; a < m; ++a) {
      if (prev_same[a] < 0) class_size.push_back(1);
      else {
        int root = a;
        while (prev_same[root] >= 0) root = prev_same[root];
        int idx = 0;  // class index = number of roots before `root`
        for (int b = 0; b < root; ++b) idx += prev_same[b] < 0;
        class_size[idx] += 1;
      }
    }
    std::vector<double> ways(k + 1, 0.0);  // ways[t] = canonical t-sets over the classes so far
    ways[0] = 1.0;
    for (int sz : class_size)
      for (int t = k; t >= 1; --t)
        for (int c = 1; c <= std::min(sz, t); ++c) ways[t] += ways[t - c];
    log_space = std::log(std::max(1.0, ways[k]));
  }
  std::vector<int> cls_of(n, -1);  // symmetry class per device id (root position in F)
  for (int a = 0; a < m; ++a) {
    int root = a;
    while (prev_same[root] >= 0) root = prev_same[root];
    cls_of[F[a]] = root;
  }
  if (log_space > std::log(2.0e5)) {  // (with collect_ties the DFS re-finds the seed and lists it)
    std::vector<int> g;
    double gj = std::numeric_limits<double>::infinity();
    // packing seeds: whole groups first, fullest first -- within the fullest outer group first, or
    // ignoring the outer levels.  Greedy growth from the cheapest pair can straddle groups on a
    // partitioned node (a 40-XCP request ending up over 6 packages where 5 whole ones exist), and a
    // poor incumbent leaves the bound nothing to cut.
    double seed_span = std::numeric_limits<double>::infinity();
    for (int outer = 0; outer < 2 && !lv_.empty(); ++outer) {
      std::vector<int> order = F;
      const auto& in = lv_[0];
      const Level* out = (outer && lv_.size() > 1) ? &lv_.back() : nullptr;
      std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
        if (out) {
          const int fa = out->free[out->gid[a]], fb = out->free[out->gid[b]];
          if (fa != fb) return fa > fb;
          if (out->gid[a] != out->gid[b]) return out->gid[a] < out->gid[b];
        }
        const int fa = in.free[in.gid[a]], fb = in.free[in.gid[b]];
        if (fa != fb) return fa > fb;
        return in.gid[a] < in.gid[b];
      });
      std::vector<int> cand(order.begin(), order.begin() + k);
      std::sort(cand.begin(), cand.end());
      Terms tm;
      const double cj = evaluate(cand, &tm);
      if (cj < gj - kEps) {
        gj = cj;
        g = cand;
        seed_span = tm.span;
      }
    }
    // The greedy + 1-swap seed (O(k m) evaluations per pass) only when packing left groups
    // straddled: a span-0 packing is already the kind of set the bound needs, and the search below
    // proves or improves it either way.
    if (!(seed_span <= 0.0)) {
      std::vector<int> gg;
      double ggj = std::numeric_limits<double>::infinity();
      greedy(k, F, &gg, &ggj, false, &cls_of);
      if (ggj < gj - kEps || g.empty()) {
        gj = ggj;
        g = gg;
      }
    }
    best_j = gj;
    for (int dev : g) best_pos.push_back((int)(std::lower_bound(F.begin(), F.end(), dev) - F.begin()));
  }

  std::function<void(int, double, double, double, double)> dfs = [&](int start, double pairsum, double pairmax, double accsum,
                                                                    double defmax) {
    if (aborted) return;
    const int d = (int)chosen.size();
    if (d == k) {
      ++leaves;
      double j = leaf_objective(pairsum, pairmax, accsum, defmax);
      if (j < best_j - kEps) {
        best_j = j;
        best_pos = chosen;
        if (collect_ties) tie_pos.assign(1, chosen);
      } else if (collect_ties && j <= best_j + kEps && tie_pos.size() < max_ties) {
        tie_pos.push_back(chosen);
      }
      return;
    }
    if (++nodes > node_limit) {
      aborted = true;
      return;
    }
    const int r = k - d;
    // lower bound over completions drawn from F[start..m)
    if (std::isfinite(best_j)) {
      double comm_lb = 1.0, bott_lb = 1.0;
      if (k >= 2) {
        int cnt = m - start;
        for (int c = 0; c < cnt; ++c) scratch[c] = cross[d][start + c] + 0.5 * pre[start + c][r - 1];
        std::nth_element(scratch.begin(), scratch.begin() + (r - 1), scratch.begin() + cnt);
        double add = 0;
        for (int c = 0; c < r; ++c) add += scratch[c];
        // nth_element leaves the r smallest in [0, r) in arbitrary order
        comm_lb = (pairsum + std::max(add, 0.0)) / pairs_k;
        bott_lb = std::max(pairmax, comm_lb);  // the costliest pair is at least the mean
      }
      // span look-ahead: the r devices still to choose come from positions >= start; they fit into
      // the touched groups' reachable free devices plus whole untouched groups, taken largest first,
      // so a completion touches at least that many more groups.  This is what lets packing problems
      // prune: on a CPX node (64 XCPs in 8 packages) a 24-XCP request that cannot avoid a fourth
      // package is worse than any three-package incumbent, and is cut as soon as that is certain.
      double span_lb = 0;
      for (size_t l = 0; l < lv_.size(); ++l) {
        const auto& lv = lv_[l];
        const int G = (int)lv.free.size();
        const int* reach = &suf[l][(size_t)start * G];  // free devices of each group at positions >= start
        int spare = 0, nun = 0;
        for (int g = 0; g < G; ++g) {
          if (take[l][g] > 0) spare += reach[g];
          else if (reach[g] > 0) ucap[nun++] = reach[g];
        }
        int extra = 0;
        if (r > spare) {
          std::sort(ucap.begin(), ucap.begin() + nun, std::greater<int>());
          int need = r - spare;
          for (int i = 0; i < nun && need > 0; ++i) {
            need -= ucap[i];
            ++extra;
          }
        }
        span_lb += std::max(0, touched[l] + extra - mg[l]);
      }
      // the deficit of the pairs chosen so far can only grow
      double lb = (1.0 - wb) * comm_lb + wb * bott_lb + pol_.w_span * span_lb + pol_.w_access * ((accsum + r * amin) / k) +
                  pol_.w_link_deficit * (k >= 2 ? defmax : 0.0);
      if (collect_ties ? lb > best_j + kEps : lb >= best_j - kEps) return;
    }
    for (int c = start; c <= m - r; ++c) {
      if (prev_same[c] >= 0 && !inset[prev_same[c]]) continue;  // non-canonical: its class predecessor was skipped
      const int dev = F[c];
      // push
      chosen.push_back(c);
      inset[c] = 1;
      for (size_t l = 0; l < lv_.size(); ++l) {
        int g = lv_[l].gid[dev];
        if (take[l][g]++ == 0) touched[l] += 1;
      }
      const double add_pairs = cross[d][c];
      const double new_max = d > 0 ? std::max(pairmax, xmax[d][c]) : pairmax;
      const double new_def = has_def && d > 0 ? std::max(defmax, dmax[d][c]) : defmax;
      if (d + 1 < k) {
        const double* row = &p_.cost[(size_t)dev * n];
        for (int q = c + 1; q < m; ++q) {
          cross[d + 1][q] = cross[d][q] + row[F[q]];
          xmax[d + 1][q] = d > 0 ? std::max(xmax[d][q], row[F[q]]) : row[F[q]];
        }
        if (has_def) {
          const double* drow = &p_.deficit[(size_t)dev * n];
          for (int q = c + 1; q < m; ++q) dmax[d + 1][q] = d > 0 ? std::max(dmax[d][q], drow[F[q]]) : drow[F[q]];
        }
      }
      dfs(c + 1, pairsum + add_pairs, new_max, accsum + p_.access[dev], new_def);
      // pop
      for (size_t l = 0; l < lv_.size(); ++l) {
        int g = lv_[l].gid[dev];
        if (--take[l][g] == 0) touched[l] -= 1;
      }
      chosen.pop_back();
      inset[c] = 0;
      if (aborted) return;
    }
  };
  dfs(0, 0.0, -std::numeric_limits<double>::infinity(), 0.0, 0.0);

  std::vector<int> ids;
  for (int pos : best_pos) ids.push_back(F[pos]);
  res.exact = !aborted;
  if (aborted) {  // the node budget ran out: the better of the search's best and greedy + 1-swap
    double gj = std::numeric_limits<double>::infinity();
    std::vector<int> g;
    greedy(k, F, &g, &gj, false, &cls_of);
    if (best_pos.size() != (size_t)k || gj < evaluate(ids, nullptr) - kEps) ids = g;
  }
  res.ids = ids;
  res.objective = evaluate(ids, &res.terms);
  res.feasible = true;
  if (collect_ties) {
    if (aborted || tie_pos.empty()) {
      res.ties.assign(1, ids);
    } else {
      for (const auto& t : tie_pos) {
        std::vector<int> s;
        for (int pos : t) s.push_back(F[pos]);
        res.ties.push_back(std::move(s));
      }
    }
  }
  res.nodes = nodes;
  res.leaves = leaves;
  return res;
}

Result Engine::worst(int k, uint64_t node_limit) const {
  // Exhaustive when C(m, k) fits the budget (lexicographic, first strict maximum: the same set as
  // itertools.combinations + first-maximum in core.worst); otherwise greedy ascent + 1-swap from
  // every seed with exact=false.  CPX nodes (64 XCPs, k=8: C(64,8) ~ 4.4e9) take the second path.
  Result res;
  const int n = p_.n;
  std::vector<int> F;
  for (int i = 0; i < n; ++i)
    if (p_.free[i]) F.push_back(i);
  const int m = (int)F.size();
  if (k <= 0 || m < k) return res;
  const double log_comb = std::lgamma(m + 1.0) - std::lgamma(k + 1.0) - std::lgamma(m - k + 1.0);
  std::vector<int> best;
  if (log_comb <= std::log((double)std::max<uint64_t>(node_limit, 1))) {
    std::vector<int> idx(k);
    std::iota(idx.begin(), idx.end(), 0);
    double bj = -std::numeric_limits<double>::infinity();
    std::vector<int> cur(k);
    while (true) {
      for (int i = 0; i < k; ++i) cur[i] = F[idx[i]];
      double j = evaluate(cur, nullptr);
      ++res.leaves;
      if (j > bj + kEps) {
        bj = j;
        best = cur;
      }
      int i = k - 1;
      while (i >= 0 && idx[i] == m - k + i) --i;
      if (i < 0) break;
      ++idx[i];
      for (int q = i + 1; q < k; ++q) idx[q] = idx[q - 1] + 1;
    }
  } else {
    double bj = -std::numeric_limits<double>::infinity();
    greedy(k, F, &best, &bj, /*maximise=*/true);
    res.exact = false;
  }
  res.ids = best;
  res.objective = evaluate(best, &res.terms);
  res.feasible = true;
  return res;
}

}  // namespace gtk
