#!/usr/bin/env python3
"""Hand-made mutants of the control plane's decision code, each run against the tests that should
catch it (a mutation-testing pass; README "Mutation testing of the control plane").

    python tools/mutants.py                  # every group
    python tools/mutants.py --only ledger    # one group (ledger, cache, plugin, informer, rbac, numa, cordon, objective, dp, guard,
                                             # banding, gaia, repartition, extender, contract)

Each mutant replaces one line (or a few) of a source file, runs the group's tests with pytest-xdist,
and restores the file whatever happens.  ``CAUGHT`` = some test failed, ``SURVIVED`` = the tests did
not notice: either a missing test or an equivalent mutant (listed with ``equivalent=True`` and a
reason; they are reported, not failed).  The guard's mutants rebuild ``libgtk_vgpu.so`` and its
sanitizer self-tests, before and after.  Refuses to run on a tree with uncommitted changes to the
files it mutates.  Exit status 1 when a non-equivalent mutant survives.
"""
import argparse
import os
import subprocess
import sys
from dataclasses import dataclass
from typing import List

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@dataclass
class Mutant:
    group: str
    path: str
    old: str
    new: str
    equivalent: bool = False
    why: str = ""


CACHE = "gpu_topology_on_k8s_amd/extender/cache.py"
SCHED = "gpu_topology_on_k8s_amd/extender/scheduler.py"
LEDGER = "gpu_topology_on_k8s_amd/extender/ledger.py"
PLUGIN = "gpu_topology_on_k8s_amd/deviceplugin/plugin.py"
DP = "gpu_topology_on_k8s_amd/parallel/dp.py"
GUARD = "csrc/vgpu/vgpu_guard.cpp"
CHECKS = "gpu_topology_on_k8s_amd/ops/checks.py"
GAIA = "gpu_topology_on_k8s_amd/placement/gaia.py"
REPART = "gpu_topology_on_k8s_amd/deviceplugin/repartition.py"
ANN = "gpu_topology_on_k8s_amd/k8s/annotations.py"
INFORMER = "gpu_topology_on_k8s_amd/k8s/informer.py"
RBAC = "gpu_topology_on_k8s_amd/k8s/rbac.py"
NUMA_ALIGN = "gpu_topology_on_k8s_amd/placement/numa_align.py"
PLUGIN_MAIN = "gpu_topology_on_k8s_amd/deviceplugin/__main__.py"
KUBELET = "gpu_topology_on_k8s_amd/deviceplugin/kubelet.py"
CORE = "gpu_topology_on_k8s_amd/placement/core.py"
ENGINE = "csrc/placement/engine.cpp"

MUTANTS: List[Mutant] = [
    # allocation ledger (cross-extender bind safety)
    Mutant("ledger", CACHE, "if k not in self.settled_at and now - self._first_seen(k, now) <= g_s",
           "if now - self._first_seen(k, now) <= g_s"),
    Mutant("ledger", CACHE, "            if key not in self.allocs:  # being bound by another extender",
           "            if False:  # being bound by another extender"),
    Mutant("ledger", LEDGER, "                api.patch_lease(self.namespace, lease_name(node), {key: value}, resource_version=lease_rv)",
           "                api.patch_lease(self.namespace, lease_name(node), {key: value}, resource_version=None)"),
    Mutant("ledger", LEDGER, "            api.patch_node(node, annotations={key: dump_ledger(entries, node_gen + 1, uids)}, resource_version=node_rv)",
           "            api.patch_node(node, annotations={key: dump_ledger(entries, node_gen + 1, uids)}, resource_version=None)"),
    Mutant("ledger", CACHE, "            st.present[key] = str(meta(obj).get(\"uid\", \"\"))\n            st.resettle()", "            pass"),
    Mutant("ledger", SCHED, "                        entries[key] = (tuple(d.ids), now)", "                        pass"),
    Mutant("ledger", CACHE, "                if self.settled_at.get(k) == (t, uid) or self.present.get(k) == uid:",
           "                if k in self.settled_at or k in self.present:"),
    Mutant("ledger", CACHE, "seen[k] = prev if prev is not None and prev[:2] == (ids, at) else (ids, at, now)",
           "seen[k] = prev if prev is not None and prev[0] == ids else (ids, at, now)"),
    Mutant("ledger", SCHED, "                self._ledger_release(node, key)", "                pass"),
    Mutant("ledger", SCHED, "                    if self.cache.refresh_node(node) is not st:",
           "                    if self.cache.refresh_node(node) is not st and False:", equivalent=True,
           why="the node object is re-created only when a node is deleted and re-added mid-bind"),
    Mutant("ledger", SCHED, "                if attempt and time.monotonic() - started > self.cfg.bind_budget_s:",
           "                if False:"),
    Mutant("ledger", SCHED, "            if self.cfg.ledger and recorded is not None and time.monotonic() - recorded > LEDGER_GRACE_S / 2:",
           "            if False:"),
    Mutant("ledger", CACHE, "                floor = None if floor is None or lrv is None else max(floor, lrv)",
           "                floor = floor"),
    # overlay / LIST epochs (the cache's view of this process's binds)
    Mutant("cache", CACHE, "                after_bind = list_epoch > self._overlay_epoch.get((st.name, key), 0)",
           "                after_bind = True"),
    Mutant("cache", CACHE, "                elif after_bind and consistent:", "                elif consistent:"),
    Mutant("cache", CACHE, "        consistent = self.consistent_lists if consistent is None else consistent",
           "        consistent = self.consistent_lists"),
    Mutant("cache", CACHE, "                self._overlay_epoch[(node, pod)] = self._next_epoch()",
           "                self._overlay_epoch[(node, pod)] = 0"),
    Mutant("cache", CACHE, "            self._overlay_epoch[(node, pod)] = math.inf", "            self._overlay_epoch[(node, pod)] = 0"),
    Mutant("cache", CACHE, "        if list_epoch < st.list_epoch:", "        if False:"),
    Mutant("cache", CACHE, "            if a.assigned or (now - a.assume_time) <= ttl:", "            if a.assigned:"),
    Mutant("cache", CACHE, '        return self._next_epoch() if kind == "Pod" else None', "        return None"),
    Mutant("cache", CACHE, "                    if after_bind:  # a LIST started after the bind: authoritative from now on",
           "                    if True:  # a LIST started after the bind: authoritative from now on", equivalent=True,
           why="a LIST that shows the pod carries its annotation: dropping the overlay entry early loses nothing"),
    # device plugin
    Mutant("plugin", PLUGIN,
           "            if c.pa is not None and ids_s <= set(c.pa.group) and (nxt == n or (nxt is None and c.adm is None)):",
           "            if c.pa is not None and (nxt == n or (nxt is None and c.adm is None)):"),
    Mutant("plugin", PLUGIN, 'pod = self.api.patch_pod_annotations(md.get("namespace", "default"), md["name"], ann,\n'
                             '                                                         resource_version=md.get("resourceVersion"))',
           'pod = self.api.patch_pod_annotations(md.get("namespace", "default"), md["name"], ann,\n'
           '                                                         resource_version=None)'),
    Mutant("plugin", PLUGIN, "                orphans.setdefault(owners[0], set()).update(rest)", "                pass"),
    Mutant("plugin", PLUGIN, "                target = set().union(*(unit_of[d] for d in ids)) - others",
           "                target = set(ids)"),
    Mutant("plugin", PLUGIN, "        unit = self._chain[0] | ids_s if linked else set(ids_s)", "        unit = set(ids_s)"),
    Mutant("plugin", PLUGIN, "                reused = set(ids) if self._gpa_must is None else self._gpa_must & set(ids)",
           "                reused = set(ids)"),
    Mutant("plugin", PLUGIN, "                    or (rec is not None and (pod is None or meta(pod).get(\"uid\", \"\") != rec.uid)))",
           "                    or False)", equivalent=True,
           why="defence in depth: a call that reuses nothing never links, and an ended pod's record leaves _admissions"),
    Mutant("plugin", PLUGIN, "            if nxt is not None and nxt != size:", "            if False:"),
    Mutant("plugin", PLUGIN, "        out.sort(key=lambda c: (c.adm is None or c.adm.done == 0, c.pa is None,",
           "        out.sort(key=lambda c: (False, c.pa is None,"),
    Mutant("plugin", PLUGIN, "        healthy = [a for a in avail if 0 <= a < self.topology.n and self._health.get(a, True)]",
           "        healthy = [a for a in avail if 0 <= a < self.topology.n]"),
    Mutant("plugin", PLUGIN, "            unhealthy = [i for i in ids if not self._health.get(i, True)]", "            unhealthy = []"),
    Mutant("plugin", PLUGIN, "            if not ids:\n                continue  # not admitted yet (or not ours)",
           "            if False:\n                continue  # not admitted yet (or not ours)"),
    Mutant("plugin", PLUGIN, "                ann[ANN_ASSUME_TIME] = str(int(self.clock()))", "                pass"),
    Mutant("plugin", PLUGIN, '            if pod_phase(p) != "Pending" and (pa is None or pa.assigned):',
           '            if pod_phase(p) != "Pending":'),
    Mutant("plugin", PLUGIN, '            if pod_phase(p) != "Pending" and (pa is None or pa.assigned):', '            if False:'),
    Mutant("plugin", PLUGIN, "        if self.cfg.container_ipc_mode:  # before the pod's own env", "        if False:  # before the pod's own env"),
    Mutant("plugin", PLUGIN, '            return int(res.get("k", 0)) >= int(json.loads(old).get("k", 0))', "            return True"),
    Mutant("plugin", KUBELET, '        if getattr(p.options, "pre_start_required", False):\n            try:',
           "        if False:\n            try:"),
    # informer (client-go reflector semantics)
    Mutant("informer", INFORMER, "                failures += 1\n                self.last_error = str(e)",
           "                failures += 1\n                rv = None\n                self.last_error = str(e)"),
    Mutant("informer", INFORMER, "                                                         resource_version=None if cont else rv_param,",
           "                                                         resource_version=rv_param,"),
    Mutant("informer", INFORMER, '                items, cont, rv_param = [], "", None', '                items, cont = [], ""'),
    Mutant("informer", INFORMER, "        return d * (1.0 + self.jitter * self._rng.uniform(-1.0, 1.0))", "        return d"),
    Mutant("informer", INFORMER, "        d = min(self.max_backoff, self.backoff * (2 ** max(0, failures - 1)))",
           "        d = self.backoff * (2 ** max(0, failures - 1))"),
    Mutant("informer", INFORMER, "self.on_event(t, kind, self.transform(kind, obj) if self.transform is not None else obj)",
           "self.on_event(t, kind, obj)"),
    Mutant("informer", INFORMER, "                    failures = 0\n                    new_rv", "                    new_rv"),
    Mutant("informer", CACHE, "        if sync and stale and self.informer is None:", "        if sync and stale and not self.informed():"),
    Mutant("informer", SCHED, "        if k and not self.ready:\n            self.metrics.request(\"filter\", \"not_ready\")",
           "        if False:\n            self.metrics.request(\"filter\", \"not_ready\")"),
    # per-identity RBAC of the deploy manifests
    Mutant("rbac", RBAC, "        if self.identity.own_node_only and node != self.node_name:", "        if False:"),
    Mutant("rbac", RBAC, "and (self.namespace is None or self.namespace == namespace))", ")"),
    Mutant("rbac", RBAC, "                out[m.group(1)].own_node_only = True", "                pass"),
    # placement under the kubelet's Topology Manager
    Mutant("numa", NUMA_ALIGN, "            if needed < len(aligned):", "            if needed <= len(aligned):", equivalent=True,
           why="needed == aligned: the plugin, asked over exactly the aligned devices, answers all of them"),
    Mutant("numa", NUMA_ALIGN, "            in_mask = sum(1 for d in all_devices if numa.get(d, -1) in mask)",
           "            in_mask = sum(1 for d in available if numa.get(d, -1) in mask)"),
    Mutant("numa", NUMA_ALIGN, "        elif pref == best[1] and (len(mask), _mask_value(mask)) < (len(best[0]), _mask_value(best[0])):",
           "        elif pref == best[1] and (len(mask), sorted(mask)) < (len(best[0]), sorted(best[0])):"),
    Mutant("numa", NUMA_ALIGN, "        for combo in itertools.combinations(sorted(nodes), width):",
           "        for combo in itertools.combinations(sorted(nodes, reverse=True), width):", equivalent=True,
           why="the merge compares equally narrow hints by their bitmask value, whatever the iteration order"),
    Mutant("numa", NUMA_ALIGN, "            if any(numa.get(d, -1) >= 0 and numa[d] not in mask for d in reusable):", "            if False:"),
    Mutant("numa", NUMA_ALIGN, '    admit = policy == "best-effort" or pref', "    admit = True"),
    Mutant("numa", NUMA_ALIGN, '        if kind == "init":\n            reuse |= got', '        if False:\n            reuse |= got'),
    Mutant("numa", PLUGIN, "                if self._gpa_must is None and self.cfg.topology_manager.active and not self._continuing():",
           "                if False:"),
    Mutant("numa", SCHED, "            if tm.active and fraction is None and steps:\n                ids, why = self._choose_aligned(",
           "            if False:\n                ids, why = self._choose_aligned("),
    Mutant("numa", SCHED, "                            if tm.active and fraction is None and steps:",
           "                            if False:"),
    # placement objective: the link-deficit term (Python and the native engine)
    Mutant("objective", CORE, "        dft = float(p.deficit[np.ix_(ids, ids)].max())", "        dft = 0.0"),
    Mutant("objective", CORE, "        out[m] = np.maximum(0.0, c[m] / best - 1.0 - LINK_DEFICIT_BAND)",
           "        out[m] = np.maximum(0.0, c[m] / best - 1.0)"),
    Mutant("objective", ENGINE, "          for (int q = c + 1; q < m; ++q) dmax[d + 1][q] = d > 0 ? std::max(dmax[d][q], drow[F[q]]) : drow[F[q]];",
           "          for (int q = c + 1; q < m; ++q) dmax[d + 1][q] = 0.0;"),
    Mutant("objective", ENGINE, "                  pol_.w_link_deficit * (k >= 2 ? defmax : 0.0);\n      if (collect_ties",
           "                  0.0;\n      if (collect_ties", equivalent=True,
           why="a weaker lower bound prunes less; the search stays exact"),
    # operator GPU cordon
    Mutant("cordon", PLUGIN, "                self._holds.setdefault(i, self.CORDON_HOLD)  #", "                pass  #"),
    Mutant("cordon", PLUGIN, "            out |= {g.index for g in t.gpus if g.physical == t.gpus[i].physical}", "            out.add(i)"),
    Mutant("cordon", PLUGIN_MAIN, "    plugin.poll_node()  # a cordoned GPU is never advertised Healthy", "    pass  # a cordoned GPU is never advertised Healthy"),
    # data-parallel reduction
    Mutant("dp", DP, "        return b.start + self.rank * c, b.start + (self.rank + 1) * c", "        return b.start, b.start + c"),
    Mutant("dp", DP, "                if b.work is None:\n                    self._launch(b)", "                if False:\n                    self._launch(b)"),
    Mutant("dp", DP, "        return 1.0 / self.world if self.average else 1.0", "        return 1.0"),
    Mutant("dp", DP, "            self.snapshot[b.start:b.end].copy_(view)", "            pass"),
    Mutant("dp", DP, "            buf.copy_(view)", "            pass"),
    # vGPU guard (rebuilt per mutant)
    Mutant("guard", GUARD, "      if (total + (long long)bytes > s.limit[dev]) return false;", "      if (false) return false;"),
    Mutant("guard", GUARD, "  if (s.used[dev] + (long long)bytes > s.limit[dev]) return false;", "  if (false) return false;"),
    Mutant("guard", GUARD, "    if (s.ptrs.count(*ptr)) return e;  // the runtime took it from a device pool: counted there",
           "    if (false) return e;"),
    Mutant("guard", GUARD, "        if (i == s.mine || slot_alive(s.acct_fd, i)) total += s.table->slot[i].used[dev];",
           "        if (i == s.mine) total += s.table->slot[i].used[dev];"),
    Mutant("guard", GUARD, "    if (o >= 0) s.limit[o] = l.bytes;", "    if (o >= 0) s.limit[0] = l.bytes;"),
    Mutant("guard", GUARD, "    if (o < 0) ++unmatched, o = unmatched_ordinal(a, \"hbm_limit_bdf\", l.addr, l.fallback);",
           "    if (o < 0) ++unmatched;"),
    Mutant("guard", GUARD, "    if (any)  // an empty intersection would stop the queue: the share's own mask applies instead",
           "    if (true)"),
    # probe banding
    Mutant("banding", CHECKS, "            if abs(meas[p] - med) <= band * med and meas[p] >= floors[p]:",
           "            if abs(meas[p] - med) <= band * med:"),
    Mutant("banding", CHECKS, "                if abs(med - pmed) <= cls_band * pmed:", "                if False:"),
    Mutant("banding", CHECKS, "            band = max(cls_band, min(float(sp[p]), BAND_SPREAD_CAP))", "            band = cls_band"),
    Mutant("banding", CHECKS, "            band = max(cls_band, min(float(sp[p]), BAND_SPREAD_CAP))",
           "            band = max(cls_band, float(sp[p]))"),
    Mutant("banding", CHECKS,
           "    return int(topo.link_type[a, b]), int(topo.hops[a, b]), int(topo.physical[a]) == int(topo.physical[b])",
           "    return int(topo.link_type[a, b]), int(topo.hops[a, b]), True"),
    # Gaia algorithms
    Mutant("gaia", GAIA, "        leaf = _pick(cands, lambda l: (round(l.resources, 9), l.access_cost), tie_break, rng)",
           "        leaf = _pick(cands, lambda l: (l.access_cost,), tie_break, rng)"),
    Mutant("gaia", GAIA, "    pool = cands if cands else leaves", "    pool = leaves"),
    Mutant("gaia", GAIA, "        lambda c: (c.link_cost, m * (_min_access(c, m) / m), c.free_whole - m),",
           "        lambda c: (c.link_cost, c.free_whole - m),"),
    Mutant("gaia", GAIA, "    cands = [l for l in leaves if l.used > 1e-12 and m <= l.resources + 1e-12]",
           "    cands = [l for l in leaves if m <= l.resources + 1e-12]", equivalent=True,
           why="an unused leaf has resources 1.0, so best fit prefers any fitting fragment anyway"),
    # partition switch
    Mutant("repartition", REPART, '            changed = bool(res.get("layout_changed", res["ok"]))', '            changed = bool(res["ok"])'),
    Mutant("repartition", REPART, "                return idle_fn() and not (h is not None and h.contended())",
           "                return idle_fn()"),
    Mutant("repartition", REPART, "        if contract.partition_failed_key in ann:", "        if False:"),
    # wire contract (pod / node annotations)
    Mutant("contract", ANN, "        if g is None or any(i < 0 for i in g):", "        if g is None:"),
    Mutant("contract", ANN, "                g = parse_group(ann.get(ANN_GPU_ID_ALIAS))  # diagram alias, read-only", "                pass"),
    Mutant("contract", ANN, '        assigned = str(ann.get(ANN_ASSIGNED, "false")).lower() == "true"',
           '        assigned = str(ann.get(ANN_ASSIGNED, "false")) == "true"'),
    Mutant("contract", ANN, '    return [int(x) for x in s.split(",") if x.strip() != ""]', '    return [int(x) for x in s.split(",")]'),
    Mutant("contract", ANN, "    except (ValueError, TypeError, KeyError, AttributeError):\n        return {}",
           "    except (ValueError,):\n        return {}"),
    # extender node evaluation
    Mutant("extender", SCHED, "        rank = obj + node_packing_term(free, k, t.n, self.cfg.policy)", "        rank = obj"),
    Mutant("extender", SCHED, "                if dev_mem <= 0:", "                if False:"),
    Mutant("extender", SCHED, '        if s > 1 and unit != "slice":', "        if False:"),
]

TESTS = {
    "ledger": ["tests/test_extender_ledger.py", "tests/test_extender.py", "tests/test_cluster_features.py", "tests/test_churn.py",
               "tests/test_rbac.py"],
    "cache": ["tests/test_cluster_features.py", "tests/test_extender.py", "tests/test_extender_ledger.py", "tests/test_churn.py",
              "tests/test_informer.py"],
    "plugin": ["tests/test_deviceplugin.py", "tests/test_cluster_features.py", "tests/test_preferred_allocation_props.py",
               "tests/test_daemons.py", "tests/test_health.py", "tests/test_sim.py", "tests/test_churn.py",
               "tests/test_reprobe_admission.py", "tests/test_partition.py", "tests/test_shares.py",
               "tests/test_multicontainer.py"],
    "informer": ["tests/test_informer.py", "tests/test_cluster_features.py", "tests/test_rbac.py"],
    "rbac": ["tests/test_rbac.py", "tests/test_config_cli.py"],
    "numa": ["tests/test_topology_manager.py"],
    "cordon": ["tests/test_cordon.py"],
    "objective": ["tests/test_placement.py", "tests/test_placement_ab.py"],
    "dp": ["tests/test_dp_check.py", "tests/test_llama_dp_cpu.py", "tests/test_checkpoint.py"],
    "guard": ["tests/test_vgpu_guard.py"],
    "banding": ["tests/test_probe_banding.py", "tests/test_probe_checks.py"],
    "gaia": ["tests/test_gaia_conformance.py", "tests/test_placement.py"],
    "repartition": ["tests/test_partition.py", "tests/test_daemons.py"],
    "extender": ["tests/test_shares.py", "tests/test_extender.py", "tests/test_cluster_features.py"],
    "contract": ["tests/test_k8s.py", "tests/test_extender.py", "tests/test_extender_fuzz.py", "tests/test_extender_ledger.py",
                 "tests/test_deviceplugin.py", "tests/test_cluster_features.py"],
}

GUARD_TARGETS = "vgpu_guard,vgpu_selftest_asan,vgpu_selftest_tsan"
NATIVE_TARGETS = {GUARD: GUARD_TARGETS, ENGINE: "_placement,engine_selftest"}  # mutated sources rebuilt per mutant


def _rebuild(path: str) -> bool:
    p = subprocess.run([sys.executable, "-m", "gpu_topology_on_k8s_amd._native.build", "--only", NATIVE_TARGETS[path]], cwd=REPO,
                       capture_output=True, text=True, timeout=900)
    return p.returncode == 0


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--only", default="", help="comma-separated groups")
    ap.add_argument("-n", type=int, default=6, help="pytest-xdist workers")
    a = ap.parse_args()
    groups = [g for g in a.only.split(",") if g] or list(TESTS)
    todo = [m for m in MUTANTS if m.group in groups]
    paths = sorted({m.path for m in todo})
    dirty = subprocess.run(["git", "status", "--porcelain", "--", *paths], cwd=REPO, capture_output=True, text=True).stdout
    if dirty.strip():
        print("refusing: uncommitted changes in\n" + dirty, file=sys.stderr)
        return 2
    bad = 0
    for m in todo:
        path = os.path.join(REPO, m.path)
        src = open(path).read()
        if m.old not in src:
            print(f"MISSING   [{m.group}] {m.old.strip()[:90]}")
            bad += 1
            continue
        try:
            open(path, "w").write(src.replace(m.old, m.new, 1))
            if m.path in NATIVE_TARGETS and not _rebuild(m.path):
                print(f"NOBUILD   [{m.group}] {m.old.strip()[:90]}")
                continue
            p = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-n", str(a.n), "-m", "not gpu",
                                *TESTS[m.group]], cwd=REPO, capture_output=True, text=True, timeout=1800)
            caught = p.returncode != 0
            tag = "CAUGHT  " if caught else ("EQUIV   " if m.equivalent else "SURVIVED")
            if not caught and not m.equivalent:
                bad += 1
            note = f"  ({m.why})" if m.equivalent and not caught else ""
            print(f"{tag}  [{m.group}] {m.old.strip()[:90].replace(chr(10), ' ')}{note}", flush=True)
        finally:
            open(path, "w").write(src)
    for path in sorted({m.path for m in todo if m.path in NATIVE_TARGETS}):
        _rebuild(path)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
