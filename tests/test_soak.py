"""Every round-6 feature at once, under random churn: nodes whose kubelets run different Topology
Manager policies, multi-container / init / sidecar pods, operator GPU cordons coming and going, the
extender as two replicas (kube-scheduler HA) each on its own informer, every component as its deploy
ServiceAccount, and extender and device plugin restarts in between.  Invariants after every
step: a bound pod is admitted (no kubelet rejection) with exactly the GROUP the extender bound
(reconcile off), no new pod lands on a cordoned GPU, no request is refused by RBAC."""
import random
import time

import pytest

from gpu_topology_on_k8s_amd.k8s import Contract, PodAssignment
from gpu_topology_on_k8s_amd.k8s.objects import annotations as obj_annotations
from gpu_topology_on_k8s_amd.placement.numa_align import TopologyManager
from gpu_topology_on_k8s_amd.sim import SimCluster
from gpu_topology_on_k8s_amd.topology import fixtures as fx
from gpu_topology_on_k8s_amd.topology.shares import time_slice

C = Contract()


def _shape(rng):
    r = rng.random()
    if r < 0.45:
        return {"gpus": rng.choice([1, 1, 2, 2, 3, 4, 8])}
    if r < 0.7:
        return {"gpus": 0, "split": list(rng.choice([(1, 1), (1, 2), (2, 2), (1, 3)]))}
    if r < 0.85:
        app = rng.choice([1, 2, 3])
        return {"gpus": 0, "split": [app], "init": [rng.choice([1, 2, app])]}
    return {"gpus": 0, "split": [rng.choice([1, 2])], "sidecars": [1]}


def _physical(t, i):
    """Every device of device i's physical GPU (a cordon names the whole GPU: all its slices)."""
    return {g.index for g in t.gpus if g.physical == t.gpus[i].physical}


def _wait(pred, timeout=5.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if pred():
            return True
        time.sleep(0.02)
    return False


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_everything_at_once_under_churn(seed):
    rng = random.Random(seed)
    tms = {"plain": TopologyManager(), "aligned": TopologyManager("best-effort", "container"),
           "strict": TopologyManager("single-numa-node", "pod"), "sliced": TopologyManager("best-effort", "container")}
    nodes = {n: (time_slice(fx.f7_mi355x(), 2) if n == "sliced" else fx.f7_mi355x()) for n in tms}
    with SimCluster(nodes, topology_manager=tms, informer=True, rbac=True, replicas=2) as c:
        live, cordoned, placed = [], {}, 0
        for i in range(150):
            ev = rng.random()
            if live and ev < 0.3:
                c.complete(live.pop(rng.randrange(len(live))))
            elif ev < 0.34:  # a component restarts: the extender (stateless) or a node's plugin
                if rng.random() < 0.5:
                    c.restart_extender()
                else:
                    c.restart_plugin(rng.choice(list(tms)))
            elif ev < 0.42:  # the operator cordons or releases a GPU somewhere
                node = rng.choice(list(tms))
                want = "" if cordoned.get(node) else str(rng.randrange(nodes[node].n))
                c.api.patch_node(node, annotations={C.cordon_key: want})
                c.nodes[node].plugin.poll_node()
                cordoned[node] = want
            # the informer delivers what just changed before the next decision
            assert _wait(lambda: all(
                {g.index for g in e.cache.get(n, sync=False).topology.gpus if not g.healthy}
                == (_physical(nodes[n], int(cordoned[n])) if cordoned.get(n) else set()) for n in tms for e in c.extenders))
            name = f"p{i}"
            if rng.random() < 0.2:  # time slices: one pool of their own (the sliced node)
                c.submit(name, **rng.choice([{"gpus": 1}, {"gpus": 2}, {"gpus": 0, "split": [1, 1]}]), slices=True)
            else:
                c.submit(name, **_shape(rng))
            (r,) = c.schedule_pending()
            if r.node is None:
                c.delete(name)
                continue
            assert not r.error, r  # bound means admitted: no TopologyAffinityError, no Allocate refusal
            assert sorted(r.devices) == sorted(r.allocated), r
            pa = PodAssignment.from_annotations(obj_annotations(c.api.get_pod("default", name)))
            assert pa.assigned and sorted(pa.group) == sorted(r.allocated), (r, pa)
            if cordoned.get(r.node):
                assert not _physical(nodes[r.node], int(cordoned[r.node])) & set(r.allocated), (r, cordoned)
            live.append(name)
            placed += 1
            if i % 10 == 9:  # every claim was exact: the pod-resources reconcile finds nothing to fix
                assert c.reconcile() == 0, i
        assert placed >= 40
        assert c.denied == []
        assert not any(n.kubelet.rejected for n in c.nodes.values())
