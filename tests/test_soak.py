"""Every round-6 feature at once, under random churn: nodes whose kubelets run different Topology
Manager policies, multi-container / init / sidecar pods, operator GPU cordons coming and going, the
extender on its informer, every component as its deploy ServiceAccount.  Invariants after every
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
           "strict": TopologyManager("single-numa-node", "pod")}
    with SimCluster({n: fx.f7_mi355x() for n in tms}, topology_manager=tms, informer=True, rbac=True) as c:
        live, cordoned, placed = [], {}, 0
        for i in range(150):
            ev = rng.random()
            if live and ev < 0.3:
                c.complete(live.pop(rng.randrange(len(live))))
            elif ev < 0.38:  # the operator cordons or releases a GPU somewhere
                node = rng.choice(list(tms))
                want = "" if cordoned.get(node) else str(rng.randrange(8))
                c.api.patch_node(node, annotations={C.cordon_key: want})
                c.nodes[node].plugin.poll_node()
                cordoned[node] = want
            # the informer delivers what just changed before the next decision
            assert _wait(lambda: all(
                {g.index for g in c.extender.cache.get(n, sync=False).topology.gpus if not g.healthy}
                == ({int(cordoned[n])} if cordoned.get(n) else set()) for n in tms))
            name = f"p{i}"
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
                assert int(cordoned[r.node]) not in r.allocated, (r, cordoned)
            live.append(name)
            placed += 1
        assert placed >= 40
        assert c.denied == []
        assert not any(n.kubelet.rejected for n in c.nodes.values())
