"""Randomised churn through the whole in-process cluster: pods of 1-8 GPUs
arrive (sometimes scheduled concurrently), finish, the extender restarts, a kubelet restarts, and
the apiserver fails binds — after every operation the allocations must stay consistent everywhere:
disjoint per node, the size requested, the pod's GROUP annotation == the kubelet's allocation, and
the extender's per-node usage == the live pods' devices."""
import random
import time

import pytest

from gpu_topology_on_k8s_amd.k8s.annotations import PodAssignment
from gpu_topology_on_k8s_amd.k8s.objects import annotations as obj_annotations
from gpu_topology_on_k8s_amd.sim import SimCluster
from gpu_topology_on_k8s_amd.topology import fixtures as fx


def _annotation_mismatches(c, live):
    out = []
    for key, node in live.items():
        ns, name = key.split("/")
        kub = c.nodes[node].kubelet.allocated[c.nodes[node].resource].get(key) or ()
        a = PodAssignment.from_annotations(obj_annotations(c.api.get_pod(ns, name)))
        if a is None or not a.assigned or sorted(a.group) != sorted(int(i) for i in kub):
            out.append((key, a, kub))
    return out


def _shape(rng, k):
    """Pod shape for a k-device request: one container, several app containers, or an init container
    (smaller or as large as the pod) in front — each Allocate'd per container by the fake kubelet."""
    r = rng.random()
    if k < 2 or r < 0.4:
        return {}
    if r < 0.75:
        cut = rng.randint(1, k - 1)
        return {"split": [cut, k - cut]}
    return {"split": [k], "init": [rng.randint(1, k)]}


def _check(c, live, request, strict=False):
    if strict:  # sequential admissions: Allocate alone must keep GROUP == the kubelet's allocation
        assert not _annotation_mismatches(c, live)
    c.reconcile()  # the plugins' periodic pass (kubelet pod-resources -> GROUP annotations), run now
    per_node = {}
    for key, node in live.items():
        ns, name = key.split("/")
        kub = c.nodes[node].kubelet.allocated[c.nodes[node].resource].get(key)
        assert kub is not None, f"{key} lost its kubelet allocation"
        ids = sorted(int(i) for i in kub)
        assert len(ids) == request[key], (key, ids)
        a = PodAssignment.from_annotations(obj_annotations(c.api.get_pod(ns, name)))
        assert a is not None and sorted(a.group) == ids, (key, a, ids)
        per_node.setdefault(node, []).extend(ids)
    for node in c.nodes:
        ids = per_node.get(node, [])
        assert len(ids) == len(set(ids)), f"double allocation on {node}: {sorted(ids)}"
        assert c.used_devices(node) == sorted(ids), (node, c.used_devices(node), sorted(ids))


@pytest.mark.parametrize("seed,informer", [(11, False), (12, False), (13, False), (21, True), (22, True)])
def test_random_churn_keeps_allocations_consistent(seed, informer):
    rng = random.Random(seed)
    with SimCluster({f"n{i}": fx.f7_mi355x() for i in range(3)}, informer=informer) as c:
        live, request, nxt, multi = {}, {}, 0, 0
        for _ in range(36):
            op = rng.random()
            strict = True
            if op < 0.55:
                for _ in range(rng.randint(1, 3)):
                    k = rng.choice([1, 1, 2, 2, 4, 8])
                    shape = _shape(rng, k)
                    c.submit(f"p{nxt}", 0 if shape else k, **shape)
                    request[f"default/p{nxt}"] = k
                    multi += bool(shape)
                    nxt += 1
                concurrent = rng.random() < 0.5
                strict = not concurrent  # concurrent binds + admissions may swap same-size pods
                for r in c.schedule_pending(concurrent=concurrent):
                    assert not r.error.startswith("admission"), r  # the extender never binds onto held devices
                    if r.node and r.allocated:
                        live[r.pod] = r.node
            elif op < 0.8 and live:
                key = rng.choice(sorted(live))
                c.complete(key.split("/")[1])
                live.pop(key)
            elif op < 0.87:
                c.restart_extender()
            elif op < 0.93:
                n = c.nodes[rng.choice(sorted(c.nodes))]
                before = n.plugin.registered
                n.kubelet.restart()
                t0 = time.time()
                while n.plugin.registered <= before and time.time() - t0 < 10:
                    time.sleep(0.02)
                n.kubelet.wait_for(c.resource)
            else:
                c.api.inject("bind_pod", 500, times=1)
            _check(c, live, request, strict=strict)
        assert multi > 0  # multi-container / init-container pods really were in the mix
        # drain: everything finishes, every node is empty again
        for key in sorted(live):
            c.complete(key.split("/")[1])
        live.clear()
        _check(c, live, request)


def test_out_of_order_admission_is_reconciled_from_pod_resources():
    """Two 1-GPU pods assumed on one node, admitted by the kubelet in the other order: Allocate cannot
    tell them apart, so their GROUP annotations end up swapped; the plugin's pod-resources pass
    restores GROUP == what the kubelet gave each pod (and records an Event)."""
    from gpu_topology_on_k8s_amd.deviceplugin.podresources import list_pod_resources
    from gpu_topology_on_k8s_amd.k8s.objects import pod_key

    with SimCluster({"n": fx.f7_mi355x()}) as c:
        c.submit("a", 1)
        c.submit("b", 1)
        ra, rb = c.schedule_pending(admit=False)  # both bound + assumed, neither admitted yet
        assert ra.node == rb.node == "n" and set(ra.devices) != set(rb.devices)
        kub = c.nodes["n"].kubelet
        kub.admit(c.api.get_pod("default", "b"), c.resource)  # b first: the kubelet's order, not the assume order
        kub.admit(c.api.get_pod("default", "a"), c.resource)
        truth = list_pod_resources(kub.pod_resources_socket)
        assert set(truth) == {"default/a", "default/b"}
        got = {k: sorted(int(i) for i in v[c.resource]) for k, v in truth.items()}

        def ann(name):
            return sorted(PodAssignment.from_annotations(obj_annotations(c.api.get_pod("default", name))).group)

        swapped = ann("a") != got["default/a"]
        assert swapped, (ann("a"), ann("b"), got)  # the ambiguity this pass exists for
        assert c.reconcile() == (2 if swapped else 0)
        assert ann("a") == got["default/a"] and ann("b") == got["default/b"]
        assert c.reconcile() == 0  # idempotent
        if swapped:
            assert any(e["reason"] == "GPUAllocationReconciled" for e in c.api.events)
        assert pod_key(c.api.get_pod("default", "a")) == "default/a"


@pytest.mark.parametrize("seed", [31, 32])
def test_random_churn_on_cpx_nodes_with_fractions(seed):
    """CPX nodes (8 packages x 8 XCPs): whole-XCP-count pods and Gaia fractions (gpu-fraction, one
    package, best fit) churn together; besides the invariants above, every fraction stays inside one
    package."""
    from gpu_topology_on_k8s_amd.k8s import Contract

    C = Contract()
    rng = random.Random(seed)
    with SimCluster({"c0": fx.f8_mi355x_cpx(), "c1": fx.f8_mi355x_cpx()}) as c:
        live, request, frac, nxt = {}, {}, set(), 0
        for _ in range(30):
            if rng.random() < 0.6:
                for _ in range(rng.randint(1, 4)):
                    name = f"p{nxt}"
                    nxt += 1
                    if rng.random() < 0.5:
                        f = rng.choice([0.125, 0.25, 0.5])
                        c.submit(name, int(f * 8), annotations={C.fraction_key: str(f)})
                        frac.add(f"default/{name}")
                        request[f"default/{name}"] = int(f * 8)
                    else:
                        k = rng.choice([1, 2, 8, 16])
                        c.submit(name, k)
                        request[f"default/{name}"] = k
                for r in c.schedule_pending(concurrent=rng.random() < 0.3):
                    if r.node and r.allocated:
                        live[r.pod] = r.node
            elif live:
                key = rng.choice(sorted(live))
                c.complete(key.split("/")[1])
                live.pop(key)
            _check(c, live, request)
            for key in frac & set(live):
                ids = c.nodes[live[key]].kubelet.allocated[c.resource][key]
                assert len({int(i) // 8 for i in ids}) == 1, (key, ids)


@pytest.mark.parametrize("seed", [41, 42])
def test_random_churn_on_time_sliced_nodes(seed):
    """SPX nodes advertised as 4 time slices per GPU (topology/shares.py): fractional pods, whole-GPU
    pods (4 slices each) and multi-GPU pods churn together; besides the invariants above every
    fraction stays on one GPU, and every container got its share and disjoint CU masks."""
    from gpu_topology_on_k8s_amd.k8s import Contract
    from gpu_topology_on_k8s_amd.topology.shares import time_slice

    C = Contract()
    rng = random.Random(seed)
    with SimCluster({"s0": time_slice(fx.f7_mi355x(), 4), "s1": time_slice(fx.f7_mi355x(), 4)}) as c:
        live, request, frac, nxt, placed = {}, {}, set(), 0, 0
        for _ in range(30):
            if rng.random() < 0.6:
                for _ in range(rng.randint(1, 4)):
                    name = f"p{nxt}"
                    nxt += 1
                    if rng.random() < 0.5:
                        f = rng.choice([0.25, 0.5, 0.75])
                        c.submit(name, int(f * 4), slices=True, annotations={C.fraction_key: str(f)})
                        frac.add(f"default/{name}")
                        request[f"default/{name}"] = int(f * 4)
                    else:
                        k = 4 * rng.choice([1, 2, 4])
                        c.submit(name, k, slices=True)
                        request[f"default/{name}"] = k
                for r in c.schedule_pending(concurrent=rng.random() < 0.3):
                    if r.node and r.allocated:
                        live[r.pod] = r.node
            elif live:
                key = rng.choice(sorted(live))
                c.complete(key.split("/")[1])
                live.pop(key)
            _check(c, live, request)
            placed += len(live)
            masks = {}
            for key in frac & set(live):
                node = live[key]
                ids = c.nodes[node].kubelet.allocated[c.nodes[node].resource][key]
                gpus = {int(i) // 4 for i in ids}
                assert len(gpus) == 1, (key, ids)
                envs = dict(c.nodes[node].kubelet.responses[key].container_responses[0].envs)
                assert float(envs["GTK_GPU_FRACTION"]) == request[key] / 4
                cus = set()
                for part in envs["HSA_CU_MASK"].split(":")[1].split(","):
                    lo, _, hi = part.partition("-")
                    cus |= set(range(int(lo), int(hi or lo) + 1))
                prev = masks.setdefault((node, gpus.pop()), set())
                assert not (prev & cus), (key, envs["HSA_CU_MASK"])  # neighbours on one GPU never share a CU
                prev |= cus
        assert placed > 0 and any(k in frac for k in request)  # the slice pool really was exercised


def test_reconcile_leaves_bound_but_not_admitted_pods_alone():
    """The kubelet has not admitted a bound pod yet (its pod-resources show no devices for it): the
    reconcile pass must not touch the extender's assumption (stamping an empty GROUP as ASSIGNED would
    hide the devices the extender set aside for it)."""
    with SimCluster({"n": fx.f7_mi355x()}) as c:
        c.submit("a", 2)
        (r,) = c.schedule_pending(admit=False)
        before = PodAssignment.from_annotations(obj_annotations(c.api.get_pod("default", "a")))
        assert c.reconcile() == 0
        after = PodAssignment.from_annotations(obj_annotations(c.api.get_pod("default", "a")))
        assert after == before and not after.assigned and sorted(after.group) == sorted(r.devices)


def test_reconcile_restores_a_lost_assignment_with_the_full_contract():
    """An admitted pod whose annotations were lost (a failed patch, a user edit) gets all three back from
    the kubelet's allocation: GROUP, ASSIGNED=true and an ASSUME_TIME."""
    from gpu_topology_on_k8s_amd.k8s.annotations import ANN_ASSIGNED, ANN_ASSUME_TIME, ANN_GROUP

    with SimCluster({"n": fx.f7_mi355x()}) as c:
        c.submit("a", 2)
        (r,) = c.schedule_pending()
        c.api.patch_pod_annotations("default", "a", {ANN_GROUP: None, ANN_ASSIGNED: None, ANN_ASSUME_TIME: None})
        assert c.reconcile() == 1
        ann = obj_annotations(c.api.get_pod("default", "a"))
        assert ann[ANN_GROUP] == ",".join(str(i) for i in sorted(r.allocated)) and ann[ANN_ASSIGNED] == "true"
        assert int(ann[ANN_ASSUME_TIME]) > 0


def test_allocate_for_an_unannotated_pod_skips_running_ones():
    """A pod scheduled around the extender is matched by its GPU count among the node's PENDING pods
    without a GROUP; a running pod of the same size (already admitted) is not a candidate."""
    from gpu_topology_on_k8s_amd.k8s.objects import make_pod

    with SimCluster({"n": fx.f7_mi355x()}) as c:
        plugin = c.nodes["n"].plugin
        old = make_pod("a-legacy-running", gpus=2, node="n")
        old["status"] = {"phase": "Running"}
        c.api.create_pod(old)
        c.api.create_pod(make_pod("b-legacy-new", gpus=2, node="n"))
        claimed = plugin._claim_pod([4, 5])
        assert claimed["metadata"]["name"] == "b-legacy-new"
        assert PodAssignment.from_annotations(obj_annotations(c.api.get_pod("default", "a-legacy-running"))) is None
