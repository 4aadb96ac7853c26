"""Least-privilege deploy (reference ``design.md:76-86,223-246``, who writes
what): the device plugin and the extender run as separate ServiceAccounts, the plugin confined to its
own node, the extender's ledger in Leases of its namespace and no write access to Nodes.  The rules
are read from the rendered manifests (``deploy/gpu-topology.yaml``) and enforced on the fake apiserver
(k8s/rbac.py) while the whole flow runs."""
import threading
import time

import pytest
import yaml

from gpu_topology_on_k8s_amd.config import EXTENDER_SA, NAMESPACE, PLUGIN_SA, render_manifests
from gpu_topology_on_k8s_amd.extender import ExtenderConfig, TopologyExtender
from gpu_topology_on_k8s_amd.k8s import Contract, FakeAPIServer, PodAssignment
from gpu_topology_on_k8s_amd.k8s.annotations import encode_node_annotations
from gpu_topology_on_k8s_amd.k8s.api import ApiError
from gpu_topology_on_k8s_amd.k8s.objects import annotations as obj_annotations
from gpu_topology_on_k8s_amd.k8s.objects import make_node, make_pod
from gpu_topology_on_k8s_amd.k8s.rbac import RBACView, identities_from_manifests, sa_username
from gpu_topology_on_k8s_amd.sim import SimCluster
from gpu_topology_on_k8s_amd.topology import fixtures as fx

PLUGIN = sa_username(NAMESPACE, PLUGIN_SA)
EXT = sa_username(NAMESPACE, EXTENDER_SA)


def _ids():
    return identities_from_manifests(yaml.safe_load_all(render_manifests()))


def test_each_service_account_holds_exactly_its_verbs():
    ids = _ids()
    assert set(ids) == {PLUGIN, EXT}  # the old shared "gpu-topology" account is gone
    assert ids[PLUGIN].grants() == {
        (None, "", "nodes"): {"get", "patch"},
        (None, "", "pods"): {"get", "list", "watch", "patch"},
        (None, "", "events"): {"create", "patch"},
    }
    assert ids[EXT].grants() == {
        (None, "", "nodes"): {"get", "list", "watch"},
        (None, "", "pods"): {"get", "list", "watch", "patch"},
        (None, "", "pods/binding"): {"create"},
        (None, "", "events"): {"create", "patch"},
        (NAMESPACE, "coordination.k8s.io", "leases"): {"get", "list", "watch", "create", "patch"},
    }
    assert ids[PLUGIN].own_node_only and not ids[EXT].own_node_only
    docs = list(yaml.safe_load_all(render_manifests()))
    sas = {d["metadata"]["name"]: d["spec"]["template"]["spec"]["serviceAccountName"] for d in docs if d["kind"] == "DaemonSet"}
    assert sas == {"amd-gpu-topology-device-plugin": PLUGIN_SA, "gpu-topology-scheduler-extender": EXTENDER_SA}
    vap = next(d for d in docs if d["kind"] == "ValidatingAdmissionPolicy")
    assert PLUGIN in vap["spec"]["matchConditions"][0]["expression"]
    assert any("authentication.kubernetes.io/node-name" in v["expression"] for v in vap["spec"]["validations"])
    binding = next(d for d in docs if d["kind"] == "ValidatingAdmissionPolicyBinding")
    assert binding["spec"] == {"policyName": vap["metadata"]["name"], "validationActions": ["Deny"]}


def test_the_committed_manifest_holds_the_same_identities():
    from pathlib import Path

    text = (Path(__file__).resolve().parent.parent / "deploy" / "gpu-topology.yaml").read_text()
    got = identities_from_manifests(yaml.safe_load_all(text))
    assert {k: v.grants() for k, v in got.items()} == {k: v.grants() for k, v in _ids().items()}


def _api_with_node(*names):
    api = FakeAPIServer()
    c = Contract()
    for n in names:
        api.create_node(make_node(n, annotations=encode_node_annotations(fx.f7_mi355x(), c), capacity={c.resource_name: "8"}))
    return api


def test_the_plugin_identity_cannot_bind_or_touch_another_node():
    api = _api_with_node("a", "b")
    ids = _ids()
    plugin = RBACView(api, ids[PLUGIN], node_name="a")
    plugin.patch_node("a", annotations={"x": "1"})  # its own node: fine
    for call in (lambda: plugin.patch_node("b", annotations={"x": "1"}),
                 lambda: plugin.bind_pod("default", "p", "", "a"),
                 lambda: plugin.list_nodes(),
                 lambda: plugin.create_lease(NAMESPACE, {"metadata": {"name": "gpu-ledger.a"}})):
        with pytest.raises(ApiError) as ei:
            call()
        assert ei.value.code == 403
    api.create_pod(make_pod("on-b", gpus=1, node="b"))
    api.create_pod(make_pod("on-a", gpus=1, node="a"))
    with pytest.raises(ApiError):
        plugin.patch_pod_annotations("default", "on-b", {"ALIYUN_COM_GPU_ASSIGNED": "true"})
    plugin.patch_pod_annotations("default", "on-a", {"ALIYUN_COM_GPU_ASSIGNED": "true"})
    assert any("own node" in d for d in plugin.denied)


def test_the_extender_identity_cannot_write_nodes_or_other_namespaces():
    api = _api_with_node("a")
    ext = RBACView(api, _ids()[EXT])
    with pytest.raises(ApiError) as ei:
        ext.patch_node("a", annotations={"x": "1"})
    assert ei.value.code == 403 and "cannot patch resource \"nodes\"" in ei.value.message
    with pytest.raises(ApiError):
        ext.create_lease("default", {"metadata": {"name": "gpu-ledger.a"}})
    ext.create_lease(NAMESPACE, {"metadata": {"name": "gpu-ledger.a"}})


def test_two_extenders_under_their_rbac_never_share_a_device():
    """The ledger race of tests/test_extender_ledger.py with both instances running as the deploy
    ServiceAccount: the Lease ledger works with no Node write access, and the round-5 Node store is
    refused with the fix named."""
    api = _api_with_node("n1")
    for i in range(2):
        api.create_pod(make_pod(f"p{i}", gpus=1))
    ident = _ids()[EXT]
    exts = [TopologyExtender(RBACView(api, ident), ExtenderConfig(resync_s=0.0, events=False)) for _ in range(2)]
    gate = threading.Barrier(2, timeout=10)
    for e in exts:
        real = e.cache.refresh_node
        first = [True]

        def refresh(name, _real=real, _first=first):
            st = _real(name)
            if _first[0]:
                _first[0] = False
                gate.wait()
            return st

        e.cache.refresh_node = refresh
    out = {}

    def go(i):
        pod = api.get_pod("default", f"p{i}")
        out[i] = exts[i].bind("default", f"p{i}", pod["metadata"]["uid"], "n1").ids

    ts = [threading.Thread(target=go, args=(i,)) for i in (0, 1)]
    [t.start() for t in ts]
    [t.join(timeout=30) for t in ts]
    assert not set(out[0]) & set(out[1]), out
    assert exts[0].metrics.ledger_conflicts + exts[1].metrics.ledger_conflicts >= 1
    old = TopologyExtender(RBACView(api, ident), ExtenderConfig(resync_s=0.0, events=False, ledger_store="node"))
    api.create_pod(make_pod("p2", gpus=1))
    with pytest.raises(ApiError) as ei:
        old.bind("default", "p2", api.get_pod("default", "p2")["metadata"]["uid"], "n1")
    assert ei.value.code == 403 and "`patch` on nodes" in str(ei.value)


@pytest.mark.parametrize("informer", [False, True])
def test_the_whole_flow_runs_under_the_deploy_rbac(informer):
    """Topology publication, filter / sort / bind with the Lease ledger, per-container Allocate with the
    ASSIGNED flip, the reconcile pass and Events — all as the deploy ServiceAccounts: nothing is refused."""
    with SimCluster({"n0": fx.f7_mi355x(), "n1": fx.f7_mi355x()}, rbac=True, informer=informer) as c:
        c.submit("a", 4)
        c.submit("b", 0, split=[2, 2])
        c.submit("c", 0, split=[2], init=[3])
        rs = c.schedule_pending()
        assert all(r.allocated for r in rs), rs
        assert c.reconcile() == 0
        for r in rs:
            pa = PodAssignment.from_annotations(obj_annotations(c.api.get_pod("default", r.pod.split("/")[1])))
            assert pa.assigned and sorted(pa.group) == sorted(r.allocated)
        c.complete("a")
        c.complete("b")  # c holds devices on one node only: the other one is empty again
        deadline = time.time() + 10  # the informer's watch delivers the completions
        while time.time() < deadline and all(c.extender.cache.get(n, sync=False).used(time.time(), 300) for n in ("n0", "n1")):
            time.sleep(0.05)
        c.submit("d", 8)
        (rd,) = c.schedule_pending()
        assert rd.node and len(rd.allocated) == 8
        leases = [k for k in c.api.leases if k[0] == NAMESPACE]
        assert leases  # the ledger lives in Leases
        assert not any(Contract().ledger_key in obj_annotations(c.api.get_node(n)) for n in ("n0", "n1"))
        assert c.denied == []
