"""The extender's HTTP verbs under malformed and adversarial payloads (hypothesis).

kube-scheduler sends well-formed JSON, but the extender also sees pods written by users, with any
annotation value, resource quantity or container layout.  The extender is ``ignorable: false``, so
a 500 or a hung handler blocks every GPU pod.  Whatever arrives, every verb must answer with its
wire type: a HostPriorityList, an ExtenderFilterResult, an ExtenderBindingResult or
ExtenderPreemptionResult, with an ``Error`` string when it cannot act, or a 400 for a body that is
not JSON at all.  Binds that do go through must never hand out a device twice.
"""
import asyncio
import json
import logging
import os

from aiohttp.test_utils import TestClient, TestServer
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from gpu_topology_on_k8s_amd.extender import ExtenderConfig, TopologyExtender
from gpu_topology_on_k8s_amd.extender.server import make_app
from gpu_topology_on_k8s_amd.k8s import Contract, FakeAPIServer, PodAssignment
from gpu_topology_on_k8s_amd.k8s.annotations import encode_node_annotations
from gpu_topology_on_k8s_amd.k8s.objects import make_node, make_pod
from gpu_topology_on_k8s_amd.topology import fixtures as fx
from gpu_topology_on_k8s_amd.topology.shares import time_slice

C = Contract()
PREFIX = "/gputopology-scheduler"

# values a user can put on a pod: plausible, boundary and garbage
_values = st.one_of(st.sampled_from(["", "0", "1", "-1", "0.5", "1.5", "nan", "inf", "1e9", "abc", "96Gi", "0.0001", "8",
                                     "3,4", " 2 ", "true", "Gi"]),
                    st.text(max_size=12))
_quantity = st.one_of(st.sampled_from(["0", "1", "2", "4", "8", "9", "64", "-2", "1.5", "x", "", "100000000000"]),
                      st.integers(-3, 100).map(str))
_json_scalar = st.one_of(st.none(), st.booleans(), st.integers(-5, 5), st.text(max_size=8))


def _pod(name, limits, annotations, extra_containers):
    containers = [{"name": "c", "resources": {"limits": limits}}] + extra_containers
    return {"metadata": {"name": name, "namespace": "default", "uid": f"uid-{name}", "annotations": annotations},
            "spec": {"containers": containers}}


pods = st.builds(
    _pod,
    name=st.sampled_from(["p0", "p1", "p2", "ghost"]),
    limits=st.dictionaries(st.sampled_from([C.resource_name, C.slice_resource, "aliyun.com/gpu", "cpu"]), _quantity, max_size=3),
    annotations=st.dictionaries(st.sampled_from([C.fraction_key, C.memory_key, C.numa_pref_key, C.multi_node_key,
                                                 "ALIYUN_COM_GPU_GROUP", "ALIYUN_COM_GPU_ASSIGNED"]), _values, max_size=4),
    extra_containers=st.lists(st.one_of(_json_scalar, st.fixed_dictionaries({"resources": st.one_of(_json_scalar, st.fixed_dictionaries(
        {"limits": st.one_of(_json_scalar, st.dictionaries(st.just(C.resource_name), _quantity, max_size=1))}))})), max_size=2),
)
node_names = st.lists(st.sampled_from(["n1", "s1", "missing", ""]), max_size=4)
bodies = st.one_of(
    st.fixed_dictionaries({"Pod": st.one_of(pods, _json_scalar), "NodeNames": st.one_of(node_names, _json_scalar)}),
    st.fixed_dictionaries({"pod": pods, "nodenames": node_names}),
    st.fixed_dictionaries({"Pod": pods, "Nodes": st.one_of(_json_scalar, st.fixed_dictionaries({"items": st.lists(
        st.one_of(_json_scalar, st.fixed_dictionaries({"metadata": st.fixed_dictionaries({"name": st.sampled_from(["n1", "s1", "zz"])})})),
        max_size=3)}))}),
    st.dictionaries(st.sampled_from(["Pod", "NodeNames", "Nodes", "PodName"]), _json_scalar, max_size=3),
    st.lists(_json_scalar, max_size=3),
    _json_scalar,
)
binds = st.fixed_dictionaries({"PodName": st.one_of(st.sampled_from(["p0", "p1", "p2", "ghost"]), _json_scalar),
                               "PodNamespace": st.sampled_from(["default", "other", ""]),
                               "PodUID": st.one_of(st.sampled_from(["uid-p0", "uid-p1", "uid-p2", "wrong"]), _json_scalar),
                               "Node": st.one_of(st.sampled_from(["n1", "s1", "missing"]), _json_scalar)})


def _cluster():
    api = FakeAPIServer()
    t = fx.f7_mi355x()
    api.create_node(make_node("n1", annotations=encode_node_annotations(t, C), capacity={C.resource_name: "8"}))
    s = time_slice(fx.f7_mi355x(n=2), 4)
    api.create_node(make_node("s1", annotations=encode_node_annotations(s, C), capacity={C.slice_resource: "8"}))
    api.create_pod(make_pod("held", gpus=2, node="n1", annotations=PodAssignment([0, 1], True, 1).to_annotations()))
    for n, k in (("p0", 1), ("p1", 4), ("p2", 2)):
        api.create_pod(make_pod(n, gpus=k))
    return api, TopologyExtender(api, ExtenderConfig(resync_s=0.0, events=False))


def _check_shape(verb, status, body):
    assert status in (200, 400), (verb, status, body)
    if status == 400:
        return
    if verb in ("sort", "prioritize"):
        assert isinstance(body, list) and all(set(h) >= {"Host", "Score"} and 0 <= h["Score"] <= 10 for h in body)
    elif verb == "filter":
        assert isinstance(body, dict) and isinstance(body.get("Error", ""), str)
    elif verb == "bind":
        assert isinstance(body, dict) and isinstance(body.get("Error"), str)
    elif verb == "preempt":
        assert isinstance(body, dict)


@settings(max_examples=int(os.environ.get("GTK_FUZZ_EXAMPLES", "150")), deadline=None, suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
@given(calls=st.lists(st.one_of(st.tuples(st.sampled_from(["sort", "prioritize", "filter", "preempt"]), bodies),
                                st.tuples(st.just("bind"), binds),
                                st.tuples(st.just("raw"), st.binary(max_size=40))), min_size=1, max_size=8))
def test_every_verb_answers_in_its_wire_type(calls):
    api, ext = _cluster()
    crashes = []

    class Catch(logging.Handler):  # a verb that fell into its exception path logs at ERROR
        def emit(self, record):
            crashes.append(record.getMessage() + (f": {record.exc_info[1]!r}" if record.exc_info else ""))

    handler = Catch(level=logging.ERROR)
    logging.getLogger("gpu_topology_on_k8s_amd.extender.server").addHandler(handler)

    async def main():
        async with TestClient(TestServer(make_app(ext))) as client:
            for verb, body in calls:
                if verb == "raw":
                    r = await client.post(f"{PREFIX}/sort", data=body)
                    assert r.status in (200, 400)
                    continue
                r = await client.post(f"{PREFIX}/{verb}", data=json.dumps(body))
                text = await r.text()
                _check_shape(verb, r.status, json.loads(text) if r.status == 200 else None)

    try:
        asyncio.run(main())
    finally:
        logging.getLogger("gpu_topology_on_k8s_amd.extender.server").removeHandler(handler)
    assert not crashes, crashes  # malformed input is answered, never an exception inside a verb
    # the invariant the verbs protect: no device of a node is held twice
    for node in ("n1", "s1"):
        seen = set()
        for pod in api.list_pods():
            if (pod.get("spec") or {}).get("nodeName") != node:
                continue
            grp = ((pod.get("metadata") or {}).get("annotations") or {}).get("ALIYUN_COM_GPU_GROUP")
            if not grp:
                continue
            ids = {int(x) for x in grp.split(",") if x.strip().lstrip("-").isdigit()}
            assert not (ids & seen), (node, ids, seen)
            seen |= ids
