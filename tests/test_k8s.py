"""Cluster-state contract, fake apiserver semantics, REST client on the wire."""
import json

import pytest

from gpu_topology_on_k8s_amd.k8s import (
    ANN_ASSIGNED, ANN_ASSUME_TIME, ANN_GROUP, ApiError, Conflict, Contract, FakeAPIServer, NotFound, PodAssignment,
    RestKubeAPI, serve_http,
)
from gpu_topology_on_k8s_amd.k8s.annotations import (
    decode_node_annotations, encode_node_annotations, format_group, pair_annotations, parse_group, parse_pair_annotations,
)
from gpu_topology_on_k8s_amd.k8s.objects import make_node, make_pod, parse_quantity, pod_gpu_request
from gpu_topology_on_k8s_amd.topology import fixtures as fx


# ------------------------------------------------------------------ annotations
def test_pair_annotation_keys_amd():
    t = fx.f7_mi355x()
    ann = pair_annotations(t)
    assert len(ann) == 28  # C(8,2)
    assert ann["GPU_XGMI_0_1"] == "xGMI 1 hop"
    assert "GPU_XGMI_0_0" not in ann  # no diagonal (design.md:17-19)


def test_pair_annotation_keys_reference_taxonomy():
    """design.md:78-82 shape: GPU_<ABBR>_<i>_<j>: <description>."""
    t = fx.f1_nvlink_host()
    ann = pair_annotations(t)
    assert ann["GPU_NV3_0_1"] == "Three NVLink links"
    assert ann["GPU_PHB_0_2"] == "Host PCI bridge"
    assert parse_pair_annotations({"GPU_SYS_0_1": "Cross CPU socket", "foo": "x"}) == {(0, 1): "SYS"}


def test_single_gpu_node_publishes_no_pairs():
    t = fx.f7_mi355x(n=1)
    assert pair_annotations(t) == {}


def test_node_annotation_roundtrip():
    t = fx.f7_mi355x(link_gbps=70.0, noise=0.05, seed=1)
    t.probe = {"method": "p2p_read_lds", "ts": 1700000000}
    c = Contract()
    ann = encode_node_annotations(t, c)
    assert ann[c.probe_time_key] == "1700000000"
    json.loads(ann[c.topology_key])
    u = decode_node_annotations(ann, c, node_name="n7")
    assert u.node_name == "n7"
    assert (u.cost == t.cost).all()


def test_decode_from_pairs_only():
    """A node annotated by a reference-style plugin (pairs only) still yields a usable model."""
    t = fx.f1_nvlink_host()
    u = decode_node_annotations(pair_annotations(t))
    assert u.n == 8
    assert u.cost[0, 1] < u.cost[0, 2]
    assert decode_node_annotations({}) is None
    amd = decode_node_annotations({"GPU_XGMI_0_1": "xGMI 1 hop"})
    assert amd.n == 2


def test_pod_assignment_codec():
    pa = PodAssignment.assumed([0, 1, 2, 3], now=1561717704)
    ann = pa.to_annotations()
    assert ann == {ANN_GROUP: "0,1,2,3", ANN_ASSIGNED: "false", ANN_ASSUME_TIME: "1561717704"}  # design.md:225-232
    back = PodAssignment.from_annotations(ann)
    assert back.group == [0, 1, 2, 3] and not back.assigned and back.assume_time == 1561717704
    alias = PodAssignment.from_annotations({"gpu-id": "0,2"})  # diagram alias, read-only
    assert alias.group == [0, 2]
    assert PodAssignment.from_annotations({}) is None
    assert parse_group("") == [] and parse_group(None) is None and format_group([3, 1]) == "3,1"


def test_pod_gpu_request():
    p = make_pod("a", gpus=4)
    assert pod_gpu_request(p, ["amd.com/gpu"]) == 4
    p2 = make_pod("b", gpus=2, resource="aliyun.com/gpu-count")
    assert pod_gpu_request(p2, ["amd.com/gpu", "aliyun.com/gpu-count"]) == 2
    p2["spec"]["initContainers"] = [{"name": "i", "resources": {"limits": {"amd.com/gpu": "3"}}}]
    assert pod_gpu_request(p2, ["amd.com/gpu", "aliyun.com/gpu-count"]) == 3
    with pytest.raises(ValueError):
        parse_quantity("0.5")


# ------------------------------------------------------------------ fake apiserver
def test_fake_apiserver_semantics():
    api = FakeAPIServer()
    api.create_node(make_node("n1"))
    api.create_pod(make_pod("p", gpus=1))
    with pytest.raises(Conflict):
        api.create_pod(make_pod("p"))
    pod = api.get_pod("default", "p")
    rv = pod["metadata"]["resourceVersion"]
    api.patch_pod_annotations("default", "p", {"a": "1"}, resource_version=rv)
    with pytest.raises(Conflict):
        api.patch_pod_annotations("default", "p", {"a": "2"}, resource_version=rv)  # stale
    api.patch_pod_annotations("default", "p", {"a": None})
    assert "a" not in api.get_pod("default", "p")["metadata"]["annotations"]
    api.bind_pod("default", "p", pod["metadata"]["uid"], "n1")
    assert api.list_pods(node_name="n1")[0]["spec"]["nodeName"] == "n1"
    with pytest.raises(Conflict):
        api.bind_pod("default", "p", "", "n1")  # already bound
    with pytest.raises(NotFound):
        api.get_pod("default", "nope")
    api.inject("bind_pod", 500, times=2)
    api.create_pod(make_pod("q"))
    for _ in range(2):
        with pytest.raises(ApiError) as ei:
            api.bind_pod("default", "q", "", "n1")
        assert ei.value.code == 500
    api.bind_pod("default", "q", "", "n1")
    events = []
    api.watch(lambda e, k, o: events.append((e, k, o["metadata"]["name"])))
    api.delete_pod("default", "q")
    assert events == [("DELETED", "Pod", "q")]


def test_label_selector():
    api = FakeAPIServer()
    api.create_node(make_node("a", labels={"gpu": "mi355x", "zone": "z1"}))
    api.create_node(make_node("b", labels={"gpu": "other"}))
    assert [n["metadata"]["name"] for n in api.list_nodes("gpu=mi355x")] == ["a"]
    assert [n["metadata"]["name"] for n in api.list_nodes("gpu!=mi355x")] == ["b"]
    assert [n["metadata"]["name"] for n in api.list_nodes("zone")] == ["a"]


# ------------------------------------------------------------------ REST client over HTTP
def test_rest_client_against_fake_over_http():
    api = FakeAPIServer()
    srv, url = serve_http(api, token="s3cret")
    try:
        rest = RestKubeAPI(url, token="s3cret")
        api.create_node(make_node("n1", labels={"x": "y"}))
        api.create_pod(make_pod("p", gpus=2, namespace="ml"))
        assert rest.get_node("n1")["metadata"]["labels"] == {"x": "y"}
        assert [n["metadata"]["name"] for n in rest.list_nodes("x=y")] == ["n1"]
        rest.patch_node("n1", annotations={"GPU_XGMI_0_1": "xGMI 1 hop"}, labels={"x": None})
        n = api.get_node("n1")
        assert n["metadata"]["annotations"]["GPU_XGMI_0_1"] == "xGMI 1 hop" and "x" not in n["metadata"]["labels"]
        pod = rest.get_pod("ml", "p")
        rest.patch_pod_annotations("ml", "p", {ANN_GROUP: "0,1"}, resource_version=pod["metadata"]["resourceVersion"])
        with pytest.raises(Conflict):
            rest.patch_pod_annotations("ml", "p", {ANN_GROUP: "2,3"}, resource_version=pod["metadata"]["resourceVersion"])
        rest.bind_pod("ml", "p", pod["metadata"]["uid"], "n1")
        assert [p["metadata"]["name"] for p in rest.list_pods(node_name="n1")] == ["p"]
        assert rest.list_pods(node_name="n2") == []
        assert len(rest.list_pods(namespace="ml")) == 1
        with pytest.raises(NotFound):
            rest.get_pod("ml", "zzz")
        bad = RestKubeAPI(url, token="wrong")
        with pytest.raises(ApiError) as ei:
            bad.get_node("n1")
        assert ei.value.code == 401
    finally:
        srv.shutdown()


def test_in_cluster_requires_env(monkeypatch):
    monkeypatch.delenv("KUBERNETES_SERVICE_HOST", raising=False)
    with pytest.raises(RuntimeError):
        RestKubeAPI.in_cluster()


def test_rest_client_rereads_a_rotated_token(tmp_path):
    """Projected service-account tokens rotate: after a 401 the client re-reads its token file once
    and retries (and re-reads it anyway once it is older than TOKEN_REFRESH_S)."""
    api = FakeAPIServer()
    api.create_node(make_node("n1"))
    srv, url = serve_http(api, token="new-token")
    try:
        tf = tmp_path / "token"
        tf.write_text("old-token\n")
        rest = RestKubeAPI(url, token="old-token", token_file=str(tf))
        tf.write_text("new-token\n")  # the kubelet rotated it
        assert rest.get_node("n1")["metadata"]["name"] == "n1"
        assert rest._token == "new-token"
        static = RestKubeAPI(url, token="old-token")  # no file: nothing to re-read, the 401 stands
        with pytest.raises(ApiError) as ei:
            static.get_node("n1")
        assert ei.value.code == 401
    finally:
        srv.shutdown()


def test_pod_assignment_parsing_edge_cases():
    """GROUP must name device indices: a negative one makes the annotation no assignment at all (the pod
    then counts by its resource request); ASSIGNED is read case-insensitively, as Go's strconv.ParseBool
    accepts "True" and "TRUE" from the reference's writers."""
    from gpu_topology_on_k8s_amd.k8s.annotations import ANN_ASSIGNED, ANN_ASSUME_TIME, ANN_GROUP, PodAssignment

    assert PodAssignment.from_annotations({ANN_GROUP: "-1"}) is None
    assert PodAssignment.from_annotations({ANN_GROUP: "0,-2"}) is None
    for v in ("true", "True", "TRUE"):
        pa = PodAssignment.from_annotations({ANN_GROUP: "1,3", ANN_ASSIGNED: v, ANN_ASSUME_TIME: "1561717704"})
        assert pa.assigned and pa.group == [1, 3] and pa.assume_time == 1561717704
    assert not PodAssignment.from_annotations({ANN_GROUP: "1", ANN_ASSIGNED: "false"}).assigned
