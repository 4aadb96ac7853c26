"""The extender's informer at scale, client-go style (reference
``design.md:234`` usage tracking, SURVEY §3.2 hot loop): paginated watch-cache LISTs, server-side
filtering of terminal pods, objects trimmed to what the cache reads, watches resumed from the last
resourceVersion after a transient error (relist only on 410 Gone), exponential back-off with jitter."""
import time

import pytest

from gpu_topology_on_k8s_amd.extender import ExtenderConfig, TopologyExtender
from gpu_topology_on_k8s_amd.k8s import Contract, FakeAPIServer, PodAssignment, serve_http
from gpu_topology_on_k8s_amd.k8s.annotations import encode_node_annotations
from gpu_topology_on_k8s_amd.k8s.api import ApiError, Gone, RestKubeAPI
from gpu_topology_on_k8s_amd.k8s.informer import Informer
from gpu_topology_on_k8s_amd.k8s.objects import LIVE_POD_SELECTOR, make_node, make_pod, match_fields, trim_node, trim_pod
from gpu_topology_on_k8s_amd.topology import fixtures as fx

C = Contract()


def meta_name(o):
    return o["metadata"]["name"]


def _wait(pred, timeout=10.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if pred():
            return True
        time.sleep(0.02)
    return False


def _bulky(pod):
    """What real pod objects carry besides what the extender reads."""
    pod["metadata"]["managedFields"] = [{"manager": "kubectl", "fieldsV1": {"f:spec": {"x" * 40: {}}}}] * 4
    pod["metadata"]["annotations"]["kubectl.kubernetes.io/last-applied-configuration"] = "{" + "y" * 800 + "}"
    c = pod["spec"]["containers"][0]
    c["env"] = [{"name": f"VAR{i}", "value": "v" * 30} for i in range(20)]
    c["volumeMounts"] = [{"name": f"vol{i}", "mountPath": f"/mnt/{i}"} for i in range(5)]
    pod["status"]["conditions"] = [{"type": t, "status": "True", "lastTransitionTime": "2026-01-01T00:00:00Z"}
                                   for t in ("PodScheduled", "Initialized", "ContainersReady", "Ready")]
    return pod


def _cluster(n_nodes=6, pods_per_node=5, terminal_every=3):
    api = FakeAPIServer()
    topo = fx.f7_mi355x()
    for i in range(n_nodes):
        api.create_node(make_node(f"n{i}", annotations=encode_node_annotations(topo, C), capacity={C.resource_name: "8"}))
    k = 0
    for i in range(n_nodes):
        for j in range(pods_per_node):
            pod = make_pod(f"p{k}", gpus=1, node=f"n{i}", annotations=PodAssignment([j], True, 100).to_annotations())
            pod["status"]["phase"] = "Succeeded" if k % terminal_every == 0 else "Running"
            api.create_pod(_bulky(pod))
            k += 1
    return api


def test_fake_apiserver_enforces_limit_and_continue():
    api = _cluster()
    items, rv, cont = api.list_page("Pod", limit=7)
    assert len(items) == 7 and cont
    seen = [p["metadata"]["name"] for p in items]
    while cont:
        page, rv2, nxt = api.list_page("Pod", limit=7, continue_token=cont)
        assert rv2 == rv  # every page is the same snapshot
        seen += [p["metadata"]["name"] for p in page]
        with pytest.raises(Gone):  # a continue token is single use
            api.list_page("Pod", limit=7, continue_token=cont)
        cont = nxt
    assert sorted(seen) == sorted(f"p{k}" for k in range(30))
    _, _, cont = api.list_page("Pod", limit=7)
    api.expire_continue_tokens()
    with pytest.raises(Gone):
        api.list_page("Pod", limit=7, continue_token=cont)
    assert api.bytes_served["Pod"] > 0 and api.list_requests["Pod"] >= 6


def test_watch_cache_list_ignores_limit_unless_it_pages():
    api = _cluster()
    items, _, cont = api.list_page("Pod", limit=5, resource_version="0")
    assert len(items) == 30 and cont == ""  # an older apiserver's watch cache answers in one piece
    api.watch_cache_pages = True
    items, _, cont = api.list_page("Pod", limit=5, resource_version="0")
    assert len(items) == 5 and cont


def test_field_selector_and_trim():
    api = _cluster()
    live, _, _ = api.list_page("Pod", field_selector=LIVE_POD_SELECTOR)
    assert len(live) == 20 and all(p["status"]["phase"] == "Running" for p in live)
    assert match_fields(live[0], "spec.nodeName=n0,status.phase==Running") or live[0]["spec"]["nodeName"] != "n0"
    t = trim_pod(live[0])
    assert "managedFields" not in t["metadata"] and "env" not in t["spec"]["containers"][0]
    assert set(t["metadata"]["annotations"]) == {"ALIYUN_COM_GPU_GROUP", "ALIYUN_COM_GPU_ASSIGNED", "ALIYUN_COM_GPU_ASSUME_TIME"}
    assert t["spec"]["containers"][0]["resources"] == live[0]["spec"]["containers"][0]["resources"]
    n = api.get_node("n0")
    n["status"]["images"] = [{"names": ["x" * 100], "sizeBytes": 1}] * 50
    tn = trim_node(n)
    assert "images" not in tn["status"] and tn["metadata"]["annotations"] == n["metadata"]["annotations"]
    assert tn["status"]["allocatable"] == {C.resource_name: "8"}


@pytest.mark.parametrize("wire", ["inproc", "rest"])
def test_informer_pages_filters_and_trims(wire):
    api = _cluster()
    api.watch_cache_pages = True
    srv = None
    client = api
    if wire == "rest":
        srv, url = serve_http(api)
        client = RestKubeAPI(url)
    ext = TopologyExtender(client, ExtenderConfig(resync_s=0.0))
    inf = ext.cache.make_informer(page_size=4, watch_timeout=2.0)
    try:
        inf.start()
        assert inf.wait_synced(10)
        assert inf.last_list["Pod"]["items"] == 20 and inf.last_list["Pod"]["pages"] == 5
        assert inf.last_list["Pod"]["consistent"] == 0.0  # served by the watch cache
        assert sorted(ext.cache.get("n0", sync=False).used(time.time(), 300)) == [1, 2, 4]  # p0 and p3 are terminal
        # a running pod finishes: the filtered watch delivers it as DELETED, its device is free again
        api.set_pod_phase("default", "p1", "Succeeded")
        assert _wait(lambda: 1 not in ext.cache.get("n0", sync=False).used(time.time(), 300))
        assert inf.relists() == 0
    finally:
        inf.stop()
        if srv is not None:
            srv.shutdown()


@pytest.mark.parametrize("wire", ["inproc", "rest"])
def test_watch_disconnects_resume_without_relisting(wire):
    """Injected watch failures — a connection reset mid-stream and a 503 at watch start — are resumed
    from the last resourceVersion: zero relists, and no event is lost."""
    api = _cluster(n_nodes=2, pods_per_node=2)
    srv = None
    client = api
    if wire == "rest":
        srv, url = serve_http(api)
        client = RestKubeAPI(url)
    ext = TopologyExtender(client, ExtenderConfig(resync_s=0.0))
    inf = ext.cache.make_informer(watch_timeout=2.0, backoff=0.02, max_backoff=0.1)
    try:
        inf.start()
        assert inf.wait_synced(10)
        api.cut_watch("Pod", after=1)  # the watch open now breaks after one more event ...
        api.inject("watch_Pod", 503, times=2)  # ... and the next two attempts are refused
        for i in range(4):
            api.create_pod(make_pod(f"new{i}", gpus=1, node="n1",
                                    annotations=PodAssignment([4 + i], True, 100).to_annotations()))
            time.sleep(0.05)
        assert _wait(lambda: {4, 5, 6, 7} <= ext.cache.get("n1", sync=False).used(time.time(), 300))
        assert inf.lists["Pod"] == 1, inf.lists  # zero relists
        assert inf.watch_errors["Pod"] >= 1 and inf.watch_resumes["Pod"] >= 1
    finally:
        inf.stop()
        if srv is not None:
            srv.shutdown()


def test_gone_relists_and_expired_continue_restarts_consistently():
    api = _cluster(n_nodes=2, pods_per_node=4, terminal_every=100)
    api.watch_cache_pages = True
    lists = []
    real = api.list_page
    first = {"done": False}

    def list_page(kind, limit=0, continue_token="", resource_version=None, field_selector=None, namespace=None):
        if kind == "Pod" and continue_token and not first["done"]:
            first["done"] = True
            api.expire_continue_tokens()  # compaction between page 1 and page 2
        lists.append((kind, bool(continue_token), resource_version))
        return real(kind, limit, continue_token, resource_version, field_selector, namespace)

    api.list_page = list_page
    got = {}
    inf = Informer(api, lambda k, items: got.__setitem__(k, len(items)), lambda t, k, o: None, page_size=3, watch_timeout=1.0,
                   backoff=0.02)
    try:
        inf.start()
        assert inf.wait_synced(10)
        assert got["Pod"] == 8 and inf.last_list["Pod"]["consistent"] == 1.0  # restarted as a quorum read
        assert ("Pod", False, None) in lists
        # a 410 on the watch (the version left the window) is the one thing that relists
        n = inf.lists["Pod"]
        orig = api.watch_stream

        def gone_once(kind, *a, **kw):
            if kind != "Pod":
                return orig(kind, *a, **kw)
            api.watch_stream = orig
            raise Gone("too old")

        api.watch_stream = gone_once
        assert _wait(lambda: inf.lists["Pod"] == n + 1, timeout=10)
    finally:
        inf.stop()


def test_backoff_is_exponential_capped_and_jittered():
    inf = Informer(FakeAPIServer(), lambda *a: None, lambda *a: None, backoff=0.5, max_backoff=8.0, jitter=0.2, seed=1)
    ds = [inf._delay(f) for f in range(1, 9)]
    for f, d in enumerate(ds, 1):
        base = min(8.0, 0.5 * 2 ** (f - 1))
        assert 0.8 * base <= d <= 1.2 * base
    assert len({round(d, 6) for d in ds[-3:]}) == 3  # capped but not in lock-step


def test_a_watch_cache_list_does_not_drop_a_bind_it_cannot_show():
    """A watch-cache LIST taken after a bind may not show the pod yet: unlike a quorum read, its
    absence must not free the bind's devices (extender/cache.py overlay)."""
    api = FakeAPIServer()
    api.create_node(make_node("n", annotations=encode_node_annotations(fx.f7_mi355x(), C), capacity={C.resource_name: "8"}))
    ext = TopologyExtender(api, ExtenderConfig(resync_s=0.0))
    cache = ext.cache
    cache.get("n")
    cache.assume("n", "default/x", [2, 3])
    cache.bound("n", "default/x")
    cache.on_list("Pod", [], cache.begin_list("Pod"), consistent=False)
    assert {2, 3} <= cache.get("n", sync=False).used(time.time(), 300)
    cache.on_list("Pod", [], cache.begin_list("Pod"), consistent=True)
    assert not {2, 3} & cache.get("n", sync=False).used(time.time(), 300)


def test_watch_events_are_transformed_and_a_delivered_event_resets_the_backoff():
    """Watch events go through the same trim as LIST items (a bulky pod never lands in the cache), and
    the back-off restarts from its base once a watch delivers again: a cluster that had a bad minute
    does not pay its longest delay on the next, unrelated disconnect."""
    api = _cluster(n_nodes=1, pods_per_node=1)
    got = []
    inf = Informer(api, lambda k, items: None, lambda t, k, o: got.append((t, o)), kinds=("Pod",),
                   transform=lambda k, o: trim_pod(o), watch_timeout=2.0, backoff=0.01, max_backoff=0.05)
    delays = []
    real = inf._delay
    inf._delay = lambda f: (delays.append(f), real(f))[1]
    api.inject("watch_Pod", 503, times=2)  # the first two watches are refused ...
    try:
        inf.start()
        assert inf.wait_synced(10)
        api.create_pod(_bulky(make_pod("late0", gpus=1, node="n0")))
        assert _wait(lambda: any(meta_name(o) == "late0" for _, o in got))
        api.cut_watch("Pod", after=0)  # ... then, after a delivered event, the open watch breaks
        api.create_pod(make_pod("late1", gpus=1, node="n0"))
        assert _wait(lambda: len(delays) >= 3)
        assert delays[:3] == [1, 2, 1], delays
        assert _wait(lambda: any(meta_name(o) == "late1" for _, o in got))  # resumed, not lost
        assert inf.relists() == 0
        o = next(o for _, o in got if meta_name(o) == "late0")
        assert "managedFields" not in o["metadata"] and "env" not in o["spec"]["containers"][0]
    finally:
        inf.stop()


def test_continue_pages_carry_no_resource_version():
    """The apiserver refuses a page request that names both a continue token and a resourceVersion;
    the informer sends the version on the first page only."""
    api = _cluster()
    api.watch_cache_pages = True
    _, _, cont = api.list_page("Pod", limit=4, resource_version="0")
    with pytest.raises(ApiError) as ei:
        api.list_page("Pod", limit=4, continue_token=cont, resource_version="0")
    assert ei.value.code == 400
    inf = Informer(api, lambda k, items: None, lambda *a: None, kinds=("Pod",), page_size=4, watch_timeout=1.0)
    items, _, consistent = inf._list("Pod")
    assert len(items) == 30 and not consistent and inf.pages["Pod"] == 8


def test_informer_health_is_on_the_extenders_metrics():
    """An operator sees a relist storm (or its absence) on /metrics: per-kind LISTs, pages, events,
    resumed and broken watches, and the size of the last LIST."""
    api = _cluster(n_nodes=2, pods_per_node=3)
    api.watch_cache_pages = True
    ext = TopologyExtender(api, ExtenderConfig(resync_s=0.0))
    assert b"gtk_extender_informer_lists" not in ext.metrics.exposition()  # polling: nothing to report
    inf = ext.cache.make_informer(page_size=2, watch_timeout=2.0, backoff=0.02, max_backoff=0.1)
    try:
        inf.start()
        assert inf.wait_synced(10)
        api.cut_watch("Pod", after=0)
        api.create_pod(make_pod("late", gpus=1, node="n0"))
        assert _wait(lambda: inf.watch_errors["Pod"] >= 1 and inf.events["Pod"] >= 1)
        text = ext.metrics.exposition().decode()
    finally:
        inf.stop()
    assert 'gtk_extender_informer_lists_total{kind="Pod"} 1.0' in text
    assert 'gtk_extender_informer_list_pages_total{kind="Pod"} 2.0' in text  # 4 live pods, 2 per page
    assert 'gtk_extender_informer_watch_errors_total{kind="Pod"} 1.0' in text
    assert 'gtk_extender_informer_last_list_items{kind="Pod"} 4.0' in text
    assert "gtk_extender_informer_synced 1.0" in text


def test_before_the_first_sync_nothing_relists_per_request():
    """An extender whose informer is still listing (a restart at 100,000 pods takes ~50 s) never
    falls back to a cluster-wide LIST per request: filter and sort decline GPU pods until it has
    synced (kube-scheduler retries them), /readyz answers 503, bind still works on its own refresh of
    the node, and once the informer has synced everything is served from it."""
    import requests

    from gpu_topology_on_k8s_amd.sim.cluster import HttpExtender

    api = _cluster(n_nodes=2, pods_per_node=1)
    ext = TopologyExtender(api, ExtenderConfig(resync_s=0.0))
    inf = ext.cache.make_informer(watch_timeout=2.0)  # attached, not started yet: still listing
    http = HttpExtender(ext)
    http.start()
    try:
        lists = api.calls.get("list_pods", 0) + api.calls.get("list_nodes", 0)
        pod = api.create_pod(make_pod("want", gpus=2))
        ok, failed = ext.filter(pod, ["n0", "n1"])
        assert ok == [] and set(failed.values()) == {ext.NOT_READY}
        assert ext.prioritize(pod, ["n0", "n1"]) == [("n0", 0), ("n1", 0)]
        assert ext.filter(make_pod("cpu", gpus=0), ["n0"])[0] == ["n0"]  # not ours: passes
        ext.preempt(pod, {"n0": ([], 0)})  # the verbs that read the cache without a gate
        ext.defrag(2)
        ext.cache.get("n1")
        assert api.calls.get("list_pods", 0) + api.calls.get("list_nodes", 0) == lists  # no cluster LIST
        assert requests.get(f"{http.url}/readyz", timeout=5).status_code == 503
        d = ext.bind("default", "want", pod["metadata"]["uid"], "n1")  # its own refresh of n1
        assert d is not None and len(d.ids) == 2
        inf.start()
        assert inf.wait_synced(10)
        assert requests.get(f"{http.url}/readyz", timeout=5).status_code == 200
        pod2 = api.create_pod(make_pod("want2", gpus=2))
        assert _wait(lambda: ext.filter(pod2, ["n0", "n1"])[0] == ["n0", "n1"])
        assert "not_ready" in ext.metrics.exposition().decode()
    finally:
        inf.stop()
        http.stop()
