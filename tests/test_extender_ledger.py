"""Bind safety across extender instances.

Each :class:`TopologyExtender` serialises select -> annotate -> bind per node with an in-process lock,
but the extender runs as several instances (a DaemonSet on the control-plane nodes; two leaders across
a scheduler failover).  Every bind therefore records its device set in the node's allocation ledger
(``<prefix>/gpu-ledger``) with the ledger object's resourceVersion as a precondition; a second instance
that decided on the same state gets 409, re-reads and re-decides.  Two instances share one
FakeAPIServer here, which enforces the precondition as the apiserver does; each has its own cache.
Every test runs with the ledger in a per-node coordination.k8s.io Lease (the default) and in the
round-5 Node annotation.
"""
import threading

import pytest

from gpu_topology_on_k8s_amd.extender import ExtenderConfig, TopologyExtender
from gpu_topology_on_k8s_amd.extender.ledger import lease_name
from gpu_topology_on_k8s_amd.k8s import Contract, FakeAPIServer
from gpu_topology_on_k8s_amd.k8s.annotations import encode_node_annotations, parse_ledger
from gpu_topology_on_k8s_amd.k8s.api import NotFound
from gpu_topology_on_k8s_amd.k8s.objects import annotations as obj_annotations
from gpu_topology_on_k8s_amd.k8s.objects import make_node, make_pod
from gpu_topology_on_k8s_amd.topology import fixtures as fx

STORE = {"store": "lease"}
NS = "kube-system"


@pytest.fixture(autouse=True, params=["lease", "node"])
def store(request):
    STORE["store"] = request.param
    yield request.param
    STORE["store"] = "lease"


def _cfg(**kw):
    return ExtenderConfig(resync_s=0.0, events=False, ledger_store=STORE["store"], ledger_namespace=NS, **kw)


def _ledger(api, node="n1"):
    """The node's ledger entries where the store in use keeps them."""
    if STORE["store"] == "node":
        return parse_ledger(obj_annotations(api.get_node(node)))
    try:
        return parse_ledger(obj_annotations(api.get_lease(NS, lease_name(node))))
    except NotFound:
        return {}


def _set_ledger(api, raw, node="n1"):
    """Another writer's ledger value, written where the store in use reads it."""
    c = Contract()
    if STORE["store"] == "node":
        api.patch_node(node, annotations={c.ledger_key: raw})
        return
    try:
        api.patch_lease(NS, lease_name(node), {c.ledger_key: raw})
    except NotFound:
        api.create_lease(NS, {"metadata": {"name": lease_name(node), "annotations": {c.ledger_key: raw}}})


class Clock:
    def __init__(self, t=1_700_000_000.0):
        self.t = t

    def __call__(self):
        return self.t


def _two(ledger=True, n_pods=0, k=1):
    api = FakeAPIServer()
    c = Contract()
    t = fx.f7_mi355x()
    api.create_node(make_node("n1", labels={c.label_model: "MI355X"}, annotations=encode_node_annotations(t, c),
                              capacity={c.resource_name: str(t.n)}))
    clock = Clock()
    exts = [TopologyExtender(api, _cfg(ledger=ledger), clock=clock) for _ in range(2)]
    for i in range(n_pods):
        api.create_pod(make_pod(f"p{i}", gpus=k))
    return api, exts, clock


def _bind(api, ext, name):
    pod = api.get_pod("default", name)
    return ext.bind("default", name, pod["metadata"]["uid"], "n1")


def _lockstep(exts):
    """Both instances read the node before either writes anything (the failover window, made certain):
    their first refresh before a bind waits for the other's."""
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


def _race(api, exts):
    out = {}

    def go(i):
        out[i] = _bind(api, exts[i], f"p{i}").ids

    ts = [threading.Thread(target=go, args=(i,)) for i in (0, 1)]
    [t.start() for t in ts]
    [t.join(timeout=30) for t in ts]
    return out


def test_without_the_ledger_two_instances_hand_out_the_same_device():
    """The hazard being fixed: two instances deciding on the same state pick the same best device."""
    api, exts, _ = _two(ledger=False, n_pods=2)
    _lockstep(exts)
    out = _race(api, exts)
    assert set(out[0]) & set(out[1])


def test_with_the_ledger_the_second_instance_redecides():
    api, exts, _ = _two(ledger=True, n_pods=2)
    _lockstep(exts)
    out = _race(api, exts)
    assert not set(out[0]) & set(out[1]), out
    assert exts[0].metrics.ledger_conflicts + exts[1].metrics.ledger_conflicts >= 1
    groups = [obj_annotations(api.get_pod("default", f"p{i}"))["ALIYUN_COM_GPU_GROUP"] for i in (0, 1)]
    assert groups[0] != groups[1]


def test_fifty_concurrent_pods_on_one_node_never_overlap():
    api, exts, _ = _two(ledger=True, n_pods=50)
    res = {}
    gate = threading.Barrier(50, timeout=30)

    def go(i):
        gate.wait()
        try:
            res[i] = _bind(api, exts[i % 2], f"p{i}").ids
        except Exception as e:  # noqa: BLE001 - no free device / ledger contention: kube-scheduler retries
            res[i] = e

    ts = [threading.Thread(target=go, args=(i,)) for i in range(50)]
    [t.start() for t in ts]
    [t.join(timeout=60) for t in ts]
    got = [r for r in res.values() if isinstance(r, tuple)]
    flat = [d for g in got for d in g]
    assert len(flat) == len(set(flat)) and len(flat) <= 8, got
    # the pods that lost retry, one at a time (what kube-scheduler does): the node fills exactly
    for i in sorted(res):
        if not isinstance(res[i], tuple) and len(flat) < 8:
            res[i] = _bind(api, exts[i % 2], f"p{i}").ids
            flat += list(res[i])
    assert sorted(flat) == list(range(8))
    ann = {i: obj_annotations(api.get_pod("default", f"p{i}")).get("ALIYUN_COM_GPU_GROUP") for i in range(50)}
    held = [int(x) for v in ann.values() if v for x in v.split(",")]
    assert sorted(held) == list(range(8))  # GROUP annotations: every device exactly once


def test_ledger_entries_settle_and_lapse():
    """An entry covers a bind in flight only: once a LIST shows the pod on the node its own annotation
    governs (the next ledger write drops the entry), and an entry whose pod never appears lapses after
    the grace period (a bind that failed after recording its devices)."""
    from gpu_topology_on_k8s_amd.extender.cache import LEDGER_CLOCK_SKEW_S, LEDGER_GRACE_S
    from gpu_topology_on_k8s_amd.k8s.annotations import dump_ledger

    api, exts, clock = _two(ledger=True, n_pods=3)
    d0 = _bind(api, exts[0], "p0")
    led = _ledger(api)
    assert set(led) == {"default/p0"} and led["default/p0"][0] == d0.ids
    d1 = _bind(api, exts[1], "p1")
    led = _ledger(api)
    assert set(led) == {"default/p1"}  # p0 settled (listed on the node): dropped
    assert not set(d0.ids) & set(d1.ids)
    # a lost bind: recorded, never annotated nor bound
    c = Contract()
    _set_ledger(api, dump_ledger({"default/ghost": ((7,), clock.t)}, 99))
    d2 = _bind(api, exts[0], "p2")
    assert 7 not in d2.ids
    api.delete_pod("default", "p2")
    clock.t += LEDGER_GRACE_S + LEDGER_CLOCK_SKEW_S + 1  # old by the writers' clocks too (exts[1] never saw them)
    api.create_pod(make_pod("p3", gpus=6))
    d3 = _bind(api, exts[1], "p3")
    assert 7 in d3.ids  # the ghost's device is free again


def test_failed_bind_releases_its_ledger_entry():
    api, exts, _ = _two(ledger=True, n_pods=1)
    api.inject("bind_pod", 500)
    try:
        _bind(api, exts[0], "p0")
    except Exception:  # noqa: BLE001 - the injected apiserver failure
        pass
    assert "default/p0" not in _ledger(api)


def test_malformed_or_foreign_ledger_values_do_not_break_binds():
    """A ledger another writer mangled (not JSON, wrong shapes, device ids off the node) reads as
    empty or is ignored where it names no device of the node; the next bind rewrites it."""
    from gpu_topology_on_k8s_amd.k8s.annotations import dump_ledger

    c = Contract()
    bad = ["not json", "[1, 2]", '{"a": {"x/y": {"g": "zz", "t": 1}}}', '{"a": [], "gen": "q"}',
           dump_ledger({"default/other": ((99, -3), 1_700_000_000.0)}, 5)]
    for i, raw in enumerate(bad):
        api, exts, _ = _two(ledger=True, n_pods=1, k=8)
        _set_ledger(api, raw)
        d = _bind(api, exts[0], "p0")
        assert sorted(d.ids) == list(range(8)), (raw, d)
        led = _ledger(api)
        assert led["default/p0"][0] == tuple(d.ids)


def test_ledger_without_its_rbac_verbs_fails_the_bind_with_the_fix_and_can_be_turned_off():
    """RBAC without the ledger's verbs (`create` on leases / `patch` on nodes): the ledger write is
    refused (403) and the bind fails with a message naming the missing verb and --bind-ledger off; with
    the ledger off the same bind succeeds (a single extender's node lock only)."""
    import pytest

    from gpu_topology_on_k8s_amd.extender.__main__ import main as extender_main  # noqa: F401 - the flag exists
    from gpu_topology_on_k8s_amd.k8s.api import ApiError

    api, exts, _ = _two(ledger=True, n_pods=2)
    api.inject("create_lease" if STORE["store"] == "lease" else "patch_node", 403, times=100)
    with pytest.raises(ApiError) as ei:
        _bind(api, exts[0], "p0")
    want = "leases" if STORE["store"] == "lease" else "`patch` on nodes"
    assert ei.value.code == 403 and "--bind-ledger off" in str(ei.value) and want in str(ei.value)
    off = TopologyExtender(api, _cfg(ledger=False))
    assert len(_bind(api, off, "p1").ids) == 1


@pytest.mark.parametrize("seed", [5, 7, 11])
def test_two_extenders_under_churn_never_share_a_device(seed):
    """Randomised churn across two extender instances on one apiserver: pods of 1-4 GPUs are bound
    concurrently through either instance (4 workers) while others complete; after every round the live
    pods' GROUP annotations on the node are disjoint, and every device a bind handed out is one no
    other live pod holds."""
    import random
    from concurrent.futures import ThreadPoolExecutor

    api, exts, clock = _two(ledger=True)
    rng = random.Random(seed)
    live, n, bound = {}, 0, 0
    lock = threading.Lock()

    def bind(name):
        try:
            ids = _bind(api, exts[rng.randrange(2)], name).ids
            # the container starts: Allocate flips ASSIGNED (an assumption never confirmed would expire
            # after the assume TTL by design, and this test's clock runs far past it)
            api.patch_pod_annotations("default", name, {"ALIYUN_COM_GPU_ASSIGNED": "true"})
            return name, ids
        except Exception:  # noqa: BLE001 - no room / ledger contention: kube-scheduler would retry later
            api.delete_pod("default", name)
            return name, None

    with ThreadPoolExecutor(4) as pool:
        for _ in range(40):
            names = []
            for _ in range(rng.randint(1, 4)):
                n += 1
                api.create_pod(make_pod(f"c{n}", gpus=rng.randint(1, 4)))
                names.append(f"c{n}")
            for name, ids in pool.map(bind, names):
                if ids is not None:
                    with lock:
                        live[name] = set(ids)
                        bound += 1
            held = [d for s in live.values() for d in s]
            assert len(held) == len(set(held)), live
            ann = [obj_annotations(api.get_pod("default", k)).get("ALIYUN_COM_GPU_GROUP") for k in live]
            flat = [int(x) for v in ann if v for x in v.split(",")]
            assert len(flat) == len(set(flat)), ann
            for k in rng.sample(sorted(live), k=min(len(live), rng.randint(0, 3))):  # some pods finish
                api.delete_pod("default", k)
                del live[k]
            clock.t += rng.choice([0.5, 2.0, 40.0])  # sometimes past the ledger grace
    assert n > 60 and bound > 30, (n, bound)


def test_a_newer_node_object_never_meets_an_older_pod_list():
    """The decision sees the node object and the pod LIST of one refresh.  Interleaving forced: B's bind
    has refreshed (no pod bound yet) when A binds p0 and then p1 -- A's second ledger write drops p0,
    which A's LIST showed bound -- and a concurrent refresh in B applies that newer node object.  Had B
    decided on it with its older LIST, p0's device would look free and the newer object's
    resourceVersion would pass the precondition; B's 7-GPU pod must not get p0's (or p1's) device."""
    from gpu_topology_on_k8s_amd.extender.scheduler import NoFeasiblePlacement

    api, exts, _ = _two(ledger=True, n_pods=2)
    api.create_pod(make_pod("big", gpus=7))
    a, b = exts
    refreshed, go = threading.Event(), threading.Event()
    real = b.cache.refresh_node
    first = [True]

    def paused_refresh(name):
        st = real(name)
        if first[0]:
            first[0] = False
            refreshed.set()
            assert go.wait(10)
        return st

    b.cache.refresh_node = paused_refresh
    out = {}

    def bind_big():
        try:
            out["big"] = _bind(api, b, "big").ids
        except NoFeasiblePlacement as e:
            out["big"] = e

    tb = threading.Thread(target=bind_big)
    tb.start()
    assert refreshed.wait(10)
    d0, d1 = _bind(api, a, "p0"), _bind(api, a, "p1")
    assert "default/p0" not in _ledger(api)  # settled, dropped by A
    def other_refresh():  # B's other refresh: the newer node object and ledger
        b.cache.update_node_object(api.get_node("n1"))
        if STORE["store"] == "lease":
            b.cache.update_lease_object("n1", api.get_lease(NS, lease_name("n1")))

    tc = threading.Thread(target=other_refresh)
    tc.start()
    tc.join(timeout=0.3)
    go.set()
    tb.join(timeout=30)
    tc.join(timeout=30)
    assert not tb.is_alive() and not tc.is_alive()
    taken = set(d0.ids) | set(d1.ids)
    assert isinstance(out["big"], NoFeasiblePlacement) or not set(out["big"]) & taken, (out, taken)


def test_an_instance_whose_clock_runs_ahead_still_honours_a_bind_in_flight():
    """The ledger entry's timestamp is the writer's clock.  An instance 90 s ahead (more than the grace)
    must still count a fresh entry: it ages entries from when it first saw them.  Once it has seen an
    entry for longer than the grace with no pod behind it, the entry lapses on its own clock."""
    from gpu_topology_on_k8s_amd.extender.cache import LEDGER_GRACE_S
    from gpu_topology_on_k8s_amd.k8s.annotations import dump_ledger

    api = FakeAPIServer()
    c = Contract()
    t = fx.f7_mi355x()
    api.create_node(make_node("n1", labels={c.label_model: "MI355X"}, annotations=encode_node_annotations(t, c),
                              capacity={c.resource_name: str(t.n)}))
    behind, ahead = Clock(1_700_000_000.0), Clock(1_700_000_090.0)
    a = TopologyExtender(api, _cfg(ledger=True), clock=behind)
    b = TopologyExtender(api, _cfg(ledger=True), clock=ahead)
    # A has recorded its decision (devices 0-3) but not yet annotated or bound the pod
    _set_ledger(api, dump_ledger({"default/inflight": ((0, 1, 2, 3), behind.t)}, 1))
    api.create_pod(make_pod("big", gpus=5))
    with pytest.raises(Exception):
        _bind(api, b, "big")  # only 4 devices are free: the in-flight entry holds 0-3
    api.create_pod(make_pod("four", gpus=4))
    assert not set(_bind(api, b, "four").ids) & {0, 1, 2, 3}
    b.cache.refresh_node("n1")  # a resync LISTs "four" on the node: its own annotation governs from now on
    ahead.t += LEDGER_GRACE_S + 1  # B has now seen the in-flight entry for longer than the grace: a lost bind
    api.delete_pod("default", "four")
    assert len(_bind(api, b, "big").ids) == 5


def test_a_reused_pod_name_in_flight_is_not_taken_for_its_settled_predecessor():
    """StatefulSet pods come back under the same name.  B has seen "db" bound (its ledger entry settled);
    db is deleted and re-created, and A records the new db's devices in the ledger but has not bound it
    yet.  B, deciding in that window, must count the new entry: the old pod's settlement does not carry
    over to a new incarnation that no LIST has shown."""
    from gpu_topology_on_k8s_amd.extender.scheduler import NoFeasiblePlacement

    api, exts, _ = _two(ledger=True)
    a, b = exts
    api.create_pod(make_pod("db", gpus=4))
    first = _bind(api, a, "db")
    b.cache.refresh_node("n1")  # B's LIST shows db on the node: settled in B's view
    api.delete_pod("default", "db")
    api.create_pod(make_pod("db", gpus=4))
    api.create_pod(make_pod("all", gpus=8))
    recorded, go = threading.Event(), threading.Event()
    real_commit = a._commit

    def paused_commit(*args, **kw):  # A: devices recorded in the ledger, pod not yet annotated or bound
        recorded.set()
        assert go.wait(10)
        return real_commit(*args, **kw)

    a._commit = paused_commit
    out = {}
    ta = threading.Thread(target=lambda: out.setdefault("db", _bind(api, a, "db")))
    ta.start()
    assert recorded.wait(10)
    try:
        out["all"] = _bind(api, b, "all").ids
    except NoFeasiblePlacement as e:
        out["all"] = e
    go.set()
    ta.join(timeout=30)
    assert not ta.is_alive()
    assert isinstance(out["all"], NoFeasiblePlacement), (out, first.ids)


def test_a_reused_pod_name_on_the_same_devices_is_a_new_entry():
    """As above, but long after the first incarnation and on the SAME devices: the new bind's entry has
    the old key and the old device set, and is still a new entry (new bind time) that ages from when B
    first sees it, not from when B saw the old one."""
    from gpu_topology_on_k8s_amd.extender.cache import LEDGER_GRACE_S
    from gpu_topology_on_k8s_amd.extender.scheduler import NoFeasiblePlacement

    api, exts, clock = _two(ledger=True)
    a, b = exts
    api.create_pod(make_pod("db", gpus=4))
    first = _bind(api, a, "db")
    a.cache.refresh_node("n1")
    b.cache.refresh_node("n1")  # both have seen db bound and its entry
    api.delete_pod("default", "db")
    clock.t += LEDGER_GRACE_S + 1
    api.create_pod(make_pod("db", gpus=4))
    api.create_pod(make_pod("all", gpus=8))
    recorded, go = threading.Event(), threading.Event()
    real_commit = a._commit
    chosen = {}

    def paused_commit(pod, namespace, name, uid, node, key, d, *rest):
        chosen["ids"] = d.ids
        recorded.set()
        assert go.wait(10)
        return real_commit(pod, namespace, name, uid, node, key, d, *rest)

    a._commit = paused_commit
    ta = threading.Thread(target=lambda: _bind(api, a, "db"))
    ta.start()
    assert recorded.wait(10)
    assert tuple(chosen["ids"]) == tuple(first.ids)  # the same devices again
    try:
        got = _bind(api, b, "all").ids
    except NoFeasiblePlacement as e:
        got = e
    go.set()
    ta.join(timeout=30)
    assert not ta.is_alive()
    assert isinstance(got, NoFeasiblePlacement), got


def test_an_ended_pod_s_entry_holds_nothing_once_its_pod_was_seen():
    """The watch shows the pod bound (its entry settles, whichever of the pod's and the ledger's events
    comes first); the pod then ends within the grace period: its devices are free at once, not after
    the entry lapses (found under the informer, where no LIST follows a bind)."""
    api, exts, clock = _two(ledger=True, n_pods=1, k=4)
    a, b = exts
    d = _bind(api, a, "p0")
    pod = api.get_pod("default", "p0")
    st = b.cache.get("n1")
    b.cache.on_event("MODIFIED", "Pod", pod)  # the pod's event first, the ledger's after
    b.cache.update_lease_object("n1", api.get_lease(NS, lease_name("n1"))) if STORE["store"] == "lease" else \
        b.cache.update_node_object(api.get_node("n1"))
    assert "default/p0" in st.ledger and "default/p0" in st.settled
    api.set_pod_phase("default", "p0", "Succeeded")
    b.cache.on_event("MODIFIED", "Pod", api.get_pod("default", "p0"))
    assert not set(d.ids) & st.used(clock.t, 300)  # within the grace, yet free


def test_a_mixed_fleet_during_the_ledger_migration_never_shares_a_device():
    """docs/MIGRATION.md: a round-5 extender (Node annotation) and an upgraded one in `both` mode bind
    on one node concurrently: each sees the other's binds in flight."""
    api = FakeAPIServer()
    c = Contract()
    t = fx.f7_mi355x()
    api.create_node(make_node("n1", labels={c.label_model: "MI355X"}, annotations=encode_node_annotations(t, c),
                              capacity={c.resource_name: str(t.n)}))
    old = TopologyExtender(api, ExtenderConfig(resync_s=0.0, events=False, ledger_store="node"))
    new = TopologyExtender(api, ExtenderConfig(resync_s=0.0, events=False, ledger_store="both", ledger_namespace=NS))
    for i in range(2):
        api.create_pod(make_pod(f"p{i}", gpus=1))
    _lockstep([old, new])
    out = _race(api, [old, new])
    assert not set(out[0]) & set(out[1]), out
    assert parse_ledger(obj_annotations(api.get_node("n1")))  # the old writer's view is kept current
    assert parse_ledger(obj_annotations(api.get_lease(NS, lease_name("n1"))))


def test_a_bind_too_slow_to_beat_its_ledger_grace_is_rolled_back(monkeypatch):
    """ADVICE r5 (cache.py:41): another extender stops counting a ledger entry LEDGER_GRACE_S after it
    first saw it, bound or not.  A bind whose pod annotation took longer than half that (a throttled
    apiserver) must not go on to bind: it is rolled back, its entry released, and kube-scheduler retries."""
    from gpu_topology_on_k8s_amd.extender import scheduler as sch
    from gpu_topology_on_k8s_amd.k8s.api import ApiError

    monkeypatch.setattr(sch, "LEDGER_GRACE_S", 0.2)
    api, exts, _ = _two(ledger=True, n_pods=1)
    real = exts[0]._patch_with_retry

    def slow(*a, **kw):
        import time as _t

        _t.sleep(0.15)
        return real(*a, **kw)

    exts[0]._patch_with_retry = slow
    with pytest.raises(ApiError) as ei:
        _bind(api, exts[0], "p0")
    assert ei.value.code == 503 and "ledger grace" in str(ei.value)
    pod = api.get_pod("default", "p0")
    assert not (pod.get("spec") or {}).get("nodeName") and "ALIYUN_COM_GPU_GROUP" not in obj_annotations(pod)
    assert "default/p0" not in _ledger(api)
    assert exts[0].metrics.bind_aborts.labels("ledger_grace")._value.get() == 1


def test_the_bind_retry_loop_has_a_time_budget():
    """ADVICE r5 (scheduler.py:487): informer events for a node wait while a bind holds its lock; a ledger
    that keeps conflicting ends the bind after `bind_budget_s`, not after the apiserver's patience."""
    import time as _t

    from gpu_topology_on_k8s_amd.k8s.api import ApiError

    api = FakeAPIServer()
    c = Contract()
    t = fx.f7_mi355x()
    api.create_node(make_node("n1", labels={c.label_model: "MI355X"}, annotations=encode_node_annotations(t, c),
                              capacity={c.resource_name: str(t.n)}))
    ext = TopologyExtender(api, _cfg(ledger=True, bind_budget_s=0.1, ledger_attempts=100))
    api.create_pod(make_pod("p0", gpus=1))
    real = ext.cache.refresh_node

    def slow_refresh(name):
        _t.sleep(0.04)
        return real(name)

    ext.cache.refresh_node = slow_refresh
    api.inject("create_lease" if STORE["store"] == "lease" else "patch_node", 409, times=1000)
    t0 = _t.monotonic()
    with pytest.raises(ApiError) as ei:
        _bind(api, ext, "p0")
    assert ei.value.code == 409 and "budget" in str(ei.value) and _t.monotonic() - t0 < 1.0
    assert ext.metrics.bind_aborts.labels("budget")._value.get() == 1
    assert ext.metrics.bind_lock_seconds._sum.get() > 0


def test_a_binds_pod_list_is_a_watch_cache_read_no_older_than_its_ledger():
    """Each bind refreshes its node: the node, the ledger, then the node's pods — read from the
    apiserver's watch cache but no older than the ledger and node just read (resourceVersionMatch=
    NotOlderThan), instead of an etcd range over every pod of the cluster.  A cache that cannot catch
    up (504) gets a consistent read; over HTTP the query carries the floor."""
    from gpu_topology_on_k8s_amd.k8s import serve_http
    from gpu_topology_on_k8s_amd.k8s.api import ApiError, RestKubeAPI

    api, exts, _ = _two(ledger=True, n_pods=3)
    floors = []
    real = api.list_pods

    def spy(node_name=None, namespace=None, cached=False, not_older_than=None):
        # the refresh has just read the node and the ledger: its floor is the newer of the two
        rvs = [int(api.get_node("n1")["metadata"]["resourceVersion"])]
        if STORE["store"] == "lease" and ("kube-system", "gpu-ledger.n1") in api.leases:
            rvs.append(int(api.get_lease("kube-system", "gpu-ledger.n1")["metadata"]["resourceVersion"]))
        floors.append((not_older_than, max(rvs)))
        return real(node_name=node_name, namespace=namespace, cached=cached, not_older_than=not_older_than)

    api.list_pods = spy
    _bind(api, exts[0], "p0")
    _bind(api, exts[1], "p1")
    node_rv = int(api.get_node("n1")["metadata"]["resourceVersion"])
    assert len(floors) >= 2 and all(f is not None and int(f) == want for f, want in floors), floors
    assert api.min_rv_reads["Pod"] >= 2
    # a watch cache that cannot catch up: the bind still decides on a consistent read
    def too_new(node_name=None, namespace=None, cached=False, not_older_than=None):
        if not_older_than is not None:
            raise ApiError(504, "Timeout: Too large resource version")
        return real(node_name=node_name, namespace=namespace, cached=cached)

    api.list_pods = too_new
    d = _bind(api, exts[0], "p2")
    assert d is not None and len(d.ids) == 1
    api.list_pods = real
    srv, url = serve_http(api)
    try:
        before = api.min_rv_reads["Pod"]
        got = RestKubeAPI(url).list_pods(node_name="n1", not_older_than=str(node_rv))
        assert len(got) == 3 and api.min_rv_reads["Pod"] == before + 1
        with pytest.raises(ApiError) as ei:
            RestKubeAPI(url).list_pods(node_name="n1", not_older_than=str(10 ** 9))
        assert ei.value.code == 504
    finally:
        srv.shutdown()


def test_the_ledger_lease_is_owned_by_its_node():
    """A node's ledger Lease carries an ownerReference to the Node: the garbage collector removes it
    with the node, so Leases of deleted nodes do not pile up in the extender's namespace."""
    if STORE["store"] != "lease":
        pytest.skip("the Node store has no separate object")
    api, exts, _ = _two(ledger=True, n_pods=1)
    _bind(api, exts[0], "p0")
    lease = api.get_lease("kube-system", "gpu-ledger.n1")
    node = api.get_node("n1")
    assert lease["metadata"]["ownerReferences"] == [{"apiVersion": "v1", "kind": "Node", "name": "n1",
                                                     "uid": node["metadata"]["uid"]}]
