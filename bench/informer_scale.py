#!/usr/bin/env python3
"""The extender's informer on a synthetic large cluster.

A fake apiserver (k8s/fake.py) holding ``--nodes`` MI355X nodes and ``--pods`` pods (realistic object
bulk: managedFields, env, volume mounts, status conditions; a quarter of them terminal) is served over
HTTP.  For each informer mode an extender process of its own (so its RSS is its own) LISTs and WATCHes
it through the REST client:

* ``legacy``   — round 5: one unpaginated consistent LIST of every pod and node, objects kept whole;
* ``clientgo`` — a watch-cache LIST (``resourceVersion=0``), terminal pods filtered server-side, objects
  trimmed to what the cache reads; the apiserver answers it whole, as apiservers before the paginated
  watch cache ignore ``limit`` there;
* ``paged``    — the same with an apiserver that pages it (limit/continue, 500 a page): the LIST never
  sits in the extender's memory whole.

Recorded per mode: LIST time to synced, LIST requests and JSON bytes the apiserver served, the
extender's peak RSS and the RSS it keeps after the sync (freed heap returned with ``malloc_trim``),
one /prioritize over every node.  In the ``clientgo`` and ``paged`` modes the apiserver
then cuts the open pod watch and refuses the next watch attempts (503): the extender must see the
pods created meanwhile with **zero** relists.

    python bench/informer_scale.py --nodes 5000 --pods 100000 --out profiles/sched/informer_scale.json
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _rss_mb(trim: bool = False) -> float:
    """Resident set size; ``trim`` first hands freed heap back to the kernel (glibc ``malloc_trim``), so
    the number is what the process keeps, not the high-water mark of a LIST it has already dropped."""
    import gc

    import psutil

    if trim:
        import ctypes

        gc.collect()
        try:
            ctypes.CDLL("libc.so.6").malloc_trim(0)
        except OSError:
            pass
    return psutil.Process().memory_info().rss / 2 ** 20


def _peak_mb() -> float:
    """This process's RSS high-water mark (``VmHWM``: reset at exec, unlike ``ru_maxrss``, which would
    carry the parent's footprint over from the fork)."""
    with open("/proc/self/status") as f:
        for line in f:
            if line.startswith("VmHWM:"):
                return int(line.split()[1]) / 1024
    return float("nan")


def child(url: str, mode: str, n_nodes: int) -> None:
    """The extender side: sync, report, then (clientgo) wait for the parent's injected watch faults."""
    import gc

    from gpu_topology_on_k8s_amd.extender import ExtenderConfig, TopologyExtender
    from gpu_topology_on_k8s_amd.k8s.api import RestKubeAPI
    from gpu_topology_on_k8s_amd.k8s.informer import Informer
    from gpu_topology_on_k8s_amd.k8s.objects import make_pod

    rss0 = _rss_mb(trim=True)
    api = RestKubeAPI(url, timeout=600.0)
    ext = TopologyExtender(api, ExtenderConfig(resync_s=0.0))
    if mode == "legacy":
        inf = Informer(api, ext.cache.on_list, ext.cache.on_event, begin_list=ext.cache.begin_list, page_size=0,
                       watch_cache=False, watch_timeout=60.0)
        ext.cache.attach_informer(inf)
    else:  # clientgo: a watch-cache LIST the apiserver answers whole; paged: one it pages (limit/continue)
        inf = ext.cache.make_informer(page_size=500, watch_timeout=60.0, backoff=0.05, max_backoff=0.5)
    t0 = time.perf_counter()
    inf.start()
    assert inf.wait_synced(1200)
    sync_s = time.perf_counter() - t0
    peak = _peak_mb()
    rss = _rss_mb(trim=True)
    names = [f"n{i}" for i in range(n_nodes)]
    pod = make_pod("probe-pod", gpus=4)
    t1 = time.perf_counter()
    prio = ext.prioritize(pod, names)
    prio_ms = (time.perf_counter() - t1) * 1e3
    out = {"mode": mode, "sync_s": round(sync_s, 2), "rss_mb_before": round(rss0, 1), "rss_mb_peak": round(peak, 1),
           "rss_mb_synced": round(rss, 1), "rss_mb_cache": round(rss - rss0, 1),
           "pod_list": inf.last_list.get("Pod"), "node_list": inf.last_list.get("Node"),
           "prioritize_all_nodes_ms": round(prio_ms, 1), "nodes_scored": len(prio),
           "nodes_with_free_4": sum(1 for _, score in prio if score > 0)}
    print("SYNCED " + json.dumps(out), flush=True)
    if mode != "legacy":
        line = sys.stdin.readline().strip()  # "GO <count>": the parent cut the watch and created pods
        want = int(line.split()[1])
        t2 = time.perf_counter()
        deadline = time.monotonic() + 120
        while time.monotonic() < deadline:
            got = sum(1 for st in ext.cache.nodes() for k in st.allocs if k.startswith(f"default/late-{mode}-"))
            if got >= want:
                break
            time.sleep(0.05)
        out2 = {"late_pods_seen": got, "late_pods_created": want, "catch_up_s": round(time.perf_counter() - t2, 2),
                "pod_lists": inf.lists["Pod"], "pod_relists": inf.relists("Pod"), "watch_errors": inf.watch_errors["Pod"],
                "watch_resumes": inf.watch_resumes["Pod"]}
        print("FAULTS " + json.dumps(out2), flush=True)
    inf.stop()


def build_cluster(n_nodes: int, n_pods: int, terminal_frac: float):
    """A FakeAPIServer filled directly (no watch history: only changes after the LIST are watched)."""
    from gpu_topology_on_k8s_amd.k8s import Contract, FakeAPIServer, PodAssignment
    from gpu_topology_on_k8s_amd.k8s.annotations import encode_node_annotations
    from gpu_topology_on_k8s_amd.k8s.objects import make_node, make_pod
    from gpu_topology_on_k8s_amd.topology import fixtures as fx

    C = Contract()
    api = FakeAPIServer(history=100_000)
    ann = encode_node_annotations(fx.f7_mi355x(), C)
    images = [{"names": [f"registry.example.com/team/image-{j}:v{j}"], "sizeBytes": 10 ** 9} for j in range(30)]
    for i in range(n_nodes):
        node = make_node(f"n{i}", labels={"kubernetes.io/hostname": f"n{i}", C.label_model: "MI355X"}, annotations=ann,
                         capacity={C.resource_name: "8", "cpu": "256", "memory": "3Ti"})
        node["metadata"]["managedFields"] = [{"manager": "kubelet", "fieldsV1": {"f:status": {"f:images": {}}}}] * 3
        node["status"]["images"] = images
        node["status"]["conditions"] = [{"type": t, "status": "False"} for t in ("MemoryPressure", "DiskPressure", "PIDPressure")]
        node["metadata"]["uid"] = f"node-uid-{i}"
        api._rv += 1
        node["metadata"]["resourceVersion"] = str(api._rv)
        api.nodes[node["metadata"]["name"]] = node
    per_node = max(1, n_pods // n_nodes)
    k = 0
    for i in range(n_nodes):
        used = 0
        for j in range(per_node):
            terminal = (k % 100) < terminal_frac * 100
            g = 1 if used < 8 and not terminal and j % 3 == 0 else 0
            a = PodAssignment([used], True, 1_700_000_000).to_annotations() if g else {}
            pod = make_pod(f"p{k}", gpus=g, node=f"n{i}", annotations=a, labels={"app": f"svc-{k % 50}"})
            md = pod["metadata"]
            md["uid"] = f"pod-uid-{k}"
            md["creationTimestamp"] = "2026-10-01T00:00:00Z"
            md["managedFields"] = [{"manager": "kube-controller-manager", "operation": "Update",
                                    "fieldsV1": {"f:metadata": {"f:labels": {f"f:k{x}": {} for x in range(6)}}}}] * 3
            md["annotations"]["kubectl.kubernetes.io/last-applied-configuration"] = "{" + "x" * 600 + "}"
            c = pod["spec"]["containers"][0]
            c["env"] = [{"name": f"ENV_{x}", "value": f"value-{x}-" + "v" * 20} for x in range(15)]
            c["volumeMounts"] = [{"name": f"vol-{x}", "mountPath": f"/var/run/vol-{x}", "readOnly": True} for x in range(4)]
            c["command"] = ["python", "-m", "serve", "--port", "8080"]
            pod["spec"]["volumes"] = [{"name": f"vol-{x}", "configMap": {"name": f"cm-{x}"}} for x in range(4)]
            pod["status"] = {"phase": "Succeeded" if terminal else "Running", "podIP": f"10.{i % 250}.{j}.{k % 250}",
                             "conditions": [{"type": t, "status": "True", "lastTransitionTime": "2026-10-01T00:00:00Z"}
                                            for t in ("PodScheduled", "Initialized", "ContainersReady", "Ready")],
                             "containerStatuses": [{"name": "c0", "ready": True, "restartCount": 0,
                                                    "image": "registry.example.com/team/app:v1", "imageID": "sha256:" + "a" * 64}]}
            used += g
            api._rv += 1
            md["resourceVersion"] = str(api._rv)
            api.pods[("default", md["name"])] = pod
            k += 1
    return api, k


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--nodes", type=int, default=5000)
    ap.add_argument("--pods", type=int, default=100_000)
    ap.add_argument("--terminal", type=float, default=0.25, help="fraction of pods that are Succeeded")
    ap.add_argument("--modes", default="legacy,clientgo,paged")
    ap.add_argument("--late-pods", type=int, default=200, help="pods created while the watch is broken")
    ap.add_argument("--out", default="")
    ap.add_argument("--child", default="")
    ap.add_argument("--url", default="")
    a = ap.parse_args()
    if a.child:
        child(a.url, a.child, a.nodes)
        return 0
    import json as _json

    from gpu_topology_on_k8s_amd.k8s import PodAssignment, serve_http
    from gpu_topology_on_k8s_amd.k8s.objects import make_pod

    t0 = time.perf_counter()
    api, n_pods = build_cluster(a.nodes, a.pods, a.terminal)
    sample = next(iter(api.pods.values()))
    report = {"nodes": a.nodes, "pods": n_pods, "terminal_fraction": a.terminal,
              "pod_json_bytes_sample": len(_json.dumps(sample)), "build_s": round(time.perf_counter() - t0, 1),
              "modes": {}}
    srv, url = serve_http(api)
    try:
        for mode in a.modes.split(","):
            api.watch_cache_pages = mode == "paged"  # an apiserver that pages watch-cache LISTs (k8s >= 1.31)
            b0, r0 = dict(api.bytes_served), dict(api.list_requests)
            p = subprocess.Popen([sys.executable, os.path.abspath(__file__), "--child", mode, "--url", url, "--nodes", str(a.nodes)],
                                 stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, cwd=REPO)
            res = {}
            for line in p.stdout:
                if line.startswith("SYNCED "):
                    res.update(_json.loads(line[7:]))
                    res["list_bytes"] = {k: api.bytes_served[k] - b0.get(k, 0) for k in ("Node", "Pod")}
                    res["list_requests"] = {k: api.list_requests[k] - r0.get(k, 0) for k in ("Node", "Pod")}
                    print(f"[informer_scale] {mode}: synced in {res['sync_s']}s, peak RSS {res['rss_mb_peak']} MB, kept "
                          f"{res['rss_mb_cache']} MB, {res['list_bytes']['Pod'] / 2 ** 20:.0f} MB of pods listed in "
                          f"{res['list_requests']['Pod']} requests", flush=True)
                    if mode != "legacy":
                        api.cut_watch("Pod", after=0)
                        api.inject("watch_Pod", 503, times=3)
                        for i in range(a.late_pods):
                            api.create_pod(make_pod(f"late-{mode}-{i}", gpus=1, node=f"n{i % a.nodes}",
                                                    annotations=PodAssignment([7], True, 1_700_000_000).to_annotations()))
                        p.stdin.write(f"GO {a.late_pods}\n")
                        p.stdin.flush()
                elif line.startswith("FAULTS "):
                    res["watch_faults"] = _json.loads(line[7:])
                    print(f"[informer_scale] {mode}: after a cut watch + 3 refused watches: {res['watch_faults']}", flush=True)
            p.wait(timeout=1200)
            res["exit"] = p.returncode
            report["modes"][mode] = res
    finally:
        srv.shutdown()
    text = _json.dumps(report, indent=1)
    print(text)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            f.write(text + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
