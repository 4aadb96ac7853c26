"""Helpers over Kubernetes object JSON (plain dicts, exactly what the apiserver returns)."""
from __future__ import annotations

from typing import Any, Dict, Iterable, List, Optional, Sequence, Tuple

__all__ = [
    "meta", "annotations", "labels", "pod_key", "pod_node", "pod_phase", "pod_is_terminal", "pod_gpu_request",
    "pod_device_steps", "make_pod", "make_node", "parse_quantity", "field_value", "match_fields", "trim_pod",
    "trim_node", "LIVE_POD_SELECTOR",
]

Obj = Dict[str, Any]


def meta(o: Obj) -> Obj:
    return o.setdefault("metadata", {})


def annotations(o: Obj) -> Dict[str, str]:
    return meta(o).get("annotations") or {}


def labels(o: Obj) -> Dict[str, str]:
    return meta(o).get("labels") or {}


def pod_key(p: Obj) -> str:
    m = meta(p)
    return f"{m.get('namespace', 'default')}/{m.get('name', '')}"


def pod_node(p: Obj) -> str:
    return (p.get("spec") or {}).get("nodeName") or ""


def pod_phase(p: Obj) -> str:
    return (p.get("status") or {}).get("phase") or "Pending"


def pod_is_terminal(p: Obj) -> bool:
    """Succeeded/Failed pods hold no devices (a deleting pod still does until it is gone)."""
    return pod_phase(p) in ("Succeeded", "Failed")


def parse_quantity(q: Any) -> int:
    """Integer extended-resource quantity ("4", 4, "4.0"); fractions are not allowed by k8s for
    extended resources, so anything else is rejected."""
    try:
        v = float(q) if isinstance(q, (int, float)) and not isinstance(q, bool) else float(str(q).strip())
        ok = v == v and abs(v) != float("inf") and v == int(v) and v >= 0
    except (TypeError, ValueError, OverflowError):
        ok = False
    if not ok:
        raise ValueError(f"extended resources must be non-negative integers, got {q!r}")
    return int(v)


def _container_request(c: Any, names: List[str]) -> int:
    res = c.get("resources") if isinstance(c, dict) else None
    for section in ("limits", "requests"):
        vals = res.get(section) if isinstance(res, dict) else None
        for n in names if isinstance(vals, dict) else ():
            if n in vals:
                return parse_quantity(vals[n])
    return 0


def _containers(p: Obj, key: str) -> list:
    spec = p.get("spec") if isinstance(p, dict) else None
    cs = spec.get(key) if isinstance(spec, dict) else None
    return cs if isinstance(cs, list) else []


def _is_sidecar(c: Any) -> bool:
    """A restartable init container (``restartPolicy: Always``, k8s >= 1.28): it keeps running beside
    the app containers, so it holds its devices for the pod's lifetime instead of lending them on."""
    return isinstance(c, dict) and c.get("restartPolicy") == "Always"


def pod_gpu_request(p: Obj, resource_names: Iterable[str]) -> int:
    """Devices a pod holds on its node, as the scheduler counts them (``PodRequests``): app containers
    and sidecars run together; a regular init container runs alone, beside the sidecars started before
    it, so the pod needs max(sum(app) + sum(sidecars), max over init_i of init_i + sidecars before i)."""
    names = list(resource_names)
    sidecars = peak = 0
    for c in _containers(p, "initContainers"):
        r = _container_request(c, names)
        if _is_sidecar(c):
            sidecars += r
            peak = max(peak, sidecars)
        else:
            peak = max(peak, r + sidecars)
    main = sum(_container_request(c, names) for c in _containers(p, "containers"))
    return max(main + sidecars, peak)


def pod_device_steps(p: Obj, resource_names: Iterable[str]) -> List[Tuple[str, int, str]]:
    """The kubelet device manager's ``Allocate`` calls for a pod, in the order it makes them:
    ``(container name, devices, kind)`` for every container that requests one of ``resource_names``,
    init containers first (``kind`` ``init`` or ``sidecar``), then the app containers (``app``).  The
    kubelet calls ``GetPreferredAllocation`` / ``Allocate`` once per such container with that
    container's own count; a regular init container's devices are handed on to the containers after
    it (they run after it has exited), a sidecar's are not."""
    names = list(resource_names)
    out: List[Tuple[str, int, str]] = []
    for key, kind in (("initContainers", "init"), ("containers", "app")):
        for i, c in enumerate(_containers(p, key)):
            r = _container_request(c, names)
            if r > 0:
                k = "sidecar" if kind == "init" and _is_sidecar(c) else kind
                out.append((str(c.get("name") or f"{key}[{i}]"), r, k))
    return out


def field_value(o: Obj, path: str) -> str:
    """The string value of a dotted field path (``status.phase``, ``spec.nodeName``), "" if absent —
    what a field selector compares (a missing ``status.phase`` is an empty string, as in the apiserver)."""
    cur: Any = o
    for part in path.split("."):
        cur = cur.get(part) if isinstance(cur, dict) else None
    return "" if cur is None else str(cur)


def match_fields(o: Obj, selector: Optional[str]) -> bool:
    """A field selector (``a.b=v``, ``a.b==v``, ``a.b!=v``, comma = AND) against an object."""
    for term in (selector or "").split(","):
        term = term.strip()
        if not term:
            continue
        if "!=" in term:
            k, v = term.split("!=", 1)
            if field_value(o, k.strip()) == v.strip():
                return False
        else:
            k, v = term.replace("==", "=").split("=", 1)
            if field_value(o, k.strip()) != v.strip():
                return False
    return True


#: what the extender's informer asks the apiserver for: pods that may hold devices (terminal ones
#: never do, and a long-lived cluster keeps many of them)
LIVE_POD_SELECTOR = "status.phase!=Succeeded,status.phase!=Failed"

_META_KEEP = ("name", "namespace", "uid", "resourceVersion", "creationTimestamp", "deletionTimestamp")


def _keep_annotation(key: str, prefix: str) -> bool:
    return key.startswith(("ALIYUN_COM_GPU_", "GPU_", "GPUPKG_", prefix + "/")) or key == "gpu-id"


def _trim_meta(o: Obj, prefix: str, keep_labels: bool) -> Obj:
    md = meta(o)
    out: Obj = {k: md[k] for k in _META_KEEP if k in md}
    ann = md.get("annotations") or {}
    out["annotations"] = {k: v for k, v in ann.items() if _keep_annotation(k, prefix)} if isinstance(ann, dict) else {}
    if keep_labels:
        out["labels"] = dict(md.get("labels") or {})
    return out


def trim_pod(p: Obj, prefix: str = "gputopology.amd.com") -> Obj:
    """The parts of a Pod the extender's cache reads (the informer's transform, like client-go's
    ``SetTransform``): identity, the GPU contract's annotations, node, phase and the containers'
    resource requests.  ``managedFields``, env, volumes, status conditions and the rest are dropped:
    a 100k-pod cluster is then held in tens of MB instead of GBs."""
    spec = p.get("spec") if isinstance(p.get("spec"), dict) else {}
    out_spec: Obj = {k: spec[k] for k in ("nodeName", "schedulerName") if k in spec}
    for key in ("containers", "initContainers"):
        cs = spec.get(key)
        if isinstance(cs, list):
            out_spec[key] = [{k: c[k] for k in ("name", "resources", "restartPolicy") if isinstance(c, dict) and k in c}
                             for c in cs]
    st = p.get("status") if isinstance(p.get("status"), dict) else {}
    return {"metadata": _trim_meta(p, prefix, keep_labels=False), "spec": out_spec,
            "status": {"phase": st["phase"]} if "phase" in st else {}}


def trim_node(n: Obj, prefix: str = "gputopology.amd.com") -> Obj:
    """The parts of a Node the extender's cache reads: identity, labels, the topology contract's
    annotations and the capacity/allocatable counts (``status.images`` alone can be 100 kB a node)."""
    st = n.get("status") if isinstance(n.get("status"), dict) else {}
    return {"metadata": _trim_meta(n, prefix, keep_labels=True),
            "status": {k: st[k] for k in ("capacity", "allocatable") if k in st}}


def make_pod(
    name: str,
    gpus: int = 0,
    namespace: str = "default",
    resource: str = "amd.com/gpu",
    annotations: Optional[Dict[str, str]] = None,
    labels: Optional[Dict[str, str]] = None,
    containers: int = 1,
    node: str = "",
    scheduler_name: str = "default-scheduler",
    split: Optional[Sequence[int]] = None,
    init: Sequence[int] = (),
    sidecars: Sequence[int] = (),
) -> Obj:
    """A pod requesting ``gpus`` devices in its first container, or ``split[i]`` in app container i;
    ``init`` adds regular init containers and ``sidecars`` restartable ones (devices each)."""
    cs: List[Obj] = []
    per = list(split) if split is not None else [gpus] + [0] * (containers - 1)
    for i, n in enumerate(per):
        c: Obj = {"name": f"c{i}", "image": "rocm/pytorch:latest"}
        if n:
            c["resources"] = {"limits": {resource: str(n)}}
        cs.append(c)
    inits: List[Obj] = []
    for kind, counts in (("sidecar", sidecars), ("init", init)):
        for i, n in enumerate(counts):
            c = {"name": f"{kind}{i}", "image": "rocm/pytorch:latest"}
            if n:
                c["resources"] = {"limits": {resource: str(n)}}
            if kind == "sidecar":
                c["restartPolicy"] = "Always"
            inits.append(c)
    spec: Obj = {"containers": cs, "schedulerName": scheduler_name}
    if inits:
        spec["initContainers"] = inits
    if node:
        spec["nodeName"] = node
    return {
        "apiVersion": "v1",
        "kind": "Pod",
        "metadata": {"name": name, "namespace": namespace, "annotations": dict(annotations or {}), "labels": dict(labels or {})},
        "spec": spec,
        "status": {"phase": "Pending"},
    }


def make_node(name: str, labels: Optional[Dict[str, str]] = None, annotations: Optional[Dict[str, str]] = None,
              capacity: Optional[Dict[str, str]] = None) -> Obj:
    cap = dict(capacity or {})
    return {
        "apiVersion": "v1",
        "kind": "Node",
        "metadata": {"name": name, "labels": dict(labels or {}), "annotations": dict(annotations or {})},
        "status": {"capacity": cap, "allocatable": dict(cap)},
    }
