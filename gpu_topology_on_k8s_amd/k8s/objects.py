"""Helpers over Kubernetes object JSON (plain dicts, exactly what the apiserver returns)."""
from __future__ import annotations

from typing import Any, Dict, Iterable, List, Optional, Sequence, Tuple

__all__ = [
    "meta", "annotations", "labels", "pod_key", "pod_node", "pod_phase", "pod_is_terminal", "pod_gpu_request",
    "pod_device_steps", "make_pod", "make_node", "parse_quantity",
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
