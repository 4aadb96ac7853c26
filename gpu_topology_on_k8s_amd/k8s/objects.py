"""Helpers over Kubernetes object JSON (plain dicts, exactly what the apiserver returns)."""
from __future__ import annotations

from typing import Any, Dict, Iterable, List, Optional

__all__ = [
    "meta", "annotations", "labels", "pod_key", "pod_node", "pod_phase", "pod_is_terminal", "pod_gpu_request",
    "make_pod", "make_node", "parse_quantity",
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


def pod_gpu_request(p: Obj, resource_names: Iterable[str]) -> int:
    """Devices requested by a pod: sum over containers of limits (or requests) of the resource;
    init containers run sequentially, so the pod needs max(sum(containers), max(init))."""
    names = list(resource_names)
    spec = p.get("spec") if isinstance(p, dict) else None
    spec = spec if isinstance(spec, dict) else {}

    def one(c: Obj) -> int:
        res = c.get("resources") if isinstance(c, dict) else None
        for section in ("limits", "requests"):
            vals = res.get(section) if isinstance(res, dict) else None
            for n in names if isinstance(vals, dict) else ():
                if n in vals:
                    return parse_quantity(vals[n])
        return 0

    def containers(key: str) -> list:
        cs = spec.get(key)
        return cs if isinstance(cs, list) else []

    main = sum(one(c) for c in containers("containers"))
    init = max([one(c) for c in containers("initContainers")] or [0])
    return max(main, init)


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
) -> Obj:
    cs: List[Obj] = []
    for i in range(containers):
        c: Obj = {"name": f"c{i}", "image": "rocm/pytorch:latest"}
        if gpus and i == 0:
            c["resources"] = {"limits": {resource: str(gpus)}}
        cs.append(c)
    spec: Obj = {"containers": cs, "schedulerName": scheduler_name}
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
