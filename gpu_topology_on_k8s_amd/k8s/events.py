"""Kubernetes Events for scheduling and allocation outcomes.

The deploy manifest grants ``events: create`` (``deploy/gpu-topology.yaml``); the extender records a
``Warning``/``FailedGPUTopologyBind`` on the pod when a bind fails and a ``Normal``/``GPUTopologyBound``
when it succeeds, and the device plugin records ``FailedGPUAllocate`` on the node when the kubelet
asks for devices it cannot hand out.  Events are best effort: a failure to record one is logged and
never fails the operation it describes.
"""
from __future__ import annotations

import datetime
import logging
import uuid
from typing import Any, Dict, Optional

from .objects import meta

log = logging.getLogger(__name__)

__all__ = ["record_event"]


def _now() -> str:
    return datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def record_event(api, obj: Dict[str, Any], reason: str, message: str, type_: str = "Normal",
                 component: str = "gpu-topology", host: str = "") -> Optional[Dict[str, Any]]:
    """Create a core/v1 Event about ``obj`` (a Pod or Node dict); returns it, or None on failure."""
    if api is None:
        return None
    md = meta(obj)
    kind = obj.get("kind") or ("Node" if "namespace" not in md and (obj.get("status") or {}).get("allocatable") is not None else "Pod")
    ns = md.get("namespace", "default") if kind == "Pod" else "default"
    ts = _now()
    ev = {
        "apiVersion": "v1",
        "kind": "Event",
        "metadata": {"name": f"{md.get('name', 'obj')}.{uuid.uuid4().hex[:12]}", "namespace": ns},
        "involvedObject": {"apiVersion": "v1", "kind": kind, "name": md.get("name", ""),
                           **({"namespace": ns} if kind == "Pod" else {}), **({"uid": md["uid"]} if md.get("uid") else {})},
        "reason": reason,
        "message": message[:1024],
        "type": type_,
        "source": {"component": component, **({"host": host} if host else {})},
        "firstTimestamp": ts,
        "lastTimestamp": ts,
        "count": 1,
        "reportingComponent": component,
    }
    try:
        return api.create_event(ns, ev)
    except Exception as e:  # noqa: BLE001 - events never fail the operation they describe
        log.info("recording event %s on %s/%s failed: %s", reason, ns, md.get("name"), e)
        return None
