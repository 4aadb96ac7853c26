"""Operator-requested hardware repartitioning of a node (``--partition-control on``).

The operator labels a node ``<prefix>/compute-partition-request=CPX`` (and optionally
``<prefix>/memory-partition-request=NPS4``).  The device plugin owns the node's GPUs, so it makes
the switch itself.  Device IDs, and with them every pod's GROUP annotation, change with the partition
mode, so the switch follows the rules of a time-slice relabel (``__main__.py``) and of an idle-time
re-probe (``plugin.reprobe``):

1. it happens only while no pod holds a device of the node;
2. the node is marked ``<prefix>/probing: <deadline>`` first, so the extender's filter, sort, bind
   and preempt skip it.  After a settle window, for binds already past the extender, the node must
   still be idle;
3. the switch itself is :func:`topology.partition.apply_partition` (amdsmi, needs root);
4. a Kubernetes Event records the outcome.  A refused switch (no permission, a mode the package
   does not offer) clears the mark and is recorded as ``<prefix>/partition-change-failed`` on the
   node; it is not tried again until the label asks for something else.  After a switch the mark
   stays: the node's published layout is the old one until the plugin restarts (exit 75, like any
   layout change) and publishes the new one, and the restarted plugin clears it then
   (``DevicePluginServer._clear_stale_mark``; the mark's deadline covers a plugin that never
   comes back).  At start-up the switch runs before discovery, so the first registration already
   shows the new layout.
"""
from __future__ import annotations

import contextlib
import logging
import math
import time
from typing import Callable, ContextManager, Optional, Tuple

from ..k8s.annotations import Contract
from ..k8s.events import record_event
from ..topology.partition import PartitionError, apply_partition, normalise, partition_info

log = logging.getLogger("gtk.deviceplugin.partition")

__all__ = ["partition_request", "repartition"]


def partition_request(api, node_name: str, contract: Contract) -> Tuple[Optional[str], Optional[str], dict]:
    """(compute, memory, node) the node's labels ask for; (None, None, node) without a request."""
    node = api.get_node(node_name)
    labels = (node.get("metadata") or {}).get("labels") or {}
    return (labels.get(contract.partition_request_label) or None, labels.get(contract.memory_partition_request_label) or None,
            node)


def _event(api, node_name: str, reason: str, msg: str, type_: str) -> None:
    record_event(api, {"kind": "Node", "metadata": {"name": node_name}}, reason, msg, type_,
                 component="gpu-topology-device-plugin", host=node_name)


def repartition(api, node_name: str, contract: Contract, idle_fn: Callable[[], bool], lib: Optional[str] = None,
                reload_driver: bool = False, settle_s: float = 2.0, mark_s: float = 600.0, time_slices: int = 1,
                wait: Callable[[float], bool] = lambda s: (time.sleep(s), False)[1],
                clock: Callable[[], float] = time.time, hold: Optional[Callable[[], ContextManager]] = None
                ) -> Tuple[str, str]:
    """One reconciliation pass.  -> (outcome, message), outcome one of
    ``none`` (no request), ``same`` (already there), ``invalid``, ``skipped`` (this request failed
    before), ``unavailable`` (amdsmi reports no package: nothing recorded, the next pass asks again),
    ``busy`` (pods hold devices), ``stopped`` (``wait`` returned True), ``ok``, ``failed`` (nothing
    changed), ``partial`` (failed, but the device layout changed on the way -- a compute step took on
    some packages, or a memory step and its driver reload ran before a later step failed: the plugin
    must restart like after ``ok``).

    ``hold`` (``DevicePluginServer.allocation_hold``) holds the plugin's Allocate from the moment the
    node is marked until the switch is over.  An Allocate that arrives meanwhile (a bind already past
    the extender, or a pod that bypassed it) makes the node busy: the switch is abandoned before it
    starts (or the driver reload is held back) and the Allocate proceeds on the old layout.  One that
    arrives while an amdsmi step is already running waits for it, and is then refused, because its
    device IDs name the old layout (the kubelet fails the pod; the plugin restarts)."""
    if api is None or not node_name:
        return "none", "no apiserver"
    want_c, want_m, node = partition_request(api, node_name, contract)
    if want_c is None and want_m is None:
        return "none", ""
    try:
        want_c, want_m = normalise(want_c, want_m)
    except PartitionError as e:
        return "invalid", str(e)
    tag = f"{want_c or '-'}/{want_m or '-'}"
    info = partition_info(lib)
    if not info:  # not "already there": there is nothing to compare (amdsmi down or no GPU visible)
        return "unavailable", f"{tag} requested; amdsmi reports no GPU packages"
    if all((not want_c or p["compute"] == want_c) and (not want_m or p["memory"] == want_m) for p in info):
        ann = (node.get("metadata") or {}).get("annotations") or {}
        if contract.partition_failed_key in ann:
            api.patch_node(node_name, annotations={contract.partition_failed_key: None})
        return "same", f"already {tag}"
    failed = ((node.get("metadata") or {}).get("annotations") or {}).get(contract.partition_failed_key, "")
    if failed.startswith(tag + ":"):
        return "skipped", f"{tag} failed before ({failed[len(tag) + 1:].strip()}); change the label to try again"
    if want_c and want_c != "SPX" and time_slices > 1:
        # time slices split whole (SPX) GPUs; the two kinds of fraction are not stacked
        why = (f"the node is time-sliced ({time_slices} per GPU, {contract.time_slices_label}): remove that label "
               "before asking for XCP partitions")
        api.patch_node(node_name, annotations={contract.partition_failed_key: f"{tag}: {why}"})
        _event(api, node_name, "FailedGPUPartitionChange", f"{tag}: {why}", "Warning")
        return "failed", why
    if not idle_fn():
        return "busy", f"{tag} requested; waiting until no pod holds a device"
    api.patch_node(node_name, annotations={contract.probing_key: str(int(math.ceil(clock() + mark_s)))})
    switched = False
    try:
        with (hold() if hold is not None else contextlib.nullcontext()) as h:
            def still_idle() -> bool:
                return idle_fn() and not (h is not None and h.contended())

            if settle_s > 0 and wait(settle_s):
                return "stopped", ""
            if not still_idle():
                return "busy", f"{tag} requested; a pod arrived while the node was being marked"
            before = f"{info[0]['compute']}/{info[0]['memory']}" if info else "?"
            log.warning("switching GPU partitions %s -> %s (node idle)", before, tag)
            if h is not None:
                h.started = True
            try:
                res = apply_partition(want_c, want_m, lib=lib, reload_driver=reload_driver, before_reload=still_idle)
            except Exception as e:  # noqa: BLE001 - PartitionError, or amdsmi without the setters: recorded, not retried
                res = {"ok": False, "reason": str(e)[:500]}
            # the old device IDs are stale exactly when the exposed devices changed: a compute step that
            # took (even if a later one failed), a memory step only once the driver reloaded -- not a
            # memory mode pending a reload, nor a reload held back for an arriving Allocate
            changed = bool(res.get("layout_changed", res["ok"]))
            if h is not None:
                h.switched = changed
        if res["ok"]:
            switched = True
            api.patch_node(node_name, annotations={contract.partition_failed_key: None})
            _event(api, node_name, "GPUPartitionChanged", f"GPU partitions {before} -> {tag}", "Normal")
            return "ok", f"{before} -> {tag}"
        api.patch_node(node_name, annotations={contract.partition_failed_key: f"{tag}: {res['reason']}"[:1000]})
        _event(api, node_name, "FailedGPUPartitionChange", f"{before} -> {tag}: {res['reason']}", "Warning")
        if changed:
            switched = True  # keep the mark: the restarted plugin publishes the changed layout and clears it
            return "partial", f"{before} -> {tag} partly applied: {res['reason']}"
        return "failed", res["reason"]
    finally:
        if not switched:  # after a switch the restarted plugin clears it, once the new layout is published
            api.patch_node(node_name, annotations={contract.probing_key: None})
