"""Where the extenders' allocation ledger lives.

Every bind records its device set in a per-node ledger under an optimistic-concurrency precondition,
so two extender instances that decided on the same state cannot hand out one device twice
(extender/scheduler.py ``bind``; ``design.md:223-246`` "who writes what").  Round 5 kept the ledger in
an annotation of the Node object, which made every extender hold ``patch`` on every Node and fanned
each bind out to every node watcher in the cluster.

The ledger now lives in one ``coordination.k8s.io/v1`` **Lease per node** in the extender's own
namespace (``gpu-ledger.<node>``), in the same annotation (``<prefix>/gpu-ledger``) with the same
JSON, written with the Lease's ``resourceVersion`` as precondition (a missing Lease is created; a
concurrent create answers 409 AlreadyExists, the same conflict).  The extender then needs no write
access to Nodes at all: ``leases`` verbs in one namespace only (deploy/gpu-topology.yaml).

``store``:
  * ``lease`` — the default;
  * ``node``  — round 5's Node annotation (a single-version fleet that has not moved yet);
  * ``both``  — the rolling-upgrade mode (docs/MIGRATION.md): read the entries of both, write both
    (the Lease first), so old and new extenders see each other's binds in flight.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

from ..k8s.annotations import Contract, dump_ledger, ledger_gen, ledger_uids, parse_ledger
from ..k8s.api import KubeAPI, NotFound
from ..k8s.objects import annotations as obj_annotations
from ..k8s.objects import meta

__all__ = ["LedgerStore", "LEASE_PREFIX", "lease_name", "lease_node", "STORES"]

LEASE_PREFIX = "gpu-ledger."
STORES = ("lease", "node", "both")

Entries = Dict[str, Tuple[Tuple[int, ...], float]]


def lease_name(node: str) -> str:
    return LEASE_PREFIX + node


def lease_node(lease: dict, contract: Contract = Contract()) -> Optional[str]:
    """The node a ledger Lease is for (its ``<prefix>/node`` annotation, else its name), or None when
    the Lease is not a ledger."""
    name = str(meta(lease).get("name", ""))
    if not name.startswith(LEASE_PREFIX):
        return None
    return obj_annotations(lease).get(f"{contract.prefix}/node") or name[len(LEASE_PREFIX):]


class LedgerStore:
    def __init__(self, store: str = "lease", namespace: str = "kube-system", contract: Contract = Contract()):
        if store not in STORES:
            raise ValueError(f"ledger store must be one of {STORES}, got {store!r}")
        self.store = store
        self.namespace = namespace
        self.contract = contract

    @property
    def uses_lease(self) -> bool:
        return self.store in ("lease", "both")

    @property
    def uses_node(self) -> bool:
        return self.store in ("node", "both")

    def read_lease(self, api: KubeAPI, node: str) -> Optional[dict]:
        """The node's ledger Lease, or None if it does not exist yet."""
        try:
            return api.get_lease(self.namespace, lease_name(node))
        except NotFound:
            return None

    def lease_object(self, node: str, value: str, node_uid: str = "") -> dict:
        """A node's ledger Lease.  With the node's UID it is owned by the Node, so the garbage collector
        deletes it with the node (a namespaced dependent may have a cluster-scoped owner; without
        ``blockOwnerDeletion`` this needs no permission on the Node)."""
        c = self.contract
        md = {"name": lease_name(node), "namespace": self.namespace,
              "labels": {"app.kubernetes.io/part-of": "gpu-topology-amd", "app.kubernetes.io/component": "gpu-ledger"},
              "annotations": {c.ledger_key: value, f"{c.prefix}/node": node}}
        if node_uid:
            md["ownerReferences"] = [{"apiVersion": "v1", "kind": "Node", "name": node, "uid": node_uid}]
        return {"apiVersion": "coordination.k8s.io/v1", "kind": "Lease", "metadata": md,
                "spec": {"holderIdentity": "gpu-topology-extender"}}

    def write(self, api: KubeAPI, node: str, entries: Entries, lease_rv: Optional[str], lease_gen: int,
              node_rv: str, node_gen: int, uids: Optional[Dict[str, str]] = None, node_uid: str = "") -> None:
        """Record ``entries`` (with their pods' ``uids``) as the node's ledger, conditional on the
        versions the decision saw.  Raises :class:`~..k8s.api.Conflict` when another writer got there
        first."""
        key = self.contract.ledger_key
        if self.uses_lease:
            value = dump_ledger(entries, lease_gen + 1, uids)
            if lease_rv is None:
                api.create_lease(self.namespace, self.lease_object(node, value, node_uid))  # 409 AlreadyExists: a race lost
            else:
                api.patch_lease(self.namespace, lease_name(node), {key: value}, resource_version=lease_rv)
        if self.uses_node:
            api.patch_node(node, annotations={key: dump_ledger(entries, node_gen + 1, uids)}, resource_version=node_rv)

    def release(self, api: KubeAPI, node: str, pod_key: str) -> bool:
        """Drop one entry (a failed bind), conditionally; -> True when done or nothing to do.  Raises
        Conflict for the caller to retry."""
        key = self.contract.ledger_key
        if self.uses_lease:
            lease = self.read_lease(api, node)
            if lease is not None:
                ann = obj_annotations(lease)
                entries = parse_ledger(ann, self.contract)
                if pod_key in entries:
                    del entries[pod_key]
                    api.patch_lease(self.namespace, lease_name(node),
                                    {key: dump_ledger(entries, ledger_gen(ann, self.contract) + 1, ledger_uids(ann, self.contract))},
                                    resource_version=str(meta(lease).get("resourceVersion", "")))
        if self.uses_node:
            n = api.get_node(node)
            ann = obj_annotations(n)
            entries = parse_ledger(ann, self.contract)
            if pod_key in entries:
                del entries[pod_key]
                api.patch_node(node, annotations={key: dump_ledger(entries, ledger_gen(ann, self.contract) + 1,
                                                                   ledger_uids(ann, self.contract))},
                               resource_version=str(meta(n).get("resourceVersion", "")))
        return True
