"""Per-identity RBAC, enforced on the in-memory apiserver.

:func:`identities_from_manifests` reads the ServiceAccounts' rules out of the rendered deploy manifests
(config.py ``render_manifests``: the very objects ``deploy/gpu-topology.yaml`` holds) — ClusterRoles
through ClusterRoleBindings, Roles through RoleBindings (their namespace only) — plus the
``ValidatingAdmissionPolicy`` that confines a ServiceAccount to its own node.  :class:`RBACView` is a
:class:`~.api.KubeAPI` that checks every call of one identity against them before passing it to the
apiserver behind it and answers 403 Forbidden like the apiserver's authorizer (or admission) would.
The device plugin and the extender run through such views in the tests and the cluster simulation,
so a verb missing from the deploy RBAC fails a functional test, not a production rollout.
"""
from __future__ import annotations

import re
import threading
from dataclasses import dataclass, field
from typing import Any, Dict, Iterable, List, Optional, Tuple

from .api import ApiError, KubeAPI
from .objects import meta

__all__ = ["Rule", "Identity", "RBACView", "identities_from_manifests", "sa_username"]

Obj = Dict[str, Any]

_KIND_RESOURCE = {"Node": ("", "nodes"), "Pod": ("", "pods"), "Lease": ("coordination.k8s.io", "leases")}


def sa_username(namespace: str, name: str) -> str:
    return f"system:serviceaccount:{namespace}:{name}"


@dataclass(frozen=True)
class Rule:
    groups: Tuple[str, ...]
    resources: Tuple[str, ...]
    verbs: Tuple[str, ...]
    namespace: Optional[str] = None  # None: cluster-wide (a ClusterRoleBinding)

    def allows(self, verb: str, group: str, resource: str, namespace: Optional[str]) -> bool:
        return ((group in self.groups or "*" in self.groups) and (resource in self.resources or "*" in self.resources)
                and (verb in self.verbs or "*" in self.verbs) and (self.namespace is None or self.namespace == namespace))


@dataclass
class Identity:
    username: str
    rules: List[Rule] = field(default_factory=list)
    own_node_only: bool = False  # a ValidatingAdmissionPolicy confines its node / pod writes to its own node

    def allows(self, verb: str, group: str, resource: str, namespace: Optional[str] = None) -> bool:
        return any(r.allows(verb, group, resource, namespace) for r in self.rules)

    def grants(self) -> Dict[Tuple[Optional[str], str, str], set]:
        """(namespace or None, apiGroup, resource) -> verbs: the identity's effective permissions."""
        out: Dict[Tuple[Optional[str], str, str], set] = {}
        for r in self.rules:
            for g in r.groups:
                for res in r.resources:
                    out.setdefault((r.namespace, g, res), set()).update(r.verbs)
        return out


def identities_from_manifests(docs: Iterable[Obj]) -> Dict[str, Identity]:
    """ServiceAccount username -> its :class:`Identity`, from manifest objects."""
    docs = [d for d in docs if isinstance(d, dict)]
    roles = {(d["kind"], meta(d).get("namespace"), meta(d)["name"]): d.get("rules") or []
             for d in docs if d.get("kind") in ("Role", "ClusterRole")}
    out: Dict[str, Identity] = {}
    for d in docs:
        if d.get("kind") not in ("RoleBinding", "ClusterRoleBinding"):
            continue
        ns = meta(d).get("namespace") if d["kind"] == "RoleBinding" else None
        ref = d["roleRef"]
        rules = roles.get((ref["kind"], ns if ref["kind"] == "Role" else None, ref["name"]), [])
        for sub in d.get("subjects") or []:
            if sub.get("kind") != "ServiceAccount":
                continue
            ident = out.setdefault(sa_username(sub["namespace"], sub["name"]), Identity(sa_username(sub["namespace"], sub["name"])))
            for r in rules:
                ident.rules.append(Rule(tuple(r.get("apiGroups") or []), tuple(r.get("resources") or []),
                                        tuple(r.get("verbs") or []), ns))
    for d in docs:  # the own-node admission policy, matched to the identity its matchConditions name
        if d.get("kind") != "ValidatingAdmissionPolicy":
            continue
        for mc in (d.get("spec") or {}).get("matchConditions") or []:
            m = re.search(r"request\.userInfo\.username == '([^']+)'", mc.get("expression", ""))
            if m and m.group(1) in out and any("node-name" in v.get("expression", "")
                                               for v in (d.get("spec") or {}).get("validations") or []):
                out[m.group(1)].own_node_only = True
    return out


class RBACView(KubeAPI):
    """``api`` as seen by ``identity`` (with the token's node-name claim ``node_name``)."""

    def __init__(self, api: KubeAPI, identity: Identity, node_name: str = ""):
        self.api = api
        self.identity = identity
        self.node_name = node_name
        self.denied: List[str] = []  # every refusal, for tests to assert on
        self._lock = threading.Lock()

    def __getattr__(self, name):  # test / simulation helpers of the apiserver (create_pod, inject, calls ...)
        return getattr(self.api, name)

    def _forbid(self, msg: str) -> None:
        with self._lock:
            self.denied.append(msg)
        raise ApiError(403, msg)

    def _check(self, verb: str, group: str, resource: str, namespace: Optional[str] = None, name: str = "") -> None:
        if not self.identity.allows(verb, group, resource, namespace):
            where = f" in the namespace \"{namespace}\"" if namespace else " at the cluster scope"
            self._forbid(f"{resource}{'.' + group if group else ''} \"{name}\" is forbidden: User \"{self.identity.username}\" "
                         f"cannot {verb} resource \"{resource}\" in API group \"{group}\"{where}")

    def _own_node(self, node: str, what: str) -> None:
        if self.identity.own_node_only and node != self.node_name:
            self._forbid(f"admission webhook denied {what}: the GPU device plugin may only change its own node "
                         f"({self.node_name!r}) and the pods bound to it")

    # ------------------------------------------------------------------ nodes
    def get_node(self, name):
        self._check("get", "", "nodes", name=name)
        return self.api.get_node(name)

    def list_nodes(self, label_selector=None):
        self._check("list", "", "nodes")
        return self.api.list_nodes(label_selector)

    def patch_node(self, name, annotations=None, labels=None, resource_version=None):
        self._check("patch", "", "nodes", name=name)
        self._own_node(name, f"patch of node {name}")
        return self.api.patch_node(name, annotations, labels, resource_version)

    # ------------------------------------------------------------------ pods
    def get_pod(self, namespace, name):
        self._check("get", "", "pods", namespace, name)
        return self.api.get_pod(namespace, name)

    def list_pods(self, node_name=None, namespace=None, cached=False, not_older_than=None):
        self._check("list", "", "pods", namespace)
        return self.api.list_pods(node_name=node_name, namespace=namespace, cached=cached, not_older_than=not_older_than)

    def patch_pod_annotations(self, namespace, name, annotations, resource_version=None):
        self._check("patch", "", "pods", namespace, name)
        if self.identity.own_node_only:
            pod = self.api.get_pod(namespace, name)
            self._own_node((pod.get("spec") or {}).get("nodeName") or "", f"patch of pod {namespace}/{name}")
        return self.api.patch_pod_annotations(namespace, name, annotations, resource_version)

    def bind_pod(self, namespace, name, uid, node):
        self._check("create", "", "pods/binding", namespace, name)
        return self.api.bind_pod(namespace, name, uid, node)

    def create_event(self, namespace, event):
        self._check("create", "", "events", namespace)
        return self.api.create_event(namespace, event)

    # ------------------------------------------------------------------ leases
    def get_lease(self, namespace, name):
        self._check("get", "coordination.k8s.io", "leases", namespace, name)
        return self.api.get_lease(namespace, name)

    def create_lease(self, namespace, lease):
        self._check("create", "coordination.k8s.io", "leases", namespace, meta(lease).get("name", ""))
        return self.api.create_lease(namespace, lease)

    def patch_lease(self, namespace, name, annotations, resource_version=None):
        self._check("patch", "coordination.k8s.io", "leases", namespace, name)
        return self.api.patch_lease(namespace, name, annotations, resource_version)

    # ------------------------------------------------------------------ LIST + WATCH
    def list_with_version(self, kind, node_name=None):
        g, r = _KIND_RESOURCE[kind]
        self._check("list", g, r)
        return self.api.list_with_version(kind, node_name)

    def list_page(self, kind, limit=0, continue_token="", resource_version=None, field_selector=None, namespace=None):
        g, r = _KIND_RESOURCE[kind]
        self._check("list", g, r, namespace)
        return self.api.list_page(kind, limit, continue_token, resource_version, field_selector, namespace)

    def watch_stream(self, kind, resource_version, timeout=60.0, stop=None, field_selector=None, namespace=None):
        g, r = _KIND_RESOURCE[kind]
        self._check("watch", g, r, namespace)
        return self.api.watch_stream(kind, resource_version, timeout, stop, field_selector=field_selector, namespace=namespace)
