"""Kubernetes API access: the interface the extender and device plugin use, and a thin REST client.

The reference talks to the apiserver to annotate nodes (``design.md:76-82``), patch pod annotations
(``design.md:223-246``), list pods and bind (``design.md:119``).  :class:`KubeAPI` is exactly that
surface.  :class:`RestKubeAPI` speaks the real REST API (in-cluster service account or kubeconfig-
less explicit URL/token); :class:`~.fake.FakeAPIServer` implements the same interface in memory for
tests and the in-process cluster simulation, and can also be served over HTTP so the REST client is
exercised on the wire.
"""
from __future__ import annotations

import json
import logging
import os
import threading
import time
from typing import Any, Dict, Iterator, List, Optional, Tuple
from urllib.parse import quote

log = logging.getLogger(__name__)

__all__ = ["ApiError", "Conflict", "NotFound", "Gone", "KubeAPI", "RestKubeAPI"]

Obj = Dict[str, Any]


class ApiError(RuntimeError):
    def __init__(self, code: int, message: str = ""):
        super().__init__(f"{code}: {message}")
        self.code = code
        self.message = message


class Conflict(ApiError):
    def __init__(self, message: str = "conflict"):
        super().__init__(409, message)


class NotFound(ApiError):
    def __init__(self, message: str = "not found"):
        super().__init__(404, message)


class Gone(ApiError):
    """410: a watch's resourceVersion fell out of the apiserver's window; relist."""

    def __init__(self, message: str = "gone"):
        super().__init__(410, message)


def raise_for(code: int, message: str) -> None:
    if code == 404:
        raise NotFound(message)
    if code == 410:
        raise Gone(message)
    if code == 409:
        raise Conflict(message)
    raise ApiError(code, message)


class KubeAPI:
    """Subset of the Kubernetes API used by this framework."""

    def get_node(self, name: str) -> Obj:
        raise NotImplementedError

    def list_nodes(self, label_selector: Optional[str] = None) -> List[Obj]:
        raise NotImplementedError

    def patch_node(self, name: str, annotations: Optional[Dict[str, Optional[str]]] = None,
                   labels: Optional[Dict[str, Optional[str]]] = None, resource_version: Optional[str] = None) -> Obj:
        """JSON merge patch of node metadata (a ``None`` value deletes the key); with
        ``resource_version`` the patch is conditional (409 when the node changed since)."""
        raise NotImplementedError

    def get_pod(self, namespace: str, name: str) -> Obj:
        raise NotImplementedError

    def list_pods(self, node_name: Optional[str] = None, namespace: Optional[str] = None, cached: bool = False,
                  not_older_than: Optional[str] = None) -> List[Obj]:
        """Pods (of one node / namespace).  ``cached``: served from the apiserver's watch cache
        (``resourceVersion=0``: no etcd range over every pod of the cluster, possibly a little stale);
        for periodic passes that tolerate it (the device plugin's reconcile).  ``not_older_than``: a
        watch-cache read that reflects at least that resourceVersion (``resourceVersionMatch=
        NotOlderThan``; 504 when the cache cannot catch up)."""
        raise NotImplementedError

    def patch_pod_annotations(self, namespace: str, name: str, annotations: Dict[str, Optional[str]],
                              resource_version: Optional[str] = None) -> Obj:
        """Merge-patch pod annotations; with ``resource_version`` the patch is conditional (409 on mismatch)."""
        raise NotImplementedError

    def bind_pod(self, namespace: str, name: str, uid: str, node: str) -> None:
        raise NotImplementedError

    def create_event(self, namespace: str, event: Obj) -> Obj:
        """POST a core/v1 Event (see :func:`.events.record_event`)."""
        raise NotImplementedError

    def list_with_version(self, kind: str, node_name: Optional[str] = None) -> Tuple[List[Obj], str]:
        """(items, list resourceVersion) of ``kind`` in {"Node", "Pod"}: one unpaginated LIST."""
        raise NotImplementedError

    # coordination.k8s.io/v1 Lease: the extender's per-node allocation ledger lives in one Lease per node
    # in its own namespace (extender/ledger.py), so the extender needs no write access to Node objects
    def get_lease(self, namespace: str, name: str) -> Obj:
        raise NotImplementedError

    def create_lease(self, namespace: str, lease: Obj) -> Obj:
        """Create a Lease; 409 Conflict (AlreadyExists) when one of that name exists."""
        raise NotImplementedError

    def patch_lease(self, namespace: str, name: str, annotations: Dict[str, Optional[str]],
                    resource_version: Optional[str] = None) -> Obj:
        """Merge-patch a Lease's annotations; with ``resource_version`` conditional (409 on mismatch)."""
        raise NotImplementedError

    def list_page(self, kind: str, limit: int = 0, continue_token: str = "", resource_version: Optional[str] = None,
                  field_selector: Optional[str] = None, namespace: Optional[str] = None) -> Tuple[List[Obj], str, str]:
        """One page of a LIST of ``kind``: (items, list resourceVersion, continue token or "").
        ``resource_version="0"`` lets the apiserver answer from its watch cache (no etcd quorum read,
        possibly a little stale; older apiservers then ignore ``limit``); ``None`` is a consistent
        read.  Pages after the first pass only ``continue_token``.  An expired continue token raises
        :class:`Gone`."""
        raise NotImplementedError

    def watch_stream(self, kind: str, resource_version: str, timeout: float = 60.0,
                     stop: Optional[threading.Event] = None, field_selector: Optional[str] = None,
                     namespace: Optional[str] = None) -> Iterator[Tuple[str, Obj]]:
        """(event type, object) after ``resource_version`` until ``timeout``: the WATCH half.  With a
        ``field_selector`` an object that stops matching arrives as DELETED.  ``namespace``: for the
        namespaced kinds (Lease), that namespace only."""
        raise NotImplementedError


def _selector_q(label_selector: Optional[str]) -> str:
    return f"?labelSelector={quote(label_selector)}" if label_selector else ""


class RestKubeAPI(KubeAPI):
    """Minimal REST client (``requests``): JSON merge patches, pods/binding subresource."""

    SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"

    #: projected service-account tokens rotate (the kubelet rewrites the file well before expiry):
    #: a long-running daemon re-reads the file at most this often, and immediately after a 401
    TOKEN_REFRESH_S = 60.0

    def __init__(self, base_url: str, token: Optional[str] = None, ca_file: Optional[str] = None, verify: bool = True,
                 timeout: float = 10.0, token_file: Optional[str] = None):
        import requests

        self.base = base_url.rstrip("/")
        self.timeout = timeout
        self._local = threading.local()
        self._requests = requests
        self._headers = {"Accept": "application/json"}
        self._token_file = token_file
        self._token = token or ""
        self._token_read = time.monotonic()
        self._verify = ca_file if (verify and ca_file) else verify

    @classmethod
    def in_cluster(cls) -> "RestKubeAPI":
        host, port = os.environ.get("KUBERNETES_SERVICE_HOST"), os.environ.get("KUBERNETES_SERVICE_PORT", "443")
        if not host:
            raise RuntimeError("not running in a cluster (KUBERNETES_SERVICE_HOST unset); pass --apiserver")
        tf = os.path.join(cls.SA_DIR, "token")
        with open(tf) as f:
            token = f.read().strip()
        if ":" in host and not host.startswith("["):
            host = f"[{host}]"
        return cls(f"https://{host}:{port}", token=token, ca_file=os.path.join(cls.SA_DIR, "ca.crt"), token_file=tf)

    def _bearer(self, force: bool = False) -> str:
        """The current token, re-read from ``token_file`` when stale (or ``force``: after a 401)."""
        if self._token_file and (force or time.monotonic() - self._token_read > self.TOKEN_REFRESH_S):
            try:
                with open(self._token_file) as f:
                    self._token = f.read().strip()
            except OSError as e:
                log.warning("re-reading %s failed: %s", self._token_file, e)
            self._token_read = time.monotonic()
        return self._token

    def _auth(self, force: bool = False) -> Dict[str, str]:
        tok = self._bearer(force)
        return {"Authorization": f"Bearer {tok}"} if tok else {}

    def _session(self):
        s = getattr(self._local, "s", None)
        if s is None:
            s = self._requests.Session()
            s.headers.update(self._headers)
            self._local.s = s
        return s

    def _do(self, method: str, path: str, body: Any = None, content_type: str = "application/json") -> Obj:
        headers = self._auth()
        data = None
        if body is not None:
            headers["Content-Type"] = content_type
            data = json.dumps(body)
        r = self._session().request(method, self.base + path, data=data, headers=headers, timeout=self.timeout, verify=self._verify)
        if r.status_code == 401 and self._token_file:  # rotated token: re-read once and retry
            headers.update(self._auth(force=True))
            r = self._session().request(method, self.base + path, data=data, headers=headers, timeout=self.timeout,
                                        verify=self._verify)
        if r.status_code >= 400:
            try:
                msg = r.json().get("message", r.text)
            except ValueError:
                msg = r.text
            raise_for(r.status_code, msg)
        return r.json() if r.content else {}

    def get_node(self, name: str) -> Obj:
        return self._do("GET", f"/api/v1/nodes/{quote(name)}")

    def list_nodes(self, label_selector: Optional[str] = None) -> List[Obj]:
        return self._do("GET", "/api/v1/nodes" + _selector_q(label_selector)).get("items", [])

    def patch_node(self, name, annotations=None, labels=None, resource_version=None) -> Obj:
        md: Obj = {}
        if annotations is not None:
            md["annotations"] = annotations
        if labels is not None:
            md["labels"] = labels
        if resource_version is not None:  # the apiserver enforces it as a precondition (409 Conflict)
            md["resourceVersion"] = str(resource_version)
        return self._do("PATCH", f"/api/v1/nodes/{quote(name)}", {"metadata": md}, "application/merge-patch+json")

    def get_pod(self, namespace: str, name: str) -> Obj:
        return self._do("GET", f"/api/v1/namespaces/{quote(namespace)}/pods/{quote(name)}")

    def list_pods(self, node_name: Optional[str] = None, namespace: Optional[str] = None, cached: bool = False,
                  not_older_than: Optional[str] = None) -> List[Obj]:
        path = f"/api/v1/namespaces/{quote(namespace)}/pods" if namespace else "/api/v1/pods"
        q = ([f"fieldSelector={quote(f'spec.nodeName={node_name}')}"] if node_name else []) + (["resourceVersion=0"] if cached else [])
        if not_older_than and not cached:
            q += [f"resourceVersion={quote(str(not_older_than))}", "resourceVersionMatch=NotOlderThan"]
        return self._do("GET", path + ("?" + "&".join(q) if q else "")).get("items", [])

    def patch_pod_annotations(self, namespace, name, annotations, resource_version=None) -> Obj:
        md: Obj = {"annotations": annotations}
        if resource_version is not None:
            md["resourceVersion"] = str(resource_version)
        return self._do("PATCH", f"/api/v1/namespaces/{quote(namespace)}/pods/{quote(name)}", {"metadata": md},
                        "application/merge-patch+json")

    def bind_pod(self, namespace: str, name: str, uid: str, node: str) -> None:
        body = {
            "apiVersion": "v1",
            "kind": "Binding",
            "metadata": {"name": name, "namespace": namespace, **({"uid": uid} if uid else {})},
            "target": {"apiVersion": "v1", "kind": "Node", "name": node},
        }
        self._do("POST", f"/api/v1/namespaces/{quote(namespace)}/pods/{quote(name)}/binding", body)

    def create_event(self, namespace: str, event: Obj) -> Obj:
        return self._do("POST", f"/api/v1/namespaces/{quote(namespace)}/events", event)

    _KIND_PATH = {"Node": "/api/v1/nodes", "Pod": "/api/v1/pods"}

    @staticmethod
    def _lease_path(namespace: str, name: str = "") -> str:
        p = f"/apis/coordination.k8s.io/v1/namespaces/{quote(namespace)}/leases"
        return p + (f"/{quote(name)}" if name else "")

    def _kind_path(self, kind: str, namespace: Optional[str]) -> str:
        if kind == "Lease":
            return self._lease_path(namespace or "default")
        return self._KIND_PATH[kind]

    def get_lease(self, namespace, name):
        return self._do("GET", self._lease_path(namespace, name))

    def create_lease(self, namespace, lease):
        return self._do("POST", self._lease_path(namespace), lease)

    def patch_lease(self, namespace, name, annotations, resource_version=None):
        md: Obj = {"annotations": annotations}
        if resource_version is not None:
            md["resourceVersion"] = str(resource_version)
        return self._do("PATCH", self._lease_path(namespace, name), {"metadata": md}, "application/merge-patch+json")

    def list_with_version(self, kind: str, node_name: Optional[str] = None) -> Tuple[List[Obj], str]:
        path = self._KIND_PATH[kind]
        if node_name and kind == "Pod":
            path += "?fieldSelector=" + quote(f"spec.nodeName={node_name}")
        d = self._do("GET", path)
        return d.get("items", []), str((d.get("metadata") or {}).get("resourceVersion", ""))

    def list_page(self, kind, limit=0, continue_token="", resource_version=None, field_selector=None, namespace=None):
        q = []
        if limit:
            q.append(f"limit={int(limit)}")
        if continue_token:
            q.append("continue=" + quote(continue_token))
        elif resource_version is not None:
            q.append("resourceVersion=" + quote(str(resource_version)))
        if field_selector:
            q.append("fieldSelector=" + quote(field_selector))
        d = self._do("GET", self._kind_path(kind, namespace) + ("?" + "&".join(q) if q else ""))
        md = d.get("metadata") or {}
        return d.get("items", []), str(md.get("resourceVersion", "")), str(md.get("continue") or "")

    def watch_stream(self, kind: str, resource_version: str, timeout: float = 60.0,
                     stop: Optional[threading.Event] = None, field_selector: Optional[str] = None,
                     namespace: Optional[str] = None) -> Iterator[Tuple[str, Obj]]:
        """``GET {path}?watch=1&resourceVersion=..&timeoutSeconds=..&allowWatchBookmarks=true`` read
        line by line; BOOKMARKs are yielded (they carry only a resourceVersion), an ERROR 410 raises
        :class:`Gone`."""
        url = (f"{self.base}{self._kind_path(kind, namespace)}?watch=1&allowWatchBookmarks=true"
               f"&resourceVersion={quote(str(resource_version))}&timeoutSeconds={int(max(1, timeout))}")
        if field_selector:
            url += "&fieldSelector=" + quote(field_selector)
        with self._session().get(url, stream=True, timeout=(self.timeout, timeout + 30), verify=self._verify,
                                 headers=self._auth()) as r:
            if r.status_code >= 400:
                raise_for(r.status_code, r.text[:300])
            for line in r.iter_lines():
                if stop is not None and stop.is_set():
                    return
                if not line:
                    continue
                ev = json.loads(line)
                t, obj = ev.get("type", ""), ev.get("object") or {}
                if t == "ERROR":
                    raise_for(int(obj.get("code", 500)), str(obj.get("message", "watch error")))
                yield t, obj
