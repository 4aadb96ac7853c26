"""In-memory Kubernetes apiserver (same :class:`~.api.KubeAPI` surface) with fault injection.

Used by the test-suite and by the in-process cluster simulation (``sim/``) because this
environment has no kind/kubectl/docker.  Semantics that matter for
correctness are modelled: ``resourceVersion`` bumps on every write, conditional patches return
409, binding a pod that already has a node returns 409, JSON merge patch (``None`` deletes), and
watchers get ADDED/MODIFIED/DELETED events.  :meth:`FakeAPIServer.inject` makes the next N calls of
an operation fail with a given HTTP code (apiserver 409/500).

:func:`serve_http` exposes the fake over the REST paths :class:`~.api.RestKubeAPI` uses, so the REST
client is tested on the wire as well.
"""
from __future__ import annotations

import copy
import json
import threading
import time
import uuid
from collections import OrderedDict, defaultdict, deque
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Callable, Dict, Iterator, List, Optional, Tuple
from urllib.parse import parse_qs, unquote, urlparse

from .api import ApiError, Conflict, Gone, KubeAPI, NotFound, raise_for
from .objects import match_fields, meta

__all__ = ["FakeAPIServer", "serve_http"]

Obj = Dict[str, Any]
Watcher = Callable[[str, str, Obj], None]  # (event, kind, object)


def _merge(dst: Obj, patch: Obj) -> Obj:
    """RFC 7386 JSON merge patch."""
    for k, v in patch.items():
        if v is None:
            dst.pop(k, None)
        elif isinstance(v, dict) and isinstance(dst.get(k), dict):
            _merge(dst[k], v)
        else:
            dst[k] = copy.deepcopy(v)
    return dst


def _match_labels(obj: Obj, selector: Optional[str]) -> bool:
    if not selector:
        return True
    lb = meta(obj).get("labels") or {}
    for term in selector.split(","):
        term = term.strip()
        if not term:
            continue
        if "!=" in term:
            k, v = term.split("!=", 1)
            if lb.get(k.strip()) == v.strip():
                return False
        elif "=" in term:
            k, v = term.split("=", 1)
            if lb.get(k.strip().rstrip("=")) != v.strip().lstrip("="):
                return False
        elif lb.get(term) is None:
            return False
    return True


class FakeAPIServer(KubeAPI):
    def __init__(self, history: int = 100_000):
        self._lock = threading.RLock()
        self._changed = threading.Condition(self._lock)
        self._rv = 0
        self.nodes: Dict[str, Obj] = {}
        self.pods: Dict[Tuple[str, str], Obj] = {}
        self.leases: Dict[Tuple[str, str], Obj] = {}  # coordination.k8s.io/v1 Leases by (namespace, name)
        self.events: List[Obj] = []
        self._faults: Dict[str, List[Tuple[int, int]]] = defaultdict(list)  # op -> [(code, remaining)]
        self._watchers: List[Watcher] = []
        # watch cache: (rv, type, kind, object) of every change; a watch older than the window gets 410
        self._history: "deque[Tuple[int, str, str, Obj]]" = deque(maxlen=history)
        self.calls: Dict[str, int] = defaultdict(int)
        self.latency_s = 0.0
        # paginated LISTs (list_page): the rest of a LIST, serialized at the LIST's resourceVersion,
        # by continue token; the oldest are dropped (their tokens then answer 410, as after etcd
        # compaction).  ``watch_cache_pages``: whether a resourceVersion=0 LIST (served from the watch
        # cache) honours ``limit`` — apiservers before the paginated watch cache ignore it
        self._pages: "OrderedDict[str, Tuple[List[str], str]]" = OrderedDict()
        self.max_open_lists = 64
        self.watch_cache_pages = False
        self.bytes_served: Dict[str, int] = defaultdict(int)  # kind -> JSON bytes of LIST responses
        self.list_requests: Dict[str, int] = defaultdict(int)  # kind -> LIST requests (pages)
        self.cache_reads: Dict[str, int] = defaultdict(int)  # kind -> LISTs served from the watch cache (resourceVersion=0)
        self.min_rv_reads: Dict[str, int] = defaultdict(int)  # kind -> watch-cache LISTs with resourceVersionMatch=NotOlderThan
        self._watch_cuts: Dict[str, List[int]] = defaultdict(list)  # kind -> cut the next watch after n events
        self._open_watches: Dict[str, Dict[int, List[Optional[int]]]] = defaultdict(dict)  # kind -> id -> [cut]
        self._watch_ids = 0

    # ------------------------------------------------------------------ infrastructure
    def _next_rv(self) -> str:
        self._rv += 1
        return str(self._rv)

    def inject(self, op: str, code: int = 500, times: int = 1) -> None:
        """Make the next ``times`` calls of ``op`` (method name, e.g. ``bind_pod``) fail with ``code``."""
        with self._lock:
            self._faults[op].append((code, times))

    def _enter(self, op: str) -> None:
        self.calls[op] += 1
        if self.latency_s:
            time.sleep(self.latency_s)
        q = self._faults.get(op)
        if q:
            code, left = q[0]
            if left <= 1:
                q.pop(0)
            else:
                q[0] = (code, left - 1)
            raise_for(code, f"injected fault on {op}")

    def watch(self, fn: Watcher) -> None:
        with self._lock:
            self._watchers.append(fn)

    def _emit(self, event: str, kind: str, obj: Obj) -> None:
        self._history.append((int(meta(obj).get("resourceVersion") or self._rv), event, kind, copy.deepcopy(obj)))
        self._changed.notify_all()
        for w in list(self._watchers):
            w(event, kind, copy.deepcopy(obj))

    # ------------------------------------------------------------------ LIST+WATCH (informers)
    def list_with_version(self, kind: str, node_name: Optional[str] = None) -> Tuple[List[Obj], str]:
        """(items, list resourceVersion): what ``GET /api/v1/{nodes,pods}`` returns."""
        items, rv, _ = self.list_page(kind, field_selector=f"spec.nodeName={node_name}" if node_name and kind == "Pod" else None)
        return items, rv

    def list_page(self, kind, limit=0, continue_token="", resource_version=None, field_selector=None, namespace=None):
        """One page of a LIST (``GET ...?limit=&continue=&resourceVersion=&fieldSelector=``).  The
        whole LIST is serialized at its resourceVersion on the first page (a consistent snapshot, as
        the apiserver reads etcd at one revision); later pages are served from it."""
        with self._lock:
            self._enter({"Node": "list_nodes", "Pod": "list_pods"}.get(kind, f"list_{kind}"))
            if continue_token:
                if resource_version not in (None, ""):  # as the apiserver's validation answers
                    raise ApiError(400, "specifying resource version is not allowed when using continue")
                snap = self._pages.pop(continue_token, None)
                if snap is None:
                    raise Gone("the provided continue parameter is too old")
                encoded, list_rv = snap
            else:
                src = {"Node": self.nodes, "Pod": self.pods, "Lease": self.leases}[kind]
                encoded = [json.dumps(o) for _, o in sorted(src.items()) if match_fields(o, field_selector)
                           and (namespace is None or meta(o).get("namespace") == namespace)]
                list_rv = str(self._rv)
                if str(resource_version) == "0":
                    self.cache_reads[kind] += 1
                    if not self.watch_cache_pages:
                        limit = 0
            page, rest = (encoded[:limit], encoded[limit:]) if limit else (encoded, [])
            token = ""
            if rest:
                token = uuid.uuid4().hex
                self._pages[token] = (rest, list_rv)
                while len(self._pages) > self.max_open_lists:
                    self._pages.popitem(last=False)
            self.list_requests[kind] += 1
            self.bytes_served[kind] += sum(len(e) for e in page)
        return [json.loads(e) for e in page], list_rv, token

    def expire_continue_tokens(self) -> None:
        """Every open paginated LIST loses its snapshot (etcd compaction): the next page answers 410."""
        with self._lock:
            self._pages.clear()

    def cut_watch(self, kind: str, after: int = 0) -> None:
        """Every watch of ``kind`` open now (or, with none open, the next one) breaks — a connection
        reset — after delivering ``after`` more events."""
        with self._lock:
            if self._open_watches.get(kind):
                for slot in self._open_watches[kind].values():
                    slot[0] = after
            else:
                self._watch_cuts[kind].append(after)

    def watch_stream(self, kind: str, resource_version: str, timeout: float = 60.0,
                     stop: Optional[threading.Event] = None, field_selector: Optional[str] = None,
                     namespace: Optional[str] = None) -> Iterator[Tuple[str, Obj]]:
        """Changes of ``kind`` after ``resource_version``, blocking up to ``timeout`` s for new ones
        (``GET ...?watch=1``).  Raises :class:`Gone` when the window no longer reaches back that far.
        With ``field_selector``, a change to an object that does not match is delivered as DELETED
        (the object left the selection) and an ADDED one is not delivered."""
        with self._lock:
            self._enter(f"watch_{kind}")
            if self._history and int(resource_version or 0) < self._history[0][0] - 1 \
                    and len(self._history) == self._history.maxlen:
                raise Gone(f"resourceVersion {resource_version} is too old")
            self._watch_ids += 1
            wid, slot = self._watch_ids, [self._watch_cuts[kind].pop(0) if self._watch_cuts.get(kind) else None]
            self._open_watches[kind][wid] = slot
        try:
            yield from self._watch_events(kind, int(resource_version or 0), time.monotonic() + timeout, stop, field_selector,
                                          namespace, slot)
        finally:
            with self._lock:
                self._open_watches[kind].pop(wid, None)

    def _watch_events(self, kind, since, deadline, stop, field_selector, namespace, slot):
        cut: Optional[int] = None
        sent = 0
        while stop is None or not stop.is_set():
            with self._lock:
                if cut is None and slot[0] is not None:  # a cut requested while this watch is open
                    cut = sent + slot[0]
                batch = [(t, o) for rv, t, k, o in self._history if rv > since and k == kind
                         and (namespace is None or meta(o).get("namespace") == namespace)]
                if self._history:
                    since = max(since, self._history[-1][0])
                if not batch:
                    left = deadline - time.monotonic()
                    if left <= 0:
                        return
                    self._changed.wait(min(left, 0.25))
                    continue
            for t, o in batch:
                if field_selector and not match_fields(o, field_selector):
                    if t == "ADDED":
                        continue
                    t = "DELETED"
                if cut is not None and sent >= cut:
                    raise ConnectionResetError(f"watch of {kind} cut after {sent} events (injected)")
                sent += 1
                yield t, copy.deepcopy(o)

    def create_event(self, namespace: str, event: Obj) -> Obj:
        with self._lock:
            self._enter("create_event")
            ev = copy.deepcopy(event)
            meta(ev).setdefault("namespace", namespace)
            meta(ev)["resourceVersion"] = self._next_rv()
            self.events.append(ev)
            return copy.deepcopy(ev)

    # ------------------------------------------------------------------ object creation (tests/sim)
    def create_node(self, node: Obj) -> Obj:
        with self._lock:
            node = copy.deepcopy(node)
            md = meta(node)
            md.setdefault("uid", str(uuid.uuid4()))
            md["resourceVersion"] = self._next_rv()
            self.nodes[md["name"]] = node
            self._emit("ADDED", "Node", node)
            return copy.deepcopy(node)

    def create_pod(self, pod: Obj) -> Obj:
        with self._lock:
            pod = copy.deepcopy(pod)
            md = meta(pod)
            md.setdefault("namespace", "default")
            md.setdefault("uid", str(uuid.uuid4()))
            md.setdefault("creationTimestamp", time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()))
            key = (md["namespace"], md["name"])
            if key in self.pods:
                raise Conflict(f"pod {key} exists")
            md["resourceVersion"] = self._next_rv()
            self.pods[key] = pod
            self._emit("ADDED", "Pod", pod)
            return copy.deepcopy(pod)

    def delete_pod(self, namespace: str, name: str) -> None:
        with self._lock:
            pod = self.pods.pop((namespace, name), None)
            if pod is None:
                raise NotFound(f"pod {namespace}/{name}")
            meta(pod)["resourceVersion"] = self._next_rv()
            self._emit("DELETED", "Pod", pod)

    def set_pod_phase(self, namespace: str, name: str, phase: str, reason: str = "", message: str = "") -> Obj:
        with self._lock:
            pod = self._pod(namespace, name)
            st = pod.setdefault("status", {})
            st["phase"] = phase
            if reason:  # e.g. the kubelet's UnexpectedAdmissionError
                st["reason"], st["message"] = reason, message
            meta(pod)["resourceVersion"] = self._next_rv()
            self._emit("MODIFIED", "Pod", pod)
            return copy.deepcopy(pod)

    def update_node_status(self, name: str, capacity: Dict[str, str], allocatable: Optional[Dict[str, str]] = None) -> Obj:
        """What the kubelet does after ListAndWatch (diagram step 2)."""
        with self._lock:
            node = self._node(name)
            st = node.setdefault("status", {})
            st.setdefault("capacity", {}).update(capacity)
            st.setdefault("allocatable", {}).update(allocatable if allocatable is not None else capacity)
            meta(node)["resourceVersion"] = self._next_rv()
            self._emit("MODIFIED", "Node", node)
            return copy.deepcopy(node)

    # ------------------------------------------------------------------ KubeAPI
    def _node(self, name: str) -> Obj:
        n = self.nodes.get(name)
        if n is None:
            raise NotFound(f"node {name}")
        return n

    def _pod(self, namespace: str, name: str) -> Obj:
        p = self.pods.get((namespace, name))
        if p is None:
            raise NotFound(f"pod {namespace}/{name}")
        return p

    def get_node(self, name: str) -> Obj:
        with self._lock:
            self._enter("get_node")
            return copy.deepcopy(self._node(name))

    def list_nodes(self, label_selector: Optional[str] = None) -> List[Obj]:
        with self._lock:
            self._enter("list_nodes")
            return [copy.deepcopy(n) for n in self.nodes.values() if _match_labels(n, label_selector)]

    def patch_node(self, name, annotations=None, labels=None, resource_version=None) -> Obj:
        with self._lock:
            self._enter("patch_node")
            node = self._node(name)
            if resource_version is not None and str(resource_version) != meta(node).get("resourceVersion"):
                raise Conflict(f"node {name}: resourceVersion {resource_version} is stale")
            md: Obj = {}
            if annotations is not None:
                md["annotations"] = annotations
            if labels is not None:
                md["labels"] = labels
            _merge(node, {"metadata": md})
            meta(node)["resourceVersion"] = self._next_rv()
            self._emit("MODIFIED", "Node", node)
            return copy.deepcopy(node)

    def get_pod(self, namespace: str, name: str) -> Obj:
        with self._lock:
            self._enter("get_pod")
            return copy.deepcopy(self._pod(namespace, name))

    def list_pods(self, node_name: Optional[str] = None, namespace: Optional[str] = None, cached: bool = False,
                  not_older_than: Optional[str] = None) -> List[Obj]:
        with self._lock:
            self._enter("list_pods")
            if not_older_than is not None:
                if int(not_older_than) > self._rv:  # the apiserver waits ~3 s for its cache, then gives up
                    raise ApiError(504, f"Timeout: Too large resource version: {not_older_than}, current: {self._rv}")
                self.min_rv_reads["Pod"] += 1
            if cached:
                self.cache_reads["Pod"] += 1
            out = []
            for (ns, _), p in self.pods.items():
                if namespace and ns != namespace:
                    continue
                if node_name is not None and (p.get("spec") or {}).get("nodeName", "") != node_name:
                    continue
                out.append(copy.deepcopy(p))
            return out

    def patch_pod_annotations(self, namespace, name, annotations, resource_version=None) -> Obj:
        with self._lock:
            self._enter("patch_pod_annotations")
            pod = self._pod(namespace, name)
            if resource_version is not None and str(resource_version) != meta(pod).get("resourceVersion"):
                raise Conflict(f"pod {namespace}/{name}: resourceVersion {resource_version} is stale")
            _merge(pod, {"metadata": {"annotations": annotations}})
            meta(pod)["resourceVersion"] = self._next_rv()
            self._emit("MODIFIED", "Pod", pod)
            return copy.deepcopy(pod)

    def get_lease(self, namespace: str, name: str) -> Obj:
        with self._lock:
            self._enter("get_lease")
            lease = self.leases.get((namespace, name))
            if lease is None:
                raise NotFound(f"lease {namespace}/{name}")
            return copy.deepcopy(lease)

    def create_lease(self, namespace: str, lease: Obj) -> Obj:
        with self._lock:
            self._enter("create_lease")
            lease = copy.deepcopy(lease)
            md = meta(lease)
            md["namespace"] = namespace
            key = (namespace, md["name"])
            if key in self.leases:
                raise Conflict(f"leases.coordination.k8s.io \"{md['name']}\" already exists")
            lease.setdefault("apiVersion", "coordination.k8s.io/v1")
            lease.setdefault("kind", "Lease")
            md.setdefault("uid", str(uuid.uuid4()))
            md["resourceVersion"] = self._next_rv()
            self.leases[key] = lease
            self._emit("ADDED", "Lease", lease)
            return copy.deepcopy(lease)

    def patch_lease(self, namespace, name, annotations, resource_version=None) -> Obj:
        with self._lock:
            self._enter("patch_lease")
            lease = self.leases.get((namespace, name))
            if lease is None:
                raise NotFound(f"lease {namespace}/{name}")
            if resource_version is not None and str(resource_version) != meta(lease).get("resourceVersion"):
                raise Conflict(f"lease {namespace}/{name}: resourceVersion {resource_version} is stale")
            _merge(lease, {"metadata": {"annotations": annotations}})
            meta(lease)["resourceVersion"] = self._next_rv()
            self._emit("MODIFIED", "Lease", lease)
            return copy.deepcopy(lease)

    def bind_pod(self, namespace: str, name: str, uid: str, node: str) -> None:
        with self._lock:
            self._enter("bind_pod")
            pod = self._pod(namespace, name)
            if uid and meta(pod).get("uid") != uid:
                raise Conflict(f"pod {namespace}/{name}: uid mismatch")
            if (pod.get("spec") or {}).get("nodeName"):
                raise Conflict(f"pod {namespace}/{name} is already assigned to node {pod['spec']['nodeName']}")
            self._node(node)
            pod.setdefault("spec", {})["nodeName"] = node
            pod.setdefault("status", {})["phase"] = "Pending"
            meta(pod)["resourceVersion"] = self._next_rv()
            self._emit("MODIFIED", "Pod", pod)


# ---------------------------------------------------------------------------------------- HTTP
class _Handler(BaseHTTPRequestHandler):
    api: FakeAPIServer = None  # type: ignore[assignment]
    token: Optional[str] = None
    # HTTP/1.1 as the apiserver speaks it: keep-alive, and watches streamed with chunked encoding (a
    # client reading an unframed HTTP/1.0 body buffers events until its read size fills)
    protocol_version = "HTTP/1.1"

    def log_message(self, *a):  # quiet
        pass

    def _send(self, code: int, body: Obj) -> None:
        data = json.dumps(body).encode()
        self.send_response(code)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)

    def _body(self) -> Obj:
        n = int(self.headers.get("Content-Length") or 0)
        return json.loads(self.rfile.read(n) or b"{}")

    def _route(self, method: str) -> None:
        if self.token and self.headers.get("Authorization") != f"Bearer {self.token}":
            return self._send(401, {"kind": "Status", "code": 401, "message": "Unauthorized"})
        u = urlparse(self.path)
        parts = [unquote(p) for p in u.path.strip("/").split("/")]
        q = parse_qs(u.query)
        try:
            if parts[:4] == ["apis", "coordination.k8s.io", "v1", "namespaces"] and len(parts) >= 6 and parts[5] == "leases":
                return self._lease_route(method, parts[4], parts[6] if len(parts) > 6 else "", q)
            if parts[:2] != ["api", "v1"]:
                raise NotFound(u.path)
            rest = parts[2:]
            watch = (q.get("watch") or ["0"])[0] in ("1", "true")
            fs = (q.get("fieldSelector") or [""])[0]
            if rest in (["nodes"], ["pods"]) and method == "GET" and watch:
                return self._watch("Node" if rest == ["nodes"] else "Pod", (q.get("resourceVersion") or ["0"])[0],
                                   float((q.get("timeoutSeconds") or ["60"])[0]), fs or None)
            if rest == ["pods"] and method == "GET" and (q.get("resourceVersionMatch") or [""])[0] == "NotOlderThan":
                node_name = fs.split("=", 1)[1] if fs.startswith("spec.nodeName=") else None
                items = self.api.list_pods(node_name=node_name, not_older_than=(q.get("resourceVersion") or ["0"])[0])
                return self._send(200, {"kind": "PodList", "metadata": {"resourceVersion": str(self.api._rv)}, "items": items})
            if rest in (["nodes"], ["pods"]) and method == "GET":
                kind = "Node" if rest == ["nodes"] else "Pod"
                items, rv, cont = self.api.list_page(kind, int((q.get("limit") or ["0"])[0]), (q.get("continue") or [""])[0],
                                                     (q.get("resourceVersion") or [None])[0], fs or None)
                md = {"resourceVersion": rv, **({"continue": cont} if cont else {})}
                return self._send(200, {"kind": f"{kind}List", "metadata": md, "items": items})
            if len(rest) == 2 and rest[0] == "nodes":
                if method == "GET":
                    return self._send(200, self.api.get_node(rest[1]))
                if method == "PATCH":
                    md = self._body().get("metadata", {})
                    return self._send(200, self.api.patch_node(rest[1], md.get("annotations"), md.get("labels"),
                                                               md.get("resourceVersion")))
            node_name = None
            if fs.startswith("spec.nodeName="):
                node_name = fs.split("=", 1)[1]
            if len(rest) == 3 and rest[0] == "namespaces" and rest[2] == "events" and method == "POST":
                return self._send(201, self.api.create_event(rest[1], self._body()))
            if len(rest) >= 3 and rest[0] == "namespaces" and rest[2] == "pods":
                ns = rest[1]
                if len(rest) == 3 and method == "GET":
                    return self._send(200, {"kind": "PodList", "items": self.api.list_pods(
                        node_name=node_name, namespace=ns, cached=(q.get("resourceVersion") or [""])[0] == "0")})
                if len(rest) == 4:
                    if method == "GET":
                        return self._send(200, self.api.get_pod(ns, rest[3]))
                    if method == "PATCH":
                        md = self._body().get("metadata", {})
                        return self._send(200, self.api.patch_pod_annotations(ns, rest[3], md.get("annotations") or {},
                                                                            md.get("resourceVersion")))
                if len(rest) == 5 and rest[4] == "binding" and method == "POST":
                    b = self._body()
                    self.api.bind_pod(ns, rest[3], (b.get("metadata") or {}).get("uid", ""), b["target"]["name"])
                    return self._send(201, {"kind": "Status", "status": "Success", "code": 201})
            raise NotFound(f"{method} {u.path}")
        except ApiError as e:
            return self._send(e.code, {"kind": "Status", "status": "Failure", "code": e.code, "message": e.message})

    def _lease_route(self, method: str, ns: str, name: str, q: Dict[str, List[str]]) -> None:
        if not name and method == "GET":
            if (q.get("watch") or ["0"])[0] in ("1", "true"):
                return self._watch("Lease", (q.get("resourceVersion") or ["0"])[0], float((q.get("timeoutSeconds") or ["60"])[0]),
                                   namespace=ns)
            items, rv, cont = self.api.list_page("Lease", int((q.get("limit") or ["0"])[0]), (q.get("continue") or [""])[0],
                                                 (q.get("resourceVersion") or [None])[0], namespace=ns)
            return self._send(200, {"kind": "LeaseList", "metadata": {"resourceVersion": rv, **({"continue": cont} if cont else {})},
                                    "items": items})
        if not name and method == "POST":
            return self._send(201, self.api.create_lease(ns, self._body()))
        if name and method == "GET":
            return self._send(200, self.api.get_lease(ns, name))
        if name and method == "PATCH":
            md = self._body().get("metadata", {})
            return self._send(200, self.api.patch_lease(ns, name, md.get("annotations") or {}, md.get("resourceVersion")))
        raise NotFound(f"{method} leases/{name}")

    def _chunk(self, data: bytes) -> None:
        self.wfile.write(f"{len(data):x}\r\n".encode() + data + b"\r\n")
        self.wfile.flush()

    def _watch(self, kind: str, rv: str, timeout: float, field_selector: Optional[str] = None,
               namespace: Optional[str] = None) -> None:
        """Watch response: one JSON ``{"type", "object"}`` line per chunk (chunked transfer encoding,
        as the apiserver streams it) until ``timeoutSeconds``.  An injected cut drops the connection
        without the final chunk (the client sees a broken stream)."""
        try:
            stream = self.api.watch_stream(kind, rv, timeout, field_selector=field_selector, namespace=namespace)
            first = next(stream, None)
        except Gone as e:
            return self._send(200, {"type": "ERROR", "object": {"kind": "Status", "code": 410, "reason": "Expired",
                                                                "message": e.message}})
        except ConnectionResetError:
            self.close_connection = True
            return
        self.send_response(200)
        self.send_header("Content-Type", "application/json")
        self.send_header("Transfer-Encoding", "chunked")
        self.end_headers()
        try:
            if first is not None:
                self._chunk((json.dumps({"type": first[0], "object": first[1]}) + "\n").encode())
                for t, o in stream:
                    self._chunk((json.dumps({"type": t, "object": o}) + "\n").encode())
            self.wfile.write(b"0\r\n\r\n")
            self.wfile.flush()
        except (BrokenPipeError, ConnectionResetError):
            self.close_connection = True

    def do_GET(self):
        self._route("GET")

    def do_PATCH(self):
        self._route("PATCH")

    def do_POST(self):
        self._route("POST")


def serve_http(api: FakeAPIServer, host: str = "127.0.0.1", port: int = 0, token: Optional[str] = None):
    """Serve ``api`` over HTTP in a daemon thread; returns ``(server, base_url)``.  ``server.shutdown()`` stops it."""
    handler = type("FakeKubeHandler", (_Handler,), {"api": api, "token": token})
    srv = ThreadingHTTPServer((host, port), handler)
    srv.daemon_threads = True
    t = threading.Thread(target=srv.serve_forever, name="fake-apiserver", daemon=True)
    t.start()
    return srv, f"http://{host}:{srv.server_address[1]}"
