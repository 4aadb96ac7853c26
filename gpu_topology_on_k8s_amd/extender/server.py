"""HTTP front-end of the extender (kube-scheduler extender v1 JSON over aiohttp).

Reference endpoint (``design.md:98-100``): ``http://127.0.0.1:32743/gputopology-scheduler`` with
``/sort`` (prioritize) and ``/bind``.  Served here under the same prefix and port by default:

  POST {prefix}/sort        ExtenderArgs -> HostPriorityList           (reference verb name)
  POST {prefix}/prioritize  alias of /sort
  POST {prefix}/filter      ExtenderArgs -> ExtenderFilterResult       (optional)
  POST {prefix}/bind        ExtenderBindingArgs -> ExtenderBindingResult
  POST {prefix}/preempt     ExtenderPreemptionArgs -> ExtenderPreemptionResult (topology-aware victims)
  GET  {prefix}/healthz, {prefix}/readyz (503 until the informer has synced), /metrics (Prometheus text), /version, /debug/nodes (cache snapshot),
       /defrag?gpus=k (the fewest pod moves after which a k-GPU pod fits well: placement/defrag.py)

kube-scheduler marshals Go structs without json tags, so request keys are capitalised (``Pod``,
``Nodes``, ``NodeNames``, ``PodName`` ...); Go's decoder matches keys case-insensitively, so the
responses use the same capitalised names.  Lower-case request keys are accepted too.
"""
from __future__ import annotations

import asyncio
import json
import logging
from concurrent.futures import ThreadPoolExecutor
from typing import Any, Dict, List, Optional, Tuple

from aiohttp import web

from .. import __version__
from .scheduler import TopologyExtender

log = logging.getLogger(__name__)

__all__ = ["make_app", "run", "DEFAULT_PORT", "DEFAULT_PREFIX"]

DEFAULT_PORT = 32743
DEFAULT_PREFIX = "/gputopology-scheduler"
EXTENDER_KEY = web.AppKey("extender", TopologyExtender)


def _get(d: Any, key: str, default=None):
    if not isinstance(d, dict):
        return default
    if key in d:
        return d[key]
    lk = key.lower()
    for k, v in d.items():
        if k.lower() == lk:
            return v
    return default


def _obj(x: Any) -> Dict[str, Any]:
    """A JSON object from the request, or {} for anything else (null, a list, a scalar)."""
    return x if isinstance(x, dict) else {}


def _candidates(args: Dict[str, Any]) -> Tuple[List[str], Optional[Dict[str, dict]], bool]:
    """(node names, {name: node object} when full nodes were sent, whether NodeNames mode).  Entries
    that are not node names / node objects are dropped: the pod is scored on the rest."""
    names = _get(args, "NodeNames")
    if names is not None:
        return [n for n in (names if isinstance(names, list) else []) if isinstance(n, str) and n], None, True
    items = _get(_obj(_get(args, "Nodes")), "items")
    objs: Dict[str, dict] = {}
    for n in items if isinstance(items, list) else []:
        name = _get(_obj(_get(n, "metadata")), "name")
        if isinstance(name, str) and name:
            objs[name] = n
    return list(objs), objs, False


def make_app(ext: TopologyExtender, prefix: str = DEFAULT_PREFIX, workers: int = 8) -> web.Application:
    pool = ThreadPoolExecutor(max_workers=workers, thread_name_prefix="extender")
    prefix = "/" + prefix.strip("/") if prefix.strip("/") else ""

    async def run_blocking(fn, *a):
        return await asyncio.get_running_loop().run_in_executor(pool, fn, *a)

    async def body(request: web.Request) -> Dict[str, Any]:
        try:
            args = await request.json(loads=json.loads)
        except Exception as e:
            raise web.HTTPBadRequest(text=f"invalid JSON: {e}")
        if not isinstance(args, dict):
            raise web.HTTPBadRequest(text="the extender arguments must be a JSON object")
        return args

    async def prioritize(request: web.Request) -> web.Response:
        args = await body(request)
        pod = _obj(_get(args, "Pod"))
        names, objs, _ = _candidates(args)
        try:
            res = await run_blocking(ext.prioritize, pod, names, objs)
            ext.metrics.request("prioritize", "ok")
        except Exception as e:  # never fail scheduling because of the extender: score 0
            log.exception("prioritize failed")
            ext.metrics.request("prioritize", "error")
            res = [(n, 0) for n in names]
            return web.json_response([{"Host": h, "Score": s} for h, s in res], headers={"X-Extender-Error": str(e)[:200]})
        return web.json_response([{"Host": h, "Score": s} for h, s in res])

    async def filter_(request: web.Request) -> web.Response:
        args = await body(request)
        pod = _obj(_get(args, "Pod"))
        names, objs, names_mode = _candidates(args)
        try:
            ok, failed = await run_blocking(ext.filter, pod, names, objs)
        except Exception as e:
            log.exception("filter failed")
            ext.metrics.request("filter", "error")
            return web.json_response({"Nodes": None, "NodeNames": None, "FailedNodes": {}, "FailedAndUnresolvableNodes": {},
                                      "Error": str(e)})
        ext.metrics.request("filter", "ok")
        out: Dict[str, Any] = {"FailedNodes": failed, "FailedAndUnresolvableNodes": {}, "Error": ""}
        if names_mode:
            out["NodeNames"] = ok
            out["Nodes"] = None
        else:
            out["Nodes"] = {"metadata": {}, "items": [objs[n] for n in ok]}
            out["NodeNames"] = None
        return web.json_response(out)

    async def bind(request: web.Request) -> web.Response:
        args = await body(request)
        try:
            for key in ("PodName", "Node"):
                if not isinstance(_get(args, key), str) or not _get(args, key):
                    raise ValueError(f"ExtenderBindingArgs.{key} must be a non-empty string")
            for key in ("PodNamespace", "PodUID"):
                if not isinstance(_get(args, key, ""), str):
                    raise ValueError(f"ExtenderBindingArgs.{key} must be a string")
            d = await run_blocking(ext.bind, _get(args, "PodNamespace", "default"), _get(args, "PodName"), _get(args, "PodUID", ""),
                                   _get(args, "Node"))
            ext.metrics.request("bind", "ok")
            out = {"Error": ""}
            if d is not None:
                out["Devices"] = list(d.ids)  # extra field, ignored by kube-scheduler
            return web.json_response(out)
        except Exception as e:
            log.warning("bind failed: %s", e)
            ext.metrics.request("bind", "error")
            return web.json_response({"Error": str(e)})

    async def preempt(request: web.Request) -> web.Response:
        args = await body(request)
        pod = _obj(_get(args, "Pod"))
        victims: Dict[str, Tuple[List[str], int]] = {}
        meta_v = _obj(_get(args, "NodeNameToMetaVictims"))
        full_v = _obj(_get(args, "NodeNameToVictims"))
        for node, v in list(full_v.items()) + list(meta_v.items()):
            pods = _get(v, "Pods")
            uids = [str(_get(p, "UID") or _get(_obj(_get(p, "metadata")), "uid", "")) for p in (pods if isinstance(pods, list) else [])]
            try:
                pdb = int(_get(v, "NumPDBViolations", 0) or 0)
            except (TypeError, ValueError):
                pdb = 0
            victims[node] = ([u for u in uids if u and u != "None"], pdb)
        try:
            res = await run_blocking(ext.preempt, pod, victims)
            ext.metrics.request("preempt", "ok")
        except Exception as e:  # the scheduler's own victims stand
            log.exception("preempt failed")
            ext.metrics.request("preempt", "error")
            res = victims
        return web.json_response({"NodeNameToMetaVictims": {
            n: {"Pods": [{"UID": u} for u in uids], "NumPDBViolations": pdb} for n, (uids, pdb) in res.items()}})

    async def healthz(request: web.Request) -> web.Response:
        return web.Response(text="ok")

    async def readyz(request: web.Request) -> web.Response:
        """Ready once the informer has listed the cluster (the DaemonSet's readinessProbe)."""
        if ext.ready:
            return web.Response(text="ok")
        return web.Response(status=503, text=ext.NOT_READY)

    async def metrics(request: web.Request) -> web.Response:
        return web.Response(body=ext.metrics.exposition(), content_type="text/plain", charset="utf-8")

    async def version(request: web.Request) -> web.Response:
        return web.json_response({"version": __version__, "policy": ext.cfg.policy_name, "resource": ext.cfg.contract.resource_name})

    async def defrag(request: web.Request) -> web.Response:
        try:
            k = int(request.query.get("gpus", "8"))
            moves = int(request.query.get("max_moves", "3"))
            min_score = float(request.query.get("min_score", "0"))
        except ValueError:
            return web.json_response({"error": "gpus, max_moves and min_score must be numbers"}, status=400)
        return web.json_response({"gpus": k, "plan": await run_blocking(ext.defrag, k, moves, min_score)})

    async def debug_nodes(request: web.Request) -> web.Response:
        return web.json_response(await run_blocking(ext.cache.snapshot))

    async def on_cleanup(app):
        pool.shutdown(wait=False, cancel_futures=True)

    app = web.Application(client_max_size=64 << 20)
    app.router.add_post(f"{prefix}/sort", prioritize)
    app.router.add_post(f"{prefix}/prioritize", prioritize)
    app.router.add_post(f"{prefix}/filter", filter_)
    app.router.add_post(f"{prefix}/bind", bind)
    app.router.add_post(f"{prefix}/preempt", preempt)
    for p in (f"{prefix}/healthz", "/healthz"):
        app.router.add_get(p, healthz)
    for p in (f"{prefix}/readyz", "/readyz"):
        app.router.add_get(p, readyz)
    app.router.add_get(f"{prefix}/metrics", metrics)
    app.router.add_get("/metrics", metrics)
    app.router.add_get(f"{prefix}/version", version)
    app.router.add_get(f"{prefix}/debug/nodes", debug_nodes)
    app.router.add_get(f"{prefix}/defrag", defrag)
    app.on_cleanup.append(on_cleanup)
    app[EXTENDER_KEY] = ext
    return app


def tls_context(cert_file: str, key_file: str, client_ca: str = ""):
    """Server TLS for the extender; with ``client_ca`` every caller must present a certificate that CA
    signed (mutual TLS: kube-scheduler's extender ``tlsConfig.certFile/keyFile``), which is what makes
    ``/bind`` safe to serve beyond loopback."""
    import ssl

    ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
    ctx.minimum_version = ssl.TLSVersion.TLSv1_2
    ctx.load_cert_chain(cert_file, key_file)
    if client_ca:
        ctx.load_verify_locations(client_ca)
        ctx.verify_mode = ssl.CERT_REQUIRED
    return ctx


def run(ext: TopologyExtender, host: str = "127.0.0.1", port: int = DEFAULT_PORT, prefix: str = DEFAULT_PREFIX,
        resync_period: float = 5.0, ssl_context=None) -> None:
    """Serve until interrupted.  Without an informer the cache is re-listed every ``resync_period``
    seconds off the request path; with one, WATCH events keep it current and nothing polls."""
    app = make_app(ext, prefix)

    async def resync_loop(app):
        async def loop():
            while True:
                if ext.cache.informer is None:
                    try:
                        await asyncio.get_running_loop().run_in_executor(None, ext.cache.sync_all)
                    except Exception as e:
                        log.warning("cache resync failed: %s", e)
                await asyncio.sleep(resync_period)

        task = asyncio.create_task(loop())
        yield
        task.cancel()

    app.cleanup_ctx.append(resync_loop)
    log.info("extender listening on %s://%s:%d%s (policy=%s)", "https" if ssl_context else "http", host, port, prefix,
             ext.cfg.policy_name)
    web.run_app(app, host=host, port=port, access_log=None, print=None, ssl_context=ssl_context)
