"""Scheduler-extender daemon.

    python -m gpu_topology_on_k8s_amd.extender --port 32743 --policy exact

Serves ``/gputopology-scheduler/{sort,prioritize,filter,bind}`` (design.md:98-100) against the
in-cluster apiserver (or ``--apiserver URL``).
"""
from __future__ import annotations

import argparse
import os
import logging
import sys

from ..k8s.annotations import Contract
from ..placement import PlacementPolicy
from .scheduler import ExtenderConfig, TopologyExtender
from .server import DEFAULT_PORT, DEFAULT_PREFIX, run


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--host", default="127.0.0.1",
                    help="listen address; kube-scheduler calls the extender on loopback (design.md:98), and /bind "
                         "is unauthenticated, so do not expose it beyond the node without TLS + auth in front")
    ap.add_argument("--port", type=int, default=DEFAULT_PORT)
    ap.add_argument("--url-prefix", default=DEFAULT_PREFIX)
    ap.add_argument("--resource-name", default="amd.com/gpu", help="extended resource of whole GPUs (or XCP partitions)")
    ap.add_argument("--slice-resource-name", default="amd.com/gpu-slice",
                    help="extended resource of time slices (nodes whose device plugin runs with --time-slices): a separate pool")
    ap.add_argument("--annotation-prefix", default="gputopology.amd.com")
    ap.add_argument("--policy", default="exact", choices=["exact", "gaia", "design"])
    ap.add_argument("--tie-break", default="first", choices=["first", "random"])
    ap.add_argument("--assume-ttl", type=float, default=300.0)
    ap.add_argument("--partition-aware", default="on", choices=["on", "off"],
                    help="CPX/DPX/QPX nodes: group XCPs by physical GPU (on) or treat each as a stand-alone GPU (off)")
    ap.add_argument("--resync", type=float, default=5.0, help="polling period without the informer")
    ap.add_argument("--list-page-size", type=int, default=500,
                    help="informer LIST page size (limit/continue; 0 = one unpaginated LIST)")
    ap.add_argument("--list-from-watch-cache", default="on", choices=["on", "off"],
                    help="first LIST with resourceVersion=0 (served by the apiserver's watch cache, no etcd quorum read)")
    ap.add_argument("--informer", default="on", choices=["on", "off"],
                    help="keep the node/pod view current with LIST+WATCH (on) or by polling every --resync s (off)")
    ap.add_argument("--scheduler-names", default="",
                    help="comma list of spec.schedulerName values whose pods may be bound (empty = any)")
    ap.add_argument("--apiserver", default="")
    ap.add_argument("--token", default="")
    ap.add_argument("--ca-file", default="", help="CA bundle that signs --apiserver's certificate (default: system CAs)")
    ap.add_argument("--insecure-skip-tls-verify", action="store_true",
                    help="do not verify --apiserver's certificate (test clusters only: the bearer token goes to whoever answers)")
    ap.add_argument("--tls-cert", default="", help="serve HTTPS with this certificate (PEM)")
    ap.add_argument("--tls-key", default="", help="private key of --tls-cert (PEM)")
    ap.add_argument("--client-ca", default="",
                    help="require callers to present a certificate signed by this CA (mutual TLS; kube-scheduler's "
                         "extender tlsConfig.certFile/keyFile) — needed before serving beyond loopback")
    ap.add_argument("--ledger-store", default="lease", choices=["lease", "node", "both"],
                    help="where the allocation ledger lives: a coordination.k8s.io Lease per node (default), the "
                         "round-5 Node annotation, or both during a rolling upgrade (docs/MIGRATION.md)")
    ap.add_argument("--ledger-namespace", default=os.environ.get("POD_NAMESPACE", "kube-system"),
                    help="namespace of the ledger Leases (the extender's own)")
    ap.add_argument("--bind-ledger", default="on", choices=["on", "off"],
                    help="record every bind's devices in the node's allocation ledger (<prefix>/gpu-ledger, see "
                         "--ledger-store) with the ledger's resourceVersion as a precondition, so extender replicas never "
                         "hand out one GPU twice; off = the per-process node lock only (a single extender)")
    ap.add_argument("--bind-budget", type=float, default=10.0,
                    help="seconds a bind may spend re-deciding on ledger conflicts before it answers 409 and lets "
                         "kube-scheduler retry (informer events for that node wait while a bind holds its lock)")
    ap.add_argument("--log-level", default="INFO")
    a = ap.parse_args(argv)
    logging.basicConfig(level=a.log_level, format='{"ts":"%(asctime)s","lvl":"%(levelname)s","mod":"%(name)s","msg":"%(message)s"}')
    from ..k8s.api import RestKubeAPI

    api = (RestKubeAPI(a.apiserver, token=a.token or None, ca_file=a.ca_file or None, verify=not a.insecure_skip_tls_verify)
           if a.apiserver else RestKubeAPI.in_cluster())
    cfg = ExtenderConfig(contract=Contract(resource_name=a.resource_name, prefix=a.annotation_prefix, slice_resource=a.slice_resource_name), policy_name=a.policy,
                         policy=PlacementPolicy(tie_break=a.tie_break, partition_aware=a.partition_aware == "on"),
                         assume_ttl=a.assume_ttl, resync_s=a.resync,
                         scheduler_names=tuple(x.strip() for x in a.scheduler_names.split(",") if x.strip()),
                         ledger=a.bind_ledger == "on", ledger_store=a.ledger_store, ledger_namespace=a.ledger_namespace,
                         bind_budget_s=a.bind_budget)
    ext = TopologyExtender(api, cfg)
    if a.informer == "on":
        ext.cache.make_informer(page_size=a.list_page_size, watch_cache=a.list_from_watch_cache == "on").start()
    ssl_context = None
    if a.tls_cert or a.tls_key:
        from .server import tls_context

        ssl_context = tls_context(a.tls_cert, a.tls_key, a.client_ca)
    elif a.client_ca:
        print("--client-ca needs --tls-cert and --tls-key", file=sys.stderr)
        return 2
    if a.host not in ("127.0.0.1", "localhost", "::1") and not a.client_ca:
        logging.getLogger("gtk.extender").warning(
            "listening on %s without --client-ca: /bind is reachable by anything that can reach this address", a.host)
    run(ext, a.host, a.port, a.url_prefix, resync_period=a.resync, ssl_context=ssl_context)
    return 0


if __name__ == "__main__":
    sys.exit(main())
