"""``python -m gpu_topology_on_k8s_amd <command>`` — operator tool.

  topo      discover the node (amdsmi / sysfs / fake) and print the matrix, JSON or annotations
  probe     run the HIP link probe (MFMA warm-up + LDS-staged copies) and print GB/s / cost
  ring      K6: every member of a subset pulls from its peers at once; the busBW ceiling of a ring
  select    run the placement core on a topology (file, discovery or fake) for k devices
  config    emit the scheduler config: ``scheduler`` (KubeSchedulerConfiguration), ``policy``
            (the reference's legacy Policy JSON, design.md:92-113) or ``manifests`` (deploy YAML)
  validate  RCCL all-reduce over the allocated devices (GTK_GPU_GROUP or --devices): the
            placement validator of SURVEY.md §3.5 (flow step 8)
  sim       run a small in-process cluster and print the scheduling decisions
  doctor    node / pod readiness checks (device nodes, discovery, extensions, IPC mode, CPU affinity,
            a pod's GROUP, cpuset and share guard), one JSON line each; --gpu adds HIP checks
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from typing import List, Optional

import yaml


def _topology(a):
    from .topology.discovery import discover
    from .topology.model import Topology

    if getattr(a, "topology", None):
        with open(a.topology) as f:
            t = Topology.from_json(f.read())
    else:
        t = discover(a.discovery, fake_n=a.fake_gpus)
    if getattr(a, "time_slices", 1) > 1:  # what a device plugin run with --time-slices advertises
        from .topology.shares import time_slice

        t = time_slice(t, a.time_slices)
    return t


def _ints(s: Optional[str]) -> List[int]:
    return [int(x) for x in s.split(",") if x.strip()] if s else []


def cmd_partition(a) -> int:
    """``gtk partition show`` (read-only) / ``gtk partition set --compute CPX [--memory NPS4] --yes``."""
    from .topology.partition import PartitionError, apply_partition, partition_info

    if a.action == "show":
        for p in partition_info():
            print(json.dumps(p))
        return 0
    if not (a.compute or a.memory):
        print("partition set: give --compute and/or --memory", file=sys.stderr)
        return 2
    if not a.yes:
        print("partition set re-partitions every GPU of this node (device IDs change, running GPU processes break): "
              "stop them and pass --yes", file=sys.stderr)
        return 2
    try:
        r = apply_partition(a.compute, a.memory, reload_driver=a.reload_driver)
    except PartitionError as e:
        print(f"partition set: {e}", file=sys.stderr)
        return 1
    print(json.dumps({k: r[k] for k in ("ok", "reason", "steps", "reload_required", "reloaded")}))
    return 0 if r["ok"] else 1


def cmd_topo(a) -> int:
    from .k8s.annotations import Contract, encode_node_annotations

    t = _topology(a)
    if a.output == "json":
        print(t.to_json(indent=None))
    elif a.output == "annotations":
        print(json.dumps(encode_node_annotations(t, Contract(resource_name=a.resource_name)), indent=1))
    else:
        print(f"{t.n} devices via {t.source}")
        print(t.render())
    return 0


def cmd_probe(a) -> int:
    from .ops.probe import probe_topology

    t = _topology(a)
    probe_topology(t, preset=a.preset, mode=a.mode)
    if a.out:  # written before the ingress stage, so a failure there keeps the pairwise matrix
        with open(a.out, "w") as f:
            f.write(t.to_json())
    if a.ingress:
        from .ops.probe import measure_ingress

        measure_ingress(t, t.probe.get("devices", list(range(t.n))), preset=a.preset)
        if a.out:
            with open(a.out, "w") as f:
                f.write(t.to_json())
    print(t.render())
    print(json.dumps({"probe": t.probe, "hbm_gbps": [None if x != x else round(float(x), 1) for x in t.hbm_gbps]}))
    return 0


def cmd_ring(a) -> int:
    """K6 concurrent ring probe over HIP ordinals (``--devices``) or a node-local GROUP resolved by
    PCI address; prints one JSON line with ``ring_bound_gbps``."""
    from .ops.probe import measure_ring

    devs = validate_devices(a)
    if len(devs) < 2:
        print("gtk ring: needs at least 2 devices", file=sys.stderr)
        return 2
    print(json.dumps(measure_ring(devs, preset=a.preset, patterns=[p for p in a.patterns.split(",") if p])))
    return 0


def cmd_ipc(a) -> int:
    """Cross-process GPU memory through HIP IPC, the mapping RCCL's P2P transport uses between ranks.
    This process exports patterned buffers on ``--device``; a child opens the handles on
    ``--reader-device`` and runs a probe kernel on the mappings (``--mode``):

    * ``read``   (K1) streams one buffer into its own with the LDS-DMA kernel and verifies it;
    * ``write``  (K2) pushes its own pattern into the exported buffer (remote stores); the owner
      verifies what landed in its memory;
    * ``gather`` (K5) pulls ``--segments`` exported buffers in one launch, each segment verified.

    Prints one JSON line, and exits 1 when the export, the import or a check fails."""
    import subprocess

    from ._native import load

    probe = load("_probe")
    if a.child:  # the importing side
        handles = [bytes.fromhex(h) for h in a.handles.split(",")]
        seeds = [int(s) for s in a.seeds.split(",")]
        if a.child == "read":
            r = dict(probe.ipc_read_bw(handles[0], a.reader_device, a.bytes, seeds[0], a.iters))
        elif a.child == "write":
            r = dict(probe.ipc_write_bw(handles[0], a.reader_device, a.bytes, seeds[0], a.iters), ok=True)
        else:
            r = dict(probe.ipc_gather_bw(handles, a.reader_device, a.bytes, seeds, a.iters))
        print(json.dumps(r))
        return 0 if r["ok"] else 1
    nbuf = a.segments if a.mode == "gather" else 1
    if not 1 <= nbuf <= 16:
        print("gtk ipc: --segments must be 1..16", file=sys.stderr)
        return 2
    out = {"mode": a.mode, "ipc_mode_legacy": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY"), "bytes": a.bytes,
           "device": a.device, "reader_device": a.reader_device}
    if a.mode == "gather":
        out["segments"] = nbuf
    seeds = [(a.seed + 7919 * i) & 0xFFFFFFFF for i in range(nbuf)]
    try:
        bufs = [probe.IpcBuffer(a.device, a.bytes, s) for s in seeds]
    except RuntimeError as e:
        out.update(ok=False, stage="export (hipIpcGetMemHandle)", error=str(e)[:300])
        print(json.dumps(out))
        return 1
    # the writer pushes a pattern the exported buffer does not already hold, so a no-op write fails
    child_seeds = [s ^ 0xA5A5A5A5 for s in seeds] if a.mode == "write" else seeds
    p = subprocess.run([sys.executable, "-m", "gpu_topology_on_k8s_amd", "ipc", "--child", a.mode,
                        "--handles", ",".join(b.handle().hex() for b in bufs), "--seeds", ",".join(map(str, child_seeds)),
                        "--bytes", str(a.bytes), "--reader-device", str(a.reader_device), "--iters", str(a.iters)],
                       capture_output=True, text=True, timeout=a.timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if p.returncode != 0 or not lines:
        out.update(ok=False, stage=f"import (hipIpcOpenMemHandle) / {a.mode}", error=(p.stderr or p.stdout)[-300:])
        print(json.dumps(out))
        return 1
    r = json.loads(lines[-1])
    ok = bool(r["ok"])
    if a.mode == "write":
        ok = ok and bufs[0].holds(child_seeds[0])
    out.update(ok=ok, ms_per_iter=round(r["ms_per_iter"], 4))
    out[{"read": "read_gbps", "write": "write_gbps", "gather": "ingress_gbps"}[a.mode]] = round(r["gbps"], 1)
    print(json.dumps(out))
    return 0 if ok else 1


def cmd_select(a) -> int:
    from .placement import PlacementPolicy, select, worst
    from .placement.gaia import gaia_schedule, tree_from_topology

    t = _topology(a)
    used = _ints(a.used)
    if a.fraction:
        # a fraction of ONE GPU: XCP partitions (CPX/DPX/QPX) or time slices, Gaia Fragment best fit
        import math

        from .placement import place_fraction
        from .topology.shares import cu_mask_env, share_fractions

        per = max(int((t.physical == p).sum()) for p in set(t.physical.tolist()))
        if per <= 1:
            print("gtk select: --fraction needs a partitioned (CPX/DPX/QPX) or time-sliced node (--time-slices S)",
                  file=sys.stderr)
            return 2
        k = max(1, math.ceil(a.fraction * per - 1e-9))
        ids = place_fraction(t, k, used)
        out = {"ids": list(ids), "policy": "fragment", "devices_per_gpu": per,
               "gpu": int(t.gpus[ids[0]].physical), "share": round(share_fractions(t, ids)[int(t.gpus[ids[0]].physical)], 4)}
        if cu_mask_env(t, ids):
            out["hsa_cu_mask"] = cu_mask_env(t, ids)
        print(json.dumps(out))
        return 0
    if a.k <= 0:
        print("gtk select: give -k N (devices) or --fraction m", file=sys.stderr)
        return 2
    if a.policy == "gaia":
        ids = gaia_schedule(tree_from_topology(t, used), a.k)
        print(json.dumps({"ids": ids, "policy": "gaia"}))
        return 0
    pl = select(t, a.k, used=used, policy=PlacementPolicy())
    out = {"ids": list(pl.ids), "score": round(pl.score, 4), "objective": round(pl.objective, 6), "exact": pl.exact,
           "terms": {k: round(v, 6) for k, v in pl.terms.items()}}
    if a.worst or a.explain:
        w = worst(t, a.k, used=used)
        out["worst"] = {"ids": list(w.ids), "score": round(w.score, 4)}
    if a.explain:
        # what bench.py's placement_terms carries: the terms of the chosen, worst and kubelet-default
        # subsets, the terms that separate each from the choice and the gain its ring-bound link predicts
        from .placement.explain import default_subset, explain_subsets

        out["explain"] = explain_subsets(t, {"chosen": pl.ids, "worst": w.ids, "default": default_subset(t, a.k, used)},
                                         used=used)
    print(json.dumps(out))
    return 0


def cmd_defrag(a) -> int:
    """Plan the fewest pod moves after which a k-GPU pod fits (placement/defrag.py) from the
    apiserver's nodes and pods; prints the plan, changes nothing."""
    from .deviceplugin.__main__ import make_api
    from .extender import ExtenderConfig, TopologyExtender
    from .k8s.annotations import Contract

    api = make_api(a.apiserver, a.token, a.ca_file, a.insecure_skip_tls_verify)
    if api is None:
        print("gtk defrag: no apiserver (--apiserver URL, or run in a cluster)", file=sys.stderr)
        return 2
    ext = TopologyExtender(api, ExtenderConfig(contract=Contract(resource_name=a.resource_name), resync_s=0.0, events=False))
    print(json.dumps({"gpus": a.k, "plan": ext.defrag(a.k, a.max_moves, a.min_score)}))
    return 0


def cmd_status(a) -> int:
    """Per-node GPU view from the apiserver, as the extender sees it: devices, used, free,
    fragmentation index, and the best placement score for each request size (or '-' if none fits)."""
    from .deviceplugin.__main__ import make_api
    from .extender import ExtenderConfig, TopologyExtender
    from .extender.metrics import node_fragmentation
    from .k8s.annotations import Contract
    from .placement.numa_align import tm_from_labels
    api = make_api(a.apiserver, a.token, a.ca_file, a.insecure_skip_tls_verify)
    if api is None:
        print("gtk status: no apiserver (--apiserver URL, or run in a cluster)", file=sys.stderr)
        return 2
    ext = TopologyExtender(api, ExtenderConfig(contract=Contract(resource_name=a.resource_name), resync_s=0.0, events=False))
    ext.cache.sync_all()
    sizes = _ints(a.sizes)
    rows = []
    now = ext.clock()
    for st in sorted(ext.cache.nodes(), key=lambda s: s.name):
        with st.lock:
            t = st.topology
            if t is None:
                continue
            used = st.used(now, ext.cfg.assume_ttl)
            free, frag, _ = node_fragmentation(t, used, st.unknown)
            per_gpu = max((int((t.physical == p).sum()) for p in set(t.physical.tolist())), default=1)
            row = {"node": st.name, "devices": t.n, "per_gpu": per_gpu,
                   "used": len(used) + st.unknown, "free": free, "fragmentation": round(frag, 3), "best_score": {}}
            if per_gpu > 1:  # partitioned / time-sliced: the share of every physical GPU in use
                row["gpu_share_used"] = {str(p): round(sum(1 for g in t.gpus if g.physical == p and g.index in used) /
                                                       sum(1 for g in t.gpus if g.physical == p), 3)
                                         for p in sorted(set(t.physical.tolist()))}
        row["partition"] = f"{t.gpus[0].partition}/{t.gpus[0].memory_partition}" if t.gpus else ""
        row["probing"] = bool(getattr(st, "probing_until", 0.0) > now)  # re-probe / repartition: the extender skips it
        row["unhealthy"] = [g.index for g in t.gpus if not g.healthy]
        tm = tm_from_labels(st.labels, ext.cfg.contract.prefix)
        if tm.active:  # the kubelet aligns devices to NUMA nodes: the scores below already account for it
            row["topology_manager"] = f"{tm.policy}/{tm.scope}"
        try:  # the operator's partition request and a refusal the plugin recorded
            md = api.get_node(st.name).get("metadata") or {}
            c = ext.cfg.contract
            req = [(md.get("labels") or {}).get(k) for k in (c.partition_request_label, c.memory_partition_request_label)]
            if any(req):
                row["partition_request"] = "/".join(x or "-" for x in req)
            failed = (md.get("annotations") or {}).get(c.partition_failed_key)
            if failed:
                row["partition_change_failed"] = failed
            cordon = (md.get("annotations") or {}).get(c.cordon_key)
            if cordon:
                row["cordoned"] = cordon  # the operator's out-of-service GPUs (the plugin holds them Unhealthy)
        except Exception:  # noqa: BLE001 - the node vanished meanwhile: the row stands without it
            pass
        # a sliced node is scored for slice requests (its own pool), every other node for whole devices
        res = ext.cfg.contract.slice_resource if int(max((g.shares for g in t.gpus), default=1)) > 1 else ext.cfg.contract.resource_name
        row["resource"] = res
        for k in sizes:
            probe_pod = {"metadata": {"name": "status", "namespace": "default"},
                         "spec": {"containers": [{"name": "c", "resources": {"limits": {res: str(k)}}}]}}
            d, _ = ext._eval_state(probe_pod, st.name, st, k)
            row["best_score"][str(k)] = None if d is None else round(d.score, 2)
        rows.append(row)
    if a.output == "json":
        print(json.dumps(rows))
        return 0
    head = f"{'NODE':<20}{'DEV':>5}{'USED':>6}{'FREE':>6}{'DOWN':>6}{'FRAG':>7}  " + "  ".join(f"k={k:<4}" for k in sizes) + "  NOTES"
    print(head)
    for r in rows:
        cells = "  ".join(f"{('-' if r['best_score'][str(k)] is None else format(r['best_score'][str(k)], '.2f')):<6}" for k in sizes)
        notes = ", ".join(x for x in (f"cordoned {r['cordoned']}" if r.get("cordoned") else "",
                                      f"topology-manager {r['topology_manager']}" if r.get("topology_manager") else "",
                                      "probing" if r.get("probing") else "") if x)
        print(f"{r['node']:<20}{r['devices']:>5}{r['used']:>6}{r['free']:>6}{len(r['unhealthy']):>6}{r['fragmentation']:>7.3f}  {cells}  {notes}")
    return 0


def cmd_config(a) -> int:
    from .config import legacy_policy, render_manifests, scheduler_configuration

    if a.kind == "kind":
        from .config import render_kind

        out = render_kind(a.resource_name, image=a.image)
        if a.out_dir:
            os.makedirs(a.out_dir, exist_ok=True)
            for name, text in out.items():
                with open(os.path.join(a.out_dir, name), "w") as f:
                    f.write(text)
                if name.endswith(".sh"):
                    os.chmod(os.path.join(a.out_dir, name), 0o755)
        else:
            print(out["gpu-topology-kind.yaml"], end="")
        return 0
    if a.kind == "alerts":
        from .config import prometheus_rules

        print(yaml.safe_dump(prometheus_rules(), sort_keys=False), end="")
    elif a.kind == "policy":
        print(json.dumps(legacy_policy(a.resource_name, with_filter=a.filter), indent=2))
    elif a.kind == "scheduler":
        print(yaml.safe_dump(scheduler_configuration(a.resource_name, with_filter=a.filter, tls_dir=a.tls_dir or None),
                             sort_keys=False), end="")
    else:
        print(render_manifests(a.resource_name, image=a.image, time_slices=a.time_slices,
                               partition_control=a.partition_control, topology_manager_policy=a.topology_manager_policy,
                               topology_manager_scope=a.topology_manager_scope), end="")
    return 0


def validate_devices(a, env=None) -> List[int]:
    """HIP ordinals to validate: ``--devices`` (ordinals) as given; else the pod's node-local GROUP
    (``--group`` or ``GTK_GPU_GROUP``) resolved through ``GTK_GPU_BDFS`` / ``--topology`` by PCI
    address (:func:`topology.identity.resolve_group`); else every visible device."""
    from .topology.identity import ENV_BDFS, group_from_env, hip_device_bdfs, resolve_group

    if a.devices:
        return _ints(a.devices)
    env = os.environ if env is None else env
    group, bdfs = group_from_env(env)
    if a.group:
        group = _ints(a.group)
        bdfs = [b for b in (a.bdfs or "").split(",") if b.strip()]
    elif a.bdfs:
        bdfs = [b for b in a.bdfs.split(",") if b.strip()]
    vis = hip_device_bdfs() if a.visible_bdfs is None else [b for b in a.visible_bdfs.split(",") if b.strip()]
    if not group:
        return list(range(len(vis)))
    topo = None
    if a.topology:
        from .topology.model import Topology

        with open(a.topology) as f:
            topo = Topology.from_json(f.read())
    if bdfs and len(bdfs) != len(group):
        raise SystemExit(f"{ENV_BDFS} has {len(bdfs)} entries for GROUP {group}")
    return resolve_group(group, bdfs=bdfs or None, topology=topo, visible_bdfs=vis)


def cmd_validate(a) -> int:
    from ._native import load
    from .topology.cpus import bind_workload

    devs = validate_devices(a)
    # Gaia B6: the validator's host threads (RCCL proxies) on the pod's cores (GTK_CPUSET from Allocate)
    cpu_rep = bind_workload(a.cpu_bind, "")
    if a.resolve_only:
        print(json.dumps({"hip_devices": devs}))
        return 0
    rccl = load("_rccl")
    sizes = rccl.size_sweep(a.min_bytes, a.max_bytes, a.factor)
    pts = rccl.local_sweep(devs, sizes, a.dtype, a.iters, a.warmup, False, True)
    wrong = sum(p["wrong"] for p in pts)
    peak = max(pts, key=lambda p: p["busbw_gbps"] if len(devs) > 1 else p["algbw_gbps"])
    for p in pts:
        print(json.dumps({"k": len(devs), "devices": devs, **p}))
    print(json.dumps({"summary": True, "k": len(devs), "devices": devs, "wrong": wrong, "peak_bytes": peak["bytes"],
                      "peak_algbw_gbps": round(peak["algbw_gbps"], 2), "peak_busbw_gbps": round(peak["busbw_gbps"], 2),
                      "cpuset_applied": {k: cpu_rep.get(k) for k in ("applied", "source", "cpus", "n", "reason")}}))
    return 1 if wrong else 0


def cmd_sim(a) -> int:
    from .sim import SimCluster
    from .topology import fixtures as fx

    with SimCluster({f"node{i}": fx.f7_mi355x(link_gbps=76.5, noise=0.03, seed=i) for i in range(a.nodes)},
                    policy_name=a.policy) as c:
        for i, k in enumerate(_ints(a.pods)):
            c.submit(f"pod{i}-{k}gpu", k)
        for r in c.schedule_pending():
            print(json.dumps({"pod": r.pod, "node": r.node, "devices": list(r.allocated), "score": r.score,
                              "sched_ms": round(r.sched_ms, 3), "admit_ms": round(r.admit_ms, 3), "error": r.error}))
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="gtk", description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)

    def disc(p):
        p.add_argument("--discovery", default="auto", choices=["auto", "amdsmi", "sysfs", "fake"])
        p.add_argument("--fake-gpus", type=int, default=None)
        p.add_argument("--topology", default="", help="topology JSON file instead of discovery")
        p.add_argument("--time-slices", type=int, default=1, help="view every GPU as this many time slices (device plugin --time-slices)")

    p = sub.add_parser("topo")
    disc(p)
    p.add_argument("--output", default="table", choices=["table", "json", "annotations"])
    p.add_argument("--resource-name", default="amd.com/gpu")
    p.set_defaults(fn=cmd_topo)
    p = sub.add_parser("probe")
    disc(p)
    p.add_argument("--preset", default="quick", choices=["quick", "full"])
    p.add_argument("--mode", default="read", choices=["read", "write"])
    p.add_argument("--ingress", action="store_true", help="also measure each GPU's all-peer ingress (K5 gather)")
    p.add_argument("--out", default="")
    p.set_defaults(fn=cmd_probe)
    p = sub.add_parser("ring", help="K6: concurrent ring-pattern probe of a device subset (busBW ceiling)")
    p.add_argument("--devices", default="", help="HIP ordinals (skips GROUP resolution)")
    p.add_argument("--group", default="", help="node-local device indices (default: $GTK_GPU_GROUP)")
    p.add_argument("--bdfs", default="", help="PCI addresses of --group, same order (default: $GTK_GPU_BDFS)")
    p.add_argument("--topology", default="", help="node topology JSON mapping GROUP indices to PCI addresses")
    p.add_argument("--visible-bdfs", default=None, help=argparse.SUPPRESS)
    p.add_argument("--preset", default="quick", choices=["quick", "full"])
    p.add_argument("--patterns", default="all,ring", help="K6 peer patterns: all (every link of the subset), ring (pred+succ)")
    p.set_defaults(fn=cmd_ring)
    p = sub.add_parser("ipc", help="cross-process GPU memory through HIP IPC (RCCL's P2P mapping): K1 read, K2 write "
                                   "or K5 gather kernels on the imported mappings")
    p.add_argument("--mode", default="read", choices=["read", "write", "gather"])
    p.add_argument("--segments", type=int, default=7, help="--mode gather: exported buffers pulled in one launch (1..16)")
    p.add_argument("--device", type=int, default=0, help="HIP ordinal that owns (exports) the buffers")
    p.add_argument("--reader-device", type=int, default=0, help="HIP ordinal of the importing process (a peer on a node)")
    p.add_argument("--bytes", type=int, default=256 << 20)
    p.add_argument("--seed", type=int, default=0x5EED)
    p.add_argument("--iters", type=int, default=5)
    p.add_argument("--timeout", type=float, default=180.0)
    p.add_argument("--child", default="", choices=["", "read", "write", "gather"], help=argparse.SUPPRESS)
    p.add_argument("--handles", default="", help=argparse.SUPPRESS)
    p.add_argument("--seeds", default="", help=argparse.SUPPRESS)
    p.set_defaults(fn=cmd_ipc)
    p = sub.add_parser("select")
    disc(p)
    p.add_argument("-k", type=int, default=0)
    p.add_argument("--fraction", type=float, default=0.0,
                   help="0 < m < 1 of one GPU (Gaia Fragment) on a partitioned or --time-slices node, instead of -k")
    p.add_argument("--used", default="")
    p.add_argument("--policy", default="exact", choices=["exact", "gaia"])
    p.add_argument("--worst", action="store_true")
    p.add_argument("--explain", action="store_true",
                   help="the objective's terms for the chosen, worst and kubelet-default (lowest free ids) subsets, "
                        "the terms that separate them and the gain their slowest ring link predicts")
    p.set_defaults(fn=cmd_select)
    p = sub.add_parser("defrag", help="plan pod moves that make a k-GPU pod placeable (read-only)")
    p.add_argument("-k", type=int, default=8)
    p.add_argument("--max-moves", type=int, default=3)
    p.add_argument("--min-score", type=float, default=0.0, help="only placements scoring at least this (0..10) count")
    p.add_argument("--apiserver", default="")
    p.add_argument("--token", default="")
    p.add_argument("--ca-file", default="")
    p.add_argument("--insecure-skip-tls-verify", action="store_true")
    p.add_argument("--resource-name", default="amd.com/gpu")
    p.set_defaults(fn=cmd_defrag)
    p = sub.add_parser("status", help="per-node GPU usage, fragmentation and best placement score per size (read-only)")
    p.add_argument("--sizes", default="1,2,4,8")
    p.add_argument("--output", default="table", choices=["table", "json"])
    p.add_argument("--apiserver", default="")
    p.add_argument("--token", default="")
    p.add_argument("--ca-file", default="")
    p.add_argument("--insecure-skip-tls-verify", action="store_true")
    p.add_argument("--resource-name", default="amd.com/gpu")
    p.set_defaults(fn=cmd_status)
    p = sub.add_parser("config")
    p.add_argument("kind", choices=["scheduler", "policy", "manifests", "kind", "alerts"])
    p.add_argument("--out-dir", default="", help="kind: write every file of deploy/kind/ here")
    p.add_argument("--resource-name", default="amd.com/gpu")
    p.add_argument("--filter", action="store_true")
    p.add_argument("--image", default="rocm/gpu-topology-k8s:latest")
    p.add_argument("--time-slices", type=int, default=1, help="manifests: device plugin --time-slices (fractional GPUs on SPX nodes)")
    p.add_argument("--topology-manager-policy", default="", choices=["", "none", "best-effort", "restricted", "single-numa-node"],
                   help="manifests: the GPU nodes' kubelet --topology-manager-policy, published by the device plugin so the "
                        "extender binds the devices the kubelet will allocate")
    p.add_argument("--topology-manager-scope", default="", choices=["", "container", "pod"],
                   help="manifests: the GPU nodes' kubelet --topology-manager-scope")
    p.add_argument("--partition-control", action="store_true",
                   help="manifests: device plugin --partition-control on (switches partition modes on node labels; /sys writable)")
    p.add_argument("--tls-dir", default="", help="scheduler: call the extender over mutual TLS with tls.crt/tls.key/ca.crt from here")
    p.set_defaults(fn=cmd_config)
    p = sub.add_parser("validate")
    p.add_argument("--devices", default="", help="HIP ordinals (skips GROUP resolution)")
    p.add_argument("--group", default="", help="node-local device indices (default: $GTK_GPU_GROUP)")
    p.add_argument("--bdfs", default="", help="PCI addresses of --group, same order (default: $GTK_GPU_BDFS)")
    p.add_argument("--topology", default="", help="node topology JSON mapping GROUP indices to PCI addresses")
    p.add_argument("--visible-bdfs", default=None, help=argparse.SUPPRESS)  # tests: stand-in for hipDeviceGetPCIBusId
    p.add_argument("--resolve-only", action="store_true", help="print the HIP ordinals and exit")
    p.add_argument("--min-bytes", type=int, default=1 << 20)
    p.add_argument("--max-bytes", type=int, default=1 << 30)
    p.add_argument("--factor", type=int, default=4)
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp16", "fp32"])
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--cpu-bind", default="env", choices=["env", "off"], help="pin to GTK_CPUSET (the pod's cores) or not")
    p.set_defaults(fn=cmd_validate)
    p = sub.add_parser("doctor", help="node / pod readiness checks (JSON lines); exit 1 on any failure")
    p.add_argument("--discovery", default="auto", choices=["auto", "amdsmi", "sysfs", "fake"])
    p.add_argument("--fake-gpus", type=int, default=None)
    p.add_argument("--gpu", action="store_true", help="also initialise HIP: device count, gfx950, MFMA warm-up")
    p.add_argument("--dev-root", default="/dev")
    p.add_argument("--plugin-dir", default="/var/lib/kubelet/device-plugins")
    p.add_argument("--kubelet-config", default="/var/lib/kubelet/config.yaml",
                   help="KubeletConfiguration whose Topology Manager policy the device plugin must be given")
    p.set_defaults(fn=lambda a: __import__("gpu_topology_on_k8s_amd.doctor", fromlist=["main"]).main(a))
    p = sub.add_parser("partition", help="GPU compute / memory partition modes: show, or set (root; the node must be idle)")
    p.add_argument("action", choices=["show", "set"])
    p.add_argument("--compute", default=None, help="set: SPX | DPX | QPX | CPX")
    p.add_argument("--memory", default=None, help="set: NPS1 | NPS2 | NPS4 | NPS8")
    p.add_argument("--reload-driver", action="store_true", help="set: reload amdgpu to complete a memory-partition change")
    p.add_argument("--yes", action="store_true", help="set: really change the hardware (every GPU process must be stopped)")
    p.set_defaults(fn=cmd_partition)
    p = sub.add_parser("sim")
    p.add_argument("--nodes", type=int, default=2)
    p.add_argument("--pods", default="4,4,2,1,1,8")
    p.add_argument("--policy", default="exact", choices=["exact", "gaia", "design"])
    p.set_defaults(fn=cmd_sim)
    a = ap.parse_args(argv)
    return a.fn(a)


if __name__ == "__main__":
    sys.exit(main())
