"""Device-plugin daemon (DaemonSet entry point).

    python -m gpu_topology_on_k8s_amd.deviceplugin --resource-name amd.com/gpu --probe quick

Bring-up: discover the node (amdsmi, KFD sysfs fallback), optionally seed the
link-cost matrix with the HIP probe (MFMA warm-up + LDS-staged p2p reads), publish the topology
annotations, serve the kubelet ``v1beta1`` API and register.  Health is re-polled from the same
discovery backend.
"""
from __future__ import annotations

import argparse
import logging
import os
import signal
import sys
import threading
import time
from typing import Optional, Tuple

from ..k8s.annotations import Contract
from ..placement import PlacementPolicy
from ..topology.discovery import discover
from ..topology.shares import time_slice
from .health import HealthMonitor, HealthPolicy
from .plugin import DevicePluginServer, PluginConfig, node_is_idle, startup_topology
from .proto import DEVICE_PLUGIN_PATH


def make_api(apiserver: str, token: str, ca_file: str = "", insecure: bool = False):
    from ..k8s.api import RestKubeAPI

    if apiserver == "none":
        return None
    if apiserver:
        return RestKubeAPI(apiserver, token=token or None, ca_file=ca_file or None, verify=not insecure)
    if os.environ.get("KUBERNETES_SERVICE_HOST"):
        return RestKubeAPI.in_cluster()
    return None


def node_time_slices(api, node_name: str, contract: Contract, default: int, node: Optional[dict] = None) -> int:
    """Time slices for this node: the operator's node label ``<prefix>/time-slices`` when set (one
    DaemonSet serves a cluster where only some nodes are shared), else ``--time-slices``.  ``node``:
    the Node object already read (no second GET)."""
    if node is None and (api is None or not node_name):
        return default
    try:
        labels = ((node if node is not None else api.get_node(node_name)).get("metadata") or {}).get("labels") or {}
    except Exception as e:  # noqa: BLE001 - the flag still applies
        logging.getLogger("gtk.deviceplugin").warning("reading node %s labels failed: %s", node_name, e)
        return default
    raw = labels.get(contract.time_slices_label)
    if raw is None:
        return default
    try:
        return max(1, int(raw))
    except ValueError:
        logging.getLogger("gtk.deviceplugin").warning("ignoring %s=%r (not an integer)", contract.time_slices_label, raw)
        return default


def startup_time_slices(api, node_name: str, contract: Contract, default: int,
                        resource_names=("amd.com/gpu", "amd.com/gpu-slice")) -> Tuple[int, str]:
    """Time slices a (re)starting plugin advertises, and why.

    The wanted count is the node label (or ``--time-slices``).  Device IDs depend on it, so if the
    count published by the previous plugin run (``<prefix>/time-slices-active``) differs and any pod
    still holds a device, the previous count is kept: the running pods' GROUP annotations and the
    kubelet's checkpointed IDs name devices of that layout (a crash / OOM / rollout restart must not
    re-number them).  The main loop's idle check performs the switch later (exit 75 + restart)."""
    want = node_time_slices(api, node_name, contract, default)
    if api is None or not node_name:
        return want, ""
    try:
        raw = ((api.get_node(node_name).get("metadata") or {}).get("annotations") or {}).get(contract.active_slices_key)
        active = int(raw) if raw not in (None, "") else None
    except Exception:  # noqa: BLE001 - nothing published (first start) or unreadable: use the label
        active = None
    if active is None or active == want:
        return want, ""
    if node_is_idle(api, node_name, resource_names):
        return want, f"time slices per GPU {active} -> {want} (node idle)"
    return active, (f"keeping {active} time slices per GPU: pods hold devices of that layout; "
                    f"the switch to {want} waits until the node is idle")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--resource-name", default="amd.com/gpu", help="extended resource of whole GPUs (or XCP partitions)")
    ap.add_argument("--slice-resource-name", default="amd.com/gpu-slice",
                    help="extended resource a time-sliced node (--time-slices S > 1) advertises its slices under instead: "
                         "whole GPUs and slices are separate pools, so --resource-name always means whole devices")
    ap.add_argument("--annotation-prefix", default="gputopology.amd.com")
    ap.add_argument("--socket-dir", default=DEVICE_PLUGIN_PATH)
    ap.add_argument("--socket-name", default="amd-gpu-topology.sock")
    ap.add_argument("--node-name", default=os.environ.get("NODE_NAME", ""))
    ap.add_argument("--discovery", default="auto", choices=["auto", "amdsmi", "sysfs", "fake"])
    ap.add_argument("--fake-gpus", type=int, default=None, help="fake backend device count (kind / CPU-only nodes)")
    ap.add_argument("--probe", default="off", choices=["off", "quick", "full"])
    ap.add_argument("--apiserver", default="", help="apiserver URL; default in-cluster; 'none' disables annotations")
    ap.add_argument("--token", default="")
    ap.add_argument("--ca-file", default="", help="CA bundle that signs --apiserver's certificate (default: system CAs)")
    ap.add_argument("--insecure-skip-tls-verify", action="store_true",
                    help="do not verify --apiserver's certificate (test clusters only: the bearer token goes to whoever answers)")
    ap.add_argument("--dev-root", default="/dev", help="where the ROCm device nodes live (a placeholder dir on kind)")
    ap.add_argument("--cdi-dir", default="/var/run/cdi", help="--device-specs cdi: where the CDI spec is written")
    ap.add_argument("--device-specs", default="auto", choices=["auto", "strict", "stub", "cdi"],
                    help="Allocate DeviceSpecs: strict = kfd + render/card nodes, fail if missing; stub = only nodes "
                         "that exist under --dev-root (kind / fake GPUs); cdi = CDI device names resolved by the spec written to "
                         "--cdi-dir (CDI-enabled runtimes); auto = stub for --discovery fake, else strict")
    ap.add_argument("--xgmi-link-loss", default="degrade", choices=["degrade", "unhealthy"],
                    help="a GPU whose xGMI link drops: degrade = republish the pair at its new link class and keep the "
                         "GPU schedulable; unhealthy = advertise the GPU Unhealthy")
    ap.add_argument("--prestart-validate", action="store_true",
                    help="validate every placement with an RCCL all-reduce over the container's devices before it starts")
    ap.add_argument("--metrics-port", type=int, default=0, help="serve Prometheus /metrics on this port (0 = off)")
    ap.add_argument("--metrics-host", default="0.0.0.0")
    ap.add_argument("--health-interval", type=float, default=10.0)
    ap.add_argument("--pod-resources-socket", default="/var/lib/kubelet/pod-resources/kubelet.sock",
                    help="kubelet pod-resources API; GROUP annotations are reconciled against it ('' = off)")
    ap.add_argument("--reconcile-interval", type=float, default=10.0,
                    help="seconds between pod-resources reconciliation passes (0 = off)")
    ap.add_argument("--admission-settle", type=float, default=5.0,
                    help="a Pending pod is reconciled only once no Allocate has come for this many seconds (the "
                         "kubelet allocates a pod container by container)")
    ap.add_argument("--topology-manager-policy", default="", choices=["", "none", "best-effort", "restricted", "single-numa-node"],
                    help="the kubelet's --topology-manager-policy, published as a node label so the extender picks "
                         "the devices the kubelet will offer ('' = read --kubelet-config, else none)")
    ap.add_argument("--topology-manager-scope", default="", choices=["", "container", "pod"],
                    help="the kubelet's --topology-manager-scope ('' = read --kubelet-config, else container)")
    ap.add_argument("--kubelet-config", default="/var/lib/kubelet/config.yaml",
                    help="KubeletConfiguration to read topologyManagerPolicy / topologyManagerScope from when the "
                         "flags above are not given (skipped when absent)")
    ap.add_argument("--reprobe-interval", type=float, default=0.0,
                    help="re-measure the links (child process) every N s while no pod holds a device; 0 = never")
    ap.add_argument("--reprobe-tolerance", type=float, default=0.15,
                    help="republish the topology when a measured pair moved by more than this fraction")
    ap.add_argument("--probe-mark-seconds", type=float, default=300.0,
                    help="a re-probe marks the node <prefix>/probing for at most this long; the extender skips it meanwhile")
    ap.add_argument("--probe-settle-seconds", type=float, default=2.0,
                    help="after marking, wait this long for binds already in flight before re-checking that the node is idle")
    ap.add_argument("--probe-yield-seconds", type=float, default=20.0,
                    help="an Allocate arriving mid-probe cancels it and waits at most this long for the GPUs to be released")
    ap.add_argument("--partition-aware", default="on", choices=["on", "off"],
                    help="GetPreferredAllocation on CPX/DPX/QPX nodes: group XCPs by physical GPU (on) or not (off)")
    ap.add_argument("--nic-env", default="on", choices=["on", "off"],
                    help="Allocate sets NCCL_IB_HCA / GTK_NICS to the RDMA NICs behind the allocated GPUs' PCIe switches")
    ap.add_argument("--gpu-events", default="auto", choices=["auto", "off"],
                    help="amdsmi GPU event notification (reset / VM fault / thermal throttle) on its own thread; "
                         "auto = on wherever amdsmi offers it")
    ap.add_argument("--time-slices", type=int, default=1,
                    help="advertise every (SPX) GPU as this many time slices: Gaia fractional requests on unpartitioned "
                         "nodes (a pod holding j slices holds j/S of one GPU; topology/shares.py); 1 = whole GPUs. "
                         "The node label <annotation-prefix>/time-slices overrides it per node")
    ap.add_argument("--label-check-interval", type=float, default=30.0,
                    help="seconds between checks of the node's time-slices label (a change restarts the plugin once idle)")
    ap.add_argument("--container-ipc-mode", default=None,
                    help="HSA_ENABLE_IPC_MODE_LEGACY for every allocated container (default: this plugin's own value, "
                         "0 in the rendered manifests; '' to set none). 0 lets RCCL's multi-process IPC work on hosts whose "
                         "driver exports IPC handles only as dma-bufs")
    ap.add_argument("--share-guard", default="preload", choices=["off", "env", "preload"],
                    help="--time-slices: mount and preload libgtk_vgpu.so into pods holding part of a GPU, which caps their HIP "
                         "allocations at the share's HBM and forces their CU mask (preload = an /etc/ld.so.preload mount plus "
                         "LD_PRELOAD, which survives a container that overrides its env; env = LD_PRELOAD only; "
                         "off = cooperative shares)")
    ap.add_argument("--share-guard-dir", default="/var/lib/gtk-vgpu",
                    help="host directory (hostPath, same path inside the DaemonSet) for the guard library and per-allocation configs")
    ap.add_argument("--share-cu-mask", default="on", choices=["on", "off"],
                    help="--time-slices: confine a pod holding part of a GPU to its slices' compute units (HSA_CU_MASK)")
    ap.add_argument("--partition-control", default="off", choices=["off", "on"],
                    help="switch the GPUs' compute / memory partition mode to what the node labels "
                         "<annotation-prefix>/compute-partition-request (SPX|DPX|QPX|CPX) and "
                         "memory-partition-request (NPS1|NPS4...) ask for, once no pod holds a device "
                         "(needs a privileged DaemonSet; deviceplugin/repartition.py)")
    ap.add_argument("--partition-driver-reload", action="store_true",
                    help="--partition-control: reload the amdgpu driver to complete a memory-partition change "
                         "(otherwise the new NPS mode waits for a reload by the operator)")
    ap.add_argument("--log-level", default="INFO")
    a = ap.parse_args(argv)
    logging.basicConfig(level=a.log_level, format='{"ts":"%(asctime)s","lvl":"%(levelname)s","mod":"%(name)s","msg":"%(message)s"}')
    log = logging.getLogger("gtk.deviceplugin")

    api = make_api(a.apiserver, a.token, a.ca_file, a.insecure_skip_tls_verify)
    contract = Contract(resource_name=a.resource_name, prefix=a.annotation_prefix, slice_resource=a.slice_resource_name)
    names = (a.resource_name, a.slice_resource_name, "aliyun.com/gpu", "aliyun.com/gpu-count")
    partition_control = a.partition_control == "on" and a.discovery in ("auto", "amdsmi") and api is not None

    def repartition_pass(idle_fn, wait, hold=None):
        from .repartition import repartition

        outcome, msg = repartition(api, a.node_name, contract, idle_fn, reload_driver=a.partition_driver_reload,
                                   settle_s=a.probe_settle_seconds, wait=wait, hold=hold,
                                   time_slices=node_time_slices(api, a.node_name, contract, a.time_slices))
        if outcome in ("ok", "partial", "failed", "invalid"):
            (log.warning if outcome != "ok" else log.info)("partition request: %s: %s", outcome, msg)
        return outcome, msg

    if partition_control:  # before discovery: the first registration already shows the new layout
        try:
            repartition_pass(lambda: node_is_idle(api, a.node_name, names), lambda s: (time.sleep(s), False)[1])
        except Exception as e:  # noqa: BLE001 - the node keeps its layout; the loop tries again
            log.warning("partition request at start-up failed: %s", e)
    a.time_slices, why = startup_time_slices(api, a.node_name, contract, a.time_slices,
                                             (a.resource_name, a.slice_resource_name, "aliyun.com/gpu", "aliyun.com/gpu-count"))
    if why:
        log.warning("%s", why)
    # Slicing needs SPX GPUs.  On a partitioned node the label's count cannot apply: the plugin
    # advertises the XCPs unsliced, and the label check below compares the label against what it
    # *could* apply (1), not against the label itself, so it never restarts for a count it cannot
    # honour (an exit-75 loop every label-check interval).
    partitioned = False
    if a.time_slices > 1:
        try:
            parts = discover(a.discovery, node_name=a.node_name, fake_n=a.fake_gpus)
            partitioned = any(g.physical != g.index for g in parts.gpus)
            if partitioned:
                log.error("time slices (%d per GPU) need SPX GPUs, and this node is partitioned (%s): advertising its "
                          "XCPs unsliced", a.time_slices, parts.gpus[0].partition)
                a.time_slices = 1
        except Exception as e:  # noqa: BLE001 - discovery fails again below, with its own error
            log.warning("discovery before slicing failed: %s", e)

    def applicable_slices(want: int) -> int:
        return 1 if partitioned else want
    unapplied_warned = False
    # a sliced node is a pool of its own: it registers its slices under the slice resource and
    # offers no whole GPUs (the extender's filter keeps the two kinds of request apart)
    advertised = a.slice_resource_name if a.time_slices > 1 else a.resource_name

    def node_topology():
        return time_slice(discover(a.discovery, node_name=a.node_name, fake_n=a.fake_gpus), a.time_slices)

    topo = node_topology()
    probe_fn = None
    if a.probe != "off" and a.discovery != "fake":
        # in a child process: the plugin lives as long as the node and must not hold HIP contexts
        # and probe buffers on every GPU it hands out to pods
        from ..ops.probe import probe_in_child

        def probe_fn():
            probed, msg = probe_in_child(a.probe, backend=a.discovery)
            log.info("probe: %s", msg)
            return None if probed is None else time_slice(probed, a.time_slices)
    topo, how = startup_topology(topo, api, a.node_name, contract, names, probe_fn)
    log.info("link matrix: %s; topology:\n%s", how, topo.render())

    health = HealthMonitor(topo, node_topology, HealthPolicy(xgmi_links=a.xgmi_link_loss == "unhealthy"))

    specs = a.device_specs if a.device_specs != "auto" else ("stub" if a.discovery == "fake" else "strict")
    tm = topology_manager_of(a)
    cfg = PluginConfig(resource_name=advertised, socket_dir=a.socket_dir, socket_name=a.socket_name, dev_root=a.dev_root,
                       node_name=a.node_name, contract=contract, device_specs=specs, prestart_validate=a.prestart_validate,
                       health_interval=a.health_interval, reprobe_interval=a.reprobe_interval,
                       reprobe_tolerance=a.reprobe_tolerance, pod_resources_socket=a.pod_resources_socket,
                       probe_mark_s=a.probe_mark_seconds, probe_settle_s=a.probe_settle_seconds,
                       probe_yield_s=a.probe_yield_seconds,
                       reconcile_interval=a.reconcile_interval, admission_settle_s=a.admission_settle, cdi_dir=a.cdi_dir, nic_env=a.nic_env == "on",
                       share_cu_mask=a.share_cu_mask == "on", share_guard=a.share_guard, guard_dir=a.share_guard_dir,
                       policy=PlacementPolicy(partition_aware=a.partition_aware == "on"), topology_manager=tm,
                       container_ipc_mode=a.container_ipc_mode)
    events = None
    if a.gpu_events == "auto" and a.discovery in ("auto", "amdsmi"):
        from .events import GpuEventWatcher

        events = GpuEventWatcher.try_open()
    reprobe = None
    if (a.reprobe_interval > 0 or events is not None) and a.discovery != "fake":
        from ..ops.probe import probe_in_child

        def reprobe(cancel=None):
            # an Allocate arriving mid-probe sets `cancel`: the probe child is killed and the pod's
            # container starts on released links (plugin.reprobe)
            probed = probe_in_child(a.probe if a.probe != "off" else "quick", backend=a.discovery, cancel=cancel)[0]
            return None if probed is None else time_slice(probed, a.time_slices)
    plugin = DevicePluginServer(topo, cfg, api=api, health_fn=health if a.discovery != "fake" else None, reprobe_fn=reprobe)
    plugin.event_source = events
    plugin.metrics.liveness = plugin.liveness  # /healthz: the DaemonSet's livenessProbe
    if a.metrics_port:
        from .metrics import serve_metrics

        serve_metrics(plugin.metrics, a.metrics_host, a.metrics_port)
    done = threading.Event()
    for sig in (signal.SIGINT, signal.SIGTERM):  # installed before serving: a stop never races start-up
        signal.signal(sig, lambda *_: done.set())
    plugin.poll_node()  # a cordoned GPU is never advertised Healthy, not even until the first label check
    plugin.start()
    ticks = 0
    while not done.wait(1.0):
        ticks += 1
        if ticks % max(1, int(a.label_check_interval)) == 0 and api is not None:
            # one GET of the node: the operator's GPU cordon (<prefix>/cordoned-gpus) and time-slice label
            node = plugin.poll_node()
            label = node_time_slices(api, a.node_name, contract, a.time_slices, node=node) if node is not None else a.time_slices
            want = applicable_slices(label)
            if want != label and not unapplied_warned:
                log.warning("node label asks for %d time slices per GPU; a partitioned node cannot be sliced, "
                            "so its XCPs stay unsliced (switch the node to SPX to apply the label)", label)
                unapplied_warned = True
            if want != a.time_slices:
                # device IDs change with the slicing: switch only when no pod holds a device, or the
                # running pods' GROUP annotations would name devices of the old layout
                if plugin.node_idle():
                    plugin.layout_change_reason = f"time slices per GPU {a.time_slices} -> {want} (node label)"
                    plugin.layout_change.set()
                elif ticks % 300 == 0:
                    log.warning("time slices per GPU %d -> %d requested by the node label; waiting until no pod holds a device",
                                a.time_slices, want)
        if partition_control and ticks % max(1, int(a.label_check_interval)) == 0 and not plugin.layout_change.is_set():
            if not plugin.maintenance.acquire(blocking=False):
                outcome, msg = "busy", "a link re-probe holds the GPUs"
            else:
                try:
                    outcome, msg = repartition_pass(plugin.node_idle, done.wait, plugin.allocation_hold)
                except Exception as e:  # noqa: BLE001 - reported; the next pass tries again
                    outcome, msg = "error", str(e)
                    log.warning("partition request: %s", e)
                finally:
                    plugin.maintenance.release()
            if outcome not in ("none", "same"):
                plugin.metrics.partition_changes.labels(outcome).inc()
            if outcome in ("ok", "partial"):  # the device layout changed: re-register it
                plugin.layout_change_reason = f"GPU partitions {msg} (node label)"
                plugin.layout_change.set()
            elif outcome == "busy" and ticks % 300 == 0:
                log.warning("partition request: %s", msg)
        if plugin.layout_change.is_set():  # partition switch / device hot-(un)plug / new slicing: restart cleanly
            log.warning("exiting for a restart: %s", plugin.layout_change_reason)
            # the published layout is stale until the restarted plugin publishes the new one (and
            # clears this mark): the extender keeps away from the node meanwhile
            plugin._mark_probing(time.time() + a.probe_mark_seconds)
            plugin.stop()
            return 75  # EX_TEMPFAIL: the DaemonSet restarts the container, which re-discovers
    plugin.stop()
    return 0


def topology_manager_of(a) -> "TopologyManager":
    """The node's Topology Manager: the flags, else the kubelet's config file, else ``none``."""
    from ..placement.numa_align import TopologyManager, read_kubelet_config

    base = TopologyManager()
    if (not a.topology_manager_policy or not a.topology_manager_scope) and a.kubelet_config and os.path.exists(a.kubelet_config):
        try:
            base = read_kubelet_config(a.kubelet_config)
        except Exception as e:  # noqa: BLE001 - an unreadable or malformed file must not stop the plugin
            logging.getLogger("gtk.deviceplugin").warning("reading the topology manager from %s failed: %s", a.kubelet_config, e)
    return TopologyManager(a.topology_manager_policy or base.policy, a.topology_manager_scope or base.scope)


if __name__ == "__main__":
    sys.exit(main())

