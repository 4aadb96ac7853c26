"""Scheduler configuration generators and deploy-manifest rendering.

* :func:`legacy_policy` — the reference's kube-scheduler ``Policy`` JSON (``design.md:92-113``):
  one extender at ``http://127.0.0.1:32743/gputopology-scheduler`` with ``PrioritizeVerb: sort``,
  ``bindVerb: bind``, ``nodeCacheCapable: true``, managed resource ``aliyun.com/gpu``.  Policy was
  removed in Kubernetes 1.23, so this is only for old clusters.
* :func:`scheduler_configuration` — the same extender as a ``KubeSchedulerConfiguration``
  (``kubescheduler.config.k8s.io/v1``) ``extenders:`` stanza for current clusters, optionally with
  the ``filter`` and ``preempt`` verbs this framework adds.
* :func:`render_manifests` — DaemonSet (device plugin, Prometheus ``/metrics`` on :32744), DaemonSet
  (extender on every control-plane node's host network, listening on 127.0.0.1 only: each
  kube-scheduler replica calls its own node's extender on loopback, and ``/bind`` is unauthenticated,
  so no Service exposes it), RBAC and the scheduler ConfigMap, as one multi-document YAML (``deploy/``).
"""
from __future__ import annotations

import json
from typing import Any, Dict, List, Optional

import yaml

from .extender.server import DEFAULT_PORT, DEFAULT_PREFIX
from .k8s.annotations import COMPAT_RESOURCE, DEFAULT_RESOURCE, DEFAULT_SLICE_RESOURCE

__all__ = ["legacy_policy", "scheduler_configuration", "render_manifests", "render_kind", "extender_url"]

NAMESPACE = "kube-system"
PLUGIN_METRICS_PORT = 32744
IMAGE = "rocm/gpu-topology-k8s:latest"


def extender_url(host: str = "127.0.0.1", port: int = DEFAULT_PORT, prefix: str = DEFAULT_PREFIX, https: bool = False) -> str:
    return f"{'https' if https else 'http'}://{host}:{port}{prefix}"


def legacy_policy(resource: str = COMPAT_RESOURCE, url: Optional[str] = None, with_filter: bool = False) -> Dict[str, Any]:
    ext: Dict[str, Any] = {
        "urlPrefix": url or extender_url(),
        "PrioritizeVerb": "sort",
        "bindVerb": "bind",
        "enableHttps": False,
        "nodeCacheCapable": True,
        "managedResources": [{"name": resource, "ignoredByScheduler": False}],
        "ignorable": False,
    }
    if with_filter:
        ext["filterVerb"] = "filter"
    return {"kind": "Policy", "apiVersion": "v1", "extenders": [ext]}


def scheduler_configuration(resource: str = DEFAULT_RESOURCE, url: Optional[str] = None, with_filter: bool = True,
                            scheduler_name: str = "default-scheduler", weight: int = 5,
                            extra_resources: Optional[List[str]] = None, with_preempt: bool = True,
                            tls_dir: Optional[str] = None, slice_resource: str = DEFAULT_SLICE_RESOURCE) -> Dict[str, Any]:
    """``tls_dir``: call the extender over mutual TLS (its ``--tls-cert/--tls-key/--client-ca``) with
    the scheduler's client certificate ``tls.crt``/``tls.key`` and the CA ``ca.crt`` from that directory.
    Both pools are managed: whole GPUs (``resource``) and the time slices of sliced nodes
    (``slice_resource``, topology/shares.py), so the scheduler sends pods of either to the extender."""
    names = [resource] + ([slice_resource] if slice_resource else []) + list(extra_resources or [])
    managed = [{"name": r, "ignoredByScheduler": False} for r in dict.fromkeys(names)]
    ext: Dict[str, Any] = {
        "urlPrefix": url or (extender_url().replace("http://", "https://", 1) if tls_dir else extender_url()),
        "prioritizeVerb": "sort",
        "bindVerb": "bind",
        "weight": weight,
        "enableHTTPS": False,
        "nodeCacheCapable": True,
        "managedResources": managed,
        "ignorable": False,
        "httpTimeout": "30s",
    }
    if tls_dir:
        d = tls_dir.rstrip("/")
        ext["enableHTTPS"] = True
        ext["tlsConfig"] = {"certFile": f"{d}/tls.crt", "keyFile": f"{d}/tls.key", "caFile": f"{d}/ca.crt"}
    if with_filter:
        ext["filterVerb"] = "filter"
    if with_preempt:  # topology-aware victim selection (extender/scheduler.py TopologyExtender.preempt)
        ext["preemptVerb"] = "preempt"
    return {
        "apiVersion": "kubescheduler.config.k8s.io/v1",
        "kind": "KubeSchedulerConfiguration",
        "profiles": [{"schedulerName": scheduler_name}],
        "extenders": [ext],
    }


PLUGIN_SA = "gpu-topology-device-plugin"
EXTENDER_SA = "gpu-topology-extender"
NODE_NAME_CLAIM = "authentication.kubernetes.io/node-name"


def rbac_manifests(namespace: str = NAMESPACE) -> List[Dict[str, Any]]:
    """Least-privilege identities: the privileged node agent and the binder no
    longer share one ServiceAccount.

    * ``gpu-topology-device-plugin`` (every GPU node, privileged): reads pods and its node, patches pod
      annotations (ASSIGNED / GROUP at Allocate, ``design.md:236-246``) and its node's annotations and
      labels (topology publication, ``design.md:76-82``), records Events.  No ``pods/binding``, no
      Leases.  A ``ValidatingAdmissionPolicy`` confines its writes to ITS node — the node named by the
      ``authentication.kubernetes.io/node-name`` claim of its pod-bound token (k8s >= 1.30) — and the
      pods bound there, and lets it change only the node's metadata.  A compromised GPU node can then
      neither bind pods nor relabel, taint or annotate another node.
    * ``gpu-topology-extender`` (control plane): reads nodes and pods, patches pod annotations,
      creates ``pods/binding`` (``design.md:119,223-232``), records Events, and keeps the allocation
      ledger in Leases of its own namespace (a Role there, not cluster-wide; extender/ledger.py).  It
      holds no write access to Nodes."""
    core, coord = "", "coordination.k8s.io"

    def role(kind, name, rules, ns=None):
        md = {"name": name, **({"namespace": ns} if ns else {})}
        return {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": kind, "metadata": md, "rules": rules}

    def binding(kind, name, role_kind, sa, ns=None):
        md = {"name": name, **({"namespace": ns} if ns else {})}
        return {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": kind, "metadata": md,
                "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": role_kind, "name": name},
                "subjects": [{"kind": "ServiceAccount", "name": sa, "namespace": namespace}]}

    plugin_user = f"system:serviceaccount:{namespace}:{PLUGIN_SA}"
    vap = {
        "apiVersion": "admissionregistration.k8s.io/v1",
        "kind": "ValidatingAdmissionPolicy",
        "metadata": {"name": "gpu-topology-device-plugin-own-node"},
        "spec": {
            "failurePolicy": "Fail",
            "matchConstraints": {"resourceRules": [{"apiGroups": [core], "apiVersions": ["v1"], "operations": ["UPDATE"],
                                                    "resources": ["nodes", "pods"]}]},
            "matchConditions": [{"name": "device-plugin", "expression": f"request.userInfo.username == '{plugin_user}'"}],
            "validations": [
                {"expression": f"'{NODE_NAME_CLAIM}' in request.userInfo.extra && "
                               f"(request.kind.kind == 'Node' ? object.metadata.name : object.spec.nodeName) == "
                               f"request.userInfo.extra['{NODE_NAME_CLAIM}'][0]",
                 "message": "the GPU device plugin may only change its own node and the pods bound to it"},
                {"expression": "request.kind.kind != 'Node' || object.spec == oldObject.spec",
                 "message": "the GPU device plugin may only change node metadata (annotations, labels)"},
            ],
        },
    }
    return [
        {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": PLUGIN_SA, "namespace": namespace}},
        {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": EXTENDER_SA, "namespace": namespace}},
        role("ClusterRole", PLUGIN_SA, [
            {"apiGroups": [core], "resources": ["nodes"], "verbs": ["get", "patch"]},
            {"apiGroups": [core], "resources": ["pods"], "verbs": ["get", "list", "watch", "patch"]},
            {"apiGroups": [core], "resources": ["events"], "verbs": ["create", "patch"]},
        ]),
        binding("ClusterRoleBinding", PLUGIN_SA, "ClusterRole", PLUGIN_SA),
        vap,
        {"apiVersion": "admissionregistration.k8s.io/v1", "kind": "ValidatingAdmissionPolicyBinding",
         "metadata": {"name": "gpu-topology-device-plugin-own-node"},
         "spec": {"policyName": "gpu-topology-device-plugin-own-node", "validationActions": ["Deny"]}},
        role("ClusterRole", EXTENDER_SA, [
            {"apiGroups": [core], "resources": ["nodes"], "verbs": ["get", "list", "watch"]},
            {"apiGroups": [core], "resources": ["pods"], "verbs": ["get", "list", "watch", "patch"]},
            {"apiGroups": [core], "resources": ["pods/binding"], "verbs": ["create"]},
            {"apiGroups": [core], "resources": ["events"], "verbs": ["create", "patch"]},
        ]),
        binding("ClusterRoleBinding", EXTENDER_SA, "ClusterRole", EXTENDER_SA),
        role("Role", f"{EXTENDER_SA}-ledger", [
            {"apiGroups": [coord], "resources": ["leases"], "verbs": ["get", "list", "watch", "create", "patch"]},
        ], ns=namespace),
        binding("RoleBinding", f"{EXTENDER_SA}-ledger", "Role", EXTENDER_SA, ns=namespace),
    ]


def render_manifests(resource: str = DEFAULT_RESOURCE, image: str = IMAGE, namespace: str = NAMESPACE,
                     probe: str = "quick", policy: str = "exact", time_slices: int = 1, partition_control: bool = False,
                     topology_manager_policy: str = "", topology_manager_scope: str = "") -> str:
    """The DaemonSets, RBAC and scheduler config.  ``time_slices > 1``: the device plugin advertises
    every GPU as that many time slices (fractional pods; topology/shares.py).  ``partition_control``:
    the plugin switches compute / memory partition modes on the node labels' request
    (deviceplugin/repartition.py), which writes the GPUs' sysfs, so /sys is mounted writable.
    ``topology_manager_policy`` / ``_scope``: the GPU nodes' kubelet ``--topology-manager-policy`` /
    ``--topology-manager-scope``, handed to the plugin, which publishes them for the extender
    (placement/numa_align.py); the kubelet's own config file is not mounted (its directory holds the
    pods' volumes)."""
    labels = {"app.kubernetes.io/part-of": "gpu-topology-amd"}
    docs: List[Dict[str, Any]] = rbac_manifests(namespace)
    plugin_sa, ext_sa = PLUGIN_SA, EXTENDER_SA
    docs += [
        {
            "apiVersion": "apps/v1",
            "kind": "DaemonSet",
            "metadata": {"name": "amd-gpu-topology-device-plugin", "namespace": namespace, "labels": labels},
            "spec": {
                "selector": {"matchLabels": {"name": "amd-gpu-topology-device-plugin"}},
                "template": {
                    "metadata": {"labels": {"name": "amd-gpu-topology-device-plugin", **labels}},
                    "spec": {
                        "serviceAccountName": plugin_sa,
                        "priorityClassName": "system-node-critical",
                        "nodeSelector": {"feature.node.kubernetes.io/amd-gpu": "true"},
                        "tolerations": [{"key": "amd.com/gpu", "operator": "Exists", "effect": "NoSchedule"}],
                        "containers": [{
                            "name": "device-plugin",
                            "image": image,
                            "command": ["python3", "-m", "gpu_topology_on_k8s_amd.deviceplugin",
                                        f"--resource-name={resource}", f"--probe={probe}", "--discovery=auto",
                                        "--reprobe-interval=3600", "--prestart-validate", f"--metrics-port={PLUGIN_METRICS_PORT}"]
                                       + ([f"--time-slices={int(time_slices)}"] if int(time_slices) > 1 else [])
                                       + (["--partition-control=on"] if partition_control else [])
                                       + ([f"--topology-manager-policy={topology_manager_policy}"] if topology_manager_policy else [])
                                       + ([f"--topology-manager-scope={topology_manager_scope}"] if topology_manager_scope else []),
                            "ports": [{"containerPort": PLUGIN_METRICS_PORT, "name": "metrics"}],
                            # /healthz fails when the gRPC server is down, the monitor loop is wedged or
                            # re-registration keeps failing (DevicePluginServer.liveness); start-up (discovery,
                            # link probe, a requested partition switch) gets up to 15 min before liveness counts
                            "startupProbe": {"httpGet": {"path": "/healthz", "port": PLUGIN_METRICS_PORT},
                                             "periodSeconds": 10, "failureThreshold": 90},
                            "livenessProbe": {"httpGet": {"path": "/healthz", "port": PLUGIN_METRICS_PORT},
                                              "periodSeconds": 30, "failureThreshold": 4},
                            "resources": {"requests": {"cpu": "100m", "memory": "256Mi"}, "limits": {"memory": "2Gi"}},
                            "env": [{"name": "NODE_NAME", "valueFrom": {"fieldRef": {"fieldPath": "spec.nodeName"}}},
                                    # the probe / validator children share GPU buffers across processes;
                                    # the amdgpu host driver exports IPC handles only as dma-bufs, which ROCr
                                    # uses with the legacy KFD IPC path off (docs/OPERATIONS.md "IPC")
                                    {"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"}],
                            "securityContext": {"privileged": True},
                            "volumeMounts": [
                                {"name": "device-plugins", "mountPath": "/var/lib/kubelet/device-plugins"},
                                # kubelet pod-resources API: which pod holds which device (GROUP reconcile)
                                {"name": "pod-resources", "mountPath": "/var/lib/kubelet/pod-resources", "readOnly": True},
                                {"name": "sys", "mountPath": "/sys", "readOnly": not partition_control},
                                {"name": "dev", "mountPath": "/dev"},
                                # time-sliced shares: the vGPU guard library + per-allocation configs the
                                # plugin writes here are bind-mounted into pods by Allocate (host path = this path)
                                {"name": "vgpu-guard", "mountPath": "/var/lib/gtk-vgpu"},
                            ],
                        }],
                        "volumes": [
                            {"name": "device-plugins", "hostPath": {"path": "/var/lib/kubelet/device-plugins"}},
                            {"name": "pod-resources", "hostPath": {"path": "/var/lib/kubelet/pod-resources"}},
                            {"name": "vgpu-guard", "hostPath": {"path": "/var/lib/gtk-vgpu", "type": "DirectoryOrCreate"}},
                            {"name": "sys", "hostPath": {"path": "/sys"}},
                            {"name": "dev", "hostPath": {"path": "/dev"}},
                        ],
                    },
                },
            },
        },
        {
            "apiVersion": "apps/v1",
            # one extender per control-plane node: every kube-scheduler replica calls ITS node's
            # 127.0.0.1:32743 (design.md:98); leader election keeps one scheduler (hence one extender)
            # active, and a new leader's extender rebuilds its state from the pod annotations
            "kind": "DaemonSet",
            "metadata": {"name": "gpu-topology-scheduler-extender", "namespace": namespace, "labels": labels},
            "spec": {
                "selector": {"matchLabels": {"name": "gpu-topology-scheduler-extender"}},
                "template": {
                    "metadata": {"labels": {"name": "gpu-topology-scheduler-extender", **labels}},
                    "spec": {
                        "serviceAccountName": ext_sa,
                        "hostNetwork": True,  # kube-scheduler reaches it on 127.0.0.1:32743 (design.md:98)
                        "nodeSelector": {"node-role.kubernetes.io/control-plane": ""},
                        "tolerations": [{"key": "node-role.kubernetes.io/control-plane", "operator": "Exists",
                                         "effect": "NoSchedule"}],
                        "containers": [{
                            "name": "extender",
                            "image": image,
                            "command": ["python3", "-m", "gpu_topology_on_k8s_amd.extender", f"--resource-name={resource}",
                                        "--host=127.0.0.1", f"--port={DEFAULT_PORT}", f"--policy={policy}", "--informer=on",
                                        "--scheduler-names=default-scheduler", "--ledger-store=lease",
                                        f"--ledger-namespace={namespace}"],
                            # ready once the informer has listed the cluster (filter / sort decline GPU pods before)
                            "readinessProbe": {"httpGet": {"host": "127.0.0.1", "path": "/readyz", "port": DEFAULT_PORT}},
                            "livenessProbe": {"httpGet": {"host": "127.0.0.1", "path": "/healthz", "port": DEFAULT_PORT}},
                            "resources": {"requests": {"cpu": "200m", "memory": "256Mi"}, "limits": {"memory": "2Gi"}},
                        }],
                    },
                },
            },
        },
        {
            "apiVersion": "v1",
            "kind": "ConfigMap",
            "metadata": {"name": "gpu-topology-scheduler-config", "namespace": namespace},
            "data": {
                "scheduler-config.yaml": yaml.safe_dump(scheduler_configuration(resource), sort_keys=False),
                "policy.json": json.dumps(legacy_policy(), indent=2),
            },
        },
    ]
    return yaml.safe_dump_all(docs, sort_keys=False)


def render_kind(resource: str = DEFAULT_RESOURCE, image: str = IMAGE, fake_gpus: int = 2) -> Dict[str, str]:
    """BASELINE config 1 — a kind cluster whose worker advertises ``fake_gpus`` fake CPU-backed GPUs
    and a pod that requests one.  Files (``deploy/kind/``):

    * ``kind-config.yaml`` — 1 control plane + 1 worker; the scheduler config is mounted into the
      control-plane node and passed to kube-scheduler (``--config``) through a kubeadm patch;
    * ``gpu-topology-kind.yaml`` — the manifests of :func:`render_manifests` with the device plugin in
      fake-discovery / stub-DeviceSpec mode: a kind node has no ``/dev/kfd`` or render nodes, so
      Allocate returns envs + annotations only and containerd never sees a missing host path;
    * ``pod-1gpu.yaml`` — the test pod; ``up.sh`` wires it together (needs docker + kind + kubectl).
    """
    docs = list(yaml.safe_load_all(render_manifests(resource, image=image, probe="off")))
    for d in docs:
        if d["kind"] == "DaemonSet" and d["metadata"]["name"] == "amd-gpu-topology-device-plugin":
            spec = d["spec"]["template"]["spec"]
            spec["nodeSelector"] = {"gputopology.amd.com/fake-gpus": "true"}
            c = spec["containers"][0]
            c["command"] = ["python3", "-m", "gpu_topology_on_k8s_amd.deviceplugin", f"--resource-name={resource}", "--discovery=fake",
                            f"--fake-gpus={fake_gpus}", "--probe=off", "--device-specs=stub", f"--metrics-port={PLUGIN_METRICS_PORT}"]
            c.pop("securityContext", None)
            c["volumeMounts"] = [m for m in c["volumeMounts"] if m["name"] in ("device-plugins", "pod-resources")]
            spec["volumes"] = [v for v in spec["volumes"] if v["name"] in ("device-plugins", "pod-resources")]
    kind_cfg = {
        "kind": "Cluster",
        "apiVersion": "kind.x-k8s.io/v1alpha4",
        "nodes": [
            {
                "role": "control-plane",
                "extraMounts": [{"hostPath": "./scheduler-config.yaml", "containerPath": "/etc/kubernetes/gpu-topology/scheduler-config.yaml",
                                 "readOnly": True}],
                "kubeadmConfigPatches": [yaml.safe_dump({
                    "kind": "ClusterConfiguration",
                    "scheduler": {
                        "extraArgs": {"config": "/etc/kubernetes/gpu-topology/scheduler-config.yaml"},
                        "extraVolumes": [{"name": "gpu-topology", "hostPath": "/etc/kubernetes/gpu-topology",
                                          "mountPath": "/etc/kubernetes/gpu-topology", "readOnly": True, "pathType": "Directory"}],
                    },
                }, sort_keys=False)],
            },
            {"role": "worker", "labels": {"gputopology.amd.com/fake-gpus": "true"}},
        ],
    }
    pod = {
        "apiVersion": "v1",
        "kind": "Pod",
        "metadata": {"name": "gpu-topology-smoke", "namespace": "default"},
        "spec": {
            "restartPolicy": "Never",
            "containers": [{"name": "c", "image": "busybox:1.36", "command": ["sh", "-c", "env | grep GTK_ && sleep 5"],
                            "resources": {"limits": {resource: "1"}}}],
        },
    }
    half = {  # a fractional pod (Gaia Fragment): half of one GPU on a time-sliced node (docs/SHARES.md)
        "apiVersion": "v1",
        "kind": "Pod",
        "metadata": {"name": "gpu-topology-half", "namespace": "default",
                     "annotations": {"gputopology.amd.com/gpu-fraction": "0.5"}},
        "spec": {
            "restartPolicy": "Never",
            # a sliced node advertises its slices as their own resource (whole GPUs stay amd.com/gpu);
            # on a 2-slice node one slice is half a GPU
            "containers": [{"name": "c", "image": "busybox:1.36",
                            "command": ["sh", "-c", "env | grep -E 'GTK_|HSA_CU_MASK' && sleep 5"],
                            "resources": {"limits": {DEFAULT_SLICE_RESOURCE: "1"}}}],
        },
    }
    up = "\n".join([
        "#!/usr/bin/env bash",
        "# BASELINE config 1: kind + 2 fake GPUs; the pod must reach Succeeded with GTK_GPU_GROUP set.",
        "set -euo pipefail",
        'cd "$(dirname "$0")"',
        "kind create cluster --name gpu-topology --config kind-config.yaml",
        f"kind load docker-image --name gpu-topology {image}",
        "kubectl apply -f gpu-topology-kind.yaml",
        "kubectl -n kube-system rollout status ds/amd-gpu-topology-device-plugin --timeout=180s",
        "kubectl -n kube-system rollout status ds/gpu-topology-scheduler-extender --timeout=180s",
        "kubectl apply -f pod-1gpu.yaml",
        "kubectl wait --for=jsonpath='{.status.phase}'=Succeeded pod/gpu-topology-smoke --timeout=180s",
        "kubectl get pod gpu-topology-smoke -o jsonpath='{.metadata.annotations}'; echo",
        "kubectl logs gpu-topology-smoke",
        "",
    ])
    return {
        "kind-config.yaml": yaml.safe_dump(kind_cfg, sort_keys=False),
        "scheduler-config.yaml": yaml.safe_dump(scheduler_configuration(resource), sort_keys=False),
        "gpu-topology-kind.yaml": yaml.safe_dump_all(docs, sort_keys=False),
        "pod-1gpu.yaml": yaml.safe_dump(pod, sort_keys=False),
        # after `kubectl label node <worker> gputopology.amd.com/time-slices=2` (the plugin restarts with 2 slices per GPU)
        "pod-half-gpu.yaml": yaml.safe_dump(half, sort_keys=False),
        "up.sh": up,
    }


def prometheus_rules(namespace: str = NAMESPACE) -> Dict[str, Any]:
    """A ``PrometheusRule`` (prometheus-operator) with the alerts an operator of this framework needs.
    Every expression uses only metrics the plugin and the extender export (tests/test_alerts.py
    checks them against live expositions)."""
    def alert(name, expr, for_, severity, summary, action):
        return {"alert": name, "expr": expr, "for": for_, "labels": {"severity": severity},
                "annotations": {"summary": summary, "description": action}}

    extender = [
        alert("GPUTopologyExtenderNotSynced", "max(gtk_extender_informer_synced) == 0", "5m", "critical",
              "The extender's informer has not listed nodes and pods",
              "Sort and bind answer from an empty or stale view. Check the extender's apiserver access "
              "(RBAC: nodes/pods list+watch, leases in its namespace) and its log."),
        alert("GPUTopologyExtenderRelisting", "sum by (kind) (increase(gtk_extender_informer_lists_total[1h])) > 2", "0m",
              "warning", "The extender relisted {{ $labels.kind }} more than twice in an hour",
              "Each relist is a full LIST (seconds and hundreds of MB at 100,000 pods). Watches are falling out of the "
              "apiserver's window (410): check apiserver load and --list-page-size."),
        alert("GPUTopologyExtenderWatchErrors", "sum(rate(gtk_extender_informer_watch_errors_total[10m])) > 0.05", "15m",
              "warning", "The extender's watches keep breaking",
              "Watches are resumed without relisting, but a steady error rate means a flaky apiserver path (LB idle "
              "timeouts, APF throttling)."),
        alert("GPUTopologyBindAborts", "sum by (reason) (increase(gtk_extender_bind_aborts_total[15m])) > 0", "0m", "warning",
              "Binds gave up ({{ $labels.reason }})",
              "budget: ledger conflicts kept re-deciding a bind (many replicas racing on one node); ledger_grace: a pod "
              "PATCH took longer than 15 s (apiserver throttling). kube-scheduler retries the pods."),
        alert("GPUTopologyLedgerConflicts", "sum(rate(gtk_extender_ledger_conflicts_total[5m])) > 1", "15m", "info",
              "Extender replicas keep colliding on the same nodes",
              "Conflicts are safe (the loser re-decides) but cost latency; fewer replicas or a scheduler leader "
              "election reduce them."),
        alert("GPUTopologyFragmented",
              "max(gtk_extender_placeable_nodes{k=\"8\"}) == 0 and sum(gtk_extender_node_free_devices) >= 8", "30m", "info",
              "No node can host an 8-GPU pod although 8 or more GPUs are free",
              "Free GPUs are scattered. `gtk defrag --size 8` plans the fewest pod moves that free a node."),
    ]
    plugin = [
        alert("GPUTopologyKubeletOverridesGroups", "sum by (pod) (increase(gtk_plugin_group_overridden_total[1h])) > 0", "0m",
              "warning", "The kubelet allocated other GPUs than the extender bound ({{ $labels.pod }})",
              "Usually the node's kubelet runs a Topology Manager policy the device plugin was not told about: pass "
              "--topology-manager-policy / --topology-manager-scope (`gtk doctor` names them)."),
        alert("GPUTopologyDeviceUnhealthy",
              "count by (pod) (gtk_plugin_device_healthy == 0) > on (pod) (max by (pod) (gtk_plugin_cordoned_devices))",
              "10m", "warning", "GPUs are Unhealthy beyond the ones the operator cordoned ({{ $labels.pod }})",
              "RAS errors, a reset in progress or a lost xGMI link (see the node's GPUUnhealthy Events)."),
        alert("GPUTopologyAllocateRefused",
              "sum by (pod, outcome) (increase(gtk_plugin_allocations_total{outcome=~\"invalid|unhealthy|missing|stale_layout\"}[15m])) > 0",
              "0m", "critical", "Allocate refused pods ({{ $labels.outcome }}) on {{ $labels.pod }}",
              "The kubelet does not retry a refused Allocate: those pods ended Failed (UnexpectedAdmissionError)."),
        alert("GPUTopologyPlacementValidationFailed",
              "sum by (pod) (increase(gtk_plugin_placement_validations_total{result!=\"ok\"}[1h])) > 0", "0m", "warning",
              "The pre-start RCCL all-reduce failed on a placement ({{ $labels.pod }})",
              "A container did not start because its GPUs failed the collective (FailedGPUPlacementValidation Events)."),
        alert("GPUTopologyPluginNotRegistered", "max by (pod) (gtk_plugin_registrations_total) == 0", "10m", "critical",
              "The device plugin never registered with the kubelet ({{ $labels.pod }})",
              "The node advertises no GPUs. Check the device-plugins hostPath mount and the kubelet."),
    ]
    return {"apiVersion": "monitoring.coreos.com/v1", "kind": "PrometheusRule",
            "metadata": {"name": "gpu-topology-amd", "namespace": namespace, "labels": {"app.kubernetes.io/part-of": "gpu-topology-amd"}},
            "spec": {"groups": [{"name": "gpu-topology-extender", "rules": extender},
                                {"name": "gpu-topology-device-plugin", "rules": plugin}]}}
