"""Scheduler configuration generators and deploy-manifest rendering.

* :func:`legacy_policy` — the reference's kube-scheduler ``Policy`` JSON (``design.md:92-113``):
  one extender at ``http://127.0.0.1:32743/gputopology-scheduler`` with ``PrioritizeVerb: sort``,
  ``bindVerb: bind``, ``nodeCacheCapable: true``, managed resource ``aliyun.com/gpu``.  Policy was
  removed in Kubernetes 1.23, so this is only for old clusters.
* :func:`scheduler_configuration` — the same extender as a ``KubeSchedulerConfiguration``
  (``kubescheduler.config.k8s.io/v1``) ``extenders:`` stanza for current clusters, optionally with
  the ``filter`` verb this framework adds.
* :func:`render_manifests` — DaemonSet (device plugin), Deployment + Service (extender), RBAC and
  the scheduler ConfigMap, as one multi-document YAML (``deploy/``).
"""
from __future__ import annotations

import json
from typing import Any, Dict, List, Optional

import yaml

from .extender.server import DEFAULT_PORT, DEFAULT_PREFIX
from .k8s.annotations import COMPAT_RESOURCE, DEFAULT_RESOURCE

__all__ = ["legacy_policy", "scheduler_configuration", "render_manifests", "extender_url"]

NAMESPACE = "kube-system"
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
                            extra_resources: Optional[List[str]] = None) -> Dict[str, Any]:
    managed = [{"name": r, "ignoredByScheduler": False} for r in [resource] + list(extra_resources or [])]
    ext: Dict[str, Any] = {
        "urlPrefix": url or extender_url(),
        "prioritizeVerb": "sort",
        "bindVerb": "bind",
        "weight": weight,
        "enableHTTPS": False,
        "nodeCacheCapable": True,
        "managedResources": managed,
        "ignorable": False,
        "httpTimeout": "30s",
    }
    if with_filter:
        ext["filterVerb"] = "filter"
    return {
        "apiVersion": "kubescheduler.config.k8s.io/v1",
        "kind": "KubeSchedulerConfiguration",
        "profiles": [{"schedulerName": scheduler_name}],
        "extenders": [ext],
    }


def render_manifests(resource: str = DEFAULT_RESOURCE, image: str = IMAGE, namespace: str = NAMESPACE,
                     probe: str = "quick", policy: str = "exact") -> str:
    sa = "gpu-topology"
    labels = {"app.kubernetes.io/part-of": "gpu-topology-amd"}
    docs: List[Dict[str, Any]] = [
        {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": sa, "namespace": namespace}},
        {
            "apiVersion": "rbac.authorization.k8s.io/v1",
            "kind": "ClusterRole",
            "metadata": {"name": "gpu-topology"},
            "rules": [
                {"apiGroups": [""], "resources": ["nodes"], "verbs": ["get", "list", "watch", "patch"]},
                {"apiGroups": [""], "resources": ["pods"], "verbs": ["get", "list", "watch", "patch", "update"]},
                {"apiGroups": [""], "resources": ["pods/binding", "bindings"], "verbs": ["create"]},
                {"apiGroups": [""], "resources": ["events"], "verbs": ["create", "patch"]},
            ],
        },
        {
            "apiVersion": "rbac.authorization.k8s.io/v1",
            "kind": "ClusterRoleBinding",
            "metadata": {"name": "gpu-topology"},
            "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": "gpu-topology"},
            "subjects": [{"kind": "ServiceAccount", "name": sa, "namespace": namespace}],
        },
        {
            "apiVersion": "apps/v1",
            "kind": "DaemonSet",
            "metadata": {"name": "amd-gpu-topology-device-plugin", "namespace": namespace, "labels": labels},
            "spec": {
                "selector": {"matchLabels": {"name": "amd-gpu-topology-device-plugin"}},
                "template": {
                    "metadata": {"labels": {"name": "amd-gpu-topology-device-plugin", **labels}},
                    "spec": {
                        "serviceAccountName": sa,
                        "priorityClassName": "system-node-critical",
                        "nodeSelector": {"feature.node.kubernetes.io/amd-gpu": "true"},
                        "tolerations": [{"key": "amd.com/gpu", "operator": "Exists", "effect": "NoSchedule"}],
                        "containers": [{
                            "name": "device-plugin",
                            "image": image,
                            "command": ["python3", "-m", "gpu_topology_on_k8s_amd.deviceplugin",
                                        f"--resource-name={resource}", f"--probe={probe}", "--discovery=auto",
                                        "--reprobe-interval=3600"],
                            "env": [{"name": "NODE_NAME", "valueFrom": {"fieldRef": {"fieldPath": "spec.nodeName"}}},
                                    {"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"}],
                            "securityContext": {"privileged": True},
                            "volumeMounts": [
                                {"name": "device-plugins", "mountPath": "/var/lib/kubelet/device-plugins"},
                                {"name": "sys", "mountPath": "/sys", "readOnly": True},
                                {"name": "dev", "mountPath": "/dev"},
                            ],
                        }],
                        "volumes": [
                            {"name": "device-plugins", "hostPath": {"path": "/var/lib/kubelet/device-plugins"}},
                            {"name": "sys", "hostPath": {"path": "/sys"}},
                            {"name": "dev", "hostPath": {"path": "/dev"}},
                        ],
                    },
                },
            },
        },
        {
            "apiVersion": "apps/v1",
            "kind": "Deployment",
            "metadata": {"name": "gpu-topology-scheduler-extender", "namespace": namespace, "labels": labels},
            "spec": {
                "replicas": 1,
                "selector": {"matchLabels": {"name": "gpu-topology-scheduler-extender"}},
                "template": {
                    "metadata": {"labels": {"name": "gpu-topology-scheduler-extender", **labels}},
                    "spec": {
                        "serviceAccountName": sa,
                        "hostNetwork": True,  # kube-scheduler reaches it on 127.0.0.1:32743 (design.md:98)
                        "nodeSelector": {"node-role.kubernetes.io/control-plane": ""},
                        "tolerations": [{"key": "node-role.kubernetes.io/control-plane", "operator": "Exists",
                                         "effect": "NoSchedule"}],
                        "containers": [{
                            "name": "extender",
                            "image": image,
                            "command": ["python3", "-m", "gpu_topology_on_k8s_amd.extender", f"--resource-name={resource}",
                                        f"--port={DEFAULT_PORT}", f"--policy={policy}"],
                            "ports": [{"containerPort": DEFAULT_PORT, "name": "http"}],
                            "readinessProbe": {"httpGet": {"path": "/healthz", "port": DEFAULT_PORT}},
                            "livenessProbe": {"httpGet": {"path": "/healthz", "port": DEFAULT_PORT}},
                        }],
                    },
                },
            },
        },
        {
            "apiVersion": "v1",
            "kind": "Service",
            "metadata": {"name": "gpu-topology-scheduler-extender", "namespace": namespace, "labels": labels},
            "spec": {"selector": {"name": "gpu-topology-scheduler-extender"},
                     "ports": [{"port": DEFAULT_PORT, "targetPort": DEFAULT_PORT, "name": "http"}]},
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
