"""kubelet pod-resources API ``v1`` (``PodResourcesLister.List``) from a hand-written descriptor.

Why: ``Allocate`` carries device IDs but not the pod.  The plugin steers the
kubelet to the annotated GROUP through ``GetPreferredAllocation``, but when two assumed pods of the
same size wait on one node the kubelet may admit them in another order than they were assumed, and
the annotations then name each other's devices (found by ``tests/test_churn.py``).  The kubelet's
pod-resources socket (``/var/lib/kubelet/pod-resources/kubelet.sock``) is the ground truth of which
pod holds which device, so the plugin reconciles the ``ALIYUN_COM_GPU_GROUP`` annotations against it
(:meth:`DevicePluginServer.reconcile`).

Field names and numbers mirror ``k8s.io/kubelet/pkg/apis/podresources/v1/api.proto`` (the parts
this plugin reads); the method path is the upstream ``/v1.PodResourcesLister/List``.
"""
from __future__ import annotations

from typing import Callable, Dict, Iterable, List, Tuple

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

__all__ = ["POD_RESOURCES_SOCKET", "LIST_METHOD", "ListPodResourcesRequest", "ListPodResourcesResponse", "list_pod_resources",
           "pod_resources_handler", "build_response"]

POD_RESOURCES_SOCKET = "/var/lib/kubelet/pod-resources/kubelet.sock"
SERVICE = "v1.PodResourcesLister"
LIST_METHOD = f"/{SERVICE}/List"

_F = descriptor_pb2.FieldDescriptorProto
_STRING, _INT64, _MSG = _F.TYPE_STRING, _F.TYPE_INT64, _F.TYPE_MESSAGE
_OPT, _REP = _F.LABEL_OPTIONAL, _F.LABEL_REPEATED

_MESSAGES = [
    ("ListPodResourcesRequest", []),
    ("ListPodResourcesResponse", [("pod_resources", 1, _MSG, _REP, ".v1.PodResources")]),
    ("PodResources", [("name", 1, _STRING, _OPT, None), ("namespace", 2, _STRING, _OPT, None),
                      ("containers", 3, _MSG, _REP, ".v1.ContainerResources")]),
    ("ContainerResources", [("name", 1, _STRING, _OPT, None), ("devices", 2, _MSG, _REP, ".v1.ContainerDevices"),
                            ("cpu_ids", 3, _INT64, _REP, None)]),
    ("ContainerDevices", [("resource_name", 1, _STRING, _OPT, None), ("device_ids", 2, _STRING, _REP, None),
                          ("topology", 3, _MSG, _OPT, ".v1.TopologyInfo")]),
    ("TopologyInfo", [("nodes", 1, _MSG, _REP, ".v1.NUMANode")]),
    ("NUMANode", [("ID", 1, _INT64, _OPT, None)]),
]


def _build_file() -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto(name="gtk/podresources/v1/api.proto", package="v1", syntax="proto3")
    for name, fields in _MESSAGES:
        m = fd.message_type.add(name=name)
        for fname, num, typ, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=typ, label=label)
            if tname:
                f.type_name = tname
    s = fd.service.add(name="PodResourcesLister")
    s.method.add(name="List", input_type=".v1.ListPodResourcesRequest", output_type=".v1.ListPodResourcesResponse")
    return fd


_POOL = descriptor_pool.DescriptorPool()
_POOL.Add(_build_file())
_FD = _POOL.FindFileByName("gtk/podresources/v1/api.proto")
ListPodResourcesRequest = message_factory.GetMessageClass(_FD.message_types_by_name["ListPodResourcesRequest"])
ListPodResourcesResponse = message_factory.GetMessageClass(_FD.message_types_by_name["ListPodResourcesResponse"])


def list_pod_resources(socket_path: str = POD_RESOURCES_SOCKET, timeout: float = 5.0) -> Dict[str, Dict[str, List[str]]]:
    """``namespace/name`` -> resource name -> device IDs (all containers of the pod), from the kubelet."""
    import grpc

    with grpc.insecure_channel(f"unix://{socket_path}") as ch:
        call = ch.unary_unary(LIST_METHOD, request_serializer=ListPodResourcesRequest.SerializeToString,
                              response_deserializer=ListPodResourcesResponse.FromString)
        resp = call(ListPodResourcesRequest(), timeout=timeout)
    out: Dict[str, Dict[str, List[str]]] = {}
    for pr in resp.pod_resources:
        per = out.setdefault(f"{pr.namespace}/{pr.name}", {})
        for c in pr.containers:
            for d in c.devices:
                per.setdefault(d.resource_name, []).extend(d.device_ids)
    return out


def build_response(allocations: Iterable[Tuple]) -> "ListPodResourcesResponse":
    """``(pod key, container, resource, device ids)`` rows (or ``(pod key, resource, ids)``, one
    container named ``main``) -> a List response."""
    resp = ListPodResourcesResponse()
    pods: Dict[str, object] = {}
    conts: Dict[Tuple[str, str], object] = {}
    for row in allocations:
        key, cname, resource, ids = row if len(row) == 4 else (row[0], "main", row[1], row[2])
        pr = pods.get(key)
        if pr is None:
            ns, name = key.split("/", 1)
            pr = resp.pod_resources.add(name=name, namespace=ns)
            pods[key] = pr
        c = conts.get((key, cname))
        if c is None:
            c = conts[(key, cname)] = pr.containers.add(name=cname)
        c.devices.add(resource_name=resource, device_ids=list(ids))
    return resp


def pod_resources_handler(list_fn: Callable[[], "ListPodResourcesResponse"]):
    """A grpc generic handler serving ``List`` from ``list_fn`` (the in-process kubelet)."""
    import grpc

    h = {"List": grpc.unary_unary_rpc_method_handler(lambda req, ctx: list_fn(),
                                                     request_deserializer=ListPodResourcesRequest.FromString,
                                                     response_serializer=ListPodResourcesResponse.SerializeToString)}
    return grpc.method_handlers_generic_handler(SERVICE, h)
