"""kubelet device-plugin API ``v1beta1`` built from a hand-written FileDescriptorProto.

``protoc`` / ``grpc_tools`` are not available in this image, so the message
classes are created at import time from a descriptor that mirrors the upstream
``k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1/api.proto`` field-for-field (names, numbers, types
and labels), which is all the wire format depends on.  Service method paths are the upstream ones
(``/v1beta1.Registration/Register``, ``/v1beta1.DevicePlugin/Allocate`` ...), so a real kubelet
talks to this plugin unchanged.

Reference: ``design.md:84-86`` (ListAndWatch advertises the resource) and ``design.md:236-246``
(Allocate); ``GetPreferredAllocation`` is the kubelet API's topology hook used so the kubelet's
own device accounting matches the extender's GROUP annotation.
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

__all__ = [
    "VERSION", "KUBELET_SOCKET", "DEVICE_PLUGIN_PATH", "HEALTHY", "UNHEALTHY", "REGISTRATION_SERVICE", "DEVICE_PLUGIN_SERVICE",
    "Empty", "DevicePluginOptions", "RegisterRequest", "ListAndWatchResponse", "TopologyInfo", "NUMANode", "Device",
    "PreStartContainerRequest", "PreStartContainerResponse", "PreferredAllocationRequest",
    "ContainerPreferredAllocationRequest", "PreferredAllocationResponse", "ContainerPreferredAllocationResponse",
    "AllocateRequest", "ContainerAllocateRequest", "CDIDevice", "AllocateResponse", "ContainerAllocateResponse", "Mount",
    "DeviceSpec", "METHODS",
]

VERSION = "v1beta1"
DEVICE_PLUGIN_PATH = "/var/lib/kubelet/device-plugins/"
KUBELET_SOCKET = DEVICE_PLUGIN_PATH + "kubelet.sock"
HEALTHY = "Healthy"
UNHEALTHY = "Unhealthy"
REGISTRATION_SERVICE = "v1beta1.Registration"
DEVICE_PLUGIN_SERVICE = "v1beta1.DevicePlugin"

_F = descriptor_pb2.FieldDescriptorProto
_STRING, _BOOL, _INT64, _INT32, _MSG = _F.TYPE_STRING, _F.TYPE_BOOL, _F.TYPE_INT64, _F.TYPE_INT32, _F.TYPE_MESSAGE
_OPT, _REP = _F.LABEL_OPTIONAL, _F.LABEL_REPEATED

# (message name, [(field name, number, type, label, type_name or None, json_name or None)])
_MESSAGES = [
    ("DevicePluginOptions", [("pre_start_required", 1, _BOOL, _OPT, None, None),
                             ("get_preferred_allocation_available", 2, _BOOL, _OPT, None, None)]),
    ("RegisterRequest", [("version", 1, _STRING, _OPT, None, None), ("endpoint", 2, _STRING, _OPT, None, None),
                         ("resource_name", 3, _STRING, _OPT, None, None),
                         ("options", 4, _MSG, _OPT, ".v1beta1.DevicePluginOptions", None)]),
    ("Empty", []),
    ("ListAndWatchResponse", [("devices", 1, _MSG, _REP, ".v1beta1.Device", None)]),
    ("TopologyInfo", [("nodes", 1, _MSG, _REP, ".v1beta1.NUMANode", None)]),
    ("NUMANode", [("ID", 1, _INT64, _OPT, None, "ID")]),
    ("Device", [("ID", 1, _STRING, _OPT, None, "ID"), ("health", 2, _STRING, _OPT, None, None),
                ("topology", 3, _MSG, _OPT, ".v1beta1.TopologyInfo", None)]),
    ("PreStartContainerRequest", [("devices_ids", 1, _STRING, _REP, None, "devicesIDs")]),
    ("PreStartContainerResponse", []),
    ("PreferredAllocationRequest", [("container_requests", 1, _MSG, _REP, ".v1beta1.ContainerPreferredAllocationRequest", None)]),
    ("ContainerPreferredAllocationRequest", [("available_deviceIDs", 1, _STRING, _REP, None, None),
                                             ("must_include_deviceIDs", 2, _STRING, _REP, None, None),
                                             ("allocation_size", 3, _INT32, _OPT, None, None)]),
    ("PreferredAllocationResponse", [("container_responses", 1, _MSG, _REP, ".v1beta1.ContainerPreferredAllocationResponse", None)]),
    ("ContainerPreferredAllocationResponse", [("deviceIDs", 1, _STRING, _REP, None, None)]),
    ("AllocateRequest", [("container_requests", 1, _MSG, _REP, ".v1beta1.ContainerAllocateRequest", None)]),
    ("ContainerAllocateRequest", [("devices_ids", 1, _STRING, _REP, None, "devicesIDs")]),
    ("CDIDevice", [("name", 1, _STRING, _OPT, None, None)]),
    ("AllocateResponse", [("container_responses", 1, _MSG, _REP, ".v1beta1.ContainerAllocateResponse", None)]),
    ("ContainerAllocateResponse", [("envs", 1, _MSG, _REP, ".v1beta1.ContainerAllocateResponse.EnvsEntry", None),
                                   ("mounts", 2, _MSG, _REP, ".v1beta1.Mount", None),
                                   ("devices", 3, _MSG, _REP, ".v1beta1.DeviceSpec", None),
                                   ("annotations", 4, _MSG, _REP, ".v1beta1.ContainerAllocateResponse.AnnotationsEntry", None),
                                   ("cdi_devices", 5, _MSG, _REP, ".v1beta1.CDIDevice", None)]),
    ("Mount", [("container_path", 1, _STRING, _OPT, None, None), ("host_path", 2, _STRING, _OPT, None, None),
               ("read_only", 3, _BOOL, _OPT, None, None)]),
    ("DeviceSpec", [("container_path", 1, _STRING, _OPT, None, None), ("host_path", 2, _STRING, _OPT, None, None),
                    ("permissions", 3, _STRING, _OPT, None, None)]),
]
_MAP_ENTRIES = {"ContainerAllocateResponse": ["EnvsEntry", "AnnotationsEntry"]}

# (service, [(method, input, output, server_streaming)])
_SERVICES = [
    ("Registration", [("Register", "RegisterRequest", "Empty", False)]),
    ("DevicePlugin", [("GetDevicePluginOptions", "Empty", "DevicePluginOptions", False),
                      ("ListAndWatch", "Empty", "ListAndWatchResponse", True),
                      ("GetPreferredAllocation", "PreferredAllocationRequest", "PreferredAllocationResponse", False),
                      ("Allocate", "AllocateRequest", "AllocateResponse", False),
                      ("PreStartContainer", "PreStartContainerRequest", "PreStartContainerResponse", False)]),
]


def _build_file() -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto(name="gtk/deviceplugin/v1beta1/api.proto", package="v1beta1", syntax="proto3")
    for name, fields in _MESSAGES:
        m = fd.message_type.add(name=name)
        for fname, num, typ, label, tname, jname in fields:
            f = m.field.add(name=fname, number=num, type=typ, label=label)
            if tname:
                f.type_name = tname
            if jname:
                f.json_name = jname
        for entry in _MAP_ENTRIES.get(name, []):
            e = m.nested_type.add(name=entry)
            e.field.add(name="key", number=1, type=_STRING, label=_OPT)
            e.field.add(name="value", number=2, type=_STRING, label=_OPT)
            e.options.map_entry = True
    for sname, methods in _SERVICES:
        s = fd.service.add(name=sname)
        for mname, inp, out, stream in methods:
            s.method.add(name=mname, input_type=f".v1beta1.{inp}", output_type=f".v1beta1.{out}", server_streaming=stream)
    return fd


_POOL = descriptor_pool.DescriptorPool()
_FILE = _POOL.Add(_build_file())
_FD = _POOL.FindFileByName("gtk/deviceplugin/v1beta1/api.proto")


def _cls(name: str):
    return message_factory.GetMessageClass(_FD.message_types_by_name[name])


Empty = _cls("Empty")
DevicePluginOptions = _cls("DevicePluginOptions")
RegisterRequest = _cls("RegisterRequest")
ListAndWatchResponse = _cls("ListAndWatchResponse")
TopologyInfo = _cls("TopologyInfo")
NUMANode = _cls("NUMANode")
Device = _cls("Device")
PreStartContainerRequest = _cls("PreStartContainerRequest")
PreStartContainerResponse = _cls("PreStartContainerResponse")
PreferredAllocationRequest = _cls("PreferredAllocationRequest")
ContainerPreferredAllocationRequest = _cls("ContainerPreferredAllocationRequest")
PreferredAllocationResponse = _cls("PreferredAllocationResponse")
ContainerPreferredAllocationResponse = _cls("ContainerPreferredAllocationResponse")
AllocateRequest = _cls("AllocateRequest")
ContainerAllocateRequest = _cls("ContainerAllocateRequest")
CDIDevice = _cls("CDIDevice")
AllocateResponse = _cls("AllocateResponse")
ContainerAllocateResponse = _cls("ContainerAllocateResponse")
Mount = _cls("Mount")
DeviceSpec = _cls("DeviceSpec")

#: full method path -> (request class, response class, server streaming)
METHODS = {
    f"/v1beta1.{s}/{m}": (globals()[i], globals()[o], stream) for s, ms in _SERVICES for m, i, o, stream in ms
}


def service_descriptor(name: str):
    return _FD.services_by_name[name]
