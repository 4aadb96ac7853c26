"""kubelet device plugin (``v1beta1`` gRPC) for MI355X devices, plus a fake kubelet for tests/simulation."""
from .kubelet import AdmissionError, FakeKubelet
from .plugin import DevicePluginServer, PluginConfig

__all__ = ["AdmissionError", "FakeKubelet", "DevicePluginServer", "PluginConfig"]
