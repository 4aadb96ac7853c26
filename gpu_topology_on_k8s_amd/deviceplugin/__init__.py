"""kubelet device plugin (``v1beta1`` gRPC) for MI355X devices, plus a fake kubelet for tests/simulation."""
from .kubelet import AdmissionError, FakeKubelet
from .metrics import PluginMetrics, serve_metrics
from .plugin import DevicePluginServer, PluginConfig, placeholder_dev_tree

__all__ = ["AdmissionError", "FakeKubelet", "DevicePluginServer", "PluginConfig", "PluginMetrics", "placeholder_dev_tree",
           "serve_metrics"]
