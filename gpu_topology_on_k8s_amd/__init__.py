"""MI355X-native topology-aware GPU scheduling for Kubernetes.

Layers: native discovery + HIP link probe (``topology``, ``ops``), placement core
(``placement``), kubelet device plugin (``deviceplugin``), scheduler extender (``extender``),
Kubernetes API client / in-memory fake (``k8s``), RCCL placement validation and DP training
(``parallel``, ``models``), in-process cluster simulation (``sim``).
"""
__version__ = "0.1.0"
