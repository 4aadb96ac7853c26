"""Topology-aware kube-scheduler extender: prioritize ("sort"), bind, filter."""
from .cache import Alloc, ClusterCache, NodeState
from .metrics import ExtenderMetrics
from .scheduler import Decision, ExtenderConfig, TopologyExtender

__all__ = ["Alloc", "ClusterCache", "NodeState", "ExtenderMetrics", "Decision", "ExtenderConfig", "TopologyExtender"]
