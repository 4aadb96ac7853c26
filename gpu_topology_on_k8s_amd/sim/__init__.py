"""In-process cluster simulation (fake apiserver + mini scheduler + extender + kubelets + device plugins)."""
from .cluster import HttpExtender, ScheduleResult, SimCluster

__all__ = ["HttpExtender", "ScheduleResult", "SimCluster"]
