"""Topology discovery (amdsmi / KFD sysfs / fake), model, annotation codec and link probing."""
from .model import DEFAULT_REF_GBPS, GPUInfo, LinkType, RefLinkClass, Topology, default_link_cost

__all__ = ["DEFAULT_REF_GBPS", "GPUInfo", "LinkType", "RefLinkClass", "Topology", "default_link_cost"]
