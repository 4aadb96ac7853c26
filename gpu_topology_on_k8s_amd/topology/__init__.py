"""Topology discovery (amdsmi / KFD sysfs / fake), model, annotation codec and link probing."""
from .model import DEFAULT_REF_GBPS, GPUInfo, LinkType, RefLinkClass, Topology, default_link_cost
from .shares import cu_mask_env, physical_group, share_fractions, slices_per_gpu, time_slice

__all__ = ["DEFAULT_REF_GBPS", "GPUInfo", "LinkType", "RefLinkClass", "Topology", "default_link_cost",
           "time_slice", "slices_per_gpu", "physical_group", "share_fractions", "cu_mask_env"]
