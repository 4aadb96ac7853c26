"""Hardware partition control: switch a node's GPUs between SPX/DPX/QPX/CPX and NPS memory modes.

Gaia virtualises a GPU in two tiers (paper p.3 §III.A "GPU resource virtualization"): the device
plugin splits it into vGPUs, and the container side enforces them.  On MI355X the hardware does the
splitting: a CPX package is 8 XCPs with their own compute units, each a device of its own (SURVEY.md
B3/B8), and NPS modes split the HBM.  Discovery (``csrc/topo/topo_reader.cpp``) reads the mode a node
is in.  This module changes it, through the same dlopen'ed amdsmi:

* :func:`partition_info` reports per package the current compute and memory modes and the ones the
  package offers (accelerator partition profiles and NPS capabilities).  It is read-only.
* :func:`apply_partition` switches every package, in the order the modes allow.  A finer compute
  mode goes first (SPX -> CPX, then NPS4, which needs CPX on MI300-class parts).  A coarser one goes
  last (NPS4 -> NPS1, then SPX).  A memory change takes effect only after an amdgpu driver reload,
  which needs every GPU process on the node gone.  It is done only when the caller allows it.

The device plugin drives this from a node label (``<prefix>/compute-partition-request``,
``--partition-control on``), only while no pod holds a device and with the node marked so that the
extender stops binding there.  Switching needs root (the privileged DaemonSet).  Anything else gets
``permission denied`` from amdsmi, which is reported, never retried in a loop.
"""
from __future__ import annotations

import os
from typing import Callable, Dict, List, Optional, Sequence, Tuple

from .._native import load

__all__ = ["COMPUTE_XCPS", "MEMORY_MODES", "PartitionError", "amdsmi_lib", "partition_info", "plan_steps",
           "apply_partition", "status_name", "normalise"]

#: XCPs per package in each compute partition mode of an 8-XCD MI355X
COMPUTE_XCPS: Dict[str, int] = {"SPX": 1, "DPX": 2, "TPX": 3, "QPX": 4, "CPX": 8}
MEMORY_MODES = ("NPS1", "NPS2", "NPS4", "NPS8")

# amdsmi_status_t values an operator can act on (amdsmi.h)
_STATUS = {0: "ok", 1: "invalid argument", 2: "not supported by this driver or device",
           3: "not yet implemented", 8: "device busy", 10: "permission denied (needs root: the privileged DaemonSet)",
           54: "amdgpu driver restart failed (see dmesg)", 55: "setting unavailable on this device or combination"}


class PartitionError(RuntimeError):
    pass


def status_name(code: int) -> str:
    return _STATUS.get(int(code), f"amdsmi status {int(code)}")


def amdsmi_lib(lib: Optional[str] = None) -> str:
    return lib or os.environ.get("GTK_AMDSMI_LIB", "") or "libamd_smi.so"


def normalise(compute: Optional[str], memory: Optional[str]) -> Tuple[Optional[str], Optional[str]]:
    """Upper-case and validate a requested (compute, memory) pair; '' / None = leave as is."""
    c = (compute or "").strip().upper() or None
    m = (memory or "").strip().upper() or None
    if c is not None and c not in COMPUTE_XCPS:
        raise PartitionError(f"unknown compute partition {compute!r} (one of {', '.join(COMPUTE_XCPS)})")
    if m is not None and m not in MEMORY_MODES:
        raise PartitionError(f"unknown memory partition {memory!r} (one of {', '.join(MEMORY_MODES)})")
    return c, m


def partition_info(lib: Optional[str] = None) -> List[dict]:
    """Per package, in socket order: ``bdf``, ``compute``, ``memory``, ``xcps`` and the
    ``compute_modes`` / ``memory_modes`` it offers (empty when the driver does not say)."""
    return [dict(d) for d in load("_topo").partition_info(amdsmi_lib(lib))]


def plan_steps(cur_compute: str, cur_memory: str, want_compute: Optional[str],
               want_memory: Optional[str]) -> List[Tuple[str, str]]:
    """Ordered ``(what, mode)`` steps from the current to the wanted modes (see the module doc)."""
    steps: List[Tuple[str, str]] = []
    c = want_compute if want_compute and want_compute != cur_compute else None
    m = want_memory if want_memory and want_memory != cur_memory else None
    if c and m:
        finer = COMPUTE_XCPS[c] >= COMPUTE_XCPS.get(cur_compute, 1)
        steps = [("compute", c), ("memory", m)] if finer else [("memory", m), ("compute", c)]
    elif c:
        steps = [("compute", c)]
    elif m:
        steps = [("memory", m)]
    return steps


def _check_offered(info: Sequence[dict], compute: Optional[str], memory: Optional[str]) -> None:
    for p in info:
        if compute and p.get("compute_modes") and compute not in p["compute_modes"]:
            raise PartitionError(f"package {p['bdf']} offers compute modes {p['compute_modes']}, not {compute}")
        if memory and p.get("memory_modes") and memory not in p["memory_modes"]:
            raise PartitionError(f"package {p['bdf']} offers memory modes {p['memory_modes']}, not {memory}")


def apply_partition(compute: Optional[str] = None, memory: Optional[str] = None, lib: Optional[str] = None,
                    reload_driver: bool = False, before_reload: Optional[Callable[[], bool]] = None) -> dict:
    """Switch every package to ``compute`` / ``memory`` (None = keep).  The caller guarantees that no
    process uses the GPUs.  -> ``{"ok", "steps", "before", "after", "reason", "reload_required",
    "reloaded", "layout_changed"}``; ``ok`` is False (with ``reason``) when amdsmi refused a step.
    Nothing is retried.  ``layout_changed``: the devices the node exposes changed, whatever ``ok`` says
    -- a compute step took effect on some package (its XCP count changed at once), or a memory step
    was followed by a driver reload.  A memory mode only pending a reload changes nothing yet.
    ``before_reload`` is asked right before a driver reload (the most disruptive step); False stops
    the switch there (the caller saw a pod claim a device since its own idle check)."""
    compute, memory = normalise(compute, memory)
    lib = amdsmi_lib(lib)
    mod = load("_topo")
    before = partition_info(lib)
    if not before:
        raise PartitionError("amdsmi found no GPU packages")
    _check_offered(before, compute, memory)
    cur_c = before[0]["compute"]
    cur_m = before[0]["memory"]
    mixed = any(p["compute"] != cur_c or p["memory"] != cur_m for p in before)
    steps = plan_steps("" if mixed else cur_c, "" if mixed else cur_m, compute, memory)
    out = {"ok": True, "before": before, "steps": [], "reason": "", "reload_required": False, "reloaded": False,
           "layout_changed": False}
    for what, mode in steps:
        res = [(bdf, int(code)) for bdf, code in mod.set_partition_step(lib, what, mode)]
        out["steps"].append({"set": what, "mode": mode, "packages": [{"bdf": b, "status": status_name(c)} for b, c in res]})
        if what == "compute" and any(c == 0 for _, c in res):
            out["layout_changed"] = True  # effective at once on every package that accepted it
        bad = [(b, c) for b, c in res if c != 0]
        if bad:
            out["ok"] = False
            out["reason"] = f"{what} partition {mode}: " + "; ".join(f"{b}: {status_name(c)}" for b, c in bad)
            break
        if what == "memory":
            if not reload_driver:
                # the new NPS mode is pending until the driver reloads; a compute step planned after
                # it may depend on it, so stop here and say so
                out["reload_required"] = True
                out["ok"] = False
                out["reason"] = (f"memory partition {mode} is pending an amdgpu driver reload "
                                 "(allow it with --partition-driver-reload, or reload the driver by hand)")
                break
            if before_reload is not None and not before_reload():
                out["ok"] = False
                out["reason"] = f"memory partition {mode} set; the driver reload was held back: the node is no longer idle"
                out["reload_required"] = True
                break
            code = int(mod.driver_reload(lib))
            out["steps"].append({"set": "driver-reload", "status": status_name(code)})
            if code != 0:
                out["ok"] = False
                out["reason"] = f"amdgpu driver reload: {status_name(code)}"
                break
            out["reloaded"] = True
            out["layout_changed"] = True
    out["after"] = partition_info(lib)
    if out["ok"]:
        wrong = [p["bdf"] for p in out["after"]
                 if (compute and p["compute"] != compute) or (memory and p["memory"] != memory)]
        if wrong:
            out["ok"] = False
            out["reason"] = f"packages {wrong} still report {out['after'][0]['compute']}/{out['after'][0]['memory']}"
    return out
