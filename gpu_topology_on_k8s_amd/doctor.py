"""``gtk doctor`` — is this node (or this pod) set up the way the framework needs it?

Every check is one line of JSON (``name``, ``status`` ok|warn|fail|skip, ``detail``), so the
DaemonSet's init step, an operator, or a pod's entry point can act on it.  Node checks:

* ``kfd`` / ``render-nodes``    the ROCm device nodes Allocate hands to containers (``design.md:239``
                                names ``NVIDIA_VISIBLE_DEVICES``; here ``/dev/kfd`` + ``/dev/dri/renderD*``);
* ``discovery``                 amdsmi, else KFD sysfs, finds the GPUs and their link classes (A1);
* ``native``                    the in-tree extensions and the vGPU guard are built;
* ``ipc-mode``                  ``HSA_ENABLE_IPC_MODE_LEGACY=0`` for cross-process GPU memory (RCCL P2P/IPC);
* ``cpu-affinity``              every GPU's local cores intersect this process's allowed CPUs (Gaia B6);
* ``device-plugin-dir``         the kubelet's device-plugin socket directory is writable;
* ``partition``                 each package's compute / memory partition mode and the modes it offers
                                (amdsmi, read-only; what ``--partition-control`` may switch to);
* ``topology-manager``          the kubelet's Topology Manager policy and scope (its KubeletConfiguration),
                                which the device plugin must be given so the extender binds what the
                                kubelet will allocate (placement/numa_align.py).

Pod checks (when ``GTK_GPU_GROUP`` is set, i.e. inside a container Allocate configured):

* ``pod-group``                 GROUP maps onto this container's HIP devices by PCI address;
* ``pod-cpuset``                ``GTK_CPUSET`` is usable here (not disjoint from the allowed CPUs);
* ``pod-share``                 a partial-GPU pod has its CU mask and the vGPU guard in force.

``--gpu`` adds the checks that initialise HIP (device count, gfx950, an MFMA warm-up, an exact RCCL
all-reduce over the visible devices); without it
the command never touches a GPU, so it is safe on a node whose GPUs are busy.
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Optional

__all__ = ["run_checks", "main"]

Check = Dict[str, object]


def _c(name: str, status: str, detail: str = "", **extra) -> Check:
    return {"name": name, "status": status, "detail": detail, **extra}


def check_dev(dev_root: str = "/dev") -> List[Check]:
    out = []
    kfd = os.path.join(dev_root, "kfd")
    out.append(_c("kfd", "ok" if os.path.exists(kfd) else "fail", kfd if os.path.exists(kfd) else f"{kfd} missing"))
    dri = os.path.join(dev_root, "dri")
    renders = sorted(n for n in (os.listdir(dri) if os.path.isdir(dri) else []) if n.startswith("renderD"))
    out.append(_c("render-nodes", "ok" if renders else "fail", ",".join(renders) or f"no renderD* under {dri}"))
    return out


def check_discovery(backend: str = "auto", fake_n: Optional[int] = None):
    """-> (checks, topology or None)."""
    import numpy as np

    from .topology.discovery import discover
    from .topology.model import LinkType

    try:
        t = discover(backend, fake_n=fake_n)
    except Exception as e:  # noqa: BLE001 - DiscoveryError or a broken library: the check's result
        return [_c("discovery", "fail", str(e)[:300])], None
    kinds = sorted({LinkType(int(x)).name for x in t.link_type[~np.eye(t.n, dtype=bool)]}) if t.n > 1 else []
    detail = f"{t.n} devices via {t.source}; gfx {sorted({g.gfx for g in t.gpus})}; NUMA {sorted({g.numa for g in t.gpus})}"
    return [_c("discovery", "ok" if t.n > 0 else "fail", detail, devices=t.n, source=t.source, link_types=kinds)], t


def check_native() -> List[Check]:
    from ._native import NativeUnavailable, available, binary

    missing = [m for m in ("_topo", "_placement", "_probe", "_rccl", "_fused") if not available(m)]
    out = [_c("native", "fail" if missing else "ok", f"missing {missing}" if missing else "all extensions import")]
    try:
        binary("libgtk_vgpu.so")
        out.append(_c("vgpu-guard", "ok", "bin/libgtk_vgpu.so built"))
    except NativeUnavailable as e:
        out.append(_c("vgpu-guard", "warn", f"{e}: time-sliced shares would stay cooperative"))
    return out


def check_ipc(env: Dict[str, str]) -> Check:
    v = env.get("HSA_ENABLE_IPC_MODE_LEGACY")
    if v == "0":
        return _c("ipc-mode", "ok", "HSA_ENABLE_IPC_MODE_LEGACY=0 (dma-buf IPC handles)")
    return _c("ipc-mode", "warn", f"HSA_ENABLE_IPC_MODE_LEGACY={v!r}: RCCL's P2P/IPC transport between processes needs 0 "
                                  "on hosts whose driver exports only dma-buf handles")


def check_cpu_affinity(topo, allowed=None) -> Check:
    from .topology.cpus import format_cpulist, parse_cpulist

    allowed = set(os.sched_getaffinity(0)) if allowed is None else set(allowed)
    bad = [g.index for g in topo.gpus if g.cpu_affinity and not (parse_cpulist(g.cpu_affinity) & allowed)]
    unknown = [g.index for g in topo.gpus if not g.cpu_affinity]
    if bad:
        return _c("cpu-affinity", "warn", f"devices {bad}: none of their local cores is allowed here ({format_cpulist(allowed)})")
    if unknown and len(unknown) == topo.n:
        return _c("cpu-affinity", "warn", "no local_cpulist for any device: GTK_CPUSET recommendations will be empty")
    return _c("cpu-affinity", "ok", f"every device's local cores intersect the allowed CPUs ({len(allowed)})")


def check_partition(backend: str) -> Check:
    if backend not in ("auto", "amdsmi"):
        return _c("partition", "skip", f"--discovery {backend}: partition modes are read through amdsmi")
    from .topology.partition import partition_info

    try:
        info = partition_info()
    except Exception as e:  # noqa: BLE001 - no amdsmi here: not a failure of the node
        return _c("partition", "skip", f"amdsmi unavailable: {str(e)[:200]}")
    if not info:
        return _c("partition", "warn", "amdsmi lists no GPU packages")
    modes = sorted({f"{p['compute']}/{p['memory']}" for p in info})
    offers = sorted({m for p in info for m in p["compute_modes"]}, key=lambda m: "SDTQC".index(m[0]) if m[0] in "SDTQC" else 9)
    nps = sorted({m for p in info for m in p["memory_modes"]})
    return _c("partition", "ok" if len(modes) == 1 else "warn",
              f"{len(info)} package(s) in {', '.join(modes)}" + ("" if len(modes) == 1 else " (mixed modes)")
              + f"; offered: {','.join(offers) or '?'} / {','.join(nps) or '?'}",
              packages=info)


def check_topology_manager(kubelet_config: str = "/var/lib/kubelet/config.yaml") -> Check:
    """The kubelet's ``topologyManagerPolicy`` / ``topologyManagerScope`` and the device plugin flags
    that must carry them (skip when the file is not readable here)."""
    from .placement.numa_align import read_kubelet_config

    if not kubelet_config or not os.path.exists(kubelet_config):
        return _c("topology-manager", "skip", f"{kubelet_config} not readable here: pass the kubelet's policy to the device "
                                              "plugin with --topology-manager-policy / --topology-manager-scope")
    try:
        tm = read_kubelet_config(kubelet_config)
    except Exception as e:  # noqa: BLE001 - the check's result
        return _c("topology-manager", "fail", f"{kubelet_config}: {e}")
    if not tm.active:
        return _c("topology-manager", "ok", "policy none: the kubelet takes the plugin's preferred devices as they are",
                  policy=tm.policy, scope=tm.scope)
    unmodelled = _unmodelled_tm_options(kubelet_config)
    if unmodelled:
        return _c("topology-manager", "warn", f"policy {tm.policy}, scope {tm.scope} with topologyManagerPolicyOptions "
                                              f"{', '.join(unmodelled)}: the extender replays the default merge (equally narrow "
                                              "hints tie-break on the lowest NUMA bitmask), so where these options make the "
                                              "kubelet pick other NUMA nodes the plugin's GROUP is overridden "
                                              "(gtk_plugin_group_overridden_total) and the reconcile corrects the annotations",
                  policy=tm.policy, scope=tm.scope, options=unmodelled)
    return _c("topology-manager", "ok", f"policy {tm.policy}, scope {tm.scope}: run the device plugin with "
                                        f"--topology-manager-policy={tm.policy} --topology-manager-scope={tm.scope} "
                                        "(or --kubelet-config on this file)", policy=tm.policy, scope=tm.scope)


#: kubelet Topology Manager policy options that leave the device hints and their merge as the
#: extender replays them (placement/numa_align.py); any other option enabled is reported
_TM_OPTIONS_MODELLED = {"max-allowable-numa-nodes"}


def _unmodelled_tm_options(kubelet_config: str) -> List[str]:
    """``topologyManagerPolicyOptions`` the extender does not model and the file enables (e.g.
    ``prefer-closest-numa-nodes``, which breaks ties between equally narrow hints by NUMA distance)."""
    import yaml

    with open(kubelet_config) as f:
        cfg = yaml.safe_load(f) or {}
    opts = cfg.get("topologyManagerPolicyOptions") or {}
    if not isinstance(opts, dict):
        return []
    return sorted(str(k) for k, v in opts.items()
                  if k not in _TM_OPTIONS_MODELLED and str(v).strip().lower() not in ("false", "0", ""))


def check_plugin_dir(path: str) -> Check:
    if not os.path.isdir(path):
        return _c("device-plugin-dir", "skip", f"{path} absent (not a kubelet node, or not mounted)")
    return _c("device-plugin-dir", "ok" if os.access(path, os.W_OK) else "fail",
              f"{path} {'writable' if os.access(path, os.W_OK) else 'not writable'}")


def check_pod(env: Dict[str, str], visible_bdfs: Optional[List[str]] = None, allowed=None) -> List[Check]:
    from .topology.cpus import format_cpulist, parse_cpulist
    from .topology.identity import group_from_env, hip_device_bdfs, resolve_group

    group, bdfs = group_from_env(env)
    if not group:
        return [_c("pod-group", "skip", "GTK_GPU_GROUP not set: not a container the device plugin configured")]
    out = []
    vis = hip_device_bdfs() if visible_bdfs is None else visible_bdfs
    try:
        hip = resolve_group(group, bdfs=bdfs or None, visible_bdfs=vis)
        out.append(_c("pod-group", "ok", f"GROUP {group} -> HIP {hip}", hip_devices=hip))
    except ValueError as e:
        out.append(_c("pod-group", "fail", str(e)[:300]))
    allowed = set(os.sched_getaffinity(0)) if allowed is None else set(allowed)
    cs = parse_cpulist(env.get("GTK_CPUSET", ""))
    if not cs:
        out.append(_c("pod-cpuset", "warn", "no GTK_CPUSET (discovery had no local_cpulist)"))
    elif not cs & allowed:
        out.append(_c("pod-cpuset", "warn", f"GTK_CPUSET {format_cpulist(cs)} is disjoint from the allowed CPUs "
                                            f"{format_cpulist(allowed)} (the kubelet CPU manager placed the pod elsewhere)"))
    else:
        out.append(_c("pod-cpuset", "ok", f"{len(cs & allowed)} of GTK_CPUSET's cores usable"))
    fr = [float(x) for x in env.get("GTK_GPU_FRACTION", "").split(",") if x.strip()]
    if fr and min(fr) < 1.0:
        problems = []
        guarded = env.get("GTK_VGPU_ACTIVE") == "1"
        # an address-keyed guard config clears HSA_CU_MASK and masks every queue itself (vgpu_guard.cpp)
        mask = env.get("HSA_CU_MASK") or ("per queue, by the guard" if guarded else "")
        if not mask:
            problems.append("no HSA_CU_MASK")
        if not guarded:
            problems.append("the vGPU guard is not loaded (HBM share unenforced)")
        out.append(_c("pod-share", "warn" if problems else "ok",
                      "; ".join(problems) if problems else f"share {fr}, CU mask {mask}, guard active"))
    return out


def check_gpu() -> List[Check]:
    from .ops import probe

    out = []
    n = probe.device_count()
    out.append(_c("hip-devices", "ok" if n > 0 else "fail", f"{n} visible"))
    if n == 0:
        return out
    props = probe.device_props(0)
    out.append(_c("gfx", "ok" if str(props["gcn_arch"]).startswith("gfx950") else "warn", str(props["gcn_arch"])))
    w = probe.warmup(0, 20.0)
    out.append(_c("mfma", "ok" if w["tflops"] > 1000 else "warn", f"{w['tflops']:.0f} TF/s dense bf16 on device 0",
                  tflops=round(float(w["tflops"]), 1)))
    try:  # RCCL loads and sums exactly (one rank per visible device; cross-device links: `gtk validate`)
        from ._native import load

        pts = load("_rccl").local_sweep(list(range(n)), [1 << 20], "bf16", 1, 1, False, True)
        wrong = sum(int(p["wrong"]) for p in pts)
        out.append(_c("rccl", "ok" if wrong == 0 else "fail",
                      f"{n}-rank all-reduce of 1 MiB bf16: {'exact' if wrong == 0 else f'{wrong} wrong elements'}"))
    except Exception as e:  # noqa: BLE001 - the check's result
        out.append(_c("rccl", "fail", str(e)[:300]))
    return out


def run_checks(backend: str = "auto", fake_n: Optional[int] = None, gpu: bool = False, dev_root: str = "/dev",
               plugin_dir: str = "/var/lib/kubelet/device-plugins", env: Optional[Dict[str, str]] = None,
               visible_bdfs: Optional[List[str]] = None, allowed=None,
               kubelet_config: str = "/var/lib/kubelet/config.yaml") -> List[Check]:
    env = dict(os.environ) if env is None else env
    checks: List[Check] = []
    if backend != "fake":
        checks += check_dev(dev_root)
    found, topo = check_discovery(backend, fake_n)
    checks += found
    if topo is not None:
        checks.append(check_cpu_affinity(topo, allowed))
        checks.append(check_partition(backend))
    checks += check_native()
    checks.append(check_ipc(env))
    checks.append(check_plugin_dir(plugin_dir))
    checks.append(check_topology_manager(kubelet_config))
    checks += check_pod(env, visible_bdfs=visible_bdfs if visible_bdfs is not None else ([] if backend == "fake" else None),
                        allowed=allowed)
    if gpu:
        checks += check_gpu()
        checks += check_guard(env)  # after the runtime started: the guard has resolved its config
    return checks


def check_guard(env: Dict[str, str]) -> List[Check]:
    """Inside a guarded partial-GPU pod, once the GPU runtime has started: every address-keyed entry of
    the guard's config matched a GPU the runtime enumerated (an unmatched one used to leave
    the share unenforced while this doctor reported it enforced).  The guard reports each unmatched
    entry on stderr and applies it to the fallback ordinal the plugin wrote."""
    if env.get("GTK_VGPU_ACTIVE") != "1":
        return []
    import ctypes

    try:
        fn = ctypes.CDLL(None).gtk_vgpu_unmatched
    except AttributeError:
        return [_c("pod-guard", "fail", "GTK_VGPU_ACTIVE is set but libgtk_vgpu.so is not loaded in this process")]
    n = int(fn())
    if n < 0:
        return [_c("pod-guard", "skip", "the GPU runtime has not enumerated its devices in this process")]
    if n:
        return [_c("pod-guard", "fail", f"{n} address-keyed guard entr{'y' if n == 1 else 'ies'} matched no GPU the runtime "
                                        "enumerated (see the gtk-vgpu lines on stderr): applied to the plugin's fallback "
                                        "ordinal when it wrote one, else unenforced", unmatched=n)]
    return [_c("pod-guard", "ok", "every address-keyed guard entry matched a GPU")]


def main(a) -> int:
    checks = run_checks(a.discovery, a.fake_gpus, a.gpu, a.dev_root, a.plugin_dir,
                        kubelet_config=getattr(a, "kubelet_config", "/var/lib/kubelet/config.yaml"))
    for c in checks:
        print(json.dumps(c))
    worst = "fail" if any(c["status"] == "fail" for c in checks) else ("warn" if any(c["status"] == "warn" for c in checks) else "ok")
    print(json.dumps({"summary": True, "status": worst, "checks": len(checks)}))
    return 1 if worst == "fail" else 0
