"""Container Device Interface (CDI) spec for the advertised devices.

The reference hands devices to the container through nvidia-docker's ``NVIDIA_VISIBLE_DEVICES``
(``design.md:239``, diagram step ⑦).  The default here is plain kubelet ``DeviceSpec`` mounts
(``/dev/kfd`` + ``/dev/dri/renderD*``); ``--device-specs cdi`` instead answers ``Allocate`` with
fully-qualified CDI names (``amd.com/gpu=<index>``, the GROUP numbering) and writes the spec that
resolves them, so a CDI-enabled runtime (containerd >= 1.7, CRI-O) performs the device injection.

Spec (``cdiVersion`` 0.6.0): one device per advertised GPU/XCP with its render and card nodes, and
``/dev/kfd`` as a common edit (every ROCm container needs it).  Written atomically (temp file +
rename) because the runtime may read the directory at any time.
"""
from __future__ import annotations

import json
import os
import tempfile
from typing import Dict, List, Sequence

from ..topology.model import Topology

__all__ = ["CDI_VERSION", "cdi_name", "build_spec", "write_spec"]

CDI_VERSION = "0.6.0"


def cdi_name(kind: str, index: int) -> str:
    """Fully-qualified CDI device name of topology index ``index``."""
    return f"{kind}={int(index)}"


def _nodes(topo: Topology, i: int, dev_root: str) -> List[Dict[str, object]]:
    g = topo.gpus[i]
    root = dev_root.rstrip("/")
    minor = g.render_node
    out: List[Dict[str, object]] = [{"path": f"/dev/dri/renderD{minor}", "hostPath": f"{root}/dri/renderD{minor}"}]
    if g.card >= 0:
        out.append({"path": f"/dev/dri/card{g.card}", "hostPath": f"{root}/dri/card{g.card}"})
    return out


def build_spec(topo: Topology, kind: str = "amd.com/gpu", dev_root: str = "/dev", only_existing: bool = False) -> Dict[str, object]:
    """The CDI spec of every device of ``topo``.  ``only_existing`` drops nodes absent under
    ``dev_root`` (kind / fake GPUs), mirroring the ``stub`` DeviceSpec mode."""
    def keep(nodes: Sequence[Dict[str, object]]) -> List[Dict[str, object]]:
        return [n for n in nodes if not only_existing or os.path.exists(str(n["hostPath"]))]

    devices = []
    for g in topo.gpus:
        edits: Dict[str, object] = {"deviceNodes": keep(_nodes(topo, g.index, dev_root)),
                                    "env": [f"GTK_CDI_DEVICE_{g.index}={g.bdf or g.index}"]}
        devices.append({"name": str(g.index), "containerEdits": edits})
    kfd = keep([{"path": "/dev/kfd", "hostPath": f"{dev_root.rstrip('/')}/kfd"}])
    return {"cdiVersion": CDI_VERSION, "kind": kind, "devices": devices, "containerEdits": {"deviceNodes": kfd}}


def write_spec(spec: Dict[str, object], cdi_dir: str, file_name: str = "") -> str:
    """Atomically write ``spec`` as ``<cdi_dir>/<vendor>-<class>.json``; returns the path."""
    os.makedirs(cdi_dir, exist_ok=True)
    name = file_name or str(spec["kind"]).replace("/", "-") + ".json"
    path = os.path.join(cdi_dir, name)
    fd, tmp = tempfile.mkstemp(prefix=".gtk-cdi-", dir=cdi_dir)
    try:
        with os.fdopen(fd, "w") as f:
            json.dump(spec, f, indent=1)
        os.chmod(tmp, 0o644)
        os.replace(tmp, path)
    except BaseException:
        try:
            os.unlink(tmp)
        except FileNotFoundError:
            pass
        raise
    return path
