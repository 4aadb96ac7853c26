"""Compact wire form of a :class:`Topology` for the node annotation.

The apiserver caps the *total* annotations of an object at 256 KiB.  The readable v1 JSON
(``Topology.to_dict``: one dict per device, nested float lists) of a probed 64-XCP CPX node plus one
``GPU_<ABBR>_i_j`` key per device pair was ~200 KB before adding the amdsmi weight and max-bandwidth
matrices, so a real CPX node could fail to publish at all.  Version 2:

* device fields are columns, and a column whose values are all equal is one scalar;
* every matrix is ``"<dtype>:<base64(zlib(bytes))>"`` — link classes and hops as u8, amdsmi weights
  as u32, measured GB/s as f16 (GB/s up to 65504 at 0.05 % resolution, far below run-to-run probe
  noise), amdsmi max-bandwidth as u32;
* ``cost`` is omitted whenever it is what :meth:`Topology.recompute_cost` derives from the other
  fields, which is every probed node.  Measured bandwidth is quantised to f16 *in the model*
  (:meth:`Topology.set_measured_bw`) so the device plugin and the extender derive bit-identical
  costs and break ties identically.

The decoder accepts v1 and v2.  The encoded size of a fully probed 64-XCP node is asserted by
``tests/test_cluster_features.py``.
"""
from __future__ import annotations

import base64
import math
import zlib
from dataclasses import fields
from typing import Any, Dict, Optional

import numpy as np

__all__ = ["encode_v2", "decode_v2", "pack_matrix", "unpack_matrix"]

_DT = {"u8": np.uint8, "u16": np.uint16, "u32": np.uint32, "i32": np.int32, "f16": np.float16, "f32": np.float32,
       "f64": np.float64}


def pack_matrix(a: np.ndarray, dtype: str) -> str:
    arr = np.ascontiguousarray(np.asarray(a).astype(_DT[dtype]))
    return f"{dtype}:{base64.b64encode(zlib.compress(arr.tobytes(), 9)).decode()}"


def unpack_matrix(s: str, n: int) -> np.ndarray:
    dtype, _, payload = s.partition(":")
    raw = zlib.decompress(base64.b64decode(payload))
    return np.frombuffer(raw, dtype=_DT[dtype]).astype(np.float64).reshape(n, n)


def _int_dtype(a: np.ndarray) -> str:
    hi = float(np.nanmax(a)) if a.size else 0.0
    lo = float(np.nanmin(a)) if a.size else 0.0
    if lo >= 0 and hi < 256:
        return "u8"
    if lo >= 0 and hi < 2**32:
        return "u32"
    return "f64"


def encode_v2(topo) -> Dict[str, Any]:
    from .model import GPUInfo

    n = topo.n
    cols: Dict[str, Any] = {}
    for f in fields(GPUInfo):
        if f.name == "index":
            continue
        vals = [getattr(g, f.name) for g in topo.gpus]
        if f.name == "physical" and vals == list(range(n)):
            continue  # SPX default
        if vals and all(v == vals[0] for v in vals):
            if vals[0] != f.default:
                cols[f.name] = vals[0]
        else:
            cols[f.name] = vals
    m: Dict[str, str] = {
        "link_type": pack_matrix(topo.link_type, "u8"),
        "hops": pack_matrix(np.clip(topo.hops, 0, 255), "u8"),
    }
    if topo.bw_gbps is not None and np.isfinite(topo.bw_gbps).any():
        m["bw_gbps"] = pack_matrix(topo.bw_gbps, "f16")
    if topo.weight is not None and np.any(topo.weight):
        m["weight"] = pack_matrix(topo.weight, _int_dtype(topo.weight))
    if topo.ref_class is not None:
        m["ref_class"] = pack_matrix(topo.ref_class, "u8")
    probe = dict(topo.probe or {})
    for key in ("raw_gbps", "spread"):  # the probe's per-link medians and repeat spreads (ops/checks.py banding)
        v = probe.pop(key, None)
        if v is not None:
            a = np.array([[np.nan if x is None else float(x) for x in row] for row in v], dtype=np.float64)
            if a.shape == (n, n):
                m[key] = pack_matrix(a, "f16")
    mx = probe.pop("amdsmi_max_bw_mbps", None)
    if mx is not None:
        mx = np.asarray(mx, dtype=np.float64)
        if mx.shape == (n, n) and np.any(mx):
            m["max_bw_mbps"] = pack_matrix(mx, _int_dtype(mx))
    d: Dict[str, Any] = {"version": 2, "n": n, "node": topo.node_name, "source": topo.source, "ref_gbps": topo.ref_gbps,
                         "gpus": cols, "m": m, "probe": probe}
    if topo.hbm_gbps is not None and np.isfinite(topo.hbm_gbps).any():
        d["hbm_gbps"] = [None if not math.isfinite(v) else round(float(v), 1) for v in topo.hbm_gbps]
    if topo.numa_distance:
        d["numa_distance"] = {str(k): list(v) for k, v in topo.numa_distance.items()}
    if topo.nics:
        d["nics"] = topo.nics
        d["gpu_nic"] = topo.gpu_nic
    # cost only when it is not derivable (fixtures with explicit costs)
    probe_copy = _decode_no_cost(d)
    if not np.array_equal(np.round(probe_copy.cost, 6), np.round(topo.cost, 6)):
        m["cost"] = pack_matrix(np.round(topo.cost, 6), "f64")
    return d


def _decode_no_cost(d: Dict[str, Any]):
    return decode_v2({**d, "m": {k: v for k, v in d["m"].items() if k != "cost"}})


def decode_v2(d: Dict[str, Any]):
    from .model import GPUInfo, Topology

    n = int(d["n"])
    cols = d.get("gpus") or {}
    gpus = []
    for i in range(n):
        kw: Dict[str, Any] = {"index": i}
        for k, v in cols.items():
            kw[k] = v[i] if isinstance(v, list) else v
        gpus.append(GPUInfo(**kw))
    m = d.get("m") or {}

    def mat(key) -> Optional[np.ndarray]:
        return unpack_matrix(m[key], n) if key in m else None

    probe = dict(d.get("probe") or {})
    for key in ("raw_gbps", "spread"):
        a = mat(key)
        if a is not None:
            probe[key] = [[None if not math.isfinite(x) else float(x) for x in row] for row in a.tolist()]
    mx = mat("max_bw_mbps")
    if mx is not None:
        probe["amdsmi_max_bw_mbps"] = mx.tolist()
    hbm = d.get("hbm_gbps")
    lt, hops, rc = mat("link_type"), mat("hops"), mat("ref_class")
    return Topology(
        gpus=gpus,
        link_type=lt.astype(np.int32),
        hops=hops.astype(np.int32),
        weight=mat("weight"),
        bw_gbps=mat("bw_gbps"),
        cost=mat("cost"),
        ref_gbps=float(d.get("ref_gbps", 76.5)),
        node_name=str(d.get("node", "")),
        source=str(d.get("source", "unknown")),
        probe=probe,
        ref_class=None if rc is None else rc.astype(np.int32),
        hbm_gbps=None if hbm is None else np.array([np.nan if v is None else v for v in hbm], dtype=np.float64),
        numa_distance={int(k): [int(x) for x in v] for k, v in d["numa_distance"].items()} if d.get("numa_distance") else None,
        nics=d.get("nics") or None,
        gpu_nic=d.get("gpu_nic") or None,
    )
