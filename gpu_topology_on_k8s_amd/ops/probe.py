"""Python front-end of the HIP/CDNA4 link probe (``csrc/probe/probe.hip``).

Seeds the link-cost matrix at node start (BASELINE.json north_star):

    mfma_warmup (K4)  ->  p2p read (K1) for every ordered pair  ->  GB/s matrix  ->  cost matrix

With one visible GPU only the diagonal (K3 HBM self-copy) is measurable; off-diagonal entries are
left unmeasured (nan) and the cost model falls back to the discovered link class.
"""
from __future__ import annotations

import logging
import os
import subprocess
import sys
import tempfile
import time
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .._native import load
from ..topology.identity import DeviceMap
from ..topology.model import Topology

log = logging.getLogger(__name__)

__all__ = ["device_count", "device_props", "warmup", "copy_bw", "gather_bw", "measure_matrix", "measure_ingress",
           "probe_topology", "probe_in_child", "ingress_bound", "ring_peers", "ring_bw", "measure_ring", "ring_in_child",
           "PROBE_PRESETS"]

#: bytes per transfer / timed iterations / repeats of every pair (the link's median is published, its
#: spread decides which links are noise-equivalent: ops/checks.py band_links); sizes exceed the 256 MiB
#: Infinity Cache for "full".
PROBE_PRESETS: Dict[str, Dict[str, int]] = {
    "quick": {"bytes": 64 << 20, "iters": 3, "warmup": 1, "repeats": 5},
    "full": {"bytes": 512 << 20, "iters": 10, "warmup": 2, "repeats": 5},
}

#: the K3 HBM self-copy reads and writes at least this much in every preset: 2 x 1 GiB is far past the
#: 256 MiB Infinity Cache, which a quick preset's 2 x 64 MiB would fit (profiles/r06_prof: 3.1-3.2 TB/s
#: at 64 MiB, 2.8 TB/s at 512 MiB)
HBM_COPY_MIN_BYTES = 1 << 30


def _p():
    return load("_probe")


def device_count() -> int:
    return int(_p().device_count())


def device_props(dev: int) -> Dict[str, object]:
    return dict(_p().device_props(dev))


def warmup(dev: int, ms: float = 50.0, random_operands: bool = False) -> Dict[str, object]:
    """K4: run MFMA until ``ms`` elapsed so the measured copies see lifted clocks.  ``random_operands``:
    cycle pseudo-random bf16 fragments instead (the power-limited MFMA rate real GEMM data sees)."""
    return dict(_p().mfma_warmup(dev, float(ms), 4096, bool(random_operands)))


def copy_bw(src: int, dst: int, nbytes: int = 256 << 20, iters: int = 10, warmup_iters: int = 2, mode: str = "read",
            kind: str = "lds", nontemporal: bool = False, blocks_per_cu: int = 8) -> Dict[str, object]:
    exec_dev = dst if mode == "read" else src
    return dict(_p().copy_bw(src, dst, exec_dev, int(nbytes), int(iters), int(warmup_iters), kind, bool(nontemporal), int(blocks_per_cu)))


def gather_bw(dst: int, srcs: Sequence[int], nbytes: int = 64 << 20, iters: int = 3, warmup_iters: int = 1) -> Dict[str, object]:
    """K5: one kernel on ``dst`` reads ``nbytes`` from every device in ``srcs`` at once (aggregate ingress)."""
    return dict(_p().gather_bw(int(dst), [int(s) for s in srcs], int(nbytes), int(iters), int(warmup_iters)))


def ring_peers(k: int, pattern: str = "all") -> List[List[int]]:
    """Member indices each of ``k`` ring members pulls from in K6: ``all`` = every other member (the
    union of the rings RCCL lays over a full mesh: every link of the subset, both directions);
    ``ring`` = predecessor and successor of one bidirectional ring (2 links per member, 1 at k = 2)."""
    if k < 2:
        raise ValueError("a ring needs at least 2 members")
    if pattern == "all":
        return [[p for p in range(k) if p != m] for m in range(k)]
    if pattern == "ring":
        return [sorted({(m - 1) % k, (m + 1) % k} - {m}) for m in range(k)]
    raise ValueError(f"pattern must be all|ring, got {pattern!r}")


def ring_bw(devs: Sequence[int], pattern: str = "all", nbytes: int = 64 << 20, iters: int = 3,
            warmup_iters: int = 1) -> Dict[str, object]:
    """K6: every member (HIP ordinal ``devs[m]``) gathers from its ``pattern`` peers at the same time;
    ``bound_gbps`` = the slowest member's ingress (the ceiling of a ring all-reduce's busBW)."""
    r = dict(_p().ring_bw([int(d) for d in devs], ring_peers(len(devs), pattern), int(nbytes), int(iters), int(warmup_iters)))
    r["pattern"] = pattern
    return r


def measure_ring(devs: Sequence[int], preset: str = "quick", patterns: Sequence[str] = ("all", "ring")) -> Dict[str, object]:
    """K6 over the HIP ordinals ``devs`` for each pattern; ``ring_bound_gbps`` is the ``all`` pattern's
    bound (every link of the subset loaded at once: what RCCL's rings do together on a full mesh)."""
    cfg = PROBE_PRESETS[preset]
    out: Dict[str, object] = {"devices": [int(d) for d in devs], "preset": preset, "bytes_per_peer": cfg["bytes"]}
    for pat in patterns:
        r = ring_bw(devs, pat, cfg["bytes"], cfg["iters"], cfg["warmup"])
        if not r["ok"]:
            raise RuntimeError(f"ring probe ({pat}) verification failed on devices {list(devs)}")
        out[pat] = {"ingress_gbps": [round(float(x), 2) for x in r["ingress_gbps"]], "bound_gbps": round(float(r["bound_gbps"]), 2),
                    "wall_ms": round(float(r["wall_ms"]), 3), "ms_member": [round(float(x), 3) for x in r["ms_member"]]}
    if "all" in out:
        out["ring_bound_gbps"] = out["all"]["bound_gbps"]
    return out


def ring_in_child(devs: Sequence[int], preset: str = "quick", timeout: float = 120.0) -> Tuple[Optional[Dict[str, object]], str]:
    """:func:`measure_ring` in a child process (``gtk ring --devices``): the caller keeps no HIP
    context or buffers on the subset's GPUs.  Returns ``(result | None, message)``."""
    import json

    cmd = [sys.executable, "-m", "gpu_topology_on_k8s_amd", "ring", "--devices", ",".join(str(int(d)) for d in devs),
           "--preset", preset]
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=root)
    except subprocess.TimeoutExpired:
        return None, f"ring probe timed out after {timeout:.0f}s"
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if p.returncode != 0 or not lines:
        return None, f"ring probe exited {p.returncode}: {(p.stderr or p.stdout).strip()[-400:]}"
    return json.loads(lines[-1]), "ok"


def _device_map(topo: Topology, dmap: Optional[DeviceMap]) -> DeviceMap:
    if dmap is not None:
        return dmap
    m = DeviceMap.for_topology(topo)
    if not m.by_bdf and m.n_visible != topo.n:
        log.warning("topology has %d devices, HIP sees %d and no PCI address matches: probing HIP ordinals "
                    "0..%d as topology indices", topo.n, m.n_visible, len(m.hip_of_index) - 1)
    return m


def measure_ingress(topo: Topology, devs: Sequence[int], preset: str = "quick",
                    dmap: Optional[DeviceMap] = None, by_package: bool = True) -> List[Optional[float]]:
    """Aggregate ingress GB/s of every topology device in ``devs`` reading from all the others
    concurrently (K5); stored in ``topo.probe["ingress_all_gbps"]`` (None where fewer than two
    devices).  Topology indices are turned into HIP ordinals by PCI address (:class:`DeviceMap`).
    On a partitioned node (``by_package``) the first XCP of each package gathers from the first XCP
    of every other package and the number is shared by the package's XCPs (8 gathers on a CPX node,
    not 64 x 63-way)."""
    cfg = PROBE_PRESETS[preset]
    m = _device_map(topo, dmap)
    devs = [d for d in devs if d in m.hip_of_index]
    out: List[Optional[float]] = [None] * topo.n
    phys = topo.physical
    rep_of = {d: d for d in devs}
    if by_package and len(set(phys.tolist())) < topo.n:
        first: Dict[int, int] = {}
        for d in devs:
            first.setdefault(int(phys[d]), d)
        rep_of = {d: first[int(phys[d])] for d in devs}
    reps = sorted(set(rep_of.values()))
    for d in reps:
        hd = m.hip(d)
        peers = [m.hip(s) for s in reps if s != d and bool(_p().can_access_peer(hd, m.hip(s)))]
        if not peers:
            continue
        r = gather_bw(hd, peers, cfg["bytes"], cfg["iters"], cfg["warmup"])
        if not r["ok"]:
            raise RuntimeError(f"ingress probe verification failed on device {d}")
        out[d] = round(float(r["gbps"]), 2)
    for d in devs:
        out[d] = out[rep_of[d]]
    topo.probe = dict(topo.probe, ingress_all_gbps=out)
    return out


def ingress_bound(topo: Topology, subset: Sequence[int]) -> Optional[float]:
    """Probe-derived ceiling of an all-reduce's busBW on ``subset``: each member's ingress over its
    |subset|-1 links (sum of the measured pairwise reads, capped by its measured all-peer ingress),
    minimum over members.  busBW = bytes each GPU sends / time, so it cannot exceed this."""
    subset = list(subset)
    if len(subset) < 2 or topo.bw_gbps is None:
        return None
    ing = (topo.probe or {}).get("ingress_all_gbps") or [None] * topo.n
    best = None
    for d in subset:
        links = [float(topo.bw_gbps[s, d]) for s in subset if s != d]
        if not all(np.isfinite(links)):
            return None
        cap = sum(links)
        if ing[d] is not None:
            cap = min(cap, float(ing[d]))
        best = cap if best is None else min(best, cap)
    return best


def measure_matrix(devs: Sequence[int], nbytes: int = 64 << 20, iters: int = 3, warmup_iters: int = 1, mode: str = "read",
                   kind: str = "lds") -> np.ndarray:
    return np.array(_p().probe_matrix(list(devs), int(nbytes), int(iters), int(warmup_iters), mode, kind), dtype=np.float64)


def _probe_pairs(topo: Topology, devs: Sequence[int], by_package: bool):
    """Ordered (src, dst) pairs to measure, and for a partitioned node the representative pair of
    every device pair (None when each pair is measured).

    On a CPX/DPX/QPX node the XCPs of one package share that package's xGMI links and HBM, so the
    node is measured per PACKAGE pair (first visible XCP of each; plus one on-package pair and one
    self-copy per package) and every XCP pair takes its packages' number: 8 x 8 measurements instead
    of 64 x 64 on a CPX node, and XCPs of one package stay exactly interchangeable for the placement
    engine's symmetry breaking (measured noise would otherwise tell them apart)."""
    phys = topo.physical
    partitioned = len(set(phys.tolist())) < topo.n
    if not (by_package and partitioned):
        return [(i, j) for i in devs for j in devs], None
    members: Dict[int, List[int]] = {}
    for d in devs:
        members.setdefault(int(phys[d]), []).append(d)
    first = {p: ms[0] for p, ms in members.items()}
    second = {p: ms[1] for p, ms in members.items() if len(ms) > 1}
    pairs = [(first[p], first[p]) for p in first]
    pairs += [(first[p], second[p]) for p in second]
    pairs += [(first[p], first[q]) for p in first for q in first if p != q]
    rep = {}
    for i in devs:
        for j in devs:
            p, q = int(phys[i]), int(phys[j])
            if i == j:
                rep[(i, j)] = (first[p], first[p])
            elif p == q:
                rep[(i, j)] = (first[p], second.get(p, first[p]))
            else:
                rep[(i, j)] = (first[p], first[q])
    return pairs, rep


def probe_topology(topo: Topology, preset: str = "quick", devs: Optional[List[int]] = None, mode: str = "read",
                   kind: str = "lds", warm_ms: float = 50.0, dmap: Optional[DeviceMap] = None,
                   by_package: bool = True) -> Topology:
    """Measure every visible pair and fold it into ``topo`` (in place; also returned).

    ``devs`` are *topology indices* (default: every device this process can reach).  Each is run on
    the HIP ordinal with the same PCI address, so a probe under ``HIP_VISIBLE_DEVICES`` or inside a
    pod writes its numbers into the right rows of the node matrix.  ``by_package``: on a partitioned
    node measure package pairs and share the numbers among their XCPs (:func:`_probe_pairs`)."""
    cfg = PROBE_PRESETS[preset]
    ndev = device_count()
    if ndev == 0:
        raise RuntimeError("no HIP devices visible: cannot probe")
    m = _device_map(topo, dmap)
    devs = m.visible_indices() if devs is None else [d for d in devs if d in m.hip_of_index]
    if not devs:
        raise RuntimeError("none of the requested topology devices is visible to HIP")
    t0 = time.time()
    w = warmup(m.hip(devs[0]), warm_ms)
    bw = np.full((topo.n, topo.n), np.nan)
    spread = np.full((topo.n, topo.n), np.nan)
    hbm = np.full(topo.n, np.nan)
    pairs, rep = _probe_pairs(topo, devs, by_package)
    reps = max(1, int(cfg.get("repeats", 1)))
    for i, j in pairs:
        hi, hj = m.hip(i), m.hip(j)
        if i != j and not bool(_p().can_access_peer(hj if mode == "read" else hi, hi if mode == "read" else hj)):
            continue
        vals = []
        nbytes = cfg["bytes"] if i != j else max(cfg["bytes"], HBM_COPY_MIN_BYTES)
        for _ in range(reps if i != j else 1):
            r = copy_bw(hi, hj, nbytes, cfg["iters"], cfg["warmup"], mode=mode, kind=kind)
            if not r["ok"]:
                raise RuntimeError(f"probe verification failed for {i}->{j}")
            vals.append(float(r["gbps"]))
        if i == j:
            hbm[i] = vals[0]
        else:
            med = float(np.median(vals))
            bw[i, j] = med
            spread[i, j] = (max(vals) - min(vals)) / med if med > 0 else np.nan
    if rep is not None:  # partitioned node: every XCP pair takes its packages' measurement
        for i in devs:
            hbm[i] = hbm[rep[(i, i)][0]] if np.isnan(hbm[i]) else hbm[i]
        for i in devs:
            for j in devs:
                if i != j and np.isnan(bw[i, j]):
                    a, b = rep[(i, j)]
                    bw[i, j], spread[i, j] = bw[a, b], spread[a, b]
    topo.hbm_gbps = hbm
    from .checks import band_links

    banded, band_report = band_links(topo, bw, spread)

    def _rows(x, nd):
        return [[None if not np.isfinite(v) else round(float(v), nd) for v in row] for row in x]

    topo.set_measured_bw(
        banded,
        {
            "raw_gbps": _rows(bw, 2),
            "spread": _rows(spread, 4),
            "repeats": reps,
            "banding": band_report,
            "method": f"p2p_{mode}_{kind}",
            "preset": preset,
            "bytes": cfg["bytes"],
            "iters": cfg["iters"],
            "devices": devs,
            "hip_ordinals": [m.hip(d) for d in devs],
            "device_map": "bdf" if m.by_bdf else "identity",
            "pairs_measured": len(pairs),
            "granularity": "package" if rep is not None else "device",
            "mfma_warmup_tflops": round(float(w["tflops"]), 1),
            "ts": int(time.time()),
            "seconds": round(time.time() - t0, 3),
        },
    )
    return topo


def probe_in_child(preset: str = "quick", backend: str = "auto", timeout: float = 150.0,
                   ingress: bool = True, cancel=None) -> Tuple[Optional[Topology], str]:
    """Discovery + K4 warm-up + K1 p2p read of every visible ordered pair (+ K5 ingress) in a CHILD
    process (``gtk probe --out``), returned as a probed :class:`Topology`.

    Long-lived callers (the device-plugin DaemonSet, rank 0 of the bench) must not keep HIP contexts
    and probe buffers on every GPU of the node: the child takes them and exits, and a failure there
    (fault, timeout) cannot take the caller down.  The pairwise matrix is written before the ingress
    stage runs, so an ingress failure still returns it.  ``cancel`` (a ``threading.Event``): once set,
    the child is killed and reaped — its GPU memory and queues are gone when this returns — and the
    result is ``(None, "cancelled")`` (the device plugin yields its links to an arriving pod this
    way).  Returns ``(Topology | None, message)``."""
    fd, path = tempfile.mkstemp(prefix="gtk_probe_", suffix=".json")
    os.close(fd)
    cmd = [sys.executable, "-m", "gpu_topology_on_k8s_amd", "probe", "--preset", preset, "--discovery", backend, "--out", path]
    if ingress:
        cmd.append("--ingress")
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    try:
        p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, cwd=root)
        deadline = time.monotonic() + timeout
        out = err_text = ""
        while True:
            try:
                out, err_text = p.communicate(timeout=0.2)
                break
            except subprocess.TimeoutExpired:
                if cancel is not None and cancel.is_set():
                    p.kill()
                    p.communicate()
                    return None, "cancelled"
                if time.monotonic() >= deadline:
                    p.kill()
                    p.communicate()
                    return None, f"probe timed out after {timeout:.0f}s"
        err = f"probe exited {p.returncode}: {(err_text or out).strip()[-400:]}"
        with open(path) as f:
            text = f.read()
        if not text:
            return None, err
        return Topology.from_json(text), ("ok" if p.returncode == 0 else "pairwise only; ingress stage failed: " + err)
    except (OSError, ValueError, KeyError) as e:
        return None, f"probe output unreadable: {e}"
    finally:
        try:
            os.unlink(path)
        except OSError:
            pass
