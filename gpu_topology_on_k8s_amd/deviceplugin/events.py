"""GPU event notifications for the device plugin (SURVEY.md §5.3 failure detection).

The RAS health pass (:mod:`.health`) polls every ``--health-interval`` seconds; a GPU reset, however,
kills every queue on the device the moment it starts, and pods admitted in between would land on a
GPU that is going away.  amdsmi delivers such events as they happen
(``amdsmi_init_gpu_event_notification`` / ``amdsmi_get_gpu_event_notification``, read natively by
``csrc/topo/topo_reader.cpp`` ``EventWatcher``); this module runs that watcher on its own thread and
hands each event, keyed by PCI address, to :meth:`DevicePluginServer.gpu_event`.

The reference has no health signal at all (``design.md:84-86``: an ``isUsed`` bit per device).
"""
from __future__ import annotations

import logging
import os
import threading
from typing import Callable, List, Optional, Sequence, Tuple

log = logging.getLogger(__name__)

__all__ = ["GpuEventWatcher", "DEFAULT_KINDS"]

DEFAULT_KINDS = ("GPU_PRE_RESET", "GPU_POST_RESET", "VMFAULT", "THERMAL_THROTTLE")

Event = Tuple[str, str, str]  # (PCI address, kind, message)


class GpuEventWatcher:
    """Polls amdsmi GPU events and forwards them to the plugin.  ``source`` (tests) is any object with
    ``poll(timeout_ms, max_events) -> [(bdf, kind, message)]`` and ``close()``; by default the native
    ``_topo.EventWatcher`` over ``lib`` (``$GTK_AMDSMI_LIB`` or ``libamd_smi.so``)."""

    def __init__(self, lib: Optional[str] = None, kinds: Sequence[str] = DEFAULT_KINDS, poll_ms: int = 1000,
                 source=None):
        self.poll_ms = int(poll_ms)
        if source is None:
            from .._native import load

            lib = lib or os.environ.get("GTK_AMDSMI_LIB", "") or "libamd_smi.so"
            source = load("_topo").EventWatcher(lib, list(kinds))
        self.source = source
        self.delivered: List[Event] = []
        self.unmatched = 0  # events for a PCI address this plugin does not advertise

    @classmethod
    def try_open(cls, lib: Optional[str] = None, **kw) -> Optional["GpuEventWatcher"]:
        """The watcher, or None (logged) where amdsmi or its event API is unavailable (sysfs-only or
        fake nodes, no permission on the device files): the RAS poll still runs."""
        try:
            return cls(lib, **kw)
        except Exception as e:  # noqa: BLE001 - optional capability
            log.info("GPU event notification unavailable (%s); relying on the health poll", e)
            return None

    def run(self, plugin, stop: threading.Event, index_of: Optional[Callable[[str], Optional[int]]] = None) -> None:
        """Thread body: poll until ``stop``, then close the native watcher."""
        try:
            while not stop.is_set():
                try:
                    events = self.source.poll(self.poll_ms, 64)
                except Exception as e:  # noqa: BLE001 - keep watching; a broken source backs off
                    log.warning("GPU event poll failed: %s", e)
                    stop.wait(5.0)
                    continue
                for bdf, kind, msg in events:
                    idx = (index_of or _index_by_bdf(plugin))(bdf)
                    if idx is None:
                        self.unmatched += 1
                        continue
                    self.delivered.append((bdf, kind, msg))
                    try:
                        plugin.gpu_event(idx, kind, msg)
                    except Exception as e:  # noqa: BLE001
                        log.warning("GPU event %s on %s not applied: %s", kind, bdf, e)
        finally:
            try:
                self.source.close()
            except Exception:  # noqa: BLE001
                pass


def _index_by_bdf(plugin) -> Callable[[str], Optional[int]]:
    def find(bdf: str) -> Optional[int]:
        key = (bdf or "").lower()
        for g in plugin.topology.gpus:
            if g.bdf and g.bdf.lower() == key:
                return g.index
        return None

    return find
