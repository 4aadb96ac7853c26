"""In-tree native extensions (built by ``python -m gpu_topology_on_k8s_amd._native.build``).

``load(name)`` imports one of ``_topo``, ``_placement``, ``_probe``, ``_rccl``, ``_fused`` and raises
:class:`NativeUnavailable` with the build command when it is missing — GPU paths never silently
fall back to Python.
"""
from __future__ import annotations

import importlib
from pathlib import Path
from types import ModuleType
from typing import Dict

HERE = Path(__file__).resolve().parent
_CACHE: Dict[str, ModuleType] = {}


class NativeUnavailable(ImportError):
    pass


def load(name: str) -> ModuleType:
    if name in _CACHE:
        return _CACHE[name]
    try:
        mod = importlib.import_module(f"{__name__}.{name}")
    except ImportError as e:  # pragma: no cover - message path
        raise NativeUnavailable(
            f"native extension {name!r} is not built or failed to load ({e}); run "
            f"`python -m gpu_topology_on_k8s_amd._native.build`"
        ) from e
    _CACHE[name] = mod
    return mod


def available(name: str) -> bool:
    try:
        load(name)
        return True
    except NativeUnavailable:
        return False


def binary(name: str) -> Path:
    p = HERE / "bin" / name
    if not p.exists():
        raise NativeUnavailable(f"native binary {name!r} missing; run `python -m gpu_topology_on_k8s_amd._native.build`")
    return p
