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


#: extensions that call the HIP runtime (built by hipcc against /opt/rocm)
_HIP_MODULES = ("_probe", "_rccl", "_fused")


def load(name: str) -> ModuleType:
    """Import one in-tree extension.

    The PyTorch wheel ships its own HIP/HSA runtime and RCCL (``torch/lib``, no SONAME).  Python
    loads extension modules RTLD_LOCAL, so an extension imported BEFORE torch brings up
    ``/opt/rocm``'s runtime, and a later ``import torch`` adds a second HSA runtime to the process;
    RCCL (torch's, which ``_rccl``'s calls bind to once torch is in the global scope) then finds "no
    ROCm-capable device".  So torch is imported first whenever it is installed, and every HIP call of
    the process goes through one runtime."""
    if name in _CACHE:
        return _CACHE[name]
    if name in _HIP_MODULES:
        try:
            import torch  # noqa: F401 - must precede the extension (one HIP runtime per process)
        except ImportError:  # pragma: no cover - torch-less images use /opt/rocm's runtime
            pass
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
