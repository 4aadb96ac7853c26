"""Build every native component in-tree (no JIT cache, no pip install).

    python -m gpu_topology_on_k8s_amd._native.build [--force] [--only _probe,_rccl] [-j 8]

Targets (all land in ``gpu_topology_on_k8s_amd/_native/``):
  _topo       C++  (g++)    amdsmi (dlopen) + KFD sysfs topology reader
  bin/libfake_amdsmi.so     stand-in amdsmi for CPU tests of the reader's multi-GPU paths
  bin/topo_selftest         ASan/UBSan host build of the sysfs reader, fed corrupted trees
  _placement  C++  (g++)    branch-and-bound placement engine
  bin/engine_selftest       ASan/UBSan host build of the engine checked against brute force
  _probe      HIP  (hipcc)  gfx950 link/HBM probe kernels + MFMA warm-up
  _rccl       HIP  (hipcc)  RCCL all-reduce validator (librccl)
  _fused      HIP  (hipcc)  PyTorch custom ops for the Llama-3 workload (torch headers)
  bin/rccl_allreduce_bench  standalone validator binary
  bin/libgtk_vgpu.so        C++  (g++)    ROCr-level HBM/CU guard preloaded into time-sliced pods (csrc/vgpu)
  bin/fake_hip/libamdhip64.so             stand-in HIP runtime for CPU tests of the guard
  bin/fake_hip/libhsa-runtime64.so        stand-in ROCr runtime under it
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shlex
import subprocess
import sys
import sysconfig
from dataclasses import dataclass, field
from pathlib import Path
from typing import Dict, List, Optional

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
CSRC = REPO / "csrc"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("GTK_OFFLOAD_ARCH", "gfx950")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _py_includes() -> List[str]:
    import pybind11

    return [f"-I{sysconfig.get_paths()['include']}", f"-I{pybind11.get_include()}"]


def _torch_flags() -> List[str]:
    import torch
    from torch.utils import cpp_extension as ce

    inc = [f"-I{p}" for p in ce.include_paths()]
    libdir = str(Path(torch.__file__).parent / "lib")
    return inc + [
        "-D__HIP_PLATFORM_AMD__=1",
        "-DUSE_ROCM=1",
        "-DTORCH_EXTENSION_NAME=_fused",
        f"-D_GLIBCXX_USE_CXX11_ABI={int(torch._C._GLIBCXX_USE_CXX11_ABI)}",
        f"-L{libdir}",
        "-lc10",
        "-ltorch",
        "-ltorch_cpu",
        "-ltorch_python",
        "-lc10_hip",
        "-ltorch_hip",
        f"-Wl,-rpath,{libdir}",
    ]


@dataclass
class Target:
    name: str
    sources: List[Path]
    compiler: str  # "gxx" | "hipcc"
    out: Path
    extra: List[str] = field(default_factory=list)
    deps: List[Path] = field(default_factory=list)
    pybind: bool = True
    torch: bool = False
    shared: bool = True
    src_flags: Dict[str, List[str]] = field(default_factory=dict)  # extra compile flags per source file name

    def command(self) -> List[str]:
        if self.compiler == "hipcc":
            cmd = [str(ROCM / "bin" / "hipcc"), f"--offload-arch={ARCH}", "-O3", "-std=c++17"]
        else:
            cmd = ["g++", "-O3", "-std=c++17", "-Wall", "-Wno-unused-function"]
        if self.shared:
            cmd += ["-shared", "-fPIC", "-fvisibility=hidden"]
        cmd += [f"-I{ROCM / 'include'}", f"-I{CSRC}"]
        if self.pybind:
            cmd += _py_includes()
        cmd += [str(s) for s in self.sources]
        if self.torch:
            cmd += _torch_flags()
        cmd += self.extra
        cmd += ["-o", str(self.out)]
        return cmd

    def compile_flags(self) -> List[str]:
        """Per-object compile command prefix (multi-source hipcc targets: one object per source)."""
        cmd = [str(ROCM / "bin" / "hipcc"), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden",
               f"-I{ROCM / 'include'}", f"-I{CSRC}"]
        if self.pybind:
            cmd += _py_includes()
        if self.torch:
            cmd += [f for f in _torch_flags() if f.startswith(("-I", "-D"))]
        return cmd

    def link_flags(self) -> List[str]:
        flags = [f for f in _torch_flags() if not f.startswith(("-I", "-D"))] if self.torch else []
        return flags + [f for f in self.extra if not f.startswith(("-I", "-D"))]

    def up_to_date(self) -> bool:
        if not self.out.exists():
            return False
        t = self.out.stat().st_mtime
        inputs = list(self.sources) + list(self.deps) + [Path(__file__)]
        return all(p.stat().st_mtime <= t for p in inputs if p.exists())


def targets() -> List[Target]:
    rocm_lib = str(ROCM / "lib")
    return [
        Target("_topo", [CSRC / "topo" / "topo_reader.cpp"], "gxx", HERE / f"_topo{EXT}", ["-ldl"]),
        # host-only sanitizer build of the sysfs reader; run by tests/test_topo_reader_asan.py
        Target("topo_selftest", [CSRC / "topo" / "topo_selftest.cpp"], "gxx", HERE / "bin" / "topo_selftest",
               ["-g", "-O1", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer",
                "-ldl"], deps=[CSRC / "topo" / "topo_reader.cpp"], pybind=False, shared=False),
        Target("fake_amdsmi", [CSRC / "topo" / "fake_amdsmi.cpp"], "gxx", HERE / "bin" / "libfake_amdsmi.so",
               ["-fvisibility=default"], pybind=False),
        Target("_placement", [CSRC / "placement" / "engine.cpp", CSRC / "placement" / "engine_module.cpp"], "gxx",
               HERE / f"_placement{EXT}", deps=[CSRC / "placement" / "engine.h"]),
        # host-only sanitizer build of the engine; run by tests/test_placement.py
        Target("engine_selftest", [CSRC / "placement" / "engine.cpp", CSRC / "placement" / "engine_selftest.cpp"], "gxx",
               HERE / "bin" / "engine_selftest", ["-g", "-O1", "-fsanitize=address,undefined", "-fno-omit-frame-pointer"],
               deps=[CSRC / "placement" / "engine.h"], pybind=False, shared=False),
        Target("_probe", [CSRC / "probe" / "probe.hip"], "hipcc", HERE / f"_probe{EXT}"),
        Target("_rccl", [CSRC / "rccl" / "rccl_module.hip"], "hipcc", HERE / f"_rccl{EXT}",
               [f"-L{rocm_lib}", "-lrccl", f"-Wl,-rpath,{rocm_lib}"], deps=[CSRC / "rccl" / "rccl_core.h"]),
        Target("rccl_allreduce_bench", [CSRC / "rccl" / "rccl_allreduce_bench.hip"], "hipcc",
               HERE / "bin" / "rccl_allreduce_bench", [f"-L{rocm_lib}", "-lrccl", f"-Wl,-rpath,{rocm_lib}"],
               deps=[CSRC / "rccl" / "rccl_core.h"], pybind=False, shared=False),
        # container-side tier of a time-sliced share (Gaia vGPU): HBM cap + forced CU mask, preloaded into
        # the pod by Allocate (--share-guard); host-only C++, resolves the real HIP entry points at run time
        Target("vgpu_guard", [CSRC / "vgpu" / "vgpu_guard.cpp"], "gxx", HERE / "bin" / "libgtk_vgpu.so",
               ["-fvisibility=hidden", "-ldl", "-pthread"], pybind=False),
        # stand-in ROCr + HIP runtimes for CPU tests of the guard, layered like the real pair (the HIP
        # stand-in links the ROCr one as libhsa-runtime64.so, found next to it)
        Target("fake_hsa", [CSRC / "vgpu" / "fake_hsa.cpp"], "gxx", HERE / "bin" / "fake_hip" / "libhsa-runtime64.so",
               ["-fvisibility=default", "-pthread", "-Wl,-soname,libhsa-runtime64.so"], pybind=False),
        Target("fake_hip", [CSRC / "vgpu" / "fake_hip.cpp"], "gxx", HERE / "bin" / "fake_hip" / "libamdhip64.so",
               ["-fvisibility=default", f"-L{HERE / 'bin' / 'fake_hip'}", "-l:libhsa-runtime64.so", "-Wl,--disable-new-dtags", "-Wl,-rpath,$ORIGIN"],
               deps=[HERE / "bin" / "fake_hip" / "libhsa-runtime64.so"], pybind=False),
        # the guard under ThreadSanitizer and under ASan/UBSan (host code only), stressed by many threads
        # against the stand-in runtimes (tests/test_vgpu_guard.py)
        Target("vgpu_selftest_tsan", [CSRC / "vgpu" / "vgpu_guard.cpp", CSRC / "vgpu" / "vgpu_selftest.cpp"], "gxx",
               HERE / "bin" / "vgpu_selftest_tsan",
               ["-g", "-O1", "-fsanitize=thread", "-pthread", "-ldl", f"-L{HERE / 'bin' / 'fake_hip'}", "-l:libamdhip64.so",
                "-l:libhsa-runtime64.so", "-Wl,--disable-new-dtags", f"-Wl,-rpath,{HERE / 'bin' / 'fake_hip'}"],
               deps=[HERE / "bin" / "fake_hip" / "libamdhip64.so"], pybind=False, shared=False),
        Target("vgpu_selftest_asan", [CSRC / "vgpu" / "vgpu_guard.cpp", CSRC / "vgpu" / "vgpu_selftest.cpp"], "gxx",
               HERE / "bin" / "vgpu_selftest_asan",
               ["-g", "-O1", "-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-pthread", "-ldl",
                f"-L{HERE / 'bin' / 'fake_hip'}", "-l:libamdhip64.so", "-l:libhsa-runtime64.so", "-Wl,--disable-new-dtags",
                f"-Wl,-rpath,{HERE / 'bin' / 'fake_hip'}"],
               deps=[HERE / "bin" / "fake_hip" / "libamdhip64.so"], pybind=False, shared=False),
        # attention.hip: MFMAs whose accumulators the code does not pin to AGPRs take the VGPR form even in
        # the one-wave-per-SIMD dK/dV kernel (its S / dP chains feed the softmax VALU directly; the dV/dK
        # accumulators are pinned to AGPRs by their asm constraints).  The other kernels of the file fit
        # 256 VGPRs and select that form anyway.
        Target("_fused", sorted((CSRC / "ops").glob("*.hip")), "hipcc", HERE / f"_fused{EXT}",
               deps=sorted((CSRC / "ops").glob("*.h")), pybind=True, torch=True,
               src_flags={"attention.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]}),
    ]


OBJ = HERE / "obj"  # per-source objects of multi-source hipcc targets (git- and gpurun-ignored)


def _run(cmd: List[str], what: str, verbose: bool) -> None:
    if verbose:
        print(" ".join(shlex.quote(c) for c in cmd), flush=True)
    p = subprocess.run(cmd, capture_output=True, text=True)
    if p.returncode != 0:
        raise RuntimeError(f"build of {what} failed ({p.returncode}):\n{' '.join(cmd)}\n{p.stdout}\n{p.stderr}")


def _build_objects(t: Target, force: bool, verbose: bool, jobs: int) -> str:
    """Multi-source hipcc target: compile every source to its own object in parallel (only the
    sources changed since their object was built), then link.  The gfx950 device code of each
    translation unit is self-contained, so no relocatable device code is needed."""
    odir = OBJ / t.name
    odir.mkdir(parents=True, exist_ok=True)
    dep_t = max([p.stat().st_mtime for p in list(t.deps) + [Path(__file__)] if p.exists()] or [0.0])
    flags = t.compile_flags()

    def one(src: Path) -> Path:
        obj = odir / (src.stem + ".o")
        if force or not obj.exists() or obj.stat().st_mtime < max(src.stat().st_mtime, dep_t):
            _run(flags + t.src_flags.get(src.name, []) + ["-c", str(src), "-o", str(obj)], f"{t.name}:{src.name}", verbose)
        return obj

    with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, len(t.sources)))) as ex:
        objs = list(ex.map(one, t.sources))
    if not force and t.out.exists() and all(o.stat().st_mtime <= t.out.stat().st_mtime for o in objs) and t.up_to_date():
        return f"ok   {t.name} (up to date)"
    t.out.parent.mkdir(parents=True, exist_ok=True)
    _run([str(ROCM / "bin" / "hipcc"), f"--offload-arch={ARCH}", "-shared", "-fPIC"] + [str(o) for o in objs]
         + t.link_flags() + ["-o", str(t.out)], t.name, verbose)
    return f"built {t.name} -> {t.out.relative_to(REPO)} ({len(objs)} objects)"


def build_one(t: Target, force: bool = False, verbose: bool = False, jobs: int = 4) -> str:
    missing = [s for s in t.sources if not s.exists()]
    if not t.sources or missing:
        return f"skip {t.name} (no sources)"
    if not force and t.up_to_date():
        return f"ok   {t.name} (up to date)"
    if t.compiler == "hipcc" and t.shared and len(t.sources) > 1:
        return _build_objects(t, force, verbose, jobs)
    t.out.parent.mkdir(parents=True, exist_ok=True)
    cmd = t.command()
    if verbose:
        print(" ".join(shlex.quote(c) for c in cmd), flush=True)
    p = subprocess.run(cmd, capture_output=True, text=True)
    if p.returncode != 0:
        raise RuntimeError(f"build of {t.name} failed ({p.returncode}):\n{' '.join(cmd)}\n{p.stdout}\n{p.stderr}")
    return f"built {t.name} -> {t.out.relative_to(REPO)}"


def build(force: bool = False, only: Optional[List[str]] = None, jobs: int = 4, verbose: bool = False) -> List[str]:
    ts = [t for t in targets() if not only or t.name in only]
    msgs: List[str] = []
    errors: List[str] = []
    # targets that link another target's output (the stand-in HIP runtime links the stand-in ROCr, the
    # guard self-tests link both) are built in a later wave than what they link: topological layers
    producer = {t.out: t for t in targets()}

    def depth(t: Target) -> int:
        return 1 + max((depth(producer[d]) for d in t.deps if d in producer), default=-1)

    layers = [depth(t) for t in ts]
    waves = [[t for t, d in zip(ts, layers) if d == k] for k in range(max(layers, default=-1) + 1)]
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for wave in waves:
            futs = {ex.submit(build_one, t, force, verbose, jobs): t for t in wave}
            for f in cf.as_completed(futs):
                try:
                    msgs.append(f.result())
                except Exception as e:  # noqa: BLE001 - report all failures together
                    errors.append(str(e))
    if errors:
        raise RuntimeError("\n\n".join(errors))
    return sorted(msgs)


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", default="")
    ap.add_argument("-j", "--jobs", type=int, default=4)
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    only = [s for s in a.only.split(",") if s] or None
    for m in build(a.force, only, a.jobs, a.verbose):
        print(m)
    return 0


if __name__ == "__main__":
    sys.exit(main())
