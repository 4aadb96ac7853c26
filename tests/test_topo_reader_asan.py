"""The KFD sysfs reader (``csrc/topo/topo_reader.cpp``) under AddressSanitizer + UBSan, fed corrupted trees.

SURVEY.md §5.2 asks for the host-side C++ built with ``-fsanitize=address,undefined``.  The reader parses
files the node's kernel writes, which a driver bug, a partial hot-unplug or a half-written RAS file can
leave in any state; it must never crash the device plugin.  ``bin/topo_selftest`` is the reader compiled
with the sanitizers (``csrc/topo/topo_selftest.cpp``, no Python).  This test writes the 8 x MI355X
fixture tree, makes copies with random corruptions per seed -- garbage, empty, huge, negative and very
long values, deleted files and directories, stray non-numeric entries -- and runs the binary over all of
them: every tree must give a result or a clean exception, and no sanitizer may report.
"""
import os
import random
import shutil
import subprocess

import pytest

from gpu_topology_on_k8s_amd._native import NativeUnavailable, binary
from gpu_topology_on_k8s_amd.topology import fixtures as fx

VALUES = ["", "\n", "garbage", "-1", "18446744073709551615", "99999999999999999999999999",
          "0x7f", "3.5", "nan", "ue: -4\nce: x", "\x00\xff\xfe", "1 2 3 4 5 6 7", "x" * 200000]
KEYS = ("node_from", "node_to", "type", "weight", "simd_count", "simd_per_cu", "location_id", "domain",
        "drm_render_minor", "unique_id", "gfx_target_version", "local_mem_size")
NAMES = ["foo", ".hidden", "99999999999999999999", "card", "cardX", "node", "nodeQ", "-3", "0000"]


def _selftest():
    try:
        return str(binary("topo_selftest"))
    except NativeUnavailable as e:
        pytest.skip(str(e))


def _mutate(root: str, rng: random.Random) -> None:
    files, dirs = [], []
    for d, ds, fs in os.walk(root, followlinks=False):
        dirs += [os.path.join(d, x) for x in ds]
        files += [os.path.join(d, x) for x in fs]
    for _ in range(rng.randint(1, 6)):
        op = rng.random()
        if op < 0.55 and files:
            f = rng.choice(files)
            if os.path.isfile(f) and not os.path.islink(f):
                with open(f, "w", errors="surrogateescape") as h:
                    if rng.random() < 0.5:
                        h.write(rng.choice(VALUES))
                    else:
                        h.write("\n".join(f"{k} {rng.choice(VALUES)}" for k in KEYS))
        elif op < 0.7 and files:
            f = rng.choice(files)
            if os.path.lexists(f):
                os.unlink(f)
        elif op < 0.8 and dirs:
            d = rng.choice(dirs)
            if os.path.isdir(d) and not os.path.islink(d):
                shutil.rmtree(d, ignore_errors=True)
        elif dirs:
            d = rng.choice(dirs)
            if os.path.isdir(d) and not os.path.islink(d):
                os.makedirs(os.path.join(d, rng.choice(NAMES)), exist_ok=True)


def _roots(p):
    return [p["kfd"], p["drm"], p["pci"], p["node"], p["ib"]]


def _run(exe, args):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    p = subprocess.run([exe] + args, capture_output=True, text=True, env=env, timeout=600)
    log = p.stdout + p.stderr
    assert "AddressSanitizer" not in log and "runtime error:" not in log and "LeakSanitizer" not in log, log[-4000:]
    assert p.returncode == 0, log[-4000:]
    return p.stdout.splitlines()


def test_selftest_reads_the_intact_fixture(tmp_path):
    exe = _selftest()
    p = fx.write_fake_kfd_sysfs(str(tmp_path), nics=True, ras={1: {"umc": (2, 5), "gfx": (1, 0), "bad_pages": 3}})
    assert _run(exe, _roots(p)) == ["ok 8 8"]


def test_sysfs_reader_survives_corrupted_trees_under_asan(tmp_path):
    exe = _selftest()
    base = str(tmp_path / "base")
    paths = fx.write_fake_kfd_sysfs(base, nics=True, ras={1: {"umc": (2, 5), "gfx": (1, 0), "bad_pages": 3}})
    seeds = int(os.environ.get("GTK_TOPO_FUZZ_SEEDS", "200"))
    args = []
    for seed in range(seeds):
        work = str(tmp_path / f"s{seed}")
        shutil.copytree(base, work, symlinks=True)
        _mutate(work, random.Random(seed))
        args += [r.replace(base, work) for r in _roots(paths)]
    lines = _run(exe, args)
    assert len(lines) == seeds, lines[-5:]
    ok = sum(1 for x in lines if x.startswith("ok "))
    # most corruptions leave a readable node: a stray or garbage entry is skipped, not fatal
    assert ok >= seeds // 2, lines
