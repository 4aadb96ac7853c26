"""The CMake build (CMakeLists.txt / CMakePresets.json): host code configures,
builds under ASan + UBSan and passes the placement-engine self-test (exact search vs brute force)."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("cmake") is None or shutil.which("ninja") is None, reason="cmake/ninja not installed")
def test_cmake_asan_host_build_and_selftest(tmp_path):
    b = tmp_path / "asan"
    run = lambda *cmd: subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=600)
    p = run("cmake", "-S", REPO, "-B", str(b), "-G", "Ninja", "-DCMAKE_BUILD_TYPE=Debug", "-DGTK_HIP=OFF", "-DGTK_SANITIZE=ON",
            "-DGTK_INPLACE=OFF")
    assert p.returncode == 0, p.stdout + p.stderr
    p = run("cmake", "--build", str(b), "-j", "4")
    assert p.returncode == 0, p.stdout[-4000:] + p.stderr[-4000:]
    p = subprocess.run(["ctest", "--output-on-failure"], cwd=b, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0 and "100% tests passed" in p.stdout, p.stdout[-4000:]
