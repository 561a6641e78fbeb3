"""CPU check of the Kendall engine's bit-parallel pair counting (visreps_amd/csrc/kcount.h):
the same header the HIP kernels include, compiled for the host with g++ and compared with
brute-force counts over random streams, segment starts and range splits."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_kcount_against_brute_force(tmp_path):
    exe = tmp_path / "kcount_test"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "visreps_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "kcount_test.cpp"), "-o", str(exe)],
                   check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "kcount ok" in r.stdout
