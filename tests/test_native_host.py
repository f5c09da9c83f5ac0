"""Runs the native host unit-test binary (tests/native/test_host.cpp)."""
import os
import subprocess


def test_native_host_unit_tests_under_asan_ubsan(mcg):
    """Host code (CPU reference CG, partitioner, halo plan, generators) under ASan + UBSan."""
    root = mcg.repo_root()
    subprocess.run(["make", "-C", root, "asan"], check=True, capture_output=True, timeout=600)
    p = subprocess.run([os.path.join(root, "build", "test_host_asan")], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr
    assert "all passed" in p.stdout and "ERROR" not in p.stderr


def test_native_host_unit_tests(mcg):
    exe = os.path.join(mcg.repo_root(), "build", "test_host")
    p = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    assert "all passed" in p.stdout
