"""Runs the native host unit-test binary (tests/native/test_host.cpp)."""
import os
import subprocess


def test_native_host_unit_tests(mcg):
    exe = os.path.join(mcg.repo_root(), "build", "test_host")
    p = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    assert "all passed" in p.stdout
