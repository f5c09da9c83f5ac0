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


def test_cmake_build_configures_and_builds_host_tests(mcg, tmp_path):
    """The CMake build (alternative to the Makefile) configures and builds the host unit tests."""
    root = mcg.repo_root()
    b = str(tmp_path / "b")
    subprocess.run(["cmake", "-S", root, "-B", b, "-G", "Ninja"], check=True, capture_output=True, timeout=300)
    subprocess.run(["cmake", "--build", b, "--target", "test_host", "-j4"], check=True, capture_output=True,
                   timeout=600)
    p = subprocess.run([os.path.join(b, "test_host")], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and "all passed" in p.stdout
