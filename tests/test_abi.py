"""CPU: the C-ABI library builds, loads, and exports exactly what include/orbg.h declares.

No compute call is made here (no GPU in the build container); orbg_create must fail
loudly with ORBG_EIO rather than fall back to anything on the CPU.
"""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "orbg.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(orbg_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def liborbg():
    from orb_slam2_test_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "orb_slam2_test_amd", "csrc")])
    return _lib


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("orbg_create", "orbg_extract", "orbg_get_level", "orbg_hamming_knn2",
                 "orbg_search_for_initialization", "orbg_ba_linearize",
                 "orbg_extract_batch_device", "orbg_match_batch_device", "orbg_destroy"):
        assert must in names


def test_library_exports_every_declared_symbol(liborbg):
    lib = liborbg.lib()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_library_is_gfx950_hip_and_oracle_free(liborbg):
    out = subprocess.run(["nm", "-D", "--defined-only", liborbg.LIB_PATH], capture_output=True,
                         text=True).stdout
    assert "orc_" not in out, "product library must not contain oracle code"
    blob = open(liborbg.LIB_PATH, "rb").read()
    assert b"gfx950" in blob, "device code object for gfx950 missing"
    assert b"__hip_fatbin" in blob or b"HIP_CLANG" in blob or b".hip_fatbin" in blob


def test_params_default_and_pattern(liborbg, ref_tables):
    p = liborbg.default_params()
    assert (p.nfeatures, round(p.scale_factor, 6), p.nlevels, p.ini_th_fast, p.min_th_fast) == (
        2000, 1.2, 8, 20, 7)
    assert list(p.gauss_k) == [18, 34, 48, 56, 48, 34, 18]
    pat = np.zeros(1024, np.int32)
    assert liborbg.lib().orbg_get_pattern(liborbg.ptr(pat)) == 0
    assert pat.tolist() == ref_tables["bit_pattern_31"]
    assert liborbg.lib().orbg_abi_version() == 1


def test_descriptor_distance_host_entry(liborbg):
    rng = np.random.default_rng(5)
    a = rng.integers(0, 256, 32, dtype=np.uint8)
    b = rng.integers(0, 256, 32, dtype=np.uint8)
    assert liborbg.lib().orbg_descriptor_distance(liborbg.ptr(a), liborbg.ptr(b)) == int(
        np.unpackbits(a ^ b).sum())


def test_no_cpu_fallback_without_gpu(liborbg):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    h = C.c_void_p()
    rc = liborbg.lib().orbg_create(0, None, C.byref(h))
    assert rc == liborbg.ORBG_EIO
    assert "no HIP device" in liborbg.last_error()
    from orb_slam2_test_amd import ORBextractor
    with pytest.raises(RuntimeError):
        ORBextractor(1000, 1.2, 8, 20, 7)


def test_invalid_arguments_rejected(liborbg):
    L = liborbg.lib()
    assert L.orbg_create(0, None, None) == liborbg.ORBG_EINVAL
    assert L.orbg_extract(None, None, 0, 0, 0, None, None, 0, None) == liborbg.ORBG_EINVAL
    assert L.orbg_sync(None) == liborbg.ORBG_EINVAL


def test_cpp_compat_header_compiles():
    """The C++ drop-in classes (compat/) compile against the C ABI with g++, and without a
    GPU the Extractor constructor throws (ORBG_EIO): no CPU fallback behind them either."""
    comp = os.path.join(ROOT, "orb_slam2_test_amd", "compat")
    src = os.path.join(comp, "compat_selftest.cpp")
    subprocess.check_call(["g++", "-std=c++17", "-Wall", "-Werror", "-fsyntax-only", "-I",
                           os.path.join(ROOT, "include"), "-I", comp, src])
    exe = os.path.join(ROOT, "orb_slam2_test_amd", "lib", "compat_selftest")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "orb_slam2_test_amd", "csrc")])
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible (tests/test_gpu_compat.py runs the selftest)")
    r = subprocess.run([exe, "nogpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "no HIP device" in r.stdout
