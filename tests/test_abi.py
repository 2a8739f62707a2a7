"""The C-ABI library loads and exports every symbol include/lmm/*.h declares (CPU only)."""
import ctypes as ct
import os
import re

import pytest

from simgrid_amd import lmm as L

INCLUDE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "lmm")


def declared_functions():
    names = set()
    for h in ("lmm_hip.h", "lmm_system.h"):
        text = open(os.path.join(INCLUDE, h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"\b(lmm\w*)\s*\(", text):
            names.add(m.group(1))
    return sorted(names)


def test_headers_declare_something():
    names = declared_functions()
    assert "lmmhip_solve" in names and "lmm_solve" in names and len(names) > 50


@pytest.mark.parametrize("name", declared_functions())
def test_symbol_exported(name):
    lib = ct.CDLL(L.LIB_PATH)
    assert hasattr(lib, name), name


def test_python_binding_covers_every_symbol():
    assert set(declared_functions()) <= set(L.SIGNATURES)


def test_solve_without_gpu_fails_loudly():
    if L.device_count() > 0:
        pytest.skip("a GPU is visible")
    s = L.System(False)
    c = s.constraint_new(None, 1.0)
    v = s.variable_new(None, 1.0)
    s.expand(c, v, 1.0)
    with pytest.raises(L.LmmError, match="no HIP device"):
        s.solve()


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
C_DRIVE = os.path.join(ROOT, "tests", "c", "abi_drive")


def build_c_drive():
    """Compile tests/c/abi_drive.c (plain C, gcc) against include/lmm/*.h and link liblmm_amd.so."""
    import subprocess

    lib_dir = os.path.dirname(L.LIB_PATH)
    subprocess.check_call(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-O1", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "c", "abi_drive.c"), "-o", C_DRIVE, "-L", lib_dir, "-llmm_amd",
                           "-Wl,-rpath," + lib_dir, "-lm"])
    return C_DRIVE


def test_c_client_compiles_against_the_headers():
    """The boundary is a C ABI: a C99 program includes both headers and links the library."""
    assert os.path.exists(build_c_drive())


def test_build_id_matches_source_tree():
    """Build provenance: the loaded library's lmmhip_build_id() is the hash of this tree's sources
    (simgrid_amd/build_id.py), so a stale or foreign liblmm_amd.so is caught."""
    from simgrid_amd import build_id as B

    if os.environ.get("LMM_AMD_LIB"):
        pytest.skip("an A/B build was loaded on purpose")
    assert L.build_id() == B.tree_id()
