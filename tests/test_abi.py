"""The C-ABI library (CPU-side checks, no GPU calls): it loads, exports every entry point
include/eslam_gpu.h declares, the ctypes mirror has the C struct layouts, and the C++
façade header compiles."""
import ctypes as C
import os
import re
import subprocess

import pytest

import eslam_abi as A

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "eslam_gpu.h")
LIB = os.path.join(ROOT, "slam-eslam_amd", "lib", "libeslam_gpu.so")


def declared_functions():
    text = open(HDR).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"^[a-z_][\w \*]*?\b(eslam_\w+)\s*\(", text, flags=re.M)
    return sorted(set(n for n in names if not n.startswith("eslam_comm")))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        import sys
        sys.path.insert(0, os.path.join(ROOT, "slam-eslam_amd"))
        import build_lib
        build_lib.build(verbose=False)
    return C.CDLL(LIB)


def test_exports_every_declared_symbol(lib):
    names = declared_functions()
    assert len(names) >= 28, names
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_library_built_from_these_sources(lib):
    """provenance: the shipped library reports the SHA-256 of the current sources and flags"""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "slam-eslam_amd"))
    import build_lib
    lib.eslam_gpu_build_id.restype = C.c_char_p
    assert lib.eslam_gpu_build_id().decode() == build_lib.source_hash()


def test_abi_version(lib):
    lib.eslam_gpu_abi_version.restype = C.c_int
    assert lib.eslam_gpu_abi_version() == 8


def test_config_default_matches_reference_defaults(lib):
    c = A.Config()
    lib.eslam_config_default(C.byref(c))
    ref = A.default_config()
    for f, _ in A.Config._fields_:
        a, b = getattr(c, f), getattr(ref, f)
        if hasattr(a, "__len__"):
            a, b = list(a), list(b)
        assert a == b, f
    # src/Configuration.hpp:85-111
    assert (c.seed, c.particle_count, c.min_effective) == (42, 250, 50)
    assert (c.measurement_error, c.discount_factor, c.spread_threshold) == (0.1, 0.9, 0.9)


STRUCTS = {"eslam_config": A.Config, "eslam_mls_grid": A.MlsGrid, "eslam_contact_point": A.ContactPoint,
           "eslam_step_input": A.StepInput, "eslam_particles": A.Particles, "eslam_update_info": A.UpdateInfo,
           "eslam_rng_state": A.RngState, "eslam_kernel_times": A.KernelTimes, "eslam_comm": A.Comm,
           "eslam_cpoint": A.CPoint, "eslam_particle_record": A.ParticleRecord, "eslam_scan_patch": A.ScanPatch}


def test_struct_layouts_match_ctypes(tmp_path):
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "eslam_gpu.h"', "int main(void){"]
    for cname, py in STRUCTS.items():
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0;}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", f"-I{os.path.join(ROOT, 'include')}", str(src), "-o", str(exe)], check=True)
    out = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                        check=True).stdout.split("\n") if l)
    for cname, py in STRUCTS.items():
        assert int(out[cname]) == C.sizeof(py), cname
        for f, _ in py._fields_:
            assert int(out[f"{cname}.{f}"]) == getattr(py, f).offset, f"{cname}.{f}"


def test_cpp_facade_compiles(tmp_path):
    src = os.path.join(ROOT, "tests", "cpp", "test_facade.cpp")
    subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Wextra", "-Werror",
                    f"-I{os.path.join(ROOT, 'include')}", src], check=True)
