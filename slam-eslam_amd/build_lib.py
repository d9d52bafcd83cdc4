"""Build libeslam_gpu.so (gfx950) in-tree with hipcc -- no cmake, no JIT cache.

    python slam-eslam_amd/build_lib.py            # rebuild unless the library's build id matches
    python slam-eslam_amd/build_lib.py --force

The library is the product: HIP kernels + the C ABI of include/eslam_gpu.h.
-ffp-contract=off keeps device and host arithmetic bit-identical to the CPU oracle.
Machine-LICM is disabled for the kernels' translation unit only: it hoists the ~150 fp64
polynomial constants of the contact model out of the particle loop and drives
k_project_weight to 256 VGPRs / occupancy 1.

Provenance: the SHA-256 of every source, header and flag is compiled into the library
(eslam_gpu_build_id()).  A build is skipped only when the existing library reports the hash
of the current sources, so a run never loads a binary that was not built from them
(tests/test_abi.py checks the shipped library the same way).
"""
import ctypes
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT_DIR = os.path.join(HERE, "lib")
LIB = os.path.join(OUT_DIR, "libeslam_gpu.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("ESLAM_OFFLOAD_ARCH", "gfx950")

SOURCES = ["eslam_kernels.hip", "eslam_hash.hip", "eslam_ctx.hip"]
HEADERS = [os.path.join(CSRC, "eslam_internal.h"), os.path.join(ROOT, "include", "eslam_gpu.h"),
           os.path.join(ROOT, "include", "eslam_detmath.h")]
FLAGS = ["-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
         "-mfma", "-Wall", "-Wno-unused-result", "-Wno-unused-function", f"-I{os.path.join(ROOT, 'include')}"]
PER_SOURCE = {"eslam_kernels.hip": ["-mllvm", "-disable-machine-licm"]}


def source_hash(defines=(), extra=()):
    """SHA-256 over the build inputs: every source and header, the flags, the defines."""
    h = hashlib.sha256()
    for path in [os.path.join(CSRC, s) for s in SOURCES] + HEADERS:
        h.update(os.path.basename(path).encode())
        with open(path, "rb") as fh:
            h.update(fh.read())
    flags = [f.replace(ROOT, "<root>") for f in FLAGS]      # location-independent (the GPU box's copy)
    h.update(repr((flags, PER_SOURCE, list(defines), list(extra), ARCH)).encode())
    return h.hexdigest()


def library_build_id(lib=LIB):
    """The build id compiled into a built library (None if it cannot be loaded)."""
    if not os.path.exists(lib):
        return None
    try:
        L = ctypes.CDLL(lib)
        L.eslam_gpu_build_id.restype = ctypes.c_char_p
        return L.eslam_gpu_build_id().decode()
    except (OSError, AttributeError):
        return None


def build(force=False, verbose=True, defines=(), lib=None, tag=""):
    """defines: extra -D macros (ablation builds only); lib/tag: alternative output names."""
    os.makedirs(OUT_DIR, exist_ok=True)
    lib = lib or LIB
    extra = os.environ.get("ESLAM_EXTRA_FLAGS", "").split()     # experiment builds only
    bid = source_hash(defines, extra)
    if not force and library_build_id(lib) == bid:
        return lib
    objs = []
    for src in SOURCES:
        path = os.path.join(CSRC, src)
        obj = os.path.join(OUT_DIR, src + tag + ".o")
        objs.append(obj)
        cmd = [HIPCC] + FLAGS + PER_SOURCE.get(src, []) + extra + ["-D" + d for d in defines]
        if src == "eslam_ctx.hip":
            cmd.append(f'-DESLAM_BUILD_ID="{bid}"')
        cmd += ["-c", path, "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib] + objs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return lib


FACADE_SRC = os.path.join(ROOT, "tests", "cpp", "test_facade.cpp")
FACADE_BIN = os.path.join(ROOT, "tests", "cpp", "_build", "test_facade")


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_facade_test(verbose=True):
    """g++ the C++ façade test (include/eslam_gpu.hpp over the C ABI) against the library."""
    deps = [FACADE_SRC, LIB, os.path.join(ROOT, "include", "eslam_gpu.hpp"), os.path.join(ROOT, "include", "eslam_gpu.h")]
    if not _stale(FACADE_BIN, deps):
        return FACADE_BIN
    os.makedirs(os.path.dirname(FACADE_BIN), exist_ok=True)
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", f"-I{os.path.join(ROOT, 'include')}", FACADE_SRC,
           f"-L{OUT_DIR}", "-leslam_gpu", "-Wl,-rpath,$ORIGIN/../../../slam-eslam_amd/lib", "-o", FACADE_BIN]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return FACADE_BIN


if __name__ == "__main__":
    defs = [a[2:] for a in sys.argv[1:] if a.startswith("-D")]
    tag = "_" + "_".join(d.lower() for d in defs) if defs else ""
    build(force="--force" in sys.argv, defines=defs, tag=tag,
          lib=os.path.join(OUT_DIR, f"libeslam_gpu{tag}.so") if defs else None)
