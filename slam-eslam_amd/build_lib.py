"""Build libeslam_gpu.so (gfx950) in-tree with hipcc -- no cmake, no JIT cache.

    python slam-eslam_amd/build_lib.py            # incremental
    python slam-eslam_amd/build_lib.py --force

The library is the product: HIP kernels + the C ABI of include/eslam_gpu.h.
-ffp-contract=off keeps device and host arithmetic bit-identical to the CPU oracle;
Machine-LICM is disabled because it hoists the ~150 fp64 polynomial constants of the
contact model out of the particle loop and drives the kernel to 256 VGPRs / occupancy 1.
"""
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
         "-mfma", "-mllvm", "-disable-machine-licm", "-Wall", "-Wno-unused-result", "-Wno-unused-function",
         f"-I{os.path.join(ROOT, 'include')}"]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=True, defines=(), lib=None, tag=""):
    """defines: extra -D macros (ablation builds only); lib/tag: alternative output names."""
    os.makedirs(OUT_DIR, exist_ok=True)
    lib = lib or LIB
    objs = []
    for src in SOURCES:
        path = os.path.join(CSRC, src)
        obj = os.path.join(OUT_DIR, src + tag + ".o")
        objs.append(obj)
        if force or _stale(obj, [path] + HEADERS):
            extra = os.environ.get("ESLAM_EXTRA_FLAGS", "").split()     # experiment builds only
            cmd = [HIPCC] + FLAGS + extra + ["-D" + d for d in defines] + ["-c", path, "-o", obj]
            if verbose:
                print(" ".join(cmd), flush=True)
            subprocess.run(cmd, check=True)
    if force or _stale(lib, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib] + objs
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return lib


FACADE_SRC = os.path.join(ROOT, "tests", "cpp", "test_facade.cpp")
FACADE_BIN = os.path.join(ROOT, "tests", "cpp", "_build", "test_facade")


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
