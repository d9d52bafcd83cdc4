"""Python binding of libeslam_gpu.so (the MI355X eSLAM core) through its C ABI.

This is the host-side mirror of the reference's API for tests and benchmarks:
``EmbodiedSlamFilter`` (src/EmbodiedSlamFilter.hpp:58-74) and the ``PoseEstimator`` /
``ParticleFilter<T>`` calls it forwards (src/PoseEstimator.hpp:123-134,
src/ParticleFilter.hpp:34-173).  Every call goes to the GPU; there is no CPU fallback --
a missing library or GPU raises.
"""
import ctypes as C
import os

import numpy as np

import eslam_abi as A

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ESLAM_GPU_LIB", os.path.join(HERE, "lib", "libeslam_gpu.so"))

_lib = None


class EslamError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(msg)
        self.code = code


def build_id():
    """SHA-256 of the sources the loaded library was built from (eslam_gpu_build_id)."""
    return load_library().eslam_gpu_build_id().decode()


def load_library(path=LIB_PATH):
    """Load libeslam_gpu.so and declare every entry point of include/eslam_gpu.h."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"libeslam_gpu.so not built ({path}); run __graft_entry__.build()")
    L = C.CDLL(path)
    L.eslam_gpu_build_id.restype = C.c_char_p
    if "ESLAM_GPU_LIB" not in os.environ:
        # the in-tree library must be the build of these sources (build_lib.source_hash)
        import build_lib
        want, got = build_lib.source_hash(), L.eslam_gpu_build_id().decode()
        if got != want:
            raise RuntimeError(f"{path} was built from other sources (build id {got[:12]}, sources {want[:12]}); "
                               "run __graft_entry__.build()")
    vp = C.c_void_p
    dp = C.POINTER(C.c_double)
    L.eslam_config_default.argtypes = [C.POINTER(A.Config)]
    L.eslam_config_default.restype = None
    L.eslam_gpu_abi_version.restype = C.c_int
    L.eslam_gpu_create.argtypes = [C.POINTER(A.Config), C.c_int, C.POINTER(vp)]
    L.eslam_gpu_destroy.argtypes = [vp]
    L.eslam_gpu_destroy.restype = None
    L.eslam_gpu_finish.argtypes = [vp]
    L.eslam_gpu_last_error.argtypes = [vp]
    L.eslam_gpu_last_error.restype = C.c_char_p
    L.eslam_gpu_set_stream.argtypes = [vp, vp]
    L.eslam_gpu_set_map.argtypes = [vp, C.POINTER(A.MlsGrid)]
    L.eslam_gpu_init_gaussian.argtypes = [vp, C.c_uint64, dp, dp, C.c_double, C.c_double]
    L.eslam_gpu_init_pose.argtypes = [vp, dp, dp]
    L.eslam_gpu_upload_particles.argtypes = [vp, C.c_uint64, C.POINTER(A.Particles)]
    L.eslam_gpu_download_particles.argtypes = [vp, C.POINTER(A.Particles)]
    L.eslam_gpu_write_particles.argtypes = [vp, C.c_uint64, C.c_uint64, C.POINTER(A.Particles)]
    L.eslam_gpu_map_update.argtypes = [vp, C.POINTER(A.ScanPatch), C.c_uint32]
    if hasattr(L, "eslam_gpu_map_match"):                 # absent from older builds (A/B runs)
        L.eslam_gpu_map_match.argtypes = [vp, C.POINTER(A.ScanPatch), C.c_uint32]
    L.eslam_gpu_set_particle_maps.argtypes = [vp, C.c_int]
    L.eslam_gpu_get_particle_map.argtypes = [vp, C.c_uint64, C.POINTER(C.c_uint32), C.POINTER(C.c_float),
                                             C.POINTER(C.c_float), C.c_uint32, C.POINTER(C.c_uint32)]
    L.eslam_gpu_download_records.argtypes = [vp, C.c_uint64, C.c_uint64, C.c_uint64, C.POINTER(A.ParticleRecord),
                                             C.POINTER(A.CPoint), C.c_uint32]
    L.eslam_gpu_particle_count.argtypes = [vp, C.POINTER(C.c_uint64)]
    L.eslam_gpu_step.argtypes = [vp, C.POINTER(A.StepInput), C.POINTER(C.c_int)]
    L.eslam_gpu_project.argtypes = [vp, C.POINTER(A.StepInput)]
    L.eslam_gpu_update.argtypes = [vp, C.POINTER(A.StepInput)]
    L.eslam_gpu_sync.argtypes = [vp, C.POINTER(A.UpdateInfo)]
    if hasattr(L, "eslam_gpu_debug_set_spin_limit"):     # absent from older builds (A/B runs)
        L.eslam_gpu_debug_set_spin_limit.argtypes = [vp, C.c_uint32]
    L.eslam_gpu_get_weights_sum.argtypes = [vp, dp]
    L.eslam_gpu_normalize_weights.argtypes = [vp, dp]
    L.eslam_gpu_resample.argtypes = [vp]
    L.eslam_gpu_get_best_particle_index.argtypes = [vp, C.POINTER(C.c_uint64)]
    L.eslam_gpu_get_centroid.argtypes = [vp, dp, dp]
    L.eslam_gpu_get_rng_state.argtypes = [vp, C.POINTER(A.RngState)]
    L.eslam_gpu_set_rng_state.argtypes = [vp, C.POINTER(A.RngState)]
    L.eslam_gpu_get_ancestors.argtypes = [vp, C.POINTER(C.c_uint32), C.c_uint64]
    L.eslam_gpu_enable_timing.argtypes = [vp, C.c_int]
    L.eslam_gpu_get_kernel_times.argtypes = [vp, C.POINTER(A.KernelTimes)]
    L.eslam_gpu_selftest_math.argtypes = [C.c_int, C.c_int, dp, dp, dp, C.c_uint64]
    up = C.POINTER(C.c_uint32)
    L.eslam_gpu_selftest_sort.argtypes = [C.c_int, up, up, C.c_uint64, up, up]
    if hasattr(L, "eslam_gpu_selftest_bm_radius"):       # absent from older builds (A/B runs)
        L.eslam_gpu_selftest_bm_radius.argtypes = [C.c_int, C.POINTER(C.c_uint64)]
    L.eslam_gpu_set_comm.argtypes = [vp, C.POINTER(A.Comm), C.c_uint64, C.POINTER(C.c_uint64)]
    L.eslam_gpu_rccl_unique_id.argtypes = [C.POINTER(C.c_uint8)]
    L.eslam_gpu_set_comm_rccl.argtypes = [vp, C.c_int32, C.c_int32, C.POINTER(C.c_uint8), C.c_uint64,
                                          C.POINTER(C.c_uint64)]
    L.eslam_gpu_hash_create.argtypes = [vp]
    L.eslam_gpu_init_hash.argtypes = [vp, C.c_uint64]
    L.eslam_gpu_hash_info.argtypes = [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)]
    L.eslam_gpu_hash_poses.argtypes = [vp, dp, dp, dp, dp, C.POINTER(C.c_int32)]
    _lib = L
    return L


def _dv(v):
    return (C.c_double * len(v))(*v)


class GpuFilter:
    """One eslam_ctx: the PoseEstimator / EmbodiedSlamFilter of one GPU."""

    def __init__(self, cfg=None, device=0):
        self.L = load_library()
        self.cfg = cfg if cfg is not None else A.default_config()
        h = C.c_void_p()
        rc = self.L.eslam_gpu_create(C.byref(self.cfg), device, C.byref(h))
        if rc != 0:
            raise EslamError(rc, f"eslam_gpu_create failed ({rc}) -- is an MI355X visible?")
        self.h = h
        self._grid = None

    def close(self):
        if getattr(self, "h", None):
            self.L.eslam_gpu_destroy(self.h)
            self.h = None

    def finish(self):
        """eslam_gpu_finish: collective on a sharded filter (completes an exchange still owed)."""
        if getattr(self, "h", None):
            self._check(self.L.eslam_gpu_finish(self.h))

    def __del__(self):
        self.close()

    def _check(self, rc):
        if rc != 0:
            raise EslamError(rc, self.L.eslam_gpu_last_error(self.h).decode())
        return rc

    # -- environment / init -------------------------------------------------------------
    def set_map(self, grid):
        self._grid = grid
        g = grid.view()
        self._check(self.L.eslam_gpu_set_map(self.h, C.byref(g)))

    def init_gaussian(self, n, mu, sigma, zpos, zsigma):
        self._check(self.L.eslam_gpu_init_gaussian(self.h, n, _dv(mu), _dv(sigma), zpos, zsigma))

    def init_pose(self, position, orientation):
        self._check(self.L.eslam_gpu_init_pose(self.h, _dv(position), _dv(orientation)))

    def upload(self, pa):
        v = pa.view()
        self._check(self.L.eslam_gpu_upload_particles(self.h, pa.n, C.byref(v)))

    def download(self):
        n = self.count()
        pa = A.ParticleArrays(n)
        v = pa.view()
        self._check(self.L.eslam_gpu_download_particles(self.h, C.byref(v)))
        return pa

    def write(self, first, pa):
        """eslam_gpu_write_particles: particles [first, first + pa.n) take pa's fields (a
        collective on a sharded filter: every rank calls it, pa.n may be 0)"""
        v = pa.view()
        self._check(self.L.eslam_gpu_write_particles(self.h, first, pa.n, C.byref(v)))

    def download_records(self, first=0, stride=1, count=None, max_cpoints=0):
        """eslam_gpu_download_records: particles first + k * stride as PoseParticle records
        (numpy structured array) and, with max_cpoints, their contact points
        (count x max_cpoints eslam_cpoint, numpy structured)."""
        n = self.count()
        if count is None:
            count = 0 if first >= n else (n - 1 - first) // max(stride, 1) + 1
        recs = (A.ParticleRecord * max(count, 1))()
        cps = (A.CPoint * max(count * max_cpoints, 1))() if max_cpoints else None
        self._check(self.L.eslam_gpu_download_records(self.h, first, stride, count, recs, cps, max_cpoints))
        r = np.ctypeslib.as_array(recs)[:count].copy()
        c = np.ctypeslib.as_array(cps)[:count * max_cpoints].reshape(count, max_cpoints).copy() if max_cpoints else None
        return r, c

    def set_particle_maps(self, on=True):
        """PoseEstimator::setEnvironment(..., useShared=not on) before init: per-particle maps"""
        self._check(self.L.eslam_gpu_set_particle_maps(self.h, 1 if on else 0))

    def map_update(self, patches):
        """eslam_gpu_map_update: processMap's merge of a scan into every particle's map"""
        self._check(self.L.eslam_gpu_map_update(self.h, patches, len(patches)))

    def map_match(self, patches):
        """eslam_gpu_map_match: processMap's visual weighting (match = true) against each
        particle's map: the shared grid, or its own map (per-particle maps)"""
        self._check(self.L.eslam_gpu_map_match(self.h, patches, len(patches)))

    def particle_map(self, i, cap=1024):
        """particle i's own patches: (cells, mean, stdev), tiles in slot order, cells row by row"""
        while True:
            cells = np.zeros(cap, np.uint32)
            mean = np.zeros(cap, np.float32)
            sd = np.zeros(cap, np.float32)
            c = C.c_uint32()
            self._check(self.L.eslam_gpu_get_particle_map(self.h, i, cells.ctypes.data_as(C.POINTER(C.c_uint32)),
                                                          mean.ctypes.data_as(C.POINTER(C.c_float)),
                                                          sd.ctypes.data_as(C.POINTER(C.c_float)), cap, C.byref(c)))
            if c.value <= cap:
                return cells[:c.value], mean[:c.value], sd[:c.value]
            cap = c.value

    def count(self):
        n = C.c_uint64()
        self._check(self.L.eslam_gpu_particle_count(self.h, C.byref(n)))
        return n.value

    # -- SurfaceHash ----------------------------------------------------------------------
    def hash_create(self):
        self._check(self.L.eslam_gpu_hash_create(self.h))

    def init_hash(self, n):
        self._check(self.L.eslam_gpu_init_hash(self.h, n))

    def hash_info(self):
        n = C.c_uint64()
        bins = self.cfg.hash_slope_bins
        sizes = np.zeros(bins * bins, dtype=np.uint32)
        self._check(self.L.eslam_gpu_hash_info(self.h, C.byref(n), sizes.ctypes.data_as(C.POINTER(C.c_uint32))))
        return n.value, sizes

    def hash_poses(self):
        n, _ = self.hash_info()
        out = [np.zeros(n) for _ in range(4)]
        bucket = np.zeros(n, dtype=np.int32)
        ptr = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))
        self._check(self.L.eslam_gpu_hash_poses(self.h, *[ptr(a) for a in out], bucket.ctypes.data_as(C.POINTER(C.c_int32))))
        return out + [bucket]

    # -- hot path -------------------------------------------------------------------------
    def step(self, st):
        u = C.c_int(0)
        self._check(self.L.eslam_gpu_step(self.h, C.byref(st), C.byref(u)))
        return bool(u.value)

    def project(self, st):
        self._check(self.L.eslam_gpu_project(self.h, C.byref(st)))

    def update(self, st):
        self._check(self.L.eslam_gpu_update(self.h, C.byref(st)))

    def sync(self):
        info = A.UpdateInfo()
        self._check(self.L.eslam_gpu_sync(self.h, C.byref(info)))
        return info

    def debug_set_spin_limit(self, polls):
        """Testing only: polls of K3's cross-block waits before they give up (0: at once)."""
        self._check(self.L.eslam_gpu_debug_set_spin_limit(self.h, polls))

    # -- ParticleFilter API ----------------------------------------------------------------
    def weights_sum(self):
        s = C.c_double()
        self._check(self.L.eslam_gpu_get_weights_sum(self.h, C.byref(s)))
        return s.value

    def normalize(self):
        e = C.c_double()
        self._check(self.L.eslam_gpu_normalize_weights(self.h, C.byref(e)))
        return e.value

    def resample(self):
        self._check(self.L.eslam_gpu_resample(self.h))

    def best_index(self):
        i = C.c_uint64()
        self._check(self.L.eslam_gpu_get_best_particle_index(self.h, C.byref(i)))
        return i.value

    def centroid(self):
        p = (C.c_double * 3)()
        q = (C.c_double * 4)()
        self._check(self.L.eslam_gpu_get_centroid(self.h, p, q))
        return list(p), list(q)

    def ancestors(self):
        n = self.count()
        out = np.zeros(n, dtype=np.uint32)
        self._check(self.L.eslam_gpu_get_ancestors(self.h, out.ctypes.data_as(C.POINTER(C.c_uint32)), n))
        return out

    def rng_state(self):
        s = A.RngState()
        self._check(self.L.eslam_gpu_get_rng_state(self.h, C.byref(s)))
        return s

    def set_rng_state(self, s):
        self._check(self.L.eslam_gpu_set_rng_state(self.h, C.byref(s)))

    def enable_timing(self, on=True):
        self._check(self.L.eslam_gpu_enable_timing(self.h, 1 if on else 0))

    def kernel_times(self):
        t = A.KernelTimes()
        self._check(self.L.eslam_gpu_get_kernel_times(self.h, C.byref(t)))
        return {f: getattr(t, f) for f, _ in t._fields_}


def selftest_math(fn, x, y=None, device=0):
    L = load_library()
    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.zeros_like(x)
    yp = None
    if y is not None:
        y = np.ascontiguousarray(y, dtype=np.float64)
        yp = y.ctypes.data_as(C.POINTER(C.c_double))
    rc = L.eslam_gpu_selftest_math(device, fn, x.ctypes.data_as(C.POINTER(C.c_double)), yp,
                                   out.ctypes.data_as(C.POINTER(C.c_double)), x.shape[0])
    if rc != 0:
        raise EslamError(rc, "selftest_math failed")
    return out
