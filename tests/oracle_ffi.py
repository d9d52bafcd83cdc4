"""ctypes binding of the CPU oracle (oracle/_build/liboracle.so) -- test infrastructure."""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-eslam_amd"))
import eslam_abi as A  # noqa: E402

LIB_PATH = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
# the same oracle with 288-byte particle records (-DOR_AOS, oracle/Makefile)
LIB_PATH_AOS = os.path.join(ROOT, "oracle", "_build", "liboracle_aos.so")

SUM_CONTRACT = 0
SUM_REFERENCE = 1


class CPoint(C.Structure):
    _fields_ = [("point", C.c_double * 3), ("zdiff", C.c_double), ("zvar", C.c_double), ("prob", C.c_double)]


class ContactModelS(C.Structure):
    _fields_ = [
        ("use_slip_update", C.c_int32), ("use_shape_update", C.c_int32),
        ("min_contacts", C.c_uint64), ("correction", C.c_double), ("radius", C.c_double),
        ("m", C.c_uint32),
        ("pos", (C.c_double * 3) * A.MAX_CONTACTS),
        ("contact", C.c_float * A.MAX_CONTACTS),
        ("group", C.c_int32 * A.MAX_CONTACTS),
        ("ncp", C.c_uint32),
        ("cp", CPoint * A.MAX_CONTACTS),
        ("zdelta", C.c_double), ("zvar", C.c_double), ("weight", C.c_double), ("posevar", C.c_double),
        ("shape_s2", C.c_double),
        ("nlow", C.c_uint32),
        ("low", (C.c_double * 3) * A.MAX_CONTACTS),
        ("literal", C.c_int32), ("pad_literal", C.c_int32),
    ]


MAPFN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.c_double, C.c_double,
                    C.POINTER(C.c_double), C.POINTER(C.c_double))


def build():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)


_libs = {}


def lib(aos=False):
    """The oracle library: SoA state (default) or 288-byte AoS records (aos=True)."""
    if aos in _libs:
        return _libs[aos]
    path = LIB_PATH_AOS if aos else LIB_PATH
    if not os.path.exists(path):
        build()
    L = C.CDLL(path)
    vp = C.c_void_p
    L.or_create.restype = vp
    L.or_create.argtypes = [C.POINTER(A.Config), C.c_int]
    L.or_destroy.argtypes = [vp]
    L.or_set_threads.argtypes = [vp, C.c_int]
    L.or_set_literal.argtypes = [vp, C.c_int]
    L.or_set_debug.argtypes = [vp, C.c_int]
    L.or_set_map.argtypes = [vp, C.POINTER(A.MlsGrid)]
    L.or_init_gaussian.argtypes = [vp, C.c_uint64, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_double, C.c_double]
    L.or_init_pose.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.or_upload.argtypes = [vp, C.c_uint64, C.POINTER(A.Particles)]
    L.or_download.argtypes = [vp, C.POINTER(A.Particles)]
    L.or_count.restype = C.c_uint64
    L.or_count.argtypes = [vp]
    for fn in ("or_project", "or_update"):
        getattr(L, fn).argtypes = [vp, C.POINTER(A.StepInput)]
    L.or_step.argtypes = [vp, C.POINTER(A.StepInput), C.POINTER(C.c_int)]
    L.or_last_info.argtypes = [vp, C.POINTER(A.UpdateInfo)]
    L.or_get_weights_sum.restype = C.c_double
    L.or_get_weights_sum.argtypes = [vp]
    L.or_normalize_weights.restype = C.c_double
    L.or_normalize_weights.argtypes = [vp]
    L.or_resample.argtypes = [vp]
    L.or_resample_multinomial.argtypes = [vp, C.c_uint64]
    L.or_best_index.restype = C.c_uint64
    L.or_best_index.argtypes = [vp]
    L.or_get_centroid.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.or_get_ancestors.argtypes = [vp, C.POINTER(C.c_uint32), C.c_uint64]
    L.or_get_rng_state.argtypes = [vp, C.POINTER(A.RngState)]
    L.or_set_rng_state.argtypes = [vp, C.POINTER(A.RngState)]
    L.or_map_update.argtypes = [vp, C.POINTER(A.ScanPatch), C.c_uint32]
    L.or_map_match.argtypes = [vp, C.POINTER(A.ScanPatch), C.c_uint32]
    L.or_get_particle_map.restype = C.c_uint32
    L.or_pages_in_use.restype = C.c_uint64
    L.or_pages_in_use.argtypes = [vp]
    L.or_get_particle_map.argtypes = [vp, C.c_uint64, C.POINTER(C.c_uint32), C.POINTER(C.c_float), C.POINTER(C.c_float),
                                      C.c_uint32]
    L.or_get_debug.argtypes = [vp, C.POINTER(C.c_uint32), C.POINTER(CPoint), C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.or_cm_init.argtypes = [C.POINTER(ContactModelS), C.POINTER(A.Config)]
    L.or_cm_set_contact_points.argtypes = [C.POINTER(ContactModelS), C.c_uint32, C.POINTER(A.ContactPoint), C.POINTER(C.c_double)]
    L.or_cm_evaluate_pose.argtypes = [C.POINTER(ContactModelS), C.POINTER(C.c_double), C.c_double, MAPFN, C.c_void_p]
    L.or_cm_update_z.argtypes = [C.POINTER(ContactModelS), C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.or_cm_lowest_points.restype = C.c_uint32
    L.or_cm_lowest_points.argtypes = [C.POINTER(ContactModelS), C.POINTER(C.c_double)]
    L.or_cm_update_contact_state_lph.argtypes = [C.POINTER(ContactModelS)]
    L.or_surface_param_from_points.argtypes = [C.POINTER(C.c_double), C.c_uint32, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.or_bucket_index.restype = C.c_int
    L.or_bucket_index.argtypes = [C.c_int, C.c_double, C.c_double, C.c_double]
    L.or_mls_get_patch.argtypes = [C.POINTER(A.MlsGrid), C.POINTER(C.c_double), C.c_double, C.c_double,
                                   C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.or_set_comm.argtypes = [vp, C.POINTER(A.Comm), C.c_uint64, C.POINTER(C.c_uint64)]
    L.or_hash_create.argtypes = [vp]
    L.or_init_hash.argtypes = [vp, C.c_uint64]
    L.or_hash_info.restype = C.c_uint64
    L.or_hash_info.argtypes = [vp, C.POINTER(C.c_uint32)]
    L.or_hash_poses.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_double),
                                C.POINTER(C.c_double), C.POINTER(C.c_int32)]
    L.or_dm.restype = C.c_double
    L.or_dm.argtypes = [C.c_int, C.c_double, C.c_double]
    L.or_dm_philox.argtypes = [C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint32, C.POINTER(C.c_uint32)]
    L.or_dm_philox_raw.argtypes = [C.POINTER(C.c_uint32), C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32)]
    L.or_dm_libc_rand.argtypes = [C.c_uint32, C.c_uint32, C.POINTER(C.c_int32)]
    L.or_dm_minstd_jump.restype = C.c_uint32
    L.or_dm_minstd_jump.argtypes = [C.c_uint32, C.c_uint64]
    L.or_dm_limbs_to_double.restype = C.c_double
    L.or_dm_limbs_to_double.argtypes = [C.POINTER(C.c_uint64), C.c_int]
    L.or_dm_fx128.argtypes = [C.c_double, C.c_int, C.POINTER(C.c_uint32)]
    _libs[aos] = L
    return L


def dvec(v):
    return (C.c_double * len(v))(*v)


class OracleFilter:
    """The oracle PoseEstimator / EmbodiedSlamFilter."""

    def __init__(self, cfg, sum_mode=SUM_CONTRACT, aos=False):
        self.L = lib(aos)
        self.cfg = cfg
        self.h = self.L.or_create(C.byref(cfg), sum_mode)
        self._map = None

    def __del__(self):
        if getattr(self, "h", None):
            self.L.or_destroy(self.h)
            self.h = None

    def set_threads(self, threads):
        """OpenMP threads of the per-particle loops (results identical for any count)."""
        self.L.or_set_threads(self.h, int(threads))

    def set_literal(self, on=True):
        """the reference's literal arithmetic instead of the build's contract (or_set_literal)"""
        self.L.or_set_literal(self.h, int(bool(on)))

    def set_debug(self, on=True):
        """capture the per-particle contact-model outputs of every update (or_get_debug)"""
        self.L.or_set_debug(self.h, int(bool(on)))

    def set_comm(self, comm, n_global):
        """Sharded mode over a host-memory eslam_comm (slam-eslam_amd/eslam_dist.TorchComm)."""
        self._comm = comm
        self.bounds = A.shard_bounds(n_global, comm.nranks, self.cfg.sum_chunk_rows)
        self._gb = (C.c_uint64 * len(self.bounds))(*self.bounds)
        rc = self.L.or_set_comm(self.h, C.byref(comm.struct), n_global, self._gb)
        assert rc == 0, rc

    def hash_create(self):
        assert self.L.or_hash_create(self.h) == 0

    def init_hash(self, n):
        rc = self.L.or_init_hash(self.h, n)
        assert rc == 0, rc

    def hash_info(self):
        bins = self.cfg.hash_slope_bins
        sizes = np.zeros(bins * bins, dtype=np.uint32)
        n = self.L.or_hash_info(self.h, sizes.ctypes.data_as(C.POINTER(C.c_uint32)))
        return n, sizes

    def hash_poses(self):
        n, _ = self.hash_info()
        out = [np.zeros(n) for _ in range(4)]
        bucket = np.zeros(n, dtype=np.int32)
        ptr = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))
        assert self.L.or_hash_poses(self.h, *[ptr(a) for a in out], bucket.ctypes.data_as(C.POINTER(C.c_int32))) == 0
        return out + [bucket]

    def set_map(self, grid):
        self._map = grid
        g = grid.view()
        assert self.L.or_set_map(self.h, C.byref(g)) == 0

    def init_gaussian(self, n, mu, sigma, z, zs):
        assert self.L.or_init_gaussian(self.h, n, dvec(mu), dvec(sigma), z, zs) == 0

    def init_pose(self, pos, q):
        assert self.L.or_init_pose(self.h, dvec(pos), dvec(q)) == 0

    def upload(self, pa):
        v = pa.view()
        assert self.L.or_upload(self.h, pa.n, C.byref(v)) == 0

    def download(self):
        n = self.L.or_count(self.h)
        pa = A.ParticleArrays(n)
        v = pa.view()
        assert self.L.or_download(self.h, C.byref(v)) == 0
        return pa

    def count(self):
        return self.L.or_count(self.h)

    def project(self, st):
        return self.L.or_project(self.h, C.byref(st))

    def update(self, st):
        return self.L.or_update(self.h, C.byref(st))

    def step(self, st):
        u = C.c_int(0)
        rc = self.L.or_step(self.h, C.byref(st), C.byref(u))
        assert rc == 0, rc
        return bool(u.value)

    def info(self):
        i = A.UpdateInfo()
        self.L.or_last_info(self.h, C.byref(i))
        return i

    def weights_sum(self):
        return self.L.or_get_weights_sum(self.h)

    def normalize(self):
        return self.L.or_normalize_weights(self.h)

    def resample(self):
        self.L.or_resample(self.h)

    def best_index(self):
        return self.L.or_best_index(self.h)

    def centroid(self):
        p = (C.c_double * 3)()
        q = (C.c_double * 4)()
        self.L.or_get_centroid(self.h, p, q)
        return list(p), list(q)

    def ancestors(self):
        n = self.count()
        out = np.zeros(n, dtype=np.uint32)
        rc = self.L.or_get_ancestors(self.h, out.ctypes.data_as(C.POINTER(C.c_uint32)), n)
        return out if rc == 0 else None

    def rng_state(self):
        s = A.RngState()
        self.L.or_get_rng_state(self.h, C.byref(s))
        return s

    def set_rng_state(self, s):
        self.L.or_set_rng_state(self.h, C.byref(s))

    def map_update(self, patches):
        assert self.L.or_map_update(self.h, patches, len(patches)) == 0

    def map_match(self, patches):
        assert self.L.or_map_match(self.h, patches, len(patches)) == 0

    def particle_map(self, i, cap=1024):
        while True:
            cells = np.zeros(cap, np.uint32)
            mean = np.zeros(cap, np.float32)
            sd = np.zeros(cap, np.float32)
            c = self.L.or_get_particle_map(self.h, i, cells.ctypes.data_as(C.POINTER(C.c_uint32)),
                                           mean.ctypes.data_as(C.POINTER(C.c_float)),
                                           sd.ctypes.data_as(C.POINTER(C.c_float)), cap)
            if c <= cap:
                return cells[:c], mean[:c], sd[:c]
            cap = c

    def pages_in_use(self):
        return int(self.L.or_pages_in_use(self.h))

    def debug(self):
        n = self.count()
        ncp = np.zeros(n, dtype=np.uint32)
        cp = (CPoint * (n * A.MAX_CONTACTS))()
        zd = np.zeros(n)
        zv = np.zeros(n)
        rc = self.L.or_get_debug(self.h, ncp.ctypes.data_as(C.POINTER(C.c_uint32)), cp,
                                 zd.ctypes.data_as(C.POINTER(C.c_double)), zv.ctypes.data_as(C.POINTER(C.c_double)))
        assert rc == 0, "debug capture is off (set_debug)"
        return ncp, cp, zd, zv


def dm(fn, x, y=0.0):
    return lib().or_dm(fn, x, y)
