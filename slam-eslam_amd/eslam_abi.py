"""ctypes mirror of include/eslam_gpu.h (the C ABI of the MI355X eSLAM core).

Shared by the product wrapper (eslam_amd.py), the tests and bench.py.  Field order and
types must match the header exactly; tests/test_abi.py checks sizes against the C compiler.
"""
import ctypes as C

MAX_CONTACTS = 32

OK = 0
ERR_INVALID_ARG = -1
ERR_NO_ENVIRONMENT = -2
ERR_ZERO_MEAS_VAR = -3
ERR_HASH_SAMPLE = -4
ERR_NO_MLS_GRID = -5
ERR_HIP = -6
ERR_NOT_INITIALISED = -7
ERR_UNSUPPORTED = -8
ERR_OUT_OF_MEMORY = -9

FLAG_RECORD_ANCESTORS = 0x1
FLAG_NO_MAP_LDS = 0x2
FLAG_NO_AUX_GATHER = 0x4
FLAG_RECORD_CONTACTS = 0x8
FLAG_PARTICLE_MAPS = 0x10
FLAG_PROCESS_STATICS = 0x20


class Config(C.Structure):
    _fields_ = [
        ("seed", C.c_uint64),
        ("particle_count", C.c_uint64),
        ("min_effective", C.c_uint64),
        ("initial_rotation_error", C.c_double * 3),
        ("initial_translation_error", C.c_double * 3),
        ("measurement_error", C.c_double),
        ("discount_factor", C.c_double),
        ("spread_threshold", C.c_double),
        ("spread_translation_factor", C.c_double),
        ("spread_rotation_factor", C.c_double),
        ("slip_factor", C.c_double),
        ("max_yaw_deviation", C.c_double),
        ("measurement_threshold_distance", C.c_double),
        ("measurement_threshold_angle", C.c_double),
        ("use_slip_update", C.c_int32),
        ("use_shape_update", C.c_int32),
        ("min_contacts", C.c_uint64),
        ("contact_likelihood_correction", C.c_double),
        ("contact_point_radius", C.c_double),
        ("hash_use", C.c_int32),
        ("hash_period", C.c_uint64),
        ("hash_percentage", C.c_double),
        ("hash_avg_factor", C.c_double),
        ("hash_slope_bins", C.c_uint64),
        ("hash_angular_steps", C.c_uint64),
        ("log_debug", C.c_int32),
        ("flags", C.c_uint32),
        ("local_map_pages", C.c_uint32),
        ("max_sensor_range", C.c_double),
        ("local_map_trail", C.c_uint32),
        ("sum_chunk_rows", C.c_uint32),
    ]


class MlsGrid(C.Structure):
    _fields_ = [
        ("width", C.c_uint32),
        ("height", C.c_uint32),
        ("scale_x", C.c_double),
        ("scale_y", C.c_double),
        ("offset_x", C.c_double),
        ("offset_y", C.c_double),
        ("global2local", C.c_double * 12),
        ("cell_start", C.POINTER(C.c_uint32)),
        ("patch_mean", C.POINTER(C.c_float)),
        ("patch_stdev", C.POINTER(C.c_float)),
        ("patch_height", C.POINTER(C.c_float)),
        ("n_patches", C.c_uint64),
    ]


class ContactPoint(C.Structure):
    _fields_ = [
        ("position", C.c_double * 3),
        ("contact", C.c_float),
        ("group_id", C.c_int32),
    ]


class StepInput(C.Structure):
    _fields_ = [
        ("body2odometry_rot", C.c_double * 4),
        ("body2odometry_trans", C.c_double * 3),
        ("pose_delta_trans", C.c_double * 3),
        ("position_error_zz", C.c_double),
        ("sample_mean", C.c_double * 3),
        ("sample_cov", C.c_double * 9),
        ("n_contacts", C.c_uint32),
        ("ltc_count", C.c_uint32),
        ("contacts", ContactPoint * MAX_CONTACTS),
    ]


class Particles(C.Structure):
    _fields_ = [
        ("x", C.POINTER(C.c_double)),
        ("y", C.POINTER(C.c_double)),
        ("orientation", C.POINTER(C.c_double)),
        ("zpos", C.POINTER(C.c_double)),
        ("zsigma", C.POINTER(C.c_double)),
        ("weight", C.POINTER(C.c_double)),
        ("mprob", C.POINTER(C.c_double)),
        ("floating", C.POINTER(C.c_uint8)),
        ("n_contact_points", C.POINTER(C.c_uint8)),
    ]


class ScanPatch(C.Structure):
    """eslam_scan_patch: one cell of the scan MLS merged by a map update"""
    _fields_ = [
        ("position", C.c_double * 3),
        ("stdev", C.c_double),
    ]


class CPoint(C.Structure):
    """eslam_cpoint: ContactPoint (src/PoseParticle.hpp:20-43)"""
    _fields_ = [
        ("point", C.c_double * 3),
        ("zdiff", C.c_double),
        ("zvar", C.c_double),
        ("prob", C.c_double),
    ]


class ParticleRecord(C.Structure):
    """eslam_particle_record: PoseParticle with its debug fields (src/PoseParticle.hpp:52-86)"""
    _fields_ = [
        ("position", C.c_double * 2),
        ("orientation", C.c_double),
        ("zpos", C.c_double),
        ("zsigma", C.c_double),
        ("mprob", C.c_double),
        ("weight", C.c_double),
        ("meas_pos", C.c_double * 3),
        ("meas_theta", C.c_double),
        ("index", C.c_uint64),
        ("n_cpoints", C.c_uint32),
        ("floating", C.c_uint8),
        ("pad", C.c_uint8 * 3),
    ]


class UpdateInfo(C.Structure):
    _fields_ = [
        ("effective", C.c_double),
        ("weight_sum", C.c_double),
        ("floating_weight", C.c_double),
        ("max_weight", C.c_double),
        ("data_particles", C.c_uint64),
        ("total_points", C.c_uint64),
        ("resampled", C.c_int32),
        ("uniform_reset", C.c_int32),
        ("resample_overruns", C.c_uint64),
        ("update_count", C.c_uint64),
        ("map_patches_dropped", C.c_uint64),
        ("map_stores_copied", C.c_uint64),
        ("map_stores_changed", C.c_uint64),
        ("map_patches_covered", C.c_uint64),
        ("map_cells_written", C.c_uint64),
        ("map_pages_taken", C.c_uint64),
        ("map_pages_free", C.c_uint64),
        ("map_tiles_evicted", C.c_uint64),
    ]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class RngState(C.Structure):
    _fields_ = [
        ("minstd_x", C.c_uint32),
        ("pad", C.c_uint32),
        ("project_count", C.c_uint64),
        ("init_count", C.c_uint64),
        ("hash_count", C.c_uint64),
        ("max_weight", C.c_double),
        ("ud_pose", C.c_double * 12),
        ("libc_rand", C.c_uint32 * 34),
        ("libc_rand_pos", C.c_uint32),
        ("pad2", C.c_uint32),
    ]


class KernelTimes(C.Structure):
    _fields_ = [
        ("project_weight_ms", C.c_float),
        ("finalize_ms", C.c_float),
        ("normalize_scan_ms", C.c_float),
        ("resample_ms", C.c_float),
        ("total_ms", C.c_float),
        ("map_gather_ms", C.c_float),
        ("map_cow_ms", C.c_float),
        ("map_merge_ms", C.c_float),
        ("map_total_ms", C.c_float),
        ("map_plan_ms", C.c_float),
        ("map_match_ms", C.c_float),
    ]


ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p)
ALLTOALLV_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.c_void_p,
                           C.POINTER(C.c_uint64), C.c_void_p)


class Comm(C.Structure):
    """eslam_comm (include/eslam_gpu.h)."""
    _fields_ = [
        ("user", C.c_void_p),
        ("rank", C.c_int32), ("nranks", C.c_int32),
        ("device_memory", C.c_int32), ("pad", C.c_int32),
        ("allgather", ALLGATHER_FN),
        ("alltoallv", ALLTOALLV_FN),
    ]


MAX_RANKS = 16


CHUNK_WAVES, CHUNK_CAP = 5120, 13


def chunk_rows(n_global, fixed=0):
    """dm_chunk_rows_cfg (include/eslam_detmath.h): rows of 64 lanes per canonical summation
    chunk -- eslam_config.sum_chunk_rows when set (`fixed`), else sized to whole generations of
    the weighting kernel's resident waves."""
    if fixed:
        return int(fixed)
    rows = (n_global + 63) // 64
    per = CHUNK_WAVES * CHUNK_CAP
    slots = (1 if rows <= per else -(-rows // per)) * CHUNK_WAVES
    return max(1, -(-rows // slots))


def shard_bounds(n_global, nranks, fixed=0):
    """First global index of every rank (+ n_global): near-equal shards whose starts are
    multiples of the summation chunk (64 * chunk_rows; `fixed`: eslam_config.sum_chunk_rows),
    as eslam_gpu_set_comm requires."""
    csz = 64 * chunk_rows(n_global, fixed)
    chunks = -(-n_global // csz)
    if chunks < nranks:
        raise ValueError(f"{n_global} particles cannot be split into {nranks} chunk-aligned shards")
    g = [min(n_global, (chunks * r // nranks) * csz) for r in range(nranks)] + [n_global]
    if any(g[r + 1] <= g[r] for r in range(nranks)):
        raise ValueError("empty shard")
    return g


def default_config(lib=None):
    """eslam_config_default() restated (src/Configuration.hpp:85-111 defaults)."""
    import math
    c = Config()
    c.seed = 42
    c.particle_count = 250
    c.min_effective = 50
    c.initial_rotation_error[:] = [0.0, 0.0, 0.1]
    c.initial_translation_error[:] = [0.1, 0.1, 1.0]
    c.measurement_error = 0.1
    c.discount_factor = 0.9
    c.spread_threshold = 0.9
    c.spread_translation_factor = 0.1
    c.spread_rotation_factor = 0.05
    c.slip_factor = 0.05
    c.max_yaw_deviation = 15 * math.pi / 180.0
    c.measurement_threshold_distance = 0.1
    c.measurement_threshold_angle = 10 * math.pi / 180.0
    c.use_slip_update = 0
    c.use_shape_update = 1
    c.min_contacts = 3
    c.contact_likelihood_correction = 0.33
    c.contact_point_radius = 0.01
    c.hash_use = 0
    c.hash_period = 10
    c.hash_percentage = 0.05
    c.hash_avg_factor = 0.1
    c.hash_slope_bins = 20
    c.hash_angular_steps = 16
    c.log_debug = 0
    c.flags = 0
    c.local_map_pages = 0
    c.max_sensor_range = 3.0
    c.local_map_trail = 16
    c.sum_chunk_rows = 0
    return c


# ---------------------------------------------------------------------------------------
# numpy helpers
# ---------------------------------------------------------------------------------------
def _ptr(a, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


class ParticleArrays:
    """Host SoA buffers + the eslam_particles view onto them."""

    def __init__(self, n):
        import numpy as np
        self.n = n
        self.x = np.zeros(n)
        self.y = np.zeros(n)
        self.orientation = np.zeros(n)
        self.zpos = np.zeros(n)
        self.zsigma = np.zeros(n)
        self.weight = np.zeros(n)
        self.mprob = np.zeros(n)
        self.floating = np.zeros(n, dtype=np.uint8)
        self.n_contact_points = np.zeros(n, dtype=np.uint8)

    def view(self):
        p = Particles()
        for f in ("x", "y", "orientation", "zpos", "zsigma", "weight", "mprob"):
            setattr(p, f, _ptr(getattr(self, f), C.c_double))
        p.floating = _ptr(self.floating, C.c_uint8)
        p.n_contact_points = _ptr(self.n_contact_points, C.c_uint8)
        return p

    FIELDS = ("x", "y", "orientation", "zpos", "zsigma", "weight", "mprob", "floating", "n_contact_points")

    def as_dict(self):
        return {f: getattr(self, f) for f in self.FIELDS}


class GridArrays:
    """An MLS grid held in numpy arrays + the eslam_mls_grid view onto them."""

    def __init__(self, width, height, scale, offset, cell_start, mean, stdev, height_arr=None,
                 global2local=None):
        import numpy as np
        self.width, self.height = int(width), int(height)
        self.scale = (float(scale[0]), float(scale[1]))
        self.offset = (float(offset[0]), float(offset[1]))
        self.cell_start = np.ascontiguousarray(cell_start, dtype=np.uint32)
        self.mean = np.ascontiguousarray(mean, dtype=np.float32)
        self.stdev = np.ascontiguousarray(stdev, dtype=np.float32)
        self.patch_height = None if height_arr is None else np.ascontiguousarray(height_arr, dtype=np.float32)
        self.g2l = [1.0, 0, 0, 0, 0, 1.0, 0, 0, 0, 0, 1.0, 0] if global2local is None else list(global2local)
        assert self.cell_start.shape[0] == self.width * self.height + 1
        assert int(self.cell_start[-1]) == self.mean.shape[0] == self.stdev.shape[0]

    def view(self):
        g = MlsGrid()
        g.width, g.height = self.width, self.height
        g.scale_x, g.scale_y = self.scale
        g.offset_x, g.offset_y = self.offset
        g.global2local[:] = self.g2l
        g.cell_start = _ptr(self.cell_start, C.c_uint32)
        g.patch_mean = _ptr(self.mean, C.c_float)
        g.patch_stdev = _ptr(self.stdev, C.c_float)
        g.patch_height = None if self.patch_height is None else _ptr(self.patch_height, C.c_float)
        g.n_patches = int(self.mean.shape[0])
        return g
