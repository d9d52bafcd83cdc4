/*
 * eslam_gpu.h -- C ABI of the MI355X-native eSLAM particle-filter core.
 *
 * Drop-in boundary for the per-step hot path of liyangSKD/slam-eslam:
 *
 *   EmbodiedSlamFilter::update(body2odometry, BodyContactState, ltc)   src/EmbodiedSlamFilter.cpp:353-369
 *     -> PoseEstimator::project                                         src/PoseEstimator.cpp:184-242
 *     -> PoseEstimator::update -> updateWeights                         src/PoseEstimator.cpp:244-352
 *          -> ContactModel::setContactPoints/evaluatePose/evaluateWeight/updateZPositionEstimate
 *                                                                       src/ContactModel.cpp:21-41,117-340
 *          -> GridAccess::get -> MLSMap::getPatch(p, patch, 3.0)        src/PoseEstimator.hpp:97-105
 *     -> ParticleFilter::normalizeWeights / resample_stratified         src/ParticleFilter.hpp:46-108
 *
 * Plain C: POD structs, pointers and sizes, no torch / HIP types in the signatures.  Every
 * entry point returns ESLAM_OK (0) or a negative ESLAM_ERR_* code; eslam_gpu_last_error()
 * gives the message (the reference's std::runtime_error texts where one exists).
 *
 * One context = one GPU (one process per GPU for multi-GPU; see eslam_gpu_set_comm).  A
 * context is not thread-safe.  Device memory is owned by the context; host buffers passed
 * in are owned by the caller and only read/written during the call.
 */
#ifndef ESLAM_GPU_H
#define ESLAM_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ESLAM_ABI_VERSION 8

/* maximum number of contact points of one BodyContactState handled per step
 * (asguard: 4 wheels x 5 feet = 20, src/ContactModel.cpp grouping) */
#define ESLAM_MAX_CONTACTS 32

/* ---- status codes -------------------------------------------------------------------- */
#define ESLAM_OK 0
#define ESLAM_ERR_INVALID_ARG -1
#define ESLAM_ERR_NO_ENVIRONMENT -2      /* "No environment attached." src/PoseEstimator.cpp:259-260 */
#define ESLAM_ERR_ZERO_MEAS_VAR -3       /* "using a zero measurement variance leads to singularities" src/ContactModel.cpp:122-123 */
#define ESLAM_ERR_HASH_SAMPLE -4         /* "could not sample from pose hash." src/PoseEstimator.cpp:84 */
#define ESLAM_ERR_NO_MLS_GRID -5         /* "The provided environment does not contain an mls grid." src/EmbodiedSlamFilter.cpp:104 */
#define ESLAM_ERR_HIP -6                 /* HIP runtime failure (message has details) */
#define ESLAM_ERR_NOT_INITIALISED -7     /* no particles yet */
#define ESLAM_ERR_UNSUPPORTED -8
#define ESLAM_ERR_OUT_OF_MEMORY -9
#define ESLAM_ERR_COMM -10               /* a collective callback failed */

/* ---- Configuration (src/Configuration.hpp:12-213, the fields consumed on the path) ---- */
typedef struct eslam_config {
    uint64_t seed;                         /* Configuration::seed (42)                     */
    uint64_t particle_count;               /* Configuration::particleCount (250)           */
    uint64_t min_effective;                /* Configuration::minEffective (50)             */
    double initial_rotation_error[3];      /* (0, 0, 0.1)                                  */
    double initial_translation_error[3];   /* (0.1, 0.1, 1.0)                              */
    double measurement_error;              /* 0.1                                          */
    double discount_factor;                /* 0.9                                          */
    double spread_threshold;               /* 0.9                                          */
    double spread_translation_factor;      /* 0.1                                          */
    double spread_rotation_factor;         /* 0.05                                         */
    double slip_factor;                    /* 0.05                                         */
    double max_yaw_deviation;              /* 15 deg                                       */
    double measurement_threshold_distance; /* UpdateThreshold(0.1, 10 deg).distance       */
    double measurement_threshold_angle;    /*                             .angle           */
    /* ContactModelConfiguration (src/Configuration.hpp:51-81) */
    int32_t use_slip_update;               /* false                                        */
    int32_t use_shape_update;              /* true                                         */
    uint64_t min_contacts;                 /* 3                                            */
    double contact_likelihood_correction;  /* 0.33                                         */
    double contact_point_radius;           /* 0.01                                         */
    /* SurfaceHashConfig (src/Configuration.hpp:32-49) */
    int32_t hash_use;                      /* false                                        */
    uint64_t hash_period;                  /* 10                                           */
    double hash_percentage;                /* 0.05                                         */
    double hash_avg_factor;                /* 0.1                                          */
    uint64_t hash_slope_bins;              /* 20                                           */
    uint64_t hash_angular_steps;           /* 16                                           */
    int32_t log_debug;                     /* Configuration::logDebug (false)              */
    /* build-specific knobs (not in the reference) */
    uint32_t flags;                        /* ESLAM_FLAG_*                                 */
    /* per-particle maps (ESLAM_FLAG_PARTICLE_MAPS): the device page pool, in pages of 8 x 8
     * cells per particle (0: the default, 16); the pool is shared by all particles' maps and
     * collected when a map update needs more (ESLAM_ERR_OUT_OF_MEMORY when even that fails) */
    uint32_t local_map_pages;
    /* Configuration::maxSensorRange (3.0, src/Configuration.hpp:107): a particle's own map keeps
     * the tiles of 8 x 8 cells within this range of the particle             */
    double max_sensor_range;
    /* per-particle maps (ABI 7): tiles a map keeps after its window has left them (the trail;
     * the reference's MLSMap keeps every grid it made, src/EmbodiedSlamFilter.cpp:195-207), up
     * to this many per map (default 16; 0: tiles leaving the window are forgotten).  Their
     * pages come from the same pool (local_map_pages).                                       */
    uint32_t local_map_trail;
    /* rows of 64 particles per canonical summation chunk (ABI 8; 0: dm_chunk_rows(n_global),
     * the default).  The chunk fixes the order of the fp64 partial sums, so two
     * filters agree bit for bit only with the same value.  A sharded filter of G ranks may set
     * dm_chunk_rows(n_global / G) so that every rank's weighting kernel fills the chip (16M
     * over 8 ranks: 7 instead of 13); its one-GPU equal then sets the same.  At most 31.     */
    uint32_t sum_chunk_rows;
} eslam_config;

#define ESLAM_FLAG_RECORD_ANCESTORS 0x1u   /* keep the last resample's ancestor indices     */
#define ESLAM_FLAG_NO_MAP_LDS 0x2u         /* disable the LDS map window (global lookups)   */
#define ESLAM_FLAG_NO_AUX_GATHER 0x4u      /* do not carry mprob/floating through resample  */
#define ESLAM_FLAG_PARTICLE_MAPS 0x10u     /* useSharedMap = false: every particle its own local
                                              map (eslam_gpu_map_update)                      */
#define ESLAM_FLAG_RECORD_CONTACTS 0x8u    /* keep every update's cpoints, meas_pos, meas_theta
                                              (also on with log_debug); on a sharded filter
                                              download_records is then a collective          */
#define ESLAM_FLAG_PROCESS_STATICS 0x20u  /* Q11: the hash-respawn counter (the function static
                                              of src/PoseEstimator.cpp:239) and rand() are the
                                              process's, shared by every context that sets this
                                              flag (default: each context its own); one
                                              sharded (nranks > 1) context per process may
                                              set it: eslam_gpu_set_comm refuses a second
                                              (ranks in one process would share them)        */

void eslam_config_default(eslam_config* cfg);

/* ---- multi-level surface grid (envire::MLSGrid as consumed by GridAccess::get) ----------
 * Cells are (m, n) with m along x; cell index = n * width + m.  Patches of cell c are
 * patches[cell_start[c] .. cell_start[c+1]) in stored order.  getPatch(p, patch, 3.0)
 * transforms p by global2local, finds the cell with
 *   m = floor((x - offset_x) / scale_x), n = floor((y - offset_y) / scale_y),
 * and returns the first patch whose distance to the query patch (mean = p.z,
 * stdev = sqrt(measVar)) is below 3:  |mean_p - mean_q| / sqrt(stdev_p^2 + stdev_q^2)
 * (vertical patches, height > 0, span [mean - height, mean]).                           */
typedef struct eslam_mls_grid {
    uint32_t width, height;
    double scale_x, scale_y;
    double offset_x, offset_y;
    double global2local[12];               /* 3x4 row-major affine: GridAccess::C_global2local */
    const uint32_t* cell_start;            /* width*height + 1 entries                       */
    const float* patch_mean;               /* n_patches                                      */
    const float* patch_stdev;              /* n_patches                                      */
    const float* patch_height;             /* n_patches or NULL (all horizontal)             */
    uint64_t n_patches;
} eslam_mls_grid;

/* ---- per-step input: EmbodiedSlamFilter::update(body2odometry, bs, ltc) ---------------- */
typedef struct eslam_contact_point {       /* odometry::BodyContactPoint                    */
    double position[3];                    /* body frame                                    */
    float contact;                         /* contact probability, NaN = unknown (passes)   */
    int32_t group_id;                      /* -1 = ungrouped                                */
} eslam_contact_point;

typedef struct eslam_step_input {
    double body2odometry_rot[4];           /* quaternion (w, x, y, z) of body2odometry        */
    double body2odometry_trans[3];
    /* outputs of the external odometry::FootContact after odometry.update(bs, orientation):
     * getPoseDelta().position, getPositionError()(2,2) and the Gaussian that
     * getPoseDeltaSample2D() samples (mean dx, dy, dtheta; 3x3 covariance, row-major).     */
    double pose_delta_trans[3];
    double position_error_zz;
    double sample_mean[3];
    double sample_cov[9];
    uint32_t n_contacts;
    uint32_t ltc_count;                    /* terrain classifications given (gate only)      */
    eslam_contact_point contacts[ESLAM_MAX_CONTACTS];
} eslam_step_input;

/* ---- particle state, structure of arrays (PoseParticle, src/PoseParticle.hpp:52-86) ----- */
typedef struct eslam_particles {
    double* x;                             /* position.x                                    */
    double* y;                             /* position.y                                    */
    double* orientation;
    double* zpos;
    double* zsigma;
    double* weight;
    double* mprob;
    uint8_t* floating;
    uint8_t* n_contact_points;             /* cpoints.size() of the last updateWeights       */
} eslam_particles;

/* result of one PoseEstimator::update (device-side values, read after eslam_gpu_sync) */
typedef struct eslam_update_info {
    double effective;                      /* normalizeWeights() return value                */
    double weight_sum;                     /* sum of weights before normalisation            */
    double floating_weight;                /* sum_data_weights / data_particles              */
    double max_weight;                     /* PoseEstimator::max_weight after the update      */
    uint64_t data_particles;
    uint64_t total_points;
    int32_t resampled;
    int32_t uniform_reset;                 /* sumWeights <= 0 branch taken                   */
    uint64_t resample_overruns;            /* draws beyond the cumulative sum (clamped, Q5)  */
    uint64_t update_count;
    /* the last eslam_gpu_map_update (per-particle maps): scan patches beyond a particle's
     * window (farther than max_sensor_range; summed over the particles); maps the merge
     * changed while another particle shared them (copy on write: written to a free table the
     * particle then names); maps the merge changed in all (cells, or the window moved); scan
     * patches that landed on cells the shared grid covers (not merged: the per-particle map
     * holds only cells the shared grid leaves empty)                            */
    uint64_t map_patches_dropped;
    uint64_t map_stores_copied;
    uint64_t map_stores_changed;
    uint64_t map_patches_covered;
    /* the device side of the same map update (not in the oracle: they depend on how the
     * pages were shared): cell writes (inserts and fuses), pages taken from the pool (copies
     * on write and new tiles), pages left in the pool's free list                           */
    uint64_t map_cells_written;
    uint64_t map_pages_taken;
    uint64_t map_pages_free;
    /* (ABI 7) tiles the last map update's windows left that a full trail could not keep
     * (forgotten; summed over the particles; in the oracle too)                              */
    uint64_t map_tiles_evicted;
} eslam_update_info;

/* ---- lifecycle ------------------------------------------------------------------------ */
typedef struct eslam_ctx eslam_ctx;

/* PoseEstimator(odometry, config) / EmbodiedSlamFilter(odoConfig, config): binds `device`. */
int eslam_gpu_create(const eslam_config* cfg, int device, eslam_ctx** out);
/* Never collective: an exchange a sharded filter still owes (see eslam_gpu_set_comm) is
 * dropped, so destroy is safe on one rank's error path and after the communicator is gone.
 * SPMD code calls eslam_gpu_finish on every rank first.                                  */
void eslam_gpu_destroy(eslam_ctx* ctx);
/* Collective on a sharded filter (every rank, at the same point): completes the last
 * update's deferred exchange if this rank still owes it, then waits for the stream; on one
 * GPU it only waits for the stream.  A rank whose filter a rank-local fault poisoned (e.g.
 * ESLAM_ERR_OUT_OF_MEMORY from its page pool) cannot take part: finish returns at once
 * there, and peers that still owe the exchange would wait for it.  Treat such an error as
 * fatal for the whole group (abort the communicator), as for any failed collective.       */
int eslam_gpu_finish(eslam_ctx* ctx);
const char* eslam_gpu_last_error(const eslam_ctx* ctx);
int eslam_gpu_abi_version(void);
/* SHA-256 (hex) of the sources, headers and compiler flags the library was built from
 * (slam-eslam_amd/build_lib.py source_hash): identifies the exact build a run loaded      */
const char* eslam_gpu_build_id(void);
/* run on a caller-provided hipStream_t (NULL = the context's own stream) */
int eslam_gpu_set_stream(eslam_ctx* ctx, void* hip_stream);

/* ---- environment: PoseEstimator::setEnvironment src/PoseEstimator.cpp:47-62 and
 * GridAccess::setMap src/PoseEstimator.hpp:68-95 (shared map, useShared = true).  Device
 * memory: 8 bytes per patch (+4 with heights) and about 20.2 bytes per cell (range word,
 * a 16-byte record of the cell's range and first patch, one occupancy bit)                 */
int eslam_gpu_set_map(eslam_ctx* ctx, const eslam_mls_grid* grid);

/* ---- initialisation -------------------------------------------------------------------
 * PoseEstimator::init(N, mu, sigma, zpos, zsigma)  src/PoseEstimator.cpp:88-102
 * mu/sigma = (x, y, theta).  weight = 0 (Q3), floating = true.                          */
int eslam_gpu_init_gaussian(eslam_ctx* ctx, uint64_t n, const double mu[3], const double sigma[3],
                            double zpos, double zsigma);
/* EmbodiedSlamFilter::init(env, pose, useSharedMap=true)  src/EmbodiedSlamFilter.cpp:70-177
 * pose = position[3] + quaternion (w,x,y,z); particle count / errors from the config.    */
int eslam_gpu_init_pose(eslam_ctx* ctx, const double position[3], const double orientation[4]);
/* replace the particle set (getParticles() is a mutable reference in the reference)       */
int eslam_gpu_upload_particles(eslam_ctx* ctx, uint64_t n, const eslam_particles* p);
int eslam_gpu_download_particles(eslam_ctx* ctx, eslam_particles* p);
/* edit particles [first, first + count) in place, the way the reference's callers edit the
 * vector getParticles() returns (processMap's weights, src/EmbodiedSlamFilter.cpp:183-220):
 * every non-NULL field of p (arrays of count values) overwrites that field; the particle
 * set, the per-particle maps, the RNG and the last update's records stay.  The weight scale
 * of the next update is then set from the largest weight, as eslam_gpu_upload_particles does,
 * so an edit through this call and a download / edit / upload of the whole set lead to the
 * same particles bit for bit.  On a sharded filter the call is collective, like the upload:
 * every rank makes it at the same point (count may be 0, and any field may be NULL), and
 * the ranks agree on the weight scale of the next update whichever of them wrote weights. */
int eslam_gpu_write_particles(eslam_ctx* ctx, uint64_t first, uint64_t count, const eslam_particles* p);

/* ---- per-particle local maps (useSharedMap = false) -----------------
 * EmbodiedSlamFilter::processMap(scanMap, match=false, update=true)
 * (src/EmbodiedSlamFilter.cpp:179-232) after PoseEstimator::cloneMaps (src/PoseEstimator.cpp:
 * 31-47): every particle's map is the shared grid plus its own patches in cells the grid
 * leaves empty, kept in a window of tiles of 8 x 8 cells centred on the particle that reaches
 * max_sensor_range (maxSensorRange, 3 m) in every direction.  A map update
 * moves each particle's window to the tile under the particle (the active-grid switch of
 * :195-207; tiles that leave the window are forgotten), places the scan patches at the
 * particle's pose (Translation(x, y, 0) * Rz(theta); offset patch zPos, zSigma) and, per
 * patch, inserts it into an empty cell or fuses it (variance-weighted) with the particle's
 * patch there when within 3 sigma; cells of the shared grid are not changed, and a patch
 * beyond the window is dropped (counted).  With an empty shared grid every particle starts
 * from an empty map, as the reference's clones of its empty grid template
 * (src/EmbodiedSlamFilter.cpp:131-134).  The contact update then reads each particle's own
 * map.  Particles that a resample copied share their tables and pages until a map update
 * writes them (copy on write).  set_map starts every particle's map over (empty).  Only the
 * insert-into-empty-cell rule is pinned by the reference (test/testMap.cpp:307-316);
 * envire's MLSGrid::merge is not in the reference.                                       */
typedef struct eslam_scan_patch {
    double position[3];                    /* yaw-free body frame (the scan MLS's cells)    */
    double stdev;                          /* sensor sigma of the patch                      */
} eslam_scan_patch;
/* Any count: a scan of more than 64 patches merges 64 at a time, in order (every cell sees
 * its patches in the scan's order); the update's counters add up over the parts
 * (map_stores_changed counts a map once per part that changed it).                          */
int eslam_gpu_map_update(eslam_ctx* ctx, const eslam_scan_patch* patches, uint32_t count);
/* processMap(scanMap, match = true, ...)  src/EmbodiedSlamFilter.cpp:214-221: the visual
 * weighting w *= pow(weight, 0.1f) of every particle against its own map (per-particle maps).
 * envire's MLSGrid::match is not in the reference, so the rule is this build's (DESIGN.md 5c,
 * parity unpinned): every 10th scan patch (sampling 10), placed like the merge, that lands on
 * a cell the particle's own map holds -- a tile inside both its window and the window the
 * next update centres on the particle -- scores exp(-d^2 / (2 sigma^2)), sigma 0.2f, d = the
 * patch's height + zPos - the cell's mean; weight = the mean score as a float (1 without a
 * matched cell).  Call it before eslam_gpu_map_update, as processMap does; weights are not
 * normalised.                                                                              */
int eslam_gpu_map_match(eslam_ctx* ctx, const eslam_scan_patch* patches, uint32_t count);
/* PoseEstimator::setEnvironment(env, map, useShared)  src/PoseEstimator.cpp:49-62: on = 1
 * gives every particle its own map (ESLAM_FLAG_PARTICLE_MAPS), 0 the shared map only.  Before
 * the particles are initialised (ESLAM_ERR_INVALID_ARG after).  On a sharded filter a
 * particle that a resample moves to another rank carries its own patches.                 */
int eslam_gpu_set_particle_maps(eslam_ctx* ctx, int on);
/* particle index's own patches (cell = n * width + m, mean, stdev), its window's tiles in slot
 * order and each tile's cells row by row; *count = how many it has (up to capacity written) */
int eslam_gpu_get_particle_map(eslam_ctx* ctx, uint64_t index, uint32_t* cells, float* mean, float* stdev,
                               uint32_t capacity, uint32_t* count);

/* ---- PoseParticle records with the debug fields (getParticles() for logging / viz) ------ */
/* ContactPoint  src/PoseParticle.hpp:20-43: one contact point evaluatePose pushed           */
typedef struct eslam_cpoint {
    double point[3];                       /* surface point: world x, y of the group's first
                                              valid contact and the patch mean (:163-171)   */
    double zdiff, zvar;                    /* ratio-weighted group averages                 */
    double prob;                           /* 1 (the slip update never reaches it, Q8)      */
} eslam_cpoint;

/* PoseParticle  src/PoseParticle.hpp:52-86 as the viz reads it (viz/ParticleVisualization.cpp) */
typedef struct eslam_particle_record {
    double position[2];
    double orientation, zpos, zsigma, mprob, weight;
    double meas_pos[3];                    /* (x, y, zPos) at the last updateWeights          */
    double meas_theta;                     /* orientation at the last updateWeights           */
    uint64_t index;                        /* global particle index                          */
    uint32_t n_cpoints;                    /* cpoints.size()                                 */
    uint8_t floating;
    uint8_t pad[3];
} eslam_particle_record;

/* Particles first, first + stride, ... (count of them) as records, gathered on the device
 * (one copy of count records; a strided subsample keeps logging cheap at millions of
 * particles).  With ESLAM_FLAG_RECORD_CONTACTS (or log_debug) the meas_* fields and up to
 * max_cpoints contact points per particle (cpoints: count x max_cpoints, may be NULL) are
 * those of the last update, carried through its resample like the reference's vectors;
 * otherwise meas_* are 0 and n_cpoints = the count of the last update.
 * Sharded with ESLAM_FLAG_RECORD_CONTACTS / log_debug: a collective (every rank calls it, in
 * the same order, count may be 0): a particle whose ancestor at the last update sat on another
 * rank gets that ancestor's records from it (two all_to_all_v); a rank whose own call fails
 * still takes part and makes every rank return an error.                                    */
int eslam_gpu_download_records(eslam_ctx* ctx, uint64_t first, uint64_t stride, uint64_t count,
                               eslam_particle_record* out, eslam_cpoint* cpoints, uint32_t max_cpoints);
int eslam_gpu_particle_count(const eslam_ctx* ctx, uint64_t* n);

/* ---- the hot path ----------------------------------------------------------------------- */
/* EmbodiedSlamFilter::update(body2odometry, bs, ltc): project, then the measurement update
 * when UpdateThreshold::test(udPose^-1 * body2odometry) (angle/distance swapped, Q6) or
 * ltc_count > 0.  *updated receives the bool.  Asynchronous on the context stream.
 * A zero measurement variance (measurementError = 0 and zSigma = 0; the throw of
 * src/ContactModel.cpp:122-123) returns ESLAM_ERR_ZERO_MEAS_VAR from this call: phase A has
 * run (such particles count as rejected with no contact points), phase B, normalisation and
 * the resample have not, and the update gate pose is not advanced.  Deviation: the reference
 * aborts its particle loop at the first such particle, leaving the later ones projected only. */
int eslam_gpu_step(eslam_ctx* ctx, const eslam_step_input* in, int* updated);
/* PoseEstimator::project(state, orientation)                                              */
int eslam_gpu_project(eslam_ctx* ctx, const eslam_step_input* in);
/* PoseEstimator::update(state, orientation, ltc): updateWeights, normalizeWeights, resample
 * if effective < minEffective.                                                             */
int eslam_gpu_update(eslam_ctx* ctx, const eslam_step_input* in);
/* wait for the stream; fetch the info of the last update (info may be NULL)               */
int eslam_gpu_sync(eslam_ctx* ctx, eslam_update_info* info);
/* The resample scan's blocks wait for each other (the fused finalize, the preceding tiles'
 * totals).  A wait that gives up -- never expected: the blocks it waits for are dispatched
 * first -- poisons the filter: nothing further is written, and every later call (step,
 * update, sync, download, the ParticleFilter API) returns ESLAM_ERR_HIP until init_* or
 * upload_particles starts over.  Testing only: polls before a wait gives up (default 2^18,
 * about 60 ms; 0 gives up at once, which forces the poisoned path).                        */
int eslam_gpu_debug_set_spin_limit(eslam_ctx* ctx, uint32_t polls);

/* ---- ParticleFilter<T> API (src/ParticleFilter.hpp:34-173) ------------------------------ */
int eslam_gpu_get_weights_sum(eslam_ctx* ctx, double* sum);          /* getWeightsSum :34-39     */
int eslam_gpu_normalize_weights(eslam_ctx* ctx, double* effective);  /* normalizeWeights :46-70 */
int eslam_gpu_resample(eslam_ctx* ctx);        /* resample() -> resample_stratified(N) :72-108 */
int eslam_gpu_get_best_particle_index(eslam_ctx* ctx, uint64_t* index);  /* :160-173 (Q16)  */
/* PoseEstimator::getCentroid src/PoseEstimator.cpp:354-383 (normalises in place, Q15):
 * position[3] + quaternion (w,x,y,z)                                                        */
int eslam_gpu_get_centroid(eslam_ctx* ctx, double position[3], double orientation[4]);

/* ---- resume state: RNG + the filter scalars (bit-exact resume with the particles) ------- */
typedef struct eslam_rng_state {
    uint32_t minstd_x;                     /* ParticleFilter::rand_gen state                */
    uint32_t pad;
    uint64_t project_count;                /* Philox event counter of project()              */
    uint64_t init_count;
    uint64_t hash_count;
    double max_weight;                     /* PoseEstimator::max_weight                      */
    double ud_pose[12];                    /* EmbodiedSlamFilter::udPose, 3x4 row-major      */
    uint32_t libc_rand[34];                /* SurfaceHash::sample's rand() (glibc TYPE_3)    */
    uint32_t libc_rand_pos;
    uint32_t pad2;
} eslam_rng_state;
int eslam_gpu_get_rng_state(eslam_ctx* ctx, eslam_rng_state* st);
int eslam_gpu_set_rng_state(eslam_ctx* ctx, const eslam_rng_state* st);

/* ---- SurfaceHash (useHash = true): pose hash of the map by terrain slope ----------------
 * SurfaceHash::create  src/SurfaceHash.hpp:155-231 on the map of eslam_gpu_set_map, with
 * the config's hash_slope_bins / hash_angular_steps (a sweep over segments x cells on the
 * GPU).  eslam_gpu_init_pose builds it on demand when config.hash_use is set and then
 * initialises from it (PoseEstimator::init(N, hash) src/PoseEstimator.cpp:75-86); with
 * hash_use, every hash_period-th project (starting with the first) runs sampleFromHash
 * (src/PoseEstimator.cpp:130-182, 238-240).  rand() is glibc's generator seeded with 1
 * (the reference never seeds it), one state per context.                                  */
int eslam_gpu_hash_create(eslam_ctx* ctx);
/* PoseEstimator::init(N, hash): particle i = a uniformly drawn hash pose                   */
int eslam_gpu_init_hash(eslam_ctx* ctx, uint64_t n);
/* number of hash poses; bucket_sizes (slope_bins^2 entries, bucket = bx * bins + by) or NULL */
int eslam_gpu_hash_info(eslam_ctx* ctx, uint64_t* n_poses, uint32_t* bucket_sizes);
/* the hash poses in sweep order (x, y, theta, z) and their buckets; any pointer may be NULL */
int eslam_gpu_hash_poses(eslam_ctx* ctx, double* x, double* y, double* theta, double* z, int32_t* bucket);

/* ---- multi-GPU: one context per GPU holds a contiguous shard of ONE global filter -------
 * The library is transport-agnostic: it calls the collectives below at the three exchange
 * points of an update.  In production they are torch.distributed over RCCL
 * (xGMI) on device buffers (slam-eslam_amd/eslam_dist.py); tests use gloo on host buffers.
 *   1. all_gather of the exact per-rank weighting statistics (~0.5 KB per rank)
 *      -> every rank finalises the same global floating weight, weight sum, effective N
 *   2. all_gather of the per-rank fixed-point weight totals (8 B per rank)
 *      -> global cumulative-sum offsets for the stratified draws
 *   3. all_gather of the per-destination send counts + all_to_all_v of the particles
 *      whose stratified draws land on another rank (72-byte records)
 * Results are bit-identical to the single-GPU run of the same global filter.          */
typedef struct eslam_comm {
    void* user;
    int32_t rank, nranks;
    int32_t device_memory;                 /* 1: callbacks take device pointers (RCCL)     */
    int32_t pad;
    /* recv[r * bytes .. (r+1) * bytes) <- send of rank r.  stream: the context's HIP
     * stream when device_memory (the collective is ordered after the work already on it
     * and work queued after the call returns must see its result), NULL otherwise.        */
    int (*allgather)(void* user, const void* send, void* recv, uint64_t bytes, void* stream);
    /* send_bytes[r] bytes to rank r (packed in rank order), recv_bytes[r] from rank r    */
    int (*alltoallv)(void* user, const void* send, const uint64_t* send_bytes, void* recv,
                     const uint64_t* recv_bytes, void* stream);
} eslam_comm;

/* Make this context shard [gbase, gbase + n_local) of an n_global-particle filter; call
 * before init.  shard_gbase lists the first global index of every rank (nranks + 1
 * entries, strictly increasing, last = n_global <= 2^30 - 64); every entry must be a multiple
 * of 64 * dm_chunk_rows(n_global) (the canonical summation chunk) except the last.
 * The context's config particle_count is the global count.  Sharded contexts support
 * the hot path (step/project/update/sync), init, upload/download of the local shard,
 * weights sum / normalise / resample, the best particle (global index), the centroid, the
 * hash respawn and per-particle maps, each equal to one GPU bit for bit.  comm == NULL
 * returns the context to one GPU.
 * Calls on a sharded filter follow SPMD order: every rank makes the same sequence of
 * calls that update, write, normalise, resample or reduce (they run collectives).  The
 * rank-local getters (download, records, particle maps, RNG state, hash poses) may be
 * called by any subset of ranks: the only collective they can run is the previous
 * update's deferred exchange, which every rank completes exactly once -- in a getter, in
 * its next collective call or in eslam_gpu_finish -- so the ranks stay matched.         */
int eslam_gpu_set_comm(eslam_ctx* ctx, const eslam_comm* comm, uint64_t n_global, const uint64_t* shard_gbase);

/* ---- multi-GPU over RCCL, driven from the library (no callback into the host language) --
 * SURVEY.md 8(b) "comm_init(nranks, rank, ncclUniqueId*)"; the reference has one CPU
 * filter and no distribution (src/EmbodiedSlamFilter.hpp:29-39 owns it by value).
 * eslam_gpu_rccl_unique_id: rank 0 creates the 128-byte RCCL id (ncclGetUniqueId) that the
 * caller broadcasts to every rank by any means.  eslam_gpu_set_comm_rccl: every rank then
 * joins the communicator (ncclCommInitRank, collective: all ranks must call it) and the
 * context becomes shard `rank` exactly as eslam_gpu_set_comm makes it; the exchanges are
 * ncclAllGather and grouped ncclSend/ncclRecv on the context's stream.  RCCL is loaded at
 * run time (librccl.so.1); without it these return ESLAM_ERR_UNSUPPORTED.                 */
#define ESLAM_RCCL_ID_BYTES 128
int eslam_gpu_rccl_unique_id(uint8_t id[ESLAM_RCCL_ID_BYTES]);
int eslam_gpu_set_comm_rccl(eslam_ctx* ctx, int32_t nranks, int32_t rank, const uint8_t id[ESLAM_RCCL_ID_BYTES],
                            uint64_t n_global, const uint64_t* shard_gbase);

/* ---- diagnostics ------------------------------------------------------------------------- */
/* ancestor index of every particle of the last resample (needs ESLAM_FLAG_RECORD_ANCESTORS) */
int eslam_gpu_get_ancestors(eslam_ctx* ctx, uint32_t* out, uint64_t n);
/* per-kernel timing of the last step, milliseconds (HIP events on the context stream)     */
typedef struct eslam_kernel_times {
    float project_weight_ms;
    float finalize_ms;
    float normalize_scan_ms;
    float resample_ms;
    float total_ms;
    /* eslam_gpu_map_update (per-particle maps), averaged over the map updates of the timed
     * region: the pending resample gather (sharded filters; one GPU fuses it into the merge),
     * the tables' sharing classes and the free-table list (copy on write's bookkeeping), the
     * plan (k_map_plan, the page budget and, when the free pages run short, the collection),
     * the merge kernel with its counters, and the whole call                               */
    float map_gather_ms;
    float map_cow_ms;
    float map_merge_ms;
    float map_total_ms;
    float map_plan_ms;
    /* eslam_gpu_map_match (ABI 6): the call's gather and k_map_match, averaged over the
     * matches of the timed region                                                         */
    float map_match_ms;
} eslam_kernel_times;
int eslam_gpu_enable_timing(eslam_ctx* ctx, int enable);
int eslam_gpu_get_kernel_times(eslam_ctx* ctx, eslam_kernel_times* t);
/* evaluate the deterministic math on the device for n inputs (tests/test_gpu_math.py):
 * fn: 0 exp, 1 log, 2 sin, 3 cos, 4 erfc, 5 sqrt, 6 div(x, y), 7 pdf/cdf ratio(x, y),
 *     8 pow(x, y), 9 fx61(x) as bits, 13 sin(2 pi x), 14 cos(2 pi x) (Box-Muller angle),
 *     20..25: the butterflies' lane exchange, out[i] = x[i ^ 2^(fn - 20)] (n a multiple of 256) */
int eslam_gpu_selftest_math(int device, int fn, const double* x, const double* y, double* out, uint64_t n);
/* the Box-Muller radius sqrt(-2 log u) with the range-restricted dm_log_pos / dm_sqrt_pos
 * against the general dm_log / dm_sqrt, on the device, for all 2^32 uniform words: the
 * number of words whose results differ in any bit (0 expected)                           */
int eslam_gpu_selftest_bm_radius(int device, uint64_t* mismatches);
/* the device's stable radix sort of (key, value) pairs (the hash respawn's select order)  */
int eslam_gpu_selftest_sort(int device, const uint32_t* keys, const uint32_t* vals, uint64_t n, uint32_t* keys_out,
                            uint32_t* vals_out);

#ifdef __cplusplus
}
#endif
#endif /* ESLAM_GPU_H */
