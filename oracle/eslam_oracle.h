/*
 * eslam_oracle.h -- CPU oracle: a plain-C restatement of the reference hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (slam-eslam_amd/, include/) links or
 * calls this; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg do,
 * and only as the checker / the timed CPU baseline.
 *
 * Every function cites the reference file:line it restates.  Two summation modes:
 *   OR_SUM_REFERENCE  literal reference arithmetic: sequential double sums
 *                     (src/PoseEstimator.cpp:305-310,329; src/ParticleFilter.hpp:34-108);
 *   OR_SUM_CONTRACT   the build's order-independent exact sums (DESIGN.md "sum contract"),
 *                     which the GPU reproduces bit-for-bit.
 * Random draws follow the build's RNG contract (include/eslam_detmath.h) in both modes;
 * the resample draws are the reference's own minstd_rand + uniform_real stream.
 */
#ifndef ESLAM_ORACLE_H
#define ESLAM_ORACLE_H

#include <stdint.h>
#include "../include/eslam_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ESLAM_ORACLE_MAX_RANKS 16
#define OR_SUM_CONTRACT 0
#define OR_SUM_REFERENCE 1

/* ---- ContactModel (src/ContactModel.hpp:32-166) on an arbitrary map callback ---------- */
/* bool map(const Vector3d& p, SurfacePatch& patch): q_mean/q_var describe the query patch
 * the reference constructs at src/ContactModel.cpp:151 (mean = p.z, stdev^2 = measVar).    */
typedef int (*or_map_fn)(void* user, const double p[3], double q_mean, double q_var,
                         double* mean, double* stdev);

typedef struct or_cpoint {                 /* eslam::ContactPoint src/PoseParticle.hpp:20-43 */
    double point[3];
    double zdiff, zvar, prob;
} or_cpoint;

typedef struct or_contact_model {
    /* ContactModelConfiguration */
    int32_t use_slip_update, use_shape_update;
    uint64_t min_contacts;
    double correction, radius;
    /* contactState (after setContactPoints) */
    uint32_t m;
    double pos[ESLAM_MAX_CONTACTS][3];
    float contact[ESLAM_MAX_CONTACTS];
    int32_t group[ESLAM_MAX_CONTACTS];
    /* outputs of the last evaluatePose */
    uint32_t ncp;
    or_cpoint cp[ESLAM_MAX_CONTACTS];
    double zdelta, zvar, weight, posevar;
    double shape_s2;                       /* sum of squared normalised deviations       */
    /* lowest points per group */
    uint32_t nlow;
    double low[ESLAM_MAX_CONTACTS][3];
    /* 1: the reference's literal arithmetic (or_set_literal), 0: the build's contract */
    int32_t literal;
    int32_t pad_literal;
} or_contact_model;

void or_cm_init(or_contact_model* cm, const eslam_config* cfg);
/* ContactModel::setContactPoints(state, orientation)  src/ContactModel.cpp:21-41 */
void or_cm_set_contact_points(or_contact_model* cm, uint32_t n, const eslam_contact_point* pts,
                              const double q_wxyz[4]);
/* ContactModel::evaluatePose(pose, measVar, map)  src/ContactModel.cpp:117-224
 * pose: 3x4 row-major affine.  Returns 1/0, or -1 when measVar == 0 (the throw). */
int or_cm_evaluate_pose(or_contact_model* cm, const double pose[12], double meas_var,
                        or_map_fn map, void* user);
/* ContactModel::updateZPositionEstimate  src/ContactModel.cpp:319-340 */
int or_cm_update_z(const or_contact_model* cm, double* zpos, double* zvar);
/* getLowestPointPerGroup / updateContactStateUsingLowestPointHeuristic  src/ContactModel.cpp:48-92 */
uint32_t or_cm_lowest_points(or_contact_model* cm, double* out_xyz);
void or_cm_update_contact_state_lph(or_contact_model* cm);

/* ---- SurfaceHash pieces (src/SurfaceHash.hpp) -------------------------------------------- */
void or_surface_param_from_points(const double* xyz, uint32_t n, double* slope_x, double* slope_y);
int or_bucket_index(int count, double min_val, double max_val, double value);

/* ---- MLS grid (envire::MLSGrid::getPatch semantics, see eslam_gpu.h) --------------------- */
int or_mls_get_patch(const eslam_mls_grid* g, const double p[3], double q_mean, double q_var,
                     double* mean, double* stdev);
/* the first patch of one grid cell passing the 3-sigma gate against the local height q_mean */
int or_mls_cell_patch(const eslam_mls_grid* g, uint64_t cell, double q_mean, double q_var, double* mean,
                      double* stdev);

/* ---- the filter (PoseEstimator + EmbodiedSlamFilter) -------------------------------------- */
typedef struct or_filter or_filter;

/* SurfaceHash (useHash): create from the filter's map, PoseEstimator::init(N, hash) */
int or_hash_create(or_filter* f);
int or_init_hash(or_filter* f, uint64_t n);
uint64_t or_hash_info(or_filter* f, uint32_t* bucket_sizes);
int or_hash_poses(or_filter* f, double* x, double* y, double* th, double* z, int32_t* bucket);

or_filter* or_create(const eslam_config* cfg, int sum_mode);
void or_destroy(or_filter* f);
/* host threads (OpenMP) of the per-particle project / updateWeights loops; default 1.
 * Results are identical for every thread count. */
void or_set_threads(or_filter* f, int threads);
/* Arithmetic of the per-particle formulas.  0 (default): the build's contract, which the GPU
 * reproduces bit for bit (eslam_detmath.h transcendentals, the rounding-level restatements of
 * DESIGN.md 2).  1: the reference's literal expressions -- contactLikelihoodRatio as boost's
 * pdf / cdf (here libm exp / erfc), the ratio evaluated for every point, the divisions of
 * src/ContactModel.cpp:201-203 and 270-301, the exp of every point, std::pow for m^(1/n) and
 * the discount factor, the 1-sigma test through fabs/sqrt, libm sin/cos (Eigen rotations). */
void or_set_literal(or_filter* f, int literal);
/* capture per-particle contact points / zDelta / zVar of every updateWeights (or_get_debug);
 * off by default (1.5 KB per particle) */
void or_set_debug(or_filter* f, int on);
int or_set_map(or_filter* f, const eslam_mls_grid* g);            /* copies the grid */
int or_init_gaussian(or_filter* f, uint64_t n, const double mu[3], const double sigma[3],
                     double zpos, double zsigma);
int or_init_pose(or_filter* f, const double position[3], const double q_wxyz[4]);
int or_upload(or_filter* f, uint64_t n, const eslam_particles* p);
int or_download(or_filter* f, eslam_particles* p);
uint64_t or_count(const or_filter* f);
int or_project(or_filter* f, const eslam_step_input* in);
int or_update(or_filter* f, const eslam_step_input* in);
int or_step(or_filter* f, const eslam_step_input* in, int* updated);
int or_last_info(or_filter* f, eslam_update_info* info);
double or_get_weights_sum(or_filter* f);
double or_normalize_weights(or_filter* f);
void or_resample(or_filter* f);
void or_resample_multinomial(or_filter* f, uint64_t samples);
uint64_t or_best_index(or_filter* f);
void or_get_centroid(or_filter* f, double position[3], double q_wxyz[4]);
int or_get_ancestors(or_filter* f, uint32_t* out, uint64_t n);
void or_get_rng_state(or_filter* f, eslam_rng_state* st);
void or_set_rng_state(or_filter* f, const eslam_rng_state* st);
/* sharded mode (host-memory eslam_comm only, contract sums): shard [gbase, gbase + n) of an
 * n_global filter -- the CPU statement of the multi-GPU decomposition (eslam_gpu_set_comm) */
int or_set_comm(or_filter* f, const eslam_comm* comm, uint64_t n_global, const uint64_t* shard_gbase);
/* per-particle debug of the last updateWeights: found contact points (cp: n*MAX entries) */
int or_get_debug(or_filter* f, uint32_t* ncp, or_cpoint* cp, double* zdelta, double* zvar);

/* ---- detmath wrappers for tests ------------------------------------------------------------ */
double or_dm(int fn, double x, double y);
void or_dm_philox(uint64_t seed, uint32_t stream, uint64_t ev, uint64_t gidx, uint32_t call, uint32_t out[4]);
void or_dm_philox_raw(const uint32_t ctr[4], uint32_t k0, uint32_t k1, uint32_t out[4]);
uint32_t or_dm_minstd_jump(uint32_t x, uint64_t n);
void or_dm_libc_rand(uint32_t seed, uint32_t n, int32_t* out);     /* glibc rand() after srand(seed) */
double or_dm_limbs_to_double(const uint64_t L[4], int scale);
void or_dm_fx128(double v, int scale, uint32_t limbs[4]);

/* per-particle maps (ESLAM_FLAG_PARTICLE_MAPS): processMap's merge, and a particle's patches;
 * processMap's match weighting on either map (the shared grid, or each particle's own) */
int or_map_update(or_filter* f, const eslam_scan_patch* patches, uint32_t count);
int or_map_match(or_filter* f, const eslam_scan_patch* patches, uint32_t count);
uint32_t or_get_particle_map(or_filter* f, uint64_t i, uint32_t* cells, float* mean, float* stdev, uint32_t cap);
uint64_t or_pages_in_use(or_filter* f);

#ifdef __cplusplus
}
#endif
#endif
