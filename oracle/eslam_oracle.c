/*
 * eslam_oracle.c -- CPU oracle (TEST INFRASTRUCTURE, see eslam_oracle.h).
 *
 * Plain-C restatement of the reference per-step particle-filter path.  Citations are
 * path:line into the reference (liyangSKD/slam-eslam).  Third-party arithmetic the
 * reference calls (Eigen, base-types, boost.math, boost.random, envire, odometry) is
 * restated from its published algorithm; see DESIGN.md "oracle" for what is pinned.
 *
 * Build: oracle/Makefile  (gcc -O2 -mfma -ffp-contract=off -fPIC -shared).
 */
#include "eslam_oracle.h"
#include "../include/eslam_detmath.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ========================================================================================
 * small Eigen / base-types restatements (host only)
 * ====================================================================================== */

/* Eigen::QuaternionBase::toRotationMatrix */
static void q_to_mat(const double q[4], double R[9])
{
    const double w = q[0], x = q[1], y = q[2], z = q[3];
    const double tx = 2.0 * x, ty = 2.0 * y, tz = 2.0 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w;
    const double txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0] = 1.0 - (tyy + tzz); R[1] = txy - twz;         R[2] = txz + twy;
    R[3] = txy + twz;         R[4] = 1.0 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;         R[7] = tyz + twx;         R[8] = 1.0 - (txx + tyy);
}

/* Eigen quaternion product (generic quat_product) */
static void q_mul(const double a[4], const double b[4], double r[4])
{
    double w = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
    double x = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
    double y = a[0] * b[2] + a[2] * b[0] + a[3] * b[1] - a[1] * b[3];
    double z = a[0] * b[3] + a[3] * b[0] + a[1] * b[2] - a[2] * b[1];
    r[0] = w; r[1] = x; r[2] = y; r[3] = z;
}

/* Quaternion(AngleAxis(angle, UnitZ)) */
static void q_from_yaw(double angle, double q[4])
{
    double ha = 0.5 * angle;
    q[0] = cos(ha);
    double s = sin(ha);
    q[1] = s * 0.0; q[2] = s * 0.0; q[3] = s * 1.0;
}

/* QuaternionBase::_transformVector:  uv = vec x v; uv += uv; v + w*uv + vec x uv */
static void q_rotate(const double q[4], const double v[3], double out[3])
{
    const double qx = q[1], qy = q[2], qz = q[3], w = q[0];
    double uv[3] = {qy * v[2] - qz * v[1], qz * v[0] - qx * v[2], qx * v[1] - qy * v[0]};
    uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
    double c[3] = {qy * uv[2] - qz * uv[1], qz * uv[0] - qx * uv[2], qx * uv[1] - qy * uv[0]};
    out[0] = (v[0] + w * uv[0]) + c[0];
    out[1] = (v[1] + w * uv[1]) + c[1];
    out[2] = (v[2] + w * uv[2]) + c[2];
}

/* base::getYaw = getEuler(q)[0]: atan2(m10, m00) unless gimbal-locked (base/Pose.hpp) */
static double get_yaw(const double q[4])
{
    double R[9];
    q_to_mat(q, R);
    double x = sqrt(R[8] * R[8] + R[7] * R[7]);
    if (x > 1e-12) return atan2(R[3], R[0]);
    return 0.0;
}

/* base::removeYaw(q) = AngleAxis(-getYaw(q), UnitZ) * q */
static void remove_yaw(const double q[4], double out[4])
{
    double a[4];
    q_from_yaw(-get_yaw(q), a);
    q_mul(a, q, out);
}

/* Eigen: Quaternion from a rotation matrix (quaternionbase_assign_impl, 3x3) */
static void q_from_mat(const double m[9], double q[4])
{
    double t = m[0] + m[4] + m[8];
    if (t > 0.0) {
        t = sqrt(t + 1.0);
        q[0] = 0.5 * t;
        t = 0.5 / t;
        q[1] = (m[7] - m[5]) * t;
        q[2] = (m[2] - m[6]) * t;
        q[3] = (m[3] - m[1]) * t;
    } else {
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > m[i * 4]) i = 2;
        int j = (i + 1) % 3, k = (j + 1) % 3;
        t = sqrt(m[i * 4] - m[j * 4] - m[k * 4] + 1.0);
        double v[3];
        v[i] = 0.5 * t;
        t = 0.5 / t;
        q[0] = (m[k * 3 + j] - m[j * 3 + k]) * t;
        v[j] = (m[j * 3 + i] + m[i * 3 + j]) * t;
        v[k] = (m[k * 3 + i] + m[i * 3 + k]) * t;
        q[1] = v[0]; q[2] = v[1]; q[3] = v[2];
    }
}

/* AngleAxisd(Quaternion).angle() */
static double q_angle(const double q[4])
{
    double n = sqrt(q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    if (n != 0.0) return 2.0 * atan2(n, fabs(q[0]));
    return 0.0;
}

/* UpdateThreshold::test(const Affine3d& delta)  src/Configuration.hpp:18-26 (args swapped, Q6)
 * with delta = udPose.inverse() * body2odometry                                              */
static int update_threshold_test(double thr_distance, double thr_angle, const double ud[12],
                                 const double q_b[4], const double t_b[3])
{
    double Rb[9];
    q_to_mat(q_b, Rb);
    /* Transform::inverse (Affine): linear = R^T, translation = -(R^T t) */
    double Ri[9] = {ud[0], ud[4], ud[8], ud[1], ud[5], ud[9], ud[2], ud[6], ud[10]};
    double ti[3];
    for (int r = 0; r < 3; ++r) ti[r] = -((Ri[r * 3 + 0] * ud[3] + Ri[r * 3 + 1] * ud[7]) + Ri[r * 3 + 2] * ud[11]);
    double L[9], t[3];
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c)
            L[r * 3 + c] = (Ri[r * 3 + 0] * Rb[0 * 3 + c] + Ri[r * 3 + 1] * Rb[1 * 3 + c]) + Ri[r * 3 + 2] * Rb[2 * 3 + c];
        t[r] = ((Ri[r * 3 + 0] * t_b[0] + Ri[r * 3 + 1] * t_b[1]) + Ri[r * 3 + 2] * t_b[2]) + ti[r];
    }
    double q[4];
    q_from_mat(L, q);
    double angle = q_angle(q);
    double dist = sqrt((t[0] * t[0] + t[1] * t[1]) + t[2] * t[2]);
    /* test(distance := angle, angle := translation norm) */
    return angle > thr_distance || dist > thr_angle;
}

static void set_translation_pose(double ud[12], double x, double y, double z)
{
    memset(ud, 0, 12 * sizeof(double));
    ud[0] = ud[5] = ud[10] = 1.0;
    ud[3] = x; ud[7] = y; ud[11] = z;
}

/* ========================================================================================
 * MLS grid: envire::MLSGrid::getPatch(p, patch, sigma_threshold = 3.0)
 * ====================================================================================== */
/* The query patch (src/ContactModel.cpp:151) has mean = point z and variance measVar; it
 * is compared in the grid frame, i.e. against the local z of the transformed point.  The
 * 3-sigma test is |mean_p - mean_q| < 3 sqrt(stdev_p^2 + measVar), evaluated squared.
 * Cell index (toGrid): floor((x - offset) * (1 / scale)).                               */
int or_mls_get_patch(const eslam_mls_grid* g, const double p[3], double q_mean_world, double q_var,
                     double* mean, double* stdev)
{
    const double* A = g->global2local;
    double lx = p[0], ly = p[1], lz = p[2];
    /* C_global2local * p; an exact identity is applied as the identity (differs from the
     * affine multiply only for infinite / NaN coordinates) */
    static const double id[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    int is_id = 1;
    for (int k = 0; k < 12; ++k) is_id &= A[k] == id[k];
    if (!is_id) {
        lx = ((A[0] * p[0] + A[1] * p[1]) + A[2] * p[2]) + A[3];
        ly = ((A[4] * p[0] + A[5] * p[1]) + A[6] * p[2]) + A[7];
        lz = ((A[8] * p[0] + A[9] * p[1]) + A[10] * p[2]) + A[11];
    }
    const double q_mean = lz;
    (void)q_mean_world;
    const double inv_x = 1.0 / g->scale_x, inv_y = 1.0 / g->scale_y;
    double fm = floor((lx - g->offset_x) * inv_x);
    double fn = floor((ly - g->offset_y) * inv_y);
    if (!(fm >= 0.0 && fm < (double)g->width && fn >= 0.0 && fn < (double)g->height)) return 0;
    return or_mls_cell_patch(g, (uint64_t)fn * g->width + (uint64_t)fm, q_mean, q_var, mean, stdev);
}

/* the first patch of grid cell `cell` passing the 3-sigma gate against the local height q_mean */
int or_mls_cell_patch(const eslam_mls_grid* g, uint64_t cell, double q_mean, double q_var, double* mean, double* stdev)
{
    uint32_t b = g->cell_start[cell], e = g->cell_start[cell + 1];
    for (uint32_t k = b; k < e; ++k) {
        double pm = (double)g->patch_mean[k];
        double ps = (double)g->patch_stdev[k];
        double ph = g->patch_height ? (double)g->patch_height[k] : 0.0;
        double diff;
        if (ph > 0.0) {                   /* vertical patch spans [mean - height, mean] */
            if (q_mean > pm) diff = q_mean - pm;
            else if (q_mean < pm - ph) diff = (pm - ph) - q_mean;
            else diff = 0.0;
        } else {
            diff = fabs(pm - q_mean);
        }
        if (diff * diff < 9.0 * (ps * ps + q_var)) { *mean = pm; *stdev = ps; return 1; }
    }
    return 0;
}

static int grid_map_fn(void* user, const double p[3], double q_mean, double q_var, double* mean, double* stdev)
{
    return or_mls_get_patch((const eslam_mls_grid*)user, p, q_mean, q_var, mean, stdev);
}

/* per-particle local maps: each particle's window of tiles (eslam_detmath.h
 * DM_LM_*); a page holds one tile's 64 cells, {mean, stdev} each.  Pages live in blocks that
 * never move (threads read them while others allocate) and are shared by the maps that a
 * resample copied until a map update writes them (copy on write; page identity never shows
 * in a result).                                                                            */
#define OR_PAGE_BLOCK_BITS 16u
#define OR_PAGE_BLOCKS (1u << 16)             /* at most 2^32 pages                            */
typedef struct { float v[2 * DM_LM_PAGE_CELLS]; } or_page;

/* the window of one particle's map: GridAccess::get on the particle's own map */
typedef struct {
    const eslam_mls_grid* g;
    const int32_t* ctr;                  /* the particle's window centre (2 tiles)         */
    const uint32_t* slot;                /* its row: slots (page or DM_LM_NONE), then trail */
    or_page* const* blk;                 /* page blocks                                     */
    uint32_t hx, hy, wx, wy;
    uint32_t V;                          /* trail entries after the wx * wy slots           */
} or_pmap;

static const or_page* lm_page(or_page* const* blk, uint32_t p)
{
    return blk[p >> OR_PAGE_BLOCK_BITS] + (p & ((1u << OR_PAGE_BLOCK_BITS) - 1u));
}

/* ---- the trail: a map's tiles outside its window ------------------------
 * The reference's per-particle MLSMap keeps every grid it has made; selectActiveGrid only
 * changes which one is active (src/EmbodiedSlamFilter.cpp:195-207).  Here the window holds the
 * tiles around the particle and the trail the tiles it left: V entries {a, b, page} after the
 * row's S slots (page DM_LM_NONE: an empty entry).  A tile is never in both.  When the window
 * moves, (1) the tiles leaving it go to the trail in slot order, each into the first empty
 * entry, or -- the trail full -- in place of the entry farthest from the new centre (Chebyshev
 * distance in tiles; the first such entry) when that one is farther than the tile itself,
 * which is otherwise the one forgotten; (2) every trail entry whose tile lies inside the new
 * window goes back to its slot.  A returning tile is never the one forgotten: it lies within
 * the window's reach of the new centre, every leaving tile beyond it.  Forgotten tiles are
 * counted (map_tiles_evicted).                                                              */
static int lm_trail_find(const uint32_t* trail, uint32_t V, int64_t a, int64_t b)
{
    for (uint32_t e = 0; e < V; ++e) {
        const uint32_t* t = trail + 3 * e;
        if (t[2] != DM_LM_NONE && (int64_t)(int32_t)t[0] == a && (int64_t)(int32_t)t[1] == b) return (int)e;
    }
    return -1;
}

static int64_t lm_cheb(int64_t a, int64_t b, int64_t na, int64_t nb)
{
    const int64_t da = llabs(a - na), db = llabs(b - nb);
    return da > db ? da : db;
}

/* one tile into the trail; returns 1 when a tile was forgotten */
static uint32_t lm_trail_push(uint32_t* trail, uint32_t V, int32_t na, int32_t nb, int64_t a, int64_t b, uint32_t pg)
{
    int64_t far = -1;
    uint32_t fe = 0;
    for (uint32_t e = 0; e < V; ++e) {
        uint32_t* t = trail + 3 * e;
        if (t[2] == DM_LM_NONE) {
            t[0] = (uint32_t)(int32_t)a; t[1] = (uint32_t)(int32_t)b; t[2] = pg;
            return 0;
        }
        const int64_t d = lm_cheb((int32_t)t[0], (int32_t)t[1], na, nb);
        if (d > far) { far = d; fe = e; }
    }
    if (V && far > lm_cheb(a, b, na, nb)) {
        uint32_t* t = trail + 3 * fe;
        t[0] = (uint32_t)(int32_t)a; t[1] = (uint32_t)(int32_t)b; t[2] = pg;
    }
    return 1;
}

/* the window of row (S = wx * wy slots, then the trail) moves from ctr to (na, nb); returns
 * the tiles forgotten */
static uint32_t lm_recentre(uint32_t* row, int32_t* ctr, int32_t na, int32_t nb, uint32_t hx, uint32_t hy,
                            uint32_t wx, uint32_t wy, uint32_t V)
{
    const uint32_t S = wx * wy;
    uint32_t* trail = row + S;
    uint32_t forgot = 0;
    if (ctr[0] != DM_LM_UNSET) {
        for (uint32_t sb = 0; sb < wy; ++sb)           /* (1) the leaving tiles, slot order */
            for (uint32_t sa = 0; sa < wx; ++sa) {
                const int64_t a = dm_lm_tile_of(sa, ctr[0], hx, wx), b = dm_lm_tile_of(sb, ctr[1], hy, wy);
                if (llabs(a - (int64_t)na) <= (int64_t)hx && llabs(b - (int64_t)nb) <= (int64_t)hy) continue;
                uint32_t* e = &row[sa + wx * sb];
                if (*e == DM_LM_NONE) continue;
                forgot += lm_trail_push(trail, V, na, nb, a, b, *e);
                *e = DM_LM_NONE;
            }
        for (uint32_t e = 0; e < V; ++e) {              /* (2) the returning tiles */
            uint32_t* t = trail + 3 * e;
            const int64_t a = (int32_t)t[0], b = (int32_t)t[1];
            if (t[2] == DM_LM_NONE || llabs(a - (int64_t)na) > (int64_t)hx || llabs(b - (int64_t)nb) > (int64_t)hy) continue;
            row[(uint32_t)(a % wx) + wx * (uint32_t)(b % wy)] = t[2];
            t[2] = DM_LM_NONE;
        }
    }
    ctr[0] = na;
    ctr[1] = nb;
    return forgot;
}

/* the page of tile (a, b) in a particle's map: its slot when the tile is inside the window
 * centred at ctr, else its trail entry (DM_LM_NONE: the map does not hold it)              */
static uint32_t lm_tile_page(const uint32_t* row, const int32_t* ctr, uint32_t hx, uint32_t hy, uint32_t wx, uint32_t wy,
                             uint32_t V, uint32_t a, uint32_t b)
{
    if (ctr[0] == DM_LM_UNSET) return DM_LM_NONE;
    if (dm_lm_inside(a, ctr[0], hx, wx) && dm_lm_inside(b, ctr[1], hy, wy)) return row[(a % wx) + wx * (b % wy)];
    const int k = lm_trail_find(row + wx * wy, V, a, b);
    return k >= 0 ? row[wx * wy + 3 * k + 2] : DM_LM_NONE;
}

/* per-particle maps: GridAccess::get on the particle's own map = its own patch of the cell
 * when it holds one that passes the 3-sigma gate (its copy of a grid cell, or a cell the grid
 * leaves empty), else the shared grid's                                                    */
static int particle_map_fn(void* user, const double p[3], double q_mean, double q_var, double* mean, double* stdev)
{
    const or_pmap* pm = (const or_pmap*)user;
    const eslam_mls_grid* g = pm->g;
    const double* A = g->global2local;
    static const double id[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    int is_id = 1;
    for (int k = 0; k < 12; ++k) is_id &= A[k] == id[k];
    double lx = p[0], ly = p[1], lz = p[2];
    if (!is_id) {
        lx = ((A[0] * p[0] + A[1] * p[1]) + A[2] * p[2]) + A[3];
        ly = ((A[4] * p[0] + A[5] * p[1]) + A[6] * p[2]) + A[7];
        lz = ((A[8] * p[0] + A[9] * p[1]) + A[10] * p[2]) + A[11];
    }
    const double fm = floor((lx - g->offset_x) * (1.0 / g->scale_x));
    const double fn = floor((ly - g->offset_y) * (1.0 / g->scale_y));
    if (!(fm >= 0.0 && fm < (double)g->width && fn >= 0.0 && fn < (double)g->height)) return 0;
    const uint32_t m = (uint32_t)fm, n = (uint32_t)fn;
    const uint32_t a = m >> DM_LM_TILE_BITS, b = n >> DM_LM_TILE_BITS;
    const uint32_t pg = lm_tile_page(pm->slot, pm->ctr, pm->hx, pm->hy, pm->wx, pm->wy, pm->V, a, b);
    const uint32_t j = (m & 7u) + 8u * (n & 7u);
    if (pg != DM_LM_NONE && dm_lm_holds(lm_page(pm->blk, pg)->v[2 * j + 1])) {
        const float* v = lm_page(pm->blk, pg)->v;
        const double mm = (double)v[2 * j], sd = (double)v[2 * j + 1];
        const double diff = fabs(mm - lz);
        if (diff * diff < 9.0 * (sd * sd + q_var)) { *mean = mm; *stdev = sd; return 1; }
    }
    return or_mls_get_patch(g, p, q_mean, q_var, mean, stdev);
}

/* ========================================================================================
 * ContactModel
 * ====================================================================================== */
void or_cm_init(or_contact_model* cm, const eslam_config* cfg)
{
    memset(cm, 0, sizeof(*cm));
    cm->use_slip_update = cfg->use_slip_update;
    cm->use_shape_update = cfg->use_shape_update;
    cm->min_contacts = cfg->min_contacts;
    cm->correction = cfg->contact_likelihood_correction;
    cm->radius = cfg->contact_point_radius;
}

/* src/ContactModel.cpp:21-41 */
void or_cm_set_contact_points(or_contact_model* cm, uint32_t n, const eslam_contact_point* pts, const double q[4])
{
    double yc[4];
    remove_yaw(q, yc);
    cm->m = n;
    cm->nlow = 0;
    for (uint32_t i = 0; i < n; ++i) {
        q_rotate(yc, pts[i].position, cm->pos[i]);
        cm->contact[i] = pts[i].contact;
        cm->group[i] = pts[i].group_id;
    }
}

/* ContactModel::contactLikelihoodRatio  src/ContactModel.cpp:104-115 */
static double contact_likelihood_ratio(const or_contact_model* cm, double z, double sigma)
{
    if (cm->literal) {
        /* boost::math::normal n(0, sd): pdf = exp(-(z - 0)^2 / (2 sd^2)) / (sd sqrt(2 pi)),
         * cdf = erfc(-(z - 0) / (sd sqrt 2)) / 2  (boost/math/distributions/normal.hpp) */
        const double sd = sigma * cm->correction;
        double exponent = z * z;
        exponent /= -2.0 * sd * sd;
        const double pdf = exp(exponent) / (sd * 2.50662827463100050242);
        const double cdf = erfc(-(z / (sd * 1.41421356237309504880))) / 2.0;
        return pdf / cdf;
    }
    return dm_normal_pdf_cdf_ratio(z, sigma * cm->correction);
}

/* src/ContactModel.cpp:262-317 literally: d1 += zdiff / zvar, d2 += 1 / zvar, delta = d1 / d2,
 * pz *= exp(-(odiff^2) / 2) with odiff = (zdiff - delta) / sqrt(zvar) */
static void evaluate_weight_literal(or_contact_model* cm)
{
    double d1 = 0, d2 = 0;
    for (uint32_t i = 0; i < cm->ncp; ++i) {
        d1 += cm->cp[i].zdiff / cm->cp[i].zvar;
        d2 += 1.0 / cm->cp[i].zvar;
    }
    const double delta = d1 / d2;
    double pz = 1.0, s2 = 0.0;
    for (uint32_t i = 0; i < cm->ncp; ++i) {
        const double odiff = (cm->cp[i].zdiff - delta) / sqrt(cm->cp[i].zvar);
        const double zk = exp(-(odiff * odiff) / (2.0));
        if (cm->use_shape_update) pz *= zk;
        s2 += odiff * odiff;
    }
    cm->shape_s2 = s2;
    cm->weight = pz;
    cm->zdelta = -delta;
    cm->zvar = 1.0 / d2;
}

/* ContactModel::evaluateWeight  src/ContactModel.cpp:262-317, restated at the rounding
 * level: 1/zvar is formed once per point (d1 += zdiff * (1/zvar); odiff = (zdiff - delta) *
 * sqrt(1/zvar)) and the product of exp(-odiff^2 / 2) is one exp of the summed squares.
 * The sum is kept (shape_s2) so that m^(1/n) = exp(-s2 / (2 n)) needs no log.           */
static void evaluate_weight(or_contact_model* cm)
{
    if (cm->literal) { evaluate_weight_literal(cm); return; }
    /* src/ContactModel.cpp:262-317 with rounding-level restatements:
     * 1/zvar once per point, delta = d1 * (1/d2), odiff^2 = (zdiff - delta)^2 / zvar,
     * prod exp(-odiff^2 / 2) = exp(-s2 / 2) */
    double d1 = 0, d2 = 0;
    double iv[ESLAM_MAX_CONTACTS];
    for (uint32_t i = 0; i < cm->ncp; ++i) {
        iv[i] = 1.0 / cm->cp[i].zvar;
        d1 += cm->cp[i].zdiff * iv[i];
        d2 += iv[i];
    }
    const double inv_d2 = 1.0 / d2;
    const double delta = d1 * inv_d2;
    double s2 = 0.0;
    for (uint32_t i = 0; i < cm->ncp; ++i) {
        const double d = cm->cp[i].zdiff - delta;
        s2 += (d * d) * iv[i];
    }
    /* useSlipUpdate multiplies by p.prob, which is always 1 at push time (Q8) */
    cm->shape_s2 = s2;
    cm->weight = cm->use_shape_update ? dm_exp(-0.5 * s2) : 1.0;
    cm->zdelta = -delta;
    cm->zvar = inv_d2;
}

/* contactLikelihoodRatio(z, sigma) > 1e-9 guaranteed (exact-arithmetic bounds with a wide
 * margin), sigma^2 = zvar corr^2: for a group of ONE evaluated point the ratio cancels,
 * (zdiff*r)/r = zdiff, and is not evaluated (rounding-level restatement)                */
static int ratio_surely_significant(double z, double zvar, double corr)
{
    const double s2 = zvar * (corr * corr);
    if (z <= 0.0) return s2 < 1e16;                       /* ratio >= sqrt(2/pi)/s, s < 1e8   */
    return s2 < 1600.0 && z * z < 31.36 * s2;             /* s < 40, z < 5.6 s                */
}

/* ContactModel::evaluatePose  src/ContactModel.cpp:117-224 (group quirk Q7 kept) */
int or_cm_evaluate_pose(or_contact_model* cm, const double T[12], double meas_var, or_map_fn map, void* user)
{
    cm->ncp = 0;
    if (meas_var == 0) return -1;       /* the throw of src/ContactModel.cpp:122-123 */
    or_cpoint p = {{0, 0, 0}, INFINITY, INFINITY, 1.0};
    int valid = 0, group_valid = 1;
    const double contact_threshold = 0.2;
    double contact_ratio = 0, pose_var_avg = 0;
    cm->posevar = 0;
    for (uint32_t i = 0; i < cm->m; ++i) {
        const int32_t gid = cm->group[i];
        const double* c = cm->pos[i];
        double w[3];
        w[0] = ((T[0] * c[0] + T[1] * c[1]) + T[2] * c[2]) + T[3];
        w[1] = ((T[4] * c[0] + T[5] * c[1]) + T[6] * c[2]) + T[7];
        w[2] = ((T[8] * c[0] + T[9] * c[1]) + T[10] * c[2]) + T[11];
        w[0] = w[0] - 0.0;
        w[1] = w[1] - 0.0;
        w[2] = w[2] - cm->radius;
        const float cp = cm->contact[i];
        if (group_valid && !((double)cp < contact_threshold)) {
            double mean, stdev;
            if (map(user, w, w[2], meas_var, &mean, &stdev)) {
                const double zdiff = w[2] - mean;
                const double pose_var = cm->literal ? pow(stdev, 2) : stdev * stdev;
                const double zvar = (cm->literal ? pow(stdev, 2) : stdev * stdev) + meas_var;
                const double sq = sqrt(zvar);
                const int ends = (gid == -1 || i + 1 == cm->m || gid != cm->group[i + 1]);
                if (!cm->literal && !valid && ends && ratio_surely_significant(zdiff, zvar, cm->correction)) {
                    /* single-point group: push (zdiff, zvar) directly */
                    p.point[0] = w[0]; p.point[1] = w[1]; p.point[2] = mean;
                    p.zdiff = zdiff;
                    p.zvar = zvar;
                    p.prob = 1.0;
                    cm->posevar += pose_var;
                    cm->cp[cm->ncp++] = p;
                    group_valid = 1;
                    valid = 0;
                    pose_var_avg = 0;
                    contact_ratio = 0;
                    continue;
                }
                const double ratio = contact_likelihood_ratio(cm, zdiff, sq);
                if (!valid) {
                    p.point[0] = w[0]; p.point[1] = w[1]; p.point[2] = mean;
                    p.zdiff = zdiff * ratio;
                    p.zvar = zvar * ratio;
                    p.prob = 1.0;
                    contact_ratio = ratio;
                    pose_var_avg = pose_var * ratio;
                } else {
                    p.zdiff += zdiff * ratio;
                    p.zvar += zvar * ratio;
                    contact_ratio += ratio;
                    pose_var_avg += pose_var * ratio;
                }
                valid = 1;
            } else {
                group_valid = 0;
            }
        }
        if (valid && (gid == -1 || i + 1 == cm->m || gid != cm->group[i + 1])) {
            if (group_valid && contact_ratio > 1e-9) {
                if (cm->literal) {                /* src/ContactModel.cpp:201-203 */
                    p.zdiff /= contact_ratio;
                    p.zvar /= contact_ratio;
                    cm->posevar += pose_var_avg / contact_ratio;
                } else {
                    const double inv = 1.0 / contact_ratio;
                    p.zdiff *= inv;
                    p.zvar *= inv;
                    cm->posevar += pose_var_avg * inv;
                }
                cm->cp[cm->ncp++] = p;
                /* useSlipUpdate: p.prob *= matchTerrain(...) happens after the push (Q8) */
            }
            group_valid = 1;
            valid = 0;
            pose_var_avg = 0;
            contact_ratio = 0;
        }
    }
    if ((uint64_t)cm->ncp >= cm->min_contacts) {
        evaluate_weight(cm);
        return 1;
    }
    return 0;
}

/* src/ContactModel.cpp:319-340 (1-sigma gate, Q9) */
int or_cm_update_z(const or_contact_model* cm, double* z_pos, double* z_var)
{
    const double pose_var = cm->posevar / (double)cm->ncp;
    double a = *z_var - pose_var;
    double delta_var = (a < 1e-9) ? 1e-9 : a;         /* std::max(a, 1e-9) */
    const double z_delta = cm->zdelta;
    /* |z_delta / sqrt(delta_var)| > 1 (the "3-sigma" gate is 1 sigma, Q9), squared */
    if (cm->literal ? fabs(z_delta / sqrt(delta_var)) > 1.0 : z_delta * z_delta > delta_var) return 0;
    double gain = *z_var / (*z_var + cm->zvar);
    *z_pos += gain * z_delta;
    double var_gain = delta_var / (delta_var + cm->zvar);
    delta_var = (1.0 - var_gain) * delta_var;
    *z_var = pose_var + delta_var;
    return 1;
}

/* ContactModel::lowestPointHeuristic  src/ContactModel.cpp:48-79 */
static void lowest_point_heuristic(or_contact_model* cm, int update_probabilities)
{
    cm->nlow = 0;
    int gidx[ESLAM_MAX_CONTACTS];
    int ng = 0;
    for (uint32_t i = 0; i < cm->m; ++i) {
        if (cm->group[i] >= 0) {
            gidx[ng++] = (int)i;
            if (update_probabilities) cm->contact[i] = 0;
        }
        if (ng == 0) {
            memcpy(cm->low[cm->nlow++], cm->pos[i], sizeof(double) * 3);
        } else if (i + 1 == cm->m || cm->group[i + 1] != cm->group[i]) {
            /* std::sort of (z, index) pairs: lowest z, ties by index */
            int best = gidx[0];
            for (int k = 1; k < ng; ++k) {
                int c = gidx[k];
                if (cm->pos[c][2] < cm->pos[best][2] || (cm->pos[c][2] == cm->pos[best][2] && c < best)) best = c;
            }
            memcpy(cm->low[cm->nlow++], cm->pos[best], sizeof(double) * 3);
            if (update_probabilities) cm->contact[best] = 1;
            ng = 0;
        }
    }
}

uint32_t or_cm_lowest_points(or_contact_model* cm, double* out)
{
    if (cm->nlow == 0) lowest_point_heuristic(cm, 0);
    if (out) memcpy(out, cm->low, sizeof(double) * 3 * cm->nlow);
    return cm->nlow;
}

void or_cm_update_contact_state_lph(or_contact_model* cm) { lowest_point_heuristic(cm, 1); }

/* ========================================================================================
 * SurfaceHash pieces
 * ====================================================================================== */
/* Buckets<T>::bucketIndex  src/SurfaceHash.hpp:25-29 (dm_bucket_index) */
int or_bucket_index(int count, double min_val, double max_val, double value)
{
    return dm_bucket_index(count, min_val, max_val, value);
}

/* SurfaceParam::fromPoints  src/SurfaceHash.hpp:60-110 (dm_surface_param: pivoted LDL^T) */
void or_surface_param_from_points(const double* P, uint32_t n, double* slope_x, double* slope_y)
{
    dm_surface_param(P, n, slope_x, slope_y);
}

/* ========================================================================================
 * the filter
 * ====================================================================================== */
/* Particle state layout.  The default build keeps one array per field (SoA).  Built with
 * -DOR_AOS (oracle/_build/liboracle_aos.so, bench.py's second cpu_baseline figure only) the
 * state is one 288-byte record per particle, the size of the reference's PoseParticleGA
 * (src/PoseParticle.hpp:52-86 + src/PoseEstimator.hpp:108-117): x..mprob at doubles 0..6,
 * floating and ncp at bytes 56 and 57, the rest standing in for the reference's other
 * members (contact points, meas_pos, the map handle).  Every access goes through OD / OB,
 * and a resample copies whole records, as the reference's particle vector does
 * (src/ParticleFilter.hpp:85-108).  Results are identical in both layouts. */
#ifdef OR_AOS
#define OR_REC_BYTES 288u
#define OR_DSTRIDE (OR_REC_BYTES / 8u)
#define OR_BSTRIDE OR_REC_BYTES
#else
#define OR_DSTRIDE 1u
#define OR_BSTRIDE 1u
#endif
#define OD(i) ((uint64_t)(i) * OR_DSTRIDE)
#define OB(i) ((uint64_t)(i) * OR_BSTRIDE)

struct or_filter {
    eslam_config cfg;
    int sum_mode;
    uint64_t n;
    double *x, *y, *th, *z, *zs, *w, *mprob;   /* field views (strided records with OR_AOS) */
    uint8_t *floating, *ncp;
    void* rec;                                 /* OR_AOS: the record buffer the views point into */
    /* debug of the last updateWeights */
    uint32_t* dbg_ncp;
    or_cpoint* dbg_cp;
    double *dbg_zdelta, *dbg_zvar;
    /* environment */
    int has_map;
    eslam_mls_grid map;
    uint32_t* map_cells;
    float *map_mean, *map_stdev, *map_height;
    /* random state */
    uint32_t minstd;
    uint64_t project_count, init_count, hash_count;
    /* PoseEstimator members */
    double max_weight;
    double zcomp[4];
    int wexp;
    /* EmbodiedSlamFilter members */
    double ud_pose[12];
    /* last update */
    eslam_update_info info;
    uint32_t* anc;
    int has_anc;
    /* SurfaceHash (useHash): poses in sweep order, bucket lists (stable counting sort) */
    int has_hash;
    uint64_t hash_n;
    double *hash_x, *hash_y, *hash_th, *hash_z;
    int32_t* hash_bucket;
    uint32_t* hash_bstart;               /* bins^2 + 1 */
    uint32_t* hash_blist;
    dm_libc_rand_state libc;             /* rand() of SurfaceHash::sample (glibc, seed 1) */
    /* sharded mode (or_set_comm): this filter is shard [gbase, gbase + n) of n_global */
    int sharded;
    eslam_comm comm;
    uint64_t n_global, gbase;
    uint64_t gall[ESLAM_ORACLE_MAX_RANKS + 1];
    /* host threads of the per-particle loops (or_set_threads; 1 = the reference default,
     * USE_OPENMP off).  Results do not depend on it: the loops write per-particle outputs
     * only and every sum stays sequential or in the canonical chunk order. */
    int threads;
    int literal;                         /* or_set_literal */
    int debug;                           /* or_set_debug */
    /* per-particle maps (ESLAM_FLAG_PARTICLE_MAPS): each particle's window of tiles in cells
     * the shared grid leaves empty; sized from the map at set_map / init     */
    int lm_on;                           /* pm_ctr / pm_slot allocated for the current map    */
    uint32_t lm_hx, lm_hy, lm_wx, lm_wy, lm_S;
    uint32_t lm_V;                       /* trail entries per map (eslam_config::local_map_trail) */
    uint64_t lm_R;                       /* words per particle's row: S slots + V trail entries
                                            {a, b, page} (lm_row)                               */
    int32_t* pm_ctr;                     /* n x 2: window centre tile (DM_LM_UNSET: none)     */
    uint32_t* pm_slot;                   /* n rows of lm_R words: the S window slots (page index
                                            or DM_LM_NONE), then the trail       */
    or_page** pg_blk;                    /* OR_PAGE_BLOCKS block pointers                      */
    uint32_t pg_nblk;                    /* blocks allocated                                   */
    uint64_t pg_top;                     /* pages [0, pg_top) handed out at least once         */
    uint32_t* pg_free;                   /* free pages (the last map update's collection)      */
    uint64_t pg_nfree, pg_free_cap;
    uint64_t* pm_id;                     /* n: which map a particle holds (the resample copies the
                                            id with the map; a particle that changes a map it
                                            shares, or receives one from another rank, takes a
                                            fresh id): the sharing that the GPU's copy on write
                                            keeps (map_stores_copied) */
    uint64_t pm_fresh;                   /* the next fresh id (bit 63 | gbase << 32 | counter) */
};


/* global particle count: the N of every formula of the reference */
static uint64_t NG(const or_filter* f) { return f->sharded ? f->n_global : f->n; }

static int comm_allgather(or_filter* f, const void* send, void* recv, uint64_t bytes)
{
    return f->comm.allgather(f->comm.user, send, recv, bytes, NULL);
}

/* point the field views at a state buffer: one record per particle (OR_AOS) */
static void set_views(or_filter* f, void* rec)
{
    f->rec = rec;
#ifdef OR_AOS
    double* d = rec;
    f->x = d; f->y = d + 1; f->th = d + 2; f->z = d + 3; f->zs = d + 4; f->w = d + 5; f->mprob = d + 6;
    f->floating = (uint8_t*)rec + 56; f->ncp = (uint8_t*)rec + 57;
#endif
}

static void free_state(or_filter* f)
{
#ifdef OR_AOS
    free(f->rec);
#else
    free(f->x); free(f->y); free(f->th); free(f->z); free(f->zs); free(f->w); free(f->mprob);
    free(f->floating); free(f->ncp);
#endif
    f->rec = NULL;
}

/* strided copies between the caller's field arrays and the state */
static void put_d(double* dst, const double* src, uint64_t n)
{
    if (OR_DSTRIDE == 1) { memcpy(dst, src, n * 8); return; }
    for (uint64_t i = 0; i < n; ++i) dst[OD(i)] = src[i];
}
static void get_d(double* dst, const double* src, uint64_t n)
{
    if (OR_DSTRIDE == 1) { memcpy(dst, src, n * 8); return; }
    for (uint64_t i = 0; i < n; ++i) dst[i] = src[OD(i)];
}
static void put_b(uint8_t* dst, const uint8_t* src, uint64_t n)
{
    if (OR_BSTRIDE == 1) { memcpy(dst, src, n); return; }
    for (uint64_t i = 0; i < n; ++i) dst[OB(i)] = src[i];
}
static void get_b(uint8_t* dst, const uint8_t* src, uint64_t n)
{
    if (OR_BSTRIDE == 1) { memcpy(dst, src, n); return; }
    for (uint64_t i = 0; i < n; ++i) dst[i] = src[OB(i)];
}

/* ---- per-particle local maps: storage ------------------------------------------------- */
static void lm_free(or_filter* f)
{
    free(f->pm_ctr); free(f->pm_slot); free(f->pm_id);
    f->pm_ctr = NULL; f->pm_slot = NULL; f->pm_id = NULL;
    if (f->pg_blk) {
        for (uint32_t k = 0; k < f->pg_nblk; ++k) free(f->pg_blk[k]);
        free(f->pg_blk);
    }
    free(f->pg_free);
    f->pg_blk = NULL; f->pg_nblk = 0; f->pg_top = 0;
    f->pg_free = NULL; f->pg_nfree = f->pg_free_cap = 0;
    f->lm_on = 0;
}

/* every particle's map empty, sized for the current map (none yet: nothing until set_map) */
static int lm_reset(or_filter* f)
{
    lm_free(f);
    if (!(f->cfg.flags & ESLAM_FLAG_PARTICLE_MAPS) || !f->has_map || !f->n) return 0;
    f->lm_hx = dm_lm_half(f->cfg.max_sensor_range, f->map.scale_x);
    f->lm_hy = dm_lm_half(f->cfg.max_sensor_range, f->map.scale_y);
    f->lm_wx = 2 * f->lm_hx + 1;
    f->lm_wy = 2 * f->lm_hy + 1;
    f->lm_S = f->lm_wx * f->lm_wy;
    f->lm_V = f->cfg.local_map_trail;
    f->lm_R = (uint64_t)f->lm_S + 3ull * f->lm_V;
    const uint64_t n = f->n;
    f->pm_ctr = malloc(n * 2 * sizeof(int32_t));
    f->pm_slot = malloc(n * f->lm_R * sizeof(uint32_t));
    f->pm_id = malloc(n * 8);
    f->pg_blk = calloc(OR_PAGE_BLOCKS, sizeof(or_page*));
    if (!f->pm_ctr || !f->pm_slot || !f->pm_id || !f->pg_blk) return ESLAM_ERR_OUT_OF_MEMORY;
    for (uint64_t i = 0; i < 2 * n; ++i) f->pm_ctr[i] = DM_LM_UNSET;
    memset(f->pm_slot, 0xff, n * f->lm_R * sizeof(uint32_t));
    for (uint64_t i = 0; i < n; ++i) f->pm_id[i] = f->gbase + i;
    f->pm_fresh = (1ull << 63) | ((uint64_t)f->gbase << 32);
    f->lm_on = 1;
    return 0;
}

/* a page for a map update's write: a free one, else a new one (called by one thread at a time) */
static uint32_t lm_alloc(or_filter* f)
{
    if (f->pg_nfree) return f->pg_free[--f->pg_nfree];
    const uint64_t p = f->pg_top;
    const uint32_t blk = (uint32_t)(p >> OR_PAGE_BLOCK_BITS);
    if (blk >= OR_PAGE_BLOCKS) return DM_LM_NONE;
    if (blk >= f->pg_nblk) {
        f->pg_blk[blk] = malloc(sizeof(or_page) << OR_PAGE_BLOCK_BITS);
        if (!f->pg_blk[blk]) return DM_LM_NONE;
        f->pg_nblk = blk + 1;
    }
    f->pg_top = p + 1;
    return (uint32_t)p;
}

static or_page* lm_pg(or_filter* f, uint32_t p)
{
    return f->pg_blk[p >> OR_PAGE_BLOCK_BITS] + (p & ((1u << OR_PAGE_BLOCK_BITS) - 1u));
}

static void or_free_particles(or_filter* f)
{
    free_state(f);
    free(f->anc);
    free(f->dbg_ncp); free(f->dbg_cp); free(f->dbg_zdelta); free(f->dbg_zvar);
    lm_free(f);
    f->x = f->y = f->th = f->z = f->zs = f->w = f->mprob = NULL;
    f->floating = f->ncp = NULL;
    f->anc = NULL;
    f->dbg_ncp = NULL; f->dbg_cp = NULL; f->dbg_zdelta = f->dbg_zvar = NULL;
    f->n = 0;
}

static int or_alloc_particles(or_filter* f, uint64_t n)
{
    if (f->sharded && n != f->gall[f->comm.rank + 1] - f->gall[f->comm.rank]) return ESLAM_ERR_INVALID_ARG;
    or_free_particles(f);
    f->n = n;
    size_t b = (size_t)(n ? n : 1);
#ifdef OR_AOS
    set_views(f, calloc(b, OR_REC_BYTES));
    if (!f->rec) return ESLAM_ERR_OUT_OF_MEMORY;
#else
    f->x = calloc(b, 8); f->y = calloc(b, 8); f->th = calloc(b, 8); f->z = calloc(b, 8);
    f->zs = calloc(b, 8); f->w = calloc(b, 8); f->mprob = calloc(b, 8);
    f->floating = calloc(b, 1); f->ncp = calloc(b, 1);
#endif
    f->anc = calloc(b, 4);
    if (f->debug) {
        f->dbg_ncp = calloc(b, 4);
        f->dbg_cp = calloc(b * ESLAM_MAX_CONTACTS, sizeof(or_cpoint));
        f->dbg_zdelta = calloc(b, 8); f->dbg_zvar = calloc(b, 8);
        if (!f->dbg_cp) return ESLAM_ERR_OUT_OF_MEMORY;
    }
    if (lm_reset(f)) return ESLAM_ERR_OUT_OF_MEMORY;    /* every particle's map: still empty */
    f->has_anc = 0;
    return f->x ? 0 : ESLAM_ERR_OUT_OF_MEMORY;
}

or_filter* or_create(const eslam_config* cfg, int sum_mode)
{
    or_filter* f = calloc(1, sizeof(or_filter));
    f->cfg = *cfg;
    f->sum_mode = sum_mode;
    f->threads = 1;
    f->minstd = dm_minstd_seed(cfg->seed);      /* ParticleFilter(seed) src/ParticleFilter.hpp:24-27 */
    dm_libc_srand(&f->libc, 1);                 /* the reference never calls srand() */
    f->max_weight = 0;                          /* src/PoseEstimator.cpp:13-25 */
    f->zcomp[0] = 1.0;
    f->wexp = 1;
    set_translation_pose(f->ud_pose, 1000, 0, 0);
    return f;
}

void or_set_threads(or_filter* f, int threads) { f->threads = threads > 1 ? threads : 1; }

void or_set_literal(or_filter* f, int literal) { f->literal = literal ? 1 : 0; }

void or_set_debug(or_filter* f, int on)
{
    f->debug = on ? 1 : 0;
    if (f->debug && f->n && !f->dbg_ncp) {
        const size_t b = (size_t)f->n;
        f->dbg_ncp = calloc(b, 4);
        f->dbg_cp = calloc(b * ESLAM_MAX_CONTACTS, sizeof(or_cpoint));
        f->dbg_zdelta = calloc(b, 8); f->dbg_zvar = calloc(b, 8);
    }
}

/* sin and cos of a particle angle: the contract's dm_sincos, or libm (Eigen's Rotation2D /
 * AngleAxis call std::sin / std::cos) in literal mode */
static void or_sincos(const or_filter* f, double a, double* s, double* c)
{
    if (f->literal) { *s = sin(a); *c = cos(a); }
    else dm_sincos(a, s, c);
}

/* std::pow in literal mode, the contract's dm_pow otherwise */
static double or_pow(const or_filter* f, double x, double y) { return f->literal ? pow(x, y) : dm_pow(x, y); }

void or_destroy(or_filter* f)
{
    if (!f) return;
    or_free_particles(f);
    free(f->map_cells); free(f->map_mean); free(f->map_stdev); free(f->map_height);
    free(f->hash_x); free(f->hash_y); free(f->hash_th); free(f->hash_z); free(f->hash_bucket);
    free(f->hash_bstart); free(f->hash_blist);
    free(f);
}

int or_set_map(or_filter* f, const eslam_mls_grid* g)
{
    uint64_t ncell = (uint64_t)g->width * g->height;
    free(f->map_cells); free(f->map_mean); free(f->map_stdev); free(f->map_height);
    f->map = *g;
    f->map_cells = malloc((ncell + 1) * 4);
    memcpy(f->map_cells, g->cell_start, (ncell + 1) * 4);
    size_t np = (size_t)(g->n_patches ? g->n_patches : 1);
    f->map_mean = malloc(np * 4); f->map_stdev = malloc(np * 4);
    memcpy(f->map_mean, g->patch_mean, g->n_patches * 4);
    memcpy(f->map_stdev, g->patch_stdev, g->n_patches * 4);
    f->map_height = NULL;
    if (g->patch_height) { f->map_height = malloc(np * 4); memcpy(f->map_height, g->patch_height, g->n_patches * 4); }
    f->map.cell_start = f->map_cells;
    f->map.patch_mean = f->map_mean;
    f->map.patch_stdev = f->map_stdev;
    f->map.patch_height = f->map_height;
    f->has_map = 1;
    /* the particles' own maps name cells of the previous grid: they start over, empty */
    return lm_reset(f);
}

uint64_t or_count(const or_filter* f) { return f->n; }

/* PoseEstimator::init(N, mu, sigma, zpos, zsigma)  src/PoseEstimator.cpp:88-102, with
 * samplePose2D (src/PoseEstimator.cpp:64-73) drawing its 3 normals from the INIT stream. */
int or_init_gaussian(or_filter* f, uint64_t n, const double mu[3], const double sigma[3], double zpos, double zsigma)
{
    int rc = or_alloc_particles(f, n);
    if (rc) return rc;
    for (uint64_t i = 0; i < n; ++i) {
        dm_philox_ctr d0 = dm_draw(f->cfg.seed, DM_STREAM_INIT, f->init_count, f->gbase + i, 0);
        double n0, n1, n2, n3;
        dm_box_muller32(d0.v[0], d0.v[1], &n0, &n1);
        dm_box_muller32(d0.v[2], d0.v[3], &n2, &n3);
        f->x[OD(i)] = n0 * sigma[0] + mu[0];
        f->y[OD(i)] = n1 * sigma[1] + mu[1];
        f->th[OD(i)] = n2 * sigma[2] + mu[2];
        f->z[OD(i)] = zpos;
        f->zs[OD(i)] = zsigma;
        f->w[OD(i)] = 0;            /* PoseParticle ctor: weight(0), Q3 */
        f->mprob[OD(i)] = 0;
        f->floating[OB(i)] = 1;
        f->ncp[OB(i)] = 0;
    }
    f->init_count++;
    f->wexp = 1;
    return 0;
}

/* EmbodiedSlamFilter::init(env, pose) non-hash branch  src/EmbodiedSlamFilter.cpp:109-128:
 * angle = eulerAngles(2,1,0)[0] (Eigen >= 3.3 folds it into [0, pi]), sigma from config,
 * zsigma = initialTranslationError.z + 1e-3, udPose = Translation(1000,0,0).            */
int or_init_pose(or_filter* f, const double pos[3], const double q[4])
{
    double R[9];
    q_to_mat(q, R);
    double angle = atan2(R[3], R[0]);
    if (angle < 0.0) angle += M_PI;
    double mu[3] = {pos[0], pos[1], angle};
    double sg[3] = {f->cfg.initial_translation_error[0], f->cfg.initial_translation_error[1],
                    f->cfg.initial_rotation_error[2]};
    uint64_t n = f->cfg.particle_count;
    if (f->sharded) n = f->gall[f->comm.rank + 1] - f->gall[f->comm.rank];
    int rc;
    if (f->cfg.hash_use) {                 /* hash.create(gridTemplate); filter.init(N, &hash) */
        rc = f->has_hash ? 0 : or_hash_create(f);
        if (!rc) rc = or_init_hash(f, n);
    } else {
        rc = or_init_gaussian(f, n, mu, sg, pos[2], f->cfg.initial_translation_error[2] + 1e-3);
    }
    set_translation_pose(f->ud_pose, 1000, 0, 0);
    return rc;
}

int or_upload(or_filter* f, uint64_t n, const eslam_particles* p)
{
    int rc = or_alloc_particles(f, n);
    if (rc) return rc;
    put_d(f->x, p->x, n); put_d(f->y, p->y, n); put_d(f->th, p->orientation, n);
    put_d(f->z, p->zpos, n); put_d(f->zs, p->zsigma, n); put_d(f->w, p->weight, n);
    if (p->mprob) put_d(f->mprob, p->mprob, n);
    if (p->floating) put_b(f->floating, p->floating, n);
    if (p->n_contact_points) put_b(f->ncp, p->n_contact_points, n);
    double mx = 0;
    for (uint64_t i = 0; i < n; ++i) if (f->w[OD(i)] > mx) mx = f->w[OD(i)];
    if (f->sharded) {
        double all[ESLAM_ORACLE_MAX_RANKS];
        if (comm_allgather(f, &mx, all, 8)) return ESLAM_ERR_COMM;
        for (int r = 0; r < f->comm.nranks; ++r) if (all[r] > mx) mx = all[r];
    }
    f->wexp = dm_weight_exp(mx);
    return 0;
}

int or_download(or_filter* f, eslam_particles* p)
{
    uint64_t n = f->n;
    if (p->x) get_d(p->x, f->x, n);
    if (p->y) get_d(p->y, f->y, n);
    if (p->orientation) get_d(p->orientation, f->th, n);
    if (p->zpos) get_d(p->zpos, f->z, n);
    if (p->zsigma) get_d(p->zsigma, f->zs, n);
    if (p->weight) get_d(p->weight, f->w, n);
    if (p->mprob) get_d(p->mprob, f->mprob, n);
    if (p->floating) get_b(p->floating, f->floating, n);
    if (p->n_contact_points) get_b(p->n_contact_points, f->ncp, n);
    return 0;
}

/* ---- per-step host preparation ------------------------------------------------------------ */
typedef struct {
    double yaw, zcomp[4], z_delta, z_var;
    double mu[3], L[9];
} or_prep;

static void lower_cholesky(const double S[9], double L[9])
{
    memset(L, 0, 9 * sizeof(double));
    for (int j = 0; j < 3; ++j) {
        double d = S[j * 3 + j];
        for (int k = 0; k < j; ++k) d -= L[j * 3 + k] * L[j * 3 + k];
        double ljj = d > 0.0 ? sqrt(d) : 0.0;
        L[j * 3 + j] = ljj;
        for (int i = j + 1; i < 3; ++i) {
            double s = S[i * 3 + j];
            for (int k = 0; k < j; ++k) s -= L[i * 3 + k] * L[j * 3 + k];
            L[i * 3 + j] = ljj > 0.0 ? s / ljj : 0.0;
        }
    }
}

/* src/PoseEstimator.cpp:186-192 */
static void or_prepare(const eslam_step_input* in, or_prep* p)
{
    const double* q = in->body2odometry_rot;
    p->yaw = get_yaw(q);
    remove_yaw(q, p->zcomp);
    double R[9];
    q_to_mat(q, R);
    const double* t = in->pose_delta_trans;
    p->z_delta = (R[6] * t[0] + R[7] * t[1]) + R[8] * t[2];
    p->z_var = in->position_error_zz * 2.0;
    for (int i = 0; i < 3; ++i) p->mu[i] = in->sample_mean[i];
    lower_cholesky(in->sample_cov, p->L);
}


/* ---- SurfaceHash  src/SurfaceHash.hpp:155-231 --------------------------------------------- */
static void hash_grid_view(const or_filter* f, dm_hash_grid* g)
{
    memset(g, 0, sizeof(*g));
    g->cell_start = f->map.cell_start;
    g->mean = f->map.patch_mean;
    g->mean_stride = 1;
    g->width = f->map.width;
    g->height = f->map.height;
    g->bins = (uint32_t)f->cfg.hash_slope_bins;
    g->scale_x = f->map.scale_x; g->scale_y = f->map.scale_y;
    g->offset_x = f->map.offset_x; g->offset_y = f->map.offset_y;
    g->inv_scale_x = 1.0 / f->map.scale_x; g->inv_scale_y = 1.0 / f->map.scale_y;
    dm_affine_inverse(f->map.global2local, g->g2w);
}

int or_hash_create(or_filter* f)
{
    if (!f->has_map) return ESLAM_ERR_NO_MLS_GRID;
    free(f->hash_x); free(f->hash_y); free(f->hash_th); free(f->hash_z); free(f->hash_bucket);
    free(f->hash_bstart); free(f->hash_blist);
    dm_hash_grid g;
    hash_grid_view(f, &g);
    const uint32_t steps = (uint32_t)f->cfg.hash_angular_steps, bins = g.bins;
    double* pts = malloc(sizeof(double) * 8 * (steps ? steps : 1));
    double* orient = malloc(sizeof(double) * (steps ? steps : 1));
    dm_hash_segments(steps, g.g2w, pts, orient);
    uint64_t cap = 1024, n = 0;
    f->hash_x = malloc(cap * 8); f->hash_y = malloc(cap * 8); f->hash_th = malloc(cap * 8); f->hash_z = malloc(cap * 8);
    f->hash_bucket = malloc(cap * 4);
    for (uint32_t a = 0; a < steps; ++a)
        for (uint32_t m = 0; m < g.width; ++m)
            for (uint32_t nn = 0; nn < g.height; ++nn) {
                double pose[4];
                const int b = dm_hash_item(&g, pts + 8 * a, orient[a], m, nn, pose);
                if (b < 0) continue;
                if (n == cap) {
                    cap *= 2;
                    f->hash_x = realloc(f->hash_x, cap * 8); f->hash_y = realloc(f->hash_y, cap * 8);
                    f->hash_th = realloc(f->hash_th, cap * 8); f->hash_z = realloc(f->hash_z, cap * 8);
                    f->hash_bucket = realloc(f->hash_bucket, cap * 4);
                }
                f->hash_x[n] = pose[0]; f->hash_y[n] = pose[1]; f->hash_th[n] = pose[2]; f->hash_z[n] = pose[3];
                f->hash_bucket[n] = b;
                ++n;
            }
    free(pts); free(orient);
    const uint32_t nb = bins * bins;
    f->hash_bstart = calloc(nb + 1, 4);
    for (uint64_t i = 0; i < n; ++i) f->hash_bstart[f->hash_bucket[i] + 1]++;
    for (uint32_t b = 0; b < nb; ++b) f->hash_bstart[b + 1] += f->hash_bstart[b];
    f->hash_blist = malloc((n ? n : 1) * 4);
    uint32_t* fill = malloc((nb ? nb : 1) * 4);
    memcpy(fill, f->hash_bstart, nb * 4);
    for (uint64_t i = 0; i < n; ++i) f->hash_blist[fill[f->hash_bucket[i]]++] = (uint32_t)i;   /* sweep order */
    free(fill);
    f->hash_n = n;
    f->has_hash = 1;
    return 0;
}

uint64_t or_hash_info(or_filter* f, uint32_t* bucket_sizes)
{
    if (!f->has_hash) return 0;
    const uint32_t nb = (uint32_t)f->cfg.hash_slope_bins * (uint32_t)f->cfg.hash_slope_bins;
    if (bucket_sizes)
        for (uint32_t b = 0; b < nb; ++b) bucket_sizes[b] = f->hash_bstart[b + 1] - f->hash_bstart[b];
    return f->hash_n;
}

int or_hash_poses(or_filter* f, double* x, double* y, double* th, double* z, int32_t* bucket)
{
    if (!f->has_hash) return ESLAM_ERR_NOT_INITIALISED;
    const uint64_t n = f->hash_n;
    if (x) memcpy(x, f->hash_x, n * 8);
    if (y) memcpy(y, f->hash_y, n * 8);
    if (th) memcpy(th, f->hash_th, n * 8);
    if (z) memcpy(z, f->hash_z, n * 8);
    if (bucket) memcpy(bucket, f->hash_bucket, n * 4);
    return 0;
}

/* PoseEstimator::init(N, hash)  src/PoseEstimator.cpp:75-86: particle i = poses[rand() %
 * size]; PoseParticle(position, orientation, zPos) defaults: zSigma 0, weight 0, floating
 * (mprob is uninitialised in the reference; 0 here) */
int or_init_hash(or_filter* f, uint64_t n)
{
    if (!f->has_hash || f->hash_n == 0) return ESLAM_ERR_HASH_SAMPLE;
    int rc = or_alloc_particles(f, n);
    if (rc) return rc;
    const uint64_t skip = f->gbase, total = f->sharded ? f->n_global : n;
    for (uint64_t g = 0; g < total; ++g) {
        const uint32_t idx = (uint32_t)((uint64_t)(uint32_t)dm_libc_rand(&f->libc) % f->hash_n);
        if (g < skip || g >= skip + n) continue;
        const uint64_t i = g - skip;
        f->x[OD(i)] = f->hash_x[idx]; f->y[OD(i)] = f->hash_y[idx]; f->th[OD(i)] = f->hash_th[idx]; f->z[OD(i)] = f->hash_z[idx];
        f->zs[OD(i)] = 0.0; f->w[OD(i)] = 0.0; f->mprob[OD(i)] = 0.0; f->floating[OB(i)] = 1; f->ncp[OB(i)] = 0;
    }
    f->wexp = 1;
    return 0;
}

typedef struct { float w; uint32_t i; } or_widx;

static int widx_cmp(const void* a, const void* b)
{
    const or_widx* x = (const or_widx*)a;
    const or_widx* y = (const or_widx*)b;
    if (x->w < y->w) return -1;
    if (y->w < x->w) return 1;
    return x->i < y->i ? -1 : (x->i > y->i);
}

/* PoseEstimator::sampleFromHash  src/PoseEstimator.cpp:130-182 */
static void sample_from_hash(or_filter* f, const eslam_step_input* in)
{
    /* contactModel.setContactPoints + getLowestPointPerGroup: yaw-compensated feet */
    double pos[ESLAM_MAX_CONTACTS * 3], low[ESLAM_MAX_CONTACTS * 3];
    int32_t grp[ESLAM_MAX_CONTACTS];
    const uint32_t m = in->n_contacts < ESLAM_MAX_CONTACTS ? in->n_contacts : ESLAM_MAX_CONTACTS;
    for (uint32_t i = 0; i < m; ++i) {
        q_rotate(f->zcomp, in->contacts[i].position, pos + 3 * i);
        grp[i] = in->contacts[i].group_id;
    }
    const uint32_t nlow = dm_lowest_points(pos, grp, m, low);
    double sx, sy;
    dm_surface_param(low, nlow, &sx, &sy);
    const int bins = (int)f->cfg.hash_slope_bins;
    const int b = dm_bucket_index(bins, -1.0, 1.0, sx) * bins + dm_bucket_index(bins, -1.0, 1.0, sy);
    const uint32_t bsize = f->hash_bstart[b + 1] - f->hash_bstart[b];
    const double rel = dm_pow(1.0 - 1.0 * (double)bsize / (double)f->hash_n, 3.0);
    const uint64_t N = NG(f);
    uint64_t k = (uint64_t)(((double)N * f->cfg.hash_percentage) * rel);
    if (rel < 0.8) k = 0;
    if (k > N) k = N;
    if (k == 0 || bsize == 0) return;      /* nothing replaced, no rand() drawn */
    const double weight = ((or_get_weights_sum(f) / (double)N) * f->cfg.hash_avg_factor) * rel;
    /* (float weight, global index) of every particle; sharded: all ranks' pairs, gathered
     * in rank order, so every rank sorts the one-filter list and replaces what it holds   */
    or_widx* wi = malloc(sizeof(or_widx) * (f->n ? f->n : 1));
    for (uint64_t i = 0; i < f->n; ++i) {
        float wf = (float)f->w[OD(i)];
        if (wf == 0.0f) wf = 0.0f;                /* -0 and +0 compare equal */
        wi[i].w = wf;
        wi[i].i = (uint32_t)(f->gbase + i);
    }
    or_widx* all = wi;
    uint64_t total = f->n;
    if (f->sharded) {
        const int G = f->comm.nranks;
        uint64_t maxn = 1;
        for (int r = 0; r < G; ++r) {
            const uint64_t nr = f->gall[r + 1] - f->gall[r];
            maxn = nr > maxn ? nr : maxn;
        }
        or_widx* pad = calloc(maxn, sizeof(or_widx));
        memcpy(pad, wi, f->n * sizeof(or_widx));
        or_widx* g = malloc((size_t)G * maxn * sizeof(or_widx));
        comm_allgather(f, pad, g, maxn * sizeof(or_widx));
        all = malloc((size_t)N * sizeof(or_widx));
        total = 0;
        for (int r = 0; r < G; ++r) {
            const uint64_t nr = f->gall[r + 1] - f->gall[r];
            memcpy(all + total, g + (uint64_t)r * maxn, nr * sizeof(or_widx));
            total += nr;
        }
        free(pad);
        free(g);
    }
    qsort(all, total, sizeof(or_widx), widx_cmp);
    for (uint64_t j = 0; j < k; ++j) {
        const uint32_t draw = (uint32_t)((uint64_t)(uint32_t)dm_libc_rand(&f->libc) % bsize);
        const uint32_t src = f->hash_blist[f->hash_bstart[b] + draw];
        const uint64_t gi = all[j].i;
        if (gi < f->gbase || gi >= f->gbase + f->n) continue;
        const uint64_t i = gi - f->gbase;
        f->x[OD(i)] = f->hash_x[src]; f->y[OD(i)] = f->hash_y[src]; f->th[OD(i)] = f->hash_th[src]; f->z[OD(i)] = f->hash_z[src];
        f->zs[OD(i)] = 0.5;
        f->floating[OB(i)] = 1;
        f->w[OD(i)] = weight;
    }
    if (all != wi) free(all);
    free(wi);
}

/* ---- project  src/PoseEstimator.cpp:184-242 --------------------------------------------- */
int or_project(or_filter* f, const eslam_step_input* in)
{
    if (!f->n) return ESLAM_ERR_NOT_INITIALISED;
    or_prep pp;
    or_prepare(in, &pp);
    memcpy(f->zcomp, pp.zcomp, sizeof(pp.zcomp));
    const eslam_config* c = &f->cfg;
    double spread = dm_weighting_function(f->max_weight, 0.0, c->spread_threshold, 0.0);
    int do_spread = spread > 0 && !c->hash_use;
    const double tf = c->spread_translation_factor * spread;
    const double rf = c->spread_rotation_factor * spread;
    const double* L = pp.L;
    const int64_t n = (int64_t)f->n;
#pragma omp parallel for schedule(static) num_threads(f->threads) if (f->threads > 1)
    for (int64_t i = 0; i < n; ++i) {
        double z0, z1, z2, sn0, sn1 = 0, sn2 = 0;
        const uint64_t gi = f->gbase + i;
        /* draw layout: call 0 -> Box-Muller pairs (z0, z1), (z2, sn0); call 1 -> slip test,
         * slip factor, spread pair (sn1, sn2)  (the odometry sampler and rand_uni/rand_norm
         * of src/PoseEstimator.cpp:198-236, restated on Philox) */
        dm_philox_ctr d0 = dm_draw(c->seed, DM_STREAM_PROJECT, f->project_count, gi, 0);
        dm_philox_ctr d1 = dm_draw(c->seed, DM_STREAM_PROJECT, f->project_count, gi, 1);
        dm_box_muller32(d0.v[0], d0.v[1], &z0, &z1);
        dm_box_muller32(d0.v[2], d0.v[3], &z2, &sn0);
        /* odometry.getPoseDeltaSample2D(): mu + L z */
        double dx = pp.mu[0] + L[0] * z0;
        double dy = pp.mu[1] + (L[3] * z0 + L[4] * z1);
        double dth = pp.mu[2] + ((L[6] * z0 + L[7] * z1) + L[8] * z2);
        const double u_slip = dm_u32(d1.v[0]);
        if (u_slip < c->slip_factor) dy *= dm_u32(d1.v[1]);
        double s, co;
        or_sincos(f, f->th[OD(i)], &s, &co);
        f->x[OD(i)] += co * dx - s * dy;
        f->y[OD(i)] += s * dx + co * dy;
        f->th[OD(i)] += dth;
        if (c->max_yaw_deviation > 0.0) {
            if (fabs(f->th[OD(i)] - pp.yaw) > c->max_yaw_deviation) f->w[OD(i)] *= 0.7;
        }
        f->z[OD(i)] += pp.z_delta;
        f->zs[OD(i)] = sqrt(f->zs[OD(i)] * f->zs[OD(i)] + pp.z_var);
        if (do_spread) {
            dm_box_muller32(d1.v[2], d1.v[3], &sn1, &sn2);
            f->x[OD(i)] += sn0 * tf + 0.0;
            f->y[OD(i)] += sn1 * tf + 0.0;
            f->th[OD(i)] += sn2 * rf + 0.0;
        }
    }
    f->project_count++;
    /* the static counter of src/PoseEstimator.cpp:239 (per filter here, Q11): the hash
     * respawn runs on the first project and every period-th after it */
    if (c->hash_use && f->has_hash) {
        const uint64_t period = c->hash_period ? c->hash_period : 1;
        if ((f->hash_count++ % period) == 0) sample_from_hash(f, in);
    }
    return 0;
}

/* ---- canonical chunk reduction ------------------------------------------------------------ */
typedef struct or_acc_s { uint64_t L[4]; uint32_t nan, inf; } or_acc;

/* exact cross-rank sum of k accumulators (limb sums, NaN/inf flags) */
static int combine_accs(or_filter* f, or_acc* a, int k)
{
    if (!f->sharded) return 0;
    const int G = f->comm.nranks;
    or_acc* all = malloc(sizeof(or_acc) * (size_t)k * (size_t)G);
    if (comm_allgather(f, a, all, sizeof(or_acc) * (uint64_t)k)) { free(all); return ESLAM_ERR_COMM; }
    memset(a, 0, sizeof(or_acc) * (size_t)k);
    for (int r = 0; r < G; ++r)
        for (int q = 0; q < k; ++q) {
            const or_acc* s = &all[r * k + q];
            for (int j = 0; j < 4; ++j) a[q].L[j] += s->L[j];
            a[q].nan |= s->nan;
            a[q].inf |= s->inf;
        }
    free(all);
    return 0;
}

static void acc_add_chunk(or_acc* a, double v, int scale)
{
    if (v != v) { a->nan = 1; return; }
    if (!dm_isfinite(v)) { a->inf = 1; return; }
    uint32_t l[4];
    dm_fx128_limbs(v, scale, l);
    for (int j = 0; j < 4; ++j) a->L[j] += l[j];
}

static double acc_value(const or_acc* a, int scale)
{
    if (a->nan) return NAN;
    if (a->inf) return INFINITY;
    return dm_limbs_to_double(a->L, scale);
}

/* the 64-lane xor butterfly of the device, lane 0's result */
static double butterfly64(double* v)
{
    double t[64];
    for (int o = 32; o >= 1; o >>= 1) {
        for (int l = 0; l < 64; ++l) t[l] = v[l] + v[l ^ o];
        memcpy(v, t, sizeof(t));
    }
    return v[0];
}

/* chunk sums of vals[i] restricted to sel(i) (bucket match), accumulated into acc */
/* vstride: element stride of vals (OR_DSTRIDE for the state's weights) */
static void chunk_reduce(const double* vals, uint64_t vstride, const uint8_t* bucket, int want_bucket,
                         uint64_t n, uint32_t J, or_acc* acc, int scale)
{
    const uint64_t csz = 64ull * J;
    for (uint64_t c0 = 0; c0 < n; c0 += csz) {
        double lane[64];
        for (int s = 0; s < 64; ++s) {
            double a = 0.0;
            for (uint32_t j = 0; j < J; ++j) {
                uint64_t i = c0 + 64ull * j + (uint64_t)s;
                if (i >= n) continue;
                double v = (bucket == NULL || (int)bucket[i] == want_bucket) ? vals[i * vstride] : 0.0;
                a = a + v;
            }
            lane[s] = a;
        }
        acc_add_chunk(acc, butterfly64(lane), scale);
    }
}

/* ---- updateWeights  src/PoseEstimator.cpp:257-352 ----------------------------------------- */
typedef struct {
    double fw, f[DM_NBUCKETS];
    double S, Q;          /* contract: sum of final weights and of their squares */
} or_phase;

static int or_update_weights(or_filter* f, const eslam_step_input* in, or_phase* ph)
{
    if (!f->has_map) return ESLAM_ERR_NO_ENVIRONMENT;
    const eslam_config* c = &f->cfg;
    or_contact_model cm0;
    or_cm_init(&cm0, c);
    or_cm_set_contact_points(&cm0, in->n_contacts, in->contacts, in->body2odometry_rot);
    cm0.literal = f->literal;

    uint64_t total_points = 0, data_particles = 0;
    double sum_data_weights = 0.0;      /* reference mode */
    const double last_max_weight = f->max_weight;
    double maxw = 0;
    const double me2 = c->measurement_error * c->measurement_error;
    double* a_val = malloc(f->n * 8);   /* w_A * mprob, contract mode */
    double* sw_val = malloc(f->n * 8);
    uint8_t* bucket = malloc(f->n);
    int err = 0;

    int zero_var = 0;
    const int64_t n = (int64_t)f->n;
#pragma omp parallel num_threads(f->threads) if (f->threads > 1) reduction(+ : total_points, data_particles) reduction(max : maxw) reduction(| : zero_var)
    {
    or_contact_model cm = cm0;            /* per-thread scratch of evaluatePose */
#pragma omp for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        double s, co;
        or_sincos(f, f->th[OD(i)], &s, &co);
        const double r22 = (1.0 - co) + co;
        /* Translation3d(x, y, zPos) * AngleAxisd(theta, UnitZ) */
        double T[12] = {co, -s, 0.0, f->x[OD(i)], s, co, 0.0, f->y[OD(i)], 0.0, 0.0, r22, f->z[OD(i)]};
        const double meas_var = f->literal ? pow(f->zs[OD(i)], 2) + pow(c->measurement_error, 2) : f->zs[OD(i)] * f->zs[OD(i)] + me2;
        or_pmap pmc = {&f->map, f->lm_on ? f->pm_ctr + 2 * (uint64_t)i : NULL,
                       f->lm_on ? f->pm_slot + (uint64_t)i * f->lm_R : NULL, f->pg_blk, f->lm_hx, f->lm_hy, f->lm_wx,
                       f->lm_wy, f->lm_V};
        int acc = f->lm_on ? or_cm_evaluate_pose(&cm, T, meas_var, particle_map_fn, &pmc)
                            : or_cm_evaluate_pose(&cm, T, meas_var, grid_map_fn, &f->map);
        if (acc < 0) { zero_var = 1; acc = 0; }
        sw_val[i] = 0.0;
        if (acc) {
            double zvar = f->zs[OD(i)] * f->zs[OD(i)];
            or_cm_update_z(&cm, &f->z[OD(i)], &zvar);
            f->zs[OD(i)] = sqrt(zvar);
            const double weight = cm.weight;
            f->w[OD(i)] *= weight;
            f->mprob[OD(i)] = weight;
            f->floating[OB(i)] = 0;
            maxw = (maxw < weight) ? weight : maxw;
            data_particles++;
            const uint64_t found = cm.ncp;
            /* pow(weight, 1.0/found) with weight = exp(-s2/2): exp(-s2/2 * (1/found)) */
            if (f->literal) sw_val[i] = pow(weight, 1.0 / (double)found);   /* src/PoseEstimator.cpp:309 */
            else if (!cm.use_shape_update || found == 0) sw_val[i] = dm_pow(weight, 1.0 / (double)found);
            else sw_val[i] = weight == 0.0 ? 0.0 : dm_exp((-0.5 * cm.shape_s2) * (1.0 / (double)found));
            total_points += found;
        } else {
            f->floating[OB(i)] = 1;
            f->mprob[OD(i)] = 1.0;
        }
        f->ncp[OB(i)] = (uint8_t)cm.ncp;
        bucket[i] = (uint8_t)(cm.ncp < DM_NBUCKETS - 1 ? cm.ncp : DM_NBUCKETS - 1);
        a_val[i] = f->w[OD(i)] * f->mprob[OD(i)];
        if (f->dbg_ncp) {
            f->dbg_ncp[i] = cm.ncp;
            memcpy(&f->dbg_cp[i * ESLAM_MAX_CONTACTS], cm.cp, cm.ncp * sizeof(or_cpoint));
            f->dbg_zdelta[i] = acc ? cm.zdelta : 0.0;
            f->dbg_zvar[i] = acc ? cm.zvar : 0.0;
        }
    }
    }
    if (zero_var) err = ESLAM_ERR_ZERO_MEAS_VAR;
    if (err) { free(a_val); free(sw_val); free(bucket); return err; }
    /* reference mode: the sequential sum in particle order (non-data particles add +0.0) */
    for (uint64_t i = 0; i < f->n; ++i) sum_data_weights += sw_val[i];

    const uint32_t J = dm_chunk_rows_cfg(NG(f), f->cfg.sum_chunk_rows);
    /* contract mode: every exact partial sum of the update; sharded filters combine them
     * across ranks in one exchange (the device's per-rank statistics record) */
    or_acc accs[2 * DM_NBUCKETS + 1];
    memset(accs, 0, sizeof(accs));
    const int sa = DM_FX_SCALE - f->wexp, sb = DM_FX_SCALE - 2 * f->wexp;
    if (f->sum_mode == OR_SUM_CONTRACT) {
        chunk_reduce(sw_val, 1, NULL, 0, f->n, J, &accs[2 * DM_NBUCKETS], DM_FX_SCALE);
        double* a2 = malloc(f->n * 8 + 8);
        for (uint64_t i = 0; i < f->n; ++i) a2[i] = a_val[i] * a_val[i];
        for (int b = 0; b < DM_NBUCKETS; ++b) {
            chunk_reduce(a_val, 1, bucket, b, f->n, J, &accs[b], sa);
            chunk_reduce(a2, 1, bucket, b, f->n, J, &accs[DM_NBUCKETS + b], sb);
        }
        free(a2);
        if (combine_accs(f, accs, 2 * DM_NBUCKETS + 1)) { free(a_val); free(sw_val); free(bucket); return ESLAM_ERR_COMM; }
        sum_data_weights = acc_value(&accs[2 * DM_NBUCKETS], DM_FX_SCALE);
    }
    if (f->sharded) {
        uint64_t mine[3], all[3 * ESLAM_ORACLE_MAX_RANKS];
        mine[0] = data_particles; mine[1] = total_points; memcpy(&mine[2], &maxw, 8);
        if (comm_allgather(f, mine, all, sizeof(mine))) { free(a_val); free(sw_val); free(bucket); return ESLAM_ERR_COMM; }
        data_particles = 0; total_points = 0;
        for (int r = 0; r < f->comm.nranks; ++r) {
            double m;
            data_particles += all[3 * r];
            total_points += all[3 * r + 1];
            memcpy(&m, &all[3 * r + 2], 8);
            maxw = (maxw < m) ? m : maxw;
        }
    }
    const double floating_weight = data_particles > 0 ? sum_data_weights / (double)data_particles : 1.0;
    ph->fw = floating_weight;
    const double base = c->discount_factor * floating_weight;
    for (int b = 0; b < DM_NBUCKETS; ++b) {
        uint64_t ncp = (uint64_t)b;                      /* bucket 5 = every n >= 5 */
        double expo = (double)(uint64_t)(4ull - ncp);    /* size_t arithmetic (Q2) */
        ph->f[b] = or_pow(f, base, expo);
    }
    /* phase B  src/PoseEstimator.cpp:332-345 */
    for (uint64_t i = 0; i < f->n; ++i) {
        double factor = f->mprob[OD(i)] * ph->f[bucket[i]];
        f->w[OD(i)] *= factor;
    }
    if (f->sum_mode == OR_SUM_CONTRACT) {
        double S = 0.0, Q = 0.0;
        for (int b = 0; b < DM_NBUCKETS; ++b) {
            S = S + ph->f[b] * acc_value(&accs[b], sa);
            Q = Q + (ph->f[b] * ph->f[b]) * acc_value(&accs[DM_NBUCKETS + b], sb);
        }
        ph->S = S;
        ph->Q = Q;
    }
    f->max_weight = maxw;
    if (total_points == 0) f->max_weight = last_max_weight * c->discount_factor;
    f->info.data_particles = data_particles;
    f->info.total_points = total_points;
    f->info.floating_weight = floating_weight;
    f->info.max_weight = f->max_weight;
    free(a_val); free(sw_val); free(bucket);
    return 0;
}

/* ---- normalizeWeights  src/ParticleFilter.hpp:46-70 ----------------------------------------- */
static double normalize_with(or_filter* f, double S, double Q, int have_sums)
{
    const uint64_t n = f->n;
    const uint64_t N = NG(f);
    double effective = 0;
    if (f->sum_mode == OR_SUM_REFERENCE || !have_sums) {
        if (f->sum_mode == OR_SUM_REFERENCE) {
            S = 0;
            for (uint64_t i = 0; i < n; ++i) S += f->w[OD(i)];
        } else {
            const uint32_t J = dm_chunk_rows_cfg(N, f->cfg.sum_chunk_rows);
            int e = f->wexp;
            double* w2 = malloc(n * 8 + 8);
            for (uint64_t i = 0; i < n; ++i) w2[i] = f->w[OD(i)] * f->w[OD(i)];
            or_acc AB[2];
            memset(AB, 0, sizeof(AB));
            chunk_reduce(f->w, OR_DSTRIDE, NULL, 0, n, J, &AB[0], DM_FX_SCALE - e);
            chunk_reduce(w2, 1, NULL, 0, n, J, &AB[1], DM_FX_SCALE - 2 * e);
            free(w2);
            combine_accs(f, AB, 2);
            S = acc_value(&AB[0], DM_FX_SCALE - e);
            Q = acc_value(&AB[1], DM_FX_SCALE - 2 * e);
        }
    }
    f->info.weight_sum = S;
    f->info.uniform_reset = 0;
    if (S <= 0.0) {
        f->info.uniform_reset = 1;
        for (uint64_t i = 0; i < n; ++i) {
            double* w = &f->w[OD(i)];
            *w = 1.0 / (double)N;
            effective += *w * *w;
        }
        if (f->sum_mode == OR_SUM_CONTRACT) effective = 1.0 / (double)N;   /* eff := N */
    } else {
        for (uint64_t i = 0; i < n; ++i) {
            f->w[OD(i)] /= S;
            effective += f->w[OD(i)] * f->w[OD(i)];
        }
        if (f->sum_mode == OR_SUM_CONTRACT) effective = Q / (S * S);
    }
    f->wexp = 1;
    return 1.0 / effective;
}

double or_normalize_weights(or_filter* f) { return normalize_with(f, 0, 0, 0); }

double or_get_weights_sum(or_filter* f)
{
    if (f->sum_mode == OR_SUM_REFERENCE) {
        double s = 0;
        for (uint64_t i = 0; i < f->n; ++i) s += f->w[OD(i)];
        return s;
    }
    or_acc A = {{0}};
    chunk_reduce(f->w, OR_DSTRIDE, NULL, 0, f->n, dm_chunk_rows_cfg(NG(f), f->cfg.sum_chunk_rows), &A, DM_FX_SCALE - f->wexp);
    combine_accs(f, &A, 1);
    return acc_value(&A, DM_FX_SCALE - f->wexp);
}

/* ---- resample_stratified  src/ParticleFilter.hpp:85-108 ------------------------------------ */
static void gather(or_filter* f, const uint32_t* anc, uint64_t samples)
{
#ifdef OR_AOS
    uint8_t* nr = malloc((samples ? samples : 1) * OR_REC_BYTES);  /* whole 288-byte records */
    const uint8_t* r = f->rec;
    for (uint64_t k = 0; k < samples; ++k)
        memcpy(nr + k * OR_REC_BYTES, r + (uint64_t)anc[k] * OR_REC_BYTES, OR_REC_BYTES);
    free_state(f);
    set_views(f, nr);
#else
    double *nx = malloc(samples * 8), *ny = malloc(samples * 8), *nt = malloc(samples * 8), *nz = malloc(samples * 8),
           *ns = malloc(samples * 8), *nw = malloc(samples * 8), *nm = malloc(samples * 8);
    uint8_t *nf = malloc(samples), *nc = malloc(samples);
    for (uint64_t k = 0; k < samples; ++k) {
        uint32_t i = anc[k];
        nx[k] = f->x[i]; ny[k] = f->y[i]; nt[k] = f->th[i]; nz[k] = f->z[i]; ns[k] = f->zs[i];
        nw[k] = f->w[i]; nm[k] = f->mprob[i]; nf[k] = f->floating[i]; nc[k] = f->ncp[i];
    }
    free_state(f);
    f->x = nx; f->y = ny; f->th = nt; f->z = nz; f->zs = ns; f->w = nw; f->mprob = nm; f->floating = nf; f->ncp = nc;
#endif
    if (f->lm_on) {                       /* a copied particle carries its map (cloneMaps: the
                                             slots are copied, the pages shared until written) */
        const uint64_t S = f->lm_R;          /* the slots and the trail */
        int32_t* nc = malloc(samples * 2 * sizeof(int32_t));
        uint32_t* ns = malloc(samples * S * sizeof(uint32_t));
        uint64_t* nid = malloc(samples * 8);
        for (uint64_t k = 0; k < samples; ++k) {
            const uint32_t i = anc[k];
            nc[2 * k] = f->pm_ctr[2 * (uint64_t)i];
            nc[2 * k + 1] = f->pm_ctr[2 * (uint64_t)i + 1];
            memcpy(ns + k * S, f->pm_slot + (uint64_t)i * S, S * sizeof(uint32_t));
            nid[k] = f->pm_id[i];
        }
        free(f->pm_ctr); free(f->pm_slot); free(f->pm_id);
        f->pm_ctr = nc; f->pm_slot = ns; f->pm_id = nid;
    }
}

/* shift: fixed-point shift of the contract-mode cumulative sum (device ctl->scan_shift) */
static void resample_stratified(or_filter* f, uint64_t samples, int shift)
{
    const uint64_t n = f->n;
    uint32_t* anc = f->anc;
    uint64_t overruns = 0;
    uint64_t idx = 0;
    if (f->sum_mode == OR_SUM_REFERENCE) {
        double sum_w = f->w[OD(idx)];
        for (uint64_t k = 0; k < samples; ++k) {
            f->minstd = dm_minstd_next(f->minstd);
            double sum_r = ((double)k + dm_minstd_uniform(f->minstd)) / (double)samples;
            while (sum_w < sum_r) {
                if (idx + 1 >= n) { overruns++; break; }   /* Q5: clamp instead of UB */
                ++idx;
                sum_w += f->w[OD(idx)];
            }
            anc[k] = (uint32_t)idx;
        }
    } else {
        uint64_t sum_w = dm_fx_shift(f->w[OD(idx)], shift);
        for (uint64_t k = 0; k < samples; ++k) {
            f->minstd = dm_minstd_next(f->minstd);
            double sum_r = ((double)k + dm_minstd_uniform(f->minstd)) / (double)samples;
            uint64_t t = dm_fx_shift(sum_r, shift);
            while (sum_w < t) {
                if (idx + 1 >= n) { overruns++; break; }
                ++idx;
                sum_w += dm_fx_shift(f->w[OD(idx)], shift);
            }
            anc[k] = (uint32_t)idx;
        }
    }
    f->info.resample_overruns = overruns;
    gather(f, anc, samples);
    f->has_anc = 1;
}


/* ---- sharded resample: the multi-GPU decomposition restated on the CPU -----------------
 * Particle i (global index g) with inclusive fixed-point cumulative sum C_g fills the
 * outputs [lo, hi) with lo = #{k : T_k <= C_(g-1)} (0 for g = 0) and hi = #{k : T_k <= C_g}
 * (N for the last particle: the Q5 clamp), T_k = fx((k + U_k) / N) -- the same ancestors
 * as resample_stratified.  Each rank sends every particle whose range meets another
 * rank's output slice there (all_to_all_v) and fills its own slice from what it gets.  */
typedef struct {
    double x, y, th, z, zs, w, mprob;
    uint64_t lo, hi, src;          /* global output range, global source index */
    uint8_t floating, ncp, pad[6];
    /* per-particle maps: the source particle's map travels with it (a deep copy): its window
     * centre here, its npg pages in the payload stream (or_mig_page each: the window's in slot
     * order, then the trail's in entry order)                                             */
    int32_t pm_ctr[2];
    uint32_t pm_npg, pm_pad;
    uint64_t pm_id;
} or_mig;
typedef struct {
    uint32_t slot;                 /* < S: a window slot; S + e: trail entry e of tile (a, b) */
    int32_t a, b;
    uint32_t pad;
    or_page page;
} or_mig_page;

static void resample_sharded(or_filter* f, int shift)
{
    const int G = f->comm.nranks, me = f->comm.rank;
    const uint64_t N = f->n_global, n = f->n;
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; ++i) total += dm_fx_shift(f->w[OD(i)], shift);
    uint64_t totals[ESLAM_ORACLE_MAX_RANKS];
    comm_allgather(f, &total, totals, 8);
    uint64_t off = 0;
    for (int r = 0; r < me; ++r) off += totals[r];
    /* the N stratified draws (every rank walks the whole minstd stream) */
    uint64_t* T = malloc(N * 8);
    for (uint64_t k = 0; k < N; ++k) {
        f->minstd = dm_minstd_next(f->minstd);
        T[k] = dm_fx_shift(((double)k + dm_minstd_uniform(f->minstd)) / (double)N, shift);
    }
    uint64_t* lo = malloc(n * 8 + 8);
    uint64_t* hi = malloc(n * 8 + 8);
    uint64_t c = off, k = 0, overruns = 0;
    while (k < N && T[k] <= c) ++k;
    for (uint64_t i = 0; i < n; ++i) {
        lo[i] = (f->gbase + i == 0) ? 0 : k;
        c += dm_fx_shift(f->w[OD(i)], shift);
        while (k < N && T[k] <= c) ++k;
        hi[i] = k;
        if (f->gbase + i == N - 1) { overruns = N - k; hi[i] = N; }
    }
    free(T);
    /* per-destination records */
    uint64_t cnt[ESLAM_ORACLE_MAX_RANKS] = {0};
    for (int d = 0; d < G; ++d)
        for (uint64_t i = 0; i < n; ++i) {
            const uint64_t a = lo[i] > f->gall[d] ? lo[i] : f->gall[d];
            const uint64_t b = hi[i] < f->gall[d + 1] ? hi[i] : f->gall[d + 1];
            if (a < b) cnt[d]++;
        }
    uint64_t nsend = 0;
    for (int d = 0; d < G; ++d) nsend += cnt[d];
    or_mig* send = malloc(sizeof(or_mig) * (nsend ? nsend : 1));
    uint64_t j = 0;
    for (int d = 0; d < G; ++d)
        for (uint64_t i = 0; i < n; ++i) {
            const uint64_t a = lo[i] > f->gall[d] ? lo[i] : f->gall[d];
            const uint64_t b = hi[i] < f->gall[d + 1] ? hi[i] : f->gall[d + 1];
            if (a >= b) continue;
            or_mig* m = &send[j++];
            memset(m, 0, sizeof(*m));
            m->x = f->x[OD(i)]; m->y = f->y[OD(i)]; m->th = f->th[OD(i)]; m->z = f->z[OD(i)]; m->zs = f->zs[OD(i)];
            m->w = f->w[OD(i)]; m->mprob = f->mprob[OD(i)];
            m->floating = f->floating[OB(i)]; m->ncp = f->ncp[OB(i)];
            m->lo = a; m->hi = b; m->src = f->gbase + i;
            if (f->lm_on) {
                m->pm_id = f->pm_id[i];
                m->pm_ctr[0] = f->pm_ctr[2 * i];
                m->pm_ctr[1] = f->pm_ctr[2 * i + 1];
                const uint32_t* row = f->pm_slot + i * f->lm_R;
                for (uint64_t q = 0; q < f->lm_S; ++q) m->pm_npg += row[q] != DM_LM_NONE;
                for (uint32_t e = 0; e < f->lm_V; ++e) m->pm_npg += row[f->lm_S + 3 * e + 2] != DM_LM_NONE;
            }
        }
    /* the maps' pages, in the records' order (one more all_to_all_v of byte counts the
     * receivers learn from an all_gather) */
    uint64_t pbytes[ESLAM_ORACLE_MAX_RANKS] = {0}, npay = 0;
    or_mig_page* pay = NULL;
    if (f->lm_on) {
        uint64_t q = 0;
        for (int d = 0; d < G; ++d)
            for (uint64_t r = 0; r < cnt[d]; ++r) pbytes[d] += send[q++].pm_npg * sizeof(or_mig_page);
        for (int d = 0; d < G; ++d) npay += pbytes[d] / sizeof(or_mig_page);
        pay = malloc((npay ? npay : 1) * sizeof(or_mig_page));
        uint64_t w = 0;
        for (uint64_t r = 0; r < nsend; ++r) {
            const uint64_t i = send[r].src - f->gbase;
            const uint32_t* row = f->pm_slot + i * f->lm_R;
            for (uint32_t sl = 0; sl < f->lm_S + f->lm_V; ++sl) {
                const uint32_t pg = sl < f->lm_S ? row[sl] : row[f->lm_S + 3 * (sl - f->lm_S) + 2];
                if (pg == DM_LM_NONE) continue;
                pay[w].slot = sl;
                pay[w].a = sl < f->lm_S ? 0 : (int32_t)row[f->lm_S + 3 * (sl - f->lm_S)];
                pay[w].b = sl < f->lm_S ? 0 : (int32_t)row[f->lm_S + 3 * (sl - f->lm_S) + 1];
                pay[w].pad = 0;
                pay[w].page = *lm_pg(f, pg);
                ++w;
            }
        }
    }
    free(lo); free(hi);
    uint64_t all[ESLAM_ORACLE_MAX_RANKS * ESLAM_ORACLE_MAX_RANKS];
    comm_allgather(f, cnt, all, 8ull * G);
    uint64_t sb[ESLAM_ORACLE_MAX_RANKS], rb[ESLAM_ORACLE_MAX_RANKS], nrecv = 0;
    for (int r = 0; r < G; ++r) {
        sb[r] = cnt[r] * sizeof(or_mig);
        rb[r] = all[r * G + me] * sizeof(or_mig);
        nrecv += all[r * G + me];
    }
    or_mig* recv = malloc(sizeof(or_mig) * (nrecv ? nrecv : 1));
    f->comm.alltoallv(f->comm.user, send, sb, recv, rb, NULL);
    free(send);
    or_mig_page* rpay = NULL;
    if (f->lm_on) {
        uint64_t pall[ESLAM_ORACLE_MAX_RANKS * ESLAM_ORACLE_MAX_RANKS], prb[ESLAM_ORACLE_MAX_RANKS], nr = 0;
        comm_allgather(f, pbytes, pall, 8ull * G);
        for (int r = 0; r < G; ++r) {
            prb[r] = pall[r * G + me];
            nr += prb[r];
        }
        rpay = malloc(nr ? nr : 1);
        f->comm.alltoallv(f->comm.user, pay, pbytes, rpay, prb, NULL);
        free(pay);
    }
    /* the received maps: each record's pages become pages of this rank (first page index of
     * record q: rfirst[q]); own records keep their maps' pages */
    uint64_t* rfirst = calloc(nrecv ? nrecv : 1, 8);
    uint32_t* rpg = NULL;
    if (f->lm_on) {
        uint64_t tot = 0;
        for (uint64_t q = 0; q < nrecv; ++q) { rfirst[q] = tot; tot += recv[q].pm_npg; }
        rpg = malloc((tot ? tot : 1) * 4);
        for (uint64_t q = 0; q < tot; ++q) {
            rpg[q] = lm_alloc(f);
            *lm_pg(f, rpg[q]) = rpay[q].page;
        }
    }
    uint32_t* anc = calloc(n + 1, 4);
    or_mig* src = calloc(n ? n : 1, sizeof(or_mig));
    uint64_t* srcq = calloc(n ? n : 1, 8);
    for (uint64_t q = 0; q < nrecv; ++q)
        for (uint64_t o = recv[q].lo; o < recv[q].hi; ++o) {
            src[o - f->gbase] = recv[q];
            srcq[o - f->gbase] = q;
            anc[o - f->gbase] = (uint32_t)recv[q].src;
        }
    free(recv);
    /* the new maps (slots of the sources this rank holds, the received pages for others) */
    int32_t* nctr = NULL;
    uint32_t* nslot = NULL;
    if (f->lm_on) {
        const uint64_t R = f->lm_R, S = f->lm_S;
        nctr = malloc(n * 2 * sizeof(int32_t));
        nslot = malloc(n * R * 4);
        for (uint64_t o = 0; o < n; ++o) {
            const or_mig* m = &src[o];
            nctr[2 * o] = m->pm_ctr[0];
            nctr[2 * o + 1] = m->pm_ctr[1];
            uint32_t* sl = nslot + o * R;
            if (m->src - f->gbase < n) {
                memcpy(sl, f->pm_slot + (m->src - f->gbase) * R, R * 4);
            } else {
                memset(sl, 0xff, R * 4);
                const uint64_t q0 = rfirst[srcq[o]];
                for (uint32_t k = 0; k < m->pm_npg; ++k) {
                    const or_mig_page* pp = &rpay[q0 + k];
                    if (pp->slot < S) {
                        sl[pp->slot] = rpg[q0 + k];
                    } else {
                        uint32_t* t = sl + S + 3 * (pp->slot - S);
                        t[0] = (uint32_t)pp->a; t[1] = (uint32_t)pp->b; t[2] = rpg[q0 + k];
                    }
                }
            }
        }
    }
    for (uint64_t o = 0; o < n; ++o) {
        const or_mig* m = &src[o];
        f->x[OD(o)] = m->x; f->y[OD(o)] = m->y; f->th[OD(o)] = m->th; f->z[OD(o)] = m->z; f->zs[OD(o)] = m->zs;
        f->w[OD(o)] = m->w; f->mprob[OD(o)] = m->mprob; f->floating[OB(o)] = m->floating; f->ncp[OB(o)] = m->ncp;
        f->anc[o] = anc[o];
        if (f->lm_on) {
            /* a map from another rank arrives as a copy of its own, one per record, which the
             * record's outputs share (the GPU: a table per record that they all name) */
            f->pm_id[o] = m->src - f->gbase < n ? m->pm_id : f->pm_fresh + srcq[o];
        }
    }
    if (f->lm_on) f->pm_fresh += nrecv;
    free(rfirst); free(rpg); free(rpay); free(srcq);
    if (f->lm_on) {
        free(f->pm_ctr); free(f->pm_slot);
        f->pm_ctr = nctr; f->pm_slot = nslot;
    }
    free(src); free(anc);
    f->info.resample_overruns = overruns;
    f->has_anc = 1;
}

int or_set_comm(or_filter* f, const eslam_comm* comm, uint64_t n_global, const uint64_t* shard_gbase)
{
    or_free_particles(f);
    if (!comm) { f->sharded = 0; f->n_global = 0; f->gbase = 0; return 0; }
    if (comm->device_memory || comm->nranks < 1 || comm->nranks > ESLAM_ORACLE_MAX_RANKS) return ESLAM_ERR_INVALID_ARG;
    const uint64_t csz = 64ull * dm_chunk_rows_cfg(n_global, f->cfg.sum_chunk_rows);
    if (shard_gbase[0] != 0 || shard_gbase[comm->nranks] != n_global) return ESLAM_ERR_INVALID_ARG;
    for (int r = 0; r < comm->nranks; ++r)
        if (shard_gbase[r + 1] <= shard_gbase[r] || shard_gbase[r] % csz) return ESLAM_ERR_INVALID_ARG;
    f->sharded = 1;
    f->comm = *comm;
    f->n_global = n_global;
    memcpy(f->gall, shard_gbase, sizeof(uint64_t) * (size_t)(comm->nranks + 1));
    f->gbase = shard_gbase[comm->rank];
    return 0;
}

/* standalone ParticleFilter::resample() on the weights as they are: the contract scales
 * the cumulative sum by the exact weight sum's exponent (device FIN_RESAMPLE)          */
void or_resample(or_filter* f)
{
    int shift = 60;
    if (f->sum_mode == OR_SUM_CONTRACT) {
        or_acc A = {{0}};
        chunk_reduce(f->w, OR_DSTRIDE, NULL, 0, f->n, dm_chunk_rows_cfg(NG(f), f->cfg.sum_chunk_rows), &A, DM_FX_SCALE - f->wexp);
        combine_accs(f, &A, 1);
        shift = 61 - (dm_weight_exp(acc_value(&A, DM_FX_SCALE - f->wexp)) + 1);
    }
    if (f->sharded) resample_sharded(f, shift);
    else resample_stratified(f, f->n, shift);
}

/* src/ParticleFilter.hpp:120-148 (not used by PoseEstimator; weights reset to 1/N) */
void or_resample_multinomial(or_filter* f, uint64_t samples)
{
    uint32_t* anc = calloc(samples + 1, 4);
    uint64_t m = 0;
    for (uint64_t k = 0; k < samples; ++k) {
        f->minstd = dm_minstd_next(f->minstd);
        double r = dm_minstd_uniform(f->minstd);
        double sum = 0;
        for (uint64_t i = 0; i < f->n; ++i) {
            sum += f->w[OD(i)];
            if (r <= sum) { anc[m++] = (uint32_t)i; break; }
        }
    }
    gather(f, anc, m);
    f->n = m;
    for (uint64_t i = 0; i < m; ++i) f->w[OD(i)] = 1.0 / (double)m;
    free(anc);
}

/* ---- PoseEstimator::update  src/PoseEstimator.cpp:244-255 ---------------------------------- */
int or_update(or_filter* f, const eslam_step_input* in)
{
    if (!f->n) return ESLAM_ERR_NOT_INITIALISED;
    or_phase ph;
    memset(&ph, 0, sizeof(ph));
    int rc = or_update_weights(f, in, &ph);
    if (rc) return rc;
    double eff = normalize_with(f, ph.S, ph.Q, 1);
    f->info.effective = eff;
    f->info.resampled = 0;
    f->info.resample_overruns = 0;
    if (eff < (double)f->cfg.min_effective) {
        if (f->sharded) resample_sharded(f, 60);
        else resample_stratified(f, f->n, 60);
        f->info.resampled = 1;
    }
    f->info.update_count++;
    return 0;
}

/* ---- EmbodiedSlamFilter::update(body2odometry, bs, ltc)  src/EmbodiedSlamFilter.cpp:353-369 */
int or_step(or_filter* f, const eslam_step_input* in, int* updated)
{
    int rc = or_project(f, in);
    if (rc) return rc;
    int gate = update_threshold_test(f->cfg.measurement_threshold_distance, f->cfg.measurement_threshold_angle,
                                     f->ud_pose, in->body2odometry_rot, in->body2odometry_trans);
    if (gate || in->ltc_count > 0) {
        rc = or_update(f, in);
        if (rc) return rc;
        double R[9];
        q_to_mat(in->body2odometry_rot, R);
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) f->ud_pose[r * 4 + c] = R[r * 3 + c];
            f->ud_pose[r * 4 + 3] = in->body2odometry_trans[r];
        }
        if (updated) *updated = 1;
    } else if (updated) {
        *updated = 0;
    }
    return 0;
}

int or_last_info(or_filter* f, eslam_update_info* info) { *info = f->info; return 0; }

/* src/ParticleFilter.hpp:160-173 (first maximum, strict >) */
uint64_t or_best_index(or_filter* f)
{
    uint64_t index = 0;
    double weight = -INFINITY;
    for (uint64_t i = 0; i < f->n; ++i)
        if (f->w[OD(i)] > weight) { index = i; weight = f->w[OD(i)]; }
    if (f->sharded) {          /* the same scan over the ranks' results in rank order */
        double mine[2] = {weight, (double)(f->gbase + index)}, all[2 * ESLAM_ORACLE_MAX_RANKS];
        comm_allgather(f, mine, all, sizeof(mine));
        index = 0;
        weight = -INFINITY;
        for (int r = 0; r < f->comm.nranks; ++r)
            if (all[2 * r] > weight) { index = (uint64_t)all[2 * r + 1]; weight = all[2 * r]; }
    }
    return index;
}

/* getCentroid's five sums (x w, y w, theta w, z w, w) under the sum contract: per canonical
 * chunk (64 lanes x J rows; lane l adds rows in order), an xor butterfly over the lanes
 * (distances 32 .. 1), then a fixed pairwise tree over the chunks in global order
 * (dst[i] = src[2i] + src[2i+1], an odd tail moves up).  A sharded filter all-gathers its
 * chunk records (the shards are chunk-aligned), so every rank gets the one-filter sums.    */
static void centroid_contract(or_filter* f, double out[5])
{
    const uint32_t J = dm_chunk_rows_cfg(NG(f), f->cfg.sum_chunk_rows);
    const uint64_t csz = 64ull * J;
    const uint64_t nch = (f->n + csz - 1) / csz;
    int G = f->sharded ? f->comm.nranks : 1;
    uint64_t maxch = nch ? nch : 1;
    if (f->sharded) {
        maxch = 1;
        for (int r = 0; r < G; ++r) {
            const uint64_t c = (f->gall[r + 1] - f->gall[r] + csz - 1) / csz;
            maxch = c > maxch ? c : maxch;
        }
    }
    double* mine = calloc(maxch * 5, sizeof(double));
    for (uint64_t c = 0; c < nch; ++c) {
        double lane[64][5];
        for (int l = 0; l < 64; ++l) {
            double a[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
            for (uint32_t j = 0; j < J; ++j) {
                const uint64_t i = c * csz + 64ull * j + (uint64_t)l;
                if (i >= f->n) continue;
                const double w = f->w[OD(i)];
                a[0] = a[0] + f->x[OD(i)] * w;
                a[1] = a[1] + f->y[OD(i)] * w;
                a[2] = a[2] + f->th[OD(i)] * w;
                a[3] = a[3] + f->z[OD(i)] * w;
                a[4] = a[4] + w;
            }
            memcpy(lane[l], a, sizeof(a));
        }
        for (int o = 32; o >= 1; o >>= 1) {
            double nxt[64][5];
            for (int l = 0; l < 64; ++l)
                for (int q = 0; q < 5; ++q) nxt[l][q] = lane[l][q] + lane[l ^ o][q];
            memcpy(lane, nxt, sizeof(lane));
        }
        memcpy(&mine[c * 5], lane[0], 5 * sizeof(double));
    }
    uint64_t total = nch;
    double* rec = mine;
    if (f->sharded) {
        double* all = malloc((size_t)G * maxch * 5 * sizeof(double));
        comm_allgather(f, mine, all, maxch * 5 * sizeof(double));
        rec = calloc((size_t)G * maxch * 5 + 5, sizeof(double));
        total = 0;
        for (int r = 0; r < G; ++r) {
            const uint64_t c = (f->gall[r + 1] - f->gall[r] + csz - 1) / csz;
            memcpy(&rec[total * 5], &all[(uint64_t)r * maxch * 5], c * 5 * sizeof(double));
            total += c;
        }
        free(all);
    }
    uint64_t m = total;
    while (m > 1) {
        const uint64_t h = m / 2, m2 = (m + 1) / 2;
        for (uint64_t i = 0; i < h; ++i)
            for (int q = 0; q < 5; ++q) rec[i * 5 + q] = rec[(2 * i) * 5 + q] + rec[(2 * i + 1) * 5 + q];
        if (m & 1)
            for (int q = 0; q < 5; ++q) rec[h * 5 + q] = rec[(m - 1) * 5 + q];
        m = m2;
    }
    for (int q = 0; q < 5; ++q) out[q] = total ? rec[q] : 0.0;
    if (rec != mine) free(rec);
    free(mine);
}

/* PoseEstimator::getCentroid  src/PoseEstimator.cpp:354-383: normalises the weights in place
 * (Q15), then the weighted means with theta averaged linearly.  Reference mode: the
 * sequential sums of :357-366 (sharded: each rank's sequential sums, added in rank order);
 * contract mode: centroid_contract (what the device computes, bit for bit).                */
void or_get_centroid(or_filter* f, double position[3], double q[4])
{
    or_normalize_weights(f);
    double s[5] = {0, 0, 0, 0, 0};
    if (f->sum_mode == OR_SUM_CONTRACT) {
        centroid_contract(f, s);
    } else {
        for (uint64_t i = 0; i < f->n; ++i) {
            s[0] += f->x[OD(i)] * f->w[OD(i)];
            s[1] += f->y[OD(i)] * f->w[OD(i)];
            s[2] += f->th[OD(i)] * f->w[OD(i)];
            s[3] += f->z[OD(i)] * f->w[OD(i)];
            s[4] += f->w[OD(i)];
        }
        if (f->sharded) {
            double all[5 * ESLAM_ORACLE_MAX_RANKS];
            comm_allgather(f, s, all, sizeof(s));
            for (int k = 0; k < 5; ++k) {
                s[k] = 0.0;
                for (int r = 0; r < f->comm.nranks; ++r) s[k] += all[5 * r + k];
            }
        }
    }
    const double sw = s[4];
    position[0] = s[0] / sw; position[1] = s[1] / sw; position[2] = s[3] / sw;
    const double mo = s[2] / sw;
    double a[4];
    q_from_yaw(mo, a);
    q_mul(a, f->zcomp, q);
}

int or_get_ancestors(or_filter* f, uint32_t* out, uint64_t n)
{
    if (!f->has_anc) return ESLAM_ERR_INVALID_ARG;
    memcpy(out, f->anc, (n < f->n ? n : f->n) * 4);
    return 0;
}

void or_get_rng_state(or_filter* f, eslam_rng_state* st)
{
    memset(st, 0, sizeof(*st));
    st->minstd_x = f->minstd;
    st->project_count = f->project_count;
    st->init_count = f->init_count;
    st->hash_count = f->hash_count;
    st->max_weight = f->max_weight;
    memcpy(st->ud_pose, f->ud_pose, sizeof(f->ud_pose));
    memcpy(st->libc_rand, f->libc.r, sizeof(st->libc_rand));
    st->libc_rand_pos = f->libc.i;
}

void or_set_rng_state(or_filter* f, const eslam_rng_state* st)
{
    f->minstd = st->minstd_x;
    f->project_count = st->project_count;
    f->init_count = st->init_count;
    f->hash_count = st->hash_count;
    f->max_weight = st->max_weight;
    memcpy(f->ud_pose, st->ud_pose, sizeof(f->ud_pose));
    memcpy(f->libc.r, st->libc_rand, sizeof(st->libc_rand));
    f->libc.i = st->libc_rand_pos % 34u;
}

/* EmbodiedSlamFilter::processMap(scanMap, match = false, update = true)
 * (src/EmbodiedSlamFilter.cpp:179-232) on per-particle maps.  Per particle: the map's window
 * moves to the tile under the particle (the active-grid switch of :195-207, here a window of
 * tiles reaching maxSensorRange around the particle: tiles that leave it are forgotten), then
 * every scan patch at the particle's pose (scanFrame = Translation(x, y, 0) * Rz(theta),
 * :186-189; the offset patch adds zPos and zSigma^2, :213-214) goes into the cell it lands in:
 * inserted into a cell empty in both the shared grid and the particle's map
 * (test/testMap.cpp:307-316), fused (variance-weighted) with the particle's patch there when
 * within 3 sigma (dm_lm_fuse), ignored on the shared grid's cells; a patch outside the window
 * (beyond maxSensorRange) is dropped.  A resample's copies share their pages until a write
 * (cloneMaps, src/PoseEstimator.cpp:31-47: the copies are independent, by value).          */
static int cmp_u64(const void* a, const void* b)
{
    const uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return x < y ? -1 : x > y;
}

static int or_map_update_part(or_filter* f, const eslam_scan_patch* sp, uint32_t m)
{
    if (!(f->cfg.flags & ESLAM_FLAG_PARTICLE_MAPS)) return ESLAM_ERR_INVALID_ARG;
    if (!f->has_map) return ESLAM_ERR_NO_ENVIRONMENT;
    if (!f->n) return ESLAM_ERR_NOT_INITIALISED;
    if (!f->lm_on) return ESLAM_ERR_OUT_OF_MEMORY;
    const eslam_mls_grid* g = &f->map;
    const double* A = g->global2local;
    static const double id[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    int is_id = 1;
    for (int k = 0; k < 12; ++k) is_id &= A[k] == id[k];
    const uint64_t S = f->lm_S, R = f->lm_R;
    const uint32_t hx = f->lm_hx, hy = f->lm_hy, wx = f->lm_wx, wy = f->lm_wy, V = f->lm_V;
    /* which particles share their map with another (copies of one map the resample made and
     * no map update has changed since): the ids sorted, a particle's id looked up */
    uint64_t* sorted = malloc((f->n ? f->n : 1) * 8);
    uint8_t* shared = calloc(f->n ? f->n : 1, 1);
    uint8_t* dirt = calloc(f->n ? f->n : 1, 1);
    uint32_t* ref = calloc(f->pg_top ? f->pg_top : 1, 4);
    if (!sorted || !shared || !dirt || !ref) { free(sorted); free(shared); free(dirt); free(ref); return ESLAM_ERR_OUT_OF_MEMORY; }
    memcpy(sorted, f->pm_id, f->n * 8);
    qsort(sorted, f->n, 8, cmp_u64);
    for (uint64_t i = 0; i < f->n; ++i) {
        uint64_t lo = 0, hi = f->n;          /* first index with sorted[] >= id */
        while (lo < hi) {
            const uint64_t mid = lo + (hi - lo) / 2;
            if (sorted[mid] < f->pm_id[i]) lo = mid + 1;
            else hi = mid;
        }
        shared[i] = lo + 1 < f->n && sorted[lo + 1] == f->pm_id[i];
    }
    free(sorted);
    /* the names every map holds now: a page named once belongs to one particle's map and may
     * be written in place, one named more often is copied first; one named by none is free */
    for (uint64_t i = 0; i < f->n; ++i) {
        const uint32_t* row = f->pm_slot + i * R;
        for (uint64_t q = 0; q < S; ++q)
            if (row[q] != DM_LM_NONE) ref[row[q]]++;
        for (uint32_t e = 0; e < V; ++e)
            if (row[S + 3 * e + 2] != DM_LM_NONE) ref[row[S + 3 * e + 2]]++;
    }
    f->pg_nfree = 0;
    if (f->pg_free_cap < f->pg_top) {
        free(f->pg_free);
        f->pg_free = malloc((f->pg_top ? f->pg_top : 1) * 4);
        f->pg_free_cap = f->pg_top;
        if (!f->pg_free) { free(shared); free(dirt); free(ref); f->pg_free_cap = 0; return ESLAM_ERR_OUT_OF_MEMORY; }
    }
    for (uint64_t q = f->pg_top; q-- > 0;)
        if (!ref[q]) f->pg_free[f->pg_nfree++] = (uint32_t)q;
    uint64_t dropped = 0, changed = 0, covered = 0, evicted = 0;
    int oom = 0;
    const int64_t n = (int64_t)f->n;
    /* particles are independent: the OpenMP threads of or_set_threads (same results) */
#pragma omp parallel num_threads(f->threads) if (f->threads > 1) reduction(+ : dropped, changed, covered, evicted) reduction(| : oom)
    {
    uint8_t* mine = malloc(S);            /* slot's page made this particle's own in this update */
#pragma omp for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        int dirty = 0;
        int32_t* ctr = f->pm_ctr + 2 * i;
        uint32_t* sl = f->pm_slot + (uint64_t)i * R;
        double sn, co;
        dm_sincos(f->th[OD(i)], &sn, &co);
        const double zvar = f->zs[OD(i)] * f->zs[OD(i)];
        const double bx = f->x[OD(i)] - g->offset_x, by = f->y[OD(i)] - g->offset_y;
        const int placed = dm_isfinite(bx) && dm_isfinite(by) && dm_isfinite(f->th[OD(i)]);
        if (!placed) continue;
        /* the window's centre: the tile under the particle */
        int32_t na, nb;
        if (is_id) {
            na = dm_lm_centre(f->x[OD(i)], g->offset_x, 1.0 / g->scale_x);
            nb = dm_lm_centre(f->y[OD(i)], g->offset_y, 1.0 / g->scale_y);
        } else {
            const double px = f->x[OD(i)], py = f->y[OD(i)], pz = f->z[OD(i)];
            const double lx = ((A[0] * px + A[1] * py) + A[2] * pz) + A[3];
            const double ly = ((A[4] * px + A[5] * py) + A[6] * pz) + A[7];
            na = dm_lm_centre(lx, g->offset_x, 1.0 / g->scale_x);
            nb = dm_lm_centre(ly, g->offset_y, 1.0 / g->scale_y);
        }
        if (ctr[0] != na || ctr[1] != nb) {        /* tiles leaving the window go to the trail */
            evicted += lm_recentre(sl, ctr, na, nb, hx, hy, wx, wy, V);
            dirty = 1;
        }
        memset(mine, 0, S);
        for (uint32_t k = 0; k < m; ++k) {
            const double wz = sp[k].position[2] + f->z[OD(i)];
            uint32_t cell, cm, cn;
            if (is_id) {
                cell = dm_merge_cell_mn(bx, by, co, sn, sp[k].position[0], sp[k].position[1], 1.0 / g->scale_x,
                                        1.0 / g->scale_y, g->width, g->height, &cm, &cn);
                if (cell == 0xffffffffu) continue;
            } else {
                const double wx_ = (co * sp[k].position[0] + (-sn) * sp[k].position[1]) + f->x[OD(i)];
                const double wy_ = (sn * sp[k].position[0] + co * sp[k].position[1]) + f->y[OD(i)];
                const double lx = ((A[0] * wx_ + A[1] * wy_) + A[2] * wz) + A[3];
                const double ly = ((A[4] * wx_ + A[5] * wy_) + A[6] * wz) + A[7];
                const double fm = floor((lx - g->offset_x) * (1.0 / g->scale_x));
                const double fn = floor((ly - g->offset_y) * (1.0 / g->scale_y));
                if (!(fm >= 0.0 && fm < (double)g->width && fn >= 0.0 && fn < (double)g->height)) continue;
                cm = (uint32_t)fm;
                cn = (uint32_t)fn;
                cell = cn * g->width + cm;
            }
            /* a cell the shared grid covers: the particle's copy of it (the reference's clone,
             * src/PoseEstimator.cpp:31-47, merged at :222-227) starts from the grid's patch */
            const int cov = g->cell_start[cell] != g->cell_start[cell + 1];
            covered += (uint64_t)cov;
            const uint32_t a = cm >> DM_LM_TILE_BITS, b = cn >> DM_LM_TILE_BITS;
            if (!dm_lm_inside(a, ctr[0], hx, wx) || !dm_lm_inside(b, ctr[1], hy, wy)) {
                ++dropped;          /* beyond maxSensorRange: outside the window */
                continue;
            }
            const uint32_t slot = (a % wx) + wx * (b % wy);
            const uint32_t j = (cm & 7u) + 8u * (cn & 7u);
            const double var = sp[k].stdev * sp[k].stdev + zvar;
            uint32_t pg = sl[slot];
            float mo, so;
            double gm, gs;
            if (pg != DM_LM_NONE && dm_lm_holds(lm_pg(f, pg)->v[2 * j + 1])) {
                const float* v = lm_pg(f, pg)->v;
                if (!dm_lm_fuse(v[2 * j], v[2 * j + 1], wz, var, &mo, &so)) continue;
            } else if (cov && or_mls_cell_patch(g, cell, wz, var, &gm, &gs) && dm_lm_fuse((float)gm, (float)gs, wz, var, &mo, &so)) {
                /* fused with the grid's patch that getPatch's 3-sigma gate picks for it */
            } else {
                mo = (float)wz;
                so = (float)dm_sqrt(var);
            }
            if (!mine[slot] && (pg == DM_LM_NONE || ref[pg] > 1)) {
                /* the first write to this tile: a page of the particle's own (copy on write) */
                uint32_t np;
#pragma omp critical(or_pages)
                np = lm_alloc(f);
                if (np == DM_LM_NONE) { oom = 1; break; }
                or_page* d = lm_pg(f, np);
                if (pg == DM_LM_NONE) {
                    for (uint32_t q = 0; q < DM_LM_PAGE_CELLS; ++q) { d->v[2 * q] = 0.0f; d->v[2 * q + 1] = -1.0f; }
                } else {
                    *d = *lm_pg(f, pg);
                }
                sl[slot] = pg = np;
            }
            mine[slot] = 1;
            or_page* d = lm_pg(f, pg);
            d->v[2 * j] = mo;
            d->v[2 * j + 1] = so;
            dirty = 1;
        }
        changed += (uint64_t)dirty;
        dirt[i] = (uint8_t)dirty;
    }
    free(mine);
    }
    free(ref);
    /* a changed shared map becomes the particle's own (the GPU writes it to a free table) */
    uint64_t copied = 0;
    for (uint64_t i = 0; i < f->n; ++i)
        if (dirt[i] && shared[i]) { f->pm_id[i] = f->pm_fresh++; ++copied; }
    free(shared);
    free(dirt);
    if (oom) return ESLAM_ERR_OUT_OF_MEMORY;
    f->info.map_patches_dropped += dropped;
    f->info.map_stores_changed += changed;
    f->info.map_stores_copied += copied;
    f->info.map_patches_covered += covered;
    f->info.map_tiles_evicted += evicted;
    return 0;
}

/* processMap's merge of a whole scan in parts, in order (the GPU's parts, eslam_gpu_map_update:
 * a scan of at most 64 patches in one part, a larger one 256 at a time); every cell sees its
 * patches in the scan's order, the counters add up */
#define OR_SCAN_PART_SMALL 64u
#define OR_SCAN_PART_LARGE 256u
#define OR_MATCH_SAMPLING 10u       /* src/EmbodiedSlamFilter.cpp:216 */
#define OR_MATCH_SIGMA ((double)0.2f) /* :217, a float there */
int or_map_update(or_filter* f, const eslam_scan_patch* sp, uint32_t m)
{
    f->info.map_patches_dropped = f->info.map_stores_changed = 0;
    f->info.map_stores_copied = f->info.map_patches_covered = 0;
    f->info.map_tiles_evicted = 0;
    const uint32_t part = m <= OR_SCAN_PART_SMALL ? OR_SCAN_PART_SMALL : OR_SCAN_PART_LARGE;
    for (uint32_t c0 = 0; c0 == 0 || c0 < m; c0 += part) {
        const int rc = or_map_update_part(f, sp + c0, m - c0 < part ? m - c0 : part);
        if (rc) return rc;
    }
    return 0;
}

/* processMap(scanMap, match = true): the visual weighting p.weight *= pow(weight, 0.1) of
 * src/EmbodiedSlamFilter.cpp:214-221 (sampling 10, sigma 0.2), against the particle's map: the
 * shared grid (useSharedMap = true, the match-only call of :342-344), or its own map -- the
 * grid's cells, and its own patches in the cells the grid leaves empty (per-particle maps, the
 * clone the reference merges into).  envire's MLSGrid::match is not in the reference tree, so
 * this rule is the build's own (parity unpinned): every 10th scan patch, placed
 * like the merge (offset patch zPos, zSigma), scores on the cell it lands in --
 *   a cell of the shared grid: exp(-d^2 / (2 sigma^2)) for the patch getPatch's 3-sigma gate
 *     picks against the placed patch (d = its local height - the patch's mean), 0 when none
 *     passes;
 *   an empty grid cell the particle's own map holds, in a tile inside the window the update
 *     centres on the particle (the reference selects the active grid before matching,
 *     :195-207; the tile comes from the window or the trail): exp(-d^2 / (2 sigma^2)),
 *     d = the patch's height + zPos - the cell's mean;
 * other patches do not count.  weight = the mean score as a float (1 when none counts);
 * p.weight *= pow(weight, 0.1f).                                                            */
int or_map_match(or_filter* f, const eslam_scan_patch* sp, uint32_t m)
{
    const int pmaps = (f->cfg.flags & ESLAM_FLAG_PARTICLE_MAPS) != 0;
    if (!f->has_map) return ESLAM_ERR_NO_ENVIRONMENT;
    if (!f->n) return ESLAM_ERR_NOT_INITIALISED;
    if (pmaps && !f->lm_on) return ESLAM_ERR_OUT_OF_MEMORY;
    const eslam_mls_grid* g = &f->map;
    const double* A = g->global2local;
    static const double id[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    int is_id = 1;
    for (int k = 0; k < 12; ++k) is_id &= A[k] == id[k];
    const uint32_t hx = f->lm_hx, hy = f->lm_hy, wx = f->lm_wx, wy = f->lm_wy, V = f->lm_V;
    const int64_t n = (int64_t)f->n;
#pragma omp parallel for num_threads(f->threads) if (f->threads > 1) schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        double sn, co;
        dm_sincos(f->th[OD(i)], &sn, &co);
        const double bx = f->x[OD(i)] - g->offset_x, by = f->y[OD(i)] - g->offset_y;
        if (!(dm_isfinite(bx) && dm_isfinite(by) && dm_isfinite(f->th[OD(i)]))) continue;
        const double zvar = f->zs[OD(i)] * f->zs[OD(i)];
        int32_t na = 0, nb = 0;
        if (is_id) {
            na = dm_lm_centre(f->x[OD(i)], g->offset_x, 1.0 / g->scale_x);
            nb = dm_lm_centre(f->y[OD(i)], g->offset_y, 1.0 / g->scale_y);
        } else {
            const double px = f->x[OD(i)], py = f->y[OD(i)], pz = f->z[OD(i)];
            na = dm_lm_centre(((A[0] * px + A[1] * py) + A[2] * pz) + A[3], g->offset_x, 1.0 / g->scale_x);
            nb = dm_lm_centre(((A[4] * px + A[5] * py) + A[6] * pz) + A[7], g->offset_y, 1.0 / g->scale_y);
        }
        double sum = 0.0;
        uint32_t cnt = 0;
        for (uint32_t k = 0; k < m; k += OR_MATCH_SAMPLING) {
            const double wz = sp[k].position[2] + f->z[OD(i)];
            double lz = wz;
            uint32_t cm, cn;
            if (is_id) {
                if (dm_merge_cell_mn(bx, by, co, sn, sp[k].position[0], sp[k].position[1], 1.0 / g->scale_x,
                                     1.0 / g->scale_y, g->width, g->height, &cm, &cn) == 0xffffffffu)
                    continue;
            } else {
                const double wx_ = (co * sp[k].position[0] + (-sn) * sp[k].position[1]) + f->x[OD(i)];
                const double wy_ = (sn * sp[k].position[0] + co * sp[k].position[1]) + f->y[OD(i)];
                const double lx = ((A[0] * wx_ + A[1] * wy_) + A[2] * wz) + A[3];
                const double ly = ((A[4] * wx_ + A[5] * wy_) + A[6] * wz) + A[7];
                lz = ((A[8] * wx_ + A[9] * wy_) + A[10] * wz) + A[11];
                const double fm = floor((lx - g->offset_x) * (1.0 / g->scale_x));
                const double fn = floor((ly - g->offset_y) * (1.0 / g->scale_y));
                if (!(fm >= 0.0 && fm < (double)g->width && fn >= 0.0 && fn < (double)g->height)) continue;
                cm = (uint32_t)fm;
                cn = (uint32_t)fn;
            }
            const uint64_t cell = (uint64_t)cn * g->width + cm;
            if (pmaps) {                      /* the particle's own cell first */
                const uint32_t a = cm >> DM_LM_TILE_BITS, b = cn >> DM_LM_TILE_BITS;
                if (dm_lm_inside(a, na, hx, wx) && dm_lm_inside(b, nb, hy, wy)) {
                    const uint32_t pg = lm_tile_page(f->pm_slot + (uint64_t)i * f->lm_R, f->pm_ctr + 2 * i, hx, hy, wx, wy, V, a, b);
                    const uint32_t j = (cm & 7u) + 8u * (cn & 7u);
                    if (pg != DM_LM_NONE && dm_lm_holds(lm_pg(f, pg)->v[2 * j + 1])) {
                        const double d = wz - (double)lm_pg(f, pg)->v[2 * j];
                        sum += dm_exp(-(d * d) / (2.0 * OR_MATCH_SIGMA * OR_MATCH_SIGMA));
                        ++cnt;
                        continue;
                    }
                }
            }
            if (g->cell_start[cell] != g->cell_start[cell + 1]) {        /* a cell of the shared grid */
                double mean, sd;
                const double var = sp[k].stdev * sp[k].stdev + zvar;
                if (or_mls_cell_patch(g, cell, lz, var, &mean, &sd)) {
                    const double d = lz - mean;
                    sum += dm_exp(-(d * d) / (2.0 * OR_MATCH_SIGMA * OR_MATCH_SIGMA));
                }
                ++cnt;
            }
        }
        const float wf = cnt ? (float)(sum / (double)cnt) : 1.0f;
        f->w[OD(i)] *= dm_pow((double)wf, (double)0.1f);
    }
    return 0;
}

/* particle i's own patches: the window's tiles in slot order, then the trail's in entry order,
 * each tile's cells in row order (cells n * width + m, mean, stdev); returns how many it holds */
uint32_t or_get_particle_map(or_filter* f, uint64_t i, uint32_t* cells, float* mean, float* stdev, uint32_t cap)
{
    if (!f->lm_on || i >= f->n) return 0;
    const int32_t* ctr = f->pm_ctr + 2 * i;
    const uint32_t* sl = f->pm_slot + i * f->lm_R;
    const uint32_t S = f->lm_S;
    uint32_t c = 0;
    for (uint32_t s = 0; s < S + f->lm_V; ++s) {
            const uint32_t pg = s < S ? sl[s] : sl[S + 3 * (s - S) + 2];
            if (pg == DM_LM_NONE) continue;
            const uint32_t sa = s % f->lm_wx, sb = s / f->lm_wx;
            const int64_t a = s < S ? dm_lm_tile_of(sa, ctr[0], f->lm_hx, f->lm_wx) : (int32_t)sl[S + 3 * (s - S)];
            const int64_t b = s < S ? dm_lm_tile_of(sb, ctr[1], f->lm_hy, f->lm_wy) : (int32_t)sl[S + 3 * (s - S) + 1];
            const float* v = lm_pg(f, pg)->v;
            for (uint32_t j = 0; j < DM_LM_PAGE_CELLS; ++j) {
                if (!dm_lm_holds(v[2 * j + 1])) continue;
                const uint64_t mm = (uint64_t)(8 * a) + (j & 7u), nn = (uint64_t)(8 * b) + (j >> 3);
                if (c < cap) {
                    cells[c] = (uint32_t)(nn * f->map.width + mm);
                    mean[c] = v[2 * j];
                    stdev[c] = v[2 * j + 1];
                }
                ++c;
            }
    }
    return c;
}

/* pages the particles' maps name (distinct), the pool's use */
uint64_t or_pages_in_use(or_filter* f)
{
    if (!f->lm_on) return 0;
    uint8_t* seen = calloc(f->pg_top ? f->pg_top : 1, 1);
    uint64_t c = 0;
    for (uint64_t i = 0; i < f->n; ++i) {
        const uint32_t* row = f->pm_slot + i * f->lm_R;
        for (uint32_t s = 0; s < f->lm_S + f->lm_V; ++s) {
            const uint32_t p = s < f->lm_S ? row[s] : row[f->lm_S + 3 * (s - f->lm_S) + 2];
            if (p != DM_LM_NONE && !seen[p]) { seen[p] = 1; ++c; }
        }
    }
    free(seen);
    return c;
}

int or_get_debug(or_filter* f, uint32_t* ncp, or_cpoint* cp, double* zdelta, double* zvar)
{
    if (!f->dbg_ncp) return ESLAM_ERR_NOT_INITIALISED;
    uint64_t n = f->n;
    if (ncp) memcpy(ncp, f->dbg_ncp, n * 4);
    if (cp) memcpy(cp, f->dbg_cp, n * ESLAM_MAX_CONTACTS * sizeof(or_cpoint));
    if (zdelta) memcpy(zdelta, f->dbg_zdelta, n * 8);
    if (zvar) memcpy(zvar, f->dbg_zvar, n * 8);
    return 0;
}

/* ---- detmath wrappers --------------------------------------------------------------------- */
double or_dm(int fn, double x, double y)
{
    double s, c;
    switch (fn) {
    case 0: return dm_exp(x);
    case 1: return dm_log(x);
    case 2: dm_sincos(x, &s, &c); return s;
    case 3: dm_sincos(x, &s, &c); return c;
    case 4: return dm_erfc(x);
    case 5: return dm_sqrt(x);
    case 6: return x / y;
    case 7: return dm_normal_pdf_cdf_ratio(x, y);
    case 8: return dm_pow(x, y);
    case 9: { uint64_t v = dm_fx61(x); return dm_from_bits(v); }
    case 10: return dm_erfcx_pos(x);
    case 11: return dm_ldexp(x, (int)y);
    case 12: return dm_weighting_function(x, 0.0, y, 0.0);
    case 13: dm_sincos2pi(x, &s, &c); return s;
    case 14: dm_sincos2pi(x, &s, &c); return c;
    case 15: return dm_log_bm(x);
    case 16: dm_sincos2pi32((uint32_t)x, &s, &c); return s;
    case 17: dm_sincos2pi32((uint32_t)x, &s, &c); return c;
    case 18: dm_box_muller32((uint32_t)x, (uint32_t)y, &s, &c); return s;   /* z0 */
    case 19: dm_box_muller32((uint32_t)x, (uint32_t)y, &s, &c); return c;   /* z1 */
    case 26: { float fs, fc; dm_sincos2pi32f((uint32_t)x, &fs, &fc); return fs; }
    case 27: { float fs, fc; dm_sincos2pi32f((uint32_t)x, &fs, &fc); return fc; }
    default: return NAN;
    }
}

void or_dm_philox(uint64_t seed, uint32_t stream, uint64_t ev, uint64_t gidx, uint32_t call, uint32_t out[4])
{
    dm_philox_ctr c = dm_draw(seed, stream, ev, gidx, call);
    memcpy(out, c.v, 16);
}

void or_dm_philox_raw(const uint32_t ctr[4], uint32_t k0, uint32_t k1, uint32_t out[4])
{
    dm_philox_ctr c;
    memcpy(c.v, ctr, 16);
    c = dm_philox4x32_10(c, k0, k1);
    memcpy(out, c.v, 16);
}

void or_dm_libc_rand(uint32_t seed, uint32_t n, int32_t* out)
{
    dm_libc_rand_state st;
    dm_libc_srand(&st, seed);
    for (uint32_t i = 0; i < n; ++i) out[i] = dm_libc_rand(&st);
}

uint32_t or_dm_minstd_jump(uint32_t x, uint64_t n) { return dm_mulmod31(dm_minstd_pow(n), x); }
double or_dm_limbs_to_double(const uint64_t L[4], int scale) { return dm_limbs_to_double(L, scale); }
void or_dm_fx128(double v, int scale, uint32_t limbs[4]) { dm_fx128_limbs(v, scale, limbs); }
