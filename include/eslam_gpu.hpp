// eslam_gpu.hpp -- C++ façade over the C ABI (eslam_gpu.h) with the reference's class API.
//
// The reference's callers (the Rock orogen task, viz/) use these classes directly; this
// header gives them the same names, constructors, method signatures, configuration fields
// and exception texts, over the MI355X library:
//   eslam::Configuration, ContactModelConfiguration, SurfaceHashConfig, UpdateThreshold
//                               src/Configuration.hpp:12-213
//   eslam::EmbodiedSlamFilter   src/EmbodiedSlamFilter.hpp:58-74 (contact path)
//   eslam::PoseEstimator        src/PoseEstimator.hpp:120-134
//   ParticleFilter<T>           src/ParticleFilter.hpp:34-173 (members of PoseEstimator)
//   eslam::PoseParticle / ContactPoint / PoseDistribution   src/PoseParticle.hpp:20-114
// A call site ports by switching the namespace to eslam::gpu.  The Eigen, base-types,
// odometry and envire types the reference signatures take are not in this image; the
// header carries small stand-ins with the same member names (Vector3d::x(), Affine3d::
// linear() / translation(), Quaterniond(w, x, y, z), base::Pose, BodyContactState::points,
// ...) and templated adapters (toGpu, toAffine, toContactState) that accept the real
// types by those member names.  The map handed to init() is an MlsGrid (the envire
// MLSGrid that EmbodiedSlamFilter::init finds in the environment); odometry::FootContact
// is the contact-odometry front end below.  Header-only; link libeslam_gpu.so.
#ifndef ESLAM_GPU_HPP
#define ESLAM_GPU_HPP

#include <cmath>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "eslam_gpu.h"

namespace eslam {
namespace gpu {

// ---------------------------------------------------------------------------------------
// Eigen-shaped stand-ins (the members the reference's call sites use)
// ---------------------------------------------------------------------------------------
struct Vector2d {
    double v[2] = {0, 0};
    Vector2d() = default;
    Vector2d(double x, double y) : v{x, y} {}
    double& x() { return v[0]; }
    double& y() { return v[1]; }
    double x() const { return v[0]; }
    double y() const { return v[1]; }
    double& operator[](int i) { return v[i]; }
    double operator[](int i) const { return v[i]; }
    double& operator()(int i) { return v[i]; }
    double operator()(int i) const { return v[i]; }
};

struct Vector3d {
    double v[3] = {0, 0, 0};
    Vector3d() = default;
    Vector3d(double x, double y, double z) : v{x, y, z} {}
    static Vector3d Zero() { return Vector3d(); }
    static Vector3d UnitZ() { return Vector3d(0, 0, 1); }
    double& x() { return v[0]; }
    double& y() { return v[1]; }
    double& z() { return v[2]; }
    double x() const { return v[0]; }
    double y() const { return v[1]; }
    double z() const { return v[2]; }
    double& operator[](int i) { return v[i]; }
    double operator[](int i) const { return v[i]; }
    double& operator()(int i) { return v[i]; }
    double operator()(int i) const { return v[i]; }
    double norm() const { return std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }
    Vector3d operator+(const Vector3d& o) const { return Vector3d(v[0] + o.v[0], v[1] + o.v[1], v[2] + o.v[2]); }
    Vector3d operator-(const Vector3d& o) const { return Vector3d(v[0] - o.v[0], v[1] - o.v[1], v[2] - o.v[2]); }
    Vector3d operator*(double s) const { return Vector3d(v[0] * s, v[1] * s, v[2] * s); }
};

struct Matrix3d {
    double m[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};   // row-major
    static Matrix3d Identity()
    {
        Matrix3d r;
        r.m[0] = r.m[4] = r.m[8] = 1.0;
        return r;
    }
    double& operator()(int r, int c) { return m[r * 3 + c]; }
    double operator()(int r, int c) const { return m[r * 3 + c]; }
    Vector3d operator*(const Vector3d& p) const
    {
        Vector3d o;
        for (int r = 0; r < 3; ++r) o.v[r] = (m[r * 3] * p.v[0] + m[r * 3 + 1] * p.v[1]) + m[r * 3 + 2] * p.v[2];
        return o;
    }
    Matrix3d operator*(const Matrix3d& b) const
    {
        Matrix3d o;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) o.m[r * 3 + c] = m[r * 3] * b.m[c] + m[r * 3 + 1] * b.m[3 + c] + m[r * 3 + 2] * b.m[6 + c];
        return o;
    }
    Matrix3d transpose() const
    {
        Matrix3d o;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) o.m[c * 3 + r] = m[r * 3 + c];
        return o;
    }
};

struct Quaterniond {
    double w_ = 1, x_ = 0, y_ = 0, z_ = 0;
    Quaterniond() = default;
    Quaterniond(double w, double x, double y, double z) : w_(w), x_(x), y_(y), z_(z) {}
    explicit Quaterniond(const Matrix3d& R)        // Eigen's rotation-matrix constructor
    {
        const double t = R(0, 0) + R(1, 1) + R(2, 2);
        if (t > 0) {
            const double s = std::sqrt(t + 1.0) * 2;
            w_ = 0.25 * s; x_ = (R(2, 1) - R(1, 2)) / s; y_ = (R(0, 2) - R(2, 0)) / s; z_ = (R(1, 0) - R(0, 1)) / s;
        } else if (R(0, 0) > R(1, 1) && R(0, 0) > R(2, 2)) {
            const double s = std::sqrt(1.0 + R(0, 0) - R(1, 1) - R(2, 2)) * 2;
            w_ = (R(2, 1) - R(1, 2)) / s; x_ = 0.25 * s; y_ = (R(0, 1) + R(1, 0)) / s; z_ = (R(0, 2) + R(2, 0)) / s;
        } else if (R(1, 1) > R(2, 2)) {
            const double s = std::sqrt(1.0 + R(1, 1) - R(0, 0) - R(2, 2)) * 2;
            w_ = (R(0, 2) - R(2, 0)) / s; x_ = (R(0, 1) + R(1, 0)) / s; y_ = 0.25 * s; z_ = (R(1, 2) + R(2, 1)) / s;
        } else {
            const double s = std::sqrt(1.0 + R(2, 2) - R(0, 0) - R(1, 1)) * 2;
            w_ = (R(1, 0) - R(0, 1)) / s; x_ = (R(0, 2) + R(2, 0)) / s; y_ = (R(1, 2) + R(2, 1)) / s; z_ = 0.25 * s;
        }
    }
    static Quaterniond Identity() { return Quaterniond(); }
    double w() const { return w_; }
    double x() const { return x_; }
    double y() const { return y_; }
    double z() const { return z_; }
    Quaterniond conjugate() const { return Quaterniond(w_, -x_, -y_, -z_); }
    Quaterniond inverse() const { return conjugate(); }   // unit quaternions
    Quaterniond operator*(const Quaterniond& b) const
    {
        return Quaterniond(w_ * b.w_ - x_ * b.x_ - y_ * b.y_ - z_ * b.z_, w_ * b.x_ + x_ * b.w_ + y_ * b.z_ - z_ * b.y_,
                           w_ * b.y_ - x_ * b.z_ + y_ * b.w_ + z_ * b.x_, w_ * b.z_ + x_ * b.y_ - y_ * b.x_ + z_ * b.w_);
    }
    Matrix3d toRotationMatrix() const
    {
        Matrix3d R;
        const double w = w_, x = x_, y = y_, z = z_;
        R.m[0] = 1 - 2 * (y * y + z * z); R.m[1] = 2 * (x * y - w * z); R.m[2] = 2 * (x * z + w * y);
        R.m[3] = 2 * (x * y + w * z); R.m[4] = 1 - 2 * (x * x + z * z); R.m[5] = 2 * (y * z - w * x);
        R.m[6] = 2 * (x * z - w * y); R.m[7] = 2 * (y * z + w * x); R.m[8] = 1 - 2 * (x * x + y * y);
        return R;
    }
    Vector3d operator*(const Vector3d& p) const { return toRotationMatrix() * p; }
};

struct Affine3d {
    Matrix3d R = Matrix3d::Identity();
    Vector3d t;
    static Affine3d Identity() { return Affine3d(); }
    Matrix3d& linear() { return R; }
    const Matrix3d& linear() const { return R; }
    Vector3d& translation() { return t; }
    const Vector3d& translation() const { return t; }
    Affine3d operator*(const Affine3d& b) const
    {
        Affine3d o;
        o.R = R * b.R;
        o.t = R * b.t + t;
        return o;
    }
    Vector3d operator*(const Vector3d& p) const { return R * p + t; }
    Affine3d inverse() const
    {
        Affine3d o;
        o.R = R.transpose();
        o.t = (o.R * t) * -1.0;
        return o;
    }
};

// base::Pose2D / base::Pose
struct Pose2D {
    Vector2d position;
    double orientation = 0;
    Pose2D() = default;
    Pose2D(const Vector2d& p, double o) : position(p), orientation(o) {}
};

struct Pose {
    Vector3d position;
    Quaterniond orientation;
    Pose() = default;
    Pose(const Vector3d& p, const Quaterniond& q) : position(p), orientation(q) {}
    explicit Pose(const Affine3d& T) : position(T.translation()), orientation(T.linear()) {}
    Affine3d toTransform() const
    {
        Affine3d T;
        T.R = orientation.toRotationMatrix();
        T.t = position;
        return T;
    }
};

// odometry::BodyContactPoint / BodyContactState; terrain_estimator::TerrainClassification
struct BodyContactPoint {
    Vector3d position;
    float contact = 1.0f;                 // NaN (unknown) passes the contact gate (Q13)
    int groupId = -1;
    float slip = 0.0f;
};

struct BodyContactState {
    std::vector<BodyContactPoint> points;
    double time = 0;
};

struct TerrainClassification {};          // only counted (ltc.size() > 0 forces an update)

// ---------------------------------------------------------------------------------------
// Configuration  src/Configuration.hpp:12-213 (same fields and defaults)
// ---------------------------------------------------------------------------------------
struct UpdateThreshold {
    UpdateThreshold() {}
    UpdateThreshold(double distance, double angle) : distance(distance), angle(angle) {}
    bool test(double distance, double angle) const { return distance > this->distance || angle > this->angle; }
    // test(const Eigen::Affine3d&)  src/Configuration.hpp:23-26: the rotation angle
    // (Eigen::AngleAxisd(linear()).angle() = 2 atan2(|q.vec|, |q.w|)) goes in as the distance and
    // the translation's norm as the angle (Q6, kept)
    bool test(const Affine3d& pdelta) const
    {
        const Quaterniond q(pdelta.linear());
        const double n = std::sqrt(q.x() * q.x() + q.y() * q.y() + q.z() * q.z());
        const double a = n != 0.0 ? 2.0 * std::atan2(n, std::fabs(q.w())) : 0.0;
        const Vector3d& t = pdelta.translation();
        return test(a, std::sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]));
    }
    double distance = 0;
    double angle = 0;
};

struct SurfaceHashConfig {
    bool useHash = false;
    size_t period = 10;
    double percentage = 0.05;
    double avgFactor = 0.1;
    size_t slopeBins = 20;
    size_t angularSteps = 16;
};

struct ContactModelConfiguration {
    bool useSlipUpdate = false;
    bool useShapeUpdate = true;
    size_t minContacts = 3;
    double contactLikelihoodCorrection = 0.33;
    double contactPointRadius = 0.01;
};

struct Configuration {
    unsigned long seed = 42u;
    size_t particleCount = 250;
    size_t minEffective = 50;
    Vector3d initialRotationError = Vector3d(0, 0, 0.1);
    Vector3d initialTranslationError = Vector3d(0.1, 0.1, 1.0);
    double measurementError = 0.1;
    double discountFactor = 0.9;
    double spreadThreshold = 0.9;
    double spreadTranslationFactor = 0.1;
    double spreadRotationFactor = 0.05;
    double slipFactor = 0.05;
    double maxYawDeviation = 15 * M_PI / 180.0;
    UpdateThreshold measurementThreshold = UpdateThreshold(0.1, 10 * M_PI / 180.0);
    UpdateThreshold mappingThreshold = UpdateThreshold(0.02, 5 * M_PI / 180.0);
    UpdateThreshold mappingCameraThreshold = UpdateThreshold(1.0, 30 * M_PI / 180.0);
    double gridSize = 20.0;
    double gridResolution = 0.05;
    double gridThreshold = 0.5;
    double gridPatchThickness = 0.1;
    double gridGapSize = 1.5;
    bool gridUseNegativeInformation = false;
    double maxSensorRange = 3.0;
    bool useVisualUpdate = false;
    ContactModelConfiguration contactModel;
    bool logDebug = false;
    unsigned int logParticlePeriod = 100;
    uint32_t flags = 0;                   // build-specific ESLAM_FLAG_* (not in the reference)
    uint32_t localMapPages = 0;           // build-specific: per-particle map page pool per particle (0: 16)
    uint32_t localMapTrail = 16;          // build-specific: tiles a particle's map keeps behind its window
    uint32_t sumChunkRows = 0;            // build-specific: eslam_config::sum_chunk_rows (0: by particle count)

    // the fields the MI355X path consumes, as the C ABI's POD (hash: the init() argument)
    eslam_config toC(const SurfaceHashConfig& hash = SurfaceHashConfig()) const
    {
        eslam_config c;
        eslam_config_default(&c);
        c.seed = seed;
        c.particle_count = particleCount;
        c.min_effective = minEffective;
        for (int i = 0; i < 3; ++i) {
            c.initial_rotation_error[i] = initialRotationError[i];
            c.initial_translation_error[i] = initialTranslationError[i];
        }
        c.measurement_error = measurementError;
        c.discount_factor = discountFactor;
        c.spread_threshold = spreadThreshold;
        c.spread_translation_factor = spreadTranslationFactor;
        c.spread_rotation_factor = spreadRotationFactor;
        c.slip_factor = slipFactor;
        c.max_yaw_deviation = maxYawDeviation;
        c.measurement_threshold_distance = measurementThreshold.distance;
        c.measurement_threshold_angle = measurementThreshold.angle;
        c.use_slip_update = contactModel.useSlipUpdate;
        c.use_shape_update = contactModel.useShapeUpdate;
        c.min_contacts = contactModel.minContacts;
        c.contact_likelihood_correction = contactModel.contactLikelihoodCorrection;
        c.contact_point_radius = contactModel.contactPointRadius;
        c.hash_use = hash.useHash;
        c.hash_period = hash.period;
        c.hash_percentage = hash.percentage;
        c.hash_avg_factor = hash.avgFactor;
        c.hash_slope_bins = hash.slopeBins;
        c.hash_angular_steps = hash.angularSteps;
        c.log_debug = logDebug;
        c.flags = flags;
        c.max_sensor_range = maxSensorRange;       // the reach of a particle's own map
        c.local_map_pages = localMapPages;
        c.local_map_trail = localMapTrail;
        c.sum_chunk_rows = sumChunkRows;
        return c;
    }
};

// ---------------------------------------------------------------------------------------
// adapters from the reference's own types (templated on their member names, so they take
// eslam::Configuration, Eigen::Affine3d, odometry::BodyContactState, ... as they are)
// ---------------------------------------------------------------------------------------
template <class V> inline Vector3d toVector3(const V& v) { return Vector3d(v[0], v[1], v[2]); }

// eslam::Configuration -> eslam::gpu::Configuration (src/Configuration.hpp:76-211)
template <class RefConfig> Configuration toGpu(const RefConfig& r)
{
    Configuration c;
    c.seed = r.seed;
    c.particleCount = r.particleCount;
    c.minEffective = r.minEffective;
    c.initialRotationError = toVector3(r.initialRotationError);
    c.initialTranslationError = toVector3(r.initialTranslationError);
    c.measurementError = r.measurementError;
    c.discountFactor = r.discountFactor;
    c.spreadThreshold = r.spreadThreshold;
    c.spreadTranslationFactor = r.spreadTranslationFactor;
    c.spreadRotationFactor = r.spreadRotationFactor;
    c.slipFactor = r.slipFactor;
    c.maxYawDeviation = r.maxYawDeviation;
    c.measurementThreshold = UpdateThreshold(r.measurementThreshold.distance, r.measurementThreshold.angle);
    c.mappingThreshold = UpdateThreshold(r.mappingThreshold.distance, r.mappingThreshold.angle);
    c.mappingCameraThreshold = UpdateThreshold(r.mappingCameraThreshold.distance, r.mappingCameraThreshold.angle);
    c.gridSize = r.gridSize;
    c.gridResolution = r.gridResolution;
    c.gridThreshold = r.gridThreshold;
    c.gridPatchThickness = r.gridPatchThickness;
    c.gridGapSize = r.gridGapSize;
    c.gridUseNegativeInformation = r.gridUseNegativeInformation;
    c.maxSensorRange = r.maxSensorRange;
    c.useVisualUpdate = r.useVisualUpdate;
    c.contactModel.useSlipUpdate = r.contactModel.useSlipUpdate;
    c.contactModel.useShapeUpdate = r.contactModel.useShapeUpdate;
    c.contactModel.minContacts = r.contactModel.minContacts;
    c.contactModel.contactLikelihoodCorrection = r.contactModel.contactLikelihoodCorrection;
    c.contactModel.contactPointRadius = r.contactModel.contactPointRadius;
    c.logDebug = r.logDebug;
    c.logParticlePeriod = r.logParticlePeriod;
    return c;
}

template <class RefHash> SurfaceHashConfig toGpuHash(const RefHash& r)
{
    SurfaceHashConfig h;
    h.useHash = r.useHash;
    h.period = r.period;
    h.percentage = r.percentage;
    h.avgFactor = r.avgFactor;
    h.slopeBins = r.slopeBins;
    h.angularSteps = r.angularSteps;
    return h;
}

// Eigen::Affine3d (or anything with linear()(r, c) and translation()[i])
template <class A> Affine3d toAffine(const A& T)
{
    Affine3d o;
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) o.R(r, c) = T.linear()(r, c);
        o.t[r] = T.translation()[r];
    }
    return o;
}

// odometry::BodyContactState (points[i].position / contact / groupId)
template <class BS> BodyContactState toContactState(const BS& bs)
{
    BodyContactState o;
    o.points.resize(bs.points.size());
    for (size_t i = 0; i < bs.points.size(); ++i) {
        o.points[i].position = toVector3(bs.points[i].position);
        o.points[i].contact = bs.points[i].contact;
        o.points[i].groupId = bs.points[i].groupId;
    }
    return o;
}

// ---------------------------------------------------------------------------------------
// MLS grid (the envire::MLSGrid EmbodiedSlamFilter::init takes from the environment) and
// ContactPoint / PoseParticle / PoseDistribution
// ---------------------------------------------------------------------------------------
struct MlsGrid {
    uint32_t width = 0, height = 0;
    double scaleX = 0.1, scaleY = 0.1, offsetX = 0, offsetY = 0;
    Affine3d global2local;                // GridAccess::C_global2local (src/PoseEstimator.hpp:65-71)
    std::vector<uint32_t> cellStart;      // width * height + 1 (CSR; cell = n * width + m)
    std::vector<float> mean, stdev, patchHeight;   // per patch; patchHeight empty = horizontal

    eslam_mls_grid toC() const
    {
        eslam_mls_grid g;
        std::memset(&g, 0, sizeof(g));
        g.width = width;
        g.height = height;
        g.scale_x = scaleX;
        g.scale_y = scaleY;
        g.offset_x = offsetX;
        g.offset_y = offsetY;
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) g.global2local[r * 4 + c] = global2local.R(r, c);
            g.global2local[r * 4 + 3] = global2local.t[r];
        }
        g.cell_start = cellStart.data();
        g.patch_mean = mean.data();
        g.patch_stdev = stdev.data();
        g.patch_height = patchHeight.empty() ? nullptr : patchHeight.data();
        g.n_patches = mean.size();
        return g;
    }
};

struct ContactPoint {                     // src/PoseParticle.hpp:20-43
    Vector3d point;
    double zdiff = INFINITY, zvar = INFINITY, prob = 1.0;
};

struct PoseParticle {                     // src/PoseParticle.hpp:52-86
    Vector2d position;
    double orientation = 0;
    double zPos = 0, zSigma = 0;
    double mprob = 0;
    bool floating = true;
    std::vector<ContactPoint> cpoints;    // filled with Configuration::logDebug (or ESLAM_FLAG_RECORD_CONTACTS)
    std::vector<ContactPoint> spoints;    // slip points: empty (useSlipUpdate's color matching is not on this path)
    Vector3d meas_pos;
    double meas_theta = 0;
    double weight = 0;
};

struct PoseDistribution {                 // src/PoseParticle.hpp:88-114 (without the GMM)
    double time = 0;
    std::vector<PoseParticle> particles;
    Quaterniond orientation;
    BodyContactState bodyState;
};

inline void check(eslam_ctx* ctx, int rc)
{
    if (rc != ESLAM_OK) throw std::runtime_error(eslam_gpu_last_error(ctx));
}

// ---------------------------------------------------------------------------------------
// FootContact: contact-odometry front end (stands in for odometry::FootContact, which the
// reference links from the external odometry package; its algorithm is not in the
// reference, so this one is the build's own and parity-unpinned).  Between two body
// states, every contact point in stance in both (contact >= stanceThreshold, same index)
// is taken to be fixed in the world: the body moved by the mean of R_prev p_prev - R_cur p_cur
// over those points.  The error grows with the travelled distance (constError +
// distError * |delta|, per axis).  It answers what PoseEstimator::project asks
// (src/PoseEstimator.cpp:188-198): getPoseDelta(), getPositionError() and the Gaussian
// getPoseDeltaSample2D() draws from (mean dx, dy, dyaw in the heading frame; diagonal cov).
// ---------------------------------------------------------------------------------------
struct OdometryConfiguration {
    float stanceThreshold = 0.5f;
    Vector3d constError = Vector3d(0.001, 0.001, 0.001);   // position sigma per step (m)
    Vector3d distError = Vector3d(0.05, 0.05, 0.05);       // position sigma per metre travelled
    double constYawError = 1e-3;                            // rad per step
    double distYawError = 0.01;                             // rad per metre
};

class FootContact {
public:
    explicit FootContact(const OdometryConfiguration& config = OdometryConfiguration()) : config_(config) {}

    void update(const BodyContactState& state, const Quaterniond& orientation)
    {
        delta_ = Pose();
        Vector3d d;
        int n = 0;
        if (has_prev_) {
            const Matrix3d Rp = prev_q_.toRotationMatrix(), Rc = orientation.toRotationMatrix();
            for (size_t i = 0; i < state.points.size() && i < prev_.points.size(); ++i) {
                const BodyContactPoint &a = prev_.points[i], &b = state.points[i];
                if (!(a.contact >= config_.stanceThreshold) || !(b.contact >= config_.stanceThreshold)) continue;
                d = d + (Rp * a.position - Rc * b.position);
                ++n;
            }
            if (n) d = d * (1.0 / n);
            // body frame of the previous state
            delta_.position = Rp.transpose() * d;
            delta_.orientation = prev_q_.inverse() * orientation;
            const double yaw_p = yawOf(Rp), yaw_c = yawOf(Rc);
            const double c = std::cos(-yaw_p), s = std::sin(-yaw_p);
            mean2d_[0] = c * d[0] - s * d[1];
            mean2d_[1] = s * d[0] + c * d[1];
            mean2d_[2] = wrap(yaw_c - yaw_p);
        }
        const double dist = std::sqrt(mean2d_[0] * mean2d_[0] + mean2d_[1] * mean2d_[1]);
        for (int i = 0; i < 3; ++i) {
            const double s = config_.constError[i] + config_.distError[i] * dist;
            sigma_[i] = s * s;
        }
        const double sy = config_.constYawError + config_.distYawError * dist;
        yawVar_ = sy * sy;
        prev_ = state;
        prev_q_ = orientation;
        has_prev_ = true;
        stance_ = n;
    }
    const Pose& getPoseDelta() const { return delta_; }
    Matrix3d getPositionError() const
    {
        Matrix3d P;
        P(0, 0) = sigma_[0]; P(1, 1) = sigma_[1]; P(2, 2) = sigma_[2];
        return P;
    }
    // the Gaussian of getPoseDeltaSample2D(): mean (dx, dy, dyaw), covariance row-major
    void getSampleDistribution2D(double mean[3], double cov[9]) const
    {
        std::memcpy(mean, mean2d_, sizeof(mean2d_));
        std::memset(cov, 0, 9 * sizeof(double));
        cov[0] = sigma_[0]; cov[4] = sigma_[1]; cov[8] = yawVar_;
    }
    int stancePoints() const { return stance_; }

private:
    static double yawOf(const Matrix3d& R) { return std::atan2(R(1, 0), R(0, 0)); }
    static double wrap(double a) { return std::atan2(std::sin(a), std::cos(a)); }
    OdometryConfiguration config_;
    BodyContactState prev_;
    Quaterniond prev_q_;
    bool has_prev_ = false;
    Pose delta_;
    double mean2d_[3] = {0, 0, 0};
    double sigma_[3] = {0, 0, 0};
    double yawVar_ = 0;
    int stance_ = 0;
};

// ---------------------------------------------------------------------------------------
// PoseEstimator  src/PoseEstimator.hpp:120-134 (+ the ParticleFilter<T> members it inherits)
// ---------------------------------------------------------------------------------------
// one cell of the scan's MLS (the scanMap of processMap): position in the yaw-free body
// frame, sensor sigma
struct ScanPatch {
    Vector3d position;
    double stdev = 0.0;
};

struct SurfaceHash {                      // src/SurfaceHash.hpp:155-231: built on the device
    SurfaceHashConfig config;
    void setConfiguration(const SurfaceHashConfig& c) { config = c; }
};

class PoseEstimator {
public:
    typedef PoseParticle Particle;

    // src/PoseEstimator.cpp:13-25; device: the MI355X (one per process; multi-GPU: setCommRccl)
    PoseEstimator(FootContact& odometry, const Configuration& config, int device = 0,
                  const SurfaceHashConfig& hash = SurfaceHashConfig())
        : odometry_(odometry), config_(config)
    {
        const eslam_config c = config.toC(hash);
        if (eslam_gpu_create(&c, device, &ctx_) != ESLAM_OK) throw std::runtime_error("eslam_gpu_create failed (no MI355X visible?)");
    }
    ~PoseEstimator() { eslam_gpu_destroy(ctx_); }   // never collective (include/eslam_gpu.h)
    // multi-GPU: the collective end of a sharded filter's life -- every rank calls it before
    // the filter is destroyed, completing an exchange the rank may still owe
    void finish() { check(ctx_, eslam_gpu_finish(ctx_)); }
    PoseEstimator(const PoseEstimator&) = delete;
    PoseEstimator& operator=(const PoseEstimator&) = delete;

    // setEnvironment(env, map, useShared)  src/PoseEstimator.cpp:49-62: useShared = false gives
    // every particle its own map (the shared grid plus its own patches; before init)
    void setEnvironment(const MlsGrid& env, bool useShared = true)
    {
        const eslam_mls_grid g = env.toC();
        check(ctx_, eslam_gpu_set_map(ctx_, &g));
        check(ctx_, eslam_gpu_set_particle_maps(ctx_, useShared ? 0 : 1));
    }
    // cloneMaps  src/PoseEstimator.cpp:31-47: the copies a resample made share their ancestor's
    // patches until the next map update gives each a private copy (copy on write), so there is
    // nothing to do here
    void cloneMaps() {}
    // the match half of EmbodiedSlamFilter::processMap(scanMap, match, update)
    // (src/EmbodiedSlamFilter.cpp:214-221): every particle's weight *= pow(weight, 0.1f)
    void matchMaps(const std::vector<ScanPatch>& scan)
    {
        flush();
        invalidate();
        std::vector<eslam_scan_patch> p(scan.size());
        for (size_t k = 0; k < scan.size(); ++k) {
            for (int i = 0; i < 3; ++i) p[k].position[i] = scan[k].position[i];
            p[k].stdev = scan[k].stdev;
        }
        check(ctx_, eslam_gpu_map_match(ctx_, p.data(), (uint32_t)p.size()));
    }
    // the merge half of EmbodiedSlamFilter::processMap(scanMap, match, update)
    // (src/EmbodiedSlamFilter.cpp:179-232) for per-particle maps: the scan's patches in the
    // yaw-free body frame, placed at every particle's pose
    void updateMaps(const std::vector<ScanPatch>& scan)
    {
        flush();
        std::vector<eslam_scan_patch> p(scan.size());
        for (size_t k = 0; k < scan.size(); ++k) {
            for (int i = 0; i < 3; ++i) p[k].position[i] = scan[k].position[i];
            p[k].stdev = scan[k].stdev;
        }
        check(ctx_, eslam_gpu_map_update(ctx_, p.data(), (uint32_t)p.size()));
    }

    // init(numParticles, hash)  src/PoseEstimator.cpp:75-86 (the hash is built on the device
    // from the environment's grid; the SurfaceHashConfig was given at construction)
    void init(int numParticles, SurfaceHash* hash)
    {
        if (!hash) throw std::runtime_error("could not sample from pose hash.");
        discardView();
        check(ctx_, eslam_gpu_hash_create(ctx_));
        check(ctx_, eslam_gpu_init_hash(ctx_, (uint64_t)numParticles));
    }
    // init(numParticles, mu, sigma, zpos, zsigma)  src/PoseEstimator.cpp:88-102
    void init(int numParticles, const Pose2D& mu, const Pose2D& sigma, double zpos = 0, double zsigma = 0)
    {
        const double m[3] = {mu.position.x(), mu.position.y(), mu.orientation};
        const double s[3] = {sigma.position.x(), sigma.position.y(), sigma.orientation};
        discardView();
        check(ctx_, eslam_gpu_init_gaussian(ctx_, (uint64_t)numParticles, m, s, zpos, zsigma));
    }

    // project(state, orientation)  src/PoseEstimator.cpp:184-242 (the odometry has been updated)
    void project(const BodyContactState& state, const Quaterniond& orientation)
    {
        const eslam_step_input in = makeInput(state, orientation, Vector3d(), 0);
        flush();
        invalidate();
        check(ctx_, eslam_gpu_project(ctx_, &in));
    }
    // update(state, orientation, ltc)  src/PoseEstimator.cpp:244-255
    void update(const BodyContactState& state, const Quaterniond& orientation, const std::vector<TerrainClassification>& ltc)
    {
        const eslam_step_input in = makeInput(state, orientation, Vector3d(), ltc.size());
        flush();
        invalidate();
        check(ctx_, eslam_gpu_update(ctx_, &in));
        check(ctx_, eslam_gpu_sync(ctx_, &last_));
    }

    // ParticleFilter<T>  src/ParticleFilter.hpp:34-173
    double getWeightsSum()
    {
        flush();
        double s = 0;
        check(ctx_, eslam_gpu_get_weights_sum(ctx_, &s));
        return s;
    }
    double getWeightAvg() { return getWeightsSum() / (double)size(); }
    double normalizeWeights()
    {
        flush();
        invalidate();
        double e = 0;
        check(ctx_, eslam_gpu_normalize_weights(ctx_, &e));
        return e;
    }
    void resample()
    {
        flush();
        invalidate();
        check(ctx_, eslam_gpu_resample(ctx_));
    }
    size_t getBestParticleIndex() const
    {
        flush();
        uint64_t i = 0;
        check(ctx_, eslam_gpu_get_best_particle_index(ctx_, &i));
        return (size_t)i;
    }
    // getCentroid  src/PoseEstimator.cpp:354-383 (normalises in place, Q15)
    Pose getCentroid()
    {
        flush();
        invalidate();                     // normalises the weights
        double p[3], q[4];
        check(ctx_, eslam_gpu_get_centroid(ctx_, p, q));
        return Pose(Vector3d(p[0], p[1], p[2]), Quaterniond(q[0], q[1], q[2], q[3]));
    }

    // getParticles(): the particles as a vector the caller may edit, like the reference's
    // std::vector<Particle>& (src/ParticleFilter.hpp:150-153; processMap edits weights through
    // it, src/EmbodiedSlamFilter.cpp:183-220).  The particles live in HBM: the vector is
    // downloaded on first use after the device changed them, and edits -- pose, zPos, zSigma,
    // weight, mprob, floating, the number of cpoints, or the vector's size -- are written back
    // (eslam_gpu_write_particles, or a whole new set when the size changed) before the next
    // call that uses the particles on the device.  With logDebug it carries cpoints / meas_pos /
    // meas_theta of the last update.  The reference stays valid; its contents are those of the
    // last download.
    std::vector<Particle>& getParticles()
    {
        if (!view_valid_) {
            view_ = getParticles(0, 1, size());
            shadow_.resize(view_.size());
            for (size_t i = 0; i < view_.size(); ++i) shadow_[i] = hot(view_[i]);
            view_valid_ = true;
        }
        return view_;
    }
    // particles first, first + stride, ... (count): a device-side gather, for logging; a copy
    // (edits to it are not written back)
    std::vector<Particle> getParticles(size_t first, size_t stride, size_t count)
    {
        flush();
        std::vector<eslam_particle_record> rec(count);
        // contact points per particle: at most the contacts of the last step
        const uint32_t maxc = config_.logDebug || (config_.flags & ESLAM_FLAG_RECORD_CONTACTS) ? (last_m_ ? last_m_ : 1) : 0;
        std::vector<eslam_cpoint> cp(maxc ? count * maxc : 0);
        check(ctx_, eslam_gpu_download_records(ctx_, first, stride, count, rec.data(), maxc ? cp.data() : nullptr, maxc));
        std::vector<Particle> particles(count);
        for (size_t k = 0; k < count; ++k) {
            const eslam_particle_record& r = rec[k];
            Particle& p = particles[k];
            p.position = Vector2d(r.position[0], r.position[1]);
            p.orientation = r.orientation;
            p.zPos = r.zpos;
            p.zSigma = r.zsigma;
            p.mprob = r.mprob;
            p.weight = r.weight;
            p.floating = r.floating != 0;
            p.meas_pos = Vector3d(r.meas_pos[0], r.meas_pos[1], r.meas_pos[2]);
            p.meas_theta = r.meas_theta;
            p.cpoints.clear();
            p.spoints.clear();
            if (maxc) {
                const uint32_t nc = r.n_cpoints < maxc ? r.n_cpoints : maxc;
                for (uint32_t q = 0; q < nc; ++q) {
                    const eslam_cpoint& c = cp[k * maxc + q];
                    ContactPoint o;
                    o.point = Vector3d(c.point[0], c.point[1], c.point[2]);
                    o.zdiff = c.zdiff;
                    o.zvar = c.zvar;
                    o.prob = c.prob;
                    p.cpoints.push_back(o);
                }
            } else {
                p.cpoints.resize(r.n_cpoints);        // the count (cpoints.size()) without the capture
            }
        }
        return particles;
    }
    void setParticles(const std::vector<Particle>& in)
    {
        discardView();
        replaceSet(in);
    }
    size_t size() const
    {
        uint64_t n = 0;
        check(ctx_, eslam_gpu_particle_count(ctx_, &n));
        return (size_t)n;
    }

private:
    void replaceSet(const std::vector<Particle>& in) const
    {
        const size_t n = in.size();
        std::vector<double> x(n), y(n), th(n), z(n), zs(n), w(n), mp(n);
        std::vector<uint8_t> fl(n), nc(n);
        for (size_t i = 0; i < n; ++i) {
            x[i] = in[i].position.x(); y[i] = in[i].position.y(); th[i] = in[i].orientation; z[i] = in[i].zPos;
            zs[i] = in[i].zSigma; w[i] = in[i].weight; mp[i] = in[i].mprob; fl[i] = in[i].floating;
            nc[i] = (uint8_t)in[i].cpoints.size();
        }
        eslam_particles p = {x.data(), y.data(), th.data(), z.data(), zs.data(), w.data(), mp.data(), fl.data(), nc.data()};
        check(ctx_, eslam_gpu_upload_particles(ctx_, n, &p));
    }

public:

    // multi-GPU (the reference has one CPU filter): this estimator becomes shard `rank` of
    // an nGlobal-particle filter over an RCCL communicator the library drives.  Rank 0 calls
    // rcclUniqueId(), the caller broadcasts the id, every rank calls setCommRccl
    // (collective) before init; shardGbase: the first global index of every rank + nGlobal.
    static std::vector<uint8_t> rcclUniqueId()
    {
        std::vector<uint8_t> id(ESLAM_RCCL_ID_BYTES);
        if (eslam_gpu_rccl_unique_id(id.data()) != ESLAM_OK) throw std::runtime_error("eslam_gpu_rccl_unique_id failed");
        return id;
    }
    void setCommRccl(int nranks, int rank, const std::vector<uint8_t>& id, uint64_t nGlobal,
                     const std::vector<uint64_t>& shardGbase)
    {
        if (id.size() != ESLAM_RCCL_ID_BYTES || shardGbase.size() != (size_t)nranks + 1)
            throw std::runtime_error("setCommRccl: bad id or shard table");
        check(ctx_, eslam_gpu_set_comm_rccl(ctx_, nranks, rank, id.data(), nGlobal, shardGbase.data()));
        sharded_ = nranks > 0;
    }
    // the same with caller-supplied collectives (eslam_gpu_set_comm); comm == nullptr: one GPU
    void setComm(const eslam_comm* comm, uint64_t nGlobal, const std::vector<uint64_t>& shardGbase)
    {
        check(ctx_, eslam_gpu_set_comm(ctx_, comm, nGlobal, comm ? shardGbase.data() : nullptr));
        sharded_ = comm != nullptr;
    }
    bool sharded() const { return sharded_; }

    // write the edits made to the getParticles() vector back to the device (a no-op without
    // any); every call above that uses the particles on the device runs it first.  On a
    // sharded filter the write-back is collective (eslam_gpu_write_particles): a rank holding
    // a view writes back even without edits, so the ranks stay matched as long as they call
    // getParticles() at the same points (SPMD order, include/eslam_gpu.h).  The contract is on
    // the caller: a rank that never took a view (view_valid_ false) skips the write-back, so
    // either every rank calls getParticles() at a point or none does
    void flush() const
    {
        if (!view_valid_) return;
        if (view_.size() != shadow_.size()) {          // the caller resized the set: replace it
            view_valid_ = false;
            replaceSet(view_);
            return;
        }
        size_t lo = view_.size(), hi = 0;
        for (size_t i = 0; i < view_.size(); ++i) {
            const Hot h = hot(view_[i]);
            if (std::memcmp(&h, &shadow_[i], sizeof(Hot)) != 0) {
                if (i < lo) lo = i;
                hi = i + 1;
                shadow_[i] = h;
            }
        }
        if (lo >= hi) {
            if (!sharded()) return;
            lo = hi = 0;
        }
        const size_t n = hi - lo;
        std::vector<double> x(n), y(n), th(n), z(n), zs(n), w(n), mp(n);
        std::vector<uint8_t> fl(n), nc(n);
        for (size_t k = 0; k < n; ++k) {
            const Hot& h = shadow_[lo + k];
            x[k] = h.v[0]; y[k] = h.v[1]; th[k] = h.v[2]; z[k] = h.v[3]; zs[k] = h.v[4]; w[k] = h.v[5]; mp[k] = h.v[6];
            fl[k] = h.floating; nc[k] = h.ncp;
        }
        eslam_particles p = {x.data(), y.data(), th.data(), z.data(), zs.data(), w.data(), mp.data(), fl.data(), nc.data()};
        check(ctx_, eslam_gpu_write_particles(ctx_, lo, n, &p));
    }
    // the device is about to change the particles: the next getParticles() downloads again
    void invalidate() { view_valid_ = false; }

    const eslam_update_info& lastUpdate() const { return last_; }
    eslam_ctx* handle() const { return ctx_; }
    FootContact& odometry() { return odometry_; }

    // the C ABI's per-step input: the body state, orientation and this estimator's odometry
    eslam_step_input makeInput(const BodyContactState& state, const Quaterniond& orientation, const Vector3d& translation,
                               size_t ltcCount) const
    {
        eslam_step_input in;
        std::memset(&in, 0, sizeof(in));
        in.body2odometry_rot[0] = orientation.w();
        in.body2odometry_rot[1] = orientation.x();
        in.body2odometry_rot[2] = orientation.y();
        in.body2odometry_rot[3] = orientation.z();
        for (int i = 0; i < 3; ++i) in.body2odometry_trans[i] = translation[i];
        const Pose& d = odometry_.getPoseDelta();
        for (int i = 0; i < 3; ++i) in.pose_delta_trans[i] = d.position[i];
        in.position_error_zz = odometry_.getPositionError()(2, 2);
        odometry_.getSampleDistribution2D(in.sample_mean, in.sample_cov);
        if (state.points.size() > ESLAM_MAX_CONTACTS) throw std::runtime_error("too many contact points");
        in.n_contacts = (uint32_t)state.points.size();
        last_m_ = in.n_contacts;
        in.ltc_count = (uint32_t)ltcCount;
        for (size_t i = 0; i < state.points.size(); ++i) {
            for (int k = 0; k < 3; ++k) in.contacts[i].position[k] = state.points[i].position[k];
            in.contacts[i].contact = state.points[i].contact;
            in.contacts[i].group_id = state.points[i].groupId;
        }
        return in;
    }

private:
    // the fields of a particle the device holds, as last downloaded or written back
    struct Hot {
        double v[7];                      // x, y, orientation, zPos, zSigma, weight, mprob
        uint8_t floating, ncp, pad[6];
    };
    static Hot hot(const Particle& p)
    {
        Hot h;
        std::memset(&h, 0, sizeof(h));
        h.v[0] = p.position.x(); h.v[1] = p.position.y(); h.v[2] = p.orientation; h.v[3] = p.zPos;
        h.v[4] = p.zSigma; h.v[5] = p.weight; h.v[6] = p.mprob;
        h.floating = p.floating ? 1 : 0;
        h.ncp = (uint8_t)(p.cpoints.size() & 0x7f);
        return h;
    }
    // a new particle set replaces the view without writing it back
    void discardView() const { view_valid_ = false; }

    FootContact& odometry_;
    Configuration config_;
    eslam_ctx* ctx_ = nullptr;
    eslam_update_info last_ = {};
    mutable std::vector<Particle> view_;           // getParticles()
    mutable std::vector<Hot> shadow_;              // view_ as the device holds it
    mutable bool view_valid_ = false;
    mutable uint32_t last_m_ = 0;
    bool sharded_ = false;
};

// ---------------------------------------------------------------------------------------
// EmbodiedSlamFilter  src/EmbodiedSlamFilter.hpp:58-74 (the contact path)
// ---------------------------------------------------------------------------------------
class EmbodiedSlamFilter {
public:
    // src/EmbodiedSlamFilter.cpp:13-23 (device: the MI355X this filter runs on)
    EmbodiedSlamFilter(const OdometryConfiguration& odometryConfig, const Configuration& eslamConfig, int device = 0)
        : eslamConfig_(eslamConfig), odometry_(odometryConfig), device_(device)
    {
    }

    // init(env, pose, useSharedMap, hashConfig)  src/EmbodiedSlamFilter.cpp:70-128: the grid
    // is the environment's MLS grid; with hashConfig.useHash the particles are drawn from the
    // surface hash built on the device, else around the pose
    void init(const MlsGrid& env, const Pose& pose, bool useSharedMap = true,
              const SurfaceHashConfig& hashConfig = SurfaceHashConfig())
    {
        filter_.reset(new PoseEstimator(odometry_, eslamConfig_, device_, hashConfig));
        filter_->setEnvironment(env, useSharedMap);
        filter_->invalidate();
        sharedMap_ = useSharedMap;
        const double p[3] = {pose.position.x(), pose.position.y(), pose.position.z()};
        const double q[4] = {pose.orientation.w(), pose.orientation.x(), pose.orientation.y(), pose.orientation.z()};
        check(filter_->handle(), eslam_gpu_init_pose(filter_->handle(), p, q));
        update_idx_ = 0;
    }

    // update(body2odometry, bs, ltc)  src/EmbodiedSlamFilter.cpp:353-369: odometry.update,
    // project, and the measurement update when UpdateThreshold::test passes (Q6) or ltc is
    // non-empty
    bool update(const Affine3d& body2odometry, const BodyContactState& bs, const std::vector<TerrainClassification>& ltc)
    {
        PoseEstimator& f = estimator();
        const Quaterniond orientation(body2odometry.linear());
        odometry_.update(bs, orientation);
        const eslam_step_input in = f.makeInput(bs, orientation, body2odometry.translation(), ltc.size());
        int updated = 0;
        f.flush();                        // edits made through getParticles()
        f.invalidate();
        check(f.handle(), eslam_gpu_step(f.handle(), &in, &updated));
        if (updated) ++update_idx_;
        last_state_ = bs;
        last_orientation_ = orientation;
        return updated != 0;
    }

    // processMap(scanMap, match, update)  src/EmbodiedSlamFilter.cpp:179-232 with the scan's
    // MLS as patches: update merges them into every particle's own map (useSharedMap = false;
    // the reference's update-only call, src/EmbodiedSlamFilter.cpp:340-342); match weights every
    // particle against its map first -- the shared grid (useSharedMap = true: the laser path's
    // match-only call, :342-344) or its own map (the build's match rule, eslam_gpu_map_match)
    void processMap(const std::vector<ScanPatch>& scanMap, bool match, bool update)
    {
        if (match) estimator().matchMaps(scanMap);
        if (update && !sharedMap_) estimator().updateMaps(scanMap);
    }

    std::vector<PoseParticle>& getParticles() { return estimator().getParticles(); }
    size_t getBestParticleIndex() const { return estimator().getBestParticleIndex(); }
    Affine3d getCentroid() { return estimator().getCentroid().toTransform(); }

    // the particle distribution a Rock task logs every logParticlePeriod-th update
    // (src/Configuration.hpp:203-212; PoseDistribution src/PoseParticle.hpp:88-114): true when
    // the last update is one to log (period 0: never, 1: every update)
    bool logDue() const
    {
        const unsigned p = eslamConfig_.logParticlePeriod;
        return p != 0 && update_idx_ != 0 && (update_idx_ - 1) % p == 0;
    }
    // stride: every stride-th particle (a device-side subsample for large filters)
    PoseDistribution getPoseDistribution(size_t stride = 1)
    {
        PoseDistribution d;
        PoseEstimator& f = estimator();
        const size_t n = f.size();
        if (stride == 0) stride = 1;
        d.particles = f.getParticles(0, stride, n ? (n - 1) / stride + 1 : 0);
        d.orientation = last_orientation_;
        d.bodyState = last_state_;
        d.time = last_state_.time;
        return d;
    }

    PoseEstimator& estimator()
    {
        if (!filter_) throw std::runtime_error("EmbodiedSlamFilter: init() has not been called");
        return *filter_;
    }
    const PoseEstimator& estimator() const
    {
        if (!filter_) throw std::runtime_error("EmbodiedSlamFilter: init() has not been called");
        return *filter_;
    }
    FootContact& odometry() { return odometry_; }

private:
    struct Holder {                       // unique_ptr without <memory> in the public surface
        PoseEstimator* p = nullptr;
        ~Holder() { delete p; }
        void reset(PoseEstimator* q) { delete p; p = q; }
        explicit operator bool() const { return p != nullptr; }
        PoseEstimator& operator*() const { return *p; }
        PoseEstimator* operator->() const { return p; }
    };
    Configuration eslamConfig_;
    FootContact odometry_;
    int device_;
    Holder filter_;
    bool sharedMap_ = true;
    uint64_t update_idx_ = 0;
    BodyContactState last_state_;
    Quaterniond last_orientation_;
};

}  // namespace gpu
}  // namespace eslam

#endif
