// eslam_gpu.hpp -- C++ façade over the C ABI (eslam_gpu.h) with the reference's class API.
//
// Mirrors the public surface of the reference classes that the Rock task calls, so a
// maintainer can swap the CPU filter for the MI355X one:
//   eslam::EmbodiedSlamFilter   src/EmbodiedSlamFilter.hpp:58-74
//   eslam::PoseEstimator        src/PoseEstimator.hpp:120-134
//   eslam::ParticleFilter<T>    src/ParticleFilter.hpp:34-173
// Same method names and argument meaning; errors are thrown as std::runtime_error with the
// reference's messages (eslam_gpu_last_error).  The Eigen / base-types / odometry / envire
// arguments are replaced by small POD types (this image has none of those libraries);
// INTEGRATION.md shows the adapters from the real types.  Header-only; link libeslam_gpu.so.
#ifndef ESLAM_GPU_HPP
#define ESLAM_GPU_HPP

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "eslam_gpu.h"

namespace eslam {
namespace gpu {

// eslam::Configuration (src/Configuration.hpp:76-111), the fields consumed on the path
struct Configuration : eslam_config {
    Configuration() { eslam_config_default(this); }
};

struct Pose2D {                           // base::Pose2D
    double x = 0, y = 0, orientation = 0;
};

struct Pose {                             // base::Pose / base::Affine3d as position + quaternion
    double position[3] = {0, 0, 0};
    double orientation[4] = {1, 0, 0, 0}; // w, x, y, z
};

struct BodyContactPoint {                 // odometry::BodyContactPoint
    double position[3] = {0, 0, 0};
    float contact = 1.0f;
    int groupId = -1;
};

// What odometry::FootContact yields after odometry.update(bs, orientation)
// (src/EmbodiedSlamFilter.cpp:357, src/PoseEstimator.cpp:188-198)
struct OdometryOutputs {
    double poseDeltaTranslation[3] = {0, 0, 0};   // getPoseDelta().position
    double positionErrorZZ = 0;                   // getPositionError()(2,2)
    double sampleMean[3] = {0, 0, 0};             // mean of getPoseDeltaSample2D() (dx, dy, dtheta)
    double sampleCov[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
};

struct PoseParticle {                     // eslam::PoseParticle (src/PoseParticle.hpp:52-86)
    double position[2];
    double orientation, zPos, zSigma, weight, mprob;
    bool floating;
    unsigned nContactPoints;              // cpoints.size()
};

inline void check(eslam_ctx* ctx, int rc)
{
    if (rc != ESLAM_OK) throw std::runtime_error(eslam_gpu_last_error(ctx));
}

// ParticleFilter<PoseParticleGA> + PoseEstimator on one GPU (or one shard)
class PoseEstimator {
public:
    explicit PoseEstimator(const Configuration& config, int device = 0) : config_(config)
    {
        const int rc = eslam_gpu_create(&config_, device, &ctx_);
        if (rc != ESLAM_OK) throw std::runtime_error("eslam_gpu_create failed (no MI355X visible?)");
    }
    ~PoseEstimator() { eslam_gpu_destroy(ctx_); }
    PoseEstimator(const PoseEstimator&) = delete;
    PoseEstimator& operator=(const PoseEstimator&) = delete;

    // PoseEstimator::setEnvironment(env, map, useShared=true): the MLS grid of the map
    void setEnvironment(const eslam_mls_grid& grid) { check(ctx_, eslam_gpu_set_map(ctx_, &grid)); }

    // PoseEstimator::init(numParticles, mu, sigma, zpos, zsigma)  src/PoseEstimator.cpp:88-102
    void init(int numParticles, const Pose2D& mu, const Pose2D& sigma, double zpos = 0, double zsigma = 0)
    {
        const double m[3] = {mu.x, mu.y, mu.orientation}, s[3] = {sigma.x, sigma.y, sigma.orientation};
        check(ctx_, eslam_gpu_init_gaussian(ctx_, (uint64_t)numParticles, m, s, zpos, zsigma));
    }

    // PoseEstimator::project(state, orientation)  src/PoseEstimator.cpp:184-242
    void project(const std::vector<BodyContactPoint>& state, const double orientation[4], const OdometryOutputs& odo)
    {
        const eslam_step_input in = make_input(state, orientation, nullptr, odo, 0);
        check(ctx_, eslam_gpu_project(ctx_, &in));
    }

    // PoseEstimator::update(state, orientation, ltc)  src/PoseEstimator.cpp:244-255
    void update(const std::vector<BodyContactPoint>& state, const double orientation[4], const OdometryOutputs& odo,
                size_t ltcCount = 0)
    {
        const eslam_step_input in = make_input(state, orientation, nullptr, odo, ltcCount);
        check(ctx_, eslam_gpu_update(ctx_, &in));
        check(ctx_, eslam_gpu_sync(ctx_, &last_));
    }

    // ParticleFilter<T> (src/ParticleFilter.hpp:34-173)
    double getWeightsSum()
    {
        double s = 0;
        check(ctx_, eslam_gpu_get_weights_sum(ctx_, &s));
        return s;
    }
    double getWeightAvg() { return getWeightsSum() / (double)size(); }      // :41-44
    double normalizeWeights()
    {
        double e = 0;
        check(ctx_, eslam_gpu_normalize_weights(ctx_, &e));
        return e;
    }
    void resample() { check(ctx_, eslam_gpu_resample(ctx_)); }
    size_t getBestParticleIndex()
    {
        uint64_t i = 0;
        check(ctx_, eslam_gpu_get_best_particle_index(ctx_, &i));
        return (size_t)i;
    }
    // PoseEstimator::getCentroid  src/PoseEstimator.cpp:354-383
    Pose getCentroid()
    {
        Pose p;
        check(ctx_, eslam_gpu_get_centroid(ctx_, p.position, p.orientation));
        return p;
    }

    // getParticles(): a copy (the reference hands out a mutable reference; write back with
    // setParticles)
    std::vector<PoseParticle> getParticles()
    {
        const size_t n = size();
        std::vector<double> x(n), y(n), th(n), z(n), zs(n), w(n), mp(n);
        std::vector<uint8_t> fl(n), nc(n);
        eslam_particles p = {x.data(), y.data(), th.data(), z.data(), zs.data(), w.data(), mp.data(), fl.data(), nc.data()};
        check(ctx_, eslam_gpu_download_particles(ctx_, &p));
        std::vector<PoseParticle> out(n);
        for (size_t i = 0; i < n; ++i)
            out[i] = PoseParticle{{x[i], y[i]}, th[i], z[i], zs[i], w[i], mp[i], fl[i] != 0, nc[i]};
        return out;
    }
    void setParticles(const std::vector<PoseParticle>& in)
    {
        const size_t n = in.size();
        std::vector<double> x(n), y(n), th(n), z(n), zs(n), w(n), mp(n);
        std::vector<uint8_t> fl(n), nc(n);
        for (size_t i = 0; i < n; ++i) {
            x[i] = in[i].position[0]; y[i] = in[i].position[1]; th[i] = in[i].orientation; z[i] = in[i].zPos;
            zs[i] = in[i].zSigma; w[i] = in[i].weight; mp[i] = in[i].mprob; fl[i] = in[i].floating;
            nc[i] = (uint8_t)in[i].nContactPoints;
        }
        eslam_particles p = {x.data(), y.data(), th.data(), z.data(), zs.data(), w.data(), mp.data(), fl.data(), nc.data()};
        check(ctx_, eslam_gpu_upload_particles(ctx_, n, &p));
    }
    size_t size()
    {
        uint64_t n = 0;
        check(ctx_, eslam_gpu_particle_count(ctx_, &n));
        return (size_t)n;
    }

    // multi-GPU (the reference has one CPU filter): this estimator becomes shard `rank` of an
    // nGlobal-particle filter over an RCCL communicator the library drives itself.  Rank 0
    // calls rcclUniqueId(), the caller broadcasts the id, every rank calls setCommRccl
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
    }

    const eslam_update_info& lastUpdate() const { return last_; }
    eslam_ctx* handle() { return ctx_; }

    static eslam_step_input make_input(const std::vector<BodyContactPoint>& state, const double orientation[4],
                                       const double* translation, const OdometryOutputs& odo, size_t ltcCount)
    {
        eslam_step_input in;
        std::memset(&in, 0, sizeof(in));
        std::memcpy(in.body2odometry_rot, orientation, sizeof(in.body2odometry_rot));
        if (translation) std::memcpy(in.body2odometry_trans, translation, sizeof(in.body2odometry_trans));
        std::memcpy(in.pose_delta_trans, odo.poseDeltaTranslation, sizeof(in.pose_delta_trans));
        in.position_error_zz = odo.positionErrorZZ;
        std::memcpy(in.sample_mean, odo.sampleMean, sizeof(in.sample_mean));
        std::memcpy(in.sample_cov, odo.sampleCov, sizeof(in.sample_cov));
        if (state.size() > ESLAM_MAX_CONTACTS) throw std::runtime_error("too many contact points");
        in.n_contacts = (uint32_t)state.size();
        in.ltc_count = (uint32_t)ltcCount;
        for (size_t i = 0; i < state.size(); ++i) {
            std::memcpy(in.contacts[i].position, state[i].position, sizeof(in.contacts[i].position));
            in.contacts[i].contact = state[i].contact;
            in.contacts[i].group_id = state[i].groupId;
        }
        return in;
    }

protected:
    Configuration config_;
    eslam_ctx* ctx_ = nullptr;
    eslam_update_info last_ = {};
};

// EmbodiedSlamFilter (contact path)  src/EmbodiedSlamFilter.hpp:58-74
class EmbodiedSlamFilter {
public:
    explicit EmbodiedSlamFilter(const Configuration& eslamConfig, int device = 0) : filter_(eslamConfig, device) {}

    // init(env, pose, useSharedMap=true)  src/EmbodiedSlamFilter.cpp:70-177 (non-hash branch)
    void init(const eslam_mls_grid& env, const Pose& pose)
    {
        filter_.setEnvironment(env);
        check(filter_.handle(), eslam_gpu_init_pose(filter_.handle(), pose.position, pose.orientation));
    }

    // update(body2odometry, bs, ltc)  src/EmbodiedSlamFilter.cpp:353-369; returns whether
    // the measurement update ran
    bool update(const Pose& body2odometry, const std::vector<BodyContactPoint>& bs, const OdometryOutputs& odo,
                size_t ltcCount = 0)
    {
        const eslam_step_input in =
            PoseEstimator::make_input(bs, body2odometry.orientation, body2odometry.position, odo, ltcCount);
        int updated = 0;
        check(filter_.handle(), eslam_gpu_step(filter_.handle(), &in, &updated));
        return updated != 0;
    }

    std::vector<PoseParticle> getParticles() { return filter_.getParticles(); }
    size_t getBestParticleIndex() { return filter_.getBestParticleIndex(); }
    Pose getCentroid() { return filter_.getCentroid(); }
    PoseEstimator& estimator() { return filter_; }

private:
    PoseEstimator filter_;
};

}  // namespace gpu
}  // namespace eslam

#endif
