// C++ façade (include/eslam_gpu.hpp) on the GPU.  The first block is a reference-shaped
// call site -- the Rock task's use of eslam::EmbodiedSlamFilter (src/EmbodiedSlamFilter.hpp:
// 58-74, src/Configuration.hpp field names) -- with only the namespace changed; it must give
// the same particles as the raw C ABI driven with the same inputs.  Then the reference-type
// adapters (toGpu, toAffine, toContactState on reference-shaped types), the logDebug
// records (cpoints), the hash init branch, the RCCL shard and the error mapping.
// Run by tests/test_gpu_facade.py; compiled (syntax) by tests/test_abi.py.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "eslam_gpu.hpp"

static int fails = 0;
#define EXPECT(c, msg)                                         \
    do {                                                       \
        if (!(c)) { std::printf("FAIL: %s\n", msg); ++fails; } \
    } while (0)

namespace eslam_ns = eslam::gpu;

// ---- reference-shaped types (what the real eslam::Configuration / Eigen / odometry types
// look like to the adapters: same member names, different classes) ----------------------
namespace ref {
struct Vec3 {
    double d[3];
    double operator[](int i) const { return d[i]; }
};
struct Mat3 {
    double d[9];
    double operator()(int r, int c) const { return d[r * 3 + c]; }
};
struct Affine {
    Mat3 R;
    Vec3 t;
    const Mat3& linear() const { return R; }
    const Vec3& translation() const { return t; }
};
struct UpdateThreshold { double distance, angle; };
struct ContactModelConfiguration {
    bool useSlipUpdate = false, useShapeUpdate = true;
    size_t minContacts = 2;
    double contactLikelihoodCorrection = 0.5, contactPointRadius = 0.02;
};
struct Configuration {
    unsigned long seed = 7;
    size_t particleCount = 1234, minEffective = 99;
    Vec3 initialRotationError{{0, 0, 0.2}}, initialTranslationError{{0.3, 0.3, 0.5}};
    double measurementError = 0.05, discountFactor = 0.8, spreadThreshold = 0.7, spreadTranslationFactor = 0.2,
           spreadRotationFactor = 0.1, slipFactor = 0.1, maxYawDeviation = 0.3;
    UpdateThreshold measurementThreshold{0.2, 0.3}, mappingThreshold{0.1, 0.1}, mappingCameraThreshold{1, 1};
    double gridSize = 10, gridResolution = 0.1, gridThreshold = 0.4, gridPatchThickness = 0.2, gridGapSize = 1.0;
    bool gridUseNegativeInformation = true;
    double maxSensorRange = 4;
    bool useVisualUpdate = false;
    ContactModelConfiguration contactModel;
    bool logDebug = true;
    unsigned int logParticlePeriod = 3;
};
struct BodyContactPoint { Vec3 position; float contact; int groupId; };
struct BodyContactState { std::vector<BodyContactPoint> points; };
}  // namespace ref

static eslam_ns::MlsGrid flat_grid(uint32_t W)
{
    eslam_ns::MlsGrid g;
    g.width = g.height = W;
    g.scaleX = g.scaleY = 0.1;
    g.offsetX = g.offsetY = -0.05 * W;
    g.cellStart.resize(W * W + 1);
    for (uint32_t i = 0; i <= W * W; ++i) g.cellStart[i] = i;
    g.mean.assign(W * W, 0.0f);
    g.stdev.assign(W * W, 0.05f);
    return g;
}

// four feet fixed in the world, seen from the body at (x, y, 0.18) with heading yaw
static eslam_ns::BodyContactState body_state(double x, double y, double yaw)
{
    static const double feet_w[4][2] = {{0.25, 0.0}, {-0.25, 0.0}, {0.25, -0.5}, {-0.25, -0.5}};
    eslam_ns::BodyContactState bs;
    bs.points.resize(4);
    const double c = std::cos(yaw), s = std::sin(yaw);
    for (int i = 0; i < 4; ++i) {
        const double dx = feet_w[i][0] - x, dy = feet_w[i][1] - y;
        bs.points[i].position = eslam_ns::Vector3d(c * dx + s * dy, -s * dx + c * dy, -0.18);
        bs.points[i].contact = 1.0f;
        bs.points[i].groupId = -1;
    }
    bs.time = x;
    return bs;
}

static eslam_ns::Affine3d body_pose(double x, double y, double yaw)
{
    eslam_ns::Affine3d T = eslam_ns::Affine3d::Identity();
    T.linear() = eslam_ns::Quaterniond(std::cos(yaw / 2), 0, 0, std::sin(yaw / 2)).toRotationMatrix();
    T.translation() = eslam_ns::Vector3d(x, y, 0.18);
    return T;
}

int main()
{
    const eslam_ns::MlsGrid env = flat_grid(200);

    // ---- the reference call site, namespace switched -------------------------------------
    eslam_ns::Configuration eslamConfig;
    eslamConfig.particleCount = 3000;
    eslamConfig.minEffective = 2000;
    eslamConfig.measurementThreshold = eslam_ns::UpdateThreshold(-1, -1);
    eslamConfig.contactModel.minContacts = 3;
    eslam_ns::OdometryConfiguration odometryConfig;
    eslam_ns::EmbodiedSlamFilter filter(odometryConfig, eslamConfig);
    eslam_ns::Pose startPose(eslam_ns::Vector3d(0, 0, 0.18), eslam_ns::Quaterniond::Identity());
    filter.init(env, startPose, true);
    std::vector<eslam_ns::TerrainClassification> terrainClassification;
    int updates = 0;
    double x = 0, y = 0, yaw = 0;
    for (int s = 0; s < 6; ++s) {
        yaw += 0.002;
        x += 0.02 * std::cos(yaw);
        y += 0.02 * std::sin(yaw);
        const eslam_ns::Affine3d body2odometry = body_pose(x, y, yaw);
        const eslam_ns::BodyContactState bodyState = body_state(x, y, yaw);
        const bool updated = filter.update(body2odometry, bodyState, terrainClassification);
        updates += updated ? 1 : 0;
    }
    std::vector<eslam_ns::PoseParticle>& particles = filter.getParticles();
    const size_t best = filter.getBestParticleIndex();
    const eslam_ns::Affine3d centroid = filter.getCentroid();
    EXPECT(updates == 6, "every step updates (thresholds forced)");
    EXPECT(particles.size() == 3000, "particle count");
    EXPECT(std::fabs(centroid.translation().x() - x) < 0.2, "centroid near the travelled pose");
    EXPECT(filter.odometry().stancePoints() == 4, "the contact odometry sees four feet in stance");
    {
        double mean[3], cov[9];
        filter.odometry().getSampleDistribution2D(mean, cov);
        // the body turns by 0.002 rad, then moves 2 cm along its new heading
        EXPECT(std::fabs(mean[0] - 0.02 * std::cos(0.002)) < 1e-12 && std::fabs(mean[1] - 0.02 * std::sin(0.002)) < 1e-12 &&
                   std::fabs(mean[2] - 0.002) < 1e-12,
               "contact odometry: 2 cm along the heading, 0.002 rad per step");
    }

    // ---- the same inputs through the raw C ABI -------------------------------------------
    {
        eslam_ns::FootContact odo(odometryConfig);
        eslam_ns::PoseEstimator raw(odo, eslamConfig);
        const eslam_mls_grid g = env.toC();
        EXPECT(eslam_gpu_set_map(raw.handle(), &g) == ESLAM_OK, "set_map");
        const double p0[3] = {0, 0, 0.18}, q0[4] = {1, 0, 0, 0};
        EXPECT(eslam_gpu_init_pose(raw.handle(), p0, q0) == ESLAM_OK, "init_pose");
        double rx = 0, ry = 0, ryaw = 0;
        for (int s = 0; s < 6; ++s) {
            ryaw += 0.002;
            rx += 0.02 * std::cos(ryaw);
            ry += 0.02 * std::sin(ryaw);
            const eslam_ns::Affine3d T = body_pose(rx, ry, ryaw);
            const eslam_ns::BodyContactState bs = body_state(rx, ry, ryaw);
            const eslam_ns::Quaterniond q(T.linear());
            odo.update(bs, q);
            const eslam_step_input in = raw.makeInput(bs, q, T.translation(), 0);
            int u = 0;
            EXPECT(eslam_gpu_step(raw.handle(), &in, &u) == ESLAM_OK && u == 1, "raw step");
        }
        const size_t n = particles.size();
        std::vector<double> X(n), Y(n), TH(n), Z(n), ZS(n), W(n), M(n);
        std::vector<uint8_t> FL(n), NC(n);
        eslam_particles p = {X.data(), Y.data(), TH.data(), Z.data(), ZS.data(), W.data(), M.data(), FL.data(), NC.data()};
        EXPECT(eslam_gpu_download_particles(raw.handle(), &p) == ESLAM_OK, "download");
        size_t diff = 0;
        for (size_t i = 0; i < n; ++i) {
            const eslam_ns::PoseParticle& a = particles[i];
            diff += std::memcmp(&a.position.v[0], &X[i], 8) || std::memcmp(&a.position.v[1], &Y[i], 8) ||
                    std::memcmp(&a.orientation, &TH[i], 8) || std::memcmp(&a.zPos, &Z[i], 8) ||
                    std::memcmp(&a.zSigma, &ZS[i], 8) || std::memcmp(&a.weight, &W[i], 8) ||
                    std::memcmp(&a.mprob, &M[i], 8) || a.floating != (FL[i] != 0) || a.cpoints.size() != NC[i];
        }
        EXPECT(diff == 0, "reference-shaped call site == raw ABI, bit for bit");
        EXPECT(raw.getBestParticleIndex() == best, "best particle");
    }

    // ---- getParticles() is the filter's particles: an edit through the reference reaches the
    // filter, as processMap's weighting (src/EmbodiedSlamFilter.cpp:183-220) relies on.  The
    // same edits through the raw ABI (download, edit, upload) give the same particles. --------
    {
        eslam_ns::Configuration ec = eslamConfig;
        ec.particleCount = 2000;
        eslam_ns::EmbodiedSlamFilter ef(odometryConfig, ec);
        ef.init(env, startPose, true);
        eslam_ns::FootContact odo(odometryConfig);
        eslam_ns::PoseEstimator raw(odo, ec);
        const eslam_mls_grid g = env.toC();
        EXPECT(eslam_gpu_set_map(raw.handle(), &g) == ESLAM_OK, "edit: raw set_map");
        const double p0[3] = {0, 0, 0.18}, q0[4] = {1, 0, 0, 0};
        EXPECT(eslam_gpu_init_pose(raw.handle(), p0, q0) == ESLAM_OK, "edit: raw init");
        const size_t n = 2000;
        std::vector<double> X(n), Y(n), TH(n), Z(n), ZS(n), W(n), M(n);
        std::vector<uint8_t> FL(n), NC(n);
        eslam_particles p = {X.data(), Y.data(), TH.data(), Z.data(), ZS.data(), W.data(), M.data(), FL.data(), NC.data()};
        auto factor = [](size_t i) { return 1.0 + 0.5 * (double)((i * 2654435761u) % 7u) / 7.0; };
        double ex = 0, eyaw = 0;
        for (int s = 0; s < 6; ++s) {
            eyaw += 0.002;
            ex += 0.02;
            const eslam_ns::Affine3d T = body_pose(ex, 0, eyaw);
            const eslam_ns::BodyContactState bs = body_state(ex, 0, eyaw);
            ef.update(T, bs, terrainClassification);
            const eslam_ns::Quaterniond q(T.linear());
            odo.update(bs, q);
            const eslam_step_input in = raw.makeInput(bs, q, T.translation(), 0);
            int u = 0;
            EXPECT(eslam_gpu_step(raw.handle(), &in, &u) == ESLAM_OK, "edit: raw step");
            if (s % 2 == 1) {
                // a per-particle weighting through the vector (processMap(match): w *= weight^0.1)
                std::vector<eslam_ns::PoseParticle>& ps = ef.getParticles();
                for (size_t i = 0; i < ps.size(); ++i) ps[i].weight *= factor(i);
                if (s == 3) ps[7].position = eslam_ns::Vector2d(ps[7].position.x() + 0.01, ps[7].position.y());
                EXPECT(eslam_gpu_download_particles(raw.handle(), &p) == ESLAM_OK, "edit: raw download");
                for (size_t i = 0; i < n; ++i) W[i] *= factor(i);
                if (s == 3) X[7] += 0.01;
                EXPECT(eslam_gpu_upload_particles(raw.handle(), n, &p) == ESLAM_OK, "edit: raw upload");
            }
        }
        std::vector<eslam_ns::PoseParticle>& a = ef.getParticles();
        EXPECT(eslam_gpu_download_particles(raw.handle(), &p) == ESLAM_OK, "edit: raw final download");
        size_t diff = a.size() != n;
        for (size_t i = 0; i < a.size() && i < n; ++i)
            diff += std::memcmp(&a[i].position.v[0], &X[i], 8) || std::memcmp(&a[i].position.v[1], &Y[i], 8) ||
                    std::memcmp(&a[i].orientation, &TH[i], 8) || std::memcmp(&a[i].zPos, &Z[i], 8) ||
                    std::memcmp(&a[i].zSigma, &ZS[i], 8) || std::memcmp(&a[i].weight, &W[i], 8) ||
                    std::memcmp(&a[i].mprob, &M[i], 8) || a[i].floating != (FL[i] != 0) || a[i].cpoints.size() != NC[i];
        EXPECT(diff == 0, "edits through getParticles() == download / edit / upload, bit for bit");
        EXPECT(&a == &ef.getParticles(), "getParticles() hands out the same vector");
        // processMap(scanMap, true, false) on the shared map (the laser path's match-only call,
        // src/EmbodiedSlamFilter.cpp:342-344): every particle against the shared grid
        std::vector<eslam_ns::ScanPatch> scan;
        std::vector<eslam_scan_patch> rs;
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < 4; ++j) {
                eslam_ns::ScanPatch sp;
                sp.position = eslam_ns::Vector3d(0.35 + 0.1 * i, -0.6 + 0.2 * j, -0.13);
                sp.stdev = 0.03;
                scan.push_back(sp);
                eslam_scan_patch r;
                for (int k = 0; k < 3; ++k) r.position[k] = sp.position[k];
                r.stdev = sp.stdev;
                rs.push_back(r);
            }
        const double w0 = ef.getParticles()[0].weight;
        ef.processMap(scan, true, false);
        EXPECT(eslam_gpu_map_match(raw.handle(), rs.data(), (uint32_t)rs.size()) == ESLAM_OK, "raw shared-map match");
        std::vector<eslam_ns::PoseParticle>& a2 = ef.getParticles();
        EXPECT(eslam_gpu_download_particles(raw.handle(), &p) == ESLAM_OK, "match: raw download");
        diff = a2.size() != n;
        for (size_t i = 0; i < a2.size() && i < n; ++i) diff += std::memcmp(&a2[i].weight, &W[i], 8) != 0;
        EXPECT(diff == 0, "processMap(match = true) on the shared map: façade == raw ABI, bit for bit");
        EXPECT(a2[0].weight < w0, "a scan 5 cm above the grid lowers particle 0's weight");
    }

    // ---- UpdateThreshold::test(const Affine3d&) (src/Configuration.hpp:23-26, Q6 kept) -----
    {
        const eslam_ns::UpdateThreshold th(0.1, 10 * M_PI / 180.0);
        eslam_ns::Affine3d turn = body_pose(0, 0, 0.15);
        turn.translation() = eslam_ns::Vector3d(0, 0, 0);
        eslam_ns::Affine3d small = eslam_ns::Affine3d::Identity(), big = eslam_ns::Affine3d::Identity();
        small.translation() = eslam_ns::Vector3d(0.05, 0, 0);
        big.translation() = eslam_ns::Vector3d(0.18, 0, 0);
        EXPECT(th.test(turn), "a 0.15 rad turn exceeds the distance threshold 0.1 (angle and distance swapped)");
        EXPECT(!th.test(small), "5 cm: neither 0 > 0.1 nor 0.05 > 10 deg");
        EXPECT(th.test(big), "18 cm exceeds the angle threshold 10 deg = 0.1745 (swapped)");
    }

    // ---- adapters from reference-shaped types ---------------------------------------------
    {
        ref::Configuration rc;
        const eslam_ns::Configuration c = eslam_ns::toGpu(rc);
        EXPECT(c.seed == 7 && c.particleCount == 1234 && c.minEffective == 99, "toGpu: counts");
        EXPECT(c.initialTranslationError.x() == 0.3 && c.initialRotationError.z() == 0.2, "toGpu: vectors");
        EXPECT(c.measurementThreshold.distance == 0.2 && c.measurementThreshold.angle == 0.3, "toGpu: UpdateThreshold");
        EXPECT(c.contactModel.minContacts == 2 && c.contactModel.contactPointRadius == 0.02, "toGpu: contactModel");
        EXPECT(c.logDebug && c.logParticlePeriod == 3, "toGpu: logging");
        const eslam_config cc = c.toC();
        EXPECT(cc.min_contacts == 2 && cc.discount_factor == 0.8 && cc.log_debug == 1, "toC");
        ref::Affine A{{{0, -1, 0, 1, 0, 0, 0, 0, 1}}, {{1, 2, 3}}};
        const eslam_ns::Affine3d T = eslam_ns::toAffine(A);
        EXPECT(T.linear()(0, 1) == -1 && T.translation().z() == 3, "toAffine");
        ref::BodyContactState rbs{{{{{0.1, 0.2, -0.3}}, 0.9f, 2}}};
        const eslam_ns::BodyContactState bs = eslam_ns::toContactState(rbs);
        EXPECT(bs.points.size() == 1 && bs.points[0].groupId == 2 && bs.points[0].position.z() == -0.3, "toContactState");
    }

    // ---- logDebug: cpoints / meas_pos of every particle, and the logging period ----------
    {
        eslam_ns::Configuration dc = eslamConfig;
        dc.particleCount = 500;
        dc.logDebug = true;
        dc.logParticlePeriod = 2;
        eslam_ns::EmbodiedSlamFilter df(odometryConfig, dc);
        df.init(env, startPose);
        double dx = 0;
        int logged = 0;
        for (int s = 0; s < 5; ++s) {
            dx += 0.02;
            df.update(body_pose(dx, 0, 0), body_state(dx, 0, 0), terrainClassification);
            logged += df.logDue() ? 1 : 0;
        }
        EXPECT(logged == 3, "logParticlePeriod 2: updates 1, 3, 5 are logged");
        const eslam_ns::PoseDistribution dist = df.getPoseDistribution(5);
        EXPECT(dist.particles.size() == 100, "strided distribution");
        size_t with_points = 0, bad = 0;
        for (const eslam_ns::PoseParticle& p : dist.particles) {
            if (!p.floating) {
                with_points += p.cpoints.size() == 4;
                for (const eslam_ns::ContactPoint& c : p.cpoints)
                    bad += !(std::isfinite(c.zdiff) && c.zvar > 0 && c.prob == 1.0 && std::fabs(c.point.z()) < 1e-6);
            }
            bad += p.meas_pos.x() != p.position.x() || p.meas_theta != p.orientation;
        }
        EXPECT(with_points > 50, "accepted particles carry their four contact points");
        EXPECT(bad == 0, "contact points on the flat map; meas_pos = the updated pose");
    }

    // ---- init(env, pose, true, hashConfig) draws the particles from the surface hash ------
    {
        eslam_ns::Configuration hc = eslamConfig;
        hc.particleCount = 800;
        eslam_ns::SurfaceHashConfig hashConfig;
        hashConfig.useHash = true;
        eslam_ns::EmbodiedSlamFilter hf(odometryConfig, hc);
        hf.init(env, startPose, true, hashConfig);
        EXPECT(hf.getParticles().size() == 800, "hash init: particle count");
        hf.update(body_pose(0.02, 0, 0), body_state(0.02, 0, 0), terrainClassification);
        EXPECT(hf.getParticles().size() == 800, "hash filter steps");
    }

    // ---- init(env, pose, false): per-particle maps, processMap(scanMap, false, true) ------
    {
        // the flat grid with no patches in the cells whose centre lies at x >= 0.3 m
        eslam_ns::MlsGrid pm;
        pm.width = pm.height = 200;
        pm.scaleX = pm.scaleY = 0.1;
        pm.offsetX = pm.offsetY = -10.0;
        pm.cellStart.assign(200 * 200 + 1, 0);
        for (uint32_t c = 0; c < 200u * 200u; ++c) {
            const bool mapped = -10.0 + ((c % 200) + 0.5) * 0.1 < 0.3;
            pm.cellStart[c + 1] = pm.cellStart[c] + (mapped ? 1u : 0u);
            if (mapped) { pm.mean.push_back(0.0f); pm.stdev.push_back(0.05f); }
        }
        std::vector<eslam_ns::ScanPatch> scan;
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < 4; ++j) {
                eslam_ns::ScanPatch sp;
                sp.position = eslam_ns::Vector3d(0.35 + 0.1 * i, -0.6 + 0.2 * j, -0.18);
                sp.stdev = 0.03;
                scan.push_back(sp);
            }
        eslam_ns::Configuration mc = eslamConfig;
        mc.particleCount = 2000;
        eslam_ns::EmbodiedSlamFilter mf(odometryConfig, mc);
        mf.init(pm, startPose, false);
        eslam_ns::FootContact odo(odometryConfig);
        eslam_ns::PoseEstimator raw(odo, mc);
        const eslam_mls_grid g = pm.toC();
        EXPECT(eslam_gpu_set_map(raw.handle(), &g) == ESLAM_OK && eslam_gpu_set_particle_maps(raw.handle(), 1) == ESLAM_OK,
               "raw: per-particle maps");
        const double p0[3] = {0, 0, 0.18}, q0[4] = {1, 0, 0, 0};
        EXPECT(eslam_gpu_init_pose(raw.handle(), p0, q0) == ESLAM_OK, "raw init");
        EXPECT(eslam_gpu_set_particle_maps(raw.handle(), 0) != ESLAM_OK, "the map mode is fixed once initialised");
        std::vector<eslam_scan_patch> rs(scan.size());
        for (size_t k = 0; k < scan.size(); ++k) {
            for (int i = 0; i < 3; ++i) rs[k].position[i] = scan[k].position[i];
            rs[k].stdev = scan[k].stdev;
        }
        double mx = 0;
        for (int s = 0; s < 6; ++s) {
            mx += 0.02;
            const eslam_ns::Affine3d T = body_pose(mx, 0, 0);
            const eslam_ns::BodyContactState bs = body_state(mx, 0, 0);
            mf.update(T, bs, terrainClassification);
            mf.processMap(scan, false, true);
            const eslam_ns::Quaterniond q(T.linear());
            odo.update(bs, q);
            const eslam_step_input in = raw.makeInput(bs, q, T.translation(), 0);
            int u = 0;
            EXPECT(eslam_gpu_step(raw.handle(), &in, &u) == ESLAM_OK, "raw step (maps)");
            EXPECT(eslam_gpu_map_update(raw.handle(), rs.data(), (uint32_t)rs.size()) == ESLAM_OK, "raw map update");
        }
        std::vector<eslam_ns::PoseParticle>& a = mf.getParticles();
        std::vector<eslam_ns::PoseParticle>& b = raw.getParticles();
        size_t diff = a.size() != b.size();
        for (size_t i = 0; i < a.size() && i < b.size(); ++i)
            diff += std::memcmp(&a[i].position.v[0], &b[i].position.v[0], 16) || std::memcmp(&a[i].weight, &b[i].weight, 8) ||
                    std::memcmp(&a[i].zPos, &b[i].zPos, 8) || std::memcmp(&a[i].zSigma, &b[i].zSigma, 8);
        EXPECT(diff == 0, "per-particle maps: façade == raw ABI, bit for bit");
        uint32_t cells[64], cnt = 0;
        float mean[64], sd[64];
        EXPECT(eslam_gpu_get_particle_map(mf.estimator().handle(), 0, cells, mean, sd, 64, &cnt) == ESLAM_OK && cnt > 0,
               "particle 0 holds patches from the scans");
        // processMap(scanMap, true, true): the match weighting (eslam_gpu_map_match) before the
        // merge, against the raw ABI; a scan 5 cm higher scores below 1 on the matched cells
        std::vector<eslam_ns::ScanPatch> hi = scan;
        for (auto& sp : hi) sp.position = eslam_ns::Vector3d(sp.position.x(), sp.position.y(), sp.position.z() + 0.05);
        std::vector<eslam_scan_patch> rh(rs);
        for (auto& sp : rh) sp.position[2] += 0.05;
        const double w0 = mf.getParticles()[0].weight;
        mf.processMap(hi, true, true);
        EXPECT(eslam_gpu_map_match(raw.handle(), rh.data(), (uint32_t)rh.size()) == ESLAM_OK &&
                   eslam_gpu_map_update(raw.handle(), rh.data(), (uint32_t)rh.size()) == ESLAM_OK,
               "raw match + update");
        std::vector<eslam_ns::PoseParticle>& a2 = mf.getParticles();
        raw.invalidate();                 // the raw ABI calls changed the particles behind the view
        std::vector<eslam_ns::PoseParticle>& b2 = raw.getParticles();
        diff = a2.size() != b2.size();
        for (size_t i = 0; i < a2.size() && i < b2.size(); ++i) diff += std::memcmp(&a2[i].weight, &b2[i].weight, 8) != 0;
        EXPECT(diff == 0, "processMap(match = true): façade == raw ABI, bit for bit");
        EXPECT(a2[0].weight < w0, "the higher scan lowers particle 0's weight");
    }

    // ---- one shard of a 3000-particle filter over the library's own RCCL communicator ----
    {
        eslam_ns::FootContact odo(odometryConfig);
        eslam_ns::PoseEstimator shard(odo, eslamConfig);
        shard.setCommRccl(1, 0, eslam_ns::PoseEstimator::rcclUniqueId(), 3000, std::vector<uint64_t>{0, 3000});
        shard.setEnvironment(env);
        const double p0[3] = {0, 0, 0.18}, q0[4] = {1, 0, 0, 0};
        EXPECT(eslam_gpu_init_pose(shard.handle(), p0, q0) == ESLAM_OK, "shard init");
        double sx = 0, sy = 0, syaw = 0;
        for (int s = 0; s < 6; ++s) {
            syaw += 0.002;
            sx += 0.02 * std::cos(syaw);
            sy += 0.02 * std::sin(syaw);
            const eslam_ns::Affine3d T = body_pose(sx, sy, syaw);
            const eslam_ns::BodyContactState bs = body_state(sx, sy, syaw);
            const eslam_ns::Quaterniond q(T.linear());
            odo.update(bs, q);
            const eslam_step_input in = shard.makeInput(bs, q, T.translation(), 0);
            int u = 0;
            EXPECT(eslam_gpu_step(shard.handle(), &in, &u) == ESLAM_OK, "shard step");
        }
        std::vector<eslam_ns::PoseParticle> b = shard.getParticles();
        size_t sdiff = b.size() == particles.size() ? 0 : 1;
        for (size_t i = 0; i < b.size() && !sdiff; ++i)
            sdiff += std::memcmp(&particles[i].position, &b[i].position, sizeof(double) * 2) != 0 ||
                     std::memcmp(&particles[i].weight, &b[i].weight, 8) != 0;
        EXPECT(sdiff == 0, "RCCL shard (1 rank) == single GPU, bit for bit");
    }

    // ---- error mapping: PoseEstimator::update without an environment ----------------------
    {
        eslam_ns::FootContact odo(odometryConfig);
        eslam_ns::PoseEstimator bare(odo, eslamConfig);
        bare.init(100, eslam_ns::Pose2D(), eslam_ns::Pose2D(eslam_ns::Vector2d(0.1, 0.1), 0.1), 0.18, 1.0);
        bool threw = false;
        try {
            bare.update(body_state(0, 0, 0), eslam_ns::Quaterniond::Identity(), terrainClassification);
        } catch (const std::runtime_error& e) {
            threw = std::strcmp(e.what(), "No environment attached.") == 0;
        }
        EXPECT(threw, "update without environment throws the reference message");
    }
    if (fails) return 1;
    std::printf("facade OK: %zu particles, best %zu, centroid (%.4f, %.4f, %.4f)\n", particles.size(), best,
                centroid.translation().x(), centroid.translation().y(), centroid.translation().z());
    return 0;
}
