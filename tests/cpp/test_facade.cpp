// C++ façade (include/eslam_gpu.hpp) on the GPU: the reference-shaped class API gives the
// same particles as the raw C ABI for the same inputs, and maps errors to the reference's
// std::runtime_error messages.  Run by tests/test_gpu_facade.py.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "eslam_gpu.hpp"

using namespace eslam::gpu;

static int fails = 0;
#define EXPECT(c, msg)                                         \
    do {                                                       \
        if (!(c)) { std::printf("FAIL: %s\n", msg); ++fails; } \
    } while (0)

int main()
{
    // flat 200 x 200 grid @ 0.1 m around the origin, one patch per cell
    const uint32_t W = 200;
    std::vector<uint32_t> cells(W * W + 1);
    for (uint32_t i = 0; i <= W * W; ++i) cells[i] = i;
    std::vector<float> mean(W * W, 0.0f), stdev(W * W, 0.05f);
    eslam_mls_grid grid;
    std::memset(&grid, 0, sizeof(grid));
    grid.width = grid.height = W;
    grid.scale_x = grid.scale_y = 0.1;
    grid.offset_x = grid.offset_y = -10.0;
    grid.global2local[0] = grid.global2local[5] = grid.global2local[10] = 1.0;
    grid.cell_start = cells.data();
    grid.patch_mean = mean.data();
    grid.patch_stdev = stdev.data();
    grid.n_patches = W * W;

    Configuration cfg;
    cfg.particle_count = 3000;
    cfg.min_effective = 2000;
    cfg.measurement_threshold_distance = -1;
    cfg.measurement_threshold_angle = -1;

    const double feet[4][3] = {{0.25, 0, -0.18}, {-0.25, 0, -0.18}, {0.25, -0.5, -0.18}, {-0.25, -0.5, -0.18}};
    std::vector<BodyContactPoint> bs(4);
    for (int i = 0; i < 4; ++i) std::memcpy(bs[i].position, feet[i], sizeof(feet[i]));
    OdometryOutputs odo;
    odo.poseDeltaTranslation[0] = 0.02;
    odo.positionErrorZZ = 1e-4;
    odo.sampleMean[0] = 0.02;
    odo.sampleMean[2] = 0.002;
    odo.sampleCov[0] = 1e-4; odo.sampleCov[4] = 1e-4; odo.sampleCov[8] = 1e-5;

    Pose start;
    start.position[2] = 0.18;
    EmbodiedSlamFilter filter(cfg);
    filter.init(grid, start);

    // the same through the raw C ABI
    eslam_ctx* raw = nullptr;
    EXPECT(eslam_gpu_create(&cfg, 0, &raw) == ESLAM_OK, "create");
    EXPECT(eslam_gpu_set_map(raw, &grid) == ESLAM_OK, "set_map");
    EXPECT(eslam_gpu_init_pose(raw, start.position, start.orientation) == ESLAM_OK, "init_pose");

    double yaw = 0, x = 0, y = 0;
    int updates = 0;
    for (int s = 0; s < 6; ++s) {
        yaw += 0.002;
        x += 0.02 * std::cos(yaw);
        y += 0.02 * std::sin(yaw);
        Pose b2o;
        b2o.position[0] = x; b2o.position[1] = y;
        b2o.orientation[0] = std::cos(yaw / 2); b2o.orientation[3] = std::sin(yaw / 2);
        updates += filter.update(b2o, bs, odo) ? 1 : 0;
        eslam_step_input in = PoseEstimator::make_input(bs, b2o.orientation, b2o.position, odo, 0);
        int u = 0;
        EXPECT(eslam_gpu_step(raw, &in, &u) == ESLAM_OK, "raw step");
    }
    EXPECT(updates == 6, "every step updates (thresholds forced)");
    std::vector<PoseParticle> a = filter.getParticles();
    const size_t n = a.size();
    std::vector<double> rx(n), ry(n), rt(n), rz(n), rs(n), rw(n), rm(n);
    std::vector<uint8_t> rf(n), rc(n);
    eslam_particles p = {rx.data(), ry.data(), rt.data(), rz.data(), rs.data(), rw.data(), rm.data(), rf.data(), rc.data()};
    EXPECT(eslam_gpu_download_particles(raw, &p) == ESLAM_OK, "download");
    size_t diff = 0;
    for (size_t i = 0; i < n; ++i)
        diff += std::memcmp(&a[i].position[0], &rx[i], 8) || std::memcmp(&a[i].position[1], &ry[i], 8) ||
                std::memcmp(&a[i].orientation, &rt[i], 8) || std::memcmp(&a[i].zPos, &rz[i], 8) ||
                std::memcmp(&a[i].zSigma, &rs[i], 8) || std::memcmp(&a[i].weight, &rw[i], 8) ||
                a[i].floating != (rf[i] != 0) || a[i].nContactPoints != rc[i];
    EXPECT(n == 3000, "particle count");
    EXPECT(diff == 0, "facade == raw ABI, bit for bit");
    const size_t best = filter.getBestParticleIndex();
    uint64_t rbest = 0;
    eslam_gpu_get_best_particle_index(raw, &rbest);
    EXPECT(best == rbest, "best particle");
    Pose c = filter.getCentroid();
    EXPECT(std::isfinite(c.position[0]) && std::fabs(c.position[0] - x) < 0.2, "centroid near the odometry pose");

    // one shard of a 3000-particle filter over the library's own RCCL communicator (one
    // rank): the same particles, bit for bit, as the single-GPU filter
    {
        PoseEstimator shard(cfg);
        shard.setCommRccl(1, 0, PoseEstimator::rcclUniqueId(), 3000, std::vector<uint64_t>{0, 3000});
        shard.setEnvironment(grid);
        EXPECT(eslam_gpu_init_pose(shard.handle(), start.position, start.orientation) == ESLAM_OK, "shard init");
        double syaw = 0, sx = 0, sy = 0;
        for (int s = 0; s < 6; ++s) {
            syaw += 0.002;
            sx += 0.02 * std::cos(syaw);
            sy += 0.02 * std::sin(syaw);
            Pose b2o;
            b2o.position[0] = sx; b2o.position[1] = sy;
            b2o.orientation[0] = std::cos(syaw / 2); b2o.orientation[3] = std::sin(syaw / 2);
            eslam_step_input in = PoseEstimator::make_input(bs, b2o.orientation, b2o.position, odo, 0);
            int u = 0;
            EXPECT(eslam_gpu_step(shard.handle(), &in, &u) == ESLAM_OK, "shard step");
        }
        std::vector<PoseParticle> b = shard.getParticles();
        size_t sdiff = b.size() == n ? 0 : 1;
        for (size_t i = 0; i < n && !sdiff; ++i)
            sdiff += std::memcmp(&a[i], &b[i], sizeof(double) * 6) != 0;
        EXPECT(sdiff == 0, "RCCL shard (1 rank) == single GPU, bit for bit");
    }

    // error mapping: PoseEstimator::update without an environment
    PoseEstimator bare(cfg);
    bare.init(100, Pose2D{}, Pose2D{0.1, 0.1, 0.1}, 0.18, 1.0);
    bool threw = false;
    try {
        const double q[4] = {1, 0, 0, 0};
        bare.update(bs, q, odo);
    } catch (const std::runtime_error& e) {
        threw = std::strcmp(e.what(), "No environment attached.") == 0;
    }
    EXPECT(threw, "update without environment throws the reference message");
    eslam_gpu_destroy(raw);
    if (fails) return 1;
    std::printf("facade OK: %zu particles, best %zu, centroid (%.4f, %.4f, %.4f)\n", n, best, c.position[0],
                c.position[1], c.position[2]);
    return 0;
}
