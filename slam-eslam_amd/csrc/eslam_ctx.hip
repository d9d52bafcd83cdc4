// eslam_ctx.hip -- host side of libeslam_gpu: the C ABI of include/eslam_gpu.h.
//
// Per-step host work is O(1): the reference's per-step scalar preparation
// (src/PoseEstimator.cpp:186-194: yaw, removeYaw, the odometry z delta and variance,
// the sampler's Cholesky factor; src/ContactModel.cpp:21-41: the yaw-compensated feet) and
// the EmbodiedSlamFilter update gate (src/EmbodiedSlamFilter.cpp:360).  Everything that
// touches particles runs on the GPU; the resample decision is taken on the device, so a
// step is four asynchronous launches with no host round trip.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <dlfcn.h>

#include <math.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <chrono>
#include <algorithm>
#include <atomic>
#include <vector>

#include "eslam_internal.h"

using namespace eslam_dev;

extern "C" hipError_t eslam_launch_contact_records(DevState s0, DevState s1, const MapView* map, const StepParams* p, Ctl* ctl,
                                                   const DebugRec* d, const LocalMaps* store, hipStream_t stream);
extern "C" hipError_t eslam_launch_store_init(uint32_t* sid, const LocalMaps* lm, uint64_t n, uint64_t pool, hipStream_t stream);
extern "C" hipError_t eslam_launch_store_refs(SidRef sid, uint64_t n, uint64_t pool, const CowScratch* cs, const GatherView* gv,
                                              uint32_t* tgen, hipStream_t stream);
extern "C" hipError_t eslam_launch_store_receive(SidRef sid, Ctl* ctl, const LocalMaps* lm, const MergeParams* mp, uint64_t n,
                                                 const CowScratch* cs, const void* hdr, uint64_t nrecv, uint32_t* hoff,
                                                 uint32_t* head, const void* pay, uint32_t* pgc, hipStream_t stream);
extern "C" hipError_t eslam_launch_map_plan(DevState s0, DevState s1, Ctl* ctl, const MapView* map, const LocalMaps* lm,
                                            const MergeParams* mp, uint32_t* pgc, hipStream_t stream);
extern "C" hipError_t eslam_launch_map_match(DevState s0, DevState s1, const Ctl* ctl, const MapView* map, const LocalMaps* lm,
                                             const MatchParams* mp, hipStream_t stream);
extern "C" hipError_t eslam_launch_map_merge(DevState s0, DevState s1, Ctl* ctl, const MapView* map, const LocalMaps* lm,
                                             const MergeParams* mp, hipStream_t stream);
extern "C" hipError_t eslam_launch_pay_hdr(DevState s0, DevState s1, const Ctl* ctl, const void* send, uint64_t nsend,
                                           uint64_t gbase, const LocalMaps* lm, const PaySeg* seg, void* hdr, uint32_t* off,
                                           hipStream_t stream);
extern "C" hipError_t eslam_launch_pay_pack(DevState s0, DevState s1, const Ctl* ctl, const void* send, uint64_t nsend,
                                            uint64_t gbase, const LocalMaps* lm, const void* hdr, const uint32_t* off, void* pay,
                                            hipStream_t stream);
extern "C" hipError_t eslam_launch_pack_records(DevState s0, DevState s1, const Ctl* ctl, uint64_t first, uint64_t stride,
                                                uint64_t count, uint64_t gbase, const uint32_t* anc, const DebugRec* d,
                                                eslam_particle_record* out, eslam_cpoint* cps, uint32_t max_cp,
                                                const uint64_t* slot, const double* remote, hipStream_t stream);
extern "C" hipError_t eslam_launch_gather_records(const uint32_t* req, uint64_t nreq, uint64_t gbase, const DebugRec* d,
                                                  double* items, hipStream_t stream);
extern "C" hipError_t eslam_launch_centroid_chunks(DevState s0, DevState s1, uint64_t n, uint32_t J, Ctl* ctl,
                                                   double* chunk_out, hipStream_t stream);
extern "C" hipError_t eslam_launch_centroid_tree(double* a, double* b, uint64_t m, double* out, hipStream_t stream);
extern "C" hipError_t eslam_launch_hash_candidates(const uint32_t* keys, const uint32_t* order, uint64_t cnt, uint64_t gbase,
                                                   int nranks, void* send, hipStream_t stream);
extern "C" hipError_t eslam_launch_hash_unpack(const void* recv, uint64_t m, uint32_t* keys, uint32_t* vals, hipStream_t stream);
extern "C" hipError_t eslam_launch_hash_replace_global(DevState s0, DevState s1, const Ctl* ctl, const uint32_t* gorder,
                                                       const uint32_t* draws, uint64_t k, uint64_t gbase, uint64_t n,
                                                       const uint32_t* blist, uint32_t bstart, const double* hx,
                                                       const double* hy, const double* hth, const double* hz, double weight,
                                                       hipStream_t stream);
extern "C" hipError_t eslam_radix_sort_pairs(uint32_t* keys, uint32_t* vals, uint32_t* keys_out, uint32_t* order, uint64_t n,
                                             void* tmp, size_t* tmp_bytes, hipStream_t stream);
extern "C" hipError_t eslam_launch_project_weight(int project, int weight, int maxp, DevState s0, DevState s1,
                                                  const MapView* map, const StepParams* p, Ctl* ctl, Shard* shards,
                                                  const GatherView* gv, const LocalMaps* store, hipStream_t stream,
                                                  const ChunkSel* sel, double* bspill);
extern "C" hipError_t eslam_launch_commit(Ctl* ctl, hipStream_t stream);
extern "C" hipError_t eslam_launch_weight_stats(DevState s0, DevState s1, uint64_t n, uint32_t J, Ctl* ctl, Shard* shards,
                                                hipStream_t stream);
extern "C" hipError_t eslam_launch_finalize(Shard* recs, int nrec, Ctl* ctl, const FinParams* fp, hipStream_t stream);
extern "C" hipError_t eslam_launch_normalize_scan(DevState s0, DevState s1, const ScanParams* sp, Ctl* ctl, uint64_t* tile_sum,
                                                  uint64_t* total, const FusedFin* ff, hipStream_t stream);
extern "C" hipError_t eslam_launch_normalize_segments(DevState s0, DevState s1, const ScanParams* sp, Ctl* ctl,
                                                      uint64_t* tile_pub, uint32_t* marks, uint32_t* tile_first,
                                                      const uint32_t* jt, const FusedFin* ff, hipStream_t stream);
extern "C" hipError_t eslam_launch_resample_gather(DevState s0, DevState s1, uint64_t n, uint64_t gbase, Ctl* ctl,
                                                   const GatherView* gv, uint32_t aux, hipStream_t stream);
extern "C" hipError_t eslam_launch_segments_multi(DevState s0, DevState s1, const ScanParams* sp, const PlanParams* pp, Ctl* ctl,
                                                  const uint64_t* tile_prefix, uint32_t* marks, uint32_t* tile_first,
                                                  const uint64_t* totals, const uint32_t* jt, uint2* range, uint64_t* first_last,
                                                  uint64_t* host_out, uint64_t* host_epoch, uint64_t epoch,
                                                  hipStream_t stream);
extern "C" hipError_t eslam_launch_pack(DevState s0, DevState s1, Ctl* ctl, const PlanParams* pp, const uint2* range,
                                        const uint64_t* first_last, uint64_t nsend, void* send, hipStream_t stream);
extern "C" hipError_t eslam_launch_expand(const void* recv, uint64_t nrecv, uint64_t W0, uint32_t* marks, uint32_t* row_first,
                                          hipStream_t stream);
extern "C" uint64_t eslam_record_bytes(void);
extern "C" hipError_t eslam_launch_hash_sweep(const dm_hash_grid* g, const double* pts, const double* orient, uint32_t steps,
                                              int32_t* out, hipStream_t stream);
extern "C" hipError_t eslam_launch_hash_poses(const dm_hash_grid* g, const double* pts, const double* orient, const uint64_t* ids,
                                              uint64_t count, double* hx, double* hy, double* hth, double* hz,
                                              hipStream_t stream);
extern "C" hipError_t eslam_launch_init_from_hash(DevState s0, const uint32_t* idx, uint64_t n, const double* hx,
                                                  const double* hy, const double* hth, const double* hz, hipStream_t stream);
extern "C" hipError_t eslam_hash_sort(DevState s0, DevState s1, const Ctl* ctl, uint64_t n, uint32_t* keys, uint32_t* vals,
                                      uint32_t* keys_out, uint32_t* order, void* tmp, size_t* tmp_bytes, hipStream_t stream);
extern "C" hipError_t eslam_launch_hash_replace(DevState s0, DevState s1, const Ctl* ctl, const uint32_t* order,
                                                const uint32_t* draws, uint64_t k, const uint32_t* blist, uint32_t bstart,
                                                const double* hx, const double* hy, const double* hth, const double* hz,
                                                double weight, hipStream_t stream);
extern "C" hipError_t eslam_launch_init_gaussian(DevState s0, uint64_t n, uint64_t gbase, uint64_t seed, uint64_t ev,
                                                 const double mu[3], const double sigma[3], double zpos, double zsigma,
                                                 hipStream_t stream);
extern "C" hipError_t eslam_launch_selftest_math(int fn, const double* x, const double* y, double* out, uint64_t n,
                                                 hipStream_t stream);
extern "C" hipError_t eslam_launch_best_index(DevState s0, DevState s1, uint64_t n, Ctl* ctl, uint64_t* out2,
                                              hipStream_t stream);
extern "C" hipError_t eslam_launch_centroid(DevState s0, DevState s1, uint64_t n, uint32_t J, Ctl* ctl, double* out,
                                            hipStream_t stream);

// ---------------------------------------------------------------------------------------
// small Eigen / base-types restatements (host, per step)
// ---------------------------------------------------------------------------------------
namespace {

void q_to_mat(const double q[4], double R[9])          // QuaternionBase::toRotationMatrix
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

void q_mul(const double a[4], const double b[4], double r[4])
{
    const double w = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
    const double x = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
    const double y = a[0] * b[2] + a[2] * b[0] + a[3] * b[1] - a[1] * b[3];
    const double z = a[0] * b[3] + a[3] * b[0] + a[1] * b[2] - a[2] * b[1];
    r[0] = w; r[1] = x; r[2] = y; r[3] = z;
}

void q_from_yaw(double angle, double q[4])              // Quaternion(AngleAxis(angle, UnitZ))
{
    const double ha = 0.5 * angle;
    q[0] = cos(ha);
    const double s = sin(ha);
    q[1] = s * 0.0; q[2] = s * 0.0; q[3] = s * 1.0;
}

void q_rotate(const double q[4], const double v[3], double out[3])   // _transformVector
{
    const double qx = q[1], qy = q[2], qz = q[3], w = q[0];
    double uv[3] = {qy * v[2] - qz * v[1], qz * v[0] - qx * v[2], qx * v[1] - qy * v[0]};
    uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
    const double c[3] = {qy * uv[2] - qz * uv[1], qz * uv[0] - qx * uv[2], qx * uv[1] - qy * uv[0]};
    out[0] = (v[0] + w * uv[0]) + c[0];
    out[1] = (v[1] + w * uv[1]) + c[1];
    out[2] = (v[2] + w * uv[2]) + c[2];
}

double get_yaw(const double q[4])                        // base::getYaw (getEuler()[0])
{
    double R[9];
    q_to_mat(q, R);
    const double x = sqrt(R[8] * R[8] + R[7] * R[7]);
    return x > 1e-12 ? atan2(R[3], R[0]) : 0.0;
}

void remove_yaw(const double q[4], double out[4])       // base::removeYaw
{
    double a[4];
    q_from_yaw(-get_yaw(q), a);
    q_mul(a, q, out);
}

void q_from_mat(const double m[9], double q[4])          // Eigen quaternion from 3x3
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
        const int j = (i + 1) % 3, k = (j + 1) % 3;
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

// UpdateThreshold::test(udPose.inverse() * body2odometry)  src/Configuration.hpp:18-26 (Q6)
bool update_gate(double thr_distance, double thr_angle, const double ud[12], const double q_b[4], const double t_b[3])
{
    double Rb[9];
    q_to_mat(q_b, Rb);
    const double Ri[9] = {ud[0], ud[4], ud[8], ud[1], ud[5], ud[9], ud[2], ud[6], ud[10]};
    double ti[3], L[9], t[3];
    for (int r = 0; r < 3; ++r) ti[r] = -((Ri[r * 3 + 0] * ud[3] + Ri[r * 3 + 1] * ud[7]) + Ri[r * 3 + 2] * ud[11]);
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c)
            L[r * 3 + c] = (Ri[r * 3 + 0] * Rb[0 * 3 + c] + Ri[r * 3 + 1] * Rb[1 * 3 + c]) + Ri[r * 3 + 2] * Rb[2 * 3 + c];
        t[r] = ((Ri[r * 3 + 0] * t_b[0] + Ri[r * 3 + 1] * t_b[1]) + Ri[r * 3 + 2] * t_b[2]) + ti[r];
    }
    double q[4];
    q_from_mat(L, q);
    const double n = sqrt(q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    const double angle = n != 0.0 ? 2.0 * atan2(n, fabs(q[0])) : 0.0;
    const double dist = sqrt((t[0] * t[0] + t[1] * t[1]) + t[2] * t[2]);
    return angle > thr_distance || dist > thr_angle;
}

void lower_cholesky(const double S[9], double L[9])
{
    memset(L, 0, 9 * sizeof(double));
    for (int j = 0; j < 3; ++j) {
        double d = S[j * 3 + j];
        for (int k = 0; k < j; ++k) d -= L[j * 3 + k] * L[j * 3 + k];
        const double ljj = d > 0.0 ? sqrt(d) : 0.0;
        L[j * 3 + j] = ljj;
        for (int i = j + 1; i < 3; ++i) {
            double s = S[i * 3 + j];
            for (int k = 0; k < j; ++k) s -= L[i * 3 + k] * L[j * 3 + k];
            L[i * 3 + j] = ljj > 0.0 ? s / ljj : 0.0;
        }
    }
}

void set_translation_pose(double ud[12], double x, double y, double z)
{
    memset(ud, 0, 12 * sizeof(double));
    ud[0] = ud[5] = ud[10] = 1.0;
    ud[3] = x; ud[7] = y; ud[11] = z;
}

}  // namespace

// ---------------------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------------------
// ESLAM_FLAG_PROCESS_STATICS: the reference's function-static hash-respawn counter
// (src/PoseEstimator.cpp:239) and the C library's rand() (SurfaceHash::sample), shared by every
// context of the process that sets the flag -- Q11.  Not locked, like the reference's statics.
struct ProcessStatics {
    uint64_t hash_event = 0;
    dm_libc_rand_state libc;
    ProcessStatics() { dm_libc_srand(&libc, 1); }
};
static ProcessStatics& process_statics()
{
    static ProcessStatics ps;
    return ps;
}
// sharded contexts of this process with the flag: at most one.  Ranks driven from one process
// would advance the shared counter once each per step and draw each other's rand() values, so
// their respawns and hash indices would disagree (eslam_gpu_set_comm refuses a second one)
static std::atomic<int> g_statics_sharded{0};

struct eslam_ctx {
    eslam_config cfg;
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    // particles
    uint64_t n = 0, cap = 0;
    uint64_t gbase = 0, n_global = 0;
    DevState st[2] = {};
    void* state_mem = nullptr;
    uint32_t* marks = nullptr;
    uint32_t* tile_first = nullptr;         // row_first: source of every 64-output row's first output
    uint64_t* fin_word = nullptr;           // the fused finalize's epoch word (after the tile words)
    uint32_t pub_stride = 0;                // ScanParams::pub_stride
    uint64_t fin_epoch = 0;                 // fused finalize launches so far
    uint64_t* tile_sum = nullptr;           // per scan tile: exact fixed-point weight total (sharded K3a), or
                                            // one GPU: tag << 61 | total published by K3 (zeroed at allocation)
    uint32_t scan_tag = 0;                  // the last K3 launch's tag (1..7)
    uint32_t* anc = nullptr;
    bool has_anc = false;
    // per-particle maps (ESLAM_FLAG_PARTICLE_MAPS): the tables, pages and the copy-on-write scratch
    LocalMaps lm = {};
    bool lm_ready = false;                   // lm sized for the current map and particle count
    uint32_t* sid_mem = nullptr;             // 2 x cap: DevState::sid of both state buffers
    uint32_t* cow = nullptr;                 // owner, counts, free and sharing lists + the copy count
    uint32_t* lm_off = nullptr;              // per particle: its first page in its plan block (MergeParams::off)
    void* lm_job = nullptr;                  // per particle: the plan's record (MergeParams::job)
    uint16_t* lm_codes = nullptr;            // per particle: the plan's cell codes (MergeParams::codes)
    uint64_t lm_codes_cap = 0;               //   bytes (a small part's stride; grown for a large part's)
    // the scan of a map update on the device (MergeParams::sp): two slots, each staged through
    // pinned host memory; an update waits for the update before last to have read its slot
    void* scan_host[2] = {nullptr, nullptr};
    void* scan_dev[2] = {nullptr, nullptr};
    uint64_t scan_host_cap[2] = {0, 0}, scan_dev_cap[2] = {0, 0};
    hipEvent_t scan_ev[2] = {nullptr, nullptr};
    uint32_t scan_slot = 0;
    uint32_t* lm_poff = nullptr;             // per merge block: page offsets (+ total)
    uint32_t* lm_pgc = nullptr;              // the page collection's compaction counts
    void* match_sp = nullptr;                // processMap match: the sampled scan patches (device)
    uint64_t match_cap = 0;
    uint64_t* merge_cnt = nullptr;           // the map merge's statistics slots (2 x kMergeCounterSlots) and
                                             // the copy-on-write copies since the last merge
    // logDebug records of the last update (ESLAM_FLAG_RECORD_CONTACTS / log_debug)
    DebugRec dbg = {};
    uint64_t dbg_cap = 0;
    bool dbg_valid = false;
    // statistics and control
    Shard* shards = nullptr;
    Ctl* ctl = nullptr;
    Ctl* ctl_host = nullptr;    // pinned
    uint32_t* fault_host = nullptr;         // host-mapped: kFaultTimeout when a device wait gave up
    bool poisoned = false;                  // the particle set is undefined until re-initialised
    bool poison_pages = false;              // ... because the map pages ran out (kFaultPages)
    uint32_t spin_limit = kSpinLimit;       // polls of K3's cross-block waits (debug: 0 gives up at once)
    uint32_t* jump = nullptr;
    uint32_t jump_n = 1;                    // A^n_global, cached
    uint64_t jump_n_for = 0;
    double* scratch = nullptr;  // small device scratch (centroid, best index)
    double* scratch_host = nullptr;
    // map
    bool has_map = false;
    MapView map = {};
    uint32_t* d_cells = nullptr;
    float2* d_patch = nullptr;
    float* d_height = nullptr;
    uint32_t* d_occ = nullptr;               // MapView::occ
    uint4* d_cell_tab = nullptr;             // MapView::cell_tab
    uint32_t maxp = 4;
    // host-side filter state
    uint64_t proj_event = 0, init_event = 0, hash_event = 0;
    double ud_pose[12];
    double zcomp[4] = {1, 0, 0, 0};
    // multi-GPU (eslam_gpu_set_comm): this context is shard [gbase, gbase + n) of n_global
    bool sharded = false;
    bool statics_sharded = false;            // counted in g_statics_sharded
    eslam_comm comm = {};
    std::vector<uint64_t> gall;             // first global index of every rank (+ n_global)
    Shard* recs = nullptr;                  // gathered records of all ranks
    uint64_t* mg = nullptr;                 // MgBlock (device)
    void* rccl = nullptr;                   // ncclComm_t of eslam_gpu_set_comm_rccl (owned)
    uint64_t* mg_host = nullptr;            // pinned, host-mapped (k_segments_multi writes the totals there)
    uint64_t seg_epoch = 0;                 // the last k_segments_multi launch's epoch (mg_host[kHostEpoch])
    uint2* range = nullptr;                 // per particle: [lo, hi) of its global outputs
    void* sendbuf = nullptr; uint64_t send_cap = 0;
    void* recvbuf = nullptr; uint64_t recv_cap = 0;
    // per-particle maps on a sharded filter: the migrated particles' maps (a MapPayHdr per
    // record, then their pages as MapPayPage, in the records' order) and whether their tables
    // are still owed to them
    void* sendpay = nullptr; uint64_t sendpay_cap = 0;
    void* sendhdr = nullptr; uint64_t sendhdr_cap = 0;
    void* recvhdr = nullptr; uint64_t recvhdr_cap = 0;
    uint32_t* payoff = nullptr; uint64_t payoff_cap = 0;   // header prefix (send side, then receive side)
    uint32_t* rhead = nullptr; uint64_t rhead_cap = 0;     // received records: the record carrying each one's map
    uint64_t nrecv_maps = 0;                 // records whose maps wait in recvhdr / recvpay
    double* cent = nullptr; uint64_t cent_bytes = 0;   // sharded getCentroid's chunk records (set_comm)
    double* bspill = nullptr; uint64_t bspill_cap = 0;  // K1's parked per-bucket sums (k1_bspill_bytes)
    void* recvpay = nullptr; uint64_t recvpay_cap = 0;
    bool cow_pending = false;
    // a sharded update's exchange left for the next call: the segments kernel's
    // epoch and plan; the next step runs its own-output chunks before it completes it
    bool xpend = false;
    uint64_t xpend_epoch = 0;
    PlanParams xpend_pp = {};
    hipStream_t xstream = nullptr;           // the deferred exchange's stream (overlaps the own chunks)
    hipEvent_t ev_seg = nullptr;             // recorded after the segments kernel
    hipEvent_t ev_x = nullptr;               // recorded after the exchange's expand
    void* stage = nullptr; uint64_t stage_cap = 0;   // pinned staging (host-memory comm)
    // SurfaceHash (useHash)
    double map_scale[2] = {1, 1};
    bool has_hash = false;
    uint64_t hash_n = 0;
    double* d_hash = nullptr;                // 4 x hash_n: x, y, theta, z
    uint32_t* d_hash_blist = nullptr;        // pose indices grouped by bucket, sweep order
    std::vector<uint32_t> hash_bstart;       // bins^2 + 1
    std::vector<int32_t> hash_bucket;        // per pose (sweep order)
    dm_libc_rand_state libc;                 // rand() of SurfaceHash::sample (glibc, seed 1)
    // the hash-respawn counter and rand() in use: this context's own, or the process's
    // (ESLAM_FLAG_PROCESS_STATICS: the reference's function statics, Q11)
    uint64_t* hash_ev = nullptr;
    dm_libc_rand_state* libcp = nullptr;
    void* hsend = nullptr; uint64_t hsend_cap = 0;   // sharded respawn: candidate pairs out / in
    void* hrecv = nullptr; uint64_t hrecv_cap = 0;
    void* hsort = nullptr; uint64_t hsort_cap = 0;   // their keys, vals, sorted keys, order + sort scratch
    uint32_t* d_sort = nullptr;              // keys, vals, keys_out, order (4 x cap)
    uint64_t sort_cap = 0;
    void* sort_tmp = nullptr;
    size_t sort_tmp_bytes = 0;
    uint32_t* d_draws = nullptr;
    uint64_t draws_cap = 0;
    // diagnostics
    std::string err;
    bool timing = false;
    hipEvent_t ev[5] = {};                  // events of the step being recorded
    std::vector<hipEvent_t> ring;           // 5 events per recorded step (timing mode)
    uint32_t ring_steps = 0;
    std::vector<hipEvent_t> mring;          // 5 events per recorded map update (timing mode)
    uint32_t mring_steps = 0;
    std::vector<hipEvent_t> xring;          // 2 events per recorded map match (timing mode)
    uint32_t xring_steps = 0;
    eslam_kernel_times times = {};
};

#define HIPCHK(ctx, expr)                                                                    \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess) {                                                              \
            (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(e_);                  \
            return ESLAM_ERR_HIP;                                                            \
        }                                                                                    \
    } while (0)

static constexpr uint32_t kRingSteps = 2048;

static int settle(eslam_ctx* ctx);       // completes a deferred sharded exchange (run_update_tail_multi)

// multi-GPU scratch block (uint64 words, device + pinned host mirror)
namespace mg {
constexpr int kTotal = 0;                                   // this rank's fixed-point weight total
constexpr int kTotals = kTotal + 1;                         // [kMaxRanks] gathered totals
constexpr int kMirror = kTotals + kMaxRanks;                // [3] resample, minstd_start, scan_shift (k_finalize)
constexpr int kCounts = kMirror + 3;                        // [kMaxRanks] records sent to each rank
constexpr int kCountsAll = kCounts + kMaxRanks;             // [kMaxRanks^2] gathered counts
constexpr int kSendOff = kCountsAll + kMaxRanks * kMaxRanks;   // [kMaxRanks + 1]
constexpr int kSdEd = kSendOff + kMaxRanks + 1;             // [2 kMaxRanks]
constexpr int kFirstLast = kSdEd + 2 * kMaxRanks;           // [2 kMaxRanks]
constexpr int kBest = kFirstLast + 2 * kMaxRanks;           // [2] local best (key, global index)
constexpr int kBestAll = kBest + 2;                         // [2 kMaxRanks]
constexpr int kMaxW = kBestAll + 2 * kMaxRanks;             // local max weight (bits)
constexpr int kMaxWAll = kMaxW + 1;                         // [kMaxRanks]
constexpr int kHostEpoch = kMaxWAll + kMaxRanks;           // (mg_host only) the segments kernel's epoch
constexpr int kChunks = kHostEpoch + 1;                     // [2] own-output chunks of the slice (PlanParams::chunk_sel)
constexpr int kWords = kChunks + 2;
}  // namespace mg

// timing mode: event k (0..4) of the current step, kept in a ring so a whole timed region
// of back-to-back steps is measured without synchronising between steps
static void rec(eslam_ctx* ctx, int k)
{
    if (!ctx->timing) return;
    if (ctx->ring.empty()) {
        ctx->ring.resize(5 * kRingSteps);
        for (auto& e : ctx->ring) (void)hipEventCreate(&e);   // timing is diagnostic: best effort
    }
    if (ctx->ring_steps >= kRingSteps) return;
    (void)hipEventRecord(ctx->ring[5 * ctx->ring_steps + k], ctx->stream);
    if (k == 4) ctx->ring_steps++;
}

// timing mode: event k (0..3) of the current map update (start, gather, copy on write, merge)
static void mrec(eslam_ctx* ctx, int k)
{
    if (!ctx->timing) return;
    if (ctx->mring.empty()) {
        ctx->mring.resize(5 * kRingSteps);
        for (auto& e : ctx->mring) (void)hipEventCreate(&e);
    }
    if (ctx->mring_steps >= kRingSteps) return;
    (void)hipEventRecord(ctx->mring[5 * ctx->mring_steps + k], ctx->stream);
    if (k == 4) ctx->mring_steps++;
}

// timing mode: event k (0: start, 1: end) of the current map match
static void xrec(eslam_ctx* ctx, int k)
{
    if (!ctx->timing) return;
    if (ctx->xring.empty()) {
        ctx->xring.resize(2 * kRingSteps);
        for (auto& e : ctx->xring) (void)hipEventCreate(&e);
    }
    if (ctx->xring_steps >= kRingSteps) return;
    (void)hipEventRecord(ctx->xring[2 * ctx->xring_steps + k], ctx->stream);
    if (k == 1) ctx->xring_steps++;
}

static int fail(eslam_ctx* ctx, int code, const char* msg)
{
    if (ctx) ctx->err = msg;
    return code;
}

extern "C" int eslam_gpu_abi_version(void) { return ESLAM_ABI_VERSION; }

#ifndef ESLAM_BUILD_ID
#define ESLAM_BUILD_ID "unknown"
#endif
// SHA-256 of the sources, headers and flags this library was compiled from (build_lib.py)
extern "C" const char* eslam_gpu_build_id(void) { return ESLAM_BUILD_ID; }

extern "C" void eslam_config_default(eslam_config* c)
{
    memset(c, 0, sizeof(*c));
    c->seed = 42;
    c->particle_count = 250;
    c->min_effective = 50;
    c->initial_rotation_error[2] = 0.1;
    c->initial_translation_error[0] = 0.1;
    c->initial_translation_error[1] = 0.1;
    c->initial_translation_error[2] = 1.0;
    c->measurement_error = 0.1;
    c->discount_factor = 0.9;
    c->spread_threshold = 0.9;
    c->spread_translation_factor = 0.1;
    c->spread_rotation_factor = 0.05;
    c->slip_factor = 0.05;
    c->max_yaw_deviation = 15 * M_PI / 180.0;
    c->measurement_threshold_distance = 0.1;
    c->measurement_threshold_angle = 10 * M_PI / 180.0;
    c->use_slip_update = 0;
    c->use_shape_update = 1;
    c->min_contacts = 3;
    c->contact_likelihood_correction = 0.33;
    c->contact_point_radius = 0.01;
    c->hash_use = 0;
    c->hash_period = 10;
    c->hash_percentage = 0.05;
    c->hash_avg_factor = 0.1;
    c->hash_slope_bins = 20;
    c->hash_angular_steps = 16;
    c->log_debug = 0;
    c->flags = 0;
    c->local_map_pages = 0;
    c->max_sensor_range = 3.0;
    c->local_map_trail = 16;
}

extern "C" const char* eslam_gpu_last_error(const eslam_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

static int materialize(eslam_ctx* ctx);
static int store_receive(eslam_ctx* ctx);
static int local_maps_reset(eslam_ctx* ctx);
static GatherView gather_view(eslam_ctx* ctx);

static const char* kPoisonMsg =
    "resample scan: a cross-block wait gave up (a preceding tile's total or the finalize never arrived); "
    "the particle set is undefined until the filter is re-initialised";

// a device wait that gave up poisons the filter (kFaultTimeout): seen here from the
// host-mapped word without a synchronisation, so the next call after the faulting launch
// fails instead of building on a corrupt particle set
static const char* kPagesMsg =
    "per-particle maps: the page pool cannot hold a map update's pages even after a collection "
    "(raise eslam_config.local_map_pages); the particle set is undefined until the filter is re-initialised";

static int poison_fail(eslam_ctx* ctx)
{
    return ctx->poison_pages ? fail(ctx, ESLAM_ERR_OUT_OF_MEMORY, kPagesMsg) : fail(ctx, ESLAM_ERR_HIP, kPoisonMsg);
}

static int check_poisoned(eslam_ctx* ctx)
{
    if (!ctx->poisoned) {
        const uint32_t f = __atomic_load_n(ctx->fault_host, __ATOMIC_ACQUIRE);
        if (f & (kFaultTimeout | kFaultPages)) {
            ctx->poisoned = true;
            ctx->poison_pages = (f & kFaultPages) != 0;
        }
    }
    return ctx->poisoned ? poison_fail(ctx) : ESLAM_OK;
}

static int read_ctl(eslam_ctx* ctx)
{
    HIPCHK(ctx, hipMemcpyAsync(ctx->ctl_host, ctx->ctl, sizeof(Ctl), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    return ESLAM_OK;
}

static int write_ctl(eslam_ctx* ctx)
{
    HIPCHK(ctx, hipMemcpyAsync(ctx->ctl, ctx->ctl_host, sizeof(Ctl), hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    return ESLAM_OK;
}

extern "C" int eslam_gpu_create(const eslam_config* cfg, int device, eslam_ctx** out)
{
    if (!cfg || !out) return ESLAM_ERR_INVALID_ARG;
    *out = nullptr;
    eslam_ctx* ctx = new eslam_ctx();
    ctx->cfg = *cfg;
    ctx->device = device;
    set_translation_pose(ctx->ud_pose, 1000, 0, 0);
    int rc = ESLAM_OK;
    do {
        // nD <= 64 J and the contact points <= ESLAM_MAX_CONTACTS nD share one 32-bit word (K1)
        if (cfg->sum_chunk_rows > 31) { rc = fail(ctx, ESLAM_ERR_INVALID_ARG, "sum_chunk_rows: at most 31"); break; }
        hipError_t e = hipSetDevice(device);
        if (e != hipSuccess) { ctx->err = std::string("hipSetDevice: ") + hipGetErrorString(e); rc = ESLAM_ERR_HIP; break; }
        if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) { rc = fail(ctx, ESLAM_ERR_HIP, "stream"); break; }
        ctx->own_stream = true;
        if (hipMalloc(&ctx->shards, sizeof(Shard) * kNShard) != hipSuccess ||
            hipMalloc(&ctx->ctl, sizeof(Ctl)) != hipSuccess ||
            hipHostMalloc(&ctx->ctl_host, sizeof(Ctl)) != hipSuccess ||
            hipMalloc(&ctx->jump, sizeof(uint32_t) * (2048 + 2048 + 1024)) != hipSuccess ||
            hipMalloc(&ctx->scratch, 4096) != hipSuccess ||
            hipHostMalloc(&ctx->scratch_host, 4096) != hipSuccess ||
            hipHostMalloc(&ctx->fault_host, 64) != hipSuccess) {
            rc = fail(ctx, ESLAM_ERR_OUT_OF_MEMORY, "device allocation failed");
            break;
        }
        if (hipMemset(ctx->shards, 0, sizeof(Shard) * kNShard) != hipSuccess) { rc = fail(ctx, ESLAM_ERR_HIP, "shard reset"); break; }
        memset(ctx->ctl_host, 0, sizeof(Ctl));
        memset(ctx->fault_host, 0, 64);
        ctx->ctl_host->minstd = dm_minstd_seed(cfg->seed);     // ParticleFilter(seed)
        dm_libc_srand(&ctx->libc, 1);                            // the reference never seeds rand()
        if (cfg->flags & ESLAM_FLAG_PROCESS_STATICS) {
            ProcessStatics& ps = process_statics();
            ctx->hash_ev = &ps.hash_event;
            ctx->libcp = &ps.libc;
        } else {
            ctx->hash_ev = &ctx->hash_event;
            ctx->libcp = &ctx->libc;
        }
        ctx->ctl_host->max_weight = 0.0;                         // PoseEstimator ctor
        ctx->ctl_host->wexp = 1;
        ctx->ctl_host->scan_shift = 60;
        if (hipMemcpy(ctx->ctl, ctx->ctl_host, sizeof(Ctl), hipMemcpyHostToDevice) != hipSuccess) {
            rc = fail(ctx, ESLAM_ERR_HIP, "control block upload");
            break;
        }
        // minstd jump tables
        std::vector<uint32_t> jt(2048 + 2048 + 1024);
        uint32_t a = 1;
        for (int i = 0; i < 2048; ++i) { jt[i] = a; a = dm_mulmod31(a, DM_MINSTD_A); }
        const uint32_t a11 = dm_minstd_pow(1ull << 11);
        a = 1;
        for (int i = 0; i < 2048; ++i) { jt[2048 + i] = a; a = dm_mulmod31(a, a11); }
        const uint32_t a22 = dm_minstd_pow(1ull << 22);
        a = 1;
        for (int i = 0; i < 1024; ++i) { jt[4096 + i] = a; a = dm_mulmod31(a, a22); }
        if (hipMemcpy(ctx->jump, jt.data(), jt.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
            rc = fail(ctx, ESLAM_ERR_HIP, "jump table upload");
            break;
        }
        bool ev_ok = true;
        for (auto& e2 : ctx->ev) ev_ok &= hipEventCreate(&e2) == hipSuccess;
        if (!ev_ok) { rc = fail(ctx, ESLAM_ERR_HIP, "event create"); break; }
        if (hipDeviceSynchronize() != hipSuccess) { rc = fail(ctx, ESLAM_ERR_HIP, "device synchronize"); break; }
    } while (0);
    if (rc != ESLAM_OK) {
        fprintf(stderr, "eslam_gpu_create: %s\n", ctx->err.c_str());
        eslam_gpu_destroy(ctx);
        return rc;
    }
    *out = ctx;
    return ESLAM_OK;
}

// ancestors are kept when asked for, and always while contact records are (the records of
// output i are those of its ancestor)
static bool record_contacts(const eslam_ctx* ctx)
{
    return (ctx->cfg.flags & ESLAM_FLAG_RECORD_CONTACTS) || ctx->cfg.log_debug;
}
static bool keep_ancestors(const eslam_ctx* ctx)
{
    return (ctx->cfg.flags & ESLAM_FLAG_RECORD_ANCESTORS) || record_contacts(ctx);
}

static void free_debug(eslam_ctx* ctx)
{
    (void)hipFree(ctx->dbg.meas); (void)hipFree(ctx->dbg.ncp); (void)hipFree(ctx->dbg.cp); (void)hipFree(ctx->dbg.resampled);
    ctx->dbg = DebugRec{};
    ctx->dbg_cap = 0;
    ctx->dbg_valid = false;
}

static bool particle_maps(const eslam_ctx* ctx) { return (ctx->cfg.flags & ESLAM_FLAG_PARTICLE_MAPS) != 0; }

static const LocalMaps* store_of(const eslam_ctx* ctx) { return particle_maps(ctx) ? &ctx->lm : nullptr; }

static void free_local_maps(eslam_ctx* ctx)
{
    (void)hipFree(ctx->lm.ctr); (void)hipFree(ctx->lm.slot); (void)hipFree(ctx->lm.page); (void)hipFree(ctx->lm.tgen);
    (void)hipFree(ctx->lm.owner); (void)hipFree(ctx->lm.frees); (void)hipFree(ctx->lm.mark);
    (void)hipFree(ctx->lm_off); (void)hipFree(ctx->lm_job); (void)hipFree(ctx->lm_codes); ctx->lm_codes_cap = 0; (void)hipFree(ctx->lm_poff); (void)hipFree(ctx->lm_pgc); (void)hipFree(ctx->match_sp);
    ctx->lm = LocalMaps{};
    ctx->lm_off = nullptr; ctx->lm_job = nullptr; ctx->lm_codes = nullptr; ctx->lm_poff = nullptr; ctx->lm_pgc = nullptr; ctx->match_sp = nullptr; ctx->match_cap = 0;
    ctx->lm_ready = false;
}

static void free_particles(eslam_ctx* ctx)
{
    free_debug(ctx);
    free_local_maps(ctx);
    (void)hipFree(ctx->sid_mem); (void)hipFree(ctx->cow); (void)hipFree(ctx->merge_cnt);
    ctx->merge_cnt = nullptr;
    ctx->sid_mem = nullptr;
    ctx->cow = nullptr;
    ctx->st[0].sid = ctx->st[1].sid = nullptr;
    (void)hipFree(ctx->state_mem); ctx->state_mem = nullptr;
    (void)hipFree(ctx->marks); ctx->marks = nullptr;
    (void)hipFree(ctx->tile_first); ctx->tile_first = nullptr;
    (void)hipFree(ctx->tile_sum); ctx->tile_sum = nullptr;
    (void)hipFree(ctx->anc); ctx->anc = nullptr;
    (void)hipFree(ctx->range); ctx->range = nullptr;
    ctx->n = ctx->cap = 0;
    ctx->has_anc = false;
}

static void free_map(eslam_ctx* ctx)
{
    (void)hipFree(ctx->d_cells); (void)hipFree(ctx->d_patch); (void)hipFree(ctx->d_height); (void)hipFree(ctx->d_occ);
    (void)hipFree(ctx->d_cell_tab);
    ctx->d_cells = nullptr; ctx->d_patch = nullptr; ctx->d_height = nullptr; ctx->d_occ = nullptr;
    ctx->d_cell_tab = nullptr;
    ctx->has_map = false;
}

namespace { void rccl_release(eslam_ctx* ctx); }

extern "C" void eslam_gpu_destroy(eslam_ctx* ctx)
{
    if (!ctx) return;
    // never collective: a deferred exchange still pending is dropped (eslam_gpu_finish is the
    // collective that completes it); destroy may run on an error path of one rank or after the
    // caller's communicator is gone, so it must not wait for the other ranks
    ctx->xpend = false;
    if (ctx->statics_sharded) g_statics_sharded.fetch_sub(1);
    ctx->statics_sharded = false;
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->xstream) { (void)hipStreamSynchronize(ctx->xstream); (void)hipStreamDestroy(ctx->xstream); }
    if (ctx->ev_seg) (void)hipEventDestroy(ctx->ev_seg);
    if (ctx->ev_x) (void)hipEventDestroy(ctx->ev_x);
    rccl_release(ctx);
    free_particles(ctx);
    free_map(ctx);
    (void)hipFree(ctx->shards); (void)hipFree(ctx->ctl); (void)hipHostFree(ctx->ctl_host); (void)hipFree(ctx->jump);
    (void)hipFree(ctx->scratch); (void)hipHostFree(ctx->scratch_host); (void)hipHostFree(ctx->fault_host);
    (void)hipFree(ctx->recs); (void)hipFree(ctx->mg); (void)hipHostFree(ctx->mg_host);
    (void)hipFree(ctx->sendbuf); (void)hipFree(ctx->recvbuf); (void)hipHostFree(ctx->stage);
    (void)hipFree(ctx->sendpay); (void)hipFree(ctx->recvpay); (void)hipFree(ctx->cent); (void)hipFree(ctx->bspill);
    (void)hipFree(ctx->sendhdr); (void)hipFree(ctx->recvhdr); (void)hipFree(ctx->payoff); (void)hipFree(ctx->rhead);
    (void)hipFree(ctx->d_hash); (void)hipFree(ctx->d_hash_blist); (void)hipFree(ctx->d_sort); (void)hipFree(ctx->sort_tmp); (void)hipFree(ctx->d_draws);
    (void)hipFree(ctx->hsend); (void)hipFree(ctx->hrecv); (void)hipFree(ctx->hsort);
    for (auto& e : ctx->ev) if (e) (void)hipEventDestroy(e);
    for (auto& e : ctx->ring) if (e) (void)hipEventDestroy(e);
    for (auto& e : ctx->mring) if (e) (void)hipEventDestroy(e);
    for (auto& e : ctx->xring) if (e) (void)hipEventDestroy(e);
    for (int k = 0; k < 2; ++k) {
        if (ctx->scan_ev[k]) (void)hipEventDestroy(ctx->scan_ev[k]);
        (void)hipHostFree(ctx->scan_host[k]);
        (void)hipFree(ctx->scan_dev[k]);
    }
    if (ctx->own_stream && ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

// collective on a sharded filter (every rank calls it at the same point): completes the last
// update's deferred exchange if this rank still owes it; a no-op otherwise
extern "C" int eslam_gpu_finish(eslam_ctx* ctx)
{
    if (!ctx) return ESLAM_ERR_INVALID_ARG;
    if (ctx->poisoned) { ctx->xpend = false; return ESLAM_OK; }
    if (const int rc_ = settle(ctx)) return rc_;
    if (ctx->stream) HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    return ESLAM_OK;
}

extern "C" int eslam_gpu_set_stream(eslam_ctx* ctx, void* s)
{
    if (!ctx) return ESLAM_ERR_INVALID_ARG;
    if (const int rc_ = settle(ctx)) return rc_;    // a deferred sharded exchange first
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    if (s) {
        if (ctx->own_stream) (void)hipStreamDestroy(ctx->stream);
        ctx->stream = (hipStream_t)s;
        ctx->own_stream = false;
    }
    return ESLAM_OK;
}

// 256-byte aligned SoA carve-out: 7 fp64 arrays + 1 byte array, two copies
static int alloc_particles(eslam_ctx* ctx, uint64_t n)
{
    if (n >= (1ull << 32) - 1) return fail(ctx, ESLAM_ERR_INVALID_ARG, "particle count must be < 2^32 - 1");
    if (ctx->sharded && n != ctx->gall[ctx->comm.rank + 1] - ctx->gall[ctx->comm.rank])
        return fail(ctx, ESLAM_ERR_INVALID_ARG, "sharded context: particle count must equal this rank's shard size");
    free_particles(ctx);
    const uint64_t cap = n ? n : 1;
    auto al = [](uint64_t b) { return (b + 255) & ~255ull; };
    const uint64_t per = 7 * al(cap * 8) + al(cap);
    HIPCHK(ctx, hipMalloc(&ctx->state_mem, 2 * per));
    for (int k = 0; k < 2; ++k) {
        char* p = (char*)ctx->state_mem + k * per;
        DevState& s = ctx->st[k];
        double** f[7] = {&s.x, &s.y, &s.th, &s.z, &s.zs, &s.w, &s.mprob};
        for (int j = 0; j < 7; ++j) { *f[j] = (double*)p; p += al(cap * 8); }
        s.flags = (uint8_t*)p;
    }
    const uint64_t ntiles = (cap + kBlock - 1) / kBlock;                // the smallest scan tile (scan_items)
    HIPCHK(ctx, hipMalloc(&ctx->marks, cap * 4));
    HIPCHK(ctx, hipMalloc(&ctx->tile_first, ((cap + kRow - 1) / kRow) * 4));
    // the tile words, then (in a line of its own) the fused finalize's epoch word
    // K3's kPubReplicas copies of the tile words (4 KB-aligned regions, 256 B apart beyond
    // that, so the copies fall on different memory channels), then the epoch word's line
    ctx->pub_stride = (uint32_t)(((ntiles + 511) & ~511ull) + 32);
    const uint64_t fin_at = (uint64_t)kPubReplicas * ctx->pub_stride;
    HIPCHK(ctx, hipMalloc(&ctx->tile_sum, (fin_at + 16) * 8));
    HIPCHK(ctx, hipMemset(ctx->tile_sum, 0, (fin_at + 16) * 8));          // tag / epoch 0: never published
    ctx->fin_word = ctx->tile_sum + fin_at;
    HIPCHK(ctx, hipMemset(ctx->marks, 0, cap * 4));
    if (keep_ancestors(ctx)) HIPCHK(ctx, hipMalloc(&ctx->anc, cap * 4));
    if (particle_maps(ctx)) {
        // the table names of both state buffers; the tables and pages come with the map
        // (local_maps_reset: their window size follows the map's cell size)
        HIPCHK(ctx, hipMalloc(&ctx->sid_mem, 2 * cap * 4));
        ctx->st[0].sid = ctx->sid_mem;
        ctx->st[1].sid = ctx->sid_mem + cap;
        HIPCHK(ctx, hipMalloc(&ctx->cow, cow_words(cap) * 4));
        HIPCHK(ctx, hipMalloc(&ctx->merge_cnt, kMergeCounters * kMergeCounterSlots * sizeof(uint64_t)));
        HIPCHK(ctx, hipMemset(ctx->merge_cnt, 0, kMergeCounters * kMergeCounterSlots * sizeof(uint64_t)));
    }
    ctx->n = n;
    ctx->cap = cap;
    if (ctx->sharded) {
        HIPCHK(ctx, hipMalloc(&ctx->range, cap * sizeof(uint2)));
    } else {
        ctx->n_global = n;
        ctx->gbase = 0;
    }
    return local_maps_reset(ctx);
}

// Per-particle maps, sized for the current map and particle count: every
// particle names its own empty table (cloneMaps of the reference's empty grid template,
// src/EmbodiedSlamFilter.cpp:131-134), every page free.  A window of (2h + 1)^2 tiles reaching
// maxSensorRange (dm_lm_half of the cell size); a pool of 2 x cap tables and local_map_pages
// pages per particle.  Runs at particle allocation and at set_map (the tables name cells of
// the map, so a new map starts them over).
static int local_maps_reset(eslam_ctx* ctx)
{
    free_local_maps(ctx);
    if (!particle_maps(ctx) || !ctx->has_map || !ctx->n) return ESLAM_OK;
    const double r = ctx->cfg.max_sensor_range;
    if (!(r == r) || r < 0.0 || r > 1e6) return fail(ctx, ESLAM_ERR_INVALID_ARG, "max_sensor_range must be finite and >= 0");
    LocalMaps& lm = ctx->lm;
    lm.hx = dm_lm_half(r, ctx->map_scale[0]);
    lm.hy = dm_lm_half(r, ctx->map_scale[1]);
    lm.wx = 2 * lm.hx + 1;
    lm.wy = 2 * lm.hy + 1;
    if (ctx->cfg.local_map_trail > 4096) return fail(ctx, ESLAM_ERR_INVALID_ARG, "local_map_trail: at most 4096 tiles");
    lm.V = ctx->cfg.local_map_trail;
    // a table's row: the window's slots, padded (NONE) to whole 16-byte words, then the trail's
    // V 16-byte entries
    lm.S = ((lm.wx * lm.wy + 3u) & ~3u) + 4u * lm.V;
    lm.mx = lm_magic(lm.wx);
    lm.my = lm_magic(lm.wy);
    lm.bx = lm.wx * (((1u << 29) + lm.wx - 1) / lm.wx);
    lm.by = lm.wy * (((1u << 29) + lm.wy - 1) / lm.wy);
    const uint64_t cap = ctx->cap, pool = store_pool(cap);
    const uint64_t per = ctx->cfg.local_map_pages ? ctx->cfg.local_map_pages : kDefaultMapPages;
    lm.ntables = pool;
    lm.npages = cap * per;
    if (lm.npages >= 0xffffffffull) return fail(ctx, ESLAM_ERR_INVALID_ARG, "per-particle map pool: at most 2^32 - 1 pages");
    const uint64_t ptiles = (lm.npages + kCompactTileItems - 1) / kCompactTileItems;
    HIPCHK(ctx, hipMalloc(&lm.ctr, pool * sizeof(int2)));
    HIPCHK(ctx, hipMalloc(&lm.slot, pool * lm.S * 4));
    HIPCHK(ctx, hipMalloc(&lm.tgen, pool * 4));
    HIPCHK(ctx, hipMalloc(&lm.page, lm.npages * DM_LM_PAGE_CELLS * sizeof(float2)));
    HIPCHK(ctx, hipMalloc(&lm.owner, lm.npages * 8));
    HIPCHK(ctx, hipMalloc(&lm.frees, lm.npages * 4));
    HIPCHK(ctx, hipMalloc(&lm.mark, ((lm.npages + 15) / 16) * 16));
    HIPCHK(ctx, hipMalloc(&ctx->lm_off, cap * 4));
    HIPCHK(ctx, hipMalloc(&ctx->lm_job, cap * sizeof(MergeJob)));
    ctx->lm_codes_cap = cap * 2 * kScanPartSmall;
    HIPCHK(ctx, hipMalloc(&ctx->lm_codes, ctx->lm_codes_cap));
    HIPCHK(ctx, hipMalloc(&ctx->lm_poff, ((cap + kLmBlock - 1) / kLmBlock + 1) * 4));
    HIPCHK(ctx, hipMalloc(&ctx->lm_pgc, (ptiles + 1) * 4));
    HIPCHK(ctx, eslam_launch_store_init(ctx->sid_mem, &lm, cap, pool, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    // the free list holds every page (k_store_init: frees[p] = p)
    int rc = read_ctl(ctx);
    if (rc) return rc;
    ctx->ctl_host->pg_cursor = 0;
    ctx->ctl_host->pg_nfree = lm.npages;
    ctx->ctl_host->pg_total = 0;
    ctx->ctl_host->pg_gc = 0;
    rc = write_ctl(ctx);
    if (rc) return rc;
    ctx->lm_ready = true;
    return ESLAM_OK;
}

// ---------------------------------------------------------------------------------------
// multi-GPU plumbing: the three exchanges of an update go through the user's collectives
// ---------------------------------------------------------------------------------------
static int grow(eslam_ctx* ctx, void** buf, uint64_t* cap, uint64_t bytes, bool pinned)
{
    if (bytes <= *cap) return ESLAM_OK;
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    const uint64_t want = bytes + bytes / 4 + 4096;
    if (pinned) {
        (void)hipHostFree(*buf);
        *buf = nullptr; *cap = 0;
        HIPCHK(ctx, hipHostMalloc(buf, want));
    } else {
        (void)hipFree(*buf);
        *buf = nullptr; *cap = 0;
        HIPCHK(ctx, hipMalloc(buf, want));
    }
    *cap = want;
    return ESLAM_OK;
}

// all_gather of `bytes` per rank from device memory into device memory
static int comm_allgather(eslam_ctx* ctx, const void* dsend, void* drecv, uint64_t bytes)
{
    const eslam_comm& c = ctx->comm;
    if (c.device_memory) {
        if (c.allgather(c.user, dsend, drecv, bytes, (void*)ctx->stream) != 0)
            return fail(ctx, ESLAM_ERR_COMM, "allgather callback failed");
        return ESLAM_OK;
    }
    int rc = grow(ctx, &ctx->stage, &ctx->stage_cap, bytes * (c.nranks + 1), true);
    if (rc) return rc;
    char* h = (char*)ctx->stage;
    HIPCHK(ctx, hipMemcpyAsync(h, dsend, bytes, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    if (c.allgather(c.user, h, h + bytes, bytes, nullptr) != 0) return fail(ctx, ESLAM_ERR_COMM, "allgather callback failed");
    HIPCHK(ctx, hipMemcpyAsync(drecv, h + bytes, bytes * c.nranks, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));     // the staging buffer is reused
    return ESLAM_OK;
}

static int comm_alltoallv(eslam_ctx* ctx, const void* dsend, const uint64_t* sb, void* drecv, const uint64_t* rb,
                          hipStream_t stream = nullptr)
{
    const eslam_comm& c = ctx->comm;
    if (!stream) stream = ctx->stream;
    if (c.device_memory) {
        if (c.alltoallv(c.user, dsend, sb, drecv, rb, (void*)stream) != 0)
            return fail(ctx, ESLAM_ERR_COMM, "alltoallv callback failed");
        return ESLAM_OK;
    }
    uint64_t ts = 0, tr = 0;
    for (int r = 0; r < c.nranks; ++r) { ts += sb[r]; tr += rb[r]; }
    int rc = grow(ctx, &ctx->stage, &ctx->stage_cap, ts + tr + 64, true);
    if (rc) return rc;
    char* h = (char*)ctx->stage;
    char* hr = h + ((ts + 63) & ~63ull);
    if (ts) HIPCHK(ctx, hipMemcpyAsync(h, dsend, ts, hipMemcpyDeviceToHost, stream));
    HIPCHK(ctx, hipStreamSynchronize(stream));
    if (c.alltoallv(c.user, h, sb, hr, rb, nullptr) != 0) return fail(ctx, ESLAM_ERR_COMM, "alltoallv callback failed");
    if (tr) HIPCHK(ctx, hipMemcpyAsync(drecv, hr, tr, hipMemcpyHostToDevice, stream));
    HIPCHK(ctx, hipStreamSynchronize(stream));
    return ESLAM_OK;
}

static PlanParams plan_params(eslam_ctx* ctx)
{
    PlanParams pp;
    memset(&pp, 0, sizeof(pp));
    pp.n_global = ctx->n_global;
    pp.rank = ctx->comm.rank;
    pp.nranks = ctx->comm.nranks;
    for (int r = 0; r <= ctx->comm.nranks; ++r) pp.gbase[r] = ctx->gall[r];
    pp.chunk_sel = ctx->mg + mg::kChunks;
    pp.n_local = ctx->n;
    pp.J = dm_chunk_rows_cfg(ctx->n_global, ctx->cfg.sum_chunk_rows);
    return pp;
}

// sharded getCentroid: this rank's chunk records (padded to the largest shard), all ranks'
// (G x that), and the tree's two ping-pong levels over the global chunks; 5 doubles a record
static uint64_t centroid_bytes(const uint64_t* gall, int G, uint32_t J)
{
    const uint64_t csz = 64ull * J;
    uint64_t maxch = 1, total = 0;
    for (int r = 0; r < G; ++r) {
        const uint64_t c = (gall[r + 1] - gall[r] + csz - 1) / csz;
        maxch = c > maxch ? c : maxch;
        total += c;
    }
    return (maxch + (uint64_t)G * maxch + 2 * (total ? total : 1)) * 5 * sizeof(double);
}

extern "C" int eslam_gpu_set_comm(eslam_ctx* ctx, const eslam_comm* comm, uint64_t n_global, const uint64_t* shard_gbase)
{
    if (!ctx) return ESLAM_ERR_INVALID_ARG;
    if (const int rc_ = settle(ctx)) return rc_;    // a deferred sharded exchange first
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    free_particles(ctx);
    if (ctx->statics_sharded) g_statics_sharded.fetch_sub(1);
    ctx->statics_sharded = false;
    if (!comm) {
        ctx->sharded = false;
        ctx->gall.clear();
        ctx->gbase = 0;
        ctx->n_global = 0;
        return ESLAM_OK;
    }
    if (!shard_gbase || !comm->allgather || !comm->alltoallv || comm->nranks < 1 || comm->nranks > kMaxRanks ||
        comm->rank < 0 || comm->rank >= comm->nranks)
        return fail(ctx, ESLAM_ERR_INVALID_ARG, "eslam_gpu_set_comm: bad communicator (1 <= nranks <= 16)");
    if (n_global == 0 || n_global > (1ull << 30) - 64)     // resample mark encoding (kMarkOwn)
        return fail(ctx, ESLAM_ERR_INVALID_ARG, "eslam_gpu_set_comm: n_global must be in [1, 2^30 - 64]");
    const uint64_t csz = 64ull * dm_chunk_rows_cfg(n_global, ctx->cfg.sum_chunk_rows);
    if (shard_gbase[0] != 0 || shard_gbase[comm->nranks] != n_global)
        return fail(ctx, ESLAM_ERR_INVALID_ARG, "eslam_gpu_set_comm: shard_gbase must run from 0 to n_global");
    for (int r = 0; r < comm->nranks; ++r) {
        if (shard_gbase[r + 1] <= shard_gbase[r])
            return fail(ctx, ESLAM_ERR_INVALID_ARG, "eslam_gpu_set_comm: every shard needs at least one particle");
        if (shard_gbase[r] % csz)
            return fail(ctx, ESLAM_ERR_INVALID_ARG, "eslam_gpu_set_comm: shard starts must be multiples of the summation chunk");
    }
    if (!ctx->mg) {
        HIPCHK(ctx, hipMalloc(&ctx->recs, sizeof(Shard) * kNShard * kMaxRanks));
        HIPCHK(ctx, hipMalloc(&ctx->mg, mg::kWords * 8));
        HIPCHK(ctx, hipHostMalloc(&ctx->mg_host, mg::kWords * 8));
        HIPCHK(ctx, hipMemset(ctx->recs, 0, sizeof(Shard) * kNShard * kMaxRanks));
        HIPCHK(ctx, hipMemset(ctx->mg, 0, mg::kWords * 8));
    }
    {
        // getCentroid's buffer (centroid_bytes): sized by the shard table, allocated here so
        // the per-step getCentroid of a Rock task allocates nothing
        const uint64_t need = centroid_bytes(shard_gbase, comm->nranks, dm_chunk_rows_cfg(n_global, ctx->cfg.sum_chunk_rows));
        if (need > ctx->cent_bytes) {
            (void)hipFree(ctx->cent);
            ctx->cent = nullptr;
            ctx->cent_bytes = 0;
            HIPCHK(ctx, hipMalloc(&ctx->cent, need));
            ctx->cent_bytes = need;
        }
    }
    if ((ctx->cfg.flags & ESLAM_FLAG_PROCESS_STATICS) && comm->nranks > 1) {
        if (g_statics_sharded.fetch_add(1) != 0) {
            g_statics_sharded.fetch_sub(1);
            return fail(ctx, ESLAM_ERR_INVALID_ARG,
                        "eslam_gpu_set_comm: ESLAM_FLAG_PROCESS_STATICS allows one sharded context per process "
                        "(ranks in one process would share the respawn counter and rand())");
        }
        ctx->statics_sharded = true;
    }
    ctx->comm = *comm;
    ctx->sharded = true;
    ctx->gall.assign(shard_gbase, shard_gbase + comm->nranks + 1);
    ctx->n_global = n_global;
    ctx->gbase = shard_gbase[comm->rank];
    return ESLAM_OK;
}

// ---------------------------------------------------------------------------------------
// RCCL transport (eslam_gpu_set_comm_rccl): the eslam_comm callbacks implemented in C++ on
// the context's stream, RCCL resolved at run time (the process's librccl.so.1 -- the one
// torch loaded, if any -- so one RCCL serves both)
// ---------------------------------------------------------------------------------------
namespace {
struct RcclApi {
    bool ok = false;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
};

const RcclApi& rccl_api()
{
    static RcclApi api = [] {
        RcclApi a;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return a;
#define ESLAM_SYM(f, name) a.f = reinterpret_cast<decltype(a.f)>(dlsym(h, name))
        ESLAM_SYM(get_unique_id, "ncclGetUniqueId");
        ESLAM_SYM(comm_init_rank, "ncclCommInitRank");
        ESLAM_SYM(comm_destroy, "ncclCommDestroy");
        ESLAM_SYM(all_gather, "ncclAllGather");
        ESLAM_SYM(send, "ncclSend");
        ESLAM_SYM(recv, "ncclRecv");
        ESLAM_SYM(group_start, "ncclGroupStart");
        ESLAM_SYM(group_end, "ncclGroupEnd");
        ESLAM_SYM(error_string, "ncclGetErrorString");
#undef ESLAM_SYM
        a.ok = a.get_unique_id && a.comm_init_rank && a.comm_destroy && a.all_gather && a.send && a.recv &&
               a.group_start && a.group_end && a.error_string;
        return a;
    }();
    return api;
}

int rccl_allgather_cb(void* user, const void* send, void* recv, uint64_t bytes, void* stream)
{
    eslam_ctx* ctx = static_cast<eslam_ctx*>(user);
    const RcclApi& a = rccl_api();
    return a.all_gather(send, recv, bytes, ncclUint8, static_cast<ncclComm_t>(ctx->rccl), static_cast<hipStream_t>(stream)) ==
                   ncclSuccess ? 0 : 1;
}

int rccl_alltoallv_cb(void* user, const void* send, const uint64_t* send_bytes, void* recv, const uint64_t* recv_bytes,
                      void* stream)
{
    eslam_ctx* ctx = static_cast<eslam_ctx*>(user);
    const RcclApi& a = rccl_api();
    const ncclComm_t comm = static_cast<ncclComm_t>(ctx->rccl);
    const hipStream_t st = static_cast<hipStream_t>(stream);
    uint64_t so = 0, ro = 0;
    if (a.group_start() != ncclSuccess) return 1;
    int bad = 0;
    for (int r = 0; r < ctx->comm.nranks; ++r) {
        if (send_bytes[r]) bad |= a.send(static_cast<const char*>(send) + so, send_bytes[r], ncclUint8, r, comm, st) != ncclSuccess;
        if (recv_bytes[r]) bad |= a.recv(static_cast<char*>(recv) + ro, recv_bytes[r], ncclUint8, r, comm, st) != ncclSuccess;
        so += send_bytes[r];
        ro += recv_bytes[r];
    }
    bad |= a.group_end() != ncclSuccess;
    return bad;
}

void rccl_release(eslam_ctx* ctx)
{
    if (ctx->rccl) rccl_api().comm_destroy(static_cast<ncclComm_t>(ctx->rccl));
    ctx->rccl = nullptr;
}
}  // namespace

extern "C" int eslam_gpu_rccl_unique_id(uint8_t id[ESLAM_RCCL_ID_BYTES])
{
    if (!id) return ESLAM_ERR_INVALID_ARG;
    const RcclApi& a = rccl_api();
    if (!a.ok) return ESLAM_ERR_UNSUPPORTED;
    ncclUniqueId u;
    if (a.get_unique_id(&u) != ncclSuccess) return ESLAM_ERR_COMM;
    static_assert(sizeof(u) == ESLAM_RCCL_ID_BYTES, "ncclUniqueId size");
    memcpy(id, &u, sizeof(u));
    return ESLAM_OK;
}

extern "C" int eslam_gpu_set_comm_rccl(eslam_ctx* ctx, int32_t nranks, int32_t rank, const uint8_t id[ESLAM_RCCL_ID_BYTES],
                                       uint64_t n_global, const uint64_t* shard_gbase)
{
    if (!ctx || !id) return ESLAM_ERR_INVALID_ARG;
    if (const int rc_ = settle(ctx)) return rc_;    // a deferred sharded exchange first
    const RcclApi& a = rccl_api();
    if (!a.ok) return fail(ctx, ESLAM_ERR_UNSUPPORTED, "eslam_gpu_set_comm_rccl: librccl.so.1 not found");
    if (nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks)
        return fail(ctx, ESLAM_ERR_INVALID_ARG, "eslam_gpu_set_comm_rccl: bad communicator (1 <= nranks <= 16)");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    rccl_release(ctx);
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    ncclComm_t comm = nullptr;
    const ncclResult_t r = a.comm_init_rank(&comm, nranks, u, rank);
    if (r != ncclSuccess)
        return fail(ctx, ESLAM_ERR_COMM, (std::string("ncclCommInitRank: ") + a.error_string(r)).c_str());
    ctx->rccl = comm;
    eslam_comm c;
    memset(&c, 0, sizeof(c));
    c.user = ctx;
    c.rank = rank;
    c.nranks = nranks;
    c.device_memory = 1;
    c.allgather = rccl_allgather_cb;
    c.alltoallv = rccl_alltoallv_cb;
    const int rc = eslam_gpu_set_comm(ctx, &c, n_global, shard_gbase);
    if (rc) rccl_release(ctx);
    return rc;
}

extern "C" int eslam_gpu_set_map(eslam_ctx* ctx, const eslam_mls_grid* g)
{
    if (!ctx || !g || !g->cell_start || !g->patch_mean || !g->patch_stdev) return ESLAM_ERR_INVALID_ARG;
    if (const int rc_ = settle(ctx)) return rc_;    // a deferred sharded exchange first
    if (g->width == 0 || g->height == 0) return fail(ctx, ESLAM_ERR_NO_MLS_GRID, "The provided environment does not contain an mls grid.");
    const uint64_t ncell = (uint64_t)g->width * g->height;
    if ((uint64_t)g->cell_start[ncell] != g->n_patches) return fail(ctx, ESLAM_ERR_INVALID_ARG, "cell_start[width*height] != n_patches");
    // a pending resample gather, and on a sharded filter the received maps it names, land in
    // the old pool first; local_maps_reset below then starts every map over, empty
    if (const int rc_ = materialize(ctx)) return rc_;
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    free_map(ctx);
    const uint64_t np = g->n_patches ? g->n_patches : 1;
    std::vector<float2> patch(np);
    for (uint64_t k = 0; k < g->n_patches; ++k) patch[k] = make_float2(g->patch_mean[k], g->patch_stdev[k]);
    HIPCHK(ctx, hipMalloc(&ctx->d_cells, (ncell + 1) * 4));
    HIPCHK(ctx, hipMalloc(&ctx->d_patch, np * sizeof(float2)));
    HIPCHK(ctx, hipMemcpy(ctx->d_cells, g->cell_start, (ncell + 1) * 4, hipMemcpyHostToDevice));
    HIPCHK(ctx, hipMemcpy(ctx->d_patch, patch.data(), np * sizeof(float2), hipMemcpyHostToDevice));
    if (g->patch_height) {
        HIPCHK(ctx, hipMalloc(&ctx->d_height, np * 4));
        HIPCHK(ctx, hipMemcpy(ctx->d_height, g->patch_height, g->n_patches * 4, hipMemcpyHostToDevice));
    }
    {
        // one bit per cell: the shared grid holds patches there (the map merge's per-patch test
        // is one 4-byte load instead of the cell's two range words)
        std::vector<uint32_t> occ((ncell + 31) / 32, 0u);
        for (uint64_t c = 0; c < ncell; ++c)
            if (g->cell_start[c] != g->cell_start[c + 1]) occ[c >> 5] |= 1u << (c & 31);
        HIPCHK(ctx, hipMalloc(&ctx->d_occ, occ.size() * 4));
        HIPCHK(ctx, hipMemcpy(ctx->d_occ, occ.data(), occ.size() * 4, hipMemcpyHostToDevice));
    }
    {
        // MapView::cell_tab: the cell's range and first patch in one 16-byte record
        std::vector<uint4> tab(ncell);
        for (uint64_t c = 0; c < ncell; ++c) {
            const uint32_t b = g->cell_start[c], e = g->cell_start[c + 1];
            const float2 f = e > b ? patch[b] : make_float2(0.0f, 0.0f);
            uint32_t fm, fs;
            memcpy(&fm, &f.x, 4);
            memcpy(&fs, &f.y, 4);
            tab[c] = make_uint4(fm, fs, b, e - b);
        }
        HIPCHK(ctx, hipMalloc(&ctx->d_cell_tab, ncell * sizeof(uint4)));
        HIPCHK(ctx, hipMemcpy(ctx->d_cell_tab, tab.data(), ncell * sizeof(uint4), hipMemcpyHostToDevice));
    }
    MapView& m = ctx->map;
    m.cell_start = ctx->d_cells;
    m.occ = ctx->d_occ;
    m.cell_tab = ctx->d_cell_tab;
    m.patch = ctx->d_patch;
    m.height = ctx->d_height;
    m.has_height = ctx->d_height ? 1u : 0u;
    m.width = g->width;
    m.height_cells = g->height;
    m.inv_scale_x = 1.0 / g->scale_x;
    m.inv_scale_y = 1.0 / g->scale_y;
    ctx->map_scale[0] = g->scale_x;
    ctx->map_scale[1] = g->scale_y;
    ctx->has_hash = false;                   // a new map invalidates the pose hash
    m.offset_x = g->offset_x;
    m.offset_y = g->offset_y;
    memcpy(m.g2l, g->global2local, sizeof(m.g2l));
    static const double kId[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    m.g2l_identity = 1;
    for (int k = 0; k < 12; ++k)
        if (!(g->global2local[k] == kId[k])) m.g2l_identity = 0;
    ctx->has_map = true;
    // per-particle maps name cells of the previous grid: they start over, empty
    return local_maps_reset(ctx);
}

static int reset_ctl_for_new_particles(eslam_ctx* ctx, int wexp)
{
    int rc = read_ctl(ctx);
    if (rc) return rc;
    if (ctx->poisoned || (ctx->ctl_host->err & (kFaultTimeout | kFaultPages))) {
        // a poisoned filter starts over: the fault cleared, no partial segment marks left
        ctx->ctl_host->err &= ~(uint64_t)(kFaultTimeout | kFaultPages);
        ctx->poison_pages = false;
        __atomic_store_n(ctx->fault_host, 0u, __ATOMIC_RELAXED);
        HIPCHK(ctx, hipMemsetAsync(ctx->marks, 0, ctx->cap * 4, ctx->stream));
        ctx->poisoned = false;
    }
    ctx->ctl_host->base = 0;
    ctx->ctl_host->flip = 0;
    ctx->ctl_host->gather = 0;               // a pending gather of the old set is dropped
    ctx->ctl_host->wexp = wexp;
    ctx->has_anc = false;
    return write_ctl(ctx);
}

extern "C" int eslam_gpu_init_gaussian(eslam_ctx* ctx, uint64_t n, const double mu[3], const double sigma[3], double zpos,
                                       double zsigma)
{
    if (!ctx || !mu || !sigma) return ESLAM_ERR_INVALID_ARG;
    if (const int rc_ = settle(ctx)) return rc_;    // a deferred sharded exchange first
    int rc = alloc_particles(ctx, n);
    if (rc) return rc;
    rc = reset_ctl_for_new_particles(ctx, 1);
    if (rc) return rc;
    HIPCHK(ctx, eslam_launch_init_gaussian(ctx->st[0], n, ctx->gbase, ctx->cfg.seed, ctx->init_event, mu, sigma, zpos, zsigma,
                                           ctx->stream));
    ctx->init_event++;
    return ESLAM_OK;
}

extern "C" int eslam_gpu_init_pose(eslam_ctx* ctx, const double pos[3], const double q[4])
{
    if (!ctx || !pos || !q) return ESLAM_ERR_INVALID_ARG;
    if (const int rc_ = settle(ctx)) return rc_;    // a deferred sharded exchange first
    if (!ctx->has_map) return fail(ctx, ESLAM_ERR_NO_MLS_GRID, "The provided environment does not contain an mls grid.");
    double R[9];
    q_to_mat(q, R);
    double angle = atan2(R[3], R[0]);          // eulerAngles(2,1,0)[0], folded into [0, pi]
    if (angle < 0.0) angle += M_PI;
    const double mu[3] = {pos[0], pos[1], angle};
    const double sg[3] = {ctx->cfg.initial_translation_error[0], ctx->cfg.initial_translation_error[1],
                          ctx->cfg.initial_rotation_error[2]};
    uint64_t n = ctx->cfg.particle_count;
    if (ctx->sharded) {
        if (n != ctx->n_global) return fail(ctx, ESLAM_ERR_INVALID_ARG, "sharded context: particle_count must be n_global");
        n = ctx->gall[ctx->comm.rank + 1] - ctx->gall[ctx->comm.rank];
    }
    int rc;
    if (ctx->cfg.hash_use) {                   // hash.create(gridTemplate); filter.init(N, &hash)
        rc = ctx->has_hash ? ESLAM_OK : eslam_gpu_hash_create(ctx);
        if (!rc) rc = eslam_gpu_init_hash(ctx, n);
    } else {
        rc = eslam_gpu_init_gaussian(ctx, n, mu, sg, pos[2], ctx->cfg.initial_translation_error[2] + 1e-3);
    }
    set_translation_pose(ctx->ud_pose, 1000, 0, 0);
    return rc;
}

// ---------------------------------------------------------------------------------------
// SurfaceHash (src/SurfaceHash.hpp:155-231, src/PoseEstimator.cpp:75-86, 130-182)
// ---------------------------------------------------------------------------------------
static dm_hash_grid hash_grid(eslam_ctx* ctx)
{
    dm_hash_grid g;
    memset(&g, 0, sizeof(g));
    g.cell_start = ctx->d_cells;
    g.mean = reinterpret_cast<const float*>(ctx->d_patch);   // float2 {mean, stdev}
    g.mean_stride = 2;
    g.width = ctx->map.width;
    g.height = ctx->map.height_cells;
    g.bins = (uint32_t)ctx->cfg.hash_slope_bins;
    g.scale_x = ctx->map_scale[0];
    g.scale_y = ctx->map_scale[1];
    g.offset_x = ctx->map.offset_x;
    g.offset_y = ctx->map.offset_y;
    g.inv_scale_x = ctx->map.inv_scale_x;
    g.inv_scale_y = ctx->map.inv_scale_y;
    dm_affine_inverse(ctx->map.g2l, g.g2w);
    return g;
}

extern "C" int eslam_gpu_hash_create(eslam_ctx* ctx)
{
    if (!ctx) return ESLAM_ERR_INVALID_ARG;
    if (const int rc_ = settle(ctx)) return rc_;    // a deferred sharded exchange first
    if (!ctx->has_map) return fail(ctx, ESLAM_ERR_NO_MLS_GRID, "The provided environment does not contain an mls grid.");
    const uint32_t steps = (uint32_t)ctx->cfg.hash_angular_steps, bins = (uint32_t)ctx->cfg.hash_slope_bins;
    if (steps == 0 || bins == 0 || bins > 4096) return fail(ctx, ESLAM_ERR_INVALID_ARG, "hash_angular_steps / hash_slope_bins");
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    const dm_hash_grid g = hash_grid(ctx);
    std::vector<double> pts(8 * steps), orient(steps);
    dm_hash_segments(steps, g.g2w, pts.data(), orient.data());
    const uint64_t cells = (uint64_t)g.width * g.height, total = cells * steps;
    double* d_seg = nullptr;
    int32_t* d_out = nullptr;
    uint64_t* d_ids = nullptr;
    std::vector<int32_t> out(total);
    int rc = ESLAM_OK;
    do {
        if (hipMalloc(&d_seg, sizeof(double) * 9 * steps) != hipSuccess ||
            hipMalloc(&d_out, sizeof(int32_t) * (total ? total : 1)) != hipSuccess) {
            rc = fail(ctx, ESLAM_ERR_OUT_OF_MEMORY, "hash sweep buffers");
            break;
        }
        if (hipMemcpy(d_seg, pts.data(), sizeof(double) * 8 * steps, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(d_seg + 8 * steps, orient.data(), sizeof(double) * steps, hipMemcpyHostToDevice) != hipSuccess ||
            eslam_launch_hash_sweep(&g, d_seg, d_seg + 8 * steps, steps, d_out, ctx->stream) != hipSuccess ||
            hipMemcpyAsync(out.data(), d_out, sizeof(int32_t) * total, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
            hipStreamSynchronize(ctx->stream) != hipSuccess) {
            rc = fail(ctx, ESLAM_ERR_HIP, "hash sweep");
            break;
        }
        // compact in sweep order; bucket lists by a stable counting sort
        std::vector<uint64_t> ids;
        ctx->hash_bucket.clear();
        for (uint64_t id = 0; id < total; ++id)
            if (out[id] >= 0) { ids.push_back(id); ctx->hash_bucket.push_back(out[id]); }
        const uint64_t n = ids.size();
        const uint32_t nb = bins * bins;
        ctx->hash_bstart.assign(nb + 1, 0);
        for (uint64_t i = 0; i < n; ++i) ctx->hash_bstart[ctx->hash_bucket[i] + 1]++;
        for (uint32_t b = 0; b < nb; ++b) ctx->hash_bstart[b + 1] += ctx->hash_bstart[b];
        std::vector<uint32_t> blist(n ? n : 1), fill(ctx->hash_bstart.begin(), ctx->hash_bstart.end() - 1);
        for (uint64_t i = 0; i < n; ++i) blist[fill[ctx->hash_bucket[i]]++] = (uint32_t)i;
        (void)hipFree(ctx->d_hash); ctx->d_hash = nullptr;
        (void)hipFree(ctx->d_hash_blist); ctx->d_hash_blist = nullptr;
        const uint64_t cap = n ? n : 1;
        if (hipMalloc(&ctx->d_hash, sizeof(double) * 4 * cap) != hipSuccess ||
            hipMalloc(&ctx->d_hash_blist, sizeof(uint32_t) * cap) != hipSuccess ||
            hipMalloc(&d_ids, sizeof(uint64_t) * cap) != hipSuccess) {
            rc = fail(ctx, ESLAM_ERR_OUT_OF_MEMORY, "hash pose buffers");
            break;
        }
        double* hx = ctx->d_hash;
        if ((n && hipMemcpy(d_ids, ids.data(), sizeof(uint64_t) * n, hipMemcpyHostToDevice) != hipSuccess) ||
            (n && hipMemcpy(ctx->d_hash_blist, blist.data(), sizeof(uint32_t) * n, hipMemcpyHostToDevice) != hipSuccess) ||
            eslam_launch_hash_poses(&g, d_seg, d_seg + 8 * steps, d_ids, n, hx, hx + cap, hx + 2 * cap, hx + 3 * cap,
                                    ctx->stream) != hipSuccess ||
            hipStreamSynchronize(ctx->stream) != hipSuccess) {
            rc = fail(ctx, ESLAM_ERR_HIP, "hash poses");
            break;
        }
        ctx->hash_n = n;
        ctx->has_hash = true;
    } while (0);
    (void)hipFree(d_seg); (void)hipFree(d_out); (void)hipFree(d_ids);
    return rc;
}

static const double* hash_field(eslam_ctx* ctx, int f)
{
    return ctx->d_hash + (uint64_t)f * (ctx->hash_n ? ctx->hash_n : 1);
}

extern "C" int eslam_gpu_init_hash(eslam_ctx* ctx, uint64_t n)
{
    if (!ctx) return ESLAM_ERR_INVALID_ARG;
    if (const int rc_ = settle(ctx)) return rc_;    // a deferred sharded exchange first
    if (!ctx->has_hash || ctx->hash_n == 0) return fail(ctx, ESLAM_ERR_HASH_SAMPLE, "could not sample from pose hash.");
    int rc = alloc_particles(ctx, n);
    if (rc) return rc;
    rc = reset_ctl_for_new_particles(ctx, 1);
    if (rc) return rc;
    // rand() % poses.size() per particle, in global particle order (every rank walks all)
    const uint64_t total = ctx->sharded ? ctx->n_global : n, skip = ctx->gbase;
    std::vector<uint32_t> idx(n ? n : 1);
    for (uint64_t gi = 0; gi < total; ++gi) {
        const uint32_t v = (uint32_t)((uint64_t)(uint32_t)dm_libc_rand(ctx->libcp) % ctx->hash_n);
        if (gi >= skip && gi < skip + n) idx[gi - skip] = v;
    }
    uint32_t* d_idx = nullptr;
    HIPCHK(ctx, hipMalloc(&d_idx, sizeof(uint32_t) * (n ? n : 1)));
    hipError_t e = hipMemcpy(d_idx, idx.data(), sizeof(uint32_t) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = eslam_launch_init_from_hash(ctx->st[0], d_idx, n, hash_field(ctx, 0), hash_field(ctx, 1), hash_field(ctx, 2),
                                        hash_field(ctx, 3), ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    (void)hipFree(d_idx);
    HIPCHK(ctx, e);
    return ESLAM_OK;
}

extern "C" int eslam_gpu_hash_info(eslam_ctx* ctx, uint64_t* n_poses, uint32_t* bucket_sizes)
{
    if (!ctx || !n_poses) return ESLAM_ERR_INVALID_ARG;
    *n_poses = ctx->has_hash ? ctx->hash_n : 0;
    if (bucket_sizes && ctx->has_hash)
        for (size_t b = 0; b + 1 < ctx->hash_bstart.size(); ++b) bucket_sizes[b] = ctx->hash_bstart[b + 1] - ctx->hash_bstart[b];
    return ESLAM_OK;
}

extern "C" int eslam_gpu_hash_poses(eslam_ctx* ctx, double* x, double* y, double* theta, double* z, int32_t* bucket)
{
    if (!ctx) return ESLAM_ERR_INVALID_ARG;
    if (const int rc_ = settle(ctx)) return rc_;    // a deferred sharded exchange first
    if (!ctx->has_hash) return fail(ctx, ESLAM_ERR_NOT_INITIALISED, "no pose hash");
    const uint64_t n = ctx->hash_n;
    double* dst[4] = {x, y, theta, z};
    for (int f = 0; f < 4; ++f)
        if (dst[f] && n) HIPCHK(ctx, hipMemcpy(dst[f], hash_field(ctx, f), n * 8, hipMemcpyDeviceToHost));
    if (bucket && n) memcpy(bucket, ctx->hash_bucket.data(), n * 4);
    return ESLAM_OK;
}

extern "C" int eslam_gpu_particle_count(const eslam_ctx* ctx, uint64_t* n)
{
    if (!ctx || !n) return ESLAM_ERR_INVALID_ARG;
    *n = ctx->n;
    return ESLAM_OK;
}

extern "C" int eslam_gpu_upload_particles(eslam_ctx* ctx, uint64_t n, const eslam_particles* p)
{
    if (!ctx || !p || !p->x || !p->y || !p->orientation || !p->zpos || !p->zsigma || !p->weight) return ESLAM_ERR_INVALID_ARG;
    if (const int rc_ = settle(ctx)) return rc_;    // a deferred sharded exchange first
    int rc = alloc_particles(ctx, n);
    if (rc) return rc;
    const DevState& s = ctx->st[0];
    const uint64_t b = n * 8;
    if (n) {
        HIPCHK(ctx, hipMemcpy(s.x, p->x, b, hipMemcpyHostToDevice));
        HIPCHK(ctx, hipMemcpy(s.y, p->y, b, hipMemcpyHostToDevice));
        HIPCHK(ctx, hipMemcpy(s.th, p->orientation, b, hipMemcpyHostToDevice));
        HIPCHK(ctx, hipMemcpy(s.z, p->zpos, b, hipMemcpyHostToDevice));
        HIPCHK(ctx, hipMemcpy(s.zs, p->zsigma, b, hipMemcpyHostToDevice));
        HIPCHK(ctx, hipMemcpy(s.w, p->weight, b, hipMemcpyHostToDevice));
        if (p->mprob) HIPCHK(ctx, hipMemcpy(s.mprob, p->mprob, b, hipMemcpyHostToDevice));
        else HIPCHK(ctx, hipMemset(s.mprob, 0, b));
        std::vector<uint8_t> fl(n);
        for (uint64_t i = 0; i < n; ++i) {
            const uint8_t f = p->floating ? (p->floating[i] ? 1 : 0) : 1;
            const uint8_t c = p->n_contact_points ? (p->n_contact_points[i] & 0x7f) : 0;
            fl[i] = (uint8_t)(c | (f << 7));
        }
        HIPCHK(ctx, hipMemcpy(s.flags, fl.data(), n, hipMemcpyHostToDevice));
    }
    double mx = 0;
    for (uint64_t i = 0; i < n; ++i) if (p->weight[i] > mx) mx = p->weight[i];
    if (ctx->sharded) {                      // the statistics scale must agree on every rank
        uint64_t* h = ctx->mg_host;
        memcpy(&h[mg::kMaxW], &mx, 8);
        HIPCHK(ctx, hipMemcpy(ctx->mg + mg::kMaxW, &h[mg::kMaxW], 8, hipMemcpyHostToDevice));
        rc = comm_allgather(ctx, ctx->mg + mg::kMaxW, ctx->mg + mg::kMaxWAll, 8);
        if (rc) return rc;
        HIPCHK(ctx, hipMemcpy(&h[mg::kMaxWAll], ctx->mg + mg::kMaxWAll, 8 * ctx->comm.nranks, hipMemcpyDeviceToHost));
        for (int r = 0; r < ctx->comm.nranks; ++r) {
            double v;
            memcpy(&v, &h[mg::kMaxWAll + r], 8);
            if (v > mx) mx = v;
        }
    }
    return reset_ctl_for_new_particles(ctx, dm_weight_exp(mx));
}

extern "C" int eslam_gpu_download_particles(eslam_ctx* ctx, eslam_particles* p)
{
    if (!ctx || !p) return ESLAM_ERR_INVALID_ARG;
    if (const int rc_ = settle(ctx)) return rc_;    // a deferred sharded exchange first
    if (check_poisoned(ctx)) return ESLAM_ERR_HIP;
    int rc = materialize(ctx);
    if (!rc) rc = read_ctl(ctx);
    if (rc) return rc;
    const DevState& s = ctx->st[ctx->ctl_host->base ^ ctx->ctl_host->flip];
    const uint64_t n = ctx->n, b = n * 8;
    if (!n) return ESLAM_OK;
    if (p->x) HIPCHK(ctx, hipMemcpy(p->x, s.x, b, hipMemcpyDeviceToHost));
    if (p->y) HIPCHK(ctx, hipMemcpy(p->y, s.y, b, hipMemcpyDeviceToHost));
    if (p->orientation) HIPCHK(ctx, hipMemcpy(p->orientation, s.th, b, hipMemcpyDeviceToHost));
    if (p->zpos) HIPCHK(ctx, hipMemcpy(p->zpos, s.z, b, hipMemcpyDeviceToHost));
    if (p->zsigma) HIPCHK(ctx, hipMemcpy(p->zsigma, s.zs, b, hipMemcpyDeviceToHost));
    if (p->weight) HIPCHK(ctx, hipMemcpy(p->weight, s.w, b, hipMemcpyDeviceToHost));
    if (p->mprob) HIPCHK(ctx, hipMemcpy(p->mprob, s.mprob, b, hipMemcpyDeviceToHost));
    if (p->floating || p->n_contact_points) {
        std::vector<uint8_t> fl(n);
        HIPCHK(ctx, hipMemcpy(fl.data(), s.flags, n, hipMemcpyDeviceToHost));
        for (uint64_t i = 0; i < n; ++i) {
            if (p->floating) p->floating[i] = fl[i] >> 7;
            if (p->n_contact_points) p->n_contact_points[i] = fl[i] & 0x7f;
        }
    }
    return ESLAM_OK;
}

// the largest weight of this context's particles (NaN and negative weights skipped), as
// eslam_gpu_upload_particles computes the weight scale
static int max_weight_local(eslam_ctx* ctx, double* out)
{
    const DevState& s = ctx->st[ctx->ctl_host->base ^ ctx->ctl_host->flip];
    std::vector<double> w(ctx->n);
    HIPCHK(ctx, hipMemcpy(w.data(), s.w, ctx->n * 8, hipMemcpyDeviceToHost));
    double mx = 0;
    for (uint64_t i = 0; i < ctx->n; ++i) if (w[i] > mx) mx = w[i];
    *out = mx;
    return ESLAM_OK;
}

// eslam_gpu_write_particles' rank-local part: the fields of p into [first, first + count)
static int write_particles_local(eslam_ctx* ctx, uint64_t first, uint64_t count, const eslam_particles* p)
{
    if (!count) return ESLAM_OK;
    const DevState& s = ctx->st[ctx->ctl_host->base ^ ctx->ctl_host->flip];
    const uint64_t b = count * 8;
    const double* src[7] = {p->x, p->y, p->orientation, p->zpos, p->zsigma, p->weight, p->mprob};
    double* dst[7] = {s.x, s.y, s.th, s.z, s.zs, s.w, s.mprob};
    for (int k = 0; k < 7; ++k)
        if (src[k]) HIPCHK(ctx, hipMemcpyAsync(dst[k] + first, src[k], b, hipMemcpyHostToDevice, ctx->stream));
    if (p->floating || p->n_contact_points) {
        std::vector<uint8_t> fl(count);
        HIPCHK(ctx, hipMemcpyAsync(fl.data(), s.flags + first, count, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
        for (uint64_t i = 0; i < count; ++i) {
            uint8_t f = fl[i];
            if (p->floating) f = (uint8_t)((f & 0x7f) | ((p->floating[i] ? 1 : 0) << 7));
            if (p->n_contact_points) f = (uint8_t)((f & 0x80) | (p->n_contact_points[i] & 0x7f));
            fl[i] = f;
        }
        HIPCHK(ctx, hipMemcpyAsync(s.flags + first, fl.data(), count, hipMemcpyHostToDevice, ctx->stream));
    }
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    // the weight scale of the next update, from the largest weight of the whole set exactly
    // as eslam_gpu_upload_particles computes it (one GPU: only when weights were written)
    if (p->weight && !ctx->sharded) {
        double mx = 0;
        const int rc = max_weight_local(ctx, &mx);
        if (rc) return rc;
        ctx->ctl_host->wexp = dm_weight_exp(mx);
        return write_ctl(ctx);
    }
    return ESLAM_OK;
}

extern "C" int eslam_gpu_write_particles(eslam_ctx* ctx, uint64_t first, uint64_t count, const eslam_particles* p)
{
    if (!ctx) return ESLAM_ERR_INVALID_ARG;
    // sharded: a collective (every rank calls it, count may be 0).  A rank whose own part fails
    // still takes part in the weight-scale all_gather, with a NaN that tells the others to fail
    // too, so no rank is left waiting in it (include/eslam_gpu.h)
    int rc = (!p || first > ctx->n || count > ctx->n - first) ? fail(ctx, ESLAM_ERR_INVALID_ARG, "write_particles: bad range")
                                                              : ESLAM_OK;
    if (!rc) rc = settle(ctx);                          // a deferred sharded exchange first
    if (!rc) rc = check_poisoned(ctx);
    if (!rc) rc = materialize(ctx);                     // the particles the caller saw: any pending gather done
    if (!rc) rc = read_ctl(ctx);
    if (!rc) rc = write_particles_local(ctx, first, count, p);
    if (!ctx->sharded) return rc;
    double mx = 0;
    if (!rc) rc = max_weight_local(ctx, &mx);
    if (rc) mx = NAN;
    uint64_t* h = ctx->mg_host;
    memcpy(&h[mg::kMaxW], &mx, 8);
    HIPCHK(ctx, hipMemcpy(ctx->mg + mg::kMaxW, &h[mg::kMaxW], 8, hipMemcpyHostToDevice));
    const int crc = comm_allgather(ctx, ctx->mg + mg::kMaxW, ctx->mg + mg::kMaxWAll, 8);
    if (crc) return rc ? rc : crc;
    HIPCHK(ctx, hipMemcpy(&h[mg::kMaxWAll], ctx->mg + mg::kMaxWAll, 8 * ctx->comm.nranks, hipMemcpyDeviceToHost));
    bool peer_failed = false;
    for (int r = 0; r < ctx->comm.nranks; ++r) {
        double v;
        memcpy(&v, &h[mg::kMaxWAll + r], 8);
        if (v != v) peer_failed = true;
        else if (v > mx) mx = v;
    }
    if (rc) return rc;
    if (peer_failed) return fail(ctx, ESLAM_ERR_COMM, "write_particles failed on another rank");
    ctx->ctl_host->wexp = dm_weight_exp(mx);
    return write_ctl(ctx);
}

constexpr uint64_t kRecRemote = 1ull << 63;     // k_pack_records: a slot naming a fetched item

// logDebug records on a sharded filter: particle i's records are those of its ancestor at the
// last update's resample, which may have sat on another rank.  Those are fetched from their
// ranks: the request counts all_gathered, then two all_to_all_v (the global indices asked for,
// the items: meas 4, ncp, maxc x 6 contact-point doubles).  slot[k]: the record's position on
// this rank, or kRecRemote | its item in *d_remote.  Every rank takes part; one whose own part
// failed (rc) sends counts that make every rank fail, so no rank is left waiting.
static int fetch_remote_records(eslam_ctx* ctx, int rc, uint64_t first, uint64_t stride, uint64_t count,
                                std::vector<uint64_t>& slot, double** d_remote)
{
    const int G = ctx->comm.nranks, me = ctx->comm.rank;
    const uint64_t gb = ctx->gbase, item = 8ull * (5 + 6ull * (ctx->dbg.maxc ? ctx->dbg.maxc : 1));
    std::vector<std::vector<uint32_t>> req(G);
    std::vector<uint32_t> owner_of;             // per remote slot: its owner
    auto resolve = [&]() -> int {
        if (!ctx->dbg_valid || !count) return ESLAM_OK;
        uint32_t resampled = 0;
        HIPCHK(ctx, hipMemcpy(&resampled, ctx->dbg.resampled, 4, hipMemcpyDeviceToHost));
        std::vector<uint32_t> anc;
        if (resampled) {
            anc.resize(ctx->n);
            HIPCHK(ctx, hipMemcpy(anc.data(), ctx->anc, ctx->n * 4, hipMemcpyDeviceToHost));
        }
        slot.resize(count);
        for (uint64_t k = 0; k < count; ++k) {
            const uint64_t i = first + k * stride, g = resampled ? anc[i] : gb + i;
            if (g >= gb && g < gb + ctx->n) {
                slot[k] = g - gb;
                continue;
            }
            const int o = (int)(std::upper_bound(ctx->gall.begin(), ctx->gall.end(), g) - ctx->gall.begin()) - 1;
            if (o < 0 || o >= G || o == me) return fail(ctx, ESLAM_ERR_HIP, "download_records: ancestor outside the filter");
            slot[k] = kRecRemote | req[o].size();
            owner_of.push_back((uint32_t)o);
            req[o].push_back((uint32_t)g);
        }
        return ESLAM_OK;
    };
    if (!rc) rc = resolve();
    // the request counts: row r of the gathered matrix is what rank r asks of each rank
    uint64_t* h = ctx->mg_host;
    for (int d = 0; d < G; ++d) h[mg::kCounts + d] = rc ? ~0ull : (uint64_t)req[d].size();
    HIPCHK(ctx, hipMemcpy(ctx->mg + mg::kCounts, &h[mg::kCounts], 8ull * G, hipMemcpyHostToDevice));
    const int crc = comm_allgather(ctx, ctx->mg + mg::kCounts, ctx->mg + mg::kCountsAll, 8ull * G);
    if (crc) return rc ? rc : crc;
    HIPCHK(ctx, hipMemcpy(&h[mg::kCountsAll], ctx->mg + mg::kCountsAll, 8ull * G * G, hipMemcpyDeviceToHost));
    bool peer_failed = false;
    uint64_t nin[kMaxRanks], tin = 0, tout = 0, off[kMaxRanks + 1];
    for (int r = 0; r < G; ++r) {
        for (int d = 0; d < G; ++d) peer_failed |= h[mg::kCountsAll + r * G + d] == ~0ull;
        nin[r] = h[mg::kCountsAll + r * G + me];
    }
    if (rc) return rc;
    if (peer_failed) return fail(ctx, ESLAM_ERR_COMM, "download_records failed on another rank");
    off[0] = 0;
    for (int r = 0; r < G; ++r) {
        tin += nin[r];
        off[r + 1] = off[r] + req[r].size();
    }
    tout = off[G];
    // the requests out, this rank's items for the others back
    std::vector<uint32_t> hreq;
    hreq.reserve(tout);
    for (int d = 0; d < G; ++d) hreq.insert(hreq.end(), req[d].begin(), req[d].end());
    uint32_t *d_out = nullptr, *d_in = nullptr;
    double* d_items = nullptr;
    int out = ESLAM_OK;
    auto exchange = [&]() -> int {
        HIPCHK(ctx, hipMalloc(&d_out, (tout + 1) * 4));
        HIPCHK(ctx, hipMalloc(&d_in, (tin + 1) * 4));
        HIPCHK(ctx, hipMalloc(&d_items, (tin + 1) * item));
        HIPCHK(ctx, hipMalloc(d_remote, (tout + 1) * item));
        if (tout) HIPCHK(ctx, hipMemcpy(d_out, hreq.data(), tout * 4, hipMemcpyHostToDevice));
        uint64_t sb[kMaxRanks], rb[kMaxRanks];
        for (int r = 0; r < G; ++r) { sb[r] = 4 * req[r].size(); rb[r] = 4 * nin[r]; }
        int e = comm_alltoallv(ctx, d_out, sb, d_in, rb);
        if (e) return e;
        HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
        if (tin && ctx->dbg_valid) HIPCHK(ctx, eslam_launch_gather_records(d_in, tin, gb, &ctx->dbg, d_items, ctx->stream));
        else if (tin) HIPCHK(ctx, hipMemsetAsync(d_items, 0, tin * item, ctx->stream));
        HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
        for (int r = 0; r < G; ++r) { sb[r] = item * nin[r]; rb[r] = item * req[r].size(); }
        e = comm_alltoallv(ctx, d_items, sb, *d_remote, rb);
        if (e) return e;
        HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
        return ESLAM_OK;
    };
    out = exchange();
    (void)hipFree(d_out); (void)hipFree(d_in); (void)hipFree(d_items);
    if (out) return out;
    // the fetched items in rank order: rank o's start off[o]
    uint64_t r = 0;
    for (uint64_t k = 0; k < slot.size(); ++k)
        if (slot[k] & kRecRemote) slot[k] = kRecRemote | (off[owner_of[r++]] + (slot[k] & ~kRecRemote));
    return ESLAM_OK;
}

extern "C" int eslam_gpu_download_records(eslam_ctx* ctx, uint64_t first, uint64_t stride, uint64_t count,
                                          eslam_particle_record* out, eslam_cpoint* cpoints, uint32_t max_cpoints)
{
    if (!ctx) return ESLAM_ERR_INVALID_ARG;
    // sharded with logDebug records: a collective (every rank calls it; count may be 0)
    const bool coll = ctx->sharded && record_contacts(ctx);
    if (!stride) stride = 1;
    int rc = (!out && count) ? fail(ctx, ESLAM_ERR_INVALID_ARG, "download_records: no output") : ESLAM_OK;
    if (!rc && count && (first >= ctx->n || (count - 1) > (ctx->n - 1 - first) / stride))
        rc = fail(ctx, ESLAM_ERR_INVALID_ARG, "download_records: range beyond the particles");
    if (!rc || coll) {
        const int s = settle(ctx);                // a deferred sharded exchange first
        if (!rc) rc = s;
    }
    if (!rc && check_poisoned(ctx)) rc = ESLAM_ERR_HIP;
    if (!rc) rc = materialize(ctx);               // the pending gather writes the ancestors too
    std::vector<uint64_t> slot;
    double* d_remote = nullptr;
    if (coll) {
        const int frc = fetch_remote_records(ctx, rc, first, stride, count, slot, &d_remote);
        if (!rc) rc = frc;
    }
    if (rc || !count) {
        (void)hipFree(d_remote);
        return rc;
    }
    if (!cpoints) max_cpoints = 0;
    const DebugRec none = {};
    const DebugRec& d = ctx->dbg_valid ? ctx->dbg : none;
    eslam_particle_record* d_out = nullptr;
    eslam_cpoint* d_cp = nullptr;
    uint64_t* d_slot = nullptr;
    hipError_t e = hipMalloc(&d_out, count * sizeof(eslam_particle_record));
    if (e == hipSuccess && max_cpoints) {
        e = hipMalloc(&d_cp, count * max_cpoints * sizeof(eslam_cpoint));
        if (e == hipSuccess) e = hipMemsetAsync(d_cp, 0, count * max_cpoints * sizeof(eslam_cpoint), ctx->stream);
    }
    if (e == hipSuccess && !slot.empty()) {
        e = hipMalloc(&d_slot, count * 8);
        if (e == hipSuccess) e = hipMemcpy(d_slot, slot.data(), count * 8, hipMemcpyHostToDevice);
    }
    if (e == hipSuccess)
        e = eslam_launch_pack_records(ctx->st[0], ctx->st[1], ctx->ctl, first, stride, count, ctx->gbase, ctx->anc, &d, d_out,
                                      d_cp, max_cpoints, d_slot, d_remote, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e == hipSuccess) e = hipMemcpy(out, d_out, count * sizeof(eslam_particle_record), hipMemcpyDeviceToHost);
    if (e == hipSuccess && max_cpoints) e = hipMemcpy(cpoints, d_cp, count * max_cpoints * sizeof(eslam_cpoint), hipMemcpyDeviceToHost);
    (void)hipFree(d_out);
    (void)hipFree(d_cp);
    (void)hipFree(d_slot);
    (void)hipFree(d_remote);
    if (e != hipSuccess) return fail(ctx, ESLAM_ERR_HIP, (std::string("download_records: ") + hipGetErrorString(e)).c_str());
    return ESLAM_OK;
}

// ---------------------------------------------------------------------------------------
// per-particle local maps
// ---------------------------------------------------------------------------------------
// the map-update parameters every copy-on-write pass shares (the merge, a sharded receive)
static MergeParams merge_params(eslam_ctx* ctx, const CowScratch& cs)
{
    MergeParams mp;
    memset(&mp, 0, sizeof(mp));
    mp.cnt = ctx->merge_cnt;
    mp.ref = cs.ref;
    mp.frees = cs.frees;
    mp.off = ctx->lm_off;
    mp.job = (MergeJob*)ctx->lm_job;
    mp.codes = ctx->lm_codes;
    mp.poff = ctx->lm_poff;
    mp.fault = ctx->fault_host;
    mp.n = ctx->n;
    return mp;
}

extern "C" int eslam_gpu_map_update(eslam_ctx* ctx, const eslam_scan_patch* patches, uint32_t count)
{
    if (!ctx || (!patches && count)) return ESLAM_ERR_INVALID_ARG;
    if (const int rc_ = settle(ctx)) return rc_;    // a deferred sharded exchange first
    if (!particle_maps(ctx)) return fail(ctx, ESLAM_ERR_INVALID_ARG, "map_update needs per-particle maps (ESLAM_FLAG_PARTICLE_MAPS)");
    if (!ctx->has_map) return fail(ctx, ESLAM_ERR_NO_ENVIRONMENT, "No environment attached.");
    if (!ctx->n) return fail(ctx, ESLAM_ERR_NOT_INITIALISED, "no particles");
    if (const int rc_ = check_poisoned(ctx)) return rc_;
    if (!ctx->lm_ready) return fail(ctx, ESLAM_ERR_NOT_INITIALISED, "per-particle maps not allocated");
    for (uint32_t k = 0; k < count; ++k)
        if (!dm_isfinite(patches[k].position[0]) || !dm_isfinite(patches[k].position[1]) ||
            !dm_isfinite(patches[k].position[2]) || !dm_isfinite(patches[k].stdev))
            return fail(ctx, ESLAM_ERR_INVALID_ARG, "map_update: scan patches must be finite");
    mrec(ctx, 0);
    // one GPU: a pending resample gather runs inside the merge (MergeParams::fuse: the store
    // classes and the merge read the particles through the marks), so the update reads and
    // writes the particle state once.  Sharded: the gather may hand this rank particles whose
    // stores are still in received payloads, which get local stores first (materialize).
    const bool fuse = !ctx->sharded;
    const GatherView gv = gather_view(ctx);
    if (!fuse) {
        const int rc = materialize(ctx);
        if (rc) return rc;
    }
    mrec(ctx, 1);
    // the scan on the device: this update's slot is free once the update before last is done
    const uint32_t slot = ctx->scan_slot ^= 1u;
    if (!ctx->scan_ev[slot]) HIPCHK(ctx, hipEventCreateWithFlags(&ctx->scan_ev[slot], hipEventDisableTiming));
    else HIPCHK(ctx, hipEventSynchronize(ctx->scan_ev[slot]));
    const uint64_t sbytes = (uint64_t)(count ? count : 1) * sizeof(ScanPatch);
    int rc = grow(ctx, &ctx->scan_host[slot], &ctx->scan_host_cap[slot], sbytes, true);
    if (!rc) rc = grow(ctx, &ctx->scan_dev[slot], &ctx->scan_dev_cap[slot], sbytes, false);
    // a scan of more than kScanPartSmall patches merges in parts of kScanPartLarge
    const uint32_t part = count <= kScanPartSmall ? kScanPartSmall : kScanPartLarge;
    if (!rc && part == kScanPartLarge) rc = grow(ctx, (void**)&ctx->lm_codes, &ctx->lm_codes_cap, ctx->cap * 2 * kScanPartLarge, false);
    if (rc) return rc;
    ScanPatch* sh = (ScanPatch*)ctx->scan_host[slot];
    for (uint32_t k = 0; k < count; ++k)
        sh[k] = ScanPatch{patches[k].position[0], patches[k].position[1], patches[k].position[2], patches[k].stdev};
    if (count) HIPCHK(ctx, hipMemcpyAsync(ctx->scan_dev[slot], sh, sbytes, hipMemcpyHostToDevice, ctx->stream));
    // the parts in order: every cell sees its patches in the scan's order; the parts' counters
    // add up (map_stores_changed counts a map once per part that changed it)
    for (uint32_t c0 = 0; c0 == 0 || c0 < count; c0 += part) {
        const uint32_t cm = count - c0 < part ? count - c0 : part;
        const SidRef sr{ctx->st[0].sid, ctx->st[1].sid, ctx->ctl};
        const CowScratch cs = cow_layout(ctx->cow, ctx->cap);
        HIPCHK(ctx, eslam_launch_store_refs(sr, ctx->n, store_pool(ctx->cap), &cs, fuse ? &gv : nullptr, ctx->lm.tgen,
                                            ctx->stream));
        if (!c0) mrec(ctx, 2);
        MergeParams mp = merge_params(ctx, cs);
        mp.is_id = ctx->map.g2l_identity;
        mp.gv = gv;                           // (the first part runs a pending gather; the device knows)
        mp.gbase = ctx->gbase;
        mp.fuse = fuse ? 1u : 0u;
        mp.aux = (ctx->cfg.flags & ESLAM_FLAG_NO_AUX_GATHER) ? 0u : 1u;
        mp.acc = c0 ? 1u : 0u;
        mp.m = cm;
        mp.sp = (const ScanPatch*)ctx->scan_dev[slot] + c0;
        mp.codes = ctx->lm_codes;
        HIPCHK(ctx, eslam_launch_map_plan(ctx->st[0], ctx->st[1], ctx->ctl, &ctx->map, &ctx->lm, &mp, ctx->lm_pgc, ctx->stream));
        if (!c0) mrec(ctx, 3);
        HIPCHK(ctx, eslam_launch_map_merge(ctx->st[0], ctx->st[1], ctx->ctl, &ctx->map, &ctx->lm, &mp, ctx->stream));
        if (fuse) {
            HIPCHK(ctx, eslam_launch_commit(ctx->ctl, ctx->stream));     // the gather's buffer flip, if one ran
        }
    }
    HIPCHK(ctx, hipEventRecord(ctx->scan_ev[slot], ctx->stream));
    mrec(ctx, 4);
    return ESLAM_OK;
}

// processMap(scanMap, match = true, ...)  src/EmbodiedSlamFilter.cpp:214-221 (k_map_match)
extern "C" int eslam_gpu_map_match(eslam_ctx* ctx, const eslam_scan_patch* patches, uint32_t count)
{
    if (!ctx || (!patches && count)) return ESLAM_ERR_INVALID_ARG;
    if (const int rc_ = settle(ctx)) return rc_;    // a deferred sharded exchange first
    if (!ctx->has_map) return fail(ctx, ESLAM_ERR_NO_ENVIRONMENT, "No environment attached.");
    if (!ctx->n) return fail(ctx, ESLAM_ERR_NOT_INITIALISED, "no particles");
    if (const int rc_ = check_poisoned(ctx)) return rc_;
    if (particle_maps(ctx) && !ctx->lm_ready) return fail(ctx, ESLAM_ERR_NOT_INITIALISED, "per-particle maps not allocated");
    for (uint32_t k = 0; k < count; ++k)
        if (!dm_isfinite(patches[k].position[0]) || !dm_isfinite(patches[k].position[1]) ||
            !dm_isfinite(patches[k].position[2]) || !dm_isfinite(patches[k].stdev))
            return fail(ctx, ESLAM_ERR_INVALID_ARG, "map_match: scan patches must be finite");
    xrec(ctx, 0);
    int rc = materialize(ctx);                // the weights of the particles as they stand
    if (rc) return rc;
    std::vector<ScanPatch> s;
    for (uint32_t k = 0; k < count; k += kMatchSampling)
        s.push_back(ScanPatch{patches[k].position[0], patches[k].position[1], patches[k].position[2], patches[k].stdev});
    MatchParams mp;
    mp.n = ctx->n;
    mp.m = (uint32_t)s.size();
    mp.is_id = ctx->map.g2l_identity;
    mp.sp = nullptr;
    const bool inline_sp = s.size() <= (size_t)kMaxScanPatches;   // the kernel arguments carry them
    if (inline_sp) {
        for (size_t k = 0; k < s.size(); ++k) mp.spi[k] = s[k];
    } else {
        rc = grow(ctx, &ctx->match_sp, &ctx->match_cap, s.size() * sizeof(ScanPatch), false);
        if (rc) return rc;
        HIPCHK(ctx, hipMemcpyAsync(ctx->match_sp, s.data(), s.size() * sizeof(ScanPatch), hipMemcpyHostToDevice, ctx->stream));
        mp.sp = (const ScanPatch*)ctx->match_sp;
    }
    HIPCHK(ctx, eslam_launch_map_match(ctx->st[0], ctx->st[1], ctx->ctl, &ctx->map, store_of(ctx), &mp, ctx->stream));
    xrec(ctx, 1);
    // a scan of more than 640 patches: the host's copy of the sampled ones goes away on return
    if (!inline_sp) HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    return ESLAM_OK;
}

extern "C" int eslam_gpu_set_particle_maps(eslam_ctx* ctx, int on)
{
    if (!ctx) return ESLAM_ERR_INVALID_ARG;
    if (const int rc_ = settle(ctx)) return rc_;    // a deferred sharded exchange first
    const bool cur = particle_maps(ctx);
    if ((on != 0) == cur) return ESLAM_OK;
    if (ctx->n) return fail(ctx, ESLAM_ERR_INVALID_ARG, "the map mode is chosen before the particles are initialised");
    if (on) ctx->cfg.flags |= ESLAM_FLAG_PARTICLE_MAPS;
    else ctx->cfg.flags &= ~ESLAM_FLAG_PARTICLE_MAPS;
    return ESLAM_OK;
}

extern "C" int eslam_gpu_get_particle_map(eslam_ctx* ctx, uint64_t index, uint32_t* cells, float* mean, float* stdev,
                                          uint32_t capacity, uint32_t* count)
{
    if (!ctx || !count) return ESLAM_ERR_INVALID_ARG;
    if (const int rc_ = settle(ctx)) return rc_;    // a deferred sharded exchange first
    if (!particle_maps(ctx)) return fail(ctx, ESLAM_ERR_INVALID_ARG, "no per-particle maps (ESLAM_FLAG_PARTICLE_MAPS)");
    if (index >= ctx->n) return fail(ctx, ESLAM_ERR_INVALID_ARG, "particle index out of range");
    int rc = materialize(ctx);
    if (!rc) rc = read_ctl(ctx);
    if (rc) return rc;
    *count = 0;
    if (!ctx->lm_ready) return ESLAM_OK;
    const LocalMaps& lm = ctx->lm;
    const uint32_t* sid = ctx->st[ctx->ctl_host->base ^ ctx->ctl_host->flip].sid;
    uint32_t X = 0;
    HIPCHK(ctx, hipMemcpy(&X, sid + index, 4, hipMemcpyDeviceToHost));
    int2 c;
    std::vector<uint32_t> sl(lm.S);
    HIPCHK(ctx, hipMemcpy(&c, lm.ctr + X, sizeof(int2), hipMemcpyDeviceToHost));
    HIPCHK(ctx, hipMemcpy(sl.data(), lm.slot + (uint64_t)X * lm.S, lm.S * 4, hipMemcpyDeviceToHost));
    // the window's tiles in slot order, then the trail's in entry order, each tile's cells row
    // by row (the oracle's or_get_particle_map)
    uint32_t k = 0;
    float2 cell[DM_LM_PAGE_CELLS];
    const uint32_t W = lm.wx * lm.wy, toff = lm.S - 4u * lm.V;
    const uint32_t hw = sl[toff - 1u] == DM_LM_NONE ? 0u : sl[toff - 1u];   // the trail's used entries
    for (uint32_t s = 0; s < W + hw; ++s) {
            const bool tr = s >= W;
            const uint32_t pg = tr ? sl[toff + 4u * (s - W) + 2u] : sl[s];
            if (pg == DM_LM_NONE) continue;
            const int64_t a = tr ? (int64_t)(int32_t)sl[toff + 4u * (s - W)] : dm_lm_tile_of(s % lm.wx, c.x, lm.hx, lm.wx);
            const int64_t b = tr ? (int64_t)(int32_t)sl[toff + 4u * (s - W) + 1u] : dm_lm_tile_of(s / lm.wx, c.y, lm.hy, lm.wy);
            HIPCHK(ctx, hipMemcpy(cell, lm.page + (uint64_t)pg * DM_LM_PAGE_CELLS, sizeof(cell), hipMemcpyDeviceToHost));
            for (uint32_t j = 0; j < DM_LM_PAGE_CELLS; ++j) {
                if (!dm_lm_holds(cell[j].y)) continue;
                if (k < capacity) {
                    const uint64_t m = (uint64_t)(8 * a) + (j & 7u), n = (uint64_t)(8 * b) + (j >> 3);
                    if (cells) cells[k] = (uint32_t)(n * ctx->map.width + m);
                    if (mean) mean[k] = cell[j].x;
                    if (stdev) stdev[k] = cell[j].y;
                }
                ++k;
            }
    }
    *count = k;
    return ESLAM_OK;
}

// ---------------------------------------------------------------------------------------
// the hot path
// ---------------------------------------------------------------------------------------
// the pending resample gather (consumed by the next k_project_weight or materialised)
static GatherView gather_view(eslam_ctx* ctx)
{
    GatherView gv;
    memset(&gv, 0, sizeof(gv));
    gv.marks = ctx->marks;
    gv.row_first = ctx->tile_first;
    gv.anc = ctx->anc;
    gv.recs = ctx->sharded ? (const Rec*)ctx->recvbuf : nullptr;
    gv.record = keep_ancestors(ctx) ? 1u : 0u;
    gv.multi = ctx->sharded ? 1u : 0u;
    return gv;
}

// before the particle state is read or replaced outside the hot path: run a pending
// gather (device decides; a no-op otherwise) and commit the buffer flip
// cloneMaps (src/PoseEstimator.cpp:31-47) as copy on write: a resample's copies of a particle
// share its store until a map update changes one of them (k_map_merge).  Particles received
// from another rank (sid = kSidRecord | record) get free stores filled from their records'
// payloads before anything reads a store.
static int store_receive(eslam_ctx* ctx)
{
    const SidRef sr{ctx->st[0].sid, ctx->st[1].sid, ctx->ctl};
    const CowScratch cs = cow_layout(ctx->cow, ctx->cap);
    HIPCHK(ctx, eslam_launch_store_refs(sr, ctx->n, store_pool(ctx->cap), &cs, nullptr, ctx->lm.tgen, ctx->stream));
    int rc = grow(ctx, (void**)&ctx->payoff, &ctx->payoff_cap, (ctx->nrecv_maps + 1) * 4, false);
    if (!rc) rc = grow(ctx, (void**)&ctx->rhead, &ctx->rhead_cap, (ctx->nrecv_maps + 1) * 4, false);
    if (rc) return rc;
    const MergeParams mp = merge_params(ctx, cs);
    HIPCHK(ctx, eslam_launch_store_receive(sr, ctx->ctl, &ctx->lm, &mp, ctx->n, &cs, ctx->recvhdr, ctx->nrecv_maps, ctx->payoff,
                                           ctx->rhead, ctx->recvpay, ctx->lm_pgc, ctx->stream));
    ctx->cow_pending = false;
    return ESLAM_OK;
}

static int materialize(eslam_ctx* ctx)
{
    if (!ctx->n) return ESLAM_OK;
    const GatherView gv = gather_view(ctx);
    const uint32_t aux = (ctx->cfg.flags & ESLAM_FLAG_NO_AUX_GATHER) ? 0u : 1u;
    HIPCHK(ctx, eslam_launch_resample_gather(ctx->st[0], ctx->st[1], ctx->n, ctx->gbase, ctx->ctl, &gv, aux, ctx->stream));
    // a sharded resample handed this rank particles whose stores are still in the received
    // payloads: they get local stores before anything reads a store
    if (ctx->cow_pending) return store_receive(ctx);
    return ESLAM_OK;
}

static void fill_step_params(eslam_ctx* ctx, const eslam_step_input* in, StepParams& p)
{
    memset(&p, 0, sizeof(p));
    const eslam_config& c = ctx->cfg;
    const double* q = in->body2odometry_rot;
    // PoseEstimator::project preamble  src/PoseEstimator.cpp:186-194
    p.yaw = get_yaw(q);
    double R[9];
    q_to_mat(q, R);
    const double* t = in->pose_delta_trans;
    p.z_delta = (R[6] * t[0] + R[7] * t[1]) + R[8] * t[2];
    p.z_var = in->position_error_zz * 2.0;
    for (int i = 0; i < 3; ++i) p.mu[i] = in->sample_mean[i];
    double L[9];
    lower_cholesky(in->sample_cov, L);
    p.L00 = L[0]; p.L10 = L[3]; p.L11 = L[4]; p.L20 = L[6]; p.L21 = L[7]; p.L22 = L[8];
    p.slip_factor = c.slip_factor;
    p.max_yaw_dev = c.max_yaw_deviation;
    p.spread_threshold = c.spread_threshold;
    p.spread_trans = c.spread_translation_factor;
    p.spread_rot = c.spread_rotation_factor;
    p.hash_use = c.hash_use ? 1u : 0u;
    p.seed = c.seed;
    // ContactModel::setContactPoints  src/ContactModel.cpp:21-41
    double yc[4];
    remove_yaw(q, yc);
    memcpy(ctx->zcomp, yc, sizeof(yc));
    const uint32_t m = in->n_contacts < ESLAM_MAX_CONTACTS ? in->n_contacts : ESLAM_MAX_CONTACTS;
    p.m = m;
    uint32_t ends = 0;
    for (uint32_t i = 0; i < m; ++i) {
        double pos[3];
        q_rotate(yc, in->contacts[i].position, pos);
        p.c[i].px = pos[0]; p.c[i].py = pos[1]; p.c[i].pz = pos[2];
        p.c[i].zp = 0.0 * pos[2];
        p.c[i].zz = 0.0 * pos[0] + 0.0 * pos[1];
        p.c[i].eval = !((double)in->contacts[i].contact < 0.2) ? 1u : 0u;
        const int32_t g = in->contacts[i].group_id;
        p.c[i].end = (g == -1 || i + 1 == m || g != in->contacts[i + 1].group_id) ? 1u : 0u;
        ends += p.c[i].end;
        p.eval_mask |= p.c[i].eval << i;
        p.end_mask |= p.c[i].end << i;
    }
    ctx->maxp = ends;
    // LDS window margin: foot reach + mean motion + 6 sigma of the sampled motion + 2 cells
    double reach = 0.0;
    for (uint32_t i = 0; i < m; ++i) {
        const double r = sqrt(p.c[i].px * p.c[i].px + p.c[i].py * p.c[i].py);
        reach = r > reach ? r : reach;
    }
    const double motion = sqrt(p.mu[0] * p.mu[0] + p.mu[1] * p.mu[1]) +
                          6.0 * sqrt(in->sample_cov[0] + in->sample_cov[4]);
    p.win_margin = reach + motion + 0.05;
    p.use_window = (c.flags & ESLAM_FLAG_NO_MAP_LDS) ? 0u : 1u;
    p.me2 = c.measurement_error * c.measurement_error;
    p.radius = c.contact_point_radius;
    p.corr = c.contact_likelihood_correction;
    p.min_contacts = c.min_contacts;
    p.use_shape = c.use_shape_update ? 1u : 0u;
    p.use_slip = c.use_slip_update ? 1u : 0u;
    p.n = ctx->n;
    p.gbase = ctx->gbase;
    p.n_global = ctx->n_global;
    p.J = dm_chunk_rows_cfg(ctx->n_global, ctx->cfg.sum_chunk_rows);
}

// particles per thread of the one-GPU K3: small filters take small tiles so the scan still
// spreads over every CU (256k particles: 1024 blocks instead of 128).  Exact integer tile
// totals: the tile size never changes a result.
static uint32_t scan_items(uint64_t n)
{
    // measured (round-2 A/B, profiles/r02/ab_items_256k_fused.log; bench step at 64k / 256k / 1M / 4M / 16M): 1 item +5 % at
    // 64k and 256k (over 2 items, themselves +19 % over 8 at 256k), 2 or 4 items +4 % at 1M,
    // 8 items best from 4M on (fewer tiles_before re-sums)
    if (n <= (1ull << 18)) return 1u;
    return n <= (1ull << 19) ? 2u : (n <= (2ull << 20) ? 4u : (uint32_t)kScanItems);
}

static ScanParams scan_params(eslam_ctx* ctx, uint32_t phase_b, uint32_t normalize, bool multi)
{
    ScanParams sp;
    memset(&sp, 0, sizeof(sp));
    sp.spin_limit = ctx->spin_limit;
    sp.fault = ctx->fault_host;
    sp.n = ctx->n;
    sp.gbase = ctx->gbase;
    sp.n_global = ctx->n_global;
    sp.phase_b = phase_b;
    sp.normalize = normalize;
    sp.items = multi ? (uint32_t)kScanItems : scan_items(ctx->n);
    const uint64_t tile = (uint64_t)kBlock * sp.items;
    sp.ntiles = (uint32_t)((ctx->n + tile - 1) / tile);
    sp.pub_stride = ctx->pub_stride;
    return sp;
}

static FinParams fin_params(eslam_ctx* ctx, uint32_t mode)
{
    FinParams fp;
    memset(&fp, 0, sizeof(fp));
    fp.n_global = ctx->n_global;
    fp.min_effective = ctx->cfg.min_effective;
    fp.discount = ctx->cfg.discount_factor;
    fp.spread_threshold = ctx->cfg.spread_threshold;
    fp.mode = mode;
    if (ctx->jump_n_for != ctx->n_global) {
        ctx->jump_n = dm_minstd_pow(ctx->n_global);
        ctx->jump_n_for = ctx->n_global;
    }
    fp.minstd_jump_n = ctx->jump_n;
    return fp;
}

// multi-GPU update tail:
//   the rank's 16 statistics shards -> all_gather -> every rank finalises the same global
//   scalars from all ranks' shards
//   -> normalise + this rank's fixed-point weight total -> all_gather of the totals
//   -> global stratified segments (outputs in this rank's slice are marked directly),
//      while the host reads the totals and derives every rank's output range (the
//      all_to_all_v sizes: one record per output that lands in another slice)
//   -> pack -> all_to_all_v -> expand; the gather is fused into the next k_project_weight
// a sharded step that fails after k_segments_multi has written own-slice segment marks:
// the marks buffer must be all zero for the next gather (flush_marks stores only segment
// starts) and no gather may stay pending on partial marks, so both are reset before the
// error is returned (the filter keeps the pre-resample particles)
static int abort_pending_gather(eslam_ctx* ctx, hipError_t e, int rc = ESLAM_ERR_HIP)
{
    if (e != hipSuccess) fail(ctx, ESLAM_ERR_HIP, (std::string("sharded resample: ") + hipGetErrorString(e)).c_str());
    (void)hipMemsetAsync(ctx->marks, 0, ctx->cap * 4, ctx->stream);
    (void)hipMemsetAsync(&ctx->ctl->flip, 0, sizeof(uint32_t), ctx->stream);
    (void)hipMemsetAsync(&ctx->ctl->gather, 0, sizeof(uint32_t), ctx->stream);
    (void)hipStreamSynchronize(ctx->stream);
    return rc;
}

// host spin bound of the sharded step's wait for the slice totals: the wait starts while the
// step's weighting kernel still runs; a 2 ms bound (which covers K1 + the exchanges of a 4M
// shard) measured the same as 200 us on one rank at 2M and 4M (profiles/r02/ab_spin.log)
constexpr long kSpinBoundUs = 200;

// Per-particle maps on a sharded filter: every record's map travels with it:
// a header per record (its source's table centre and page count), then the pages, each with
// its slot.  The page counts per destination come from the headers' prefix; the receivers learn
// theirs from an all_gather.  The received maps get local tables and pages in store_receive.
static int exchange_maps(eslam_ctx* ctx, uint64_t nsend, uint64_t nrecv, const uint64_t* sb, const uint64_t* rb,
                         const PlanParams& pp, hipStream_t xs)
{
    const int G = ctx->comm.nranks, me = ctx->comm.rank;
    const uint64_t R = eslam_record_bytes(), H = sizeof(MapPayHdr), P = sizeof(MapPayPage);
    int rc = grow(ctx, &ctx->sendhdr, &ctx->sendhdr_cap, (nsend ? nsend : 1) * H, false);
    if (!rc) rc = grow(ctx, &ctx->recvhdr, &ctx->recvhdr_cap, (nrecv ? nrecv : 1) * H, false);
    if (!rc) rc = grow(ctx, (void**)&ctx->payoff, &ctx->payoff_cap, (nsend + nrecv + 2) * 4, false);
    if (rc) return rc;
    PaySeg seg;
    memset(&seg, 0, sizeof(seg));
    for (int d = 0; d <= G; ++d) seg.off[d] = pp.send_off[d];
    seg.n = G;
    HIPCHK(ctx, eslam_launch_pay_hdr(ctx->st[0], ctx->st[1], ctx->ctl, ctx->sendbuf, nsend, ctx->gbase, &ctx->lm, &seg,
                                     ctx->sendhdr, ctx->payoff, xs));
    // the page counts per destination (records [send_off[d], send_off[d + 1]) go to rank d)
    std::vector<uint32_t> bound(G + 1);
    for (int d = 0; d <= G; ++d)
        HIPCHK(ctx, hipMemcpyAsync(&bound[d], ctx->payoff + pp.send_off[d], 4, hipMemcpyDeviceToHost, xs));
    HIPCHK(ctx, hipStreamSynchronize(xs));
    uint64_t* h = ctx->mg_host;
    uint64_t spg[kMaxRanks], rpg[kMaxRanks], totr = 0;
    for (int d = 0; d < G; ++d) h[mg::kCounts + d] = spg[d] = bound[d + 1] - bound[d];
    HIPCHK(ctx, hipMemcpyAsync(ctx->mg + mg::kCounts, &h[mg::kCounts], 8 * G, hipMemcpyHostToDevice, xs));
    HIPCHK(ctx, hipStreamSynchronize(xs));
    rc = comm_allgather(ctx, ctx->mg + mg::kCounts, ctx->mg + mg::kCountsAll, 8ull * G);
    if (rc) return rc;
    HIPCHK(ctx, hipMemcpy(&h[mg::kCountsAll], ctx->mg + mg::kCountsAll, 8ull * G * G, hipMemcpyDeviceToHost));
    for (int r = 0; r < G; ++r) { rpg[r] = h[mg::kCountsAll + r * G + me]; totr += rpg[r]; }
    rc = grow(ctx, &ctx->sendpay, &ctx->sendpay_cap, ((uint64_t)bound[G] + 1) * P, false);
    if (!rc) rc = grow(ctx, &ctx->recvpay, &ctx->recvpay_cap, (totr + 1) * P, false);
    if (rc) return rc;
    HIPCHK(ctx, eslam_launch_pay_pack(ctx->st[0], ctx->st[1], ctx->ctl, ctx->sendbuf, nsend, ctx->gbase, &ctx->lm, ctx->sendhdr,
                                      ctx->payoff, ctx->sendpay, xs));
    uint64_t hs[kMaxRanks], hr[kMaxRanks], ps[kMaxRanks], pr[kMaxRanks];
    for (int d = 0; d < G; ++d) {
        hs[d] = sb[d] / R * H; hr[d] = rb[d] / R * H;
        ps[d] = spg[d] * P; pr[d] = rpg[d] * P;
    }
    rc = comm_alltoallv(ctx, ctx->sendhdr, hs, ctx->recvhdr, hr, xs);
    if (!rc) rc = comm_alltoallv(ctx, ctx->sendpay, ps, ctx->recvpay, pr, xs);
    if (rc) return rc;
    ctx->nrecv_maps = nrecv;
    ctx->cow_pending = nrecv > 0;
    return ESLAM_OK;
}

static int exchange_tail(eslam_ctx* ctx, uint64_t epoch, PlanParams& pp, uint64_t* own_lo, uint64_t* own_hi,
                         hipStream_t xs = nullptr, bool* queued = nullptr);

static int run_update_tail_multi(eslam_ctx* ctx, uint32_t mode, bool timed)
{
    const int G = ctx->comm.nranks;
    int rc = comm_allgather(ctx, ctx->shards, ctx->recs, sizeof(Shard) * kNShard);
    if (rc) return rc;
    FinParams fp = fin_params(ctx, mode);
    fp.local_shards = ctx->shards;
    fp.mirror = ctx->mg + mg::kMirror;
    // an update step folds the finalize (over every rank's shards) into K3a's block 0
    const bool fused = mode == FIN_UPDATE;
    if (!fused) HIPCHK(ctx, eslam_launch_finalize(ctx->recs, G * kNShard, ctx->ctl, &fp, ctx->stream));
    if (timed) rec(ctx, 2);
    if (mode == FIN_SUM) return ESLAM_OK;
    ScanParams sp = scan_params(ctx, mode == FIN_UPDATE, mode == FIN_UPDATE || mode == FIN_NORMALIZE, true);
    sp.multi = 1;
    sp.tag = ctx->scan_tag = ctx->scan_tag % 7u + 1u;         // differs from the previous launch's
    const FusedFin ff{ctx->recs, fp, ctx->fin_word, ++ctx->fin_epoch, G * kNShard};
    HIPCHK(ctx, eslam_launch_normalize_scan(ctx->st[0], ctx->st[1], &sp, ctx->ctl, ctx->tile_sum, ctx->mg + mg::kTotal,
                                            fused ? &ff : nullptr, ctx->stream));
    rc = comm_allgather(ctx, ctx->mg + mg::kTotal, ctx->mg + mg::kTotals, 8);
    if (rc) return rc;
    uint64_t* h = ctx->mg_host;
    // the gathered totals and the finalize mirror reach the host without a copy on the
    // stream: the segments kernel's first thread writes them to the host-mapped mg_host and
    // then the launch's epoch (system-scope release)
    PlanParams pp = plan_params(ctx);
    const uint64_t epoch = ++ctx->seg_epoch;
    HIPCHK(ctx, eslam_launch_segments_multi(ctx->st[0], ctx->st[1], &sp, &pp, ctx->ctl, ctx->tile_sum, ctx->marks,
                                            ctx->tile_first, ctx->mg + mg::kTotals, ctx->jump, ctx->range,
                                            ctx->mg + mg::kFirstLast, h + mg::kTotals, h + mg::kHostEpoch, epoch,
                                            ctx->stream));
    if (timed) rec(ctx, 3);
    if (keep_ancestors(ctx)) ctx->has_anc = true;
    // an update defers the exchange to the next call, which first runs the chunks of the rank's
    // own outputs while the host waits for the totals (no particle maps: their stores travel
    // with the records and are placed by the map update)
    if (mode == FIN_UPDATE && !particle_maps(ctx)) {
        if (G > 1) {                         // one rank exchanges nothing: no side stream
            if (!ctx->xstream) {
                HIPCHK(ctx, hipStreamCreateWithFlags(&ctx->xstream, hipStreamNonBlocking));
                HIPCHK(ctx, hipEventCreateWithFlags(&ctx->ev_seg, hipEventDisableTiming));
                HIPCHK(ctx, hipEventCreateWithFlags(&ctx->ev_x, hipEventDisableTiming));
            }
            HIPCHK(ctx, hipEventRecord(ctx->ev_seg, ctx->stream));
        }
        ctx->xpend = true;
        ctx->xpend_epoch = epoch;
        ctx->xpend_pp = pp;
        if (timed) rec(ctx, 4);
        return ESLAM_OK;
    }
    uint64_t own_lo = 0, own_hi = 0;
    rc = exchange_tail(ctx, epoch, pp, &own_lo, &own_hi);
    if (timed) rec(ctx, 4);
    return rc;
}

// The exchange of a sharded resample, after k_segments_multi: wait for the gathered totals
// (host-mapped words the segments kernel writes), derive every rank's output range (the
// all_to_all_v sizes: one record per output that lands in another slice), pack, exchange,
// expand.  own_lo / own_hi: the chunks of this slice holding only its own outputs (the
// segments kernel's PlanParams::chunk_sel, computed alike).
// xs: the stream of the pack / exchange / expand (the context's stream by default; the split
// step's side stream, which waits for ev_seg, overlapping the own chunks' weighting launch)
static int exchange_tail(eslam_ctx* ctx, uint64_t epoch, PlanParams& pp, uint64_t* own_lo, uint64_t* own_hi,
                         hipStream_t xs, bool* queued)
{
    if (!xs) xs = ctx->stream;
    if (queued) *queued = false;
    const int G = ctx->comm.nranks, me = ctx->comm.rank;
    int rc = ESLAM_OK;
    uint64_t* h = ctx->mg_host;
    {
        const uint64_t csz = 64ull * pp.J;
        *own_lo = 0;
        *own_hi = (ctx->n + csz - 1) / csz;
    }
    {
        // spin on the epoch word: a blocking synchronize wakes the thread tens of microseconds
        // late, and the GPU runs dry before the next step's launches if the host is late here
        // (the segments kernel is all it has queued).  Bounded (kSpinBoundUs): past it (a hung
        // collective or kernel, or a late GPU) fall back to a blocking wait instead of burning
        // a host core next to the RCCL proxy threads.
        const auto t0 = std::chrono::steady_clock::now();
        const auto bound = std::chrono::microseconds(kSpinBoundUs);
        while (__atomic_load_n(h + mg::kHostEpoch, __ATOMIC_ACQUIRE) != epoch) {
            if (std::chrono::steady_clock::now() - t0 > bound) {
                const hipError_t q = xs == ctx->stream ? hipStreamSynchronize(xs) : hipEventSynchronize(ctx->ev_seg);
                if (q != hipSuccess) return abort_pending_gather(ctx, q);
                break;
            }
        }
        if (__atomic_load_n(h + mg::kHostEpoch, __ATOMIC_ACQUIRE) != epoch)
            return abort_pending_gather(ctx, hipErrorUnknown);
    }
    // a rank whose slice-total wait gave up all-gathers ~0: every rank stops here
    for (int r = 0; r < G; ++r)
        if (h[mg::kTotals + r] == ~0ull) {
            ctx->poisoned = true;
            (void)abort_pending_gather(ctx, hipSuccess);
            return fail(ctx, ESLAM_ERR_HIP, kPoisonMsg);
        }
    const uint64_t c_resample = h[mg::kMirror];
    const uint32_t c_minstd_start = (uint32_t)h[mg::kMirror + 1];
    const int c_scan_shift = (int)(int64_t)h[mg::kMirror + 2];
    uint64_t nrecv = 0;
    if (c_resample && G > 1) {
        // every rank's outputs [O0_r, O1_r), the same counts the device computes
        const uint64_t N = ctx->n_global;
        uint64_t O0[kMaxRanks], O1[kMaxRanks], off = 0;
        for (int r = 0; r < G; ++r) {
            const uint64_t t = h[mg::kTotals + r];
            O0[r] = r == 0 ? 0 : dm_count_draws_le(off, N, c_minstd_start, c_scan_shift);
            O1[r] = r == G - 1 ? N : dm_count_draws_le(off + t, N, c_minstd_start, c_scan_shift);
            off += t;
        }
        auto overlap = [&](int r, int d) -> uint64_t {
            const uint64_t a = O0[r] > ctx->gall[d] ? O0[r] : ctx->gall[d];
            const uint64_t b = O1[r] < ctx->gall[d + 1] ? O1[r] : ctx->gall[d + 1];
            return b > a ? b - a : 0;
        };
        const uint64_t R = eslam_record_bytes();
        uint64_t sb[kMaxRanks], rb[kMaxRanks], nsend = 0, any = 0;
        pp.send_off[0] = 0;
        for (int d = 0; d < G; ++d) {
            const uint64_t ns = d == me ? 0 : overlap(me, d);
            const uint64_t nr = d == me ? 0 : overlap(d, me);
            pp.sd[d] = O0[me] > ctx->gall[d] ? O0[me] : ctx->gall[d];
            pp.ed[d] = pp.sd[d] + ns;
            pp.send_off[d + 1] = pp.send_off[d] + ns;
            sb[d] = ns * R;
            rb[d] = nr * R;
            nsend += ns;
            nrecv += nr;
            for (int r = 0; r < G; ++r) any |= (r == d ? 0 : overlap(r, d));
        }
        if (any) {
            const bool maps = particle_maps(ctx);
            rc = grow(ctx, &ctx->sendbuf, &ctx->send_cap, nsend * R, false);
            if (!rc) rc = grow(ctx, &ctx->recvbuf, &ctx->recv_cap, nrecv * R, false);
            if (rc) return abort_pending_gather(ctx, hipSuccess, rc);
            // a side stream starts after the segments kernel (its records and ranges)
            if (xs != ctx->stream) HIPCHK(ctx, hipStreamWaitEvent(xs, ctx->ev_seg, 0));
            if (queued) *queued = true;
            const hipError_t e = eslam_launch_pack(ctx->st[0], ctx->st[1], ctx->ctl, &pp, ctx->range, ctx->mg + mg::kFirstLast,
                                                   nsend, ctx->sendbuf, xs);
            if (e != hipSuccess) return abort_pending_gather(ctx, e);
            rc = comm_alltoallv(ctx, ctx->sendbuf, sb, ctx->recvbuf, rb, xs);
            if (!rc && maps) rc = exchange_maps(ctx, nsend, nrecv, sb, rb, pp, xs);
            if (rc) return abort_pending_gather(ctx, hipSuccess, rc);
        } else {
            nrecv = 0;
        }
    }
    if (c_resample) {
        // the own-output chunks (the same function of the same totals as on the device)
        const uint64_t N = ctx->n_global;
        uint64_t off = 0;
        for (int r = 0; r < me; ++r) off += h[mg::kTotals + r];
        const uint64_t O0 = me == 0 ? 0 : dm_count_draws_le(off, N, c_minstd_start, c_scan_shift);
        const uint64_t O1 = me == G - 1 ? N : dm_count_draws_le(off + h[mg::kTotals + me], N, c_minstd_start, c_scan_shift);
        own_chunks(O0, O1, ctx->gbase, ctx->n, pp.J, own_lo, own_hi);
    }
    // marks of the migrated outputs; the gather is fused into the next k_project_weight
    HIPCHK(ctx, eslam_launch_expand(ctx->recvbuf, nrecv, ctx->gbase, ctx->marks, ctx->tile_first, xs));
    return ESLAM_OK;
}

// complete a deferred exchange before anything else reads the particles or the marks
static int settle(eslam_ctx* ctx)
{
    if (!ctx->xpend) return ESLAM_OK;
    ctx->xpend = false;
    uint64_t lo = 0, hi = 0;
    return exchange_tail(ctx, ctx->xpend_epoch, ctx->xpend_pp, &lo, &hi);
}

static int run_update_tail(eslam_ctx* ctx, uint32_t mode, bool timed)
{
    if (ctx->sharded) return run_update_tail_multi(ctx, mode, timed);
    const FinParams fp = fin_params(ctx, mode);
    // an update step folds the finalize into K3's block 0 (one launch fewer per step); the
    // standalone normalise / resample / sum keep k_finalize
    const bool fused = mode == FIN_UPDATE;
    if (!fused) HIPCHK(ctx, eslam_launch_finalize(ctx->shards, kNShard, ctx->ctl, &fp, ctx->stream));
    if (timed) rec(ctx, 2);
    ScanParams sp = scan_params(ctx, mode == FIN_UPDATE, mode == FIN_UPDATE || mode == FIN_NORMALIZE, false);
    sp.tag = ctx->scan_tag = ctx->scan_tag % 7u + 1u;         // differs from the previous launch's
    FusedFin ff{ctx->shards, fp, ctx->fin_word, ++ctx->fin_epoch, kNShard};
    HIPCHK(ctx, eslam_launch_normalize_segments(ctx->st[0], ctx->st[1], &sp, ctx->ctl, ctx->tile_sum, ctx->marks,
                                                ctx->tile_first, ctx->jump, fused ? &ff : nullptr, ctx->stream));
    if (timed) rec(ctx, 3);
    // the gather itself is fused into the next k_project_weight (or materialize())
    if (timed) rec(ctx, 4);
    if (keep_ancestors(ctx)) ctx->has_anc = true;
    return ESLAM_OK;
}

// PoseEstimator::sampleFromHash  src/PoseEstimator.cpp:130-182 (after the project kernel)
static int sample_from_hash(eslam_ctx* ctx, const eslam_step_input* in, const StepParams& p)
{
    double pos[3 * ESLAM_MAX_CONTACTS], low[3 * ESLAM_MAX_CONTACTS];
    int32_t grp[ESLAM_MAX_CONTACTS];
    for (uint32_t i = 0; i < p.m; ++i) {                      // setContactPoints: yaw-compensated feet
        pos[3 * i] = p.c[i].px; pos[3 * i + 1] = p.c[i].py; pos[3 * i + 2] = p.c[i].pz;
        grp[i] = in->contacts[i].group_id;
    }
    const uint32_t nlow = dm_lowest_points(pos, grp, p.m, low);  // getLowestPointPerGroup
    double sx, sy;
    dm_surface_param(low, nlow, &sx, &sy);
    const int bins = (int)ctx->cfg.hash_slope_bins;
    const int b = dm_bucket_index(bins, -1.0, 1.0, sx) * bins + dm_bucket_index(bins, -1.0, 1.0, sy);
    const uint32_t bsize = ctx->hash_bstart[b + 1] - ctx->hash_bstart[b];
    const double rel = dm_pow(1.0 - 1.0 * (double)bsize / (double)ctx->hash_n, 3.0);   // getRelevance^3
    const uint64_t N = ctx->n_global;
    uint64_t k = (uint64_t)(((double)N * ctx->cfg.hash_percentage) * rel);
    if (rel < 0.8) k = 0;
    if (k > N) k = N;
    if (k == 0 || bsize == 0) return ESLAM_OK;                // nothing replaced, no rand() drawn
    double S = 0.0;
    int rc = eslam_gpu_get_weights_sum(ctx, &S);
    if (rc) return rc;
    const double weight = ((S / (double)N) * ctx->cfg.hash_avg_factor) * rel;   // getWeightAvg() * avgFactor * rel
    const uint64_t n = ctx->n;
    if (ctx->sort_cap < n) {
        (void)hipFree(ctx->d_sort); ctx->d_sort = nullptr; ctx->sort_cap = 0;
        (void)hipFree(ctx->sort_tmp); ctx->sort_tmp = nullptr; ctx->sort_tmp_bytes = 0;
        HIPCHK(ctx, hipMalloc(&ctx->d_sort, sizeof(uint32_t) * 4 * n));
        size_t bytes = 0;
        HIPCHK(ctx, eslam_hash_sort(ctx->st[0], ctx->st[1], ctx->ctl, n, nullptr, nullptr, nullptr, nullptr, nullptr, &bytes,
                                    ctx->stream));
        HIPCHK(ctx, hipMalloc(&ctx->sort_tmp, bytes ? bytes : 1));
        ctx->sort_tmp_bytes = bytes;
        ctx->sort_cap = n;
    }
    uint32_t* keys = ctx->d_sort;
    uint32_t* vals = keys + n;
    uint32_t* keys_out = vals + n;
    uint32_t* order = keys_out + n;
    size_t bytes = ctx->sort_tmp_bytes;
    HIPCHK(ctx, eslam_hash_sort(ctx->st[0], ctx->st[1], ctx->ctl, n, keys, vals, keys_out, order, ctx->sort_tmp, &bytes,
                                ctx->stream));
    // sharded: the global order of the k lowest.  Rank r contributes its min(k, n_r) lowest
    // pairs (any of the k lowest lies among them); every rank sorts the same concatenation.
    const uint32_t* gorder = order;
    if (ctx->sharded) {
        const int G = ctx->comm.nranks, me = ctx->comm.rank;
        std::vector<uint64_t> cnt(G), sb(G), rb(G);
        uint64_t total = 0;
        for (int r = 0; r < G; ++r) {
            const uint64_t nr = ctx->gall[r + 1] - ctx->gall[r];
            cnt[r] = k < nr ? k : nr;
            total += cnt[r];
        }
        for (int d = 0; d < G; ++d) { sb[d] = cnt[me] * 8; rb[d] = cnt[d] * 8; }
        rc = grow(ctx, &ctx->hsend, &ctx->hsend_cap, G * cnt[me] * 8 + 8, false);
        if (!rc) rc = grow(ctx, &ctx->hrecv, &ctx->hrecv_cap, total * 8 + 8, false);
        size_t sbytes = 0;
        (void)eslam_radix_sort_pairs(nullptr, nullptr, nullptr, nullptr, total, nullptr, &sbytes, ctx->stream);
        if (!rc) rc = grow(ctx, &ctx->hsort, &ctx->hsort_cap, 16 * (total + 1) + sbytes, false);
        if (rc) return rc;
        HIPCHK(ctx, eslam_launch_hash_candidates(keys_out, order, cnt[me], ctx->gbase, G, ctx->hsend, ctx->stream));
        rc = comm_alltoallv(ctx, ctx->hsend, sb.data(), ctx->hrecv, rb.data());
        if (rc) return rc;
        uint32_t* ck = (uint32_t*)ctx->hsort;
        uint32_t* cv = ck + total + 1;
        uint32_t* sk = cv + total + 1;
        uint32_t* so = sk + total + 1;
        HIPCHK(ctx, eslam_launch_hash_unpack(ctx->hrecv, total, ck, cv, ctx->stream));
        HIPCHK(ctx, eslam_radix_sort_pairs(ck, cv, sk, so, total, so + total + 1, &sbytes, ctx->stream));
        gorder = so;
    }
    std::vector<uint32_t> draws(k);
    for (uint64_t j = 0; j < k; ++j) draws[j] = (uint32_t)((uint64_t)(uint32_t)dm_libc_rand(ctx->libcp) % bsize);
    if (ctx->draws_cap < k) {
        (void)hipFree(ctx->d_draws); ctx->d_draws = nullptr; ctx->draws_cap = 0;
        HIPCHK(ctx, hipMalloc(&ctx->d_draws, sizeof(uint32_t) * k));
        ctx->draws_cap = k;
    }
    HIPCHK(ctx, hipMemcpyAsync(ctx->d_draws, draws.data(), sizeof(uint32_t) * k, hipMemcpyHostToDevice, ctx->stream));
    if (ctx->sharded)
        HIPCHK(ctx, eslam_launch_hash_replace_global(ctx->st[0], ctx->st[1], ctx->ctl, gorder, ctx->d_draws, k, ctx->gbase,
                                                     ctx->n, ctx->d_hash_blist, ctx->hash_bstart[b], hash_field(ctx, 0),
                                                     hash_field(ctx, 1), hash_field(ctx, 2), hash_field(ctx, 3), weight,
                                                     ctx->stream));
    else
        HIPCHK(ctx, eslam_launch_hash_replace(ctx->st[0], ctx->st[1], ctx->ctl, order, ctx->d_draws, k, ctx->d_hash_blist,
                                              ctx->hash_bstart[b], hash_field(ctx, 0), hash_field(ctx, 1), hash_field(ctx, 2),
                                              hash_field(ctx, 3), weight, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));          // draws (host) must outlive the copy
    return ESLAM_OK;
}

// the device's zero-measurement-variance flag (k_finalize aborted the update): clear it and
// report the reference's exception text.  A timeout fault stays set (poisoned filter).
static int take_update_error(eslam_ctx* ctx)
{
    int rc = read_ctl(ctx);
    if (rc) return rc;
    const uint64_t err = ctx->ctl_host->err;
    if (err & (kFaultTimeout | kFaultPages)) {
        ctx->poisoned = true;
        ctx->poison_pages = (err & kFaultPages) != 0;
        return poison_fail(ctx);
    }
    if (!(err & 1ull)) return ESLAM_OK;
    ctx->ctl_host->err = 0;
    rc = write_ctl(ctx);
    if (rc) return rc;
    return fail(ctx, ESLAM_ERR_ZERO_MEAS_VAR, "using a zero measurement variance leads to singularities");
}

static int launch_step(eslam_ctx* ctx, const eslam_step_input* in, bool project, bool weight)
{
    if (!ctx->n) return fail(ctx, ESLAM_ERR_NOT_INITIALISED, "no particles");
    if (check_poisoned(ctx)) return ESLAM_ERR_HIP;
    if (weight && !ctx->has_map) return fail(ctx, ESLAM_ERR_NO_ENVIRONMENT, "No environment attached.");
    StepParams p;
    fill_step_params(ctx, in, p);
    p.proj_event = ctx->proj_event;
    // the hash respawn (static counter of src/PoseEstimator.cpp:239, per context) runs on
    // the first project and every period-th after it, between project and update
    bool respawn = false;
    if (project && ctx->cfg.hash_use && ctx->has_hash) {
        const uint64_t period = ctx->cfg.hash_period ? ctx->cfg.hash_period : 1;
        respawn = ((*ctx->hash_ev)++ % period) == 0;
    }
    // logDebug records: the update's contact points are recorded on the projected state
    const bool records = weight && record_contacts(ctx);
    // a deferred sharded exchange: the weighting launch is split around it (own-output chunks,
    // the exchange, the other chunks) unless the step takes another path first
    const bool split = ctx->xpend && !respawn && !records && !particle_maps(ctx);
    if (ctx->xpend && !split) {
        const int rc = settle(ctx);
        if (rc) return rc;
    }
    // per-particle maps: the resample gather is materialised (it carries the store names), so
    // no k_project_weight consumes one
    if (particle_maps(ctx)) {
        const int rc = materialize(ctx);
        if (rc) return rc;
    }
    // logDebug records: the project runs as its own launch first (bit-identical to the fused
    // kernel)
    if (respawn || (records && project)) {
        const GatherView gv0 = gather_view(ctx);
        HIPCHK(ctx, eslam_launch_project_weight(1, 0, (int)ctx->maxp, ctx->st[0], ctx->st[1], &ctx->map, &p, ctx->ctl,
                                                ctx->shards, &gv0, nullptr, ctx->stream, nullptr, nullptr));
        HIPCHK(ctx, eslam_launch_commit(ctx->ctl, ctx->stream));
        ctx->proj_event++;
        if (gv0.record) ctx->has_anc = true;
        if (respawn) {
            const int rc = sample_from_hash(ctx, in, p);
            if (rc) return rc;
        }
        project = false;                      // done; the update below is weight-only
        if (!weight) return ESLAM_OK;
    }
    if (records) {
        const uint32_t maxc = p.m ? p.m : 1u;
        if (ctx->dbg_cap < ctx->n || ctx->dbg.maxc < maxc) {
            free_debug(ctx);
            HIPCHK(ctx, hipMalloc(&ctx->dbg.meas, ctx->cap * 32));
            HIPCHK(ctx, hipMalloc(&ctx->dbg.ncp, ctx->cap));
            HIPCHK(ctx, hipMalloc(&ctx->dbg.cp, ctx->cap * 48ull * maxc));
            HIPCHK(ctx, hipMalloc(&ctx->dbg.resampled, 4));
            ctx->dbg.maxc = maxc;
            ctx->dbg_cap = ctx->cap;
        }
        HIPCHK(ctx, eslam_launch_contact_records(ctx->st[0], ctx->st[1], &ctx->map, &p, ctx->ctl, &ctx->dbg, store_of(ctx),
                                                 ctx->stream));
    }
    if (weight) {
        // K1's parked per-bucket sums (K1Args::bspill): one slot per chunk of this context
        const uint64_t csz = 64ull * p.J;
        const int rc = grow(ctx, (void**)&ctx->bspill, &ctx->bspill_cap, k1_bspill_bytes((ctx->n + csz - 1) / csz), false);
        if (rc) return rc;
    }
    rec(ctx, 0);
    const GatherView gv = gather_view(ctx);
    ChunkSel sel;
    memset(&sel, 0, sizeof(sel));
    if (split) {
        sel.mode = 1;                         // the own-output chunks (the segments kernel's chunk_sel)
        sel.cdev = ctx->mg + mg::kChunks;
    }
    HIPCHK(ctx, eslam_launch_project_weight(project, weight, (int)ctx->maxp, ctx->st[0], ctx->st[1], &ctx->map, &p, ctx->ctl,
                                            ctx->shards, &gv, store_of(ctx), ctx->stream, split ? &sel : nullptr, ctx->bspill));
    if (split) {
        // the previous update's exchange (its host wait overlaps the launch above), then the
        // chunks that needed its records.  A failure here leaves a half-weighted step: the
        // filter is poisoned rather than continued.
        ctx->xpend = false;
        uint64_t own_lo = 0, own_hi = 0;
        bool queued = false;
        hipStream_t xs = ctx->comm.nranks > 1 ? ctx->xstream : ctx->stream;
        const int rc = exchange_tail(ctx, ctx->xpend_epoch, ctx->xpend_pp, &own_lo, &own_hi, xs, &queued);
        if (rc) {
            ctx->poisoned = true;
            if (xs != ctx->stream) (void)hipStreamSynchronize(xs);
            return rc;
        }
        if (queued && xs != ctx->stream) {
            // the main stream continues once the records and their marks are in place
            HIPCHK(ctx, hipEventRecord(ctx->ev_x, xs));
            HIPCHK(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_x, 0));
        }
        const uint64_t csz = 64ull * p.J, nch = (ctx->n + csz - 1) / csz;
        if (own_lo > 0 || own_hi < nch) {
            sel.mode = 2;
            sel.c_lo = own_lo;
            sel.c_hi = own_hi;
            sel.cdev = nullptr;
            // the exchange may have grown (reallocated) the receive buffer: the records are read
            // through the gather view taken now, not the one of the first launch
            const GatherView gve = gather_view(ctx);
            HIPCHK(ctx, eslam_launch_project_weight(project, weight, (int)ctx->maxp, ctx->st[0], ctx->st[1], &ctx->map, &p,
                                                    ctx->ctl, ctx->shards, &gve, store_of(ctx), ctx->stream, &sel, ctx->bspill));
        }
    }
    rec(ctx, 1);
    if (project) ctx->proj_event++;
    if (gv.record) ctx->has_anc = true;
    if (weight) {
        const int rc = run_update_tail(ctx, FIN_UPDATE, true);   // finalize commits the flip
        if (rc) return rc;
        if (records) {
            // the records describe this update; its resample decision maps outputs to them
            HIPCHK(ctx, hipMemcpyAsync(ctx->dbg.resampled, &ctx->ctl->resample, 4, hipMemcpyDeviceToDevice, ctx->stream));
            ctx->dbg_valid = true;
        }
        // measVar = zSigma^2 + measurementError^2 is zero only when measurementError^2 is: in
        // that configuration the update is checked at once, so the error surfaces from this
        // call like the reference's throw (src/ContactModel.cpp:122-123) and the caller's
        // update gate pose is not advanced (src/EmbodiedSlamFilter.cpp:361-362)
        if (p.me2 == 0.0) return take_update_error(ctx);
        return ESLAM_OK;
    }
    HIPCHK(ctx, eslam_launch_commit(ctx->ctl, ctx->stream));
    rec(ctx, 2); rec(ctx, 3); rec(ctx, 4);
    return ESLAM_OK;
}

extern "C" int eslam_gpu_project(eslam_ctx* ctx, const eslam_step_input* in)
{
    if (!ctx || !in) return ESLAM_ERR_INVALID_ARG;
    return launch_step(ctx, in, true, false);
}

extern "C" int eslam_gpu_update(eslam_ctx* ctx, const eslam_step_input* in)
{
    if (!ctx || !in) return ESLAM_ERR_INVALID_ARG;
    return launch_step(ctx, in, false, true);
}

extern "C" int eslam_gpu_step(eslam_ctx* ctx, const eslam_step_input* in, int* updated)
{
    if (!ctx || !in) return ESLAM_ERR_INVALID_ARG;
    const bool gate = update_gate(ctx->cfg.measurement_threshold_distance, ctx->cfg.measurement_threshold_angle, ctx->ud_pose,
                                  in->body2odometry_rot, in->body2odometry_trans) ||
                      in->ltc_count > 0;
    const int rc = launch_step(ctx, in, true, gate);
    if (rc) return rc;
    if (gate) {
        double R[9];
        q_to_mat(in->body2odometry_rot, R);
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) ctx->ud_pose[r * 4 + c] = R[r * 3 + c];
            ctx->ud_pose[r * 4 + 3] = in->body2odometry_trans[r];
        }
    }
    if (updated) *updated = gate ? 1 : 0;
    return ESLAM_OK;
}

extern "C" int eslam_gpu_debug_set_spin_limit(eslam_ctx* ctx, uint32_t polls)
{
    if (!ctx) return ESLAM_ERR_INVALID_ARG;
    ctx->spin_limit = polls;
    return ESLAM_OK;
}

extern "C" int eslam_gpu_sync(eslam_ctx* ctx, eslam_update_info* info)
{
    if (!ctx) return ESLAM_ERR_INVALID_ARG;
    if (const int rc_ = settle(ctx)) return rc_;    // a deferred sharded exchange first
    int rc = read_ctl(ctx);
    if (rc) return rc;
    const Ctl& c = *ctx->ctl_host;
    if (info) {
        info->effective = c.eff;
        info->weight_sum = c.S;
        info->floating_weight = c.fw;
        info->max_weight = c.max_weight;
        info->data_particles = c.data_particles;
        info->total_points = c.total_points;
        info->resampled = (int32_t)c.resample;
        info->uniform_reset = (int32_t)c.uniform;
        info->resample_overruns = c.overruns;
        info->update_count = c.update_count;
        info->map_patches_dropped = c.map_dropped;
        info->map_stores_copied = c.map_copied;
        info->map_patches_covered = c.map_covered;
        info->map_stores_changed = c.map_changed;
        info->map_cells_written = c.map_written;
        info->map_pages_taken = c.map_taken;
        info->map_tiles_evicted = c.map_evicted;
        info->map_pages_free = c.pg_nfree > c.pg_cursor ? c.pg_nfree - c.pg_cursor : 0;
    }
    if (ctx->timing && ctx->ring_steps) {
        double acc[5] = {0, 0, 0, 0, 0};
        for (uint32_t k = 0; k < ctx->ring_steps; ++k) {
            hipEvent_t* e = &ctx->ring[5 * k];
            float ms;
            for (int j = 0; j < 4; ++j) { ms = 0; (void)hipEventElapsedTime(&ms, e[j], e[j + 1]); acc[j] += ms; }
            ms = 0; (void)hipEventElapsedTime(&ms, e[0], e[4]); acc[4] += ms;
        }
        eslam_kernel_times& t = ctx->times;
        const double inv = 1.0 / ctx->ring_steps;
        t.project_weight_ms = (float)(acc[0] * inv);
        t.finalize_ms = (float)(acc[1] * inv);
        t.normalize_scan_ms = (float)(acc[2] * inv);
        t.resample_ms = (float)(acc[3] * inv);
        t.total_ms = (float)(acc[4] * inv);
        ctx->ring_steps = 0;
    }
    if (ctx->timing && ctx->mring_steps) {
        double acc[5] = {0, 0, 0, 0, 0};
        for (uint32_t k = 0; k < ctx->mring_steps; ++k) {
            hipEvent_t* e = &ctx->mring[5 * k];
            float ms;
            for (int j = 0; j < 4; ++j) { ms = 0; (void)hipEventElapsedTime(&ms, e[j], e[j + 1]); acc[j] += ms; }
            ms = 0; (void)hipEventElapsedTime(&ms, e[0], e[4]); acc[4] += ms;
        }
        eslam_kernel_times& t = ctx->times;
        const double inv = 1.0 / ctx->mring_steps;
        t.map_gather_ms = (float)(acc[0] * inv);
        t.map_cow_ms = (float)(acc[1] * inv);
        t.map_plan_ms = (float)(acc[2] * inv);
        t.map_merge_ms = (float)(acc[3] * inv);
        t.map_total_ms = (float)(acc[4] * inv);
        ctx->mring_steps = 0;
    }
    if (ctx->timing && ctx->xring_steps) {
        double acc = 0;
        for (uint32_t k = 0; k < ctx->xring_steps; ++k) {
            float ms = 0;
            (void)hipEventElapsedTime(&ms, ctx->xring[2 * k], ctx->xring[2 * k + 1]);
            acc += ms;
        }
        ctx->times.map_match_ms = (float)(acc / ctx->xring_steps);
        ctx->xring_steps = 0;
    }
    return take_update_error(ctx);
}

// ---------------------------------------------------------------------------------------
// ParticleFilter<T> API
// ---------------------------------------------------------------------------------------
static int standalone(eslam_ctx* ctx, uint32_t mode)
{
    if (!ctx->n) return fail(ctx, ESLAM_ERR_NOT_INITIALISED, "no particles");
    if (check_poisoned(ctx)) return ESLAM_ERR_HIP;
    const int rc = materialize(ctx);
    if (rc) return rc;
    const uint32_t J = dm_chunk_rows_cfg(ctx->n_global, ctx->cfg.sum_chunk_rows);
    HIPCHK(ctx, eslam_launch_weight_stats(ctx->st[0], ctx->st[1], ctx->n, J, ctx->ctl, ctx->shards, ctx->stream));
    if (mode == FIN_SUM && !ctx->sharded) {
        const FinParams fp = fin_params(ctx, mode);
        HIPCHK(ctx, eslam_launch_finalize(ctx->shards, kNShard, ctx->ctl, &fp, ctx->stream));
        return ESLAM_OK;
    }
    return run_update_tail(ctx, mode, false);
}

extern "C" int eslam_gpu_get_weights_sum(eslam_ctx* ctx, double* sum)
{
    if (!ctx || !sum) return ESLAM_ERR_INVALID_ARG;
    if (const int rc_ = settle(ctx)) return rc_;    // a deferred sharded exchange first
    int rc = standalone(ctx, FIN_SUM);
    if (rc) return rc;
    rc = read_ctl(ctx);
    if (rc) return rc;
    *sum = ctx->ctl_host->S;
    return ESLAM_OK;
}

extern "C" int eslam_gpu_normalize_weights(eslam_ctx* ctx, double* effective)
{
    if (!ctx) return ESLAM_ERR_INVALID_ARG;
    if (const int rc_ = settle(ctx)) return rc_;    // a deferred sharded exchange first
    int rc = standalone(ctx, FIN_NORMALIZE);
    if (rc) return rc;
    rc = read_ctl(ctx);
    if (rc) return rc;
    if (effective) *effective = ctx->ctl_host->eff;
    return ESLAM_OK;
}

extern "C" int eslam_gpu_resample(eslam_ctx* ctx)
{
    if (!ctx) return ESLAM_ERR_INVALID_ARG;
    if (const int rc_ = settle(ctx)) return rc_;    // a deferred sharded exchange first
    ctx->dbg_valid = false;                  // the records no longer follow the particles
    return standalone(ctx, FIN_RESAMPLE);
}

extern "C" int eslam_gpu_get_best_particle_index(eslam_ctx* ctx, uint64_t* index)
{
    if (!ctx || !index) return ESLAM_ERR_INVALID_ARG;
    if (const int rc_ = settle(ctx)) return rc_;    // a deferred sharded exchange first
    if (!ctx->n) { *index = 0; return ESLAM_OK; }
    if (const int rc0 = materialize(ctx)) return rc0;
    uint64_t* out = reinterpret_cast<uint64_t*>(ctx->scratch);
    HIPCHK(ctx, eslam_launch_best_index(ctx->st[0], ctx->st[1], ctx->n, ctx->ctl, out, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ctx->scratch_host, ctx->scratch, 16, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    const uint64_t* h = reinterpret_cast<const uint64_t*>(ctx->scratch_host);
    if (!ctx->sharded) {
        *index = h[1] == ~0ull ? 0 : h[1];
        return ESLAM_OK;
    }
    // sharded: the first global maximum = the lowest rank holding the largest key
    uint64_t* m = ctx->mg_host;
    m[mg::kBest] = h[0];
    m[mg::kBest + 1] = h[1] == ~0ull ? ~0ull : ctx->gbase + h[1];
    HIPCHK(ctx, hipMemcpy(ctx->mg + mg::kBest, &m[mg::kBest], 16, hipMemcpyHostToDevice));
    const int rc = comm_allgather(ctx, ctx->mg + mg::kBest, ctx->mg + mg::kBestAll, 16);
    if (rc) return rc;
    HIPCHK(ctx, hipMemcpy(&m[mg::kBestAll], ctx->mg + mg::kBestAll, 16ull * ctx->comm.nranks, hipMemcpyDeviceToHost));
    uint64_t best = 0, idx = ~0ull;
    for (int r = 0; r < ctx->comm.nranks; ++r) {
        const uint64_t k = m[mg::kBestAll + 2 * r], i = m[mg::kBestAll + 2 * r + 1];
        if (i == ~0ull) continue;
        if (idx == ~0ull || k > best) { best = k; idx = i; }
    }
    *index = idx == ~0ull ? 0 : idx;
    return ESLAM_OK;
}

extern "C" int eslam_gpu_get_centroid(eslam_ctx* ctx, double position[3], double orientation[4])
{
    if (!ctx || !position || !orientation) return ESLAM_ERR_INVALID_ARG;
    if (const int rc_ = settle(ctx)) return rc_;    // a deferred sharded exchange first
    int rc = eslam_gpu_normalize_weights(ctx, nullptr);     // side effect, Q15
    if (rc) return rc;
    const uint32_t J = dm_chunk_rows_cfg(ctx->n_global, ctx->cfg.sum_chunk_rows);
    if (!ctx->sharded) {
        HIPCHK(ctx, eslam_launch_centroid(ctx->st[0], ctx->st[1], ctx->n, J, ctx->ctl, ctx->scratch, ctx->stream));
    } else {
        // the shards are chunk-aligned: every rank's chunk records, all-gathered (padded to
        // the largest shard) and laid out in global chunk order, feed the same fixed tree
        // as on one GPU, so every rank computes the one-GPU centroid bit for bit
        rc = materialize(ctx);
        if (rc) return rc;
        const int G = ctx->comm.nranks;
        const uint64_t csz = 64ull * J;
        std::vector<uint64_t> nch(G);
        uint64_t maxch = 1, total = 0;
        for (int r = 0; r < G; ++r) {
            nch[r] = (ctx->gall[r + 1] - ctx->gall[r] + csz - 1) / csz;
            maxch = nch[r] > maxch ? nch[r] : maxch;
            total += nch[r];
        }
        const uint64_t rec = 5 * sizeof(double);
        if (centroid_bytes(ctx->gall.data(), G, J) > ctx->cent_bytes)
            return fail(ctx, ESLAM_ERR_HIP, "getCentroid: buffer not sized by set_comm");
        double* mine = ctx->cent;
        double* all = mine + maxch * 5;
        double* a = all + G * maxch * 5;
        double* b = a + (total ? total : 1) * 5;
        hipError_t e = hipMemsetAsync(mine, 0, maxch * rec, ctx->stream);
        if (e == hipSuccess) e = eslam_launch_centroid_chunks(ctx->st[0], ctx->st[1], ctx->n, J, ctx->ctl, mine, ctx->stream);
        if (e != hipSuccess) return fail(ctx, ESLAM_ERR_HIP, hipGetErrorString(e));
        rc = comm_allgather(ctx, mine, all, maxch * rec);
        if (rc) return rc;
        uint64_t off = 0;
        for (int r = 0; r < G && e == hipSuccess; ++r) {
            if (nch[r]) e = hipMemcpyAsync(a + off * 5, all + (uint64_t)r * maxch * 5, nch[r] * rec, hipMemcpyDeviceToDevice,
                                           ctx->stream);
            off += nch[r];
        }
        if (e == hipSuccess) e = eslam_launch_centroid_tree(a, b, total, ctx->scratch, ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) return fail(ctx, ESLAM_ERR_HIP, hipGetErrorString(e));
    }
    HIPCHK(ctx, hipMemcpyAsync(ctx->scratch_host, ctx->scratch, 5 * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    const double* h = ctx->scratch_host;       // sum x w, y w, theta w, z w, w
    const double sw = h[4];
    position[0] = h[0] / sw;
    position[1] = h[1] / sw;
    position[2] = h[3] / sw;
    const double mo = h[2] / sw;
    double a[4];
    q_from_yaw(mo, a);
    q_mul(a, ctx->zcomp, orientation);
    return ESLAM_OK;
}

extern "C" int eslam_gpu_get_rng_state(eslam_ctx* ctx, eslam_rng_state* st)
{
    if (!ctx || !st) return ESLAM_ERR_INVALID_ARG;
    if (const int rc_ = settle(ctx)) return rc_;    // a deferred sharded exchange first
    int rc = read_ctl(ctx);
    if (rc) return rc;
    memset(st, 0, sizeof(*st));
    st->minstd_x = ctx->ctl_host->minstd;
    st->project_count = ctx->proj_event;
    st->init_count = ctx->init_event;
    st->hash_count = *ctx->hash_ev;
    st->max_weight = ctx->ctl_host->max_weight;
    memcpy(st->ud_pose, ctx->ud_pose, sizeof(ctx->ud_pose));
    memcpy(st->libc_rand, ctx->libcp->r, sizeof(st->libc_rand));
    st->libc_rand_pos = ctx->libcp->i;
    return ESLAM_OK;
}

extern "C" int eslam_gpu_set_rng_state(eslam_ctx* ctx, const eslam_rng_state* st)
{
    if (!ctx || !st) return ESLAM_ERR_INVALID_ARG;
    if (const int rc_ = settle(ctx)) return rc_;    // a deferred sharded exchange first
    int rc = read_ctl(ctx);
    if (rc) return rc;
    ctx->ctl_host->minstd = st->minstd_x;
    ctx->proj_event = st->project_count;
    ctx->init_event = st->init_count;
    *ctx->hash_ev = st->hash_count;
    ctx->ctl_host->max_weight = st->max_weight;
    memcpy(ctx->ud_pose, st->ud_pose, sizeof(ctx->ud_pose));
    memcpy(ctx->libcp->r, st->libc_rand, sizeof(st->libc_rand));
    ctx->libcp->i = st->libc_rand_pos % 34u;
    return write_ctl(ctx);
}

extern "C" int eslam_gpu_get_ancestors(eslam_ctx* ctx, uint32_t* out, uint64_t n)
{
    if (!ctx || !out) return ESLAM_ERR_INVALID_ARG;
    if (const int rc_ = settle(ctx)) return rc_;    // a deferred sharded exchange first
    if (!ctx->has_anc || !ctx->anc) return fail(ctx, ESLAM_ERR_INVALID_ARG, "no ancestors recorded (ESLAM_FLAG_RECORD_ANCESTORS)");
    if (const int rc = materialize(ctx)) return rc;
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    HIPCHK(ctx, hipMemcpy(out, ctx->anc, (n < ctx->n ? n : ctx->n) * 4, hipMemcpyDeviceToHost));
    return ESLAM_OK;
}

extern "C" int eslam_gpu_enable_timing(eslam_ctx* ctx, int enable)
{
    if (!ctx) return ESLAM_ERR_INVALID_ARG;
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    ctx->timing = enable != 0;
    ctx->ring_steps = 0;
    ctx->mring_steps = 0;
    ctx->xring_steps = 0;
    return ESLAM_OK;
}

extern "C" int eslam_gpu_get_kernel_times(eslam_ctx* ctx, eslam_kernel_times* t)
{
    if (!ctx || !t) return ESLAM_ERR_INVALID_ARG;
    *t = ctx->times;
    return ESLAM_OK;
}

extern "C" hipError_t eslam_launch_selftest_bm_radius(unsigned long long* bad, hipStream_t stream);

extern "C" int eslam_gpu_selftest_bm_radius(int device, uint64_t* mismatches)
{
    if (!mismatches) return ESLAM_ERR_INVALID_ARG;
    if (hipSetDevice(device) != hipSuccess) return ESLAM_ERR_HIP;
    unsigned long long* d = nullptr;
    if (hipMalloc(&d, 8) != hipSuccess) return ESLAM_ERR_OUT_OF_MEMORY;
    hipError_t e = hipMemset(d, 0, 8);
    if (e == hipSuccess) e = eslam_launch_selftest_bm_radius(d, nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    unsigned long long h = 0;
    if (e == hipSuccess) e = hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    *mismatches = h;
    return e == hipSuccess ? ESLAM_OK : ESLAM_ERR_HIP;
}

extern "C" int eslam_gpu_selftest_sort(int device, const uint32_t* keys, const uint32_t* vals, uint64_t n, uint32_t* keys_out,
                                       uint32_t* vals_out)
{
    if ((!keys || !vals || !keys_out || !vals_out) && n) return ESLAM_ERR_INVALID_ARG;
    if (hipSetDevice(device) != hipSuccess) return ESLAM_ERR_HIP;
    size_t bytes = 0;
    (void)eslam_radix_sort_pairs(nullptr, nullptr, nullptr, nullptr, n, nullptr, &bytes, nullptr);
    const uint64_t b = (n ? n : 1) * 4;
    uint32_t* d = nullptr;
    void* tmp = nullptr;
    if (hipMalloc(&d, 4 * b) != hipSuccess || hipMalloc(&tmp, bytes) != hipSuccess) return ESLAM_ERR_OUT_OF_MEMORY;
    hipError_t e = hipMemcpy(d, keys, n * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d + b / 4, vals, n * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = eslam_radix_sort_pairs(d, d + b / 4, d + 2 * b / 4, d + 3 * b / 4, n, tmp, &bytes, nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(keys_out, d + 2 * b / 4, n * 4, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(vals_out, d + 3 * b / 4, n * 4, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    (void)hipFree(tmp);
    return e == hipSuccess ? ESLAM_OK : ESLAM_ERR_HIP;
}

extern "C" int eslam_gpu_selftest_math(int device, int fn, const double* x, const double* y, double* out, uint64_t n)
{
    if (hipSetDevice(device) != hipSuccess) return ESLAM_ERR_HIP;
    double *dx = nullptr, *dy = nullptr, *dout = nullptr;
    const uint64_t b = (n ? n : 1) * 8;
    if (hipMalloc(&dx, b) != hipSuccess || hipMalloc(&dy, b) != hipSuccess || hipMalloc(&dout, b) != hipSuccess)
        return ESLAM_ERR_OUT_OF_MEMORY;
    hipError_t e = n ? hipMemcpy(dx, x, n * 8, hipMemcpyHostToDevice) : hipSuccess;
    if (e == hipSuccess) e = (y && n) ? hipMemcpy(dy, y, n * 8, hipMemcpyHostToDevice) : hipMemset(dy, 0, b);
    if (e == hipSuccess) e = eslam_launch_selftest_math(fn, dx, dy, dout, n, nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(out, dout, n * 8, hipMemcpyDeviceToHost);
    (void)hipFree(dx); (void)hipFree(dy); (void)hipFree(dout);
    return e == hipSuccess ? ESLAM_OK : ESLAM_ERR_HIP;
}
