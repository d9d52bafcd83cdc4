// eslam_internal.h -- shared between the HIP kernels and the host side of libeslam_gpu.
//
// Device memory layout (per context, one GPU):
//   state[2]   SoA fp64 x, y, theta, zpos, zsigma, weight, mprob + uint8 flags
//              (flags = n_contact_points | floating << 7); double-buffered for resample
//   marks      uint32 per particle: resample segment starts (particle index + 1)
//   row_first  uint32 per 64 outputs: source covering the row's first output
//   tile_sum   uint64 per scan tile: exact fixed-point weight total (K3a), read by K3b
//   shards     NSHARD x Shard: exact fixed-point statistics of the weighting kernel
//   ctl        Ctl: per-step scalars decided on the device (no host round trip per step)
//   jump       minstd jump-ahead tables A^(i), A^(i*2^11), A^(i*2^22)
#pragma once
#include <stdint.h>
#include "../../include/eslam_gpu.h"
#include "../../include/eslam_detmath.h"

namespace eslam_dev {

constexpr int kBlock = 256;              // threads per block (4 waves of 64)
constexpr int kWaves = kBlock / 64;
constexpr int kScanItems = 8;            // particles per thread in the scan kernel
constexpr int kScanTile = kBlock * kScanItems;   // 2048 particles per scan tile
constexpr int kGatherTile = kScanTile;           // outputs per resample-gather block
constexpr int kRow = 64;                         // outputs per row_first entry (one wave row)
constexpr int kNShard = 16;              // statistics shards (blockIdx % kNShard)
constexpr int kJumpBits = 11;
constexpr int kStatsLds = 2048;          // bytes of the statistics scratch at the LDS base
#ifndef ESLAM_WINDOW_LDS                 // experiment builds may shrink it
#define ESLAM_WINDOW_LDS 29696
#endif
// bytes of the MLS window after the statistics (1856 cells).  gfx950 allocates LDS in 1280-byte
// granules (inferred, r04i): K1 blocks of 32 736 B ran four per CU (each took 33 280 of the
// 160 KB), blocks of 31 776 B (32 000 allocated) run five: K1 180 -> 167 us at 4M
constexpr int kWindowLds = ESLAM_WINDOW_LDS;
#ifndef ESLAM_K1_ATTR                    // experiment builds may set an occupancy attribute on K1
#define ESLAM_K1_ATTR
#endif

// one statistics shard: exact sums as 4 limbs of 32-bit columns (uint64 each)
struct alignas(128) Shard {
    uint64_t A[DM_NBUCKETS][4];          // sum over chunks of  w_A * mprob        (per bucket)
    uint64_t B[DM_NBUCKETS][4];          // sum over chunks of (w_A * mprob)^2     (per bucket)
    uint64_t SW[4];                      // sum of m^(1/n) over accepted particles
    uint64_t D, TP;                      // data_particles, total_points
    uint64_t maxm;                       // bits of max accepted m (non-negative double)
    uint64_t flags;                      // bit q: accumulator q NaN, bit 16+q: infinite
    uint64_t err;                        // bit 0: zero measurement variance
    uint64_t bbox[4];                    // max of ~key(min x), key(max x), ~key(min y), key(max y)
    uint64_t pad[3];
};
static_assert(sizeof(Shard) % 128 == 0, "shard alignment");

// per-step device-side control block
struct alignas(128) Ctl {
    // committed buffer index and pending flip (latest state = base ^ flip)
    uint32_t base, flip;
    uint32_t resample;                   // decided by finalize for this update
    uint32_t uniform;                    // sumWeights <= 0 branch
    uint32_t mode;                       // finalize mode (see FinMode)
    uint32_t special;                    // 1: S NaN, 2: S inf
    uint32_t gather;                     // a resample gather is pending (marks -> state[base^1])
    uint32_t aborted;                    // the update hit the zero-measurement-variance error (phase B,
                                         // normalisation and resample skipped, as the reference's throw)
    int32_t scan_shift;                  // fixed-point shift of the resample cumulative sum
    int32_t wexp;                        // weight exponent bound for the next weighting
    double S, Q, eff, fw, max_weight;
    double f[DM_NBUCKETS];
    double inv_n;
    uint32_t minstd;                     // ParticleFilter::rand_gen state
    uint32_t minstd_start;               // state at the start of the current resample
    uint64_t tile_counter;               // dynamic tile id of the scan kernel
    uint64_t overruns;
    uint64_t data_particles, total_points;
    uint64_t update_count;
    uint64_t err;
    uint64_t bbox[4];                    // particle bounding box of the last weighting (keys)
    uint32_t k3_base;                    // the buffer the last weighting kernel wrote (base ^ flip at
                                         // its start): the fused K3 reads it while block 0 commits
    uint64_t map_dropped;                // scan patches the last map merge could not store (full stores)
    uint64_t map_changed;                // stores the last map merge changed
    uint64_t map_copied;                 // shared stores the last map merge wrote to a free store
    uint64_t map_covered;                // scan patches the last map merge saw on cells the shared grid covers
    uint64_t map_written;                // cell writes (inserts and fuses) of the last map merge
    uint64_t map_taken;                  // pages the last map merge took from the free list
    uint64_t map_evicted;                // tiles the last map update's full trails forgot
    uint64_t pg_cursor;                  // per-particle maps: next unused entry of LocalMaps::frees
    uint64_t pg_nfree;                   //   entries in LocalMaps::frees (the last collection)
    uint64_t pg_total;                   //   pages the current map update may take (its plan)
    uint32_t pg_gc;                      //   the current map update collects first
    uint32_t pg_pad;
    uint64_t fin_epoch;                  // fused finalize: the epoch of the launch whose finalize wrote
                                         // this block (checked in every block's copy of it)
};

enum FinMode : uint32_t {
    FIN_UPDATE = 0,       // updateWeights statistics -> phase B factors, normalise, maybe resample
    FIN_NORMALIZE = 1,    // standalone normalizeWeights (weights as they are)
    FIN_RESAMPLE = 2,     // standalone resample (no normalisation)
    FIN_SUM = 3,          // getWeightsSum only
};

struct DevState {
    double* x; double* y; double* th; double* z; double* zs; double* w; double* mprob;
    uint8_t* flags;
    uint32_t* sid;                       // per-particle maps only: the particle's map store
};

// Per-particle local maps (useSharedMap = false, ESLAM_FLAG_PARTICLE_MAPS): the
// shared grid plus, per particle, a window of (2 hx + 1) x (2 hy + 1) tiles of 8 x 8 cells
// around the particle (eslam_detmath.h DM_LM_*: the window reaches maxSensorRange and moves
// with the particle at every map update) and a trail of up to V tiles the window has left.
//   table  what a particle names (DevState::sid): the window centre and a row of S words: the
//          window's slots (wx * wy, padded with DM_LM_NONE to a multiple of 4; the slot of tile
//          (a, b) being (a mod wx) + wx (b mod wy), each a page id or DM_LM_NONE), then the
//          trail's V entries {a, b, page, -} (page DM_LM_NONE: empty; lm_trail_* below).
//          The resample copies the name, so copies share a table; a map update that changes
//          a table another particle also names writes the result to a free table the particle
//          then names (copy on write: a shared table is never written).
//   page   the 64 cells {mean, stdev} of one tile (stdev >= 0: the cell holds a patch).  Pages
//          are shared by tables the same way; a page is written in place only by the table
//          that owns it at the table's current generation (LocalMaps::owner == gen << 32 |
//          table), and a table's generation moves on whenever it is shared, so every page it
//          had is then frozen and copied on the next write.  Free pages come from a list the
//          map update's collection rebuilds (mark the pages live tables name, compact the
//          rest) when the list runs short.
// K1 reads the first 64 bytes (LocalMaps up to my) with one scalar load per lookup.
struct LocalMaps {
    int2* ctr;                           // per table: window centre tile (DM_LM_UNSET: an empty table)
    uint32_t* slot;                      // per table: S page ids
    float2* page;                        // per page: 64 cells {mean, stdev}, row-major (m & 7) + 8 (n & 7)
    uint32_t S, wx, wy, hx;              // S: words per table row (window slots + 4 V)
    uint32_t hy, V;                      // V: trail entries per table (the last 4 V words of a row)
    uint64_t mx, my;                     // lm_magic(wx), lm_magic(wy)
    // --- the map update and the collection only
    uint32_t bx, by;                     // multiples of wx, wy >= 2^29 (non-negative residues)
    uint32_t* tgen;                      // per table: generation (bumped when a map update finds it shared)
    uint64_t* owner;                     // per page: gen << 32 | the table that may write it in place
    uint32_t* frees;                     // the free pages, in page order, from the last collection
    uint8_t* mark;                       // per page: a live table names it (the collection's marks)
    uint64_t npages, ntables;
};
static_assert(sizeof(int2) == 8, "centre");
constexpr int kMaxRanks = 16;

// sharded filters: a particle that a resample received from another rank names no local table
// yet; its sid is kSidRecord | the record index, and the copy on write that follows the gather
// gives it a free table (and pages) filled from the record's payload (the migrated map)
constexpr uint32_t kSidRecord = 0x80000000u;
// a migrated map: the header per record (its table's centre and page count), then the pages
// of all records in the records' order, each with its slot
struct alignas(8) MapPayHdr {
    int2 ctr;
    uint32_t npg;
    uint32_t share;                      // bit 0: the previous record (same source, same destination)
                                         // carries this record's map (npg 0): they name one table;
                                         // bit 1: the map holds copies of shared-grid cells (kLmShadow)
};
// the first record of each destination's range of a sharded send (PlanParams::send_off): a
// record there always carries its map
struct PaySeg {
    uint64_t off[kMaxRanks + 1];
    int32_t n;
    int32_t pad;
};
struct alignas(8) MapPayPage {
    uint32_t slot;                       // a window slot, or kPayTrail | trail entry e of tile (a, b)
    int32_t a, b;
    uint32_t pad;
    float2 cell[DM_LM_PAGE_CELLS];
};
static_assert(sizeof(MapPayPage) == 528, "payload page");
constexpr uint32_t kPayTrail = 0x80000000u;
// a table row's word lm_trail_off - 2 (window padding): kLmShadow when the map holds its own
// copy of a cell the shared grid covers (lookups then ask the particle's cells first)
constexpr uint32_t kLmShadow = 1u;
// the tables' pool holds 2 x cap tables: at most n <= cap are named by a particle, so at least
// cap are free whenever a map update starts, and particle i may take the i-th free one (copy
// on write with a fixed, deterministic allocation of tables and no allocation counter)
inline uint64_t store_pool(uint64_t cap) { return 2 * cap; }
// a ceil(2^35 / w) multiplier: (a * m) >> 35 = floor(a / w), exactly, for a < 2^30 and
// 3 <= w <= 31 (a * m < 2^64; the rounding error a * (m w - 2^35) / (w 2^35) < 1 / w)
constexpr uint32_t kLmMagicShift = 35;
inline uint64_t lm_magic(uint32_t w) { return ((1ull << kLmMagicShift) + w - 1) / w; }
constexpr uint32_t kDefaultMapPages = 16;       // pages per particle when the config says 0

// K1 reads the first 64 bytes (the lookup header) with one scalar load per lookup
struct MapView {
    const uint32_t* cell_start;
    const float2* patch;                 // (mean, stdev) per patch
    double inv_scale_x, inv_scale_y, offset_x, offset_y;
    uint32_t width, height_cells;
    uint32_t g2l_identity;               // global2local is exactly the identity
    uint32_t has_height;                 // height != nullptr
    const float* height;                 // nullable: all horizontal
    double g2l[12];
    const uint32_t* occ;                 // bit c: the shared grid has patches in cell c (the map merge's test)
    // per cell {first patch mean, stdev (float bits), begin, count}: K1's window rows stage
    // with one 16-byte load per cell, and a lookup off the window is one load for the cell and
    // its first patch (the same values as cell_start / patch)
    const uint4* cell_tab;
};

struct ContactC {
    double px, py, zp, zz;               // yaw-compensated body-frame x, y; zp = 0.0 * pz and
                                         // zz = (0.0 * px + 0.0 * py): the zero terms of
                                         // Affine3d * p (exact, uniform per step)
    double pz;
    uint32_t eval;                       // !(contact < 0.2)
    uint32_t end;                        // group ends after this contact
};

// The head of StepParams is laid out for K1's scalar loads at the point of use (field
// order matters: see k_project_weight); the rest is read before the particle loop.
struct StepParams {
    // ---- project (PoseEstimator::project): Philox key, odometry sampler, z motion
    uint64_t seed, proj_event, gbase;    // +0
    double mu[3];                        // +24
    double L00, L10, L11, L20, L21;      // +48
    double L22, slip_factor, yaw, max_yaw_dev;   // +88
    double z_delta, z_var;               // +120
    // ---- weighting (updateWeights)
    double me2, radius, corr;            // +136
    uint64_t min_contacts;               // +160
    uint32_t use_shape;                  // +168
    uint32_t m;                          // number of contacts
    uint32_t eval_mask, end_mask;        // bit i: contact i evaluated / ends its group
    uint32_t hash_use, use_slip;
    double spread_threshold, spread_trans, spread_rot;
    // ---- sizes
    uint64_t n, n_global;
    uint32_t J;                          // canonical chunk rows
    uint32_t use_window;                 // stage the MLS window under the cloud in LDS
    double win_margin;                   // world-frame margin around the last bounding box
    ContactC c[ESLAM_MAX_CONTACTS];
};

// one particle migrating between GPUs at a multi-GPU resample (72 bytes)
struct alignas(8) Rec {
    double x, y, th, z, zs, w, mprob;
    uint64_t lohi;                       // [lo, hi) of the outputs it fills (global, clipped)
    uint64_t src;                        // flags | global source index << 8
};
static_assert(sizeof(Rec) == 72, "record size");

// multi-GPU mark encoding (monotone in output order): records from lower ranks,
// then this rank's own particles, then records from higher ranks
constexpr uint32_t kMarkOwn = 1u << 30, kMarkHigh = 1u << 31;

// a pending resample gather, consumed by the next k_project_weight (or k_resample_gather)
struct GatherView {
    uint32_t* marks;
    const uint32_t* row_first;
    uint32_t* anc;                       // ancestors (global indices) when record
    const Rec* recs;                     // multi-GPU: migrated particles
    uint32_t record;
    uint32_t multi;                      // marks use the multi-GPU source encoding
};

// which chunks a k_project_weight launch processes: all (mode 0); the own chunks named by the
// device words cdev[0..1] (mode 1); the others, [0, c_lo) and [c_hi, nchunks) (mode 2)
struct ChunkSel {
    uint32_t mode;
    uint32_t pad;
    uint64_t c_lo, c_hi;
    const uint64_t* cdev;
};

// k_project_weight's single kernel argument: its fields are read with scalar loads from the
// kernel-argument segment where they are used (offsetof), see k_project_weight
struct K1Args {
    StepParams p;
    MapView map;
    GatherView gv;
    DevState s[2];
    Ctl* ctl;
    Shard* shards;
    LocalMaps store;                     // per-particle maps (the DELTA instantiations only)
    ChunkSel sel;                        // the chunks this launch processes
    double* bspill;                      // per chunk: the per-bucket sums a wave is not in (k1_bspill_bytes)
};
// K1 keeps the per-bucket sums of the bucket its wave is in in registers; a wave whose
// particles fall into several buckets parks the others per lane in its chunk's slot here
// (DM_NBUCKETS x {A, B} x 64 lanes), so the register file holds one pair instead of six
inline uint64_t k1_bspill_bytes(uint64_t chunks) { return chunks * DM_NBUCKETS * 2 * 64 * sizeof(double); }

// one scan patch of a map update (the scan MLS of processMap, in the yaw-free body frame)
struct ScanPatch {
    double x, y, z, stdev;
};
constexpr int kMaxScanPatches = 64;
// a map update merges a scan in parts of kScanPartSmall patches (a scan of at most that many:
// one part) or of kScanPartLarge (larger scans: fewer parts, so each tile is staged about once)
constexpr uint32_t kScanPartSmall = 64, kScanPartLarge = 256;
// processMap(scanMap, match = true) (k_map_match): every kMatchSampling-th scan patch
constexpr uint32_t kMatchSampling = 10;          // src/EmbodiedSlamFilter.cpp:216
constexpr double kMatchSigma = (double)0.2f;     // :217 (a float there)
struct MatchParams {
    uint64_t n;
    uint32_t m;                          // the sampled patches in sp
    uint32_t is_id;                      // the grid's global2local is the identity
    const ScanPatch* sp;                 // device copy of the sampled patches (more than kMaxScanPatches)
    ScanPatch spi[kMaxScanPatches];      // else the sampled patches themselves (sp null)
};
constexpr int kLmBlock = 128;                   // particles per block of the page plan (k_map_plan, k_recv_plan)
constexpr uint32_t kMergeCounterSlots = 256;   // the merge's statistics, spread over slots
constexpr uint32_t kMergeCounters = 7;

// the store names of both state buffers; the copy-on-write kernels use the current one
// (base ^ flip read on the device, so the host never waits for the commit)
struct SidRef {
    uint32_t* s0;
    uint32_t* s1;
    const Ctl* ctl;
};
// the copy-on-write scratch (u32 words): ref (pool), the two compactions' tile counts, the
// free stores (pool), the received particles (cap), the received count, the free count
struct CowScratch {
    uint32_t* ref;                       // particles naming each store
    uint32_t* counts;                    // 2 x (tiles + 1)
    uint32_t* frees;                     // the stores no particle names, in store order
    uint32_t* dups;                      // the particles received from another rank (sid = kSidRecord | record)
    uint32_t* ndup;
    uint32_t* nfree;
    uint32_t tiles;                      // compaction tiles over the pool (>= the tiles over the particles)
};
constexpr int kCompactItems = 8;                // k_compact_*: items per thread
constexpr int kCompactTileItems = kBlock * kCompactItems;
inline uint64_t cow_words(uint64_t cap)
{
    const uint64_t pool = store_pool(cap), tiles = (pool + kCompactTileItems - 1) / kCompactTileItems;
    return pool + 2 * (tiles + 1) + pool + cap + 2;
}
inline CowScratch cow_layout(uint32_t* base, uint64_t cap)
{
    const uint64_t pool = store_pool(cap), tiles = (pool + kCompactTileItems - 1) / kCompactTileItems;
    CowScratch c;
    c.ref = base;
    c.counts = c.ref + pool;
    c.frees = c.counts + 2 * (tiles + 1);
    c.dups = c.frees + pool;
    c.ndup = c.dups + cap;
    c.nfree = c.ndup + 1;
    c.tiles = (uint32_t)tiles;
    return c;
}
// k_map_plan -> k_map_merge, per particle (one 128-byte record): what the plan decided, so
// the merge's first memory round trip brings everything its page moves need
constexpr uint32_t kJobPlaced = 1u, kJobShared = 2u, kJobMore = 4u, kJobMoved = 8u;   // flags; tiles of pass 1 << 8
constexpr uint32_t kJobCovered = 16u;    // a patch of this part lands on a cell the shared grid covers
struct alignas(16) MergeJob {
    uint32_t X, T;                       // the table the particle names; the table its merge writes
    uint64_t gT;                         // tgen[T] << 32 | T: the owner word of T's pages
    int32_t na, nb;                      // the window's new centre
    int32_t ox, oy;                      // its old centre (ctr[X]; the plan has moved T's window)
    uint32_t flags;
    uint32_t need;                       // bit r: tile r of pass 1 takes a new page
    uint16_t L[8];                       // pass 1's tiles (slots, ascending)
    uint32_t P[8];                       // their pages in X (DM_LM_NONE: none)
    double z, zs;                        // zPos, zSigma (the offset patch)
    uint32_t src, pad[5];                // the particle the merge reads (gather); pad to 128 B
};
static_assert(sizeof(MergeJob) == 128, "merge job");

struct MergeParams {
    uint64_t n;
    uint32_t m;                          // scan patches
    uint32_t is_id;                      // the grid's global2local is the identity
    uint64_t* cnt;                       // kMergeCounters x kMergeCounterSlots: dropped patches, changed
                                         // tables, copies, patches on covered cells, cell writes, pages
                                         // taken, tiles the trail forgot (zeroed)
    const uint32_t* ref;                 // CowScratch::ref of this update
    const uint32_t* frees;               // CowScratch::frees: particle i's table if it writes a shared map
    uint32_t* off;                       // per particle: its first page of the plan within its plan block
                                         // (k_map_plan / k_recv_plan: the exclusive prefix of the needs)
    uint32_t* poff;                      // per block of kLmBlock particles: first page offset (+ total)
    MergeJob* job;                       // per particle: k_map_plan's record for the merge
    uint16_t* codes;                     // per particle: a part's scan-patch cell codes (plan; the part's stride)
    uint32_t* fault;                     // host-mapped fault word (kFaultPages)
    GatherView gv;                       // fuse: a pending resample gather runs in the merge (one GPU)
    uint64_t gbase;
    uint32_t fuse, aux;                  // aux: carry mprob / flags (ESLAM_FLAG_NO_AUX_GATHER unset)
    uint32_t acc, pad2;                  // acc: add this merge's counters to the update's (a later 64-patch part)
    const ScanPatch* sp;                 // the part's patches (device copy of the scan)
};

// logDebug records of the last update (k_contact_records), indexed by the particle's
// position during that update: meas 4 doubles (x, y, zPos, theta), ncp, and maxc contact
// points of 6 doubles (surface point xyz, zdiff, zvar, prob)
struct DebugRec {
    double* meas;
    uint8_t* ncp;
    double* cp;
    uint32_t* resampled;                 // the update's resample decision (copied from Ctl)
    uint32_t maxc;
};

struct FinParams {
    uint64_t n_global;
    uint64_t min_effective;
    double discount;
    double spread_threshold;
    uint32_t mode;
    int32_t wexp;                        // scale exponent used by the statistics kernel
    uint32_t record;                     // 1: write update info
    uint32_t minstd_jump_n;              // A^n_global mod (2^31 - 1): the resample's N draws
    // multi-GPU only (null otherwise): the shards this rank all-gathered, zeroed once read,
    // and 3 words next to the gathered totals (resample, minstd_start, scan_shift) so the
    // host reads everything it needs for the all_to_all_v sizes with one copy
    Shard* local_shards;
    uint64_t* mirror;
};

// the finalize fused into the one-GPU K3 (k_normalize_segments<ITEMS, true>): block 0 runs
// k_finalize's block over the local shards and publishes epoch in *fin_word
struct FusedFin {
    Shard* shards;                       // the statistics shards (all ranks' on a sharded filter)
    FinParams fp;
    uint64_t* fin_word;
    uint64_t epoch;
    int nrec;                            // shards to reduce (kNShard, or kNShard x ranks)
};


struct ScanParams {
    uint64_t n, gbase, n_global;
    uint32_t phase_b;                    // apply phase-B factors
    uint32_t normalize;                  // divide by S
    uint32_t ntiles;
    uint32_t multi;                      // multi-GPU: tile prefixes + rank total, no marks
    uint32_t items;                      // particles per thread of K3: tile = kBlock * items
                                         // (2, 4 or kScanItems; sharded: kScanItems)
    uint32_t tag;                        // one GPU: this launch's tile-total tag (1..7, cycled per launch)
    uint32_t spin_limit;                 // polls of a cross-block wait before it gives up (kSpinLimit;
                                         // 0: give up at once, eslam_gpu_debug_set_spin_limit)
    uint32_t* fault;                     // host-mapped word: kFaultTimeout when a wait gave up
    uint32_t pub_stride;                 // one GPU: words between the replicas of K3's tile words
};
// K3 (one GPU) publishes each tile word in kPubReplicas copies, pub_stride words apart, and a
// tile reads the copy of its XCD (tile % kPubReplicas): every tile reads every earlier word, so
// one copy makes its few lines a hot spot of the memory system
constexpr uint32_t kPubReplicas = 8;

// A cross-block wait that gave up (a preceding tile's total or the fused finalize never
// arrived) poisons the filter: the device ORs kFaultTimeout into ctl->err and into a
// host-mapped word, writes nothing further, and every later launch that sees the bit in
// ctl->err returns at once; the host refuses the filter until it is re-initialised.
constexpr uint32_t kFaultTimeout = 4u;
// the per-particle maps' page pool could not hold a map update's pages even after a collection:
// the update wrote nothing and the filter is poisoned like a timeout (ESLAM_ERR_OUT_OF_MEMORY)
constexpr uint32_t kFaultPages = 8u;
constexpr uint32_t kSpinLimit = 1u << 18;    // x s_sleep(8) (512 clocks): ~60 ms


struct PlanParams {
    uint64_t n_global;
    int32_t rank, nranks;
    uint64_t gbase[kMaxRanks + 1];       // first global index of every rank (+ n_global)
    // per destination d != rank (host-computed from the all-gathered totals): this rank's
    // outputs in d's slice [sd[d], ed[d]) and their offsets in the send buffer
    uint64_t sd[kMaxRanks], ed[kMaxRanks];
    uint64_t send_off[kMaxRanks + 1];
    // the deferred exchange: the segments kernel writes the chunks of this rank's
    // slice whose outputs all come from its own particles, [chunk_sel[0], chunk_sel[1])
    uint64_t* chunk_sel;
    uint64_t n_local;
    uint32_t J;
};

// Chunks (64 J outputs each) of a rank's slice [W0, W0 + n) that hold only outputs of its own
// particles, whose outputs are [O0, O1) globally: the rest -- a prefix filled from lower ranks,
// a suffix from higher ranks -- needs the exchanged records.  Host and device compute it alike.
__host__ __device__ inline void own_chunks(uint64_t O0, uint64_t O1, uint64_t W0, uint64_t n, uint32_t J, uint64_t* c_lo,
                                           uint64_t* c_hi)
{
    const uint64_t csz = 64ull * J, nchunks = (n + csz - 1) / csz;
    const uint64_t lo = O0 <= W0 ? 0 : (O0 - W0 < n ? O0 - W0 : n);
    uint64_t hi = O1 <= W0 ? 0 : (O1 - W0 < n ? O1 - W0 : n);
    hi = hi < lo ? lo : hi;
    const uint64_t cl = (lo + csz - 1) / csz;
    uint64_t ch = hi == n ? nchunks : hi / csz;
    *c_lo = cl;
    *c_hi = ch < cl ? cl : ch;
}


}  // namespace eslam_dev
