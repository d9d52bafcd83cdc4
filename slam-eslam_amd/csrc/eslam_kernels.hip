// eslam_kernels.hip -- gfx950 kernels of the eSLAM per-step particle-filter update.
//
// One update of the reference (EmbodiedSlamFilter::update -> PoseEstimator::project +
// PoseEstimator::update, src/EmbodiedSlamFilter.cpp:353-369) runs as four launches with no
// host round trip:
//
//   k_project_weight  predict (src/PoseEstimator.cpp:196-237) fused with updateWeights
//                     phase A (src/PoseEstimator.cpp:276-327: ContactModel::evaluatePose,
//                     evaluateWeight, updateZPositionEstimate + the MLS lookup of
//                     GridAccess::get) and the exact per-bucket statistics
//   k_finalize        one block: floating weight, phase-B factors, normalisation sum,
//                     effective count and the resample decision (src/PoseEstimator.cpp:329,
//                     src/ParticleFilter.hpp:46-70, src/PoseEstimator.cpp:250)
//   k_normalize_scan  phase B + normalisation (src/PoseEstimator.cpp:332-345,
//                     src/ParticleFilter.hpp:46-70) and, when resampling, each tile's exact
//                     fixed-point weight total
//   k_segments        stratified resample (src/ParticleFilter.hpp:85-108): the tile prefix
//                     (sum of the preceding tile totals), a blocked fixed-point scan, the
//                     wave's draws in LDS, and the segment-start marks of every ancestor
//
// The resample gather (expand the marks by a max-scan, copy the ancestor's state) is fused
// into the next step's k_project_weight; k_resample_gather materialises a pending gather
// when the state is read (download, the standalone PoseEstimator API) before that.
//
// Everything is wave64: 256-thread blocks, butterfly reductions with __shfl_xor over 64
// lanes, ballots as 64-bit masks.  All arithmetic goes through include/eslam_detmath.h and
// the file is compiled with -ffp-contract=off, so results equal the CPU oracle bit for bit.
#include <hip/hip_runtime.h>
#include <type_traits>
#include <string.h>

#include "eslam_internal.h"

namespace eslam_dev {

// ---------------------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------------------
// lane i receives lane i ^ O's value without the LDS crossbar (ds_bpermute: ~100+ cycles of
// latency per step).  O = 1, 2: DPP quad_perm; O = 4, 8: DPP row_shl / row_shr, each writing
// only the banks (4-lane groups of a row) whose partner lies in that direction; O = 16, 32:
// gfx950's v_permlane16_swap / v_permlane32_swap (odd rows <-> even rows, upper half <->
// lower half) with both operands the value, then a per-lane pick of the swapped copy.
template <int O> __device__ __forceinline__ uint32_t xor_lane_u32(uint32_t v)
{
    static_assert(O == 1 || O == 2 || O == 4 || O == 8 || O == 16 || O == 32, "xor distance");
    if constexpr (O == 32) {
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);   // r[0]: [lo, lo], r[1]: [hi, hi]
        return (threadIdx.x & 32u) ? r[0] : r[1];
    } else if constexpr (O == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);   // r[0]: even rows, r[1]: odd rows
        return (threadIdx.x & 16u) ? r[0] : r[1];
    } else if constexpr (O == 8) {
        const int t = __builtin_amdgcn_update_dpp(0, (int)v, 0x108, 0xf, 0x3, false);     // row_shl:8, banks 0-1
        return (uint32_t)__builtin_amdgcn_update_dpp(t, (int)v, 0x118, 0xf, 0xc, false);  // row_shr:8, banks 2-3
    } else if constexpr (O == 4) {
        const int t = __builtin_amdgcn_update_dpp(0, (int)v, 0x104, 0xf, 0x5, false);     // row_shl:4, banks 0, 2
        return (uint32_t)__builtin_amdgcn_update_dpp(t, (int)v, 0x114, 0xf, 0xa, false);  // row_shr:4, banks 1, 3
    } else if constexpr (O == 2) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4e, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
    } else {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xb1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
    }
}

template <int O> __device__ __forceinline__ uint64_t xor_lane_u64(uint64_t v)
{
    return (uint64_t)xor_lane_u32<O>((uint32_t)v) | ((uint64_t)xor_lane_u32<O>((uint32_t)(v >> 32)) << 32);
}
template <int O> __device__ __forceinline__ double xor_lane(double v) { return dm_from_bits(xor_lane_u64<O>(dm_bits(v))); }
template <int O> __device__ __forceinline__ float xor_lane(float v) { return __uint_as_float(xor_lane_u32<O>(__float_as_uint(v))); }
template <int O> __device__ __forceinline__ uint32_t xor_lane(uint32_t v) { return xor_lane_u32<O>(v); }
template <int O> __device__ __forceinline__ uint64_t xor_lane(uint64_t v) { return xor_lane_u64<O>(v); }

// xor butterfly over the 64 lanes, distances 32, 16, ..., 1 (the sum contract's chunk tree:
// every stage adds the same pair in both lanes, so all lanes end with the same bits)
template <class T, class Op> __device__ __forceinline__ T wave_butterfly(T v, Op op)
{
    v = op(v, xor_lane<32>(v));
    v = op(v, xor_lane<16>(v));
    v = op(v, xor_lane<8>(v));
    v = op(v, xor_lane<4>(v));
    v = op(v, xor_lane<2>(v));
    v = op(v, xor_lane<1>(v));
    return v;
}

// one stage of a transposed xor butterfly over 2H totals per lane (see K1's chunk flush):
// the lane with bit O set keeps the upper H totals, its partner the lower H, and each adds
// the partner's copy of the totals it keeps
// transpose_add with another order-free operation (float maxima)
template <int O, int H, int N, class Op> __device__ __forceinline__ void transpose_op(float (&v)[N], uint32_t lane, Op op)
{
    const bool up = (lane & (uint32_t)O) != 0u;
#pragma unroll
    for (int j = 0; j < H; ++j) {
        const float send = up ? v[j] : v[H + j];
        const float keep = up ? v[H + j] : v[j];
        v[j] = op(keep, xor_lane<O>(send));
    }
}

template <int O, int H, int N> __device__ __forceinline__ void transpose_add(double (&v)[N], uint32_t lane)
{
    const bool up = (lane & (uint32_t)O) != 0u;
#pragma unroll
    for (int j = 0; j < H; ++j) {
        const double send = up ? v[j] : v[H + j];
        const double keep = up ? v[H + j] : v[j];
        v[j] = keep + xor_lane<O>(send);
    }
}

__device__ __forceinline__ double wave_sum_butterfly(double v)
{
    return wave_butterfly(v, [](double a, double b) { return a + b; });
}

__device__ __forceinline__ double wave_max_butterfly(double v)
{
    return wave_butterfly(v, [](double a, double b) { return (a < b) ? b : a; });
}

// inclusive max-scan over the 64 lanes with DPP (VALU lane moves, no LDS round trips):
// row_shr 1,2,4,8 inside each row of 16, then row_bcast:15 and row_bcast:31 across rows.
// 0 is the identity (lanes without a source keep it).
__device__ __forceinline__ uint32_t wave_incl_max_u32(uint32_t m)
{
    uint32_t t;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x111, 0xf, 0xf, false); m = m > t ? m : t;   // row_shr:1
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x112, 0xf, 0xf, false); m = m > t ? m : t;   // row_shr:2
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x114, 0xf, 0xf, false); m = m > t ? m : t;   // row_shr:4
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x118, 0xf, 0xf, false); m = m > t ? m : t;   // row_shr:8
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x142, 0xa, 0xf, false); m = m > t ? m : t;   // row_bcast:15
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x143, 0xc, 0xf, false); m = m > t ? m : t;   // row_bcast:31
    return m;
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v)
{
    return wave_butterfly(v, [](uint32_t a, uint32_t b) { return a + b; });
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v)
{
    return wave_butterfly(v, [](uint64_t a, uint64_t b) { return a + b; });
}

__device__ __forceinline__ uint64_t atomic_load_agent(const uint64_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void atomic_store_agent(uint64_t* p, uint64_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t jump_pow(const uint32_t* __restrict__ jt, uint64_t e)
{
    // A^e for e < 2^32 from three tables: A^(i), A^(i*2^11), A^(i*2^22)
    uint32_t a = jt[e & 2047u];
    uint32_t b = jt[2048u + ((e >> 11) & 2047u)];
    uint32_t c = jt[4096u + ((e >> 22) & 1023u)];
    return dm_mulmod31(dm_mulmod31(a, b), c);
}

// ---------------------------------------------------------------------------------------
// Diagnostic builds only (-DESLAM_STAMPS, tools/stamps.py): per-block s_memrealtime stamps
// (100 MHz, one clock for the whole device) at the phase boundaries of K1 and K3, written by
// thread 0 to arrays of their own.  The product build compiles none of it.
// ---------------------------------------------------------------------------------------
#ifdef ESLAM_STAMPS
constexpr uint32_t kStampBlocks = 32768, kStampSlots = 8;
__device__ uint64_t g_stamps_k1[kStampBlocks][kStampSlots];
__device__ uint64_t g_stamps_k3[kStampBlocks][kStampSlots];
__device__ uint64_t g_stamps_mg[kStampBlocks][kStampSlots];   // the map merge (its first group)
__device__ __forceinline__ uint64_t stamp_now()
{
    uint64_t t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
__device__ uint32_t g_stamps_grid[3];    // gridDim.x of the last stamped K1 / K3 launch
#define ESLAM_STAMP(arr, k) \
    do { \
        if (threadIdx.x == 0 && blockIdx.x < kStampBlocks) arr[blockIdx.x][(k)] = stamp_now(); \
        if ((k) == 0 && threadIdx.x == 0 && blockIdx.x == 0) g_stamps_grid[&arr == &g_stamps_k1 ? 0 : &arr == &g_stamps_k3 ? 1 : 2] = gridDim.x; \
    } while (0)
#else
#define ESLAM_STAMP(arr, k) do { } while (0)
#endif

// ---------------------------------------------------------------------------------------
// K1 kernel arguments by scalar load at the point of use.  K1 reads ~110 uniform values
// (contacts, sampler, map header, state pointers).  Loaded once at kernel entry they exceed
// the 102 SGPRs, and the compiler parks them in VGPR lanes and fetches them back with
// v_readlane (a VALU instruction) on every row.  A volatile asm load + wait cannot be
// hoisted, so each value occupies SGPRs only where it is used; the scalar cache serves the
// repeats.  Outputs are early-clobber: the loads are in flight while the address is live.
// ---------------------------------------------------------------------------------------
typedef uint32_t su2 __attribute__((ext_vector_type(2)));
typedef uint32_t su4 __attribute__((ext_vector_type(4)));
typedef uint32_t su8 __attribute__((ext_vector_type(8)));
typedef uint32_t su16 __attribute__((ext_vector_type(16)));

#define KOFF(f) ((uint32_t)offsetof(K1Args, f))

__device__ __forceinline__ uint64_t kseg() { return (uint64_t)(uintptr_t)__builtin_amdgcn_kernarg_segment_ptr(); }

__device__ __forceinline__ su2 kl2(uint32_t off)
{
    su2 r;
    asm volatile("s_load_dwordx2 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=&s"(r) : "s"(kseg()), "s"(off));
    return r;
}
__device__ __forceinline__ su4 kl4(uint32_t off)
{
    su4 r;
    asm volatile("s_load_dwordx4 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=&s"(r) : "s"(kseg()), "s"(off));
    return r;
}
__device__ __forceinline__ su8 kl8(uint32_t off)
{
    su8 r;
    asm volatile("s_load_dwordx8 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=&s"(r) : "s"(kseg()), "s"(off));
    return r;
}
__device__ __forceinline__ su16 kl16(uint32_t off)
{
    su16 r;
    asm volatile("s_load_dwordx16 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=&s"(r) : "s"(kseg()), "s"(off));
    return r;
}
// two blocks, one wait
__device__ __forceinline__ void kl8_2(uint32_t off_a, uint32_t off_b, su8& a, su2& b)
{
    asm volatile("s_load_dwordx8 %0, %2, %3\n\ts_load_dwordx2 %1, %2, %4\n\ts_waitcnt lgkmcnt(0)"
                 : "=&s"(a), "=&s"(b) : "s"(kseg()), "s"(off_a), "s"(off_b));
}
template <class V> __device__ __forceinline__ uint64_t kq(const V& r, int k)
{
    return (uint64_t)r[2 * k] | ((uint64_t)r[2 * k + 1] << 32);
}
template <class V> __device__ __forceinline__ double kd(const V& r, int k) { return dm_from_bits(kq(r, k)); }
// pointers from the kernel arguments are global memory: the explicit address space gives
// global_load/store (SGPR base + 32-bit offset, vmcnt only) instead of flat accesses
template <class T> using gmem = __attribute__((address_space(1))) T;
template <class T, class V> __device__ __forceinline__ gmem<T>* kp(const V& r, int k) { return (gmem<T>*)(uintptr_t)kq(r, k); }

// the state pointers of buffer s[b] (offset KOFF(s[b]))
struct StatePtrs {
    gmem<double> *x, *y, *th, *z, *zs, *w, *mprob;
    gmem<uint8_t>* flags;
};
__device__ __forceinline__ StatePtrs kstate(uint32_t off)
{
    const su16 r = kl16(off);
    return StatePtrs{kp<double>(r, 0), kp<double>(r, 1), kp<double>(r, 2), kp<double>(r, 3),
                     kp<double>(r, 4), kp<double>(r, 5), kp<double>(r, 6), kp<uint8_t>(r, 7)};
}

static_assert(offsetof(StepParams, mu) == 24 && offsetof(StepParams, L22) == 88 && offsetof(StepParams, z_delta) == 120 &&
                  offsetof(StepParams, me2) == 136 && offsetof(StepParams, use_shape) == 168,
              "K1 scalar-load blocks");
static_assert(offsetof(MapView, width) == 48 && offsetof(MapView, height) == 64, "map lookup header");
static_assert(offsetof(ContactC, pz) == 32 && offsetof(GatherView, record) == 32, "K1 scalar-load blocks");
static_assert(offsetof(LocalMaps, S) == 24 && offsetof(LocalMaps, hy) == 40 && offsetof(LocalMaps, mx) == 48 &&
                  offsetof(LocalMaps, my) == 56, "K1 reads the local maps' first 64 bytes");

// ---------------------------------------------------------------------------------------
// GridAccess::get -> MLSMap::getPatch(C_global2local * p, patch, 3.0)  (src/PoseEstimator.hpp:97-105)
// qv: the query patch variance (measVar).  Cell: floor((x - offset) * (1/scale)); the
// 3-sigma gate |mean_p - z| < 3 sqrt(stdev_p^2 + measVar) is evaluated squared.
// The window part of the grid under the particle cloud may be staged in LDS: identical
// values, so the result never depends on whether a cell came from LDS or global memory.
// ---------------------------------------------------------------------------------------
// One window cell in LDS: its first patch inline + its patch range in global memory, so a
// lookup is one 16-byte LDS read (further patches of multi-patch cells come from global).
struct alignas(16) WinCell {
    float mean0, stdev0;
    uint32_t begin, count;
};

// The window's bounds stay in LDS (k1_win) and are re-read where used: held in registers
// across the particle loop they would be 6 more long-lived SGPRs, which K1 cannot afford.
__shared__ __attribute__((aligned(16))) int k1_win[8];   // on, m0, m1, n0, n1, cols

struct Window {
    int on;                              // staged (block-uniform)
    const WinCell* cells;                // rows x cols (LDS)
};

struct WinBounds {
    int on, m0, m1, n0, n1, cols;        // cell range [m0,m1) x [n0,n1)
};
__device__ __forceinline__ WinBounds win_bounds()
{
    typedef int vi4 __attribute__((ext_vector_type(4)));
    typedef int vi2 __attribute__((ext_vector_type(2)));
    // volatile keeps the reads where they are used; the explicit LDS address space keeps
    // them ds_read (a volatile generic pointer became a flat load + vmcnt(0) wait)
    typedef const volatile __attribute__((address_space(3))) vi4 lds_vi4;
    typedef const volatile __attribute__((address_space(3))) vi2 lds_vi2;
    const vi4 a = *(lds_vi4*)(&k1_win[0]);
    const vi2 b = *(lds_vi2*)(&k1_win[4]);
    return WinBounds{a.x, a.y, a.z, a.w, b.x, b.y};
}

__device__ __forceinline__ bool patch_gate(const gmem<const float>* height, uint32_t k, float pmf, float psf, double lz, double qv,
                                           double& mean, double& stdev)
{
    const double pm = (double)pmf, ps = (double)psf;
    const double ph = height ? (double)height[k] : 0.0;
    double diff;
    if (ph > 0.0) {
        if (lz > pm) diff = lz - pm;
        else if (lz < pm - ph) diff = (pm - ph) - lz;
        else diff = 0.0;
    } else {
        diff = dm_fabs(pm - lz);
    }
    if (diff * diff < 9.0 * (ps * ps + qv)) { mean = pm; stdev = ps; return true; }
    return false;
}

// per-particle maps: the patch of cell (m, n), which the shared grid leaves empty, from the
// particle's table (K1Args::store) with the same 3-sigma gate as a grid patch:
// the table's centre and the tile's slot load together, then the page cell.  A tile outside
// the window comes from the table's trail (rare: the window follows the particle).
__device__ __forceinline__ bool store_patch(uint32_t sid, uint32_t m, uint32_t n, double lz, double qv, double& mean,
                                            double& stdev)
{
    const su16 h = kl16(KOFF(store));                // 64 bytes: ctr, slot, page, {S, wx}, {wy, hx}, {hy, V}, mx, my
    const uint64_t w3 = kq(h, 3), w4 = kq(h, 4), w5 = kq(h, 5);
    const uint32_t S = (uint32_t)w3, wx = (uint32_t)(w3 >> 32), wy = (uint32_t)w4, hx = (uint32_t)(w4 >> 32);
    const uint32_t hy = (uint32_t)w5, V = (uint32_t)(w5 >> 32);
    const uint32_t a = m >> DM_LM_TILE_BITS, b = n >> DM_LM_TILE_BITS;
    const uint32_t qa = (uint32_t)(((uint64_t)a * kq(h, 6)) >> kLmMagicShift);
    const uint32_t qb = (uint32_t)(((uint64_t)b * kq(h, 7)) >> kLmMagicShift);
    const uint32_t s = (a - wx * qa) + wx * (b - wy * qb);
    const uint64_t c = kp<const uint64_t>(h, 0)[sid];   // int2 {x, y}
    const gmem<const uint32_t>* row = kp<const uint32_t>(h, 1) + (uint64_t)sid * S;
    uint32_t pg = row[s];
    if (!dm_lm_inside(a, (int32_t)(uint32_t)c, hx, wx) || !dm_lm_inside(b, (int32_t)(uint32_t)(c >> 32), hy, wy)) {
        pg = DM_LM_NONE;
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        const gmem<const u4>* t = reinterpret_cast<const gmem<const u4>*>(row + (S - 4u * V));
        const uint32_t hwv = row[S - 4u * V - 1u], hw = hwv == DM_LM_NONE ? 0u : hwv;
        for (uint32_t e = 0; e < hw; ++e) {
            const u4 v = t[e];
            if (v.z != DM_LM_NONE && v.x == a && v.y == b) pg = v.z;
        }
    }
    if (pg == DM_LM_NONE) return false;
    const uint64_t pf = reinterpret_cast<const gmem<const uint64_t>*>(kp<const float2>(h, 2))
        [(uint64_t)pg * DM_LM_PAGE_CELLS + (m & 7u) + 8u * (n & 7u)];
    const float sd = __uint_as_float((uint32_t)(pf >> 32));
    if (!dm_lm_holds(sd)) return false;
    return patch_gate(nullptr, 0, __uint_as_float((uint32_t)pf), sd, lz, qv, mean, stdev);
}

// store_patch for up to N feet of one particle at once (the cells get_patch<DELTA, true>
// deferred: dm[i] = ~0 for the others): the table's centre and every foot's slot in one round
// trip, then every page cell in one; the same results as store_patch foot by foot.  A tile
// outside the window (rare) takes store_patch itself.
constexpr uint32_t kStoreTrail = 0xfffffffeu;      // store_patches: a tile outside the window
template <int N>
__device__ __forceinline__ void store_patches(uint32_t sid, const uint32_t (&dm)[N], const uint32_t (&dn)[N],
                                              const double (&lz)[N], double qv, bool (&fnd)[N], double (&mean)[N],
                                              double (&stdev)[N])
{
    const su16 h = kl16(KOFF(store));
    const uint64_t w3 = kq(h, 3), w4 = kq(h, 4), w5 = kq(h, 5);
    const uint32_t S = (uint32_t)w3, wx = (uint32_t)(w3 >> 32), wy = (uint32_t)w4, hx = (uint32_t)(w4 >> 32);
    const uint32_t hy = (uint32_t)w5;
    const gmem<const uint32_t>* row = kp<const uint32_t>(h, 1) + (uint64_t)sid * S;
    bool any = false;
#pragma unroll
    for (int i = 0; i < N; ++i) any |= dm[i] != 0xffffffffu;
    if (!any) return;
    const uint64_t c = kp<const uint64_t>(h, 0)[sid];   // int2 {x, y}
    uint32_t pg[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        pg[i] = DM_LM_NONE;
        if (dm[i] == 0xffffffffu) continue;
        const uint32_t a = dm[i] >> DM_LM_TILE_BITS, b = dn[i] >> DM_LM_TILE_BITS;
        const uint32_t qa = (uint32_t)(((uint64_t)a * kq(h, 6)) >> kLmMagicShift);
        const uint32_t qb = (uint32_t)(((uint64_t)b * kq(h, 7)) >> kLmMagicShift);
        pg[i] = row[(a - wx * qa) + wx * (b - wy * qb)];
    }
    uint64_t pf[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        pf[i] = 0;
        if (dm[i] == 0xffffffffu) continue;
        const uint32_t a = dm[i] >> DM_LM_TILE_BITS, b = dn[i] >> DM_LM_TILE_BITS;
        if (!dm_lm_inside(a, (int32_t)(uint32_t)c, hx, wx) || !dm_lm_inside(b, (int32_t)(uint32_t)(c >> 32), hy, wy)) {
            pg[i] = kStoreTrail;                         // the trail: store_patch below
        } else if (pg[i] != DM_LM_NONE) {
            pf[i] = reinterpret_cast<const gmem<const uint64_t>*>(kp<const float2>(h, 2))
                [(uint64_t)pg[i] * DM_LM_PAGE_CELLS + (dm[i] & 7u) + 8u * (dn[i] & 7u)];
        }
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {
        if (dm[i] == 0xffffffffu) continue;
        if (pg[i] == kStoreTrail) {
            fnd[i] = store_patch(sid, dm[i], dn[i], lz[i], qv, mean[i], stdev[i]);
        } else if (pg[i] != DM_LM_NONE) {
            const float sd = __uint_as_float((uint32_t)(pf[i] >> 32));
            fnd[i] = dm_lm_holds(sd) && patch_gate(nullptr, 0, __uint_as_float((uint32_t)pf[i]), sd, lz[i], qv, mean[i], stdev[i]);
        }
    }
}

// a particle's table name for get_patch<DELTA>, with bit 31 set when its map holds copies of
// shared-grid cells (kLmShadow in its row): its lookups then ask its own cells first
__device__ __forceinline__ uint32_t store_sid(uint32_t sid)
{
    const su16 h = kl16(KOFF(store));
    const uint64_t w3 = kq(h, 3), w5 = kq(h, 5);
    const uint32_t S = (uint32_t)w3, V = (uint32_t)(w5 >> 32);
    const uint32_t f = kp<const uint32_t>(h, 1)[(uint64_t)sid * S + (S - 4u * V - 2u)];
    return sid | (f == kLmShadow ? 0x80000000u : 0u);
}

// the map is K1Args::map, read by scalar loads (header: 64 bytes per lookup).  DELTA: the
// particle's own map answers for cells the shared grid leaves empty, and first for every cell
// when it holds copies of shared-grid cells (sid bit 31, store_sid).
// DEFER (DELTA, a particle without copies of grid cells): a lookup that needs the particle's
// own map does not make it but returns false with *dm, *dn = its cell (else *dm = ~0), so the
// caller makes the lookups of all its feet together (store_patches)
template <bool DELTA = false, bool DEFER = false>
__device__ __forceinline__ bool get_patch(const Window& win, double px, double py, double pz, double qv, double& mean,
                                          double& stdev, uint32_t sid = 0, uint32_t* dm = nullptr, uint32_t* dn = nullptr,
                                          double* dlz = nullptr)
{
    if constexpr (DEFER) *dm = 0xffffffffu;
    const su16 h = kl16(KOFF(map));
    const uint32_t width = h[12], hcells = h[13], ident = h[14], has_height = h[15];
    double lx = px, ly = py, lz = pz;    // an identity global2local is applied as the identity
    if (!ident) {
        const su16 a = kl16(KOFF(map.g2l));
        const su8 b = kl8(KOFF(map.g2l[8]));
        lx = ((kd(a, 0) * px + kd(a, 1) * py) + kd(a, 2) * pz) + kd(a, 3);
        ly = ((kd(a, 4) * px + kd(a, 5) * py) + kd(a, 6) * pz) + kd(a, 7);
        lz = ((kd(b, 0) * px + kd(b, 1) * py) + kd(b, 2) * pz) + kd(b, 3);
    }
    const double ux = (lx - kd(h, 4)) * kd(h, 2);
    const double uy = (ly - kd(h, 5)) * kd(h, 3);
    if constexpr (DELTA) {
        if (sid >> 31) {                     // the particle's own cell first (the oracle's particle_map_fn)
            sid &= 0x7fffffffu;
            const double fm = floor(ux), fn = floor(uy);
            if ((fm >= 0.0) & (fm < (double)width) & (fn >= 0.0) & (fn < (double)hcells) &&
                store_patch(sid, (uint32_t)fm, (uint32_t)fn, lz, qv, mean, stdev))
                return true;
        }
    }
    // fast path without branches: an in-window cell whose first patch passes the gate (the
    // window is only staged for maps without heights).  Everything else -- off the window,
    // heights, a failing first patch of a multi-patch cell -- takes the loop below.  The
    // window lies inside the grid and starts at cell 1 in both directions, so the window test
    // needs no floor: v_cvt_i32_f64 truncates (saturating; NaN -> 0), which equals the floor
    // for every value >= 0, and maps every value < 1 -- negatives, NaN -- below the window.
    int im, in;                          // v_cvt_i32_f64 itself: defined for every input
    asm("v_cvt_i32_f64 %0, %1" : "=v"(im) : "v"(ux));
    asm("v_cvt_i32_f64 %0, %1" : "=v"(in) : "v"(uy));
    const WinBounds wb = win_bounds();
    const uint32_t wm = (uint32_t)im - (uint32_t)wb.m0, wn = (uint32_t)in - (uint32_t)wb.n0;
    const bool in_win = (wb.on != 0) & (wm < (uint32_t)wb.cols) & (wn < (uint32_t)(wb.n1 - wb.n0));
    const WinCell wc = win.cells[in_win ? wn * (uint32_t)wb.cols + wm : 0u];
    const double pm = (double)wc.mean0, ps = (double)wc.stdev0;
    const double diff = dm_fabs(pm - lz);
    const bool gate0 = in_win & (wc.count > 0) & (diff * diff < 9.0 * (ps * ps + qv));
    mean = pm;
    stdev = ps;
    if (gate0) return true;
    // the cell by the floor (outside the window trunc and floor differ)
    const double fm = floor(ux), fn = floor(uy);
    asm("v_cvt_i32_f64 %0, %1" : "=v"(im) : "v"(fm));
    asm("v_cvt_i32_f64 %0, %1" : "=v"(in) : "v"(fn));
    const bool in_grid = (fm >= 0.0) & (fm < (double)width) & (fn >= 0.0) & (fn < (double)hcells);
    if constexpr (DELTA) {
        if (!in_grid || (in_win && wc.count == 1)) return false;
        if (in_win && wc.count == 0) {
            if constexpr (DEFER) {
                *dm = (uint32_t)im;
                *dn = (uint32_t)in;
                *dlz = lz;
                return false;
            }
            return store_patch(sid, (uint32_t)im, (uint32_t)in, lz, qv, mean, stdev);
        }
    } else {
        if (!in_grid || (in_win && wc.count <= 1)) return false;
    }
    const gmem<const float>* height = has_height ? kp<const float>(kl2(KOFF(map.height)), 0) : nullptr;
    const gmem<const float2>* patch = kp<const float2>(h, 1);
    uint32_t b, e;
    if (in_win) {
        b = wc.begin + 1;
        e = wc.begin + wc.count;
    } else {
        // the cell's record (MapView::cell_tab): its range and first patch in one load
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        const gmem<const u4>* tab = kp<const u4>(kl2(KOFF(map.cell_tab)), 0);
        const uint64_t cell = (uint64_t)in * width + (uint64_t)im;
        const u4 ct = tab[cell];
        b = ct.z;
        e = ct.z + ct.w;
        if constexpr (DELTA) {
            if (b == e) {
                if constexpr (DEFER) {
                    *dm = (uint32_t)im;
                    *dn = (uint32_t)in;
                    *dlz = lz;
                    return false;
                }
                return store_patch(sid, (uint32_t)im, (uint32_t)in, lz, qv, mean, stdev);
            }
        }
        if (!has_height && b < e) {
            if (patch_gate(nullptr, 0, __uint_as_float(ct.x), __uint_as_float(ct.y), lz, qv, mean, stdev)) return true;
            ++b;
        }
    }
    for (uint32_t k = b; k < e; ++k) {
        const uint64_t pf = reinterpret_cast<const gmem<const uint64_t>*>(patch)[k];   // float2 {mean, stdev}
        if (patch_gate(height, k, __uint_as_float((uint32_t)pf), __uint_as_float((uint32_t)(pf >> 32)), lz, qv, mean,
                       stdev))
            return true;
    }
    return false;
}

__device__ __forceinline__ uint64_t order_key(double w)
{
    const uint64_t b = dm_bits(w);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

__device__ __forceinline__ double key_value(uint64_t k)
{
    return dm_from_bits((k >> 63) ? (k & 0x7fffffffffffffffull) : ~k);
}

// Stage the grid cells under last step's particle cloud (+ margin) into LDS.  Every block
// computes the same window from ctl; a window that does not fit is simply not used.
__device__ Window stage_window(const MapView& m, const StepParams& p, const Ctl* ctl, double extra_margin,
                               unsigned char* lds)
{
    int* s_w = k1_win;
    Window w;
    w.on = 0;
    if (threadIdx.x == 0) {
        int on = 0;
        const uint64_t k0 = ctl->bbox[0], k1 = ctl->bbox[1], k2 = ctl->bbox[2], k3 = ctl->bbox[3];
        if (p.use_window && k0 && k1 && k2 && k3 && !m.height) {
            const double mg = p.win_margin + extra_margin;
            const double x0 = key_value(~k0) - mg, x1 = key_value(k1) + mg;
            const double y0 = key_value(~k2) - mg, y1 = key_value(k3) + mg;
            const double* A = m.g2l;
            double lx0 = 1e300, lx1 = -1e300, ly0 = 1e300, ly1 = -1e300;
            for (int c = 0; c < 4; ++c) {
                const double wx = (c & 1) ? x1 : x0, wy = (c & 2) ? y1 : y0;
                const double lx = (A[0] * wx + A[1] * wy) + A[3], ly = (A[4] * wx + A[5] * wy) + A[7];
                lx0 = lx < lx0 ? lx : lx0; lx1 = lx > lx1 ? lx : lx1;
                ly0 = ly < ly0 ? ly : ly0; ly1 = ly > ly1 ? ly : ly1;
            }
            const double fm0 = floor((lx0 - m.offset_x) * m.inv_scale_x) - 1.0;
            const double fm1 = floor((lx1 - m.offset_x) * m.inv_scale_x) + 2.0;
            const double fn0 = floor((ly0 - m.offset_y) * m.inv_scale_y) - 1.0;
            const double fn1 = floor((ly1 - m.offset_y) * m.inv_scale_y) + 2.0;
            if (dm_isfinite(fm0) && dm_isfinite(fm1) && dm_isfinite(fn0) && dm_isfinite(fn1)) {
                // the window starts at cell 1 (get_patch's floor-free window test); cells of
                // column / row 0 take the general path
                const double W = (double)m.width, H = (double)m.height_cells;
                const int m0 = (int)(fm0 < 1 ? 1 : (fm0 > W ? W : fm0));
                const int m1 = (int)(fm1 < 1 ? 1 : (fm1 > W ? W : fm1));
                const int n0 = (int)(fn0 < 1 ? 1 : (fn0 > H ? H : fn0));
                const int n1 = (int)(fn1 < 1 ? 1 : (fn1 > H ? H : fn1));
                const int rows = n1 - n0, cols = m1 - m0;
                if (rows > 0 && cols > 0 && (int64_t)rows * cols * (int64_t)sizeof(WinCell) <= kWindowLds) {
                    on = 1;
                    s_w[1] = m0; s_w[2] = m1; s_w[3] = n0; s_w[4] = n1; s_w[5] = cols;
                }
            }
        }
        s_w[0] = on;
    }
    __syncthreads();
    if (!s_w[0]) return w;
    const int wm0 = s_w[1], wn0 = s_w[3], wn1 = s_w[4], wcols = s_w[5];
    WinCell* cells = reinterpret_cast<WinCell*>(lds);
    const int ncell = (wn1 - wn0) * wcols;
    // one memory round trip per batch of kPer cells per thread: each cell's record in
    // MapView::cell_tab is already the WinCell (range + first patch)
    constexpr int kPer = 4;
    const uint4* tab = m.cell_tab;
    for (int t0 = 0; t0 < ncell; t0 += kPer * kBlock) {
        uint4 v[kPer];
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            const int t = t0 + (int)threadIdx.x + q * kBlock;
            v[q] = make_uint4(0u, 0u, 0u, 0u);
            if (t < ncell) {
                const int r = t / wcols, c = t - r * wcols;
                v[q] = tab[(uint64_t)(wn0 + r) * m.width + (uint64_t)(wm0 + c)];
            }
        }
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            const int t = t0 + (int)threadIdx.x + q * kBlock;
            if (t < ncell) {
                WinCell wc;
                wc.mean0 = __uint_as_float(v[q].x);
                wc.stdev0 = __uint_as_float(v[q].y);
                wc.begin = v[q].z;
                wc.count = v[q].w;
                cells[t] = wc;
            }
        }
    }
    __syncthreads();
    w.on = 1;
    w.cells = cells;
    return w;
}

// ---------------------------------------------------------------------------------------
// ContactModel::evaluatePose + evaluateWeight  (src/ContactModel.cpp:117-224, 262-317)
// ---------------------------------------------------------------------------------------
struct CMResult {
    uint32_t ncp;
    bool accepted;
    double weight, zdelta, zvar, posevar, s2;
};

// contactLikelihoodRatio(z, sigma) > 1e-9 guaranteed (exact-arithmetic bounds, wide margin),
// sigma^2 = zvar corr^2: a one-point group's ratio cancels ((zdiff*r)/r = zdiff) and is not
// evaluated (same predicate as the oracle)
__device__ __forceinline__ bool ratio_surely_significant(double z, double zvar, double corr)
{
    const double s2 = zvar * (corr * corr);
    if (z <= 0.0) return s2 < 1e16;
    return s2 < 1600.0 && z * z < 31.36 * s2;
}

// MAXP: bound on the contact points found (group ends); BATCH: p.m <= MAXP contacts;
// UNG (with BATCH): every contact closes its group (groupId -1 or a group of one), so the
// group logic reduces to the Q7 poisoning flag and a push per evaluated, found contact.
// StepParams (p.*) and the contacts come from scalar loads of the kernel arguments.
// lookups in flight per particle in the reduced group logic (BATCH && UNG): all MAXP by
// default; an experiment knob (fewer live registers)
#ifndef ESLAM_K1_LB
#define ESLAM_K1_LB 4
#endif
constexpr int kK1LookupBatch = ESLAM_K1_LB;

template <int MAXP, bool BATCH, bool DELTA = false, bool UNG = false>
__device__ __forceinline__ CMResult evaluate_pose(const Window& win, double co, double s, double r22, double x, double y,
                                                  double z, double meas_var, uint32_t sid)
{
    CMResult r;
    // pushed contact points.  BATCH: slot = index of the contact that closed the group, so
    // every write has a static index; the slots are summed in index order = push order.
    double cz[MAXP], cv[MAXP];
    bool ok[MAXP];
#pragma unroll
    for (int k = 0; k < MAXP; ++k) ok[k] = false;
    uint32_t ncp = 0;
    bool valid = false, group_valid = true;
    double contact_ratio = 0, pose_var_avg = 0, posevar = 0;
    double pzd = 0, pzv = 0;
    const double qv = meas_var;
    const su8 wp = kl8(KOFF(p.me2));          // me2, radius, corr, min_contacts
    const su4 wq = kl4(KOFF(p.use_shape));    // use_shape, m, eval_mask, end_mask
    const double radius = kd(wp, 1), corr = kd(wp, 2);
    const uint32_t m = wq[1], eval_mask = wq[2], end_mask = wq[3];

    auto push = [&](uint32_t i, double zd, double zv) {
        if constexpr (BATCH) {
            cz[i] = zd; cv[i] = zv; ok[i] = true;
        } else {
#pragma unroll
            for (int k = 0; k < MAXP; ++k)
                if ((uint32_t)k == ncp) { cz[k] = zd; cv[k] = zv; }
        }
        ++ncp;
    };
    // the sequential part of one contact (group logic, Q7 poisoning): found/mean/stdev are
    // the map lookup of its world point (used only when the contact is evaluated)
    auto contact = [&](uint32_t i, bool found, double mean, double stdev, double wz) {
        const bool c_eval = (eval_mask >> i) & 1u, c_end = (end_mask >> i) & 1u;
        if (group_valid && c_eval) {
            if (found) {
                const double zdiff = wz - mean;
                const double pose_var = stdev * stdev;
                const double zvar = stdev * stdev + meas_var;
                if (!valid && c_end && ratio_surely_significant(zdiff, zvar, corr)) {
                    // single-point group: (zdiff, zvar) pushed directly
                    posevar += pose_var;
                    push(i, zdiff, zvar);
                    group_valid = true;
                    valid = false;
                    pose_var_avg = 0;
                    contact_ratio = 0;
                    return;
                }
                const double ratio = dm_normal_pdf_cdf_ratio(zdiff, dm_sqrt(zvar) * corr);
                if (!valid) {
                    pzd = zdiff * ratio;
                    pzv = zvar * ratio;
                    contact_ratio = ratio;
                    pose_var_avg = pose_var * ratio;
                } else {
                    pzd += zdiff * ratio;
                    pzv += zvar * ratio;
                    contact_ratio += ratio;
                    pose_var_avg += pose_var * ratio;
                }
                valid = true;
            } else {
                group_valid = false;
            }
        }
        if (valid && c_end) {
            if (group_valid && contact_ratio > 1e-9) {
                const double inv = 1.0 / contact_ratio;
                pzd *= inv;
                pzv *= inv;
                posevar += pose_var_avg * inv;
                push(i, pzd, pzv);
            }
            group_valid = true;
            valid = false;
            pose_var_avg = 0;
            contact_ratio = 0;
        }
    };
    // pose * p with pose = Translation(x, y, z) * AngleAxis(theta, UnitZ); the zero products
    // of the affine multiply are per-step constants, and "- 0.0" is exact
    auto world = [&](uint32_t i, double& wx, double& wy, double& wz) {
        su8 c;
        su2 cpz;
        const uint32_t off = KOFF(p.c) + i * (uint32_t)sizeof(ContactC);
        kl8_2(off, off + (uint32_t)offsetof(ContactC, pz), c, cpz);   // px, py, zp, zz | pz
        const double px = kd(c, 0), py = kd(c, 1), zp = kd(c, 2), zz = kd(c, 3), pz = kd(cpz, 0);
        wx = ((co * px + (-s) * py) + zp) + x;
        wy = ((s * px + co * py) + zp) + y;
        wz = ((zz + r22 * pz) + z) - radius;
    };
    auto lookup = [&](double wx, double wy, double wz, double& mean, double& stdev) -> bool {
        return get_patch<DELTA>(win, wx, wy, wz, qv, mean, stdev, sid);
    };

    if constexpr (BATCH && UNG && kK1LookupBatch < MAXP) {
        // the reduced group logic (below) with kK1LookupBatch lookups in flight at a time
        bool alive = true;
#pragma unroll
        for (int g = 0; g < MAXP; g += kK1LookupBatch) {
            bool fnd[kK1LookupBatch];
            double mn[kK1LookupBatch], sd[kK1LookupBatch], wzs[kK1LookupBatch];
#pragma unroll
            for (int q = 0; q < kK1LookupBatch; ++q) {
                const int i = g + q;
                fnd[q] = false; mn[q] = 0.0; sd[q] = 0.0; wzs[q] = 0.0;
                if ((uint32_t)i < m) {
                    double wx, wy;
                    world((uint32_t)i, wx, wy, wzs[q]);
                    if ((eval_mask >> i) & 1u) fnd[q] = lookup(wx, wy, wzs[q], mn[q], sd[q]);
                }
            }
#pragma unroll
            for (int q = 0; q < kK1LookupBatch; ++q) {
                const int i = g + q;
                if ((uint32_t)i >= m) break;
                if (!((eval_mask >> i) & 1u)) continue;
                if (alive && fnd[q]) {
                    const double zdiff = wzs[q] - mn[q];
                    const double pose_var = sd[q] * sd[q];
                    const double zvar = sd[q] * sd[q] + meas_var;
                    double pzd_i = zdiff, pzv_i = zvar, pv_i = pose_var;
                    bool take = true;
                    if (!ratio_surely_significant(zdiff, zvar, corr)) {
                        const double ratio = dm_normal_pdf_cdf_ratio(zdiff, dm_sqrt(zvar) * corr);
                        take = ratio > 1e-9;
                        const double inv = 1.0 / ratio;
                        pzd_i = (zdiff * ratio) * inv;
                        pzv_i = (zvar * ratio) * inv;
                        pv_i = (pose_var * ratio) * inv;
                    }
                    if (take) {
                        posevar += pv_i;
                        push((uint32_t)i, pzd_i, pzv_i);
                    }
                }
                alive = alive && fnd[q];
            }
        }
    } else if constexpr (BATCH) {
        // all m <= MAXP contacts' lookups first: independent, so their memory latencies
        // overlap (a lookup the group logic then skips is harmless: pure function)
        bool fnd[MAXP];
        double mn[MAXP], sd[MAXP], wzs[MAXP];
        if constexpr (DELTA) {
            if (!(sid >> 31)) {
                // the feet the shared grid leaves to the particle's map: their lookups together
                uint32_t dm[MAXP], dn[MAXP];
                double dlz[MAXP];
#pragma unroll
                for (int i = 0; i < MAXP; ++i) {
                    fnd[i] = false; mn[i] = 0.0; sd[i] = 0.0; wzs[i] = 0.0; dm[i] = 0xffffffffu; dn[i] = 0u; dlz[i] = 0.0;
                    if ((uint32_t)i < m) {
                        double wx, wy;
                        world((uint32_t)i, wx, wy, wzs[i]);
                        if ((eval_mask >> i) & 1u)
                            fnd[i] = get_patch<true, true>(win, wx, wy, wzs[i], qv, mn[i], sd[i], sid, &dm[i], &dn[i], &dlz[i]);
                    }
                }
                store_patches<MAXP>(sid, dm, dn, dlz, qv, fnd, mn, sd);
            } else {
#pragma unroll
                for (int i = 0; i < MAXP; ++i) {
                    fnd[i] = false; mn[i] = 0.0; sd[i] = 0.0; wzs[i] = 0.0;
                    if ((uint32_t)i < m) {
                        double wx, wy;
                        world((uint32_t)i, wx, wy, wzs[i]);
                        if ((eval_mask >> i) & 1u) fnd[i] = lookup(wx, wy, wzs[i], mn[i], sd[i]);
                    }
                }
            }
        } else {
#pragma unroll
            for (int i = 0; i < MAXP; ++i) {
                fnd[i] = false; mn[i] = 0.0; sd[i] = 0.0; wzs[i] = 0.0;
                if ((uint32_t)i < m) {
                    double wx, wy;
                    world((uint32_t)i, wx, wy, wzs[i]);
                    if ((eval_mask >> i) & 1u) fnd[i] = lookup(wx, wy, wzs[i], mn[i], sd[i]);
                }
            }
        }
        if constexpr (UNG) {
            // contact() with c_end set for every contact: `valid` is false at the start of
            // each one, a surely-significant point is pushed as it is, any other one through
            // its ratio (pzd = (zdiff r) (1/r), ...), and a miss clears group_valid for good
            // (Q7: it is only reset under `valid`, which a miss never sets)
            bool alive = true;
#pragma unroll
            for (int i = 0; i < MAXP; ++i) {
                if ((uint32_t)i >= m) break;
                if (!((eval_mask >> i) & 1u)) continue;
                if (alive && fnd[i]) {
                    const double zdiff = wzs[i] - mn[i];
                    const double pose_var = sd[i] * sd[i];
                    const double zvar = sd[i] * sd[i] + meas_var;
                    double pzd_i = zdiff, pzv_i = zvar, pv_i = pose_var;
                    bool take = true;
                    if (!ratio_surely_significant(zdiff, zvar, corr)) {
                        const double ratio = dm_normal_pdf_cdf_ratio(zdiff, dm_sqrt(zvar) * corr);
                        take = ratio > 1e-9;
                        const double inv = 1.0 / ratio;
                        pzd_i = (zdiff * ratio) * inv;
                        pzv_i = (zvar * ratio) * inv;
                        pv_i = (pose_var * ratio) * inv;
                    }
                    if (take) {
                        posevar += pv_i;
                        push((uint32_t)i, pzd_i, pzv_i);
                    }
                }
                alive = alive && fnd[i];
            }
        } else {
#pragma unroll
            for (int i = 0; i < MAXP; ++i) {
                if ((uint32_t)i >= m) break;
                contact((uint32_t)i, fnd[i], mn[i], sd[i], wzs[i]);
            }
        }
    } else {
        for (uint32_t i = 0; i < m; ++i) {
            double wx, wy, wz, mean = 0.0, stdev = 0.0;
            world(i, wx, wy, wz);
            bool found = false;
            if (group_valid && ((eval_mask >> i) & 1u)) found = lookup(wx, wy, wz, mean, stdev);
            contact(i, found, mean, stdev, wz);
        }
    }
    r.ncp = ncp;
    r.posevar = posevar;
    r.accepted = (uint64_t)ncp >= kq(wp, 3);
    r.weight = r.zdelta = r.zvar = r.s2 = 0.0;
    if (r.accepted) {
        // every zvar lies in [meas_var, meas_var + 2^256] (a float stdev squared), and d2 in
        // [2^-301, 4 / meas_var]: for meas_var in [2^-400, 2^300] the reciprocals need none of
        // the division's scaling (dm_div_inrange: the same bits)
        double d1 = 0, d2 = 0, inv_d2;
        auto sums = [&](auto recip) {
#pragma unroll
            for (int k = 0; k < MAXP; ++k) {
                if (BATCH ? ok[k] : (uint32_t)k < ncp) {
                    cv[k] = recip(cv[k]);       // cv now holds 1/zvar
                    d1 += cz[k] * cv[k];
                    d2 += cv[k];
                }
            }
            inv_d2 = recip(d2);
        };
        if (meas_var >= 0x1p-400 && meas_var <= 0x1p300) sums([](double v) { return dm_div_inrange(1.0, v); });
        else sums([](double v) { return 1.0 / v; });
        const double delta = d1 * inv_d2;
        double s2 = 0.0;
#pragma unroll
        for (int k = 0; k < MAXP; ++k) {
            if (BATCH ? ok[k] : (uint32_t)k < ncp) {
                const double d = cz[k] - delta;
                s2 += (d * d) * cv[k];
            }
        }
        r.s2 = s2;
        const uint32_t use_shape = kl2(KOFF(p.use_shape))[0];
        const double pz = use_shape ? dm_exp(-0.5 * s2) : 1.0;
        r.weight = pz;
        r.zdelta = -delta;
        r.zvar = inv_d2;
    }
    return r;
}

// ---------------------------------------------------------------------------------------
// k_project_weight: PoseEstimator::project and/or updateWeights phase A, one particle per
// lane, one canonical chunk (64 lanes x J rows) per wave.
// ---------------------------------------------------------------------------------------
// ---------------------------------------------------------------------------------------
// source of a pending-gather output: expand the segment marks (inclusive max-scan) and
// decode.  Returns the local particle index, or sets *rec for a migrated particle.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t decode_source(uint32_t v, uint32_t multi, const gmem<const Rec>* __restrict__ recs,
                                                  const gmem<const Rec>** rec)
{
    *rec = nullptr;
    if (multi) {
        if (v >= kMarkOwn && v < kMarkHigh) return v - kMarkOwn;
        *rec = recs + (v >= kMarkHigh ? v - kMarkHigh : v);
        return 0;
    }
    return v;
}

// The state written by K1 (and w by K3) is streamed: each value is read once, by the next
// kernel, from another XCD.  Non-temporal stores (nt) leave fewer lines for the kernel-end L2
// writeback (interleaved A/B on MI355X: 256k +3 %, 4M +0.7 %, 16M +1.6 % per step; plain
// stores and agent-coherent sc1 stores measured beside them).  Same values, same bits.
#define K1_ST(p, v) __builtin_nontemporal_store((v), (p))

#ifndef ESLAM_K1D_WPE
#define ESLAM_K1D_WPE 3                  // K1 DELTA: three waves a SIMD hold the batched own-map lookups unspilled
#endif
template <bool PROJECT, bool WEIGHT, int MAXP, bool BATCH, bool DELTA = false, bool UNG = false>
__global__ void __launch_bounds__(kBlock) ESLAM_K1_ATTR __attribute__((amdgpu_waves_per_eu(DELTA ? ESLAM_K1D_WPE : 1))) k_project_weight(K1Args a)
{
    // Inside the particle loop every argument is read by a scalar load where it is used
    // (KOFF offsets into the K1Args kernel argument); "a." appears only outside the loop.
    ESLAM_STAMP(g_stamps_k1, 0);
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint64_t n = a.p.n;
    const uint32_t J = a.p.J;
    const uint64_t csz = 64ull * J;
    const uint64_t nchunks = (n + csz - 1) / csz;
    Ctl* ctl = a.ctl;
    if (ctl->err & kFaultTimeout) return;    // poisoned filter (a wait gave up): nothing is touched
    // a pending resample gather is fused here: read the ancestors from state[base],
    // write the updated particles to state[base ^ 1] (the latest buffer)
    const uint32_t gath = ctl->gather;
    const uint32_t cur = ctl->base ^ ctl->flip;
    if (WEIGHT && blockIdx.x == 0 && threadIdx.x == 0) ctl->k3_base = cur;
    const uint32_t st_off = __builtin_amdgcn_readfirstlane(cur ? KOFF(s[1]) : KOFF(s[0]));
    const uint32_t si_off = __builtin_amdgcn_readfirstlane(gath ? (ctl->base ? KOFF(s[1]) : KOFF(s[0])) : st_off);
    const int wexp = ctl->wexp;
    double spread = 0.0;
    bool do_spread = false;
    double tf = 0.0, rf = 0.0;
    if (PROJECT) {
        spread = dm_weighting_function(ctl->max_weight, 0.0, a.p.spread_threshold, 0.0);
        do_spread = spread > 0 && !a.p.hash_use;
        tf = a.p.spread_trans * spread;
        rf = a.p.spread_rot * spread;
    }

    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    Window win;
    win.on = 0;
    if (WEIGHT) win = stage_window(a.map, a.p, ctl, 6.0 * tf, smem + kStatsLds);
    ESLAM_STAMP(g_stamps_k1, 1);

    // order-free per-lane state, kept across chunks
    double maxm = 0.0;
    // data particles | total points << 16 per lane (nD <= J, nTP <= ESLAM_MAX_CONTACTS J);
    // werr: some particle of the wave hit a zero measurement variance (wave-uniform)
    uint32_t nDTP = 0, werr = 0, flag = 0;
    uint32_t touched = 0;                // bit b: the wave walked bucket b (wave-uniform)
    // -min x, max x, -min y, max y of the cloud, rounded to float (the window only needs a
    // box that holds the cloud; it is widened by the float rounding in bbox_keys)
    float bb[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    uint64_t limb = 0;                  // lane t < 52: column t & 3 of exact accumulator t >> 2
    const int sa = DM_FX_SCALE - wexp, sb = DM_FX_SCALE - 2 * wexp;

    // one canonical chunk (64 x J particles) per wave; its totals go to exact fixed point.
    // A sharded step may split the launch (ChunkSel): the chunks of the rank's own outputs
    // first, the chunks that need exchanged records after the exchange (exact sums: the
    // statistics do not depend on the order in which chunks are processed)
    uint64_t chunk = (uint64_t)blockIdx.x * kWaves + wave;
    bool active = chunk < nchunks;
    if (a.sel.mode == 1u) {
        active = chunk >= a.sel.cdev[0] && chunk < a.sel.cdev[1];
    } else if (a.sel.mode == 2u) {
        chunk = chunk < a.sel.c_lo ? chunk : a.sel.c_hi + (chunk - a.sel.c_lo);
        active = chunk < nchunks;
    }
    if (active) {
    const uint64_t lbase = chunk * csz;
    // the per-bucket sums A_b, B_b of the sum contract: the pair of the bucket the wave is in
    // (cur_b; usually the chunk's only one) in registers, the others parked per lane in the
    // chunk's slot of K1Args::bspill and reloaded when the wave returns to them.  Each lane's
    // sum of bucket b sees the same additions in the same order as with a register per bucket.
    constexpr uint32_t kNoBucket = 0xffu;
    double curA = 0.0, curB = 0.0;
    uint32_t cur_b = kNoBucket;
    // DELTA (per-particle maps): a wave's particles find different numbers of contact points
    // (cells only their stores hold), so its rows span several buckets and parking pairs in
    // bspill costs a store and a load per switch (K1 DELTA 0.45 -> 0.51 ms at 8M, r04h).  Its
    // kernel runs at four waves per SIMD anyway: every bucket's pair stays in registers.
    constexpr bool kRegAcc = DELTA;
    double accA[kRegAcc ? DM_NBUCKETS : 1], accB[kRegAcc ? DM_NBUCKETS : 1];
#pragma unroll
    for (int k = 0; k < (kRegAcc ? DM_NBUCKETS : 1); ++k) accA[k] = accB[k] = 0.0;
    double accSW = 0.0;

    for (uint32_t j = 0; j < J; ++j) {
        const uint64_t row0 = lbase + 64ull * j;
        if (row0 >= n) break;
        const uint64_t i = row0 + lane;
        uint32_t src = (uint32_t)i;
        const gmem<const Rec>* rc = nullptr;
        uint32_t rec_anc = 0;
        bool clr = false;                        // this output's segment mark is set
        if (gath) {
            const su8 g = kl8(KOFF(gv));              // marks, row_first, anc, recs
            const su2 gf = kl2(KOFF(gv.record));      // record, multi
            gmem<uint32_t>* marks = kp<uint32_t>(g, 0);
            // expand the segment marks of this row: inclusive max-scan + the row carry.  Both
            // loads are issued together; the mark is cleared with the row's other stores at its
            // end (vmcnt counts stores too: a store here would add its round trip to the wait
            // before the state loads)
            const uint32_t carry = kp<const uint32_t>(g, 1)[row0 / kRow] + 1u;
            uint32_t m = 0;
            if (i < n) { m = marks[i]; clr = m != 0; }
            m = wave_incl_max_u32(m);
            m = m > carry ? m : carry;
            src = decode_source(m - 1u, gf[1], kp<const Rec>(g, 3), &rc);
            rec_anc = gf[0];
        }
        // lanes past n (only in the last row of the last chunk) compute nothing but take part
        // in the row's bucket walk, so the walk's state stays wave-uniform (scalar)
        uint32_t bucket = kNoBucket;
        double am = 0.0, am2 = 0.0;
        bool rowerr = false;
        if (i < n) {
        double x, y, th, z, zs, w, mp_in = 0.0;
        uint32_t fl_in = 0;
        if (rc) {
            x = rc->x; y = rc->y; th = rc->th; z = rc->z; zs = rc->zs; w = rc->w;
            mp_in = rc->mprob; fl_in = (uint8_t)rc->src;
        } else {
            const StatePtrs si = kstate(si_off);
            x = si.x[src]; y = si.y[src]; th = si.th[src]; z = si.z[src];
            zs = si.zs[src]; w = si.w[src];
            if (!WEIGHT && gath) { mp_in = si.mprob[src]; fl_in = si.flags[src]; }
        }
        if (gath && rec_anc) {
            const su2 ga = kl2(KOFF(gv.anc));
            const uint64_t gbase = kq(kl2(KOFF(p.gbase)), 0);
            kp<uint32_t>(ga, 0)[i] = rc ? (uint32_t)(rc->src >> 8) : (uint32_t)(gbase + src);
        }
        const double w_in = w;
        double mprob = 0.0;
        uint32_t flags = 0;
        if (PROJECT) {
            const su8 key = kl8(KOFF(p.seed));       // seed, proj_event, gbase
            const uint64_t gi = kq(key, 2) + i;
            // draw layout: call 0 -> two Box-Muller pairs (z0, z1), (z2, sn0);
            // call 1 -> slip test + slip factor, spread pair (sn1, sn2)
            const dm_philox_ctr d0 = dm_draw(kq(key, 0), DM_STREAM_PROJECT, kq(key, 1), gi, 0);
            const dm_philox_ctr d1 = dm_draw(kq(key, 0), DM_STREAM_PROJECT, kq(key, 1), gi, 1);
            double z0, z1, z2, sn0;
            dm_box_muller32(d0.v[0], d0.v[1], &z0, &z1);
            dm_box_muller32(d0.v[2], d0.v[3], &z2, &sn0);
            // odometry.getPoseDeltaSample2D() = mu + L z
            const su16 P = kl16(KOFF(p.mu));         // mu0 mu1 mu2 L00 L10 L11 L20 L21
            const su8 Q = kl8(KOFF(p.L22));          // L22 slip_factor yaw max_yaw_dev
            const double dx = kd(P, 0) + kd(P, 3) * z0;
            double dy = kd(P, 1) + (kd(P, 4) * z0 + kd(P, 5) * z1);
            const double dth = kd(P, 2) + ((kd(P, 6) * z0 + kd(P, 7) * z1) + kd(Q, 0) * z2);
            if (dm_u32(d1.v[0]) < kd(Q, 1)) dy *= dm_u32(d1.v[1]);
            double s, co;
            dm_sincos(th, &s, &co);
            x += co * dx - s * dy;
            y += s * dx + co * dy;
            th += dth;
            if (kd(Q, 3) > 0.0) {
                if (dm_fabs(th - kd(Q, 2)) > kd(Q, 3)) w *= 0.7;
            }
            const su4 Z = kl4(KOFF(p.z_delta));      // z_delta z_var
            z += kd(Z, 0);
            zs = dm_sqrt_fast(zs * zs + kd(Z, 1));
            if (do_spread) {
                double sn1, sn2;
                dm_box_muller32(d1.v[2], d1.v[3], &sn1, &sn2);
                x += sn0 * tf + 0.0;
                y += sn1 * tf + 0.0;
                th += sn2 * rf + 0.0;
            }
        }
        if (WEIGHT) {
            double s, co;
            dm_sincos(th, &s, &co);
            const double r22 = (1.0 - co) + co;
            const double meas_var = zs * zs + kd(kl2(KOFF(p.me2)), 0);
            uint32_t sid = 0;
            if constexpr (DELTA) {
                // per-particle maps: the host materialises every gather first, so particle i
                // is at i; its store name sits next to the state (DevState::sid)
                sid = store_sid(kp<const uint32_t>(kl2(st_off + (uint32_t)offsetof(DevState, sid)), 0)[i]);
            }
            CMResult r = evaluate_pose<MAXP, BATCH, DELTA, UNG>(win, co, s, r22, x, y, z, meas_var, sid);
            if (meas_var == 0) {            // evaluatePose throws (src/ContactModel.cpp:122): no contact points
                rowerr = true;
                r.accepted = false;
                r.ncp = 0;
            }
            uint32_t floating;
            double sw = 0.0;
            if (r.accepted) {
                // ContactModel::updateZPositionEstimate  src/ContactModel.cpp:319-340
                double zvar = zs * zs;
                // posevar / found: a power-of-two count divides exactly as a multiplication by
                // its reciprocal (the same correctly rounded quotient)
                const double inv_n = dm_recip_small(r.ncp);     // 1.0 / found, correctly rounded
                double pose_var;
                if (r.ncp != 0u && (r.ncp & (r.ncp - 1u)) == 0u) pose_var = r.posevar * inv_n;
                else pose_var = r.posevar / (double)r.ncp;
                const double av = zvar - pose_var;
                double delta_var = (av < 1e-9) ? 1e-9 : av;
                if (!(r.zdelta * r.zdelta > delta_var)) {
                    const double gain = zvar / (zvar + r.zvar);
                    z += gain * r.zdelta;
                    const double var_gain = delta_var / (delta_var + r.zvar);
                    delta_var = (1.0 - var_gain) * delta_var;
                    zvar = pose_var + delta_var;
                }
                zs = dm_sqrt_fast(zvar);
                w *= r.weight;
                mprob = r.weight;
                floating = 0;
                maxm = (maxm < r.weight) ? r.weight : maxm;
                nDTP += 1u + (r.ncp << 16);
                // pow(weight, 1.0/found) with weight = exp(-s2/2): exp(-s2/2 * (1/found))
                const uint32_t use_shape = kl2(KOFF(p.use_shape))[0];
                if (!use_shape || r.ncp == 0) sw = dm_pow(r.weight, inv_n);
                else sw = r.weight == 0.0 ? 0.0 : dm_exp((-0.5 * r.s2) * inv_n);
            } else {
                floating = 1;
                mprob = 1.0;
            }
            bucket = r.ncp < DM_NBUCKETS - 1 ? r.ncp : DM_NBUCKETS - 1;
            am = w * mprob;
            am2 = am * am;
            accSW = accSW + sw;
            flags = (r.ncp & 0x7fu) | (floating << 7);
        } else {
            mprob = mp_in;
            flags = fl_in;
        }
        // all stores of the row at the end: one scalar load of the output pointers
        const StatePtrs st = kstate(st_off);
        if (PROJECT || gath) {
            K1_ST(st.x + i, x);
            K1_ST(st.y + i, y);
            K1_ST(st.th + i, th);
        }
        if (WEIGHT || gath) {
            K1_ST(st.mprob + i, mprob);
            K1_ST(st.flags + i, (uint8_t)flags);
        }
        if (PROJECT || WEIGHT) {
            K1_ST(st.z + i, z);
            K1_ST(st.zs + i, zs);
            if (gath || w != w_in || w != w) K1_ST(st.w + i, w);
        }
        if (clr) kp<uint32_t>(kl2(KOFF(gv.marks)), 0)[i] = 0;
        {
            // v_max_f32 returns the other operand for a NaN: NaN coordinates are skipped
            const float xf = (float)x, yf = (float)y;
            bb[0] = __builtin_fmaxf(bb[0], -xf);
            bb[1] = __builtin_fmaxf(bb[1], xf);
            bb[2] = __builtin_fmaxf(bb[2], -yf);
            bb[3] = __builtin_fmaxf(bb[3], yf);
        }
        }
        if (WEIGHT) {
            // per bucket b the lane adds am if it holds b, else +0.0 (the oracle's canonical
            // per-bucket sums add +0.0 for the other buckets' particles: the same bits).  The
            // wave walks its distinct buckets (usually one): each pass adds to one bucket's two
            // sums, chosen by a scalar branch, instead of selecting over every bucket per lane.
            // ncp <= MAXP: the buckets above MAXP stay empty.  The whole wave walks (lanes
            // without a particle add +0.0), so cur_b and touched are scalars.
            werr |= __ballot(rowerr) != 0ull ? 1u : 0u;
            uint64_t todo = __ballot(bucket != kNoBucket);
            while (todo) {
                const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)bucket, (int)__builtin_ctzll(todo));
                const bool mine = bucket == b0;
                if constexpr (kRegAcc) {
                    touched |= 1u << b0;
#pragma unroll
                    for (uint32_t k = 0; k < (uint32_t)DM_NBUCKETS; ++k) {
                        if (k == b0) {                   // scalar branch (b0 is wave-uniform)
                            accA[k] = accA[k] + (mine ? am : 0.0);
                            accB[k] = accB[k] + (mine ? am2 : 0.0);
                        }
                    }
                    todo &= ~__ballot(mine);
                    continue;
                }
                if (b0 != cur_b) {
                    // the wave moves to another bucket: park the current pair, take b0's (a
                    // bucket the wave never walked starts at +0.0)
                    gmem<double>* sp = kp<double>(kl2(KOFF(bspill)), 0) + chunk * (DM_NBUCKETS * 128) + lane;
                    if (cur_b != kNoBucket) {
                        sp[cur_b * 128] = curA;
                        sp[cur_b * 128 + 64] = curB;
                    }
                    curA = curB = 0.0;
                    if ((touched >> b0) & 1u) {
                        curA = sp[b0 * 128];
                        curB = sp[b0 * 128 + 64];
                    }
                    cur_b = b0;
                }
                touched |= 1u << b0;
                curA = curA + (mine ? am : 0.0);
                curB = curB + (mine ? am2 : 0.0);
                todo &= ~__ballot(mine);
            }
        }
    }

    if (WEIGHT) {
        // chunk totals (sub-lane sums + the xor butterfly of the sum contract) -> exact fixed
        // point -> lane columns.  The butterfly runs transposed over the 2 * NB + 1 totals
        // (padded to 16): at distances 32, 16, 8 and 4 each lane pair splits the totals it
        // holds in halves and adds the half it keeps, so total q ends in lanes 4q..4q+3 after
        // the same pairwise additions as its own butterfly (the same bits); distances 2 and 1
        // finish it there, and each lane converts its total once and keeps limb lane & 3.
        constexpr int kQ = 2 * DM_NBUCKETS + 1;
        static_assert(kQ <= 16, "16 totals over the 64 lanes");
        const uint32_t q = lane >> 2;
        double t;
        // `touched` is only updated by the lanes active in a walk: lanes past n in the last row
        // keep an older set.  Lane 0 takes part in every walk (a row runs only if row0 < n), so
        // its set is complete, and read as a scalar the branch below is wave-uniform.
        const uint32_t touched0 = touched;
        if (__builtin_popcount(touched0) <= 1) {
            // the usual wave: every row's particles in one bucket b0, so the totals of the
            // other buckets are +0.0 (nothing was added to them) and the register pair holds
            // the sums of b0.  The
            // butterfly runs over A_b0, B_b0 and SW only (transposed at distances 32 and 16:
            // total k ends in lanes 16k..16k+15), the same pairwise additions, and lane 4q + c
            // picks total q.
            const uint32_t b0 = touched0 ? (uint32_t)__builtin_ctz(touched0) : 0u;
            if constexpr (kRegAcc) {
#pragma unroll
                for (uint32_t k = 0; k < (uint32_t)DM_NBUCKETS; ++k)
                    if (k == b0) { curA = accA[k]; curB = accB[k]; }
            }
            double w4[4] = {curA, curB, accSW, 0.0};
            transpose_add<32, 2>(w4, lane);
            transpose_add<16, 1>(w4, lane);
            double u = w4[0];
            u = u + xor_lane<8>(u);
            u = u + xor_lane<4>(u);
            u = u + xor_lane<2>(u);
            u = u + xor_lane<1>(u);
            auto lane_value = [](double x, int l) {      // v_readlane of both halves
                const uint64_t b = dm_bits(x);
                const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
                const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
                return dm_from_bits(((uint64_t)hi << 32) | lo);
            };
            const double tA = lane_value(u, 0), tB = lane_value(u, 16), tS = lane_value(u, 32);
            t = q == b0 ? tA : (q == DM_NBUCKETS + b0 ? tB : (q == kQ - 1 ? tS : 0.0));
        } else {
            // several buckets: the sums of bucket k are the register pair (k == cur_b), the
            // parked pair (a bucket the wave left), or +0.0 (a bucket it never walked)
            const gmem<const double>* sp = kp<const double>(kl2(KOFF(bspill)), 0) + chunk * (DM_NBUCKETS * 128) + lane;
            double v[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                v[k] = k == kQ - 1 ? accSW : 0.0;
                if (k < 2 * DM_NBUCKETS) {
                    const uint32_t b = (uint32_t)(k < DM_NBUCKETS ? k : k - DM_NBUCKETS);
                    if constexpr (kRegAcc) v[k] = k < DM_NBUCKETS ? accA[b] : accB[b];
                    else if (b == cur_b) v[k] = k < DM_NBUCKETS ? curA : curB;
                    else if ((touched >> b) & 1u) v[k] = sp[b * 128 + (k < DM_NBUCKETS ? 0 : 64)];
                }
            }
            transpose_add<32, 8>(v, lane);
            transpose_add<16, 4>(v, lane);
            transpose_add<8, 2>(v, lane);
            transpose_add<4, 1>(v, lane);
            t = v[0];
            t = t + xor_lane<2>(t);
            t = t + xor_lane<1>(t);
        }
        const int scale = q < DM_NBUCKETS ? sa : (q < 2 * DM_NBUCKETS ? sb : DM_FX_SCALE);
        const bool nan_ = t != t, inf_ = !nan_ && !dm_isfinite(t);
        uint32_t l[4] = {0, 0, 0, 0};
        if (!nan_ && !inf_) dm_fx128_limbs(t, scale, l);          // padding totals are 0: limbs 0
        const uint32_t c = lane & 3u;
        limb += c == 0 ? l[0] : (c == 1 ? l[1] : (c == 2 ? l[2] : l[3]));
        const uint64_t mn = __ballot(nan_), mi = __ballot(inf_);
#pragma unroll
        for (int k = 0; k < kQ; ++k) {
            if ((mn >> (4 * k)) & 1ull) flag |= 1u << k;
            if ((mi >> (4 * k)) & 1ull) flag |= 1u << (k + 16);
        }
    }
    }

    ESLAM_STAMP(g_stamps_k1, 2);
    Shard* shb = a.shards + (blockIdx.x % kNShard);
    // bounding box of the cloud for the next step's LDS window (maxima, any order): the four
    // maxima in one transposed butterfly (at distances 32 and 16 each lane pair keeps half of
    // them), so value q ends in lanes 16q..16q+15 and lane 16q publishes it
    {
        transpose_op<32, 2>(bb, lane, [](float a, float b) { return __builtin_fmaxf(a, b); });
        transpose_op<16, 1>(bb, lane, [](float a, float b) { return __builtin_fmaxf(a, b); });
        float m = bb[0];
        m = __builtin_fmaxf(m, xor_lane<8>(m));
        m = __builtin_fmaxf(m, xor_lane<4>(m));
        m = __builtin_fmaxf(m, xor_lane<2>(m));
        m = __builtin_fmaxf(m, xor_lane<1>(m));
        const float xmax = __uint_as_float((uint32_t)__builtin_amdgcn_readlane((int)__float_as_uint(m), 16));
        if ((lane & 15u) == 0u && xmax > -INFINITY) {
            const uint32_t q = lane >> 4;
            // |x - (float)x| <= 2^-24 |x| + 2^-150: widen outward, then the order key
            const double v = (double)m;
            const double wv = v + (dm_fabs(v) * 0x1p-22 + 0x1p-140);
            const uint64_t k = order_key((q & 1u) ? wv : -wv);
            atomicMax((unsigned long long*)&shb->bbox[q], (unsigned long long)((q & 1u) ? k : ~k));
        }
    }

    if (!WEIGHT) return;

    // ---- exact statistics: wave columns -> block (LDS) -> sharded atomics ----
    struct StatsLds {
        uint64_t limb[kWaves][(2 * DM_NBUCKETS + 1) * 4];
        uint32_t flag[kWaves];
        uint32_t cnt[kWaves][2];
        double mx[kWaves];
    };
    static_assert(sizeof(StatsLds) <= kStatsLds, "stats scratch");
    StatsLds& sl = *reinterpret_cast<StatsLds*>(smem);
    const double wmax = wave_max_butterfly(maxm);
    // the two counts in one sum: nD <= 64 J and nTP <= ESLAM_MAX_CONTACTS nD per wave (16 bits each)
    static_assert(64u * ESLAM_CHUNK_CAP * ESLAM_MAX_CONTACTS < 65536u, "packed wave counts");
    const uint32_t wDTP = wave_sum_u32(nDTP);
    const uint32_t wD = wDTP & 0xffffu, wTP = wDTP >> 16;
    if (lane < (2 * DM_NBUCKETS + 1) * 4) sl.limb[wave][lane] = limb;
    if (lane == 0) {
        sl.flag[wave] = flag | (werr << 31);
        sl.cnt[wave][0] = wD;
        sl.cnt[wave][1] = wTP;
        sl.mx[wave] = wmax;
    }
    __syncthreads();
    Shard* sh = shb;
    const int t = threadIdx.x;
    if (t < (2 * DM_NBUCKETS + 1) * 4) {
        const int q = t >> 2, j = t & 3;
        uint64_t v = 0;
#pragma unroll
        for (int wv = 0; wv < kWaves; ++wv) v += sl.limb[wv][t];
        if (v) {
            uint64_t* dst = q < DM_NBUCKETS ? &sh->A[q][j] : (q < 2 * DM_NBUCKETS ? &sh->B[q - DM_NBUCKETS][j] : &sh->SW[j]);
            atomicAdd((unsigned long long*)dst, (unsigned long long)v);
        }
    } else if (t == 64) {
        uint64_t d = 0, tp = 0;
        uint32_t f = 0;
        double mx = 0.0;
        for (int wv = 0; wv < kWaves; ++wv) {
            d += sl.cnt[wv][0];
            tp += sl.cnt[wv][1];
            f |= sl.flag[wv];
            mx = (mx < sl.mx[wv]) ? sl.mx[wv] : mx;
        }
        if (d) atomicAdd((unsigned long long*)&sh->D, (unsigned long long)d);
        if (tp) atomicAdd((unsigned long long*)&sh->TP, (unsigned long long)tp);
        if (mx > 0.0) atomicMax((unsigned long long*)&sh->maxm, (unsigned long long)dm_bits(mx));
        if (f & 0x7fffffffu) atomicOr((unsigned long long*)&sh->flags, (unsigned long long)(f & 0x7fffffffu));
        if (f >> 31) atomicOr((unsigned long long*)&sh->err, 1ull);
    }
    ESLAM_STAMP(g_stamps_k1, 3);
}

// ---------------------------------------------------------------------------------------
// k_contact_records (Configuration::logDebug / ESLAM_FLAG_RECORD_CONTACTS): the debug fields
// updateWeights stores in every PoseParticle (src/PoseEstimator.cpp:285-287, 322-325):
// meas_pos, meas_theta and cpoints.  Runs on the projected state between a project-only and
// a weight-only k_project_weight, so the weighting sees exactly the state these records
// describe.  ContactModel::evaluatePose (src/ContactModel.cpp:117-224) evaluated in contact
// order with the same arithmetic as evaluate_pose (the same pushes, bit for bit), recording
// each pushed ContactPoint: the surface point of the group's first valid contact (world x,
// y and the patch mean, :163-171), zdiff, zvar and prob = 1 (Q8).  One particle per thread,
// map lookups through the global CSR (the same values as the LDS window).
// ---------------------------------------------------------------------------------------
template <bool DELTA>
__global__ void __launch_bounds__(kBlock) k_contact_records(K1Args a, DebugRec d)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    if (threadIdx.x < 8) k1_win[threadIdx.x] = 0;          // no LDS window: get_patch reads k1_win
    __syncthreads();
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= a.p.n) return;
    const Ctl* ctl = a.ctl;
    const DevState& st = (ctl->base ^ ctl->flip) ? a.s[1] : a.s[0];
    const double x = st.x[i], y = st.y[i], th = st.th[i], z = st.z[i], zs = st.zs[i];
    Window win;
    win.on = 0;
    win.cells = reinterpret_cast<const WinCell*>(smem);
    double s, co;
    dm_sincos(th, &s, &co);
    const double r22 = (1.0 - co) + co;
    const double meas_var = zs * zs + a.p.me2;
    d.meas[4 * i + 0] = x;
    d.meas[4 * i + 1] = y;
    d.meas[4 * i + 2] = z;
    d.meas[4 * i + 3] = th;
    uint32_t ncp = 0;
    if (meas_var != 0) {
        bool valid = false, group_valid = true;
        double contact_ratio = 0, pzd = 0, pzv = 0, gx = 0, gy = 0, gm = 0;
        const double corr = a.p.corr;
        double* cp = d.cp + (uint64_t)6 * d.maxc * i;
        auto push = [&](double px, double py, double pm, double zd, double zv) {
            if (ncp < d.maxc) {
                double* r = cp + 6 * ncp;
                r[0] = px; r[1] = py; r[2] = pm; r[3] = zd; r[4] = zv; r[5] = 1.0;
            }
            ++ncp;
        };
        for (uint32_t k = 0; k < a.p.m; ++k) {
            const ContactC& c = a.p.c[k];
            const bool c_eval = (a.p.eval_mask >> k) & 1u, c_end = (a.p.end_mask >> k) & 1u;
            const double wx = ((co * c.px + (-s) * c.py) + c.zp) + x;
            const double wy = ((s * c.px + co * c.py) + c.zp) + y;
            const double wz = ((c.zz + r22 * c.pz) + z) - a.p.radius;
            if (group_valid && c_eval) {
                double mean = 0.0, stdev = 0.0;
                if (get_patch<DELTA>(win, wx, wy, wz, meas_var, mean, stdev, DELTA ? store_sid(st.sid[i]) : 0u)) {
                    const double zdiff = wz - mean;
                    const double zvar = stdev * stdev + meas_var;
                    if (!valid && c_end && ratio_surely_significant(zdiff, zvar, corr)) {
                        push(wx, wy, mean, zdiff, zvar);       // single-point group
                        continue;
                    }
                    const double ratio = dm_normal_pdf_cdf_ratio(zdiff, dm_sqrt(zvar) * corr);
                    if (!valid) {
                        pzd = zdiff * ratio; pzv = zvar * ratio; contact_ratio = ratio;
                        gx = wx; gy = wy; gm = mean;
                    } else {
                        pzd += zdiff * ratio; pzv += zvar * ratio; contact_ratio += ratio;
                    }
                    valid = true;
                } else {
                    group_valid = false;
                }
            }
            if (valid && c_end) {
                if (group_valid && contact_ratio > 1e-9) {
                    const double inv = 1.0 / contact_ratio;
                    push(gx, gy, gm, pzd * inv, pzv * inv);
                }
                group_valid = true;
                valid = false;
                contact_ratio = 0;
            }
        }
    }
    d.ncp[i] = (uint8_t)(ncp < 255u ? ncp : 255u);
}

// eslam_gpu_download_records: particles first + k * stride as PoseParticle records with their
// debug fields.  Particle i's records are those of the particle it descends from at the last
// update's resample (anc, global indices) -- the reference copies cpoints with the particle.
// On a sharded filter the host resolves the descent first (slot[k]: the record's position on
// this rank, or kRecRemote | its item in `remote`, fetched from the rank that held it).
constexpr uint64_t kRecRemote = 1ull << 63;
__device__ __forceinline__ uint32_t rec_items(uint32_t maxc) { return 5u + 6u * maxc; }    // doubles per item

__global__ void __launch_bounds__(kBlock) k_pack_records(DevState s0, DevState s1, const Ctl* __restrict__ ctl, uint64_t first,
                                                         uint64_t stride, uint64_t count, uint64_t gbase,
                                                         const uint32_t* __restrict__ anc, DebugRec d,
                                                         eslam_particle_record* __restrict__ out,
                                                         eslam_cpoint* __restrict__ cps, uint32_t max_cp,
                                                         const uint64_t* __restrict__ slot, const double* __restrict__ remote)
{
    const uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= count) return;
    const uint64_t i = first + k * stride;
    const DevState& st = (ctl->base ^ ctl->flip) ? s1 : s0;
    eslam_particle_record r;
    r.position[0] = st.x[i];
    r.position[1] = st.y[i];
    r.orientation = st.th[i];
    r.zpos = st.z[i];
    r.zsigma = st.zs[i];
    r.mprob = st.mprob[i];
    r.weight = st.w[i];
    const uint8_t fl = st.flags[i];
    r.floating = fl >> 7;
    r.index = i + gbase;
    uint32_t n = 0;
    if (d.ncp) {
        const uint64_t s = slot ? slot[k] : (*d.resampled ? (uint64_t)anc[i] - gbase : i);
        const double *meas, *cp;
        if (s & kRecRemote) {                 // an item fetched from another rank
            const double* item = remote + (uint64_t)rec_items(d.maxc) * (s & ~kRecRemote);
            meas = item;
            n = (uint32_t)item[4];
            cp = item + 5;
        } else {
            meas = d.meas + 4 * s;
            n = d.ncp[s];
            cp = d.cp + (uint64_t)6 * d.maxc * s;
        }
        for (int q = 0; q < 3; ++q) r.meas_pos[q] = meas[q];
        r.meas_theta = meas[3];
        const uint32_t kept = n < d.maxc ? n : d.maxc;
        for (uint32_t q = 0; q < kept && q < max_cp; ++q) {
            const double* c = cp + 6 * q;
            eslam_cpoint& o = cps[(uint64_t)max_cp * k + q];
            o.point[0] = c[0]; o.point[1] = c[1]; o.point[2] = c[2];
            o.zdiff = c[3]; o.zvar = c[4]; o.prob = c[5];
        }
    } else {
        r.meas_pos[0] = r.meas_pos[1] = r.meas_pos[2] = 0.0;
        r.meas_theta = 0.0;
        n = fl & 0x7fu;
    }
    r.n_cpoints = n;
    out[k] = r;
}

// the records other ranks asked for (sharded download_records): item j = the debug fields
// of this rank's particle at global index req[j] during the last update (meas 4, ncp, cps)
__global__ void __launch_bounds__(kBlock) k_gather_records(const uint32_t* __restrict__ req, uint64_t nreq, uint64_t gbase,
                                                           DebugRec d, double* __restrict__ items)
{
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= nreq) return;
    const uint64_t s = (uint64_t)req[j] - gbase;
    double* o = items + (uint64_t)rec_items(d.maxc) * j;
    for (int q = 0; q < 4; ++q) o[q] = d.meas[4 * s + q];
    o[4] = (double)d.ncp[s];
    const double* c = d.cp + (uint64_t)6 * d.maxc * s;
    for (uint32_t q = 0; q < 6 * d.maxc; ++q) o[5 + q] = c[q];
}

// exclusive prefix sum of m counts in place, one block: chunks of 8192 counts are loaded and
// stored striped (coalesced, every load of a chunk in flight together) through LDS, where each
// thread scans 8 consecutive counts; the wave scans and a carry join the threads and chunks.
// (A thread per contiguous segment of m / 1024 counts read and wrote them one dependent load
// at a time: 73 us per call at 8M particles' 32k block sums.)
constexpr uint32_t kScanPer = 8, kScanChunk = 1024 * kScanPer;
__global__ void __launch_bounds__(1024) k_scan_excl(uint32_t* __restrict__ a, uint64_t m)
{
    __shared__ __attribute__((aligned(16))) uint32_t s_v[kScanChunk];
    __shared__ uint32_t s_w[16];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    uint32_t carry = 0;
    for (uint64_t base = 0; base < m; base += kScanChunk) {
        const uint32_t cnt = m - base < kScanChunk ? (uint32_t)(m - base) : kScanChunk;
        uint32_t v[kScanPer];
#pragma unroll
        for (uint32_t q = 0; q < kScanPer; ++q) {
            const uint32_t k = q * 1024u + tid;
            v[q] = k < cnt ? a[base + k] : 0u;
        }
#pragma unroll
        for (uint32_t q = 0; q < kScanPer; ++q) s_v[q * 1024u + tid] = v[q];
        __syncthreads();
        const uint4 lo = reinterpret_cast<const uint4*>(s_v)[2 * tid], hi = reinterpret_cast<const uint4*>(s_v)[2 * tid + 1];
        const uint32_t u[kScanPer] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        uint32_t tot = 0;
#pragma unroll
        for (uint32_t q = 0; q < kScanPer; ++q) tot += u[q];
        uint32_t incl = tot;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t x = (uint32_t)__shfl_up((int)incl, o, 64);
            incl += lane >= (uint32_t)o ? x : 0u;
        }
        if (lane == 63) s_w[wave] = incl;
        __syncthreads();
        uint32_t before = 0, all = 0;
#pragma unroll
        for (uint32_t w = 0; w < 16; ++w) {
            before += w < wave ? s_w[w] : 0u;
            all += s_w[w];
        }
        uint32_t run = carry + before + (incl - tot);
        uint32_t r[kScanPer];
#pragma unroll
        for (uint32_t q = 0; q < kScanPer; ++q) { r[q] = run; run += u[q]; }
        reinterpret_cast<uint4*>(s_v)[2 * tid] = make_uint4(r[0], r[1], r[2], r[3]);
        reinterpret_cast<uint4*>(s_v)[2 * tid + 1] = make_uint4(r[4], r[5], r[6], r[7]);
        carry += all;
        __syncthreads();
#pragma unroll
        for (uint32_t q = 0; q < kScanPer; ++q) {
            const uint32_t k = q * 1024u + tid;
            if (k < cnt) a[base + k] = s_v[k];
        }
        __syncthreads();                 // s_v and s_w are reused by the next chunk
    }
}

// ---------------------------------------------------------------------------------------
// Per-particle local maps (useSharedMap = false):
// processMap's merge of a scan into every particle's map (src/EmbodiedSlamFilter.cpp:179-232)
// and cloneMaps' independent copies (src/PoseEstimator.cpp:31-47) as copy on write of tables
// and pages (eslam_internal.h LocalMaps).
// ---------------------------------------------------------------------------------------
// fresh maps: particle i names table i (sid: both state buffers' names, 2 x n), every table
// empty, every page free and unowned
__global__ void __launch_bounds__(kBlock) k_store_init(uint32_t* __restrict__ sid, LocalMaps lm, uint64_t n, uint64_t pool,
                                                      uint64_t items)
{
    const uint64_t slots = pool * lm.S;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < items; i += (uint64_t)gridDim.x * kBlock) {
        if (i < slots) lm.slot[i] = DM_LM_NONE;
        if (i < pool) {
            lm.ctr[i] = make_int2(DM_LM_UNSET, DM_LM_UNSET);
            lm.tgen[i] = 0u;
            if (i < n) {                     // both state buffers' names (n = cap here)
                sid[i] = (uint32_t)i;
                sid[n + i] = (uint32_t)i;
            }
        }
        if (i < lm.npages) {
            lm.frees[i] = (uint32_t)i;
            lm.owner[i] = ~0ull;
        }
    }
}

__device__ __forceinline__ uint32_t* cur_sid(const SidRef& r) { return (r.ctl->base ^ r.ctl->flip) ? r.s1 : r.s0; }

// ref[s]: 0, 1 or >= 2 particles name table s (received particles name none yet; the map merge
// only asks "free", "own" or "shared").  A resample hands the copies of a particle out as
// consecutive outputs, so equal names come in runs: the first lane of a run within the wave
// raises ref to 2 with a plain store when the run is longer than one (no atomic: as sharing
// grows, long runs span many waves and one hot atomic per wave serialised at 0.6 ms per 8M),
// and adds 1 atomically otherwise.  Any interleaving ends at the right class.  A table found
// shared moves to its next generation: its pages are frozen (the copies will name them too).
__global__ void __launch_bounds__(kBlock) k_store_ref(SidRef sr, uint64_t n, uint32_t* __restrict__ ref, GatherView gv,
                                                     uint32_t fuse, uint32_t* __restrict__ tgen)
{
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t s;
    if (fuse && sr.ctl->gather) {
        // a pending resample gather that the map merge runs (MergeParams::fuse): output i will
        // name its ancestor's table (the marks expanded as in K1, state[base] read)
        const uint64_t row0 = i & ~(uint64_t)(kRow - 1);          // a row past n has no row_first entry
        const uint32_t carry = row0 < n ? gv.row_first[row0 / kRow] + 1u : 0u;
        uint32_t mk = i < n ? gv.marks[i] : 0u;
        mk = wave_incl_max_u32(mk);
        const uint32_t src = (mk > carry ? mk : carry) - 1u;
        const uint32_t* sin = sr.ctl->base ? sr.s1 : sr.s0;
        s = i < n ? sin[src] : 0xffffffffu;
    } else {
        const uint32_t* sid = cur_sid(sr);
        s = i < n ? sid[i] : 0xffffffffu;
    }
    const uint32_t prev = (uint32_t)__shfl_up((int)s, 1, 64);
    const bool head = lane == 0 || prev != s;
    const uint64_t heads = __ballot(head);
    const uint64_t above = lane == 63 ? 0ull : heads >> (lane + 1);
    const uint32_t len = above ? (uint32_t)__builtin_ctzll(above) + 1u : 64u - lane;
    if (head && !(s & kSidRecord)) {                               // 0xffffffff has the record bit
        if (len >= 2u) {
            if (ref[s] < 2u) ref[s] = 2u;
            tgen[s] += 1u;                   // racing bumps of one table only move it further
        } else if (atomicAdd(&ref[s], 1u) >= 1u) {
            tgen[s] += 1u;
        }
    }
}

// compaction, mode 0: the free tables (ref 0) in table order, over the pool; mode 1: the
// particles received from another rank (sid = kSidRecord | record), in particle order;
// mode 2: the free pages (mark 0) in page order.  gate (device word, may be null): when 0
// the launch does nothing (the collection runs only when a map update needs it)
__device__ __forceinline__ bool compact_pred(int mode, uint64_t i, const uint32_t* ref, const uint32_t* sid)
{
    if (mode == 2) return reinterpret_cast<const uint8_t*>(ref)[i] == 0u;
    return mode == 0 ? ref[i] == 0u : (sid[i] & kSidRecord) != 0u;
}

constexpr int kCompactTile = kCompactTileItems;

__global__ void __launch_bounds__(kBlock) k_compact_count(int mode, uint64_t n, const uint32_t* __restrict__ ref,
                                                          SidRef sr, uint32_t* __restrict__ counts,
                                                          const uint32_t* __restrict__ gate)
{
    if (gate && !*gate) return;
    const uint32_t* sid = mode == 1 ? cur_sid(sr) : nullptr;
    __shared__ uint32_t s_w[kWaves];
    const uint64_t base = (uint64_t)blockIdx.x * kCompactTile;
    uint32_t c = 0;
    for (int r = 0; r < kCompactItems; ++r) {
        const uint64_t i = base + (uint64_t)r * kBlock + threadIdx.x;
        if (i < n && compact_pred(mode, i, ref, sid)) ++c;
    }
    c = wave_sum_u32(c);
    if ((threadIdx.x & 63u) == 0) s_w[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) counts[blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

// offs: exclusive prefix of counts; each selected i goes to out[offs[b] + its rank in the tile]
__global__ void __launch_bounds__(kBlock) k_compact_write(int mode, uint64_t n, const uint32_t* __restrict__ ref,
                                                          SidRef sr, const uint32_t* __restrict__ offs,
                                                          uint32_t* __restrict__ out, const uint32_t* __restrict__ gate)
{
    if (gate && !*gate) return;
    const uint32_t* sid = mode == 1 ? cur_sid(sr) : nullptr;
    __shared__ uint32_t s_w[kWaves];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint64_t base = (uint64_t)blockIdx.x * kCompactTile;
    const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t run = offs[blockIdx.x];
    for (int r = 0; r < kCompactItems; ++r) {       // rounds of 256 consecutive items, in order
        const uint64_t i = base + (uint64_t)r * kBlock + threadIdx.x;
        const bool sel = i < n && compact_pred(mode, i, ref, sid);
        const uint64_t b = __ballot(sel);
        if (lane == 0) s_w[wave] = (uint32_t)__popcll(b);
        __syncthreads();
        uint32_t pos = run + (uint32_t)__popcll(b & below);
        for (uint32_t w = 0; w < wave; ++w) pos += s_w[w];
        if (sel) out[pos] = (uint32_t)i;
        run += s_w[0] + s_w[1] + s_w[2] + s_w[3];
        __syncthreads();
    }
}

// ---- the window arithmetic (eslam_detmath.h DM_LM_*, the oracle's or_map_update) -------
__device__ __forceinline__ uint32_t lm_div(uint32_t a, uint64_t m) { return (uint32_t)(((uint64_t)a * m) >> kLmMagicShift); }
__device__ __forceinline__ uint32_t lm_mod(uint32_t a, uint32_t w, uint64_t m) { return a - w * lm_div(a, m); }
// the tile of slot column s in the window [c - h, c + h] (= dm_lm_tile_of): lo + ((s - lo) mod w)
// evaluated on s + (b - lo) with b a multiple of w >= 2^29, so the residue's argument is positive
__device__ __forceinline__ int32_t lm_tile(uint32_t s, int32_t c, uint32_t h, uint32_t w, uint64_t m, uint32_t b)
{
    const int32_t lo = c - (int32_t)h;
    return lo + (int32_t)lm_mod(s + (uint32_t)((int32_t)b - lo), w, m);
}
__device__ __forceinline__ bool lm_in(int32_t a, int32_t c, uint32_t h)
{
    const int32_t d = a - c;
    return d <= (int32_t)h && -d <= (int32_t)h;
}

// ---- the trail (eslam_internal.h LocalMaps; the oracle's lm_trail_* and lm_recentre): a
// table's tiles outside its window, V entries {a, b, page, -} closing its row.  The last word
// before them (window padding: (2h + 1)^2 is odd, so there always is one) holds the trail's
// high-water mark hw (DM_LM_NONE: 0): entries from hw on are empty and are neither read nor
// copied (their words may be stale)
__device__ __forceinline__ uint32_t lm_trail_off(const LocalMaps& lm) { return lm.S - 4u * lm.V; }
__device__ __forceinline__ uint32_t lm_hw_word(uint32_t w) { return w == DM_LM_NONE ? 0u : w; }
__device__ __forceinline__ int32_t lm_cheb(int32_t a, int32_t b, int32_t na, int32_t nb)
{
    const int32_t da = a > na ? a - na : na - a, db = b > nb ? b - nb : nb - b;
    return da > db ? da : db;
}
// tile (a, b) into the trail of row: the first empty entry, else in place of the entry farthest
// from (na, nb) (the first such) when that one is farther than the tile; 1 when a tile was forgotten
__device__ __forceinline__ uint32_t lm_trail_push(const LocalMaps& lm, uint32_t* row, int32_t na, int32_t nb, int32_t a, int32_t b,
                                                  uint32_t pg)
{
    uint4* t = reinterpret_cast<uint4*>(row + lm_trail_off(lm));
    const uint32_t hw = lm_hw_word(row[lm_trail_off(lm) - 1u]);
    int32_t far = -1;
    uint32_t fe = 0;
    for (uint32_t e = 0; e < hw; ++e) {
        const uint4 v = t[e];
        if (v.z == DM_LM_NONE) {
            t[e] = make_uint4((uint32_t)a, (uint32_t)b, pg, DM_LM_NONE);
            return 0u;
        }
        const int32_t d = lm_cheb((int32_t)v.x, (int32_t)v.y, na, nb);
        if (d > far) { far = d; fe = e; }
    }
    if (hw < lm.V) {                                     // the first entry never used
        t[hw] = make_uint4((uint32_t)a, (uint32_t)b, pg, DM_LM_NONE);
        row[lm_trail_off(lm) - 1u] = hw + 1u;
        return 0u;
    }
    if (lm.V && far > lm_cheb(a, b, na, nb)) t[fe] = make_uint4((uint32_t)a, (uint32_t)b, pg, DM_LM_NONE);
    return 1u;
}

constexpr uint32_t kLmList = 8;                 // tiles one pass of the merge handles
constexpr uint16_t kCodeSkip = 0xffffu;
constexpr uint32_t kLmNoList = 0xffffffffu;

// one particle as a map update sees it: its table, its pose, the window's new centre
struct LmPart {
    uint32_t X;                          // the table it names
    bool shared;                         // another particle names X too
    bool placed;                         // finite x, y, theta (else the update skips it)
    double x, y, th, z, zs;
    double sn, co;
    int32_t na, nb;                      // the new centre
};

__device__ __forceinline__ void lm_centre(const MapView& map, const MergeParams& mp, const LmPart& q, int32_t& na, int32_t& nb)
{
    if (mp.is_id) {
        na = dm_lm_centre(q.x, map.offset_x, map.inv_scale_x);
        nb = dm_lm_centre(q.y, map.offset_y, map.inv_scale_y);
    } else {
        const double* A = map.g2l;
        const double lx = ((A[0] * q.x + A[1] * q.y) + A[2] * q.z) + A[3];
        const double ly = ((A[4] * q.x + A[5] * q.y) + A[6] * q.z) + A[7];
        na = dm_lm_centre(lx, map.offset_x, map.inv_scale_x);
        nb = dm_lm_centre(ly, map.offset_y, map.inv_scale_y);
    }
}

// scan patch k's code for this particle: (slot << 6) | cell in the tile, or kCodeSkip (off
// the grid or outside the window).  Counts the dropped patches; cell_out: the grid cell
// (0xffffffff off the grid), whose occupancy bit the callers test eight patches at a time
// (a cell the shared grid covers: merged into the particle's own copy of it, which the
// merge starts from the grid's patch)
__device__ __forceinline__ uint16_t lm_code(const MapView& map, const LocalMaps& lm, const MergeParams& mp, const LmPart& q,
                                            uint32_t k, uint32_t& cell_out, uint32_t& dropped)
{
    const double bx = q.x - map.offset_x, by = q.y - map.offset_y;
    {
        const ScanPatch sp = mp.sp[k];
        uint32_t cell, cm, cn;
        if (mp.is_id) {
            cell = dm_merge_cell_mn(bx, by, q.co, q.sn, sp.x, sp.y, map.inv_scale_x, map.inv_scale_y, map.width,
                                    map.height_cells, &cm, &cn);
        } else {
            const double wx = (q.co * sp.x + (-q.sn) * sp.y) + q.x;
            const double wy = (q.sn * sp.x + q.co * sp.y) + q.y;
            const double wz = sp.z + q.z;
            const double* A = map.g2l;
            const double lx = ((A[0] * wx + A[1] * wy) + A[2] * wz) + A[3];
            const double ly = ((A[4] * wx + A[5] * wy) + A[6] * wz) + A[7];
            const double fm = floor((lx - map.offset_x) * map.inv_scale_x);
            const double fn = floor((ly - map.offset_y) * map.inv_scale_y);
            const bool in = (fm >= 0.0) & (fm < (double)map.width) & (fn >= 0.0) & (fn < (double)map.height_cells);
            cm = in ? (uint32_t)fm : 0u;
            cn = in ? (uint32_t)fn : 0u;
            cell = in ? cn * map.width + cm : 0xffffffffu;
        }
        uint16_t code = kCodeSkip;
        cell_out = cell;
        if (cell != 0xffffffffu) {
            const uint32_t a = cm >> DM_LM_TILE_BITS, b = cn >> DM_LM_TILE_BITS;
            if (dm_lm_inside(a, q.na, lm.hx, lm.wx) && dm_lm_inside(b, q.nb, lm.hy, lm.wy)) {
                const uint32_t s = lm_mod(a, lm.wx, lm.mx) + lm.wx * lm_mod(b, lm.wy, lm.my);
                code = (uint16_t)((s << 6) | ((cm & 7u) + 8u * (cn & 7u)));
            } else {
                ++dropped;                   // beyond maxSensorRange: outside the window
            }
        }
        return code;
    }
}

// how many of eight cells the shared grid covers: the eight occupancy words in one round trip
__device__ __forceinline__ uint32_t lm_covered8(const MapView& map, const uint32_t (&cell)[8])
{
    uint32_t w[8];
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) w[j] = cell[j] != 0xffffffffu ? map.occ[cell[j] >> 5] : 0u;
    uint32_t n = 0;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) n += (w[j] >> (cell[j] & 31u)) & 1u;
    return n;
}

// every scan patch's code into LDS (patch-major, thread-minor: a part of kScanPartSmall)
__device__ __forceinline__ void lm_codes(const MapView& map, const LocalMaps& lm, const MergeParams& mp, const LmPart& q,
                                         uint16_t* codes, uint32_t& covered, uint32_t& dropped)
{
    for (uint32_t k0 = 0; k0 < mp.m; k0 += 8) {
        uint32_t cell[8];
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j) {
            cell[j] = 0xffffffffu;
            if (k0 + j < mp.m) codes[(k0 + j) * kLmBlock] = lm_code(map, lm, mp, q, k0 + j, cell[j], dropped);
        }
        covered += lm_covered8(map, cell);
    }
}

// slot s into the sorted list of the kLmList smallest distinct slots; more: a slot fell off
__device__ __forceinline__ void lm_insert(uint32_t (&L)[kLmList], uint32_t s, bool& more)
{
    bool dup = false;
#pragma unroll
    for (uint32_t r = 0; r < kLmList; ++r) dup |= L[r] == s;
    if (dup) return;
    more |= L[kLmList - 1] != kLmNoList;
#pragma unroll
    for (uint32_t r = kLmList - 1; r >= 1; --r) L[r] = L[r - 1] > s ? L[r - 1] : (L[r] > s ? s : L[r]);
    L[0] = L[0] > s ? s : L[0];
}

// a large part: every code straight to the particle's row of the codes buffer (eight per
// 16-byte store), and the first pass's tiles collected on the way (L; more: further tiles)
__device__ __forceinline__ void lm_codes_row(const MapView& map, const LocalMaps& lm, const MergeParams& mp, const LmPart& q,
                                             uint4* row, uint32_t (&L)[kLmList], bool& more, uint32_t& covered, uint32_t& dropped)
{
#pragma unroll
    for (uint32_t r = 0; r < kLmList; ++r) L[r] = kLmNoList;
    more = false;
    for (uint32_t k0 = 0; k0 < mp.m; k0 += 8) {
        uint32_t w[4], cell[8];
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j) {
            const uint32_t k = k0 + j;
            cell[j] = 0xffffffffu;
            const uint32_t c = k < mp.m ? (uint32_t)lm_code(map, lm, mp, q, k, cell[j], dropped) : (uint32_t)kCodeSkip;
            if (c != kCodeSkip) lm_insert(L, c >> 6, more);
            w[j >> 1] = (j & 1) ? (w[j >> 1] | (c << 16)) : c;
        }
        row[k0 >> 3] = make_uint4(w[0], w[1], w[2], w[3]);
        covered += lm_covered8(map, cell);
    }
}

// the up to kLmList smallest distinct slots above t of a particle's codes row
__device__ __forceinline__ void lm_collect_row(const uint4* row, uint32_t m, uint32_t t, uint32_t (&L)[kLmList])
{
#pragma unroll
    for (uint32_t r = 0; r < kLmList; ++r) L[r] = kLmNoList;
    bool more = false;
    for (uint32_t k0 = 0; k0 < m; k0 += 8) {
        const uint4 v = row[k0 >> 3];
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j) {
            const uint32_t c = (w[j >> 1] >> ((j & 1) * 16)) & 0xffffu;
            if (k0 + j >= m || c == kCodeSkip) continue;
            const uint32_t s = c >> 6;
            if (s > t) lm_insert(L, s, more);
        }
    }
}

// the up to kLmList smallest distinct slots above t (sorted; free entries kLmNoList)
__device__ __forceinline__ void lm_collect(const uint16_t* codes, uint32_t m, uint32_t t, uint32_t (&L)[kLmList])
{
#pragma unroll
    for (uint32_t r = 0; r < kLmList; ++r) L[r] = kLmNoList;
    for (uint32_t k = 0; k < m; ++k) {
        const uint16_t c = codes[k * kLmBlock];
        if (c == kCodeSkip) continue;
        const uint32_t s = (uint32_t)c >> 6;
        if (t != kLmNoList && s <= t) continue;
        bool dup = false;
#pragma unroll
        for (uint32_t r = 0; r < kLmList; ++r) dup |= L[r] == s;
        if (dup) continue;
#pragma unroll
        for (uint32_t r = kLmList - 1; r >= 1; --r) L[r] = L[r - 1] > s ? L[r - 1] : (L[r] > s ? s : L[r]);
        L[0] = L[0] > s ? s : L[0];
    }
}

__device__ __forceinline__ uint32_t lm_find(const uint32_t (&L)[kLmList], uint32_t s)
{
    uint32_t idx = kLmNoList;
#pragma unroll
    for (uint32_t r = 0; r < kLmList; ++r) idx = L[r] == s ? r : idx;
    return idx;
}

// the plan's table step (the oracle's lm_recentre; copy on write): table T's row and centre
// from X's, the window moved to (na, nb): (1) the tiles leaving it go to the trail in slot
// order, (2) the trail's tiles inside the new window go back to their slots.  T != X: X is
// shared, T a free table written whole.  A lane per particle; returns the tiles forgotten.
__device__ uint32_t lm_rewrite(const LocalMaps& lm, uint32_t X, uint32_t T, int2 oc, int32_t na, int32_t nb)
{
    uint32_t* row = lm.slot + (uint64_t)T * lm.S;
    const uint32_t toff = lm_trail_off(lm);
    if (X != T) {                                        // the window's words and the trail's used entries
        const uint4* src = reinterpret_cast<const uint4*>(lm.slot + (uint64_t)X * lm.S);
        uint4* dst = reinterpret_cast<uint4*>(row);
        const uint32_t nq = toff / 4u + lm_hw_word(lm.slot[(uint64_t)X * lm.S + toff - 1u]);
        for (uint32_t q = 0; q < nq; ++q) dst[q] = src[q];
    }
    uint32_t forgot = 0;
    if (oc.x != DM_LM_UNSET && (oc.x != na || oc.y != nb)) {
        // the window's columns and rows whose tiles leave it (bit sa / sb), then their slots in
        // slot order
        uint32_t colx = 0, rowx = 0;
        for (uint32_t sa = 0; sa < lm.wx; ++sa)
            colx |= lm_in(lm_tile(sa, oc.x, lm.hx, lm.wx, lm.mx, lm.bx), na, lm.hx) ? 0u : 1u << sa;
        for (uint32_t sb = 0; sb < lm.wy; ++sb)
            rowx |= lm_in(lm_tile(sb, oc.y, lm.hy, lm.wy, lm.my, lm.by), nb, lm.hy) ? 0u : 1u << sb;
        const uint32_t all = lm.wx >= 32u ? ~0u : (1u << lm.wx) - 1u;
        for (uint32_t sb = 0; sb < lm.wy; ++sb) {
            const int32_t b = lm_tile(sb, oc.y, lm.hy, lm.wy, lm.my, lm.by);
            for (uint32_t cols = ((rowx >> sb) & 1u) ? all : colx; cols; cols &= cols - 1u) {
                const uint32_t sa = (uint32_t)__builtin_ctz(cols);
                const uint32_t s = sa + lm.wx * sb, p = row[s];
                if (p == DM_LM_NONE) continue;
                forgot += lm_trail_push(lm, row, na, nb, lm_tile(sa, oc.x, lm.hx, lm.wx, lm.mx, lm.bx), b, p);
                row[s] = DM_LM_NONE;
            }
        }
        uint4* t = reinterpret_cast<uint4*>(row + toff);
        const uint32_t hw = lm_hw_word(row[toff - 1u]);
        for (uint32_t e = 0; e < hw; ++e) {
            const uint4 v = t[e];
            if (v.z == DM_LM_NONE || !lm_in((int32_t)v.x, na, lm.hx) || !lm_in((int32_t)v.y, nb, lm.hy)) continue;
            row[lm_mod(v.x, lm.wx, lm.mx) + lm.wx * lm_mod(v.y, lm.wy, lm.my)] = v.z;
            t[e] = make_uint4(v.x, v.y, DM_LM_NONE, DM_LM_NONE);
        }
    }
    lm.ctr[T] = make_int2(na, nb);
    return forgot;
}

// the particle of a map update: output i reads its ancestor through the marks when the merge
// runs the pending resample gather (fused), else itself
__device__ __forceinline__ uint32_t lm_source(const MergeParams& mp, uint64_t i, bool gath)
{
    uint32_t src = (uint32_t)i;
    if (gath) {
        const uint64_t row0 = i & ~(uint64_t)(kRow - 1);
        const uint32_t carry = row0 < mp.n ? mp.gv.row_first[row0 / kRow] + 1u : 0u;
        uint32_t mk = i < mp.n ? mp.gv.marks[i] : 0u;
        mk = wave_incl_max_u32(mk);
        src = (mk > carry ? mk : carry) - 1u;
    }
    return src;
}

__device__ __forceinline__ void lm_load(const DevState& in, uint32_t src, const MapView& map, const MergeParams& mp,
                                        const uint32_t* ref, LmPart& q)
{
    q.X = in.sid[src];
    q.shared = ref[q.X] > 1u;
    q.x = in.x[src]; q.y = in.y[src]; q.th = in.th[src]; q.z = in.z[src]; q.zs = in.zs[src];
    dm_sincos(q.th, &q.sn, &q.co);
    q.placed = dm_isfinite(q.x - map.offset_x) && dm_isfinite(q.y - map.offset_y) && dm_isfinite(q.th);
    q.na = q.nb = 0;
    if (q.placed) lm_centre(map, mp, q, q.na, q.nb);
}

// the exclusive prefix of the blocks' per-thread needs (off[t], thread t of the block) and the
// block's sum (*sum); s_w: kLmBlock / 64 words of LDS
__device__ __forceinline__ void block_offsets(uint32_t need, bool valid, uint32_t* off, uint32_t* sum, uint32_t* s_w)
{
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    uint32_t pfx = need;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t v = (uint32_t)__shfl_up((int)pfx, o, 64);
        pfx += lane >= (uint32_t)o ? v : 0u;
    }
    if (lane == 63) s_w[tid >> 6] = pfx;
    __syncthreads();
    uint32_t base = 0;
    for (uint32_t w = 0; w < (tid >> 6); ++w) base += s_w[w];
    if (valid) off[tid] = base + pfx - need;
    if (tid == kLmBlock - 1) *sum = base + pfx;
}

// after the scan of the plan's block sums: whether the free list holds this update's pages
// (else the collection runs first)
__global__ void k_page_budget(Ctl* __restrict__ ctl, const uint32_t* __restrict__ poff, uint32_t nblocks)
{
    const uint64_t total = poff[nblocks];
    ctl->pg_total = total;
    ctl->pg_gc = ctl->pg_cursor + total > ctl->pg_nfree ? 1u : 0u;
}

// the collection: clear the marks, mark every page a live table (ref >= 1) names, compact the
// unmarked pages into LocalMaps::frees (k_compact_* mode 2), then k_page_budget2
__global__ void __launch_bounds__(kBlock) k_pg_clear(uint8_t* __restrict__ mark, uint64_t npages, const uint32_t* __restrict__ gate)
{
    if (!*gate) return;
    uint4* m4 = reinterpret_cast<uint4*>(mark);
    const uint64_t n16 = (npages + 15) / 16;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * kBlock)
        m4[i] = make_uint4(0u, 0u, 0u, 0u);
}

// one wave per table (grid-stride): its lanes walk the slots, then the trail's pages
__global__ void __launch_bounds__(kBlock) k_pg_mark(LocalMaps lm, const uint32_t* __restrict__ ref, const uint32_t* __restrict__ gate)
{
    if (!*gate) return;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nw = (uint64_t)gridDim.x * kWaves;
    const uint32_t toff = lm.S - 4u * lm.V;
    for (uint64_t t = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6); t < lm.ntables; t += nw) {
        if (ref[t] == 0u) continue;
        const uint32_t* sl = lm.slot + t * lm.S;
        for (uint32_t s = lane; s < toff; s += 64u) {
            const uint32_t p = sl[s];
            if (p != DM_LM_NONE) lm.mark[p] = 1u;
        }
        const uint32_t hw = lm_hw_word(sl[toff - 1u]);
        for (uint32_t e = lane; e < hw; e += 64u) {
            const uint32_t p = sl[toff + 4u * e + 2u];
            if (p != DM_LM_NONE) lm.mark[p] = 1u;
        }
    }
}

__global__ void k_page_budget2(Ctl* __restrict__ ctl, const uint32_t* __restrict__ counts, uint32_t tiles,
                               uint32_t* fault)
{
    if (!ctl->pg_gc) return;
    ctl->pg_nfree = counts[tiles];
    ctl->pg_cursor = 0;
    if (ctl->pg_total > ctl->pg_nfree) {
        atomicOr((unsigned long long*)&ctl->err, (unsigned long long)kFaultPages);
        if (fault) __hip_atomic_fetch_or(fault, kFaultPages, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// processMap(scanMap, match = false, update = true) per particle (the oracle's or_map_update):
// the window moves to the tile under the particle (tiles that leave it are forgotten), then
// every scan patch, placed at the particle's pose (Translation(x, y, 0) * Rz(theta); the
// offset patch adds zPos and zSigma^2, src/EmbodiedSlamFilter.cpp:186-189, 213-214), merges
// into the cell it lands in: inserted into an empty cell (test/testMap.cpp:307-316) or fused
// (dm_lm_fuse) with the patch there.  The table the particle writes is its own (ref 1: in
// place) or, when shared, the free table frees[i] it then names.
// Two kernels.  k_map_plan (a lane per particle) does the lookups: the codes of the scan's
// cells, the tiles, their pages, whether the table owns them.  k_map_merge moves the data, a
// group of kLmLanes lanes per particle (four particles a wave), so that every access of the
// maps is a whole table or page moved by the group together (a lane per particle touching
// 8-byte cells scattered over 64 pages missed the caches on two of three accesses: r05h).
// Per particle:
//   1. the plan's record, the codes (PART / kLmLanes a lane, two to a register) and the allocation offset arrive in one
//      round trip; each patch is ranked among the earlier patches on its cell;
//   2. lane r of the group takes tile r of the first pass: a new page when the plan says the
//      table does not own it; a table copied on write or whose window moved is rewritten by
//      the group (evictions, the pass's new pages folded in);
//   3. kLmStage pages at a time are staged in LDS (each lane loads 32 B: whole 512-B pages),
//      the patches applied there rank by rank (scan order on every cell), and the changed or
//      new pages stored whole.  Tiles beyond kLmList (a later pass) are looked up by the group.
// A tile whose patches all turn out no-ops keeps the copy it got: the same values.
// 8 lanes per particle, 2 staged pages each, at most 128 VGPRs: 11.8 ms per merge at 8M against
// 12.4 for 16 lanes with 4 pages (r05 A/B, profiles/r05/ab_merge_lanes.log)
#ifndef ESLAM_LM_LANES
#define ESLAM_LM_LANES 8
#endif
#ifndef ESLAM_LM_STAGE
#define ESLAM_LM_STAGE 2
#endif
#ifndef ESLAM_LM_WPE
#define ESLAM_LM_WPE 4
#endif
constexpr uint32_t kLmLanes = ESLAM_LM_LANES;                       // lanes per particle: 8 or 16
constexpr uint32_t kLmMergeBlock = 128;
constexpr uint32_t kLmPpb = kLmMergeBlock / kLmLanes;               // particles per block
constexpr uint32_t kLmStage = ESLAM_LM_STAGE;                        // pages in LDS per particle
static_assert(kLmList <= kLmLanes && (kLmLanes == 8 || kLmLanes == 16) && kLmStage <= 4,
              "a lane per tile of a pass; 8 or 16 lanes; row masks of 8 bits per staged page in a word");
constexpr uint32_t kLmChunk = kLmLanes * 16;                         // bytes of a page a group moves per instruction
constexpr uint32_t kLmNq = DM_LM_PAGE_CELLS * 8 / kLmChunk;           // such chunks per page

// the lanes of a wave see each other's LDS writes (in-order LDS; no code motion across)
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ uint32_t grp_min(uint32_t v)
{
#pragma unroll
    for (int o = kLmLanes / 2; o >= 1; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, kLmLanes));
    return v;
}
__device__ __forceinline__ uint32_t grp_max(uint32_t v)
{
#pragma unroll
    for (int o = kLmLanes / 2; o >= 1; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, kLmLanes));
    return v;
}
__device__ __forceinline__ uint32_t grp_or(uint32_t v)
{
#pragma unroll
    for (int o = kLmLanes / 2; o >= 1; o >>= 1) v |= (uint32_t)__shfl_xor((int)v, o, kLmLanes);
    return v;
}
__device__ __forceinline__ uint32_t grp_get(uint32_t v, uint32_t l) { return (uint32_t)__shfl((int)v, (int)l, kLmLanes); }

// the first patch of shared-grid cell ct (its MapView::cell_tab record) passing getPatch's
// 3-sigma gate against the local height lz (the oracle's or_mls_cell_patch); its stdev in *sd
__device__ __forceinline__ bool grid_cell_patch(const MapView& map, uint4 ct, double lz, double qv, double& mean,
                                                double* sd = nullptr)
{
    for (uint32_t k = ct.z; k < ct.z + ct.w; ++k) {
        const float2 pf = k == ct.z ? make_float2(__uint_as_float(ct.x), __uint_as_float(ct.y)) : map.patch[k];
        const double pm = (double)pf.x, ps = (double)pf.y;
        const double ph = map.height ? (double)map.height[k] : 0.0;
        double diff;
        if (ph > 0.0) {
            if (lz > pm) diff = lz - pm;
            else if (lz < pm - ph) diff = (pm - ph) - lz;
            else diff = 0.0;
        } else {
            diff = dm_fabs(pm - lz);
        }
        if (diff * diff < 9.0 * (ps * ps + qv)) {
            mean = pm;
            if (sd) *sd = ps;
            return true;
        }
    }
    return false;
}

// k_map_plan: per particle (a lane each: kLmBlock particles a block, so the latency of its
// chain of lookups -- state, table, page, owner -- overlaps across many particles) the cell
// codes of its scan (MergeParams::codes), the first pass's tiles with their pages and whether
// the table owns them (the MergeJob record), and the pages its merge takes: one per tile its
// scan reaches that its table cannot write in place (a new tile, or a page it does not own).
// The block sums give the allocation offsets (k_scan_excl).  A tile whose writes all turn out
// no-ops leaves its page unused (free again at the next collection).
template <uint32_t PART>
__global__ void __launch_bounds__(kLmBlock) k_map_plan(DevState s0, DevState s1, const Ctl* __restrict__ ctl, MapView map,
                                                       LocalMaps lm, MergeParams mp)
{
    // a small part's codes leave through LDS (then the records); a large part's go straight to
    // the rows (their LDS would cost the kernel its occupancy)
    __shared__ __attribute__((aligned(16))) uint16_t s_code[kScanPartSmall * kLmBlock];
    // the block sums' words alias the codes: the block holds exactly 16 KiB of LDS (a 17th
    // granule cost it a block per CU)
    uint32_t* s_w = reinterpret_cast<uint32_t*>(s_code);
    static_assert(sizeof(MergeJob) * kLmBlock <= sizeof(uint16_t) * kScanPartSmall * kLmBlock, "records in s_code");
    constexpr bool kSmall = PART == kScanPartSmall;
    const uint32_t tid = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * kLmBlock, i = base + tid;
    const uint32_t nb = (uint32_t)(mp.n - base < kLmBlock ? mp.n - base : kLmBlock);     // particles of the block
    const DevState st = (ctl->base ^ ctl->flip) ? s1 : s0;
    const bool gath = mp.fuse && ctl->gather;
    const DevState in = gath ? (ctl->base ? s1 : s0) : st;
    const uint32_t src = lm_source(mp, i, gath);
    uint32_t need = 0, covered = 0, dropped = 0, forgot = 0;
    MergeJob jb;
    if (i < mp.n) {
        LmPart q;
        lm_load(in, src, map, mp, mp.ref, q);
        jb.X = q.X;
        jb.T = q.X;
        jb.gT = 0;
        jb.na = q.na;
        jb.nb = q.nb;
        jb.ox = jb.oy = DM_LM_UNSET;
        jb.flags = 0;
        jb.need = 0;
        jb.z = q.z;
        jb.zs = q.zs;
        jb.src = src;
#pragma unroll
        for (uint32_t r = 0; r < kLmList; ++r) { jb.L[r] = 0; jb.P[r] = DM_LM_NONE; }
        if (q.placed) {
            uint16_t* codes = s_code + tid;
            uint4* crow = reinterpret_cast<uint4*>(mp.codes + i * PART);
            uint32_t L[kLmList];
            bool more1 = false;
            const uint32_t cov0 = covered;
            if constexpr (kSmall) {
                lm_codes(map, lm, mp, q, codes, covered, dropped);
                lm_collect(codes, mp.m, kLmNoList, L);
            } else {
                lm_codes_row(map, lm, mp, q, crow, L, more1, covered, dropped);
            }
            const int2 oc = lm.ctr[q.X];
            const uint32_t T = q.shared ? mp.frees[i] : q.X;
            // the window moves to the particle (into T: a shared table is copied): from here on
            // every tile the scan reaches is in T's slots.  A shared table whose window stays is
            // copied by the merge (a group of lanes per particle moves the row coalesced); its
            // tiles are X's slots
            const bool moved = oc.x != q.na || oc.y != q.nb;
            if (moved) forgot = lm_rewrite(lm, q.X, T, oc, q.na, q.nb);
            const uint32_t* trow = lm.slot + (uint64_t)(moved ? T : q.X) * lm.S;
            const uint64_t gT = ((uint64_t)lm.tgen[T] << 32) | T;
            uint32_t nt = 0, bits = 0;
#pragma unroll
            for (uint32_t r = 0; r < kLmList; ++r) {
                if (L[r] == kLmNoList) continue;
                const uint32_t P = trow[L[r]];
                const bool mine = !q.shared && P != DM_LM_NONE && lm.owner[P] == gT;
                bits |= mine ? 0u : 1u << r;
                jb.L[r] = (uint16_t)L[r];
                jb.P[r] = P;
                ++nt;
            }
            need = __builtin_popcount(bits);
            // later passes (a scan reaching more than kLmList tiles): counted here, resolved by the merge
            bool more = false;
            for (uint32_t t = L[kLmList - 1]; t != kLmNoList && (kSmall || more1); t = L[kLmList - 1]) {
                if constexpr (kSmall) lm_collect(codes, mp.m, t, L);
                else lm_collect_row(crow, mp.m, t, L);
                if (L[0] == kLmNoList) break;
                more = true;
#pragma unroll
                for (uint32_t r = 0; r < kLmList; ++r) {
                    if (L[r] == kLmNoList) continue;
                    const uint32_t P = trow[L[r]];
                    need += (!q.shared && P != DM_LM_NONE && lm.owner[P] == gT) ? 0u : 1u;
                }
            }
            jb.T = T;
            jb.gT = gT;
            jb.ox = oc.x;
            jb.oy = oc.y;
            jb.need = bits;
            jb.flags = kJobPlaced | (q.shared ? kJobShared : 0u) | (more ? kJobMore : 0u) | (moved ? kJobMoved : 0u) |
                       (covered != cov0 ? kJobCovered : 0u) | (nt << 8);
        }
    }
    // the codes rows and the records leave through LDS, so every store is a whole 1-KiB line of
    // the wave (a lane per particle storing its own 128-byte record wrote 64 lines partially)
    __syncthreads();
    uint4* rows = reinterpret_cast<uint4*>(mp.codes + base * kScanPartSmall);
    for (uint32_t c = tid; kSmall && c < nb * (kScanPartSmall / 8); c += kLmBlock) {
        const uint32_t p = c / (kScanPartSmall / 8), k0 = (c % (kScanPartSmall / 8)) * 8;
        if (k0 >= mp.m) continue;
        uint32_t w[4];
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t a = k0 + 2 * j < mp.m ? s_code[(k0 + 2 * j) * kLmBlock + p] : kCodeSkip;
            const uint32_t b = k0 + 2 * j + 1 < mp.m ? s_code[(k0 + 2 * j + 1) * kLmBlock + p] : kCodeSkip;
            w[j] = a | (b << 16);
        }
        rows[c] = make_uint4(w[0], w[1], w[2], w[3]);
    }
    __syncthreads();
    uint4* srec = reinterpret_cast<uint4*>(s_code);
    if (i < mp.n) {
        const uint4* r = reinterpret_cast<const uint4*>(&jb);
#pragma unroll
        for (uint32_t k = 0; k < sizeof(MergeJob) / 16; ++k) srec[tid * (sizeof(MergeJob) / 16) + k] = r[k];
    }
    __syncthreads();
    uint4* jobs = reinterpret_cast<uint4*>(mp.job + base);
    for (uint32_t c = tid; c < nb * (sizeof(MergeJob) / 16); c += kLmBlock) jobs[c] = srec[c];
    covered = wave_sum_u32(covered);
    dropped = wave_sum_u32(dropped);
    forgot = wave_sum_u32(forgot);
    if ((tid & 63u) == 0) {                   // the update's dropped / covered patches, forgotten tiles (k_merge_counts)
        const uint32_t slot_c = (uint32_t)((blockIdx.x * (kLmBlock / 64) + (tid >> 6)) % kMergeCounterSlots);
        if (dropped) atomicAdd((unsigned long long*)&mp.cnt[slot_c], (unsigned long long)dropped);
        if (covered) atomicAdd((unsigned long long*)&mp.cnt[3 * kMergeCounterSlots + slot_c], (unsigned long long)covered);
        if (forgot) atomicAdd((unsigned long long*)&mp.cnt[6 * kMergeCounterSlots + slot_c], (unsigned long long)forgot);
    }
    __syncthreads();                          // every record has left s_code (s_w aliases it)
    block_offsets(need, i < mp.n, mp.off + (i - tid), mp.poff + blockIdx.x, s_w);
}

// the number of lower lanes of the 16-lane row holding the same code (c == 0xffffffff never
// matches): DPP row shifts, the group's lanes all active
template <int D>
__device__ __forceinline__ uint32_t row_same(uint32_t c, uint32_t l)
{
    if constexpr (D >= (int)kLmLanes) {
        return 0u;
    } else {
        const uint32_t o = (uint32_t)__builtin_amdgcn_update_dpp((int)0xffffffff, (int)c, 0x110 + D, 0xf, 0xf, false);
        return (o == c && l >= (uint32_t)D) ? 1u : 0u;     // l >= D: the lane D lower is in the group
    }
}
__device__ __forceinline__ uint32_t row_rank(uint32_t c, uint32_t l)
{
    return row_same<1>(c, l) + row_same<2>(c, l) + row_same<3>(c, l) + row_same<4>(c, l) + row_same<5>(c, l) +
           row_same<6>(c, l) + row_same<7>(c, l) + row_same<8>(c, l) + row_same<9>(c, l) + row_same<10>(c, l) +
           row_same<11>(c, l) + row_same<12>(c, l) + row_same<13>(c, l) + row_same<14>(c, l) + row_same<15>(c, l);
}

// the staged pages of a wave: for stage page rr, chunk q (kLmChunk bytes) the groups' chunks
// lie side by side (one 16-byte LDS-DMA per lane fills [rr][q] for the whole wave: 1 KiB)
constexpr uint32_t kLmWaveStage = kLmStage * kLmNq * 1024;          // bytes per wave
__device__ __forceinline__ uint32_t lm_stage_off(uint32_t rr, uint32_t ci, uint32_t g)
{
    constexpr uint32_t cpc = kLmChunk / 8;                           // cells per chunk
    return (rr * kLmNq + ci / cpc) * 1024 + g * kLmChunk + (ci % cpc) * 8;
}
// a large part's 32 codes a lane: three waves a SIMD (168 VGPRs)
#define LM_MERGE_ATTR __attribute__((amdgpu_waves_per_eu(PART == kScanPartSmall ? ESLAM_LM_WPE : ESLAM_LM_WPE_LARGE)))
#ifndef ESLAM_LM_WPE_LARGE
#define ESLAM_LM_WPE_LARGE 3
#endif
template <uint32_t PART>
__global__ void __launch_bounds__(kLmMergeBlock) LM_MERGE_ATTR k_map_merge(DevState s0, DevState s1, Ctl* __restrict__ ctl, MapView map,
                                                             LocalMaps lm, MergeParams mp)
{
    constexpr uint32_t PER = PART / kLmLanes;                       // codes a lane holds
    constexpr uint32_t NCH = PART / 8 / kLmLanes;                   // 16-byte chunks of codes a lane loads
    static_assert(PART <= 256 && NCH >= 1 && kLmStage <= 4, "a list entry holds k (8 bits), the page (2) and the cell (6)");
    __shared__ __attribute__((aligned(16))) uint16_t s_code[kLmPpb][PART];
    __shared__ __attribute__((aligned(16))) uint8_t s_stage[kLmMergeBlock / 64][kLmWaveStage];
    static_assert(PART * 2 >= 2 * kLmList * 4, "pass 0's slot / new page pairs fit a particle's s_code");
    // a small part's patch heights and deviations, read by every round (a large part's come
    // from memory: their 4 KiB would cost the kernel a block per CU)
    constexpr bool kSpLds = PART <= kScanPartSmall;
    __shared__ double2 s_sp[kSpLds ? PART : 1];
    const uint32_t tid = threadIdx.x, l = tid & (kLmLanes - 1), pl = tid / kLmLanes, g = pl % (64 / kLmLanes), wv = tid >> 6;
    // once the codes are in registers (cpk), the particle's s_code holds pass 0's (slot, new
    // page) pairs of a copied table and then each stage's list of patches
    uint32_t* const s_np = reinterpret_cast<uint32_t*>(&s_code[pl][0]);
    uint16_t* const s_lst = &s_code[pl][0];
    const uint64_t i = (uint64_t)blockIdx.x * kLmPpb + pl;
    if (ctl->err & kFaultPages) return;       // the pool could not hold the plan: nothing is written
    const bool valid = i < mp.n;
    ESLAM_STAMP(g_stamps_mg, 0);
    const DevState st = (ctl->base ^ ctl->flip) ? s1 : s0;      // by value: no private copy of the arguments
    // a pending resample gather (mp.fuse, one GPU) runs here instead of in its own launch:
    // output i reads its ancestor (the plan's src) in state[base] and the merge writes the
    // whole particle, its table name included, to st = state[base ^ 1]
    const bool gath = mp.fuse && ctl->gather;
    const DevState in = gath ? (ctl->base ? s1 : s0) : st;
    // the plan's record, the codes and this particle's first page: one round trip
    uint32_t X = 0, T = 0, flags = 0, needb = 0, src = 0, Lr = kLmNoList, Pr = DM_LM_NONE;
    uint64_t gT = 0, alloc = 0;
    int32_t na = 0, nb = 0;
    double z = 0.0, zs = 0.0;
    uint4 c4[NCH];                            // chunks l, l + kLmLanes, ... of the row (8 codes each)
#pragma unroll
    for (uint32_t q = 0; q < NCH; ++q) c4[q] = make_uint4(0u, 0u, 0u, 0u);
    if (valid) {
        const MergeJob* J = mp.job + i;
        X = J->X; T = J->T; gT = J->gT;
        flags = J->flags; needb = J->need;
        na = J->na; nb = J->nb;
        z = J->z; zs = J->zs; src = J->src;
        if (l < kLmList) { Lr = J->L[l]; Pr = J->P[l]; }
        const uint4* crow = reinterpret_cast<const uint4*>(mp.codes + i * PART);
#pragma unroll
        for (uint32_t q = 0; q < NCH; ++q)
            if ((l + kLmLanes * q) * 8 < mp.m) c4[q] = crow[l + kLmLanes * q];
        if constexpr (NCH > 1) {              // a large part's codes to LDS at once (no registers held)
#pragma unroll
            for (uint32_t q = 0; q < NCH; ++q) reinterpret_cast<uint4*>(&s_code[pl][0])[l + kLmLanes * q] = c4[q];
        }
        alloc = ctl->pg_cursor + mp.poff[i / kLmBlock] + mp.off[i];
    }
    for (uint32_t k = tid; kSpLds && k < mp.m && k < PART; k += kLmMergeBlock) s_sp[k] = make_double2(mp.sp[k].z, mp.sp[k].stdev);
    if (gath && valid) {                      // the gather's copies: a field a lane
        for (uint32_t f = l; f < 10; f += kLmLanes) switch (f) {
        case 0: st.w[i] = in.w[src]; break;
        case 1: if (mp.aux) st.mprob[i] = in.mprob[src]; break;
        case 2: if (mp.aux) st.flags[i] = in.flags[src]; break;
        case 3: if (mp.gv.record) mp.gv.anc[i] = (uint32_t)(mp.gbase + src); break;
        case 4: if (mp.gv.marks[i]) mp.gv.marks[i] = 0u; break;
        case 5: st.x[i] = in.x[src]; break;
        case 6: st.y[i] = in.y[src]; break;
        case 7: st.th[i] = in.th[src]; break;
        case 8: st.z[i] = in.z[src]; break;
        case 9: st.zs[i] = in.zs[src]; break;
        default: break;
        }
    }
    bool dirty = false, moved = false, covw = false;
    uint32_t written = 0, taken = 0;
    const bool shared = (flags & kJobShared) != 0;
    if constexpr (kSpLds) __syncthreads();    // s_sp
    if (valid && (flags & kJobPlaced)) {      // group-uniform from here on
        // ---- 1. the codes: patch k = l + kLmLanes u in lane l (round u precedes round u + 1 in
        // the scan, so the rounds apply in order and only a round's own duplicates need ranks)
        if constexpr (NCH == 1) reinterpret_cast<uint4*>(&s_code[pl][0])[l] = c4[0];
        wave_sync();
        ESLAM_STAMP(g_stamps_mg, 1);
        // two 16-bit codes a register: code(u) is patch l + kLmLanes u (round 6: against one
        // code a register and against reading them from LDS, profiles/r06/ab/ab_r06k*, ab_r06l*)
        uint32_t cpk[(PER + 1) / 2];
#pragma unroll
        for (uint32_t v = 0; v < (PER + 1) / 2; ++v) {
            const uint32_t k0 = l + kLmLanes * (2 * v), k1 = k0 + kLmLanes;
            const uint32_t c0 = k0 < mp.m ? (uint32_t)s_code[pl][k0] : (uint32_t)kCodeSkip;
            const uint32_t c1 = (2 * v + 1 < PER && k1 < mp.m) ? (uint32_t)s_code[pl][k1] : (uint32_t)kCodeSkip;
            cpk[v] = c0 | (c1 << 16);
        }
        auto code = [&](uint32_t u) -> uint32_t { return (cpk[u >> 1] >> ((u & 1u) * 16u)) & 0xffffu; };
        // the plan has moved T's window (a moved shared X copied to T): every tile of the scan is
        // in T's slots, and the merge only adds the new pages -- but a shared X whose window
        // stays is copied to T here, the pass's new pages folded in
        const bool copy = shared && !(flags & kJobMoved);
        uint32_t* tsl = lm.slot + (uint64_t)T * lm.S;
        const uint32_t* xsl = lm.slot + (uint64_t)X * lm.S;
        const uint32_t gshift = (tid & 63u) & ~(kLmLanes - 1u);
        const double zvar = zs * zs;
        uint8_t* stage = &s_stage[wv][0];
        // stage: lane l moves bytes [16 l, 16 l + 16) of each chunk of the pages, straight into LDS
        auto stage_pages = [&](const uint32_t (&Ls)[kLmStage], const uint32_t (&Ps)[kLmStage]) {
#pragma unroll
            for (uint32_t rr = 0; rr < kLmStage; ++rr) {
#pragma unroll
                for (uint32_t h = 0; h < kLmNq; ++h) {
                    uint8_t* dst = stage + (rr * kLmNq + h) * 1024;
                    if (Ls[rr] != kLmNoList && Ps[rr] != DM_LM_NONE) {
                        const uint8_t* srcp = reinterpret_cast<const uint8_t*>(lm.page + (uint64_t)Ps[rr] * DM_LM_PAGE_CELLS) +
                                              h * kLmChunk + l * 16;
                        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)srcp,
                                                         (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
                    } else {
                        *reinterpret_cast<uint4*>(dst + (tid & 63u) * 16) =
                            make_uint4(0u, __float_as_uint(-1.0f), 0u, __float_as_uint(-1.0f));
                    }
                }
            }
        };
        uint32_t cnt = (flags >> 8) & 0xffu;
        int32_t lo = -1;
        for (uint32_t pass = 0;; ++pass) {
            // lane r: tile r of the pass, its page P, whether it takes a new page NP
            bool need = false;
            uint32_t P = DM_LM_NONE, NP = DM_LM_NONE;
            bool more;
            if (pass == 0) {
                if (l >= cnt) Lr = kLmNoList;
                P = Pr;
                need = l < cnt && ((needb >> l) & 1u);
                more = (flags & kJobMore) != 0;
                lo = cnt ? (int32_t)grp_get(Lr, cnt - 1) : -1;
                // the first stage's pages are known from the record: their loads overlap the
                // allocation and the table rewrite below
                uint32_t Ls0[kLmStage], Ps0[kLmStage];
#pragma unroll
                for (uint32_t rr = 0; rr < kLmStage; ++rr) {
                    Ls0[rr] = grp_get(Lr, rr);
                    Ps0[rr] = grp_get(P, rr);
                }
                stage_pages(Ls0, Ps0);
            } else {
                Lr = kLmNoList;
                for (cnt = 0; cnt < kLmList; ++cnt) {
                    uint32_t mn = kLmNoList;
#pragma unroll
                    for (uint32_t u = 0; u < PER; ++u) {
                        const uint32_t s = code(u) >> 6;
                        if (code(u) != kCodeSkip && (int32_t)s > lo) mn = min(mn, s);
                    }
                    mn = grp_min(mn);
                    if (mn == kLmNoList) break;
                    if (l == cnt) Lr = mn;
                    lo = (int32_t)mn;
                }
                uint32_t nx = kLmNoList;
#pragma unroll
                for (uint32_t u = 0; u < PER; ++u)
                    if (code(u) != kCodeSkip && (int32_t)(code(u) >> 6) > lo) nx = min(nx, code(u) >> 6);
                more = cnt == kLmList && grp_min(nx) != kLmNoList;
                if (l < cnt) {
                    __builtin_amdgcn_s_waitcnt(0);   // the group's stores of T's row (pass 0) have landed
                    P = tsl[Lr];
                    need = !(!shared && P != DM_LM_NONE && lm.owner[P] == gT);
                }
            }
            const uint32_t gmask = (uint32_t)(__ballot(need) >> gshift) & ((1u << kLmLanes) - 1u);
            if (need) {
                NP = lm.frees[alloc + __builtin_popcount(gmask & ((1u << l) - 1u))];
                lm.owner[NP] = gT;
                ++taken;
            }
            alloc += __builtin_popcount(gmask);
            // ---- 2. the table: the new pages into T's slots (a later pass: T's slot may have
            // been written by this group above -- the same wave, in order)
            if (pass == 0 && copy) {
                // X's row to T, four words a lane (each group instruction moves 128 contiguous
                // bytes), with this pass's new pages; the trail's words as they are
                if (l < kLmList) {
                    s_np[2 * l] = Lr;
                    s_np[2 * l + 1] = NP;
                }
                const uint32_t lmin = cnt ? grp_get(Lr, 0) : 1u, lmax = cnt ? grp_get(Lr, cnt - 1) : 0u;
                const uint32_t toff = lm_trail_off(lm), nq = toff / 4u + lm_hw_word(xsl[toff - 1u]);
                wave_sync();
                for (uint32_t q = l; q < nq; q += kLmLanes) {
                    uint4 w4 = reinterpret_cast<const uint4*>(xsl)[q];
                    if (4 * q + 3 >= lmin && 4 * q <= lmax) {
                        uint32_t v[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
                        for (uint32_t e = 0; e < 4; ++e)
                            for (uint32_t r = 0; r < cnt; ++r)
                                if (s_np[2 * r] == 4 * q + e && s_np[2 * r + 1] != DM_LM_NONE) v[e] = s_np[2 * r + 1];
                        w4 = make_uint4(v[0], v[1], v[2], v[3]);
                    }
                    reinterpret_cast<uint4*>(tsl)[q] = w4;
                }
                if (l == 0) lm.ctr[T] = lm.ctr[X];
            } else if (need) {
                if (pass != 0) __builtin_amdgcn_s_waitcnt(0);
                tsl[Lr] = NP;
            }
            if (pass == 0) dirty = (flags & kJobMoved) != 0;
            // ---- 3. the pass's pages, kLmStage at a time through LDS
            for (uint32_t r0 = 0; r0 < cnt; r0 += kLmStage) {
                uint32_t Ls[kLmStage], Ps[kLmStage], Ds[kLmStage];
#pragma unroll
                for (uint32_t rr = 0; rr < kLmStage; ++rr) {
                    Ls[rr] = grp_get(Lr, r0 + rr);                 // kLmNoList beyond cnt
                    Ps[rr] = grp_get(P, r0 + rr);
                    const uint32_t npr = grp_get(NP, r0 + rr);
                    Ds[rr] = npr != DM_LM_NONE ? npr : Ps[rr];
                }
                if (pass != 0 || r0 != 0) {   // (pass 0's first stage was issued with the record)
                    wave_sync();              // the previous stage's stores have read LDS
                    stage_pages(Ls, Ps);
                }
                __builtin_amdgcn_s_waitcnt(0);
                wave_sync();
                if (pass == 0 && r0 == 0) ESLAM_STAMP(g_stamps_mg, 2);
                uint32_t wbits = 0;           // bit 8 rr + row: this lane wrote that 64-byte row of page rr
                // the stage's patches listed in scan order (k = l + kLmLanes u is u-major), then
                // applied kLmLanes at a time: a round's lanes on one cell go by rank (DPP row
                // compare), rounds in order -- every cell sees its patches in scan order
                // an entry: patch k, its staged page rr and its cell ci (k | rr << 8 | ci << 10)
                uint32_t nst = 0;
#pragma unroll
                for (uint32_t u = 0; u < PER; ++u) {
                    const uint32_t cu = code(u);
                    bool in = false;
                    uint32_t ru = 0;
#pragma unroll
                    for (uint32_t w = 0; w < kLmStage; ++w) {
                        const bool m = cu != kCodeSkip && Ls[w] == (cu >> 6);
                        in |= m;
                        ru = m ? w : ru;
                    }
                    const uint32_t gm = (uint32_t)(__ballot(in) >> gshift) & ((1u << kLmLanes) - 1u);
                    if (in)
                        s_lst[nst + __builtin_popcount(gm & ((1u << l) - 1u))] =
                            (uint16_t)((l + kLmLanes * u) | (ru << 8) | ((cu & 63u) << 10));
                    nst += __builtin_popcount(gm);
                }
                wave_sync();
                for (uint32_t j0 = 0; j0 < nst; j0 += kLmLanes) {
                    const bool act = j0 + l < nst;
                    const uint32_t e = act ? (uint32_t)s_lst[j0 + l] : 0u;
                    const uint32_t k = e & 0xffu;
                    // the patch first (every lane: k = 0 is a patch of the part), so a large part's
                    // load overlaps the ranking below
                    double2 sp;
                    if constexpr (kSpLds) {
                        sp = s_sp[k];
                    } else {
                        const ScanPatch* spk = mp.sp + k;
                        sp = make_double2(spk->z, spk->stdev);
                    }
                    const uint32_t c = act ? (e >> 8) : 0xfffffffeu - l;   // page and cell; idle lanes never match
                    const uint32_t rank = row_rank(c, l);
                    const uint32_t maxr = grp_max(act ? rank : 0u);
                    const uint32_t rr = (e >> 8) & 3u, ci = e >> 10;
                    // the patch, and for an empty cell the shared grid covers its occupancy word
                    // and record, are loaded together ahead of the ranks (cells are never emptied)
                    uint4 gct = make_uint4(0u, 0u, 0u, 0u);
                    uint32_t gocc = 0;
                    if (act) {
                        const float2 cv0 = *reinterpret_cast<const float2*>(stage + lm_stage_off(rr, ci, g));
                        if ((flags & kJobCovered) && !dm_lm_holds(cv0.y)) {
                            uint32_t sl = Ls[0];
#pragma unroll
                            for (uint32_t w = 1; w < kLmStage; ++w) sl = rr == w ? Ls[w] : sl;
                            const uint32_t sb = lm_div(sl, lm.mx), sa = sl - lm.wx * sb;
                            const uint32_t cm = 8u * (uint32_t)lm_tile(sa, na, lm.hx, lm.wx, lm.mx, lm.bx) + (ci & 7u);
                            const uint32_t cn = 8u * (uint32_t)lm_tile(sb, nb, lm.hy, lm.wy, lm.my, lm.by) + (ci >> 3);
                            const uint64_t cell = (uint64_t)cn * map.width + cm;
                            gocc = (map.occ[cell >> 5] >> (cell & 31u)) & 1u;
                            gct = map.cell_tab[cell];
                        }
                    }
                    for (uint32_t rk = 0; rk <= maxr; ++rk) {
                        if (act && rank == rk) {
                            float2* cp = reinterpret_cast<float2*>(stage + lm_stage_off(rr, ci, g));
                            const float2 cv = *cp;
                            const double wz = sp.x + z;
                            const double var = sp.y * sp.y + zvar;
                            float mo = cv.x, so = cv.y;
                            bool w = true, ins = true;
                            if (dm_lm_holds(cv.y)) {
                                w = dm_lm_fuse(cv.x, cv.y, wz, var, &mo, &so);
                                ins = false;
                            } else if (gocc) {
                                // a cell the shared grid covers: the particle's copy starts from
                                // the grid's patch the 3-sigma gate picks (the oracle alike)
                                double gm, gs;
                                if (grid_cell_patch(map, gct, wz, var, gm, &gs) &&
                                    dm_lm_fuse((float)gm, (float)gs, wz, var, &mo, &so)) {
                                    ins = false;
                                    covw = true;
                                }
                            }
                            if (ins) { mo = (float)wz; so = (float)dm_sqrt(var); }
                            if (w) {
                                *cp = make_float2(mo, so);
                                wbits |= 1u << (8u * rr + (ci >> 3));
                                ++written;
                            }
                        }
                        wave_sync();
                    }
                }
                wbits = grp_or(wbits);
                if (pass == 0 && r0 == 0) ESLAM_STAMP(g_stamps_mg, 3);
                static_assert(kLmStage <= 4 && kLmChunk == 128, "a lane's 16 bytes of a chunk lie in row 2 h + l / 4");
                // a new page goes back whole; a page the table owns, only the rows the patches changed
#pragma unroll
                for (uint32_t rr = 0; rr < kLmStage; ++rr) {
                    const uint32_t rows = (wbits >> (8u * rr)) & 0xffu;
                    const bool fresh = Ds[rr] != Ps[rr];
                    if (Ls[rr] == kLmNoList || (!fresh && !rows)) continue;
                    uint4* dp = reinterpret_cast<uint4*>(lm.page + (uint64_t)Ds[rr] * DM_LM_PAGE_CELLS);
#pragma unroll
                    for (uint32_t h = 0; h < kLmNq; ++h)
                        if (fresh || ((rows >> (2u * h + (l >> 2))) & 1u))
                            dp[kLmLanes * h + l] = *reinterpret_cast<const uint4*>(stage + (rr * kLmNq + h) * 1024 + (tid & 63u) * 16);
                }
                dirty = dirty || wbits != 0;
            }
            if (!more) break;
        }
        ESLAM_STAMP(g_stamps_mg, 4);
        if (shared && dirty) moved = true;
        if ((gath || moved) && l == 0) st.sid[i] = moved ? T : X;
        // the map now holds a copy of a shared-grid cell: its lookups ask its own cells first
        // (after T's row words have landed: the copy above may have written this word)
        if (grp_or(covw ? 1u : 0u) && l == 0) {
            __builtin_amdgcn_s_waitcnt(0);
            tsl[lm_trail_off(lm) - 2u] = kLmShadow;
        }
    } else if (valid && gath && l == 0) {
        st.sid[i] = X;
    }
    // the counters: particles once (the group's lane 0), cell writes and pages from every lane
    // (the plan counted the dropped and covered patches)
    const bool lead = l == 0;
    written = wave_sum_u32(written);
    taken = wave_sum_u32(taken);
    const uint64_t dmask = __ballot(lead && dirty), mmask = __ballot(lead && moved);
    if ((tid & 63u) == 0) {                   // one address per counter slot: no single hot atomic
        const uint32_t slot_c = (uint32_t)((blockIdx.x * (kLmMergeBlock / 64) + (tid >> 6)) % kMergeCounterSlots);
        if (written) atomicAdd((unsigned long long*)&mp.cnt[4 * kMergeCounterSlots + slot_c], (unsigned long long)written);
        if (taken) atomicAdd((unsigned long long*)&mp.cnt[5 * kMergeCounterSlots + slot_c], (unsigned long long)taken);
        if (dmask) atomicAdd((unsigned long long*)&mp.cnt[kMergeCounterSlots + slot_c], (unsigned long long)__popcll(dmask));
        if (mmask) atomicAdd((unsigned long long*)&mp.cnt[2 * kMergeCounterSlots + slot_c], (unsigned long long)__popcll(mmask));
    }
    ESLAM_STAMP(g_stamps_mg, 5);
}

// processMap(scanMap, match = true) per particle (the oracle's or_map_match; the rule is the
// build's own, envire's MLSGrid::match not being in the reference): every 10th scan patch,
// placed like the merge, scores on the cell it lands in -- a cell of the shared grid: the
// patch getPatch's 3-sigma gate picks (0 when none passes); with per-particle maps (PMAPS) an
// empty grid cell of the particle's own map, in a tile inside the window the update centres on
// the particle (from the window or the trail): its cell -- exp(-d^2 / (2 sigma^2)), sigma 0.2f
// (src/EmbodiedSlamFilter.cpp:217); the particle's weight is multiplied by pow(weight, 0.1f),
// weight the float mean score (1 when no patch counts).  A lane per particle; the sampled
// patches from the kernel arguments (scalar loads), kMatchBatch at a time: their grid records
// and table slots in one round trip, then the cells.
template <bool PMAPS>
__global__ void __launch_bounds__(kBlock) k_map_match(DevState s0, DevState s1, const Ctl* __restrict__ ctl, MapView map,
                                                      LocalMaps lm, MatchParams mp)
{
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= mp.n) return;
    const DevState st = (ctl->base ^ ctl->flip) ? s1 : s0;
    const uint32_t X = PMAPS ? st.sid[i] : 0u;
    const double x = st.x[i], y = st.y[i], th = st.th[i], z = st.z[i], zs = st.zs[i], w = st.w[i];
    const double bx = x - map.offset_x, by = y - map.offset_y;
    if (!(dm_isfinite(bx) && dm_isfinite(by) && dm_isfinite(th))) return;
    double sn, co;
    dm_sincos(th, &sn, &co);
    const double zvar = zs * zs;
    const double* A = map.g2l;
    int32_t na = 0, nb = 0;
    int2 c = make_int2(0, 0);
    const uint32_t* row = nullptr;
    if constexpr (PMAPS) {
        if (mp.is_id) {
            na = dm_lm_centre(x, map.offset_x, map.inv_scale_x);
            nb = dm_lm_centre(y, map.offset_y, map.inv_scale_y);
        } else {
            na = dm_lm_centre(((A[0] * x + A[1] * y) + A[2] * z) + A[3], map.offset_x, map.inv_scale_x);
            nb = dm_lm_centre(((A[4] * x + A[5] * y) + A[6] * z) + A[7], map.offset_y, map.inv_scale_y);
        }
        c = lm.ctr[X];
        row = lm.slot + (uint64_t)X * lm.S;
    }
    double sum = 0.0;
    uint32_t cnt = 0;
    constexpr uint32_t kMatchBatch = 8;
    for (uint32_t k0 = 0; k0 < mp.m; k0 += kMatchBatch) {
        uint4 ct[kMatchBatch];
        uint32_t pg[kMatchBatch], cj[kMatchBatch], sl[kMatchBatch];
        double wzs[kMatchBatch], lzs[kMatchBatch], var[kMatchBatch];
        bool on[kMatchBatch], own[kMatchBatch];
#pragma unroll
        for (uint32_t q = 0; q < kMatchBatch; ++q) {
            const uint32_t k = k0 + q;
            on[q] = own[q] = false;
            ct[q] = make_uint4(0u, 0u, 0u, 0u);
            pg[q] = DM_LM_NONE;
            cj[q] = sl[q] = 0;
            wzs[q] = lzs[q] = var[q] = 0.0;
            if (k >= mp.m) continue;
            const ScanPatch sp = mp.sp ? mp.sp[k] : mp.spi[k];
            const double wz = sp.z + z;
            double lz = wz;
            uint32_t cm, cn;
            if (mp.is_id) {
                if (dm_merge_cell_mn(bx, by, co, sn, sp.x, sp.y, map.inv_scale_x, map.inv_scale_y, map.width,
                                     map.height_cells, &cm, &cn) == 0xffffffffu)
                    continue;
            } else {
                const double wx = (co * sp.x + (-sn) * sp.y) + x;
                const double wy = (sn * sp.x + co * sp.y) + y;
                const double lx = ((A[0] * wx + A[1] * wy) + A[2] * wz) + A[3];
                const double ly = ((A[4] * wx + A[5] * wy) + A[6] * wz) + A[7];
                lz = ((A[8] * wx + A[9] * wy) + A[10] * wz) + A[11];
                const double fm = floor((lx - map.offset_x) * map.inv_scale_x);
                const double fn = floor((ly - map.offset_y) * map.inv_scale_y);
                if (!((fm >= 0.0) & (fm < (double)map.width) & (fn >= 0.0) & (fn < (double)map.height_cells))) continue;
                cm = (uint32_t)fm;
                cn = (uint32_t)fn;
            }
            on[q] = true;
            wzs[q] = wz;
            lzs[q] = lz;
            var[q] = sp.stdev * sp.stdev + zvar;
            ct[q] = map.cell_tab[(uint64_t)cn * map.width + cm];
            if constexpr (PMAPS) {
                const uint32_t a = cm >> DM_LM_TILE_BITS, b = cn >> DM_LM_TILE_BITS;
                if (dm_lm_inside(a, na, lm.hx, lm.wx) && dm_lm_inside(b, nb, lm.hy, lm.wy)) {
                    own[q] = true;
                    cj[q] = (cm & 7u) + 8u * (cn & 7u);
                    const bool inw = dm_lm_inside(a, c.x, lm.hx, lm.wx) && dm_lm_inside(b, c.y, lm.hy, lm.wy);
                    sl[q] = inw ? row[lm_mod(a, lm.wx, lm.mx) + lm.wx * lm_mod(b, lm.wy, lm.my)] : DM_LM_NONE;
                    if (!inw) {                  // a tile the window has left: the trail (rare)
                        const uint4* t = reinterpret_cast<const uint4*>(row + lm_trail_off(lm));
                        const uint32_t hw = lm_hw_word(row[lm_trail_off(lm) - 1u]);
                        for (uint32_t e = 0; e < hw; ++e) {
                            const uint4 v = t[e];
                            if (v.z != DM_LM_NONE && v.x == a && v.y == b) sl[q] = v.z;
                        }
                    }
                }
            }
        }
        float2 cv[kMatchBatch];
#pragma unroll
        for (uint32_t q = 0; q < kMatchBatch; ++q) {
            pg[q] = (PMAPS && own[q]) ? sl[q] : DM_LM_NONE;
            cv[q] = pg[q] != DM_LM_NONE ? lm.page[(uint64_t)pg[q] * DM_LM_PAGE_CELLS + cj[q]] : make_float2(0.0f, -1.0f);
        }
#pragma unroll
        for (uint32_t q = 0; q < kMatchBatch; ++q) {
            if (!on[q]) continue;
            if (pg[q] != DM_LM_NONE && dm_lm_holds(cv[q].y)) {     // the particle's own cell first
                const double d = wzs[q] - (double)cv[q].x;
                sum += dm_exp(-(d * d) / (2.0 * kMatchSigma * kMatchSigma));
                ++cnt;
            } else if (ct[q].w != 0u) {          // a cell of the shared grid
                double mean;
                if (grid_cell_patch(map, ct[q], lzs[q], var[q], mean)) {
                    const double d = lzs[q] - mean;
                    sum += dm_exp(-(d * d) / (2.0 * kMatchSigma * kMatchSigma));
                }
                ++cnt;
            }
        }
    }
    const float wf = cnt ? (float)(sum / (double)cnt) : 1.0f;
    st.w[i] = w * dm_pow((double)wf, (double)0.1f);
}

// the merge's statistics slots -> ctl (one block of kMergeCounterSlots threads); the free
// list's cursor moves past this update's plan
__global__ void __launch_bounds__(kMergeCounterSlots) k_merge_counts(const uint64_t* __restrict__ cnt, Ctl* __restrict__ ctl,
                                                                      uint32_t acc)
{
    __shared__ uint64_t s[kMergeCounters][kMergeCounterSlots / 64];
    const uint32_t t = threadIdx.x;
#pragma unroll
    for (uint32_t g = 0; g < kMergeCounters; ++g) {
        const uint64_t v = wave_sum_u64(cnt[g * kMergeCounterSlots + t]);
        if ((t & 63u) == 0) s[g][t >> 6] = v;
    }
    __syncthreads();
    if (t == 0) {
        uint64_t r[kMergeCounters] = {0, 0, 0, 0, 0, 0, 0};
        for (uint32_t g = 0; g < kMergeCounters; ++g)
            for (uint32_t w = 0; w < kMergeCounterSlots / 64; ++w) r[g] += s[g][w];
        // acc: a later part of a scan merged 64 patches at a time (eslam_gpu_map_update) adds
        if (acc) {
            ctl->map_dropped += r[0]; ctl->map_changed += r[1]; ctl->map_copied += r[2];
            ctl->map_covered += r[3]; ctl->map_written += r[4]; ctl->map_taken += r[5];
            ctl->map_evicted += r[6];
        } else {
            ctl->map_dropped = r[0]; ctl->map_changed = r[1]; ctl->map_copied = r[2];
            ctl->map_covered = r[3]; ctl->map_written = r[4]; ctl->map_taken = r[5];
            ctl->map_evicted = r[6];
        }
        if (!(ctl->err & kFaultPages)) ctl->pg_cursor += ctl->pg_total;
    }
}

// the free list's cursor moves past a plan (the received maps' pages)
__global__ void k_pg_advance(Ctl* __restrict__ ctl)
{
    if (!(ctl->err & kFaultPages)) ctl->pg_cursor += ctl->pg_total;
}

// ---------------------------------------------------------------------------------------
// k_weight_stats: exact sum of the weights and of their squares (standalone
// getWeightsSum / normalizeWeights / resample, src/ParticleFilter.hpp:34-70)
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) k_weight_stats(DevState s0, DevState s1, uint64_t n, uint32_t J,
                                                         Ctl* __restrict__ ctl, Shard* __restrict__ shards)
{
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint64_t lbase = ((uint64_t)blockIdx.x * kWaves + wave) * 64ull * J;
    const DevState st = (ctl->base ^ ctl->flip) ? s1 : s0;
    const int wexp = ctl->wexp;
    double a = 0.0, b = 0.0;
    for (uint32_t j = 0; j < J; ++j) {
        const uint64_t i = lbase + 64ull * j + lane;
        if (i >= n) continue;
        const double w = st.w[i];
        a = a + w;
        b = b + w * w;
    }
    __shared__ uint32_t s_limb[kWaves][2][4];
    __shared__ uint32_t s_flag[kWaves];
    uint32_t flag = 0;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        double v = q == 0 ? a : b;
        uint32_t l[4] = {0, 0, 0, 0};
        if (__ballot(v != 0.0) != 0ull) {
            v = wave_sum_butterfly(v);
            if (v != v) flag |= 1u << (q * DM_NBUCKETS);
            else if (!dm_isfinite(v)) flag |= 1u << (q * DM_NBUCKETS + 16);
            else dm_fx128_limbs(v, q == 0 ? DM_FX_SCALE - wexp : DM_FX_SCALE - 2 * wexp, l);
        }
        if (lane == 0) for (int j = 0; j < 4; ++j) s_limb[wave][q][j] = l[j];
    }
    if (lane == 0) s_flag[wave] = flag;
    __syncthreads();
    Shard* sh = shards + (blockIdx.x % kNShard);
    const int t = threadIdx.x;
    if (t < 8) {
        const int q = t >> 2, j = t & 3;
        uint64_t v = 0;
        for (int wv = 0; wv < kWaves; ++wv) v += s_limb[wv][q][j];
        if (v) atomicAdd((unsigned long long*)(q == 0 ? &sh->A[0][j] : &sh->B[0][j]), (unsigned long long)v);
    } else if (t == 64) {
        uint32_t f = 0;
        for (int wv = 0; wv < kWaves; ++wv) f |= s_flag[wv];
        if (f) atomicOr((unsigned long long*)&sh->flags, (unsigned long long)f);
    }
}

// ---------------------------------------------------------------------------------------
// k_finalize: one block.  Sums the shards exactly, then the scalar part of the update.
// ---------------------------------------------------------------------------------------
constexpr int kShardFields = 2 * DM_NBUCKETS * 4 + 4 + 5 + 4;   // A, B, SW, D, TP, maxm, flags, err, bbox

__device__ __forceinline__ double acc_value(const uint64_t* L, uint64_t flags, int qbit, int scale)
{
    if (flags & (1ull << qbit)) return __builtin_nan("");
    if (flags & (1ull << (qbit + 16))) return __builtin_inf();
    return dm_limbs_to_double(L, scale);
}

// combine field t of nrec statistics records exactly (sum / max / or by field) and zero them
// (exact integers: any grouping gives the same value)
__device__ __forceinline__ uint64_t reduce_field(Shard* recs, int nrec, int t)
{
    constexpr int kCap = kNShard;
    uint64_t acc = 0;
    const int base = 2 * DM_NBUCKETS * 4 + 4;                                  // D
    for (int k0 = 0; k0 < nrec; k0 += kCap) {
        // a group's loads first (they are independent), then combine: one memory latency
        uint64_t v[kCap];
#pragma unroll
        for (int k = 0; k < kCap; ++k) v[k] = k0 + k < nrec ? reinterpret_cast<const uint64_t*>(recs + k0 + k)[t] : 0ull;
#pragma unroll
        for (int k = 0; k < kCap; ++k)
            if (k0 + k < nrec) reinterpret_cast<uint64_t*>(recs + k0 + k)[t] = 0;
#pragma unroll
        for (int k = 0; k < kCap; ++k) {
            if (k0 + k >= nrec) break;
            if (t == base + 2 || t >= base + 5) acc = acc > v[k] ? acc : v[k];      // maxm, bbox
            else if (t == base + 3 || t == base + 4) acc |= v[k];                   // flags, err
            else acc += v[k];
        }
    }
    return acc;
}

// LDS of the finalize: the combined shard fields, the exact sums A_b, B_b, SW as doubles and
// the phase-B factors
struct FinLds {
    uint64_t s[kShardFields];
    double acc[2 * DM_NBUCKETS + 1];
    double f[DM_NBUCKETS];
};

// the finalize of one block (every thread calls it).  recs: kNShard local shards (one GPU)
// or the gathered per-rank records (multi-GPU)
__device__ __forceinline__ void finalize_block(Shard* __restrict__ recs, int nrec, Ctl* __restrict__ ctl, const FinParams& fp, FinLds& L)
{
    uint64_t* s = L.s;
    double* s_acc = L.acc;
    double* s_f = L.f;
    const int t = threadIdx.x;
    // the control fields the finalize reads, loaded with the shards (one memory round trip)
    const int wexp_ = ctl->wexp;
    uint32_t base0 = 0, flip0 = 0, minstd0 = 0;
    double last_max = 0.0;
    uint64_t updates0 = 0;
    if (t == 0) {
        base0 = ctl->base; flip0 = ctl->flip; minstd0 = ctl->minstd;
        last_max = ctl->max_weight; updates0 = ctl->update_count;
    }
    if (t < kShardFields) {
        s[t] = reduce_field(recs, nrec, t);
        // multi-GPU: the local shards were all-gathered (stream order: already read)
        if (fp.local_shards)
            for (int k = 0; k < kNShard; ++k) reinterpret_cast<uint64_t*>(fp.local_shards + k)[t] = 0;
    }
    __syncthreads();
    {
        // the 13 fixed-point -> double conversions, one per lane (same values as serially)
        const uint64_t flags_ = s[2 * DM_NBUCKETS * 4 + 7];
        if (t < 2 * DM_NBUCKETS + 1) {
            const int scale = t < DM_NBUCKETS ? DM_FX_SCALE - wexp_
                            : (t < 2 * DM_NBUCKETS ? DM_FX_SCALE - 2 * wexp_ : DM_FX_SCALE);
            s_acc[t] = acc_value(s + 4 * t, flags_, t, scale);
        }
        __syncthreads();
        // phase-B factors (0.9 fw)^(4 - n), one bucket per lane
        if (fp.mode == FIN_UPDATE && t < DM_NBUCKETS) {
            const uint64_t D_ = s[2 * DM_NBUCKETS * 4 + 4];
            const double fw_ = D_ > 0 ? s_acc[2 * DM_NBUCKETS] / (double)D_ : 1.0;
            s_f[t] = dm_pow(fp.discount * fw_, (double)(uint64_t)(4ull - (uint64_t)t));
        }
        __syncthreads();
    }
    if (t != 0) return;

    const uint64_t D = s[2 * DM_NBUCKETS * 4 + 4];
    const uint64_t TP = s[2 * DM_NBUCKETS * 4 + 5];
    const double maxm = dm_from_bits(s[2 * DM_NBUCKETS * 4 + 6]);
    const uint64_t err = s[2 * DM_NBUCKETS * 4 + 8];
    if (s[2 * DM_NBUCKETS * 4 + 10]) {                 // a weighting kernel saw particles
        for (int q = 0; q < 4; ++q) ctl->bbox[q] = s[2 * DM_NBUCKETS * 4 + 9 + q];
    }
    // commit the previous resample's buffer flip
    ctl->base = base0 ^ flip0;
    ctl->flip = 0;
    ctl->gather = 0;
    if (err) atomicOr((unsigned long long*)&ctl->err, (unsigned long long)err);   // K3 blocks may OR in too
    ctl->tile_counter = 0;
    ctl->overruns = 0;
    ctl->aborted = 0;
    const double N = (double)fp.n_global;
    if (fp.mode == FIN_UPDATE && err) {
        // evaluatePose threw (src/ContactModel.cpp:122-123): updateWeights stops after its
        // particle loop has run, before the floating weight, phase B, the max-weight update,
        // normalizeWeights and resample (src/PoseEstimator.cpp:276-352, 244-255)
        ctl->aborted = 1;
        ctl->resample = 0;
        if (fp.mirror) { fp.mirror[0] = 0; fp.mirror[1] = ctl->minstd_start; fp.mirror[2] = (uint64_t)(int64_t)ctl->scan_shift; }
        return;
    }

    double S = 0.0, Q = 0.0;
    if (fp.mode == FIN_UPDATE) {
        const double SW = s_acc[2 * DM_NBUCKETS];
        const double fw = D > 0 ? SW / (double)D : 1.0;
        for (int b = 0; b < DM_NBUCKETS; ++b) {
            const double fb = s_f[b];
            ctl->f[b] = fb;
            S = S + fb * s_acc[b];
            Q = Q + (fb * fb) * s_acc[DM_NBUCKETS + b];
        }
        ctl->fw = fw;
        const double last = last_max;
        double mw = maxm;
        if (TP == 0) mw = last * fp.discount;
        ctl->max_weight = mw;
        ctl->data_particles = D;
        ctl->total_points = TP;
        ctl->update_count = updates0 + 1;
    } else {
        S = s_acc[0];
        Q = s_acc[DM_NBUCKETS];
        for (int b = 0; b < DM_NBUCKETS; ++b) ctl->f[b] = 1.0;
    }
    ctl->S = S;
    ctl->Q = Q;
    ctl->inv_n = 1.0 / N;

    if (fp.mode == FIN_UPDATE || fp.mode == FIN_NORMALIZE) {
        double eff;
        ctl->uniform = 0;
        if (S <= 0.0) {
            ctl->uniform = 1;
            eff = 1.0 / (1.0 / N);
        } else {
            eff = 1.0 / (Q / (S * S));
        }
        ctl->eff = eff;
        ctl->wexp = 1;
        ctl->scan_shift = 60;
        ctl->resample = (fp.mode == FIN_UPDATE && eff < (double)fp.min_effective) ? 1u : 0u;
    } else if (fp.mode == FIN_RESAMPLE) {
        ctl->resample = 1;
        ctl->scan_shift = 61 - (dm_weight_exp(S) + 1);
    } else {
        ctl->resample = 0;
    }
    if (fp.mirror) {
        fp.mirror[0] = ctl->resample;
        fp.mirror[1] = ctl->resample ? minstd0 : ctl->minstd_start;      // minstd_start below
        fp.mirror[2] = (uint64_t)(int64_t)ctl->scan_shift;
    }
    if (ctl->resample) {
        ctl->minstd_start = minstd0;
        ctl->minstd = dm_mulmod31(fp.minstd_jump_n, minstd0);       // A^N, precomputed
        ctl->flip = 1;
        ctl->gather = 1;
    }
}

__global__ void __launch_bounds__(kBlock) k_finalize(Shard* __restrict__ recs, int nrec, Ctl* __restrict__ ctl, FinParams fp)
{
    __shared__ FinLds L;
    finalize_block(recs, nrec, ctl, fp, L);
}

// ---------------------------------------------------------------------------------------
// count of stratified draws T_k = fx(((k + U_k) / N), shift) that are <= c
// (U_k = boost uniform_real of the (k+1)-th minstd draw after x_start)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t fx_shift(double v, int shift) { return dm_fx_shift(v, shift); }

// dm_fx_shift(q, shift) for 0 <= q <= 1 without branches: then sh = e - 1075 + shift <= 9
// (shift <= 61), inside the general function's "m << sh" range, and q = +0 or subnormal
// (e = 0) gives 0 as there
__device__ __forceinline__ uint64_t fx_unit(double q, int shift)
{
    const uint64_t b = dm_bits(q);
    const uint32_t e = (uint32_t)(b >> 52);
    const uint64_t m = (b & 0x000fffffffffffffull) | 0x0010000000000000ull;
    const int sh = (int)e - 1075 + shift;
    const uint64_t r = sh >= 0 ? (m << (sh & 63)) : (m >> ((-sh) & 63));
    return ((e == 0u) | (sh <= -64)) ? 0ull : r;
}

// T_k = fx((k + U_k) / N): both divisions as dm_div_recip (bit-identical to "/", checked by
// tests/c/check_div.c); inv_N = 1.0 / N.  k < N < 2^32, so (k + U_k) / N <= 1.
__device__ __forceinline__ uint64_t draw_fx(uint64_t k, uint32_t x, double dN, double inv_N, int shift)
{
    return fx_unit(dm_div_recip((double)(uint32_t)k + dm_minstd_uniform_fast(x), dN, inv_N), shift);
}

__device__ __forceinline__ uint64_t count_draws_le(uint64_t c, uint64_t N, uint32_t xs, int shift,
                                                   const uint32_t* __restrict__ jt)
{
    const unsigned __int128 prod = (unsigned __int128)c * N;
    const uint64_t kstar = (uint64_t)(prod >> shift);
    const uint64_t k0 = kstar >= 1 ? kstar - 1 : 0;
    if (k0 >= N) return N;
    uint64_t cnt = k0;
    uint32_t x = dm_mulmod31(jump_pow(jt, k0 + 1), xs);
    const double dN = (double)N, inv_N = 1.0 / dN;
    for (uint64_t k = k0; k <= kstar + 1 && k < N; ++k) {
        const uint64_t T = draw_fx(k, x, dN, inv_N, shift);
        if (T <= c) cnt = k + 1;
        else break;
        x = dm_minstd_next(x);
    }
    return cnt;
}

// phase B (updateWeights' second pass, src/PoseEstimator.cpp:332-344) + normalisation
// (src/ParticleFilter.hpp:46-70) of one tile's items r * kBlock + tid, in place; v[r] is the
// final weight (0 past the filter's end).  Every load of the tile is issued first (indices
// clamped into the filter: no branches between them), so their latencies overlap instead of
// costing one memory round trip per item.
__device__ __forceinline__ uint32_t sgpr_u32(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ double sgpr_f64(double v)
{
    const uint64_t b = dm_bits(v);
    return dm_from_bits(((uint64_t)sgpr_u32((uint32_t)(b >> 32)) << 32) | sgpr_u32((uint32_t)b));
}

template <int ITEMS>
__device__ __forceinline__ void phase_b_load(const DevState& st, const ScanParams& sp, uint64_t t0, uint32_t tid,
                                             double (&v)[ITEMS], double (&mp)[ITEMS], uint32_t (&fl)[ITEMS])
{
    const uint64_t last = sp.n - 1;
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const uint64_t i = t0 + (uint64_t)(r * kBlock + (int)tid);
        v[r] = st.w[(i < sp.n ? i : last)];
    }
    if (sp.phase_b) {
#pragma unroll
        for (int r = 0; r < ITEMS; ++r) {
            const uint64_t i = t0 + (uint64_t)(r * kBlock + (int)tid);
            const uint64_t ic = i < sp.n ? i : last;
            fl[r] = st.flags[ic];
            mp[r] = st.mprob[ic];
        }
    }
}

// ctl: k_finalize's outputs (S, uniform, inv_n, f)
template <int ITEMS>
__device__ __forceinline__ void phase_b_apply(const DevState& st, const ScanParams& sp, const Ctl* ctl, uint64_t t0,
                                              uint32_t tid, double (&v)[ITEMS], const double (&mp)[ITEMS],
                                              const uint32_t (&fl)[ITEMS])
{
    // block-uniform values (the fused K3 reads them from LDS): kept in SGPRs
    const double S = sgpr_f64(ctl->S);
    const bool uniform = sgpr_u32(ctl->uniform) != 0;
    const double inv_n = sgpr_f64(ctl->inv_n);
    double f[DM_NBUCKETS];
#pragma unroll
    for (int b = 0; b < DM_NBUCKETS; ++b) f[b] = sgpr_f64(ctl->f[b]);
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const uint64_t i = t0 + (uint64_t)(r * kBlock + (int)tid);
        double x = v[r];
        if (sp.phase_b) {
            const uint32_t ncp = fl[r] & 0x7fu;
            const uint32_t bucket = ncp < DM_NBUCKETS - 1 ? ncp : DM_NBUCKETS - 1;
            double fb = f[0];
#pragma unroll
            for (int b = 1; b < DM_NBUCKETS; ++b) fb = (bucket == (uint32_t)b) ? f[b] : fb;
            const double factor = mp[r] * fb;
            x *= factor;
        }
        if (sp.normalize) x = uniform ? inv_n : x / S;
        if (i < sp.n) {
            if (sp.phase_b || sp.normalize) K1_ST(st.w + i, x);
        } else {
            x = 0.0;
        }
        v[r] = x;
    }
}

template <int ITEMS>
__device__ __forceinline__ void phase_b_tile(const DevState& st, const ScanParams& sp, const Ctl* ctl, uint64_t t0,
                                             uint32_t tid, double (&v)[ITEMS])
{
    double mp[ITEMS];
    uint32_t fl[ITEMS];
    phase_b_load<ITEMS>(st, sp, t0, tid, v, mp, fl);
    phase_b_apply<ITEMS>(st, sp, ctl, t0, tid, v, mp, fl);
}

// ---------------------------------------------------------------------------------------
// The fused finalize (one-GPU update step): block 0 of K3 runs k_finalize's block
// (finalize_block) and then publishes the launch's epoch in one word with an agent-scope
// release store; every block waits for that word (one lane polls, with a sleep) and copies
// the control block into LDS with agent-scope loads (its lines may be stale in this XCD's
// L2).  Block 0 is dispatched first and waits on nothing before it publishes, so the wait
// terminates; a bounded spin turns a violated assumption into ctl->err bit 2.  The epoch is
// a per-context launch counter: a word left by an earlier launch never equals it.
// ---------------------------------------------------------------------------------------
constexpr int kCtlWords = (int)(sizeof(Ctl) / 8);
static_assert(sizeof(Ctl) % 8 == 0 && kCtlWords <= 64, "the control block is copied by one wave");

// a cross-block wait gave up: poison the filter (kFaultTimeout in ctl->err, which every later
// launch checks, and in the host-mapped word the host checks before it trusts anything)
__device__ __forceinline__ void raise_timeout(Ctl* ctl, uint32_t* fault)
{
    atomicOr((unsigned long long*)&ctl->err, (unsigned long long)kFaultTimeout);
    if (fault) __hip_atomic_fetch_or(fault, kFaultTimeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// true (block-uniform) when the wait gave up: s_img is then not valid
__device__ __forceinline__ bool fin_wait_copy(Ctl* ctl, const uint64_t* fin_word, uint64_t epoch, uint64_t* s_img,
                                              const ScanParams& sp, uint32_t* s_flag)
{
    const uint32_t tid = threadIdx.x;
    if (tid < 64) {
        bool timeout = sp.spin_limit == 0;       // testing: give up at once
        if (tid == 0) {
            uint32_t spins = 0;
            // relaxed agent-scope polls and copies: on gfx950 an agent-scope atomic load reads
            // through this XCD's L2 to memory, where block 0's release store (a write-back of its
            // L2) has put the ctl lines.  Acquire loads (or an acquire fence) here invalidate
            // the L2 in every block: K3 53 -> 91 us at 4M, 18 -> 48 us at 256k (r03b).
            while (!timeout && atomic_load_agent(fin_word) != epoch) {
                if (spins++ >= sp.spin_limit) { timeout = true; break; }
                __builtin_amdgcn_s_sleep(8);
            }
            *s_flag = timeout ? 1u : 0u;
            if (timeout) raise_timeout(ctl, sp.fault);
        }
        // lane 0's verdict for the whole wave (the other lanes skip the copy's retry loop)
        timeout = __builtin_amdgcn_readfirstlane(timeout ? 1 : 0) != 0;
        // the copy must carry this launch's epoch (ctl->fin_epoch, written by block 0 before its
        // release): a stale copy of the line holding it would show an older one.  The relaxed
        // loads rely on gfx950's agent-scope loads missing this XCD's L2 for lines another XCD
        // wrote back.  Only the epoch's own 128-byte line is validated: were that assumption to
        // fail for another line of the block (resample, scan_shift, aborted sit in other lines),
        // this check would not see it -- it guards the common failure, not every one
        constexpr uint32_t kEpochWord = (uint32_t)(offsetof(Ctl, fin_epoch) / 8);
        if (!timeout) {
            uint64_t word = 0;
            for (int attempt = 0;; ++attempt) {
                if (tid < (uint32_t)kCtlWords) word = atomic_load_agent(reinterpret_cast<const uint64_t*>(ctl) + tid);
                if (!__any(tid == kEpochWord && word != epoch)) break;
                if (attempt == 64) {
                    if (tid == 0) { *s_flag = 1u; raise_timeout(ctl, sp.fault); }
                    break;
                }
                __builtin_amdgcn_s_sleep(8);
            }
            if (tid < (uint32_t)kCtlWords) s_img[tid] = word;
        }
    }
    __syncthreads();
    return *s_flag != 0u;
}

// ---------------------------------------------------------------------------------------
// k_normalize_scan (K3a): phase B + normalisation and the tile totals; k_segments (K3b):
// the prefix of the fixed-point weights and the segment boundaries.  No cross-tile waiting
// inside a kernel: K3b re-sums the preceding tile totals (exact integers, any order).
// ---------------------------------------------------------------------------------------


// In-tile exclusive prefix of this thread's first item (thread -> wave -> block).
// run = this thread's total; s_wtot: kWaves words of LDS.
__device__ __forceinline__ uint64_t block_excl(uint64_t run, uint64_t* s_wtot)
{
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    uint64_t tincl = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t t = __shfl_up(tincl, o, 64);
        if ((int)lane >= o) tincl += t;
    }
    if (lane == 63) s_wtot[wave] = tincl;
    __syncthreads();
    uint64_t wexcl = 0;
#pragma unroll
    for (int wv = 0; wv < kWaves; ++wv)
        if ((uint32_t)wv < wave) wexcl += s_wtot[wv];
    return wexcl + (tincl - run);
}

// mark the segment [lo, hi) (outputs relative to this rank's slice) with value v
__device__ __forceinline__ void mark_segment(uint32_t* __restrict__ marks, uint32_t* __restrict__ tile_first,
                                             uint64_t lo, uint64_t hi, uint32_t v)
{
    marks[lo] = v;
    for (uint64_t t = (lo + kRow - 1) / kRow; t * kRow < hi; ++t) tile_first[t] = v - 1u;
}

// LDS staging of one scan tile: values in particle order, skewed by one slot every 32
// doubles so both the striped writes and the blocked (8 per thread) reads are conflict-free
constexpr int kSkew = 32;

__device__ __forceinline__ int skew(int k) { return k + k / kSkew; }

// this thread's 8 consecutive values (blocked) -> fixed-point inclusive running sums
template <int ITEMS>
__device__ __forceinline__ uint64_t blocked_fx(const double* s_v, int shift, uint64_t (&c)[ITEMS])
{
    uint64_t run = 0;
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        run += fx_shift(s_v[skew((int)threadIdx.x * ITEMS + r)], shift);
        c[r] = run;
    }
    return run;
}

constexpr int kWaveChunks = 2;           // more draws than kWaveChunks * wave_draws: per-target windows

// stratified draws one wave holds in LDS at a time: its particles' share plus a row of slack
// (at least 576)
template <int ITEMS> constexpr int wave_draws() { return 64 * ITEMS + 64 > 576 ? 64 * ITEMS + 64 : 576; }

// the LDS slot of a wave's draw x, one pad slot per 8: a lane's window reads sit near draw
// 8 l + const (one target per particle, ITEMS = 8 particles per lane), and unpadded that stride
// of 8 doubles put lanes l and l + 4 on one bank (8-way within each 32-lane ds_read_b64 group);
// padded, the lanes' 8-byte reads cover the 64 banks once
__device__ __forceinline__ uint32_t draw_slot(uint32_t x) { return x + (x >> 3); }

// K3's LDS: the staged weights, then the wave's draws (the weights are dead before the
// draws are written)
template <int ITEMS> union K3Lds {
    double v[kBlock * ITEMS + kBlock * ITEMS / kSkew];
    uint64_t T[kWaves][wave_draws<ITEMS>() + wave_draws<ITEMS>() / 8];
};

// Write the marks of the tile's segment starts (relative to the slice) and the row carries
// of tile_first.  The marks buffer is all zero here (the gather clears every mark it
// reads), so only the segment starts are stored: direct stores measured ~1 µs faster per
// step than staging the tile's output range in LDS and writing it densely.
// seg_lo/seg_hi: this thread's segments (relative; empty when equal), val: their values.
template <int ITEMS>
__device__ __forceinline__ void flush_marks(uint32_t* __restrict__ marks, uint32_t* __restrict__ tile_first,
                                            const uint64_t (&seg_lo)[ITEMS], const uint64_t (&seg_hi)[ITEMS],
                                            const uint32_t (&val)[ITEMS])
{
#pragma unroll
    for (int q = 0; q < ITEMS; ++q) {
        const uint64_t lo = seg_lo[q], hi = seg_hi[q];
        if (hi <= lo) continue;
        marks[lo] = val[q];
        for (uint64_t t = (lo + kRow - 1) / kRow; t * kRow < hi; ++t) tile_first[t] = val[q] - 1u;
    }
}

// one segment's start mark and row carries (flush_marks for a single item)
__device__ __forceinline__ void flush_mark(uint32_t* __restrict__ marks, uint32_t* __restrict__ tile_first, uint64_t lo,
                                           uint64_t hi, uint32_t val)
{
    if (hi <= lo) return;
    marks[lo] = val;
    for (uint64_t t = (lo + kRow - 1) / kRow; t * kRow < hi; ++t) tile_first[t] = val - 1u;
}

constexpr uint64_t kPubMask = (1ull << 61) - 1;

// a tile's word into every replica (ScanParams::pub_stride), one lane each.  The sharded K3a
// writes every replica too (one thread): the words of a launch tag never outlive a launch in
// any copy, whichever kernel last wrote them
__device__ __forceinline__ void publish_tile(uint64_t* pub, uint32_t stride, uint32_t tile, uint64_t w)
{
    if (threadIdx.x < kPubReplicas) atomic_store_agent(pub + (uint64_t)threadIdx.x * stride + tile, w);
}
__device__ __forceinline__ void publish_tile_1(uint64_t* pub, uint32_t stride, uint32_t tile, uint64_t w)
{
#pragma unroll
    for (uint32_t r = 0; r < kPubReplicas; ++r) atomic_store_agent(pub + (uint64_t)r * stride + tile, w);
}

// sum of the published totals of tiles [0, count) (any order: exact integers).  Wave 0 reads
// them, 8 loads in flight per lane, and polls the unpublished ones with a sleep between
// polls (light on the memory system the tiles it waits for are still streaming through);
// the other waves wait at the barrier.
// A wait that gives up (sp.spin_limit polls) poisons the filter and returns ~0.
__device__ __forceinline__ uint64_t tiles_before_pub(const uint64_t* __restrict__ pub, uint32_t count, const ScanParams& sp,
                                                     uint64_t* s_red, Ctl* __restrict__ ctl)
{
    const uint32_t tag = sp.tag;
    const uint32_t tid = threadIdx.x;
    if (tid < 64) {
        uint64_t acc = 0;
        bool timeout = sp.spin_limit == 0 && count > 0;   // testing: give up at once
        for (uint32_t b0 = 0; !timeout && b0 < count; b0 += 8u * 64u) {
            uint64_t v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const uint32_t k = b0 + (uint32_t)q * 64u + tid;
                v[q] = k < count ? atomic_load_agent(pub + k) : ((uint64_t)tag << 61);
            }
            uint32_t spins = 0;
            for (;;) {
                bool ready = true;
#pragma unroll
                for (int q = 0; q < 8; ++q) ready &= (uint32_t)(v[q] >> 61) == tag;
                if (__ballot(!ready) == 0ull) break;
                if (spins++ >= sp.spin_limit) { timeout = true; break; }
                __builtin_amdgcn_s_sleep(8);
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const uint32_t k = b0 + (uint32_t)q * 64u + tid;
                    if ((uint32_t)(v[q] >> 61) != tag) v[q] = atomic_load_agent(pub + k);
                }
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) acc += v[q] & kPubMask;
        }
        acc = wave_sum_u64(acc);
        if (tid == 0) s_red[0] = timeout ? ~0ull : acc;
        if (timeout && tid == 0) raise_timeout(ctl, sp.fault);
    }
    __syncthreads();
    return s_red[0];
}

// sum of the first `count` tile totals of a finished K3a (one block, coalesced, any order:
// exact integers; the words carry K3a's launch tag above bit 61)
__device__ __forceinline__ uint64_t tiles_before(const uint64_t* __restrict__ tile_sum, uint32_t count, uint64_t* s_wtot)
{
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    uint64_t acc = 0;
    for (uint32_t k = tid; k < count; k += kBlock) acc += tile_sum[k] & kPubMask;
    acc = wave_sum_u64(acc);
    if (lane == 0) s_wtot[wave] = acc;
    __syncthreads();
    uint64_t t = 0;
#pragma unroll
    for (int wv = 0; wv < kWaves; ++wv) t += s_wtot[wv];
    __syncthreads();                     // s_wtot is reused by the caller
    return t;
}

// K3a (multi-GPU): phase B + normalisation (striped, coalesced) and, when resampling, the
// tile's exact fixed-point weight total, published as tag << 61 | total like the one-GPU
// K3's words (every launch writes every word).  The last tile waits for the others' words
// and writes this slice's total (the value all-gathered before K3b), so no separate kernel
// sums the tiles; K3b re-sums the words before its own tile (any order: exact integers).
template <int ITEMS, bool FUSED>
__global__ void __launch_bounds__(kBlock) k_normalize_scan(DevState s0, DevState s1, ScanParams sp, Ctl* __restrict__ ctl,
                                                           uint64_t* __restrict__ tile_sum, uint64_t* __restrict__ total,
                                                           FusedFin ff)
{
    __shared__ uint64_t s_wtot[kWaves], s_red[kWaves];
    __shared__ uint64_t s_img[FUSED ? kCtlWords : 1];
    __shared__ uint32_t s_flag;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t tile = blockIdx.x;
    const uint64_t tagw = (uint64_t)sp.tag << 61;
    const bool last_tile = total && tile + 1 == sp.ntiles;
    if (ctl->err & kFaultTimeout) {      // poisoned: nothing is written (the waits of the other blocks end)
        if (tid == 0) {
            publish_tile_1(tile_sum, sp.pub_stride, tile, tagw);
            if (FUSED && tile == 0) __hip_atomic_store(ff.fin_word, ff.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            if (last_tile) *total = ~0ull;
        }
        return;
    }
    if constexpr (FUSED) {
        // the update step's finalize over every rank's statistics (block 0; the sharded
        // counterpart of k_normalize_segments' fused finalize)
        if (tile == 0) {
            __shared__ FinLds s_fin;
            finalize_block(ff.shards, ff.nrec, ctl, ff.fp, s_fin);
            __syncthreads();
            if (tid == 0) {
                ctl->fin_epoch = ff.epoch;       // ordered before the publication by the release
                __hip_atomic_store(ff.fin_word, ff.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    const Ctl* cv = FUSED ? reinterpret_cast<const Ctl*>(s_img) : ctl;
    const DevState st = (FUSED ? ctl->k3_base : ctl->base) ? s1 : s0;
    const uint64_t t0 = (uint64_t)tile * (kBlock * ITEMS);
    double v[ITEMS];
    if constexpr (FUSED) {
        double mp[ITEMS];
        uint32_t fl[ITEMS];
        phase_b_load<ITEMS>(st, sp, t0, tid, v, mp, fl);
        if (fin_wait_copy(ctl, ff.fin_word, ff.epoch, s_img, sp, &s_flag)) {
            if (tid == 0) {
                publish_tile_1(tile_sum, sp.pub_stride, tile, tagw);
                if (last_tile) *total = ~0ull;               // every rank sees the fault
            }
            return;
        }
        if (cv->aborted) {               // the update threw (k_finalize): weights stay as phase A left them
            if (tid == 0) publish_tile_1(tile_sum, sp.pub_stride, tile, tagw);
            return;
        }
        phase_b_apply<ITEMS>(st, sp, cv, t0, tid, v, mp, fl);
    } else {
        if (ctl->aborted) {              // the update threw (k_finalize): weights stay as phase A left them
            if (tid == 0) publish_tile_1(tile_sum, sp.pub_stride, tile, tagw);
            return;
        }
        phase_b_tile<ITEMS>(st, sp, ctl, t0, tid, v);
    }
    const bool resample = sgpr_u32(cv->resample) != 0;
    const int shift = (int)sgpr_u32((uint32_t)cv->scan_shift);
    uint64_t fx_sum = 0;
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) fx_sum += fx_shift(v[r], shift);   // 0 past the end
    if (!resample) {
        if (tid == 0) publish_tile_1(tile_sum, sp.pub_stride, tile, tagw);
        return;
    }

    fx_sum = wave_sum_u64(fx_sum);
    if (lane == 0) s_wtot[wave] = fx_sum;
    __syncthreads();
    uint64_t t = 0;
#pragma unroll
    for (int wv = 0; wv < kWaves; ++wv) t += s_wtot[wv];
    if (tid == 0) publish_tile_1(tile_sum, sp.pub_stride, tile, tagw | (t & kPubMask));
    if (last_tile) {
        const uint64_t before = tiles_before_pub(tile_sum, tile, sp, s_red, ctl);
        if (tid == 0) *total = before == ~0ull ? ~0ull : before + t;     // ~0: every rank sees the fault
    }
}

// Draw counting (#{k : T_k <= C}) for the particles of one wave: the counts of its targets
// only read the draws [dlo, dhi) around floor(C N) of its first and last target.  Its lanes
// evaluate those draws in parallel, wave_draws at a time (lane l: k = q0 + l + 64 j, one jump
// then a 64-stride minstd step), store them in LDS, and every target reads the (at most
// three) draws of its window there.  No per-lane serial walk, no search, no divergence.
// Waves with more than kWaveChunks chunks of draws (heavy weights) evaluate each target's
// window directly (count_draws_le).
//
// count_draws_le with the draws read from LDS instead of evaluated.  The count of a target c
// is k0 = k* - 1 plus the leading draws among k0, k0 + 1, k0 + 2 (at most k* + 1, below N)
// that are <= c, k* = floor(c N) (draws below k0 are <= c, draws above k* + 1 are > c).
__device__ __forceinline__ uint64_t kstar_of(uint64_t c, uint64_t N, int shift)
{
    // c * N with N < 2^32 as two 32 x 32 -> 64 products: (hi << 32) + lo, and for shift >= 32
    // (the update path: 60) the shift needs only hi + (lo >> 32) (< 2^62, no carry out)
    if (shift >= 32) {
        const uint64_t lo = (uint64_t)(uint32_t)c * (uint32_t)N, hi = (c >> 32) * (uint64_t)(uint32_t)N;
        return (hi + (lo >> 32)) >> ((shift - 32) & 63);
    }
    return (uint64_t)(((unsigned __int128)c * N) >> shift);
}

// The window of target c as one word: bits 0..15 k0 - dlo (< kWaveChunks * wave_draws),
// 16..17 the number of window draws (k0 + d <= k* + 1, < N), bit 18 "k0 >= N" (count N),
// bits 19..21 set by draws_le_chunk: window draw d is <= c.
__device__ __forceinline__ uint32_t window_of(uint64_t c, uint64_t N, int shift, uint64_t dlo)
{
    const uint64_t kstar = kstar_of(c, N, shift);
    const uint64_t k0 = kstar >= 1 ? kstar - 1 : 0;
    if (k0 >= N) return 1u << 18;
    // draws k0 + d with k0 + d <= k* + 1 and k0 + d < N
    const uint64_t room = N - k0;
    uint32_t nd = kstar >= 1 ? 3u : 2u;
    nd = room < (uint64_t)nd ? (uint32_t)room : nd;
    return (uint32_t)(k0 - dlo) | (nd << 16);
}

// rq0, rq1: the LDS chunk [q0, q1) relative to dlo (u32: the wave's draws span < 2^16)
__device__ __forceinline__ uint32_t draws_le_chunk(uint32_t w, uint64_t c, const uint64_t* sT, uint32_t rq0, uint32_t rq1)
{
    const uint32_t r0 = w & 0xffffu;
    const uint32_t nd = (w >> 16) & 3u;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        const uint32_t r = r0 + (uint32_t)d;
        const bool in = ((uint32_t)d < nd) & (r >= rq0) & (r < rq1);
        const uint64_t t = sT[draw_slot(in ? r - rq0 : 0u)];    // slot 0 is in LDS; used only when in
        w |= (in && t <= c) ? 1u << (19 + d) : 0u;
    }
    return w;
}

__device__ __forceinline__ uint64_t count_from_window(uint32_t w, uint64_t dlo, uint64_t N)
{
    if ((w >> 18) & 1u) return N;
    const uint64_t k0 = dlo + (w & 0xffffu);
    const uint32_t le = (w >> 19) & 7u;
    // leading draws <= c (draws are nondecreasing in k; le has no bits beyond nd)
    const uint32_t lead = (le & 1u) ? ((le & 2u) ? ((le & 4u) ? 3u : 2u) : 1u) : 0u;
    return k0 + lead;
}

// The counts #{k : T_k <= base + c[r]} of one wave's targets (hi_r) and, for the lane's
// first item, the count of its predecessor (lo: lane 0 #{T_k <= base}, the others the
// previous lane's last count).  The wave's cumulative range [wlo, whi] needs only the draws
// in [dlo, dhi) (the windows k* - 1 .. k* + 1 of wlo and whi, clamped to [0, N)): its lanes
// evaluate them in parallel into LDS (sT, wave_draws at a time) and every target reads the
// (at most three) draws of its window there.  Heavy weights (more than kWaveChunks chunks of
// draws): each target's window evaluated directly.
template <int ITEMS>
__device__ __forceinline__ void wave_counts(uint64_t base, uint64_t run, const uint64_t (&c)[ITEMS], uint64_t N, int shift,
                                            uint32_t xs, const uint32_t* __restrict__ jt, uint64_t* sT,
                                            uint64_t (&hi_r)[ITEMS], uint64_t& lo)
{
    const uint32_t lane = threadIdx.x & 63u;
    const double dN = (double)N, inv_N = 1.0 / dN;
    // wave-uniform by construction: moved to SGPRs, so the window bounds, the loop and the
    // jump-ahead table reads of the first draw are scalar (readfirstlane returns int: each
    // half is widened as unsigned)
    auto rfl64 = [](uint64_t v) {
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
        const uint32_t lo_ = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
        return ((uint64_t)hi << 32) | (uint64_t)lo_;
    };
    const uint64_t wlo = rfl64(__shfl(base, 0, 64)), whi = rfl64(__shfl(base + run, 63, 64));
    const uint64_t ks_lo = kstar_of(wlo, N, shift), ks_hi = kstar_of(whi, N, shift);
    const uint64_t dlo = ks_lo >= 1 ? ks_lo - 1 : 0;
    const uint64_t dhi = ks_hi + 2 < N ? ks_hi + 2 : N;
    if (dlo >= dhi || dhi - dlo <= (uint64_t)kWaveChunks * wave_draws<ITEMS>()) {
        // le[r] bit d: draw k0_r + d of target r (r = ITEMS: wlo) is <= its target
        uint32_t win[ITEMS + 1];
#pragma unroll
        for (int r = 0; r <= ITEMS; ++r) win[r] = window_of(r < ITEMS ? base + c[r] : wlo, N, shift, dlo);
        const uint32_t a64 = jt[64], a_lane = jt[lane];            // A^64, A^lane
        for (uint64_t q0 = dlo; q0 < dhi; q0 += wave_draws<ITEMS>()) {
            const uint64_t q1 = dhi - q0 < (uint64_t)wave_draws<ITEMS>() ? dhi : q0 + wave_draws<ITEMS>();
            if (q0 + lane < q1) {
                uint32_t x = dm_mulmod31(dm_mulmod31(jump_pow(jt, q0 + 1), xs), a_lane);
#pragma unroll 4
                for (uint64_t k = q0 + lane; k < q1; k += 64) {
                    sT[draw_slot((uint32_t)(k - q0))] = draw_fx(k, x, dN, inv_N, shift);
                    x = dm_mulmod31(x, a64);
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int r = 0; r <= ITEMS; ++r)
                win[r] = draws_le_chunk(win[r], r < ITEMS ? base + c[r] : wlo, sT, (uint32_t)(q0 - dlo),
                                        (uint32_t)(q1 - dlo));
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
#pragma unroll
        for (int r = 0; r < ITEMS; ++r) hi_r[r] = count_from_window(win[r], dlo, N);
        const uint64_t K0 = count_from_window(win[ITEMS], dlo, N);
        const uint64_t prev = __shfl_up(hi_r[ITEMS - 1], 1, 64);
        lo = lane == 0 ? K0 : prev;
    } else {
#pragma unroll
        for (int r = 0; r < ITEMS; ++r) hi_r[r] = count_draws_le(base + c[r], N, xs, shift, jt);
        const uint64_t K0 = count_draws_le(wlo, N, xs, shift, jt);
        const uint64_t prev = __shfl_up(hi_r[ITEMS - 1], 1, 64);
        lo = lane == 0 ? K0 : prev;
    }
}

// ---------------------------------------------------------------------------------------
// K3 (one GPU): phase B + normalisation, the tile's exact fixed-point total, the prefix of
// the preceding tiles and the segment marks, in one pass.  Each tile publishes its total as
// one 64-bit word, tag << 61 | total (fixed point < 2^61: the weights are normalised with
// shift 60, or scaled below 2^61 by k_finalize's shift for a standalone resample); the host
// cycles the tag per launch and every launch writes every tile's word, so a word still
// holding the previous launch's value never carries the current tag.  A tile sums its
// predecessors' words (exact integers, any order), waiting for those not yet published.
// The wait needs only that a tile's predecessors get scheduled: workgroups are dispatched in
// order (per XCD), and a predecessor publishes before it waits on anything itself.  A
// bounded spin turns a violated assumption into ctl->err bit 2 instead of a hang.
// ---------------------------------------------------------------------------------------

// 8 items: the 6 waves per SIMD the unfused kernel reaches by itself (<= 80 VGPRs; the fused
// one would take 86 and run at 5)
template <int ITEMS, bool FUSED>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(ITEMS == 8 ? 6 : 1))) k_normalize_segments(DevState s0, DevState s1, ScanParams sp, Ctl* __restrict__ ctl,
                                                               uint64_t* __restrict__ tile_pub, uint32_t* __restrict__ marks,
                                                               uint32_t* __restrict__ tile_first,
                                                               const uint32_t* __restrict__ jt, FusedFin ff)
{
    __shared__ uint64_t s_wtot[kWaves], s_red[kWaves];
    __shared__ K3Lds<ITEMS> s_u;
    __shared__ uint64_t s_img[FUSED ? kCtlWords : 1];
    __shared__ uint32_t s_flag;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t tile = blockIdx.x;
    ESLAM_STAMP(g_stamps_k3, 0);
    const uint64_t tagw = (uint64_t)sp.tag << 61;
    if (ctl->err & kFaultTimeout) {      // poisoned: nothing is written (the waits of the other blocks end)
        if (tid == 0) {
            if (FUSED && tile == 0) __hip_atomic_store(ff.fin_word, ff.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
        publish_tile(tile_pub, sp.pub_stride, tile, tagw);
        return;
    }
    if constexpr (FUSED) {
        if (tile == 0) {
            __shared__ FinLds s_fin;
            finalize_block(ff.shards, ff.nrec, ctl, ff.fp, s_fin);
            __syncthreads();
            if (tid == 0) {
                ctl->fin_epoch = ff.epoch;       // ordered before the publication by the release
                __hip_atomic_store(ff.fin_word, ff.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    // the finalize's outputs: ctl itself (k_finalize ran before this launch), or its copy in
    // LDS once block 0 has published (fused)
    const Ctl* cv = FUSED ? reinterpret_cast<const Ctl*>(s_img) : ctl;
    // the buffer the weighting kernel wrote (= base after the finalize's commit)
    const DevState st = (FUSED ? ctl->k3_base : ctl->base) ? s1 : s0;
    const uint64_t t0 = (uint64_t)tile * (kBlock * ITEMS);
    bool resample = false;
    if constexpr (!FUSED) {
        if (cv->aborted) {               // the update threw (k_finalize): weights stay as phase A left them
            publish_tile(tile_pub, sp.pub_stride, tile, tagw);
            return;
        }
        resample = cv->resample != 0;
    }
    {
        // phase B + normalisation, striped (coalesced); the values are staged in LDS for the
        // blocked scan below.  Fused: the loads do not depend on the finalize, so they are
        // issued before its wait.
        double v[ITEMS];
        if constexpr (FUSED) {
            double mp[ITEMS];
            uint32_t fl[ITEMS];
            phase_b_load<ITEMS>(st, sp, t0, tid, v, mp, fl);
            ESLAM_STAMP(g_stamps_k3, 1);
            if (fin_wait_copy(ctl, ff.fin_word, ff.epoch, s_img, sp, &s_flag)) {
                publish_tile(tile_pub, sp.pub_stride, tile, tagw);
                return;
            }
            if (cv->aborted) {           // the update threw (k_finalize): weights stay as phase A left them
                publish_tile(tile_pub, sp.pub_stride, tile, tagw);
                return;
            }
            ESLAM_STAMP(g_stamps_k3, 2);
            phase_b_apply<ITEMS>(st, sp, cv, t0, tid, v, mp, fl);
            resample = sgpr_u32(cv->resample) != 0;
        } else {
            phase_b_tile<ITEMS>(st, sp, cv, t0, tid, v);
        }
#pragma unroll
        for (int r = 0; r < ITEMS; ++r) s_u.v[skew(r * kBlock + (int)tid)] = v[r];
    }
    if (!resample) {
        publish_tile(tile_pub, sp.pub_stride, tile, tagw);
        return;
    }
    __syncthreads();
    ESLAM_STAMP(g_stamps_k3, 3);
    const int shift = (int)sgpr_u32((uint32_t)cv->scan_shift);
    uint64_t c[ITEMS];
    const uint64_t run = blocked_fx(s_u.v, shift, c);
    // in-tile exclusive prefix and the tile total (wave scans -> LDS)
    uint64_t tincl = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t t = __shfl_up(tincl, o, 64);
        if ((int)lane >= o) tincl += t;
    }
    if (lane == 63) s_wtot[wave] = tincl;
    __syncthreads();                     // (s_u.v is dead after it)
    uint64_t wexcl = 0, agg = 0;
#pragma unroll
    for (int wv = 0; wv < kWaves; ++wv) {
        const uint64_t t = s_wtot[wv];
        if ((uint32_t)wv < wave) wexcl += t;
        agg += t;
    }
    ESLAM_STAMP(g_stamps_k3, 4);
    publish_tile(tile_pub, sp.pub_stride, tile, tagw | (agg & kPubMask));
    const uint64_t tb = tiles_before_pub(tile_pub + (uint64_t)(tile % kPubReplicas) * sp.pub_stride, tile, sp, s_red, ctl);
    if (tb == ~0ull) return;             // gave up waiting: poisoned, no marks
    ESLAM_STAMP(g_stamps_k3, 5);
    const uint64_t base = tb + wexcl + (tincl - run);

    const uint64_t N = sp.n_global;
    const uint32_t xs = sgpr_u32(cv->minstd_start);
    const uint64_t i0 = t0 + (uint64_t)tid * ITEMS;
    uint64_t hi_r[ITEMS];
    uint64_t lo;
    wave_counts<ITEMS>(base, run, c, N, shift, xs, jt, s_u.T[wave], hi_r, lo);
    ESLAM_STAMP(g_stamps_k3, 6);
    if (i0 == 0) lo = 0;
    // each item's segment [lo, hi) marked as it is found (no arrays of segments held)
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const uint64_t i = i0 + r;
        if (i < sp.n) {
            uint64_t hi = hi_r[r];
            if (i == N - 1) {
                if (hi < N) atomicAdd((unsigned long long*)&ctl->overruns, (unsigned long long)(N - hi));
                hi = N;
            }
            flush_mark(marks, tile_first, lo, hi, (uint32_t)(i + 1));
            lo = hi;
        }
    }
    ESLAM_STAMP(g_stamps_k3, 7);
}

// ---------------------------------------------------------------------------------------
// multi-GPU segments: the same scan, offset by the lower ranks' totals.  Outputs that land
// in this rank's slice [W0, W1) are marked directly (own particles never move); particles
// whose outputs reach another rank's slice record their range for k_pack.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void plan_bounds(const PlanParams& pp, const Ctl* ctl, const uint64_t* totals,
                                            const uint32_t* jt, uint64_t& off, uint64_t& O0, uint64_t& O1)
{
    off = 0;
    for (int r = 0; r < pp.rank; ++r) off += totals[r];
    const uint64_t N = pp.n_global;
    const uint32_t xs = ctl->minstd_start;
    const int shift = ctl->scan_shift;
    O0 = pp.rank == 0 ? 0 : count_draws_le(off, N, xs, shift, jt);
    O1 = pp.rank == pp.nranks - 1 ? N : count_draws_le(off + totals[pp.rank], N, xs, shift, jt);
}

__global__ void __launch_bounds__(kBlock) k_segments_multi(DevState s0, DevState s1, ScanParams sp, PlanParams pp,
                                                           Ctl* __restrict__ ctl, const uint64_t* __restrict__ tile_sum,
                                                           uint32_t* __restrict__ marks, uint32_t* __restrict__ tile_first,
                                                           const uint64_t* __restrict__ totals, const uint32_t* __restrict__ jt,
                                                           uint2* __restrict__ range, uint64_t* __restrict__ first_last,
                                                           uint64_t* host_out, uint64_t* host_epoch, uint64_t epoch)
{
    __shared__ uint64_t s_wtot[kWaves];
    __shared__ K3Lds<kScanItems> s_u;
    double* s_v = s_u.v;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        // the gathered totals and the finalize mirror (they follow the totals) to the host-mapped
        // buffer, then this launch's epoch: the host plans the exchange from them while the
        // kernel runs (no copy on the stream)
        for (int r = 0; r < pp.nranks; ++r) host_out[r] = totals[r];
        for (int q = 0; q < 3; ++q) host_out[kMaxRanks + q] = totals[kMaxRanks + q];
        __hip_atomic_store(host_epoch, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        // the chunks the next weighting launch may process before the exchange: all of them
        // without a resample (no gather pending), else those of the own outputs
        uint64_t c_lo = 0, c_hi = (pp.n_local + 64ull * pp.J - 1) / (64ull * pp.J);
        if (ctl->resample) {
            uint64_t off, O0, O1;
            plan_bounds(pp, ctl, totals, jt, off, O0, O1);
            own_chunks(O0, O1, pp.gbase[pp.rank], pp.n_local, pp.J, &c_lo, &c_hi);
        }
        pp.chunk_sel[0] = c_lo;
        pp.chunk_sel[1] = c_hi;
    }
    if (!ctl->resample) return;
    const uint32_t tid = threadIdx.x;
    const uint32_t tile = blockIdx.x;
    const DevState st = ctl->base ? s1 : s0;
    const uint64_t t0 = (uint64_t)tile * kScanTile;
#pragma unroll
    for (int r = 0; r < kScanItems; ++r) {
        const int k = r * kBlock + (int)tid;
        const uint64_t i = t0 + (uint64_t)k;
        s_v[skew(k)] = i < sp.n ? st.w[i] : 0.0;
    }
    __syncthreads();
    const int shift = ctl->scan_shift;
    uint64_t c[kScanItems];
    const uint64_t run = blocked_fx<kScanItems>(s_v, shift, c);
    const uint64_t tbase = tiles_before(tile_sum, tile, s_wtot) + block_excl(run, s_wtot);
    uint64_t off, O0, O1;
    plan_bounds(pp, ctl, totals, jt, off, O0, O1);
    const uint64_t base = off + tbase;
    const uint64_t N = pp.n_global;
    const uint64_t W0 = pp.gbase[pp.rank], W1 = pp.gbase[pp.rank + 1];
    const uint64_t i0 = t0 + (uint64_t)tid * kScanItems;
    uint64_t hi_r[kScanItems];
    uint64_t lo;
    wave_counts<kScanItems>(base, run, c, N, shift, ctl->minstd_start, jt, s_u.T[tid >> 6], hi_r, lo);
    if (i0 == 0) lo = O0;
    uint64_t seg_lo[kScanItems], seg_hi[kScanItems];
    uint32_t val[kScanItems];
#pragma unroll
    for (int r = 0; r < kScanItems; ++r) {
        const uint64_t i = i0 + r;
        seg_lo[r] = seg_hi[r] = 0;
        val[r] = kMarkOwn + 1u + (uint32_t)i;
        if (i >= sp.n) continue;
        uint64_t hi = hi_r[r];
        if (i + 1 == sp.n) {
            if (pp.rank == pp.nranks - 1 && hi < N)
                atomicAdd((unsigned long long*)&ctl->overruns, (unsigned long long)(N - hi));
            hi = O1;
        }
        const uint64_t a = lo > W0 ? lo : W0, b = hi < W1 ? hi : W1;
        if (a < b) { seg_lo[r] = a - W0; seg_hi[r] = b - W0; }
        // every particle a foreign destination's [first, last] run can include (empty
        // ranges too) has lo < W0 or hi > W1: record its range for k_pack
        if (lo < W0 || hi > W1) {
            range[i] = make_uint2((uint32_t)lo, (uint32_t)hi);
            if (hi > lo) {
                for (int d = 0; d < pp.nranks; ++d) {
                    if (d == pp.rank) continue;
                    const uint64_t Wd0 = pp.gbase[d], Wd1 = pp.gbase[d + 1];
                    const uint64_t Sd = O0 > Wd0 ? O0 : Wd0, Ed = O1 < Wd1 ? O1 : Wd1;
                    if (Sd >= Ed) continue;
                    if (lo <= Sd && Sd < hi) first_last[2 * d] = i;
                    if (lo <= Ed - 1 && Ed - 1 < hi) first_last[2 * d + 1] = i;
                }
            }
        }
        lo = hi;
    }
    flush_marks(marks, tile_first, seg_lo, seg_hi, val);
}

// one record per output of this rank that lands in another slice: send slot j of
// destination d is output k = sd[d] + (j - send_off[d]); its source is the particle of
// [first, last] (d's run, from k_segments_multi) whose range [lo, hi) contains k
__global__ void __launch_bounds__(kBlock) k_pack(DevState s0, DevState s1, const Ctl* __restrict__ ctl, PlanParams pp,
                                                 const uint2* __restrict__ range, const uint64_t* __restrict__ first_last,
                                                 Rec* __restrict__ send)
{
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= pp.send_off[pp.nranks]) return;
    int d = 0;
    while (j >= pp.send_off[d + 1]) ++d;
    const uint64_t k = pp.sd[d] + (j - pp.send_off[d]);
    uint64_t a = first_last[2 * d], b = first_last[2 * d + 1];   // range[a].x <= k < range[b].y
    while (a < b) {                                               // last i in [a, b] with lo_i <= k
        const uint64_t mid = a + (b - a + 1) / 2;
        if ((uint64_t)range[mid].x <= k) a = mid;
        else b = mid - 1;
    }
    const uint64_t i = a;
    const DevState st = ctl->base ? s1 : s0;
    Rec r;
    r.x = st.x[i]; r.y = st.y[i]; r.th = st.th[i]; r.z = st.z[i]; r.zs = st.zs[i]; r.w = st.w[i]; r.mprob = st.mprob[i];
    r.lohi = k | ((k + 1) << 32);
    r.src = (uint64_t)st.flags[i] | ((pp.gbase[pp.rank] + i) << 8);
    send[j] = r;
}

// records -> marks (lower ranks: 1 + j, higher ranks: kMarkHigh + 1 + j)
__global__ void __launch_bounds__(kBlock) k_expand(const Rec* __restrict__ recv, uint64_t nrecv, uint64_t W0,
                                                   uint32_t* __restrict__ marks, uint32_t* __restrict__ tile_first)
{
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= nrecv) return;
    const Rec& r = recv[j];
    const uint64_t glo = r.lohi & 0xffffffffull, ghi = r.lohi >> 32;
    if (ghi > glo) {
        const uint32_t v = ((r.src >> 8) < W0 ? 1u : kMarkHigh + 1u) + (uint32_t)j;
        mark_segment(marks, tile_first, glo - W0, ghi - W0, v);
    }
}

// ---------------------------------------------------------------------------------------
// k_resample_gather: materialise a pending resample gather (xi_k.swap(xi_kp),
// src/ParticleFilter.hpp:107) before the state is read by anything but the next
// k_project_weight, which gathers on the fly.  Weights are carried, not reset (Q4).
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) k_resample_gather(DevState s0, DevState s1, uint64_t n, uint64_t gbase,
                                                            Ctl* __restrict__ ctl, GatherView gv, uint32_t aux)
{
    if (!ctl->gather) return;
    __shared__ uint32_t s_wmax[kWaves];
    __shared__ uint32_t s_idx[kGatherTile];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t t = blockIdx.x;
    const DevState in = ctl->base ? s1 : s0;
    const DevState out = ctl->base ? s0 : s1;
    const uint64_t k0 = (uint64_t)t * kGatherTile + (uint64_t)tid * kScanItems;
    uint32_t mk[kScanItems];
    uint32_t run = 0;
#pragma unroll
    for (int r = 0; r < kScanItems; ++r) {
        const uint64_t k = k0 + r;
        uint32_t v = 0;
        if (k < n) { v = gv.marks[k]; if (v) gv.marks[k] = 0; }
        run = run > v ? run : v;
        mk[r] = run;
    }
    const uint32_t tincl = wave_incl_max_u32(run);
    if (lane == 63) s_wmax[wave] = tincl;
    __syncthreads();
    uint32_t carry = gv.row_first[(uint64_t)t * (kGatherTile / kRow)] + 1u;
    for (uint32_t wv = 0; wv < wave; ++wv) carry = carry > s_wmax[wv] ? carry : s_wmax[wv];
    uint32_t texcl = __shfl_up(tincl, 1, 64);
    if (lane == 0) texcl = 0;
    carry = carry > texcl ? carry : texcl;
#pragma unroll
    for (int r = 0; r < kScanItems; ++r) {
        const uint32_t v = mk[r] > carry ? mk[r] : carry;
        s_idx[tid * kScanItems + r] = v - 1u;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kScanItems; ++r) {
        const uint32_t slot = (uint32_t)r * kBlock + tid;
        const uint64_t k = (uint64_t)t * kGatherTile + slot;
        if (k >= n) continue;
        const gmem<const Rec>* rc;
        const uint32_t i = decode_source(s_idx[slot], gv.multi, (const gmem<const Rec>*)gv.recs, &rc);
        if (rc) {
            out.x[k] = rc->x; out.y[k] = rc->y; out.th[k] = rc->th; out.z[k] = rc->z; out.zs[k] = rc->zs; out.w[k] = rc->w;
            if (aux) { out.mprob[k] = rc->mprob; out.flags[k] = (uint8_t)rc->src; }
            if (gv.record) gv.anc[k] = (uint32_t)(rc->src >> 8);
            if (in.sid) out.sid[k] = kSidRecord | (uint32_t)(rc - (const gmem<const Rec>*)gv.recs);   // store: the record's
            continue;
        }
        out.x[k] = in.x[i];
        out.y[k] = in.y[i];
        out.th[k] = in.th[i];
        out.z[k] = in.z[i];
        out.zs[k] = in.zs[i];
        out.w[k] = in.w[i];
        if (aux) {
            out.mprob[k] = in.mprob[i];
            out.flags[k] = in.flags[i];
        }
        if (in.sid) out.sid[k] = in.sid[i];            // per-particle maps: the store's name
        if (gv.record) gv.anc[k] = (uint32_t)(gbase + i);
    }
}

// commit a consumed gather / flip outside an update (after a project-only step or a
// materialising gather): the latest state becomes state[base]
__global__ void k_commit(Ctl* __restrict__ ctl)
{
    if (threadIdx.x == 0) {
        ctl->base ^= ctl->flip;
        ctl->flip = 0;
        ctl->gather = 0;
    }
}

// ---------------------------------------------------------------------------------------
// PoseEstimator::init(N, mu, sigma, zpos, zsigma): samplePose2D per particle
// (src/PoseEstimator.cpp:64-73, 88-102) from the INIT Philox stream.
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) k_init_gaussian(DevState s0, uint64_t n, uint64_t gbase, uint64_t seed, uint64_t ev,
                                                          double mx, double my, double mt, double sx, double sy, double stt,
                                                          double zpos, double zsigma)
{
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint64_t gi = gbase + i;
    const dm_philox_ctr d0 = dm_draw(seed, DM_STREAM_INIT, ev, gi, 0);
    double n0, n1, n2, n3;
    dm_box_muller32(d0.v[0], d0.v[1], &n0, &n1);
    dm_box_muller32(d0.v[2], d0.v[3], &n2, &n3);
    s0.x[i] = n0 * sx + mx;
    s0.y[i] = n1 * sy + my;
    s0.th[i] = n2 * stt + mt;
    s0.z[i] = zpos;
    s0.zs[i] = zsigma;
    s0.w[i] = 0.0;
    s0.mprob[i] = 0.0;
    s0.flags[i] = 0x80u;   // floating = true, no contact points
}

// ---------------------------------------------------------------------------------------
// ParticleFilter::getBestParticleIndex (src/ParticleFilter.hpp:160-173): first index of the
// maximum weight; NaN never compares greater.  out[0] = max ordered key, out[1] = index.
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) k_best_max(DevState s0, DevState s1, uint64_t n, const Ctl* __restrict__ ctl,
                                                     uint64_t* out)
{
    const DevState st = (ctl->base ^ ctl->flip) ? s1 : s0;
    uint64_t best = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
        const double w = st.w[i];
        if (w == w) { const uint64_t k = order_key(w); best = best > k ? best : k; }
    }
    for (int o = 32; o >= 1; o >>= 1) { const uint64_t t = __shfl_xor(best, o, 64); best = best > t ? best : t; }
    if ((threadIdx.x & 63u) == 0 && best) atomicMax((unsigned long long*)&out[0], (unsigned long long)best);
}

__global__ void __launch_bounds__(kBlock) k_best_index(DevState s0, DevState s1, uint64_t n, const Ctl* __restrict__ ctl,
                                                       uint64_t* out)
{
    const DevState st = (ctl->base ^ ctl->flip) ? s1 : s0;
    const uint64_t key = out[0];
    uint64_t idx = ~0ull;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
        const double w = st.w[i];
        if (w == w && order_key(w) == key) { idx = i < idx ? i : idx; break; }
    }
    for (int o = 32; o >= 1; o >>= 1) { const uint64_t t = __shfl_xor(idx, o, 64); idx = idx < t ? idx : t; }
    if ((threadIdx.x & 63u) == 0 && idx != ~0ull) atomicMin((unsigned long long*)&out[1], (unsigned long long)idx);
}

// ---------------------------------------------------------------------------------------
// PoseEstimator::getCentroid sums (src/PoseEstimator.cpp:354-383): x w, y w, theta w, z w, w
// in the canonical chunk order, then a fixed pairwise tree over the chunk totals.
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) k_centroid_chunks(DevState s0, DevState s1, uint64_t n, uint32_t J,
                                                            const Ctl* __restrict__ ctl, double* __restrict__ chunk_out)
{
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint64_t chunk = (uint64_t)blockIdx.x * kWaves + wave;
    const uint64_t lbase = chunk * 64ull * J;
    if (lbase >= n) return;
    const DevState st = (ctl->base ^ ctl->flip) ? s1 : s0;
    double a[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    for (uint32_t j = 0; j < J; ++j) {
        const uint64_t i = lbase + 64ull * j + lane;
        if (i >= n) continue;
        const double w = st.w[i];
        a[0] = a[0] + st.x[i] * w;
        a[1] = a[1] + st.y[i] * w;
        a[2] = a[2] + st.th[i] * w;
        a[3] = a[3] + st.z[i] * w;
        a[4] = a[4] + w;
    }
#pragma unroll
    for (int q = 0; q < 5; ++q) {
        const double v = wave_sum_butterfly(a[q]);
        if (lane == 0) chunk_out[chunk * 5 + q] = v;
    }
}

// one level of the fixed pairwise tree: dst[i] = src[2i] + src[2i+1]; odd tail moves up
__global__ void __launch_bounds__(kBlock) k_tree_level(const double* __restrict__ src, double* __restrict__ dst, uint64_t m)
{
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const uint64_t h = m / 2;
    if (i > h || (i == h && !(m & 1))) return;
    for (int q = 0; q < 5; ++q)
        dst[i * 5 + q] = i < h ? src[(2 * i) * 5 + q] + src[(2 * i + 1) * 5 + q] : src[(m - 1) * 5 + q];
}

// device self-test of the deterministic math (tests/test_gpu_math.py)
__global__ void k_selftest_math(int fn, const double* x, const double* y, double* out, uint64_t n)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (fn >= 20 && fn <= 25) {
        // lane exchanges of the butterflies: x[i ^ 2^(fn - 20)] (n a multiple of the block)
        const double v = i < n ? x[i] : 0.0;
        double r = 0.0;
        switch (fn) {
        case 20: r = xor_lane<1>(v); break;
        case 21: r = xor_lane<2>(v); break;
        case 22: r = xor_lane<4>(v); break;
        case 23: r = xor_lane<8>(v); break;
        case 24: r = xor_lane<16>(v); break;
        default: r = xor_lane<32>(v); break;
        }
        if (i < n) out[i] = r;
        return;
    }
    if (i >= n) return;
    double s, c, r = 0;
    switch (fn) {
    case 0: r = dm_exp(x[i]); break;
    case 1: r = dm_log(x[i]); break;
    case 2: dm_sincos(x[i], &s, &c); r = s; break;
    case 3: dm_sincos(x[i], &s, &c); r = c; break;
    case 4: r = dm_erfc(x[i]); break;
    case 5: r = dm_sqrt(x[i]); break;
    case 6: r = x[i] / y[i]; break;
    case 7: r = dm_normal_pdf_cdf_ratio(x[i], y[i]); break;
    case 8: r = dm_pow(x[i], y[i]); break;
    case 9: r = dm_from_bits(dm_fx61(x[i])); break;
    case 13: dm_sincos2pi(x[i], &s, &c); r = s; break;
    case 14: dm_sincos2pi(x[i], &s, &c); r = c; break;
    case 15: r = dm_log_bm(x[i]); break;
    case 16: dm_sincos2pi32((uint32_t)x[i], &s, &c); r = s; break;
    case 17: dm_sincos2pi32((uint32_t)x[i], &s, &c); r = c; break;
    case 18: dm_box_muller32((uint32_t)x[i], (uint32_t)y[i], &s, &c); r = s; break;
    case 19: dm_box_muller32((uint32_t)x[i], (uint32_t)y[i], &s, &c); r = c; break;
    case 26: { float fs, fc; dm_sincos2pi32f((uint32_t)x[i], &fs, &fc); r = fs; } break;
    case 27: { float fs, fc; dm_sincos2pi32f((uint32_t)x[i], &fs, &fc); r = fc; } break;
    default: r = __builtin_nan("");
    }
    out[i] = r;
}

// every Box-Muller radius: the range-restricted sqrt against the general one on -2 log u, for
// all 2^32 uniform words (counts the words whose radius differs in any bit)
__global__ void __launch_bounds__(kBlock) k_selftest_bm_radius(unsigned long long* bad)
{
    uint32_t cnt = 0;
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t a = (uint64_t)blockIdx.x * kBlock + threadIdx.x; a < (1ull << 32); a += stride) {
        const float x = (float)(-2.0 * dm_log_bm(dm_u32((uint32_t)a)));
        cnt += __float_as_uint(dm_sqrtf_pos(x)) != __float_as_uint(__builtin_sqrtf(x)) ? 1u : 0u;
    }
    cnt = wave_sum_u32(cnt);
    if ((threadIdx.x & 63u) == 0 && cnt) atomicAdd(bad, (unsigned long long)cnt);
}

}  // namespace eslam_dev

// ---------------------------------------------------------------------------------------
// launchers (called by eslam_ctx.hip)
// ---------------------------------------------------------------------------------------
using namespace eslam_dev;

// One canonical chunk per wave (dm_chunk_rows sizes the chunks so that there are ~16k of
// them from 1M particles on).  A persistent grid striding over chunks was measured slower:
// its loop state spills SGPRs, and the LDS window it saves is staged from L2 anyway.
static uint32_t k1_grid(uint64_t chunks) { return (uint32_t)((chunks + kWaves - 1) / kWaves); }

extern "C" hipError_t eslam_launch_project_weight(int project, int weight, int maxp, DevState s0, DevState s1,
                                                  const MapView* map, const StepParams* p, Ctl* ctl, Shard* shards,
                                                  const GatherView* gv, const LocalMaps* store, hipStream_t stream,
                                                  const ChunkSel* sel, double* bspill)
{
    const uint64_t csz = 64ull * p->J;
    uint64_t chunks = (p->n + csz - 1) / csz;
    if (sel && sel->mode == 2u) chunks = sel->c_lo + (chunks > sel->c_hi ? chunks - sel->c_hi : 0);   // the edge chunks
    if (chunks == 0) return hipSuccess;
    const size_t lds = kStatsLds + (weight ? kWindowLds : 0);
    K1Args args;
    args.p = *p;
    args.map = *map;
    args.gv = *gv;
    args.s[0] = s0;
    args.s[1] = s1;
    args.ctl = ctl;
    args.shards = shards;
    memset(&args.store, 0, sizeof(args.store));
    if (store) args.store = *store;
    memset(&args.sel, 0, sizeof(args.sel));
    if (sel) args.sel = *sel;
    args.bspill = bspill;
    if (weight && !bspill) return hipErrorInvalidValue;
#define ESLAM_LAUNCH(P, W, M, B, ...)                                                                   \
    hipLaunchKernelGGL((k_project_weight<P, W, M, B, ##__VA_ARGS__>), dim3(k1_grid(chunks)), dim3(kBlock), lds, \
                       stream, args)
    // every contact closes its group (groupId -1 or groups of one): the reduced group logic
    const uint32_t all = p->m >= 32 ? 0xffffffffu : ((1u << p->m) - 1u);
    const bool ung = (p->end_mask & all) == all;
    if (weight && store) {
        // per-particle maps: the lookups fall back to the particle's store (every pending
        // gather has been materialised by the host)
        if (p->m <= 4 && maxp <= 4) {
            if (project) { if (ung) ESLAM_LAUNCH(true, true, 4, true, true, true); else ESLAM_LAUNCH(true, true, 4, true, true); }
            else { if (ung) ESLAM_LAUNCH(false, true, 4, true, true, true); else ESLAM_LAUNCH(false, true, 4, true, true); }
        } else {
            if (project) ESLAM_LAUNCH(true, true, ESLAM_MAX_CONTACTS, false, true);
            else ESLAM_LAUNCH(false, true, ESLAM_MAX_CONTACTS, false, true);
        }
        return hipGetLastError();
    }
    // batched contact lookups when every contact fits the MAXP-sized arrays
    if (project && !weight) ESLAM_LAUNCH(true, false, 4, false);
    else if (!project && weight) {
        if (maxp <= 4) {
            if (p->m <= 4) { if (ung) ESLAM_LAUNCH(false, true, 4, true, false, true); else ESLAM_LAUNCH(false, true, 4, true); }
            else ESLAM_LAUNCH(false, true, 4, false);
        }
        else if (maxp <= 8) { if (p->m <= 8) ESLAM_LAUNCH(false, true, 8, true); else ESLAM_LAUNCH(false, true, 8, false); }
        else ESLAM_LAUNCH(false, true, ESLAM_MAX_CONTACTS, false);
    } else {
        if (maxp <= 4) {
            if (p->m <= 4) { if (ung) ESLAM_LAUNCH(true, true, 4, true, false, true); else ESLAM_LAUNCH(true, true, 4, true); }
            else ESLAM_LAUNCH(true, true, 4, false);
        }
        else if (maxp <= 8) { if (p->m <= 8) ESLAM_LAUNCH(true, true, 8, true); else ESLAM_LAUNCH(true, true, 8, false); }
        else ESLAM_LAUNCH(true, true, ESLAM_MAX_CONTACTS, false);
    }
#undef ESLAM_LAUNCH
    return hipGetLastError();
}

extern "C" hipError_t eslam_launch_contact_records(DevState s0, DevState s1, const MapView* map, const StepParams* p, Ctl* ctl,
                                                   const DebugRec* d, const LocalMaps* store, hipStream_t stream)
{
    const uint32_t blocks = (uint32_t)((p->n + kBlock - 1) / kBlock);
    if (!blocks) return hipSuccess;
    K1Args args;
    memset(&args, 0, sizeof(args));
    args.p = *p;
    args.map = *map;
    args.s[0] = s0;
    args.s[1] = s1;
    args.ctl = ctl;
    if (store) args.store = *store;
    if (s0.sid) hipLaunchKernelGGL(k_contact_records<true>, dim3(blocks), dim3(kBlock), 16, stream, args, *d);
    else hipLaunchKernelGGL(k_contact_records<false>, dim3(blocks), dim3(kBlock), 16, stream, args, *d);
    return hipGetLastError();
}

extern "C" hipError_t eslam_launch_pack_records(DevState s0, DevState s1, const Ctl* ctl, uint64_t first, uint64_t stride,
                                                uint64_t count, uint64_t gbase, const uint32_t* anc, const DebugRec* d, eslam_particle_record* out, eslam_cpoint* cps,
                                                uint32_t max_cp, const uint64_t* slot, const double* remote, hipStream_t stream)
{
    const uint32_t blocks = (uint32_t)((count + kBlock - 1) / kBlock);
    if (!blocks) return hipSuccess;
    hipLaunchKernelGGL(k_pack_records, dim3(blocks), dim3(kBlock), 0, stream, s0, s1, ctl, first, stride, count, gbase, anc,
                       *d, out, cps, max_cp, slot, remote);
    return hipGetLastError();
}

extern "C" hipError_t eslam_launch_gather_records(const uint32_t* req, uint64_t nreq, uint64_t gbase, const DebugRec* d,
                                                  double* items, hipStream_t stream)
{
    const uint64_t blocks = (nreq + kBlock - 1) / kBlock;
    if (blocks) hipLaunchKernelGGL(k_gather_records, dim3((uint32_t)blocks), dim3(kBlock), 0, stream, req, nreq, gbase, *d, items);
    return hipGetLastError();
}

extern "C" hipError_t eslam_launch_scan_excl(uint32_t* a, uint64_t m, hipStream_t stream)
{
    if (m) hipLaunchKernelGGL(k_scan_excl, dim3(1), dim3(1024), 0, stream, a, m);
    return hipGetLastError();
}

extern "C" hipError_t eslam_launch_store_init(uint32_t* sid, const LocalMaps* lm, uint64_t n, uint64_t pool, hipStream_t stream)
{
    uint64_t items = pool * lm->S;
    if (lm->npages > items) items = lm->npages;
    const uint64_t want = (items + kBlock - 1) / kBlock;
    if (items) hipLaunchKernelGGL(k_store_init, dim3((uint32_t)(want < 65536 ? want : 65536)), dim3(kBlock), 0, stream, sid, *lm, n,
                                  pool, items);
    return hipGetLastError();
}

// one compaction (k_compact_count, the exclusive prefix over tiles + 1 entries -- entry tiles
// becomes the total, copied to *total when total is not null -- and k_compact_write) of the
// items [0, items); gate: see k_compact_count
static hipError_t compact(int mode, uint64_t items, const uint32_t* ref, SidRef sid, uint32_t* counts, uint32_t* out,
                          uint32_t* total, hipStream_t stream, const uint32_t* gate = nullptr)
{
    const uint32_t tiles = (uint32_t)((items + kCompactTile - 1) / kCompactTile);
    hipError_t e = hipMemsetAsync(counts + tiles, 0, 4, stream);
    if (e != hipSuccess) return e;
    if (tiles) hipLaunchKernelGGL(k_compact_count, dim3(tiles), dim3(kBlock), 0, stream, mode, items, ref, sid, counts, gate);
    hipLaunchKernelGGL(k_scan_excl, dim3(1), dim3(1024), 0, stream, counts, (uint64_t)tiles + 1);
    if (tiles) hipLaunchKernelGGL(k_compact_write, dim3(tiles), dim3(kBlock), 0, stream, mode, items, ref, sid, counts, out, gate);
    return total ? hipMemcpyAsync(total, counts + tiles, 4, hipMemcpyDeviceToDevice, stream) : hipGetLastError();
}

// the tables' reference counts (and generations) and the free-table list of the pool (before a
// map merge or a copy on write): cs.ref, cs.frees, *cs.nfree
extern "C" hipError_t eslam_launch_store_refs(SidRef sid, uint64_t n, uint64_t pool, const CowScratch* cs, const GatherView* gv,
                                              uint32_t* tgen, hipStream_t stream)
{
    hipError_t e = hipMemsetAsync(cs->ref, 0, pool * 4, stream);
    if (e != hipSuccess) return e;
    GatherView g;
    memset(&g, 0, sizeof(g));
    if (gv) g = *gv;
    if (n) hipLaunchKernelGGL(k_store_ref, dim3((uint32_t)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream, sid, n, cs->ref,
                              g, gv ? 1u : 0u, tgen);
    e = compact(0, pool, cs->ref, sid, cs->counts, cs->frees, cs->nfree, stream);
    return e != hipSuccess ? e : hipGetLastError();
}

// the page budget of a plan (mp->poff holds the block sums of mp->need over nblocks blocks):
// the offsets, and a collection when the free list runs short (the gated kernels return at
// once otherwise).  pgc: the collection's compaction counts (npages / kCompactTile + 1 words)
static hipError_t page_budget(Ctl* ctl, const LocalMaps* lm, const MergeParams* mp, uint32_t nblocks, uint32_t* pgc,
                              hipStream_t stream)
{
    hipLaunchKernelGGL(k_scan_excl, dim3(1), dim3(1024), 0, stream, mp->poff, (uint64_t)nblocks + 1);
    hipLaunchKernelGGL(k_page_budget, dim3(1), dim3(1), 0, stream, ctl, mp->poff, nblocks);
    const uint32_t* gate = &ctl->pg_gc;
    const uint64_t n16 = (lm->npages + 15) / 16;
    const uint64_t gcl = (n16 + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(k_pg_clear, dim3((uint32_t)(gcl < 8192 ? gcl : 8192)), dim3(kBlock), 0, stream, lm->mark, lm->npages, gate);
    const uint64_t gm = (lm->ntables + kWaves - 1) / kWaves;
    hipLaunchKernelGGL(k_pg_mark, dim3((uint32_t)(gm < 16384 ? gm : 16384)), dim3(kBlock), 0, stream, *lm, mp->ref, gate);
    const SidRef none{nullptr, nullptr, nullptr};
    hipError_t e = compact(2, lm->npages, reinterpret_cast<const uint32_t*>(lm->mark), none, pgc, lm->frees, nullptr, stream, gate);
    if (e != hipSuccess) return e;
    const uint32_t tiles = (uint32_t)((lm->npages + kCompactTile - 1) / kCompactTile);
    hipLaunchKernelGGL(k_page_budget2, dim3(1), dim3(1), 0, stream, ctl, pgc, tiles, mp->fault);
    return hipGetLastError();
}

// a map update in two halves (timed apart): the plan (k_map_plan, the page budget and, when
// the free list runs short, the collection), then the merge and its counters
extern "C" hipError_t eslam_launch_map_plan(DevState s0, DevState s1, Ctl* ctl, const MapView* map, const LocalMaps* lm,
                                            const MergeParams* mp, uint32_t* pgc, hipStream_t stream)
{
    hipError_t e = hipMemsetAsync(mp->cnt, 0, kMergeCounters * kMergeCounterSlots * sizeof(uint64_t), stream);
    if (e != hipSuccess) return e;
    const uint32_t nb = (uint32_t)((mp->n + kLmBlock - 1) / kLmBlock);
    e = hipMemsetAsync(mp->poff + nb, 0, 4, stream);
    if (e != hipSuccess) return e;
    if (nb && mp->m > kScanPartSmall)
        hipLaunchKernelGGL(k_map_plan<kScanPartLarge>, dim3(nb), dim3(kLmBlock), 0, stream, s0, s1, ctl, *map, *lm, *mp);
    else if (nb)
        hipLaunchKernelGGL(k_map_plan<kScanPartSmall>, dim3(nb), dim3(kLmBlock), 0, stream, s0, s1, ctl, *map, *lm, *mp);
    return page_budget(ctl, lm, mp, nb, pgc, stream);
}

extern "C" hipError_t eslam_launch_map_match(DevState s0, DevState s1, const Ctl* ctl, const MapView* map, const LocalMaps* lm,
                                             const MatchParams* mp, hipStream_t stream)
{
    const uint64_t blocks = (mp->n + kBlock - 1) / kBlock;
    if (blocks && lm) hipLaunchKernelGGL(k_map_match<true>, dim3((uint32_t)blocks), dim3(kBlock), 0, stream, s0, s1, ctl, *map, *lm, *mp);
    if (blocks && !lm) {
        LocalMaps none;
        memset(&none, 0, sizeof(none));
        hipLaunchKernelGGL(k_map_match<false>, dim3((uint32_t)blocks), dim3(kBlock), 0, stream, s0, s1, ctl, *map, none, *mp);
    }
    return hipGetLastError();
}

extern "C" hipError_t eslam_launch_map_merge(DevState s0, DevState s1, Ctl* ctl, const MapView* map, const LocalMaps* lm,
                                             const MergeParams* mp, hipStream_t stream)
{
    const uint32_t nb = (uint32_t)((mp->n + kLmPpb - 1) / kLmPpb);
    if (nb && mp->m > kScanPartSmall)
        hipLaunchKernelGGL(k_map_merge<kScanPartLarge>, dim3(nb), dim3(kLmMergeBlock), 0, stream, s0, s1, ctl, *map, *lm, *mp);
    else if (nb)
        hipLaunchKernelGGL(k_map_merge<kScanPartSmall>, dim3(nb), dim3(kLmMergeBlock), 0, stream, s0, s1, ctl, *map, *lm, *mp);
    hipLaunchKernelGGL(k_merge_counts, dim3(1), dim3(kMergeCounterSlots), 0, stream, mp->cnt, ctl, mp->acc);
    return hipGetLastError();
}

// ---- sharded filters: the maps travel with the migrating particles -----------------------
// k_pack's companion: each record's map header (its source's table centre and page count).
// A record is one output; the copies of one source that go to one rank are consecutive
// records, and only the first of them carries the map (the others share it: one table and one
// set of pages on the receiver, as the copies share them here)
__device__ __forceinline__ bool pay_shares(const Rec* send, uint64_t j, const PaySeg& seg)
{
    if (j == 0 || (send[j].src >> 8) != (send[j - 1].src >> 8)) return false;
    for (int32_t d = 0; d <= seg.n; ++d)
        if (seg.off[d] == j) return false;               // the first record for a destination
    return true;
}

__global__ void __launch_bounds__(kBlock) k_pay_hdr(const DevState s0, const DevState s1, const Ctl* __restrict__ ctl,
                                                   const Rec* __restrict__ send, uint64_t nsend, uint64_t gbase, LocalMaps lm,
                                                   PaySeg seg, MapPayHdr* __restrict__ hdr)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nw = (uint64_t)gridDim.x * kWaves;
    const DevState st = ctl->base ? s1 : s0;
    for (uint64_t j = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6); j < nsend; j += nw) {
        const uint64_t i = (send[j].src >> 8) - gbase;
        const uint32_t X = st.sid[i];
        const bool share = pay_shares(send, j, seg);
        const uint32_t* row = lm.slot + (uint64_t)X * lm.S;
        const uint32_t toff = lm.S - 4u * lm.V;
        uint32_t c = 0;
        if (!share) {
            for (uint32_t s = lane; s < toff; s += 64u) c += row[s] != DM_LM_NONE ? 1u : 0u;
            const uint32_t hw = lm_hw_word(row[toff - 1u]);
            for (uint32_t e = lane; e < hw; e += 64u) c += row[toff + 4u * e + 2u] != DM_LM_NONE ? 1u : 0u;
            c = wave_sum_u32(c);
        }
        if (lane == 0) {
            MapPayHdr h;
            h.ctr = lm.ctr[X];
            h.npg = c;
            h.share = (share ? 1u : 0u) | (row[toff - 2u] == kLmShadow ? 2u : 0u);
            hdr[j] = h;
        }
    }
}

// the records' pages in the records' order (off: exclusive prefix of the headers' npg), the
// window's in slot order then the trail's in entry order; one wave per record: its lanes copy
// each page's 64 cells
__global__ void __launch_bounds__(kBlock) k_pay_pack(const DevState s0, const DevState s1, const Ctl* __restrict__ ctl,
                                                    const Rec* __restrict__ send, uint64_t nsend, uint64_t gbase, LocalMaps lm,
                                                    const MapPayHdr* __restrict__ hdr, const uint32_t* __restrict__ off,
                                                    MapPayPage* __restrict__ pay)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nw = (uint64_t)gridDim.x * kWaves;
    const DevState st = ctl->base ? s1 : s0;
    for (uint64_t j = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6); j < nsend; j += nw) {
        if (hdr[j].share & 1u) continue;                 // the previous record carries the map
        const uint64_t i = (send[j].src >> 8) - gbase;
        const uint32_t X = st.sid[i];
        const uint32_t* row = lm.slot + (uint64_t)X * lm.S;
        const uint32_t toff = lm.S - 4u * lm.V;
        uint64_t q = off[j];
        const uint32_t hw = lm_hw_word(row[toff - 1u]);
        for (uint32_t s = 0; s < toff + hw; ++s) {
            const bool tr = s >= toff;
            const uint32_t p = tr ? row[toff + 4u * (s - toff) + 2u] : row[s];
            if (p == DM_LM_NONE) continue;
            if (lane == 0) {
                pay[q].slot = tr ? (kPayTrail | (s - toff)) : s;
                pay[q].a = tr ? (int32_t)row[toff + 4u * (s - toff)] : 0;
                pay[q].b = tr ? (int32_t)row[toff + 4u * (s - toff) + 1u] : 0;
                pay[q].pad = 0;
            }
            pay[q].cell[lane] = lm.page[(uint64_t)p * DM_LM_PAGE_CELLS + lane];
            ++q;
        }
    }
}

// exclusive prefix of the headers' page counts (one block; out: m + 1 words)
__global__ void __launch_bounds__(1024) k_pay_prefix(const MapPayHdr* __restrict__ hdr, uint64_t m, uint32_t* __restrict__ out)
{
    __shared__ uint32_t s_sum[1024];
    const uint64_t per = (m + 1023) / 1024;
    const uint64_t lo = threadIdx.x * per, hi = lo + per < m ? lo + per : m;
    uint32_t t = 0;
    for (uint64_t i = lo; i < hi; ++i) t += hdr[i].npg;
    s_sum[threadIdx.x] = t;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const uint32_t v = threadIdx.x >= (uint32_t)o ? s_sum[threadIdx.x - o] : 0u;
        __syncthreads();
        s_sum[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = s_sum[threadIdx.x] - t;
    for (uint64_t i = lo; i < hi; ++i) {
        out[i] = run;
        run += hdr[i].npg;
    }
    if (threadIdx.x == 1023) out[m] = s_sum[1023];
}

// the received records' map owners: head[r] = the last record at or before r that carries a
// map (the copies of one source that came together share it); one block, ranges per thread
__global__ void __launch_bounds__(1024) k_recv_heads(const MapPayHdr* __restrict__ hdr, uint64_t m, uint32_t* __restrict__ head)
{
    __shared__ uint32_t s_h[1024];
    const uint64_t per = (m + 1023) / 1024;
    const uint64_t lo = threadIdx.x * per, hi = lo + per < m ? lo + per : m;
    uint32_t h = 0;                                      // 1 + the last head of the range (0: none)
    for (uint64_t i = lo; i < hi; ++i)
        if (!(hdr[i].share & 1u)) h = (uint32_t)i + 1u;
    s_h[threadIdx.x] = h;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {                 // inclusive max-scan over the threads
        const uint32_t v = threadIdx.x >= (uint32_t)o ? s_h[threadIdx.x - o] : 0u;
        __syncthreads();
        s_h[threadIdx.x] = max(s_h[threadIdx.x], v);
        __syncthreads();
    }
    uint32_t run = threadIdx.x ? s_h[threadIdx.x - 1] : 0u;
    for (uint64_t i = lo; i < hi; ++i) {
        if (!(hdr[i].share & 1u)) run = (uint32_t)i + 1u;
        head[i] = run ? run - 1u : 0u;                   // record 0 always carries its map
    }
}

// the received records' maps: a record r that carries one takes free table frees[r] and its
// pages at hoff[r] past the free list's cursor, filled from the payload; the records sharing it
// (and every output of them) name that table, which their next map update then finds shared --
// copy on write, as the copies of a one-GPU resample.  One wave per record: its lanes copy
// each page's cells, then write the table's row (window slots, then the trail's entries
// {a, b, page, -})
__global__ void __launch_bounds__(kLmBlock) k_recv_maps(uint64_t nrec, const uint32_t* __restrict__ frees, Ctl* __restrict__ ctl,
                                                        const MapPayHdr* __restrict__ hdr, const uint32_t* __restrict__ hoff,
                                                        const MapPayPage* __restrict__ pay, LocalMaps lm)
{
    if (ctl->err & kFaultPages) return;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nw = (uint64_t)gridDim.x * (kLmBlock / 64);
    const uint32_t toff = lm.S - 4u * lm.V;
    for (uint64_t r = (uint64_t)blockIdx.x * (kLmBlock / 64) + (threadIdx.x >> 6); r < nrec; r += nw) {
        if (hdr[r].share & 1u) continue;
        const uint64_t alloc = ctl->pg_cursor + hoff[r];
        const uint32_t T = frees[r];
        const uint64_t gT = ((uint64_t)lm.tgen[T] << 32) | T;
        const uint32_t npg = hdr[r].npg;
        const uint64_t q0 = hoff[r];
        for (uint32_t q = 0; q < npg; ++q) {
            const uint32_t np = lm.frees[alloc + q];
            lm.page[(uint64_t)np * DM_LM_PAGE_CELLS + lane] = pay[q0 + q].cell[lane];
            if (lane == 0) lm.owner[np] = gT;
        }
        uint32_t* tsl = lm.slot + (uint64_t)T * lm.S;
        for (uint32_t s = lane; s < lm.S; s += 64u) {
            uint32_t v = DM_LM_NONE;
            if (s == toff - 2u) {                        // the map's copies of shared-grid cells
                v = (hdr[r].share & 2u) ? kLmShadow : DM_LM_NONE;
            } else if (s == toff - 1u) {                 // the trail's high-water mark
                for (uint32_t q = 0; q < npg; ++q) {
                    const uint32_t sl = pay[q0 + q].slot;
                    if (sl & kPayTrail) v = (v == DM_LM_NONE || (sl & ~kPayTrail) + 1u > v) ? (sl & ~kPayTrail) + 1u : v;
                }
            } else if (s < toff) {
                for (uint32_t q = 0; q < npg; ++q) v = pay[q0 + q].slot == s ? lm.frees[alloc + q] : v;
            } else {
                const uint32_t e = (s - toff) >> 2, k = (s - toff) & 3u;
                for (uint32_t q = 0; q < npg; ++q) {
                    const MapPayPage& pp = pay[q0 + q];
                    if (pp.slot != (kPayTrail | e)) continue;
                    v = k == 0u ? (uint32_t)pp.a : k == 1u ? (uint32_t)pp.b : k == 2u ? lm.frees[alloc + q] : DM_LM_NONE;
                }
            }
            tsl[s] = v;
        }
        if (lane == 0) lm.ctr[T] = hdr[r].ctr;
    }
}

// the particles a sharded resample received from record r (sid = kSidRecord | r) name the
// table of the record carrying r's map, frees[head[r]]
__global__ void __launch_bounds__(kBlock) k_recv_rename(const uint32_t* __restrict__ dups, const uint32_t* __restrict__ frees,
                                                        const uint32_t* __restrict__ head, const uint32_t* __restrict__ ndup_dev,
                                                        SidRef sr)
{
    uint32_t* sid = cur_sid(sr);
    const uint64_t ndup = *ndup_dev;
    for (uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x; j < ndup; j += (uint64_t)gridDim.x * kBlock)
        sid[dups[j]] = frees[head[sid[dups[j]] & ~kSidRecord]];
}

// the particles a sharded resample received (cs.dups, *cs.ndup, from nrecv records) get their
// records' maps: a free table and pages from the pool per record, filled from the payloads
// (needs eslam_launch_store_refs first): hdr / pay the received headers and pages, hoff
// (nrecv + 1 words) scratch
extern "C" hipError_t eslam_launch_store_receive(SidRef sid, Ctl* ctl, const LocalMaps* lm, const MergeParams* mp, uint64_t n,
                                                 const CowScratch* cs, const void* hdr, uint64_t nrecv, uint32_t* hoff,
                                                 uint32_t* head, const void* pay, uint32_t* pgc, hipStream_t stream)
{
    if (!n) return hipSuccess;
    hipError_t e = compact(1, n, cs->ref, sid, cs->counts + cs->tiles + 1, cs->dups, cs->ndup, stream);
    if (e != hipSuccess) return e;
    const MapPayHdr* h = (const MapPayHdr*)hdr;
    if (nrecv) {
        hipLaunchKernelGGL(k_pay_prefix, dim3(1), dim3(1024), 0, stream, h, nrecv, hoff);
        hipLaunchKernelGGL(k_recv_heads, dim3(1), dim3(1024), 0, stream, h, nrecv, head);
    } else {
        e = hipMemsetAsync(hoff, 0, 4, stream);
        if (e != hipSuccess) return e;
    }
    // the plan is the records' page counts: one "block" whose sum is hoff[nrecv]
    e = hipMemcpyAsync(mp->poff, hoff + nrecv, 4, hipMemcpyDeviceToDevice, stream);
    if (e == hipSuccess) e = hipMemsetAsync(mp->poff + 1, 0, 4, stream);
    if (e != hipSuccess) return e;
    e = page_budget(ctl, lm, mp, 1u, pgc, stream);
    if (e != hipSuccess) return e;
    const uint64_t gw = (nrecv + kLmBlock / 64 - 1) / (kLmBlock / 64);
    if (nrecv)
        hipLaunchKernelGGL(k_recv_maps, dim3((uint32_t)(gw < 8192 ? gw : 8192)), dim3(kLmBlock), 0, stream, nrecv, cs->frees, ctl, h,
                           hoff, (const MapPayPage*)pay, *lm);
    hipLaunchKernelGGL(k_pg_advance, dim3(1), dim3(1), 0, stream, ctl);
    const uint64_t want_r = (n + kBlock - 1) / kBlock;
    const uint32_t gr = (uint32_t)(want_r < 2048 ? want_r : 2048);
    hipLaunchKernelGGL(k_recv_rename, dim3(gr), dim3(kBlock), 0, stream, cs->dups, cs->frees, head, cs->ndup, sid);
    return hipGetLastError();
}

// a sharded resample's map payloads (after k_pack): headers, their prefix (off: nsend + 1
// words; the host reads the per-destination page counts from it), then the pages
extern "C" hipError_t eslam_launch_pay_hdr(DevState s0, DevState s1, const Ctl* ctl, const void* send, uint64_t nsend,
                                           uint64_t gbase, const LocalMaps* lm, const PaySeg* seg, void* hdr, uint32_t* off,
                                           hipStream_t stream)
{
    if (!nsend) return hipMemsetAsync(off, 0, 4, stream);
    const uint64_t g = (nsend + kWaves - 1) / kWaves;
    hipLaunchKernelGGL(k_pay_hdr, dim3((uint32_t)(g < 4096 ? g : 4096)), dim3(kBlock), 0, stream, s0, s1, ctl, (const Rec*)send,
                       nsend, gbase, *lm, *seg, (MapPayHdr*)hdr);
    hipLaunchKernelGGL(k_pay_prefix, dim3(1), dim3(1024), 0, stream, (const MapPayHdr*)hdr, nsend, off);
    return hipGetLastError();
}

extern "C" hipError_t eslam_launch_pay_pack(DevState s0, DevState s1, const Ctl* ctl, const void* send, uint64_t nsend,
                                            uint64_t gbase, const LocalMaps* lm, const void* hdr, const uint32_t* off, void* pay,
                                            hipStream_t stream)
{
    if (!nsend) return hipSuccess;
    const uint64_t g = (nsend + kWaves - 1) / kWaves;
    hipLaunchKernelGGL(k_pay_pack, dim3((uint32_t)(g < 4096 ? g : 4096)), dim3(kBlock), 0, stream, s0, s1, ctl, (const Rec*)send,
                       nsend, gbase, *lm, (const MapPayHdr*)hdr, off, (MapPayPage*)pay);
    return hipGetLastError();
}

extern "C" hipError_t eslam_launch_weight_stats(DevState s0, DevState s1, uint64_t n, uint32_t J, Ctl* ctl, Shard* shards,
                                                hipStream_t stream)
{
    const uint64_t csz = 64ull * J;
    const uint64_t chunks = (n + csz - 1) / csz;
    const uint32_t blocks = (uint32_t)((chunks + kWaves - 1) / kWaves);
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_weight_stats, dim3(blocks), dim3(kBlock), 0, stream, s0, s1, n, J, ctl, shards);
    return hipGetLastError();
}

extern "C" hipError_t eslam_launch_finalize(Shard* recs, int nrec, Ctl* ctl, const FinParams* fp, hipStream_t stream)
{
    hipLaunchKernelGGL(k_finalize, dim3(1), dim3(kBlock), 0, stream, recs, nrec, ctl, *fp);
    return hipGetLastError();
}

// ff: the update step's finalize fused into block 0 (nullptr: k_finalize ran before)
extern "C" hipError_t eslam_launch_normalize_scan(DevState s0, DevState s1, const ScanParams* sp, Ctl* ctl, uint64_t* tile_sum,
                                                  uint64_t* total, const FusedFin* ff, hipStream_t stream)
{
    if (sp->ntiles == 0) return hipSuccess;
    if (sp->tag < 1 || sp->tag > 7) return hipErrorInvalidValue;
    FusedFin none;
    memset(&none, 0, sizeof(none));
    const FusedFin& f = ff ? *ff : none;
#define ESLAM_K3A(I)                                                                                                  \
    do {                                                                                                              \
        if (ff) hipLaunchKernelGGL((k_normalize_scan<I, true>), dim3(sp->ntiles), dim3(kBlock), 0, stream, s0, s1, *sp, \
                                   ctl, tile_sum, total, f);                                                          \
        else hipLaunchKernelGGL((k_normalize_scan<I, false>), dim3(sp->ntiles), dim3(kBlock), 0, stream, s0, s1, *sp,   \
                                ctl, tile_sum, total, f);                                                             \
    } while (0)
    switch (sp->items) {
    case 2: ESLAM_K3A(2); break;
    case 4: ESLAM_K3A(4); break;
    case kScanItems: ESLAM_K3A(kScanItems); break;
    default: return hipErrorInvalidValue;
    }
#undef ESLAM_K3A
    return hipGetLastError();
}

extern "C" hipError_t eslam_launch_normalize_segments(DevState s0, DevState s1, const ScanParams* sp, Ctl* ctl,
                                                      uint64_t* tile_pub, uint32_t* marks, uint32_t* tile_first,
                                                      const uint32_t* jt, const FusedFin* ff, hipStream_t stream)
{
    if (sp->ntiles == 0) return hipSuccess;
    if (sp->tag < 1 || sp->tag > 7) return hipErrorInvalidValue;
    if (ff && (!ff->shards || !ff->fin_word || ff->fp.mode != FIN_UPDATE || ff->fp.mirror)) return hipErrorInvalidValue;
    const FusedFin none{};
#define ESLAM_SEG(I) do { \
        if (ff) hipLaunchKernelGGL((k_normalize_segments<I, true>), dim3(sp->ntiles), dim3(kBlock), 0, stream, s0, s1, *sp, ctl, \
                                   tile_pub, marks, tile_first, jt, *ff); \
        else hipLaunchKernelGGL((k_normalize_segments<I, false>), dim3(sp->ntiles), dim3(kBlock), 0, stream, s0, s1, *sp, ctl, \
                                tile_pub, marks, tile_first, jt, none); \
    } while (0)
    switch (sp->items) {
    case 1: ESLAM_SEG(1); break;
    case 2: ESLAM_SEG(2); break;
    case 4: ESLAM_SEG(4); break;
    case 8: ESLAM_SEG(8); break;
    default: return hipErrorInvalidValue;
    }
#undef ESLAM_SEG
    return hipGetLastError();
}

extern "C" hipError_t eslam_launch_resample_gather(DevState s0, DevState s1, uint64_t n, uint64_t gbase, Ctl* ctl,
                                                   const GatherView* gv, uint32_t aux, hipStream_t stream)
{
    const uint32_t tiles = (uint32_t)((n + kGatherTile - 1) / kGatherTile);
    if (tiles) hipLaunchKernelGGL(k_resample_gather, dim3(tiles), dim3(kBlock), 0, stream, s0, s1, n, gbase, ctl, *gv, aux);
    hipLaunchKernelGGL(k_commit, dim3(1), dim3(64), 0, stream, ctl);
    return hipGetLastError();
}

extern "C" hipError_t eslam_launch_commit(Ctl* ctl, hipStream_t stream)
{
    hipLaunchKernelGGL(k_commit, dim3(1), dim3(64), 0, stream, ctl);
    return hipGetLastError();
}

extern "C" hipError_t eslam_launch_segments_multi(DevState s0, DevState s1, const ScanParams* sp, const PlanParams* pp, Ctl* ctl,
                                                  const uint64_t* tile_prefix, uint32_t* marks, uint32_t* tile_first,
                                                  const uint64_t* totals, const uint32_t* jt, uint2* range, uint64_t* first_last,
                                                  uint64_t* host_out, uint64_t* host_epoch, uint64_t epoch, hipStream_t stream)
{
    if (sp->items != kScanItems) return hipErrorInvalidValue;       // the sharded scan uses full tiles
    if (sp->ntiles) hipLaunchKernelGGL(k_segments_multi, dim3(sp->ntiles), dim3(kBlock), 0, stream, s0, s1, *sp, *pp, ctl,
                                       tile_prefix, marks, tile_first, totals, jt, range, first_last, host_out, host_epoch,
                                       epoch);
    return hipGetLastError();
}

extern "C" hipError_t eslam_launch_pack(DevState s0, DevState s1, Ctl* ctl, const PlanParams* pp, const uint2* range,
                                        const uint64_t* first_last, uint64_t nsend, void* send, hipStream_t stream)
{
    const uint32_t blocks = (uint32_t)((nsend + kBlock - 1) / kBlock);
    if (blocks)
        hipLaunchKernelGGL(k_pack, dim3(blocks), dim3(kBlock), 0, stream, s0, s1, ctl, *pp, range, first_last, (Rec*)send);
    return hipGetLastError();
}

extern "C" hipError_t eslam_launch_expand(const void* recv, uint64_t nrecv, uint64_t W0, uint32_t* marks, uint32_t* row_first,
                                          hipStream_t stream)
{
    if (nrecv) hipLaunchKernelGGL(k_expand, dim3((uint32_t)((nrecv + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream,
                                  (const Rec*)recv, nrecv, W0, marks, row_first);
    return hipGetLastError();
}

extern "C" uint64_t eslam_record_bytes(void) { return sizeof(Rec); }

extern "C" hipError_t eslam_launch_init_gaussian(DevState s0, uint64_t n, uint64_t gbase, uint64_t seed, uint64_t ev,
                                                 const double mu[3], const double sigma[3], double zpos, double zsigma,
                                                 hipStream_t stream)
{
    const uint32_t blocks = (uint32_t)((n + kBlock - 1) / kBlock);
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_init_gaussian, dim3(blocks), dim3(kBlock), 0, stream, s0, n, gbase, seed, ev, mu[0], mu[1], mu[2],
                       sigma[0], sigma[1], sigma[2], zpos, zsigma);
    return hipGetLastError();
}

extern "C" hipError_t eslam_launch_selftest_math(int fn, const double* x, const double* y, double* out, uint64_t n,
                                                 hipStream_t stream)
{
    const uint32_t blocks = (uint32_t)((n + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_selftest_math, dim3(blocks), dim3(kBlock), 0, stream, fn, x, y, out, n);
    return hipGetLastError();
}

extern "C" hipError_t eslam_launch_selftest_bm_radius(unsigned long long* bad, hipStream_t stream)
{
    hipLaunchKernelGGL(k_selftest_bm_radius, dim3(4096), dim3(kBlock), 0, stream, bad);
    return hipGetLastError();
}

extern "C" hipError_t eslam_launch_best_index(DevState s0, DevState s1, uint64_t n, Ctl* ctl, uint64_t* out2,
                                              hipStream_t stream)
{
    const uint64_t init[2] = {0ull, ~0ull};
    hipError_t e = hipMemcpyAsync(out2, init, 16, hipMemcpyHostToDevice, stream);
    if (e != hipSuccess) return e;
    uint32_t blocks = (uint32_t)((n + kBlock - 1) / kBlock);
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(k_best_max, dim3(blocks), dim3(kBlock), 0, stream, s0, s1, n, ctl, out2);
    hipLaunchKernelGGL(k_best_index, dim3(blocks), dim3(kBlock), 0, stream, s0, s1, n, ctl, out2);
    return hipGetLastError();
}

// the fixed pairwise tree over m chunk records of 5 doubles at a (b: scratch of the same
// size; both are overwritten); the total goes to out
static hipError_t centroid_tree(double* a, double* b, uint64_t m, double* out, hipStream_t stream)
{
    while (m > 1) {
        const uint64_t m2 = (m + 1) / 2;
        hipLaunchKernelGGL(k_tree_level, dim3((uint32_t)((m2 + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream, a, b, m);
        double* t = a; a = b; b = t;
        m = m2;
    }
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(out, a, 5 * sizeof(double), hipMemcpyDeviceToDevice, stream);
    return e;
}

// per canonical chunk (64 x J particles) of this context: sum x w, y w, theta w, z w, w
extern "C" hipError_t eslam_launch_centroid_chunks(DevState s0, DevState s1, uint64_t n, uint32_t J, Ctl* ctl,
                                                   double* chunk_out, hipStream_t stream)
{
    const uint64_t csz = 64ull * J;
    const uint64_t chunks = (n + csz - 1) / csz;
    const uint32_t blocks = (uint32_t)((chunks + kWaves - 1) / kWaves);
    if (blocks) hipLaunchKernelGGL(k_centroid_chunks, dim3(blocks), dim3(kBlock), 0, stream, s0, s1, n, J, ctl, chunk_out);
    return hipGetLastError();
}

// sharded getCentroid: the tree over the all-gathered chunk records (m chunks at a, b scratch)
extern "C" hipError_t eslam_launch_centroid_tree(double* a, double* b, uint64_t m, double* out, hipStream_t stream)
{
    if (m == 0) return hipMemsetAsync(out, 0, 5 * sizeof(double), stream);
    return centroid_tree(a, b, m, out, stream);
}

extern "C" hipError_t eslam_launch_centroid(DevState s0, DevState s1, uint64_t n, uint32_t J, Ctl* ctl, double* out,
                                            hipStream_t stream)
{
    const uint64_t csz = 64ull * J;
    const uint64_t chunks = (n + csz - 1) / csz;
    const uint64_t cap = chunks ? chunks : 1;
    double* tmp = nullptr;
    hipError_t e = hipMallocAsync((void**)&tmp, 2 * cap * 5 * sizeof(double), stream);
    if (e != hipSuccess) return e;
    double* a = tmp;
    double* b = tmp + cap * 5;
    e = hipMemsetAsync(a, 0, 5 * sizeof(double), stream);
    if (e == hipSuccess) e = eslam_launch_centroid_chunks(s0, s1, n, J, ctl, a, stream);
    if (e == hipSuccess) e = centroid_tree(a, b, chunks, out, stream);
    (void)hipFreeAsync(tmp, stream);
    return e;
}

// blocks per CU of the main K1 instantiation (diagnostics)
extern "C" int eslam_debug_k1_occupancy(int* blocks_per_cu, int lds)
{
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k_project_weight<true, true, 4, true>, kBlock,
                                                        lds < 0 ? kStatsLds + kWindowLds : lds) == hipSuccess ? 0 : -1;
}

#ifdef ESLAM_STAMPS
// diagnostic builds: zero the stamps (before the launch to be measured: a block that returns
// early then leaves zeros, not an older launch's stamps)
extern "C" int eslam_gpu_debug_stamps_clear(void)
{
    void *a = nullptr, *b = nullptr, *c = nullptr, *g = nullptr;
    if (hipGetSymbolAddress(&a, HIP_SYMBOL(g_stamps_k1)) != hipSuccess || hipGetSymbolAddress(&b, HIP_SYMBOL(g_stamps_k3)) != hipSuccess ||
        hipGetSymbolAddress(&c, HIP_SYMBOL(g_stamps_mg)) != hipSuccess || hipGetSymbolAddress(&g, HIP_SYMBOL(g_stamps_grid)) != hipSuccess)
        return -1;
    const size_t bytes = sizeof(uint64_t) * kStampBlocks * kStampSlots;
    if (hipMemset(a, 0, bytes) != hipSuccess || hipMemset(b, 0, bytes) != hipSuccess || hipMemset(c, 0, bytes) != hipSuccess ||
        hipMemset(g, 0, 12) != hipSuccess)
        return -1;
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

// copy the stamps of the last K1 (which = 1), K3 (which = 3) or map merge (which = 5) launch; returns that launch's
// block count (its grid; blocks past kStampBlocks are not stamped), or -1
extern "C" int64_t eslam_gpu_debug_stamps(int which, uint64_t* out, uint64_t blocks)
{
    if (blocks > kStampBlocks) blocks = kStampBlocks;
    uint32_t grid[3] = {0, 0, 0};
    const hipError_t e = which == 1 ? hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps_k1), blocks * kStampSlots * 8)
                         : which == 3 ? hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps_k3), blocks * kStampSlots * 8)
                                      : hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps_mg), blocks * kStampSlots * 8);
    if (e != hipSuccess || hipMemcpyFromSymbol(grid, HIP_SYMBOL(g_stamps_grid), sizeof(grid)) != hipSuccess) return -1;
    return (int64_t)grid[which == 1 ? 0 : which == 3 ? 1 : 2];
}
#endif
