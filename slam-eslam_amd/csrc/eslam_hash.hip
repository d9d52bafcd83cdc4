// eslam_hash.hip -- SurfaceHash on the GPU (useHash = true):
//   k_hash_sweep      SurfaceHash::create: one thread per (segment, cell) of the sweep
//                     (src/SurfaceHash.hpp:155-231), the item arithmetic shared with the
//                     oracle (dm_hash_item); the host compacts the valid items in order
//   k_hash_poses      the poses of the compacted items
//   k_init_from_hash  PoseEstimator::init(N, hash)  src/PoseEstimator.cpp:75-86
//   k_hash_keys + radix sort + k_hash_replace
//                     PoseEstimator::sampleFromHash  src/PoseEstimator.cpp:130-182: the
//                     replace_count lowest (float weight, index) pairs get hash poses
//   k_radix_hist / (k_scan_excl) / k_radix_scatter
//                     a stable LSD radix sort of (u32 key, u32 value) pairs, 8 bits per
//                     pass: per-tile digit histograms, one exclusive scan in digit-major
//                     order, and a scatter that ranks each tile's elements stably with
//                     wave ballots (peers of a digit) and per-wave digit counts in LDS
// Not on the per-step hot path (init, and every hash_period-th project).
#include <hip/hip_runtime.h>

#include "eslam_internal.h"

namespace eslam_dev {

__global__ void __launch_bounds__(kBlock) k_hash_sweep(dm_hash_grid g, const double* __restrict__ pts,
                                                       const double* __restrict__ orient, uint32_t steps,
                                                       int32_t* __restrict__ out)
{
    const uint64_t cells = (uint64_t)g.width * g.height;
    const uint64_t id = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (id >= cells * steps) return;
    const uint32_t a = (uint32_t)(id / cells);
    const uint64_t rem = id - (uint64_t)a * cells;
    const uint32_t m = (uint32_t)(rem / g.height), n = (uint32_t)(rem - (uint64_t)m * g.height);
    double pose[4];
    out[id] = dm_hash_item(&g, pts + 8 * a, orient[a], m, n, pose);
}

__global__ void __launch_bounds__(kBlock) k_hash_poses(dm_hash_grid g, const double* __restrict__ pts,
                                                       const double* __restrict__ orient, const uint64_t* __restrict__ ids,
                                                       uint64_t count, double* __restrict__ hx, double* __restrict__ hy,
                                                       double* __restrict__ hth, double* __restrict__ hz)
{
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= count) return;
    const uint64_t cells = (uint64_t)g.width * g.height;
    const uint64_t id = ids[j];
    const uint32_t a = (uint32_t)(id / cells);
    const uint64_t rem = id - (uint64_t)a * cells;
    const uint32_t m = (uint32_t)(rem / g.height), n = (uint32_t)(rem - (uint64_t)m * g.height);
    double pose[4];
    dm_hash_item(&g, pts + 8 * a, orient[a], m, n, pose);
    hx[j] = pose[0]; hy[j] = pose[1]; hth[j] = pose[2]; hz[j] = pose[3];
}

// PoseParticle(position, orientation, zPos): zSigma 0, weight 0, floating; mprob 0
__global__ void __launch_bounds__(kBlock) k_init_from_hash(DevState s0, const uint32_t* __restrict__ idx, uint64_t n,
                                                           const double* __restrict__ hx, const double* __restrict__ hy,
                                                           const double* __restrict__ hth, const double* __restrict__ hz)
{
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = idx[i];
    s0.x[i] = hx[k]; s0.y[i] = hy[k]; s0.th[i] = hth[k]; s0.z[i] = hz[k];
    s0.zs[i] = 0.0; s0.w[i] = 0.0; s0.mprob[i] = 0.0;
    s0.flags[i] = (uint8_t)(1u << 7);
}

// ---- stable LSD radix sort of (key, value) pairs -------------------------------------
constexpr int kSortItems = 8;                        // elements per thread of a tile
constexpr int kSortTile = kBlock * kSortItems;       // elements per tile (block)
constexpr int kDigits = 256;

// tile b's count of every digit of bits [shift, shift + 8): hist[d * ntiles + b]
__global__ void __launch_bounds__(kBlock) k_radix_hist(const uint32_t* __restrict__ keys, uint64_t n, int shift,
                                                       uint32_t* __restrict__ hist, uint32_t ntiles)
{
    __shared__ uint32_t s_cnt[kDigits];
    s_cnt[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kSortTile;
    for (int r = 0; r < kSortItems; ++r) {
        const uint64_t e = base + (uint64_t)r * kBlock + threadIdx.x;
        if (e < n) atomicAdd(&s_cnt[(keys[e] >> shift) & 0xffu], 1u);
    }
    __syncthreads();
    hist[(uint64_t)threadIdx.x * ntiles + blockIdx.x] = s_cnt[threadIdx.x];
}

// tile b's elements to their sorted positions: offs[d * ntiles + b] (scanned histogram) +
// the element's rank among the tile's elements of digit d, in element order (stable).
// Rounds of 256 consecutive elements; in a round, lanes of one wave with the same digit
// (the AND of 8 ballots) rank by lane, waves by the per-wave digit counts in LDS.
__global__ void __launch_bounds__(kBlock) k_radix_scatter(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                          uint32_t* __restrict__ kout, uint32_t* __restrict__ vout, uint64_t n,
                                                          int shift, const uint32_t* __restrict__ offs, uint32_t ntiles)
{
    __shared__ uint32_t s_run[kDigits];              // elements of each digit placed so far
    __shared__ uint32_t s_wcnt[kWaves][kDigits];     // this round: per wave, per digit
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    s_run[tid] = offs[(uint64_t)tid * ntiles + blockIdx.x];
    for (int w = 0; w < kWaves; ++w) s_wcnt[w][tid] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kSortTile;
    const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (int r = 0; r < kSortItems; ++r) {
        const uint64_t e = base + (uint64_t)r * kBlock + tid;
        const bool valid = e < n;
        const uint32_t key = valid ? kin[e] : 0u;
        const uint32_t val = valid ? vin[e] : 0u;
        const uint32_t d = (key >> shift) & 0xffu;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        const uint32_t in_wave = (uint32_t)__popcll(peers & below);
        if (valid && in_wave == 0) s_wcnt[wave][d] = (uint32_t)__popcll(peers);
        __syncthreads();
        if (valid) {
            uint32_t pos = s_run[d] + in_wave;
            for (uint32_t w = 0; w < wave; ++w) pos += s_wcnt[w][d];
            kout[pos] = key;
            vout[pos] = val;
        }
        __syncthreads();
        uint32_t add = 0;
        for (int w = 0; w < kWaves; ++w) { add += s_wcnt[w][tid]; s_wcnt[w][tid] = 0; }
        s_run[tid] += add;
        __syncthreads();
    }
}

// sort keys of (float weight, index): ascending float order, -0 == +0, ties by index
__global__ void __launch_bounds__(kBlock) k_hash_keys(DevState s0, DevState s1, const Ctl* __restrict__ ctl, uint64_t n,
                                                      uint32_t* __restrict__ keys, uint32_t* __restrict__ vals)
{
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const DevState st = (ctl->base ^ ctl->flip) ? s1 : s0;
    float wf = (float)st.w[i];
    if (wf == 0.0f) wf = 0.0f;
    uint32_t b;
    __builtin_memcpy(&b, &wf, 4);
    keys[i] = (b >> 31) ? ~b : (b | 0x80000000u);
    vals[i] = (uint32_t)i;
}

__global__ void __launch_bounds__(kBlock) k_hash_replace(DevState s0, DevState s1, const Ctl* __restrict__ ctl,
                                                         const uint32_t* __restrict__ order, const uint32_t* __restrict__ draws,
                                                         uint64_t k, const uint32_t* __restrict__ blist, uint32_t bstart,
                                                         const double* __restrict__ hx, const double* __restrict__ hy,
                                                         const double* __restrict__ hth, const double* __restrict__ hz,
                                                         double weight)
{
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= k) return;
    const DevState st = (ctl->base ^ ctl->flip) ? s1 : s0;
    const uint32_t i = order[j];
    const uint32_t src = blist[bstart + draws[j]];
    st.x[i] = hx[src]; st.y[i] = hy[src]; st.th[i] = hth[src]; st.z[i] = hz[src];
    st.zs[i] = 0.5;
    st.flags[i] = (uint8_t)(st.flags[i] | (1u << 7));
    st.w[i] = weight;
}

// ---- sharded sampleFromHash: every rank's cnt lowest (key, global index) pairs go to every
// rank (an all_to_all_v used as an all-gather of uneven parts, rank order); the stable sort of
// their concatenation by key puts equal keys in global index order, so its first k entries
// are the one-filter order of src/PoseEstimator.cpp:146-152 on every rank
__global__ void __launch_bounds__(kBlock) k_hash_candidates(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ order,
                                                            uint64_t cnt, uint64_t gbase, int nranks, uint2* __restrict__ send)
{
    const uint64_t e = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= cnt) return;
    const uint2 pr = make_uint2(keys[e], (uint32_t)(gbase + order[e]));
    for (int d = 0; d < nranks; ++d) send[(uint64_t)d * cnt + e] = pr;
}

__global__ void __launch_bounds__(kBlock) k_hash_unpack(const uint2* __restrict__ recv, uint64_t m, uint32_t* __restrict__ keys,
                                                        uint32_t* __restrict__ vals)
{
    const uint64_t e = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= m) return;
    keys[e] = recv[e].x;
    vals[e] = recv[e].y;
}

// the j-th lowest (j < k, global order) gets hash pose draws[j] if this rank holds it
__global__ void __launch_bounds__(kBlock) k_hash_replace_global(DevState s0, DevState s1, const Ctl* __restrict__ ctl,
                                                                const uint32_t* __restrict__ gorder,
                                                                const uint32_t* __restrict__ draws, uint64_t k, uint64_t gbase,
                                                                uint64_t n, const uint32_t* __restrict__ blist, uint32_t bstart,
                                                                const double* __restrict__ hx, const double* __restrict__ hy,
                                                                const double* __restrict__ hth, const double* __restrict__ hz,
                                                                double weight)
{
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= k) return;
    const uint64_t gi = gorder[j];
    if (gi < gbase || gi >= gbase + n) return;
    const uint64_t i = gi - gbase;
    const DevState st = (ctl->base ^ ctl->flip) ? s1 : s0;
    const uint32_t src = blist[bstart + draws[j]];
    st.x[i] = hx[src]; st.y[i] = hy[src]; st.th[i] = hth[src]; st.z[i] = hz[src];
    st.zs[i] = 0.5;
    st.flags[i] = (uint8_t)(st.flags[i] | (1u << 7));
    st.w[i] = weight;
}

}  // namespace eslam_dev

using namespace eslam_dev;

static uint32_t blocks_for(uint64_t n) { return (uint32_t)((n + kBlock - 1) / kBlock); }

extern "C" hipError_t eslam_launch_scan_excl(uint32_t* a, uint64_t m, hipStream_t stream);   // eslam_kernels.hip

extern "C" hipError_t eslam_launch_hash_sweep(const dm_hash_grid* g, const double* pts, const double* orient, uint32_t steps,
                                              int32_t* out, hipStream_t stream)
{
    const uint64_t total = (uint64_t)g->width * g->height * steps;
    if (total) hipLaunchKernelGGL(k_hash_sweep, dim3(blocks_for(total)), dim3(kBlock), 0, stream, *g, pts, orient, steps, out);
    return hipGetLastError();
}

extern "C" hipError_t eslam_launch_hash_poses(const dm_hash_grid* g, const double* pts, const double* orient, const uint64_t* ids,
                                              uint64_t count, double* hx, double* hy, double* hth, double* hz,
                                              hipStream_t stream)
{
    if (count) hipLaunchKernelGGL(k_hash_poses, dim3(blocks_for(count)), dim3(kBlock), 0, stream, *g, pts, orient, ids, count,
                                  hx, hy, hth, hz);
    return hipGetLastError();
}

extern "C" hipError_t eslam_launch_init_from_hash(DevState s0, const uint32_t* idx, uint64_t n, const double* hx,
                                                  const double* hy, const double* hth, const double* hz, hipStream_t stream)
{
    if (n) hipLaunchKernelGGL(k_init_from_hash, dim3(blocks_for(n)), dim3(kBlock), 0, stream, s0, idx, n, hx, hy, hth, hz);
    return hipGetLastError();
}

// stable radix sort of n (key, value) pairs: keys/vals in, sorted into keys_out/order.
// tmp: scratch for the digit histograms and one ping-pong pair (query its size with
// tmp == NULL).  Four passes of 8 bits; the pass results alternate so the last lands in
// keys_out/order.
extern "C" hipError_t eslam_radix_sort_pairs(uint32_t* keys, uint32_t* vals, uint32_t* keys_out, uint32_t* order, uint64_t n,
                                             void* tmp, size_t* tmp_bytes, hipStream_t stream)
{
    const uint32_t ntiles = (uint32_t)((n + kSortTile - 1) / kSortTile);
    const uint64_t hist_words = (uint64_t)kDigits * (ntiles ? ntiles : 1);
    const size_t need = hist_words * 4 + 2 * (n ? n : 1) * 4;
    if (!tmp) { *tmp_bytes = need; return hipSuccess; }
    if (*tmp_bytes < need) return hipErrorInvalidValue;
    if (!n) return hipSuccess;
    uint32_t* hist = (uint32_t*)tmp;
    uint32_t* tk = hist + hist_words;
    uint32_t* tv = tk + n;
    // passes: keys -> (tk, tv) -> (keys_out, order) -> (tk, tv) -> (keys_out, order)
    const uint32_t* ki = keys;
    const uint32_t* vi = vals;
    for (int pass = 0; pass < 4; ++pass) {
        uint32_t* ko = (pass & 1) ? keys_out : tk;
        uint32_t* vo = (pass & 1) ? order : tv;
        hipLaunchKernelGGL(k_radix_hist, dim3(ntiles), dim3(kBlock), 0, stream, ki, n, 8 * pass, hist, ntiles);
        (void)eslam_launch_scan_excl(hist, hist_words, stream);
        hipLaunchKernelGGL(k_radix_scatter, dim3(ntiles), dim3(kBlock), 0, stream, ki, vi, ko, vo, n, 8 * pass, hist, ntiles);
        ki = ko;
        vi = vo;
    }
    return hipGetLastError();
}

// the k lowest particles by (float weight, index) into order[0..k): keys + the stable sort.
// tmp/tmp_bytes: caller-owned scratch (query with tmp == NULL)
extern "C" hipError_t eslam_hash_sort(DevState s0, DevState s1, const Ctl* ctl, uint64_t n, uint32_t* keys, uint32_t* vals,
                                      uint32_t* keys_out, uint32_t* order, void* tmp, size_t* tmp_bytes, hipStream_t stream)
{
    if (!tmp) return eslam_radix_sort_pairs(nullptr, nullptr, nullptr, nullptr, n, nullptr, tmp_bytes, stream);
    if (n) hipLaunchKernelGGL(k_hash_keys, dim3(blocks_for(n)), dim3(kBlock), 0, stream, s0, s1, ctl, n, keys, vals);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return eslam_radix_sort_pairs(keys, vals, keys_out, order, n, tmp, tmp_bytes, stream);
}

extern "C" hipError_t eslam_launch_hash_replace(DevState s0, DevState s1, const Ctl* ctl, const uint32_t* order,
                                                const uint32_t* draws, uint64_t k, const uint32_t* blist, uint32_t bstart,
                                                const double* hx, const double* hy, const double* hth, const double* hz,
                                                double weight, hipStream_t stream)
{
    if (k) hipLaunchKernelGGL(k_hash_replace, dim3(blocks_for(k)), dim3(kBlock), 0, stream, s0, s1, ctl, order, draws, k,
                              blist, bstart, hx, hy, hth, hz, weight);
    return hipGetLastError();
}

extern "C" hipError_t eslam_launch_hash_candidates(const uint32_t* keys, const uint32_t* order, uint64_t cnt, uint64_t gbase,
                                                   int nranks, void* send, hipStream_t stream)
{
    if (cnt) hipLaunchKernelGGL(k_hash_candidates, dim3(blocks_for(cnt)), dim3(kBlock), 0, stream, keys, order, cnt, gbase,
                                nranks, (uint2*)send);
    return hipGetLastError();
}

extern "C" hipError_t eslam_launch_hash_unpack(const void* recv, uint64_t m, uint32_t* keys, uint32_t* vals, hipStream_t stream)
{
    if (m) hipLaunchKernelGGL(k_hash_unpack, dim3(blocks_for(m)), dim3(kBlock), 0, stream, (const uint2*)recv, m, keys, vals);
    return hipGetLastError();
}

extern "C" hipError_t eslam_launch_hash_replace_global(DevState s0, DevState s1, const Ctl* ctl, const uint32_t* gorder,
                                                       const uint32_t* draws, uint64_t k, uint64_t gbase, uint64_t n,
                                                       const uint32_t* blist, uint32_t bstart, const double* hx,
                                                       const double* hy, const double* hth, const double* hz, double weight,
                                                       hipStream_t stream)
{
    if (k) hipLaunchKernelGGL(k_hash_replace_global, dim3(blocks_for(k)), dim3(kBlock), 0, stream, s0, s1, ctl, gorder, draws,
                              k, gbase, n, blist, bstart, hx, hy, hth, hz, weight);
    return hipGetLastError();
}
