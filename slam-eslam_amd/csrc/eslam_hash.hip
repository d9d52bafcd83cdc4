// eslam_hash.hip -- SurfaceHash on the GPU (useHash = true):
//   k_hash_sweep      SurfaceHash::create: one thread per (segment, cell) of the sweep
//                     (src/SurfaceHash.hpp:155-231), the item arithmetic shared with the
//                     oracle (dm_hash_item); the host compacts the valid items in order
//   k_hash_poses      the poses of the compacted items
//   k_init_from_hash  PoseEstimator::init(N, hash)  src/PoseEstimator.cpp:75-86
//   k_hash_keys + radix sort + k_hash_replace
//                     PoseEstimator::sampleFromHash  src/PoseEstimator.cpp:130-182: the
//                     replace_count lowest (float weight, index) pairs get hash poses
// Not on the per-step hot path (init, and every hash_period-th project).
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

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

}  // namespace eslam_dev

using namespace eslam_dev;

static uint32_t blocks_for(uint64_t n) { return (uint32_t)((n + kBlock - 1) / kBlock); }

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

// the k lowest particles by (float weight, index) into order[0..k): keys + stable radix sort.
// tmp/tmp_bytes: caller-owned scratch (query with tmp == NULL)
extern "C" hipError_t eslam_hash_sort(DevState s0, DevState s1, const Ctl* ctl, uint64_t n, uint32_t* keys, uint32_t* vals,
                                      uint32_t* keys_out, uint32_t* order, void* tmp, size_t* tmp_bytes, hipStream_t stream)
{
    if (!tmp) return rocprim::radix_sort_pairs(nullptr, *tmp_bytes, keys, keys_out, vals, order, (uint32_t)n, 0u, 32u, stream);
    if (n) hipLaunchKernelGGL(k_hash_keys, dim3(blocks_for(n)), dim3(kBlock), 0, stream, s0, s1, ctl, n, keys, vals);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return rocprim::radix_sort_pairs(tmp, *tmp_bytes, keys, keys_out, vals, order, (uint32_t)n, 0u, 32u, stream);
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
