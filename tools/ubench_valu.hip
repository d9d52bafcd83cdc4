// Issue cost of the VALU instructions K1 and K3 lean on (gfx950): one block of W waves on
// one CU, each lane running 8 independent chains of one instruction kind, timed with
// s_memtime (the wave's own clock) around 256 iterations.  Prints cycles per wave-instruction
// per SIMD (4 waves per block spread over the 4 SIMDs: W = 4 -> one wave per SIMD, W = 16 ->
// four).  Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_valu.hip -o /tmp/ubench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kIters = 256;

#define CHAINS8(stmt)                                                                               \
    _Pragma("unroll") for (int c = 0; c < 8; ++c) { stmt; }

template <int KIND>
__global__ void k_bench(const double* in, double* out, uint64_t* cyc)
{
    const int t = threadIdx.x;
    double d[8];
    uint32_t u[8];
    float f[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) { d[c] = in[(t + c) & 63]; u[c] = (uint32_t)(d[c] * 1e6) + c; f[c] = (float)d[c]; }
    const double k1 = in[64], k2 = in[65];
    const uint32_t m1 = 0xD2511F53u;
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; ++it) {
        if constexpr (KIND == 0) {           // v_fma_f64
            CHAINS8(d[c] = __builtin_fma(d[c], k1, k2))
        } else if constexpr (KIND == 1) {    // v_mad_u64_u32 (Philox round: hi/lo of a 32x32 product)
            CHAINS8({ const uint64_t p = (uint64_t)m1 * u[c]; u[c] = (uint32_t)(p >> 32) ^ (uint32_t)p; })
        } else if constexpr (KIND == 2) {    // v_rcp_f64
            CHAINS8(d[c] = __builtin_amdgcn_rcp(d[c]))
        } else if constexpr (KIND == 3) {    // v_rsq_f64
            CHAINS8(d[c] = __builtin_amdgcn_rsq(d[c]))
        } else if constexpr (KIND == 4) {    // v_fma_f32
            CHAINS8(f[c] = __builtin_fmaf(f[c], 1.0001f, 0.5f))
        } else if constexpr (KIND == 5) {    // v_sqrt_f32
            CHAINS8(f[c] = __builtin_amdgcn_sqrtf(f[c]))
        } else if constexpr (KIND == 6) {    // v_cvt_f64_f32 + v_cvt_f32_f64
            CHAINS8(f[c] = (float)((double)f[c] * 1.0))
        } else if constexpr (KIND == 7) {    // v_add_u32 / v_xor (integer full rate)
            CHAINS8(u[c] = (u[c] + 0x9E3779B9u) ^ m1)
        } else if constexpr (KIND == 8) {    // v_mul_lo_u32
            CHAINS8(u[c] = u[c] * m1)
        } else if constexpr (KIND == 9) {    // v_cvt_i32_f64
            CHAINS8({ int q; asm volatile("v_cvt_i32_f64 %0, %1" : "=v"(q) : "v"(d[c])); u[c] += (uint32_t)q; })
        } else if constexpr (KIND == 10) {   // v_pk_fma_f32 (two fp32 FMAs)
            typedef float f2 __attribute__((ext_vector_type(2)));
            const f2 ka = {1.0001f, 1.0002f}, kb = {0.5f, 0.25f};
#pragma unroll
            for (int c = 0; c < 8; c += 2) {
                f2 a;
                a.x = f[c];
                a.y = f[c + 1];
                a = __builtin_elementwise_fma(a, ka, kb);
                f[c] = a.x;
                f[c + 1] = a.y;
            }
        } else if constexpr (KIND == 11) {   // v_lshlrev_b64 (64-bit shift)
            CHAINS8({ uint64_t v = ((uint64_t)u[c] << 32) | u[(c + 1) & 7]; v = v << (u[c] & 31); u[c] = (uint32_t)(v >> 32) ^ (uint32_t)v; })
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    double acc = 0.0;
#pragma unroll
    for (int c = 0; c < 8; ++c) acc += d[c] + (double)u[c] + (double)f[c];
    out[blockIdx.x * blockDim.x + t] = acc;
    if ((t & 63) == 0) cyc[t >> 6] = t1 - t0;
}

static const char* kName[] = {"v_fma_f64", "v_mad_u64_u32 (+xor)", "v_rcp_f64", "v_rsq_f64", "v_fma_f32", "v_sqrt_f32",
                              "cvt f32->f64->f32 (+mul)", "v_add_u32+v_xor", "v_mul_lo_u32", "v_cvt_i32_f64 (+add)",
                              "v_pk_fma_f32 (+add)", "v_lshlrev_b64 (+ops)"};

template <int KIND>
static void run(int waves, double* in, double* out, uint64_t* cyc)
{
    hipLaunchKernelGGL(k_bench<KIND>, dim3(1), dim3(64 * waves), 0, 0, in, out, cyc);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL(k_bench<KIND>, dim3(1), dim3(64 * waves), 0, 0, in, out, cyc);
    uint64_t h[16];
    (void)hipMemcpy(h, cyc, sizeof(uint64_t) * waves, hipMemcpyDeviceToHost);
    uint64_t mx = 0;
    for (int w = 0; w < waves; ++w) mx = h[w] > mx ? h[w] : mx;
    // s_memtime counts at the shader clock; 8 chains x kIters instructions per wave
    printf("%-28s waves/SIMD %d: %.2f clocks per wave-instruction per SIMD\n", kName[KIND], waves / 4,
           (double)mx / (8.0 * kIters) / (waves / 4));
}

template <int K> static void all(int waves, double* in, double* out, uint64_t* cyc)
{
    run<K>(waves, in, out, cyc);
    if constexpr (K < 11) all<K + 1>(waves, in, out, cyc);
}

int main()
{
    double h[66];
    for (int i = 0; i < 66; ++i) h[i] = 1.0 + i * 1e-3;
    double *in, *out;
    uint64_t* cyc;
    (void)hipMalloc(&in, sizeof(h));
    (void)hipMalloc(&out, 1024 * sizeof(double));
    (void)hipMalloc(&cyc, 16 * sizeof(uint64_t));
    (void)hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
    for (int waves : {4, 16}) all<0>(waves, in, out, cyc);
    return 0;
}
