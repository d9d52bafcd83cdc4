/*
 * eslam_detmath.h -- the deterministic arithmetic contract of the eslam MI355X core.
 *
 * Every transcendental, random-number and fixed-point operation that the particle-filter
 * hot path performs is defined here, once, as a header that compiles both for the host
 * (gcc / clang, x86-64 SSE2 + FMA3) and for the device (hipcc, gfx950).  Built with
 * -ffp-contract=off on both sides, every function returns bit-identical results on the
 * CPU and on the GPU, which is what lets the device path match the CPU oracle bit-for-bit
 * (resample indices) and to the last ulp (weights).
 *
 * The reference delegates these operations to third-party code that is not vendored and
 * whose version is not pinned: glibc exp/log/sin/cos/pow, boost.math
 * normal pdf/cdf (src/ContactModel.cpp:104-115), boost.random minstd_rand + uniform_real
 * (src/ParticleFilter.hpp:87-88,177; src/PoseEstimator.cpp:15-16) and an external odometry
 * sampler (src/PoseEstimator.cpp:198).  Their results are reproduced here to ~1e-15
 * relative (transcendentals) or exactly (minstd integers, boost's integral-engine
 * uniform_real mapping), and tests/test_detmath.py checks them against mpmath / numpy.
 *
 * Only IEEE-exact primitives are used underneath: + - * / sqrt fma floor and integer ops.
 */
#ifndef ESLAM_DETMATH_H
#define ESLAM_DETMATH_H

#include <stdint.h>

#if defined(__HIPCC__)
#define DM_FN __host__ __device__ static inline __attribute__((always_inline))
#define DM_CONST static constexpr
#define DM_UNROLL _Pragma("unroll")
#else
#define DM_FN static inline
#define DM_CONST static const
#define DM_UNROLL
#endif

/* ------------------------------------------------------------------------------------ */
/* bit helpers                                                                           */
/* ------------------------------------------------------------------------------------ */
DM_FN uint64_t dm_bits(double x) { uint64_t u; __builtin_memcpy(&u, &x, 8); return u; }
DM_FN double dm_from_bits(uint64_t u) { double x; __builtin_memcpy(&x, &u, 8); return x; }
DM_FN uint32_t dm_fbits(float x) { uint32_t u; __builtin_memcpy(&u, &x, 4); return u; }
DM_FN int dm_isnan(double x) { return x != x; }
DM_FN int dm_isfinite(double x) { return (dm_bits(x) & 0x7ff0000000000000ull) != 0x7ff0000000000000ull; }
DM_FN double dm_fabs(double x) { return dm_from_bits(dm_bits(x) & 0x7fffffffffffffffull); }
DM_FN double dm_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }
/* fma(a, b, k) with k a compile-time (wave-uniform) constant.  On gfx950 the compiler
 * emits Horner steps as v_fmac_f64 with the constant moved into the destination VGPRs
 * (two v_mov_b32 per step); the VOP3 form reads it from an SGPR pair materialised by
 * the scalar unit instead.  Same IEEE fma, so host and device stay bit-identical.      */
#if defined(__HIP_DEVICE_COMPILE__)
DM_FN double dm_fmak(double a, double b, double k)
{
    double r;
    __asm__("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(k));
    return r;
}
#else
DM_FN double dm_fmak(double a, double b, double k) { return __builtin_fma(a, b, k); }
#endif
/* fma(a, b, c) with c one of the hardware's inline constants (no register at all) */
#if defined(__HIP_DEVICE_COMPILE__)
#define DM_FMA_INLINE(name, val)                                                            \
    DM_FN double name(double a, double b)                                                   \
    {                                                                                       \
        double r;                                                                           \
        __asm__("v_fma_f64 %0, %1, %2, " #val : "=v"(r) : "v"(a), "v"(b));                 \
        return r;                                                                           \
    }
#else
#define DM_FMA_INLINE(name, val) DM_FN double name(double a, double b) { return __builtin_fma(a, b, (val)); }
#endif
DM_FMA_INLINE(dm_fma_1, 1.0)
DM_FMA_INLINE(dm_fma_h, 0.5)
DM_FMA_INLINE(dm_fma_mh, -0.5)

/* Horner tables (highest degree first): p = c[0]; p = fma(p, u, c[i]).  Unrolled, every
 * coefficient is a compile-time constant (dm_fmak: an SGPR pair on the device).  Keeping
 * the tables in constant memory and scalar-loading them per evaluation was measured
 * slower (the loads raise SGPR pressure into spills).                                  */
#define DM_POLY_TABLE(name, n, ...) DM_CONST double name[n] = {__VA_ARGS__};
#define DM_POLY(name, n, u) dm_horner_k(name, n, (u))
DM_FN double dm_horner_k(const double* c, int n, double u)
{
    double p = c[0];
    DM_UNROLL
    for (int i = 1; i < n; ++i) p = dm_fmak(p, u, c[i]);
    return p;
}
DM_FN double dm_sqrt(double x) { return __builtin_sqrt(x); }
DM_FN double dm_floor(double x) { return __builtin_floor(x); }

/* a / b correctly rounded, for operands that need none of the device division's scaling
 * (|b| and |a / b| well inside the normal range, a == 0 allowed) and no special-value
 * fix-up (finite a, b != 0).  On the device it is the compiler's own fp64 division sequence
 * (v_rcp_f64, two Newton steps, the quotient and its one correction) without v_div_scale /
 * v_div_fixup, which return their inputs unchanged for such operands, so the bits are those
 * of the division; the host divides.  Callers state why their operands qualify.          */
DM_FN double dm_div_inrange(double a, double b)
{
#if defined(__HIP_DEVICE_COMPILE__)
    const double y0 = __builtin_amdgcn_rcp(b);
    double e = __builtin_fma(-b, y0, 1.0);
    const double y1 = __builtin_fma(y0, e, y0);
    e = __builtin_fma(-b, y1, 1.0);
    const double y2 = __builtin_fma(y1, e, y1);
    const double q0 = a * y2;
    const double r = __builtin_fma(-b, q0, a);
    return __builtin_fma(r, y2, q0);
#else
    return a / b;
#endif
}

/* sqrt(x) for a positive normal finite x, correctly rounded like dm_sqrt.  On the device
 * it is the compiler's own fp64 sqrt sequence (v_rsq_f64, Goldschmidt iteration, two
 * corrections) without the subnormal scaling and the zero/inf fix-up that such an x never
 * needs.  Used for the Box-Muller radius, whose argument -2 log(u), u = (a + 1/2) 2^-32,
 * lies in [2.3e-10, 44.4]; tests/test_gpu_parity.py compares it with dm_sqrt on the device
 * for all 2^32 values of a.                                                             */
DM_FN double dm_sqrt_pos(double x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = y * 0.5;
    const double r = dm_fma(-h, g, 0.5);
    g = dm_fma(g, r, g);
    h = dm_fma(h, r, h);
    double d = dm_fma(-g, g, x);
    g = dm_fma(d, h, g);
    d = dm_fma(-g, g, x);
    return dm_fma(d, h, g);
#else
    return __builtin_sqrt(x);
#endif
}

/* dm_sqrt with the range test in front: x in [2^-767, DBL_MAX] takes dm_sqrt_pos (the same
 * sequence the compiler emits there without its scaling and class fix-up, so the same
 * bits), anything else -- zero, subnormal-range, inf, NaN, negative -- the full sqrt.  On
 * the device the test is a branch that a wave skips when no lane needs the full path.    */
DM_FN double dm_sqrt_fast(double x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    if (x >= 0x1p-767 && x <= 1.7976931348623157e308) return dm_sqrt_pos(x);
    return __builtin_sqrt(x);
#else
    return __builtin_sqrt(x);
#endif
}

/* 2^k for k in [-1022, 1023], exact */
DM_FN double dm_pow2i(int k) { return dm_from_bits((uint64_t)(k + 1023) << 52); }

/* x * 2^k rounded once (IEEE round-to-nearest), including gradual underflow and overflow. */
DM_FN double dm_ldexp(double x, int k)
{
    if (x == 0.0 || !dm_isfinite(x)) return x;
    uint64_t b = dm_bits(x);
    int e = (int)((b >> 52) & 0x7ff);
    if (e == 0) { x *= 18446744073709551616.0; /* 2^64, exact */ b = dm_bits(x); e = (int)((b >> 52) & 0x7ff); k -= 64; }
    int t = e - 1023 + k;                                   /* target exponent */
    double m = dm_from_bits((b & 0x800fffffffffffffull) | 0x3ff0000000000000ull); /* +-[1,2) */
    if (t > 1023) return (m * dm_pow2i(1023)) * 2.0;        /* -> +-inf */
    if (t >= -1022) return m * dm_pow2i(t);                 /* exact */
    if (t < -1086) return m * 0.0;                          /* rounds to (signed) zero */
    return (m * dm_pow2i(t + 64)) * dm_pow2i(-64);          /* exact, then one rounding */
}

/* round-to-nearest-even integer value of |x| < 2^51, as a double (magic-number trick) */
DM_FN double dm_rint_small(double x)
{
    const double magic = 6755399441055744.0; /* 0x1.8p52 */
    double t = x + magic;
    return t - magic;
}

/* ------------------------------------------------------------------------------------ */
/* exp                                                                                   */
/* ------------------------------------------------------------------------------------ */
#define DM_LN2_HI 6.93147180369123816490e-01  /* 0x3fe62e42fee00000: 32 significant bits */
#define DM_LN2_LO 1.90821492927058770002e-10  /* ln2 - DM_LN2_HI                        */
#define DM_INV_LN2 1.44269504088896338700e+00

/* e^r on |r| <= 0.3466: e^r = 1 + r (1 + r (1/2 + r P(r))), P a degree-9 near-minimax fit
 * (tools/gen_minimax.py: Chebyshev, mpmath 60 digits; error of P's contribution < 1e-18
 * relative), fma Horner                                                                 */
DM_POLY_TABLE(dm_c_exp, 10, 2.0911229928855294e-09, 2.510037611136142e-08, 2.7557282983637385e-07,
              2.7557268479724004e-06, 2.4801587317135435e-05, 0.00019841269863040922,
              0.0013888888888886554, 0.008333333333330065, 0.041666666666666664, 0.16666666666666669)
DM_FN double dm_exp_kernel(double r)
{
    double p = DM_POLY(dm_c_exp, 10, r);
    p = dm_fma_h(p, r);
    p = dm_fma_1(p, r);
    return dm_fma_1(p, r);
}

/* Branch-free on the device's hot path: the special cases are selected afterwards (same
 * values), so several calls interleave in one basic block; only a result outside the
 * normal range takes dm_ldexp.                                                          */
DM_FN double dm_exp(double x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    /* x in [-708, 709]: ki = rint(x / ln2) lies in [-1021, 1023] and p 2^ki is normal, so the
     * scaling below is exact and equals v_ldexp_f64; the special-value selects are not
     * needed.  A branch: a wave runs the general path only when one of its lanes needs it. */
    if (x >= -708.0 && x <= 709.0) {
        const double kd = dm_rint_small(x * DM_INV_LN2);
        const double hi = x - kd * DM_LN2_HI;
        const double r = hi - kd * DM_LN2_LO;
        return __builtin_amdgcn_ldexp(dm_exp_kernel(r), (int)kd);
    }
#endif
    const int nan_ = x != x, over = x > 709.782712893384, under = x < -745.1332191019412;
    const double xs = (nan_ | over | under) ? 0.0 : x;
    double kd = dm_rint_small(xs * DM_INV_LN2);
    double hi = xs - kd * DM_LN2_HI;   /* exact: kd has <= 11 bits, LN2_HI 32 bits */
    double r = hi - kd * DM_LN2_LO;
    double p = dm_exp_kernel(r);       /* in [0.7, 1.42] */
    const int ki = (int)kd;
    /* p * 2^ki is normal (exact) for -1021 <= ki <= 1022: what dm_ldexp returns there */
    double res = (ki >= -1021 && ki <= 1022) ? p * dm_pow2i(ki) : dm_ldexp(p, ki);
    res = under ? 0.0 : res;
    res = over ? dm_from_bits(0x7ff0000000000000ull) : res;
    return nan_ ? x : res;
}

/* ------------------------------------------------------------------------------------ */
/* log                                                                                   */
/* ------------------------------------------------------------------------------------ */
/* P(z) = 2 (atanh(sqrt z)/sqrt z - 1) / z on z <= 0.02944, degree-6 minimax (Remez,
 * tools/gen_minimax.py; contribution < 1.5e-18 relative to log(1+f))                    */
DM_POLY_TABLE(dm_c_log, 7, 0.14795474282318508, 0.15314098921479188, 0.1818356240187849,
              0.22222198610842994, 0.2857142874201498, 0.39999999999416375, 0.6666666666666734)
/* log(xs 2^kadj) for a positive normal finite xs: the arithmetic of dm_log without its
 * special-case and subnormal selects */
DM_FN double dm_log_core(double xs, int kadj)
{
    const uint64_t b = dm_bits(xs);
    int k = kadj + (int)(b >> 52) - 1023;
    double m = dm_from_bits((b & 0x000fffffffffffffull) | 0x3ff0000000000000ull); /* [1,2) */
    const int big = m > 1.4142135623730951;
    m = big ? m * 0.5 : m;
    k += big;
    double f = m - 1.0;                 /* exact (Sterbenz) */
    /* (m-1)/(m+1), |s| <= 0.1716: f in [-0.293, 0.414], 2 + f in [1.70, 2.42] */
    double s = dm_div_inrange(f, 2.0 + f);
    double z = s * s;
    /* R = z P(z) ~ 2 z/3 + 2 z^2/5 + ...  (the atanh series, minimax-fitted) */
    double R = DM_POLY(dm_c_log, 7, z);
    R = R * z;
    /* log(1+f) = 2 atanh(s) = 2s + s R, and 2s = f - s f  ->  f - s (f - R) */
    double l = f - s * (f - R);
    double kd = (double)k;
    return kd * DM_LN2_HI + (l + kd * DM_LN2_LO);
}

/* log(x) of a positive normal finite x: equal to dm_log(x) bit for bit */
DM_FN double dm_log_pos(double x) { return dm_log_core(x, 0); }

DM_FN double dm_log(double x)
{
    /* branch-free: NaN, x <= 0 and +inf are selected at the end (same values) */
    const int special = !(x > 0.0) || !dm_isfinite(x);
    double xs = special ? 1.0 : x;
    const int sub = (dm_bits(xs) >> 52) == 0;
    xs = sub ? xs * 18014398509481984.0 /* 2^54 */ : xs;
    const double res = dm_log_core(xs, sub ? -54 : 0);
    if (!special) return res;
    if (x != x) return x;
    if (x <= 0.0) return x == 0.0 ? -dm_from_bits(0x7ff0000000000000ull) : dm_from_bits(0x7ff8000000000000ull);
    return x;                           /* +inf */
}

/* ------------------------------------------------------------------------------------ */
/* sin / cos                                                                             */
/* ------------------------------------------------------------------------------------ */
#define DM_PIO2_1 1.57079632673412561417e+00   /* first 33 bits of pi/2 */
#define DM_PIO2_2 6.07710050630396597660e-11   /* next 33 bits          */
#define DM_PIO2_3 2.02226624871116645580e-21   /* next 33 bits          */
#define DM_INV_PIO2 6.36619772367581382433e-01

/* sin(r) = r - r z P(z), P(z) = (1 - sin(sqrt z)/sqrt z) / z, z <= (pi/4)^2: degree-5
 * weighted minimax (Remez, tools/gen_minimax.py; |z (P - p)| < 5.4e-18)                 */
DM_POLY_TABLE(dm_c_sin, 6, -1.5896827930152048e-10, 2.505075865328765e-08, -2.7557313695226595e-06,
              0.0001984126982981695, -0.008333333333322425, 0.16666666666666632)
DM_FN double dm_sin_kernel(double r)   /* |r| <= pi/4, degree 13 */
{
    double z = r * r;
    double p = DM_POLY(dm_c_sin, 6, z);
    return dm_fma(-r * z, p, r) ;
}

/* cos(r) = 1 + z (-1/2 + z P(z)), P(z) = (cos(sqrt z) - 1 + z/2) / z^2: degree-5 weighted
 * minimax (Remez, tools/gen_minimax.py; |z^2 (P - p)| / cos r < 1.2e-18)                */
DM_POLY_TABLE(dm_c_cos, 6, -1.1358536517414803e-11, 2.0875700841892227e-09, -2.755731417929608e-07,
              2.48015872888517e-05, -0.0013888888888873056, 0.041666666666666595)
DM_FN double dm_cos_kernel(double r)   /* |r| <= pi/4, degree 14 */
{
    double z = r * r;
    double p = DM_POLY(dm_c_cos, 6, z);
    p = dm_fma_mh(p, z);
    return dm_fma_1(p, z);
}

/* quadrant q of (sin, cos) from the kernels on the reduced argument, by selects */
DM_FN void dm_quadrant(int q, double sr, double cr, double* s, double* c)
{
    const int swap = q & 1, neg_s = q & 2, neg_c = (q == 1) | (q == 2);
    const double ss = swap ? cr : sr, cc = swap ? sr : cr;
    *s = neg_s ? -ss : ss;
    *c = neg_c ? -cc : cc;
}

/* n mod 4 of the integer-valued n of dm_sincos, through a 32-bit conversion that saturates
 * (v_cvt_i32_f64 on the device, the same clamp on the host): exact for |n| < 2^31, i.e.
 * |x| < 3.3e9 rad; beyond, the quadrant of the clamped value (deterministic both sides)   */
DM_FN int dm_quadrant_of(double n)
{
#if defined(__HIP_DEVICE_COMPILE__)
    int q;
    __asm__("v_cvt_i32_f64 %0, %1" : "=v"(q) : "v"(n));
    return q & 3;
#else
    const int q = n >= 2147483647.0 ? 2147483647 : (n <= -2147483648.0 ? (-2147483647 - 1) : (int)n);
    return q & 3;
#endif
}

DM_FN void dm_sincos(double x, double* s, double* c)
{
#if defined(__HIP_DEVICE_COMPILE__)
    /* a wave whose angles are all finite takes the arithmetic without the special-value
     * selects (the same values) */
    if (__builtin_amdgcn_ballot_w64(!dm_isfinite(x)) == 0) {
        const double n = dm_rint_small(x * DM_INV_PIO2);
        const double r = ((x - n * DM_PIO2_1) - n * DM_PIO2_2) - n * DM_PIO2_3;
        dm_quadrant(dm_quadrant_of(n), dm_sin_kernel(r), dm_cos_kernel(r), s, c);
        return;
    }
#endif
    const int fin = dm_isfinite(x);
    const double xs = fin ? x : 0.0;
    /* |n| > 2^20 (|x| > 1.6e6 rad): the three-part reduction is inexact but deterministic */
    double n = dm_rint_small(xs * DM_INV_PIO2);
    double r = ((xs - n * DM_PIO2_1) - n * DM_PIO2_2) - n * DM_PIO2_3;
    double sr = dm_sin_kernel(r), cr = dm_cos_kernel(r);
    dm_quadrant(dm_quadrant_of(n), sr, cr, s, c);
    if (!fin) { *s = x - x; *c = x - x; }
}

/* 1.0 / k for k = 0..32 (correctly rounded, as the division; k = 0 -> inf) */
DM_CONST double dm_recip_tab[33] = {
    __builtin_inf(), 1.0, 0.5, 0.3333333333333333, 0.25, 0.2, 0.16666666666666666, 0.14285714285714285,
    0.125, 0.1111111111111111, 0.1, 0.09090909090909091, 0.08333333333333333, 0.07692307692307693,
    0.07142857142857142, 0.06666666666666667, 0.0625, 0.058823529411764705, 0.05555555555555555,
    0.05263157894736842, 0.05, 0.047619047619047616, 0.045454545454545456, 0.043478260869565216,
    0.041666666666666664, 0.04, 0.038461538461538464, 0.037037037037037035, 0.03571428571428571,
    0.034482758620689655, 0.03333333333333333, 0.03225806451612903, 0.03125};
DM_FN double dm_recip_small(uint32_t k) { return k <= 32 ? dm_recip_tab[k] : 1.0 / (double)k; }

/* ------------------------------------------------------------------------------------ */
/* erfc                                                                                  */
/* ------------------------------------------------------------------------------------ */
/* Piecewise polynomial fits of erfcx(t) = exp(t^2) erfc(t), t >= 0, generated by
 * tools/gen_erfcx_coeffs.py (mpmath, 60 digits; fit error < 1e-19 relative).           */
DM_CONST double dm_erfcx_c0[19] = {9.283752145234023e-18, -1.1792469674650424e-16, 1.4147642917261418e-15, -1.6990873809451645e-14, 1.9815259170250877e-13, -2.237871975539458e-12, 2.443089253356378e-11, -2.5716880604565665e-10, 2.602534528787355e-09, -2.523338988527416e-08, 2.334361521750124e-07, -2.0502402237783523e-06, 1.699015396298168e-05, -0.00013180360649459388, 0.0009473309967177142, -0.006219475256501468, 0.03653406715146833, -0.18580147330750355, 0.7703465477309968};
DM_CONST double dm_erfcx_c1[21] = {7.586363910623654e-16, -5.70498818820545e-15, 3.804139839023933e-14, -2.7298916881805636e-13, 1.923220700761848e-12, -1.316808218435804e-11, 8.78702258916541e-11, -5.707384863259472e-10, 3.6018496597373607e-09, -2.2042929675824138e-08, 1.3053024836981828e-07, -7.460049373598812e-07, 4.102614842889114e-06, -2.1633318561315704e-05, 0.00010890847460873127, -0.0005206834090754457, 0.002348268513455678, -0.009903371117665843, 0.03859289034297711, -0.13660600739194928, 0.427583576155807};
DM_CONST double dm_erfcx_c2[21] = {5.057065718502677e-15, -3.068476570068241e-14, 1.5665515071079456e-13, -9.145569832047356e-13, 5.304280116094916e-12, -2.988095123391799e-11, 1.6501687267503609e-10, -8.932988395737626e-10, 4.733487001243104e-09, -2.452313531325191e-08, 1.2405991227876422e-07, -6.119614590410515e-07, 2.938639159152759e-06, -1.3711609161098606e-05, 6.20318170584252e-05, -0.0002714121303982754, 0.001145072748839861, -0.004641494381623146, 0.017995852918522272, -0.06636487710656187, 0.23108725873039188};
DM_CONST double dm_erfcx_c3[21] = {1.3630546848219266e-15, -7.922495175389322e-15, 3.837381296081427e-14, -2.1703391711090554e-13, 1.228659481248371e-12, -6.783010963567072e-12, 3.694282205184398e-11, -1.9861768949727073e-10, 1.0530843369976437e-09, -5.5033698295504104e-09, 2.8331978822991838e-08, -1.4359644214436117e-07, 7.16045664615945e-07, -3.5103666499135004e-06, 1.6905649257776914e-05, -7.990888030554815e-05, 0.0003703524689955565, -0.001681182076746115, 0.007465433244975571, -0.032383506095021455, 0.13699945762506138};
DM_CONST double dm_erfcx_tail[15] = {7.839577105055556e-16, -4.33825604370309e-15, 2.2414082272808668e-14, -1.4112442747221709e-13, 9.543596829961645e-13, -6.9177088797188345e-12, 5.462084473729142e-11, -4.76004525046868e-10, 4.6562063848232095e-09, -5.230561185110592e-08, 6.970116167625029e-07, -1.1575329006190274e-05, 0.0002604872169531935, -0.009441218224620304, 0.9902859647173192};

DM_FN double dm_horner(const double* c, int n, double u)
{
    double p = c[0];
    DM_UNROLL
    for (int i = 1; i < n; ++i) p = dm_fmak(p, u, c[i]);
    return p;
}

/* erfcx(t) for t >= 0 (t finite) */
DM_FN double dm_erfcx_pos(double t)
{
    if (t < 0.5) return dm_horner(dm_erfcx_c0, 19, (t - 0.25) * 4.0);
    if (t < 1.5) return dm_horner(dm_erfcx_c1, 21, (t - 1.0) * 2.0);
    if (t < 3.0) return dm_horner(dm_erfcx_c2, 21, (t - 2.25) / 0.75);
    if (t < 5.0) return dm_horner(dm_erfcx_c3, 21, (t - 4.0));
    double w = 1.0 / (t * t);
    double q = dm_horner(dm_erfcx_tail, 15, w * 50.0 - 1.0);   /* u = 2 w / 0.04 - 1 */
    return q / (t * 1.7724538509055159);                        /* sqrt(pi) */
}

/* exp(-x^2) with the square split exactly (hi + lo) so |x| up to 27 keeps ~1 ulp */
DM_FN double dm_exp_negsq(double x)
{
    double hi = x * x;
    double lo = dm_fma(x, x, -hi);
    double e = dm_exp(-hi);
    return e - e * lo;
}

DM_FN double dm_erfc(double x)
{
    if (x != x) return x;
    double a = dm_fabs(x);
    if (a > 27.3) return x > 0 ? 0.0 : 2.0;
    double v = dm_exp_negsq(a) * dm_erfcx_pos(a);
    return x >= 0 ? v : 2.0 - v;
}

/* ------------------------------------------------------------------------------------ */
/* powers                                                                                */
/* ------------------------------------------------------------------------------------ */
/* x^k, k a non-negative integer <= 64, correctly rounded via double-double accumulation
 * (matches glibc's correctly-rounded pow(x, (double)k) barring exact ties).             */
DM_FN double dm_pow_ui(double x, uint32_t k)
{
    if (k == 0) return 1.0;
    if (k == 1 || x != x || x == 0.0 || !dm_isfinite(x)) {
        double r = x;
        for (uint32_t i = 1; i < k; ++i) r = r * x;
        return r;
    }
    double hi = x, lo = 0.0;
    for (uint32_t i = 1; i < k; ++i) {
        double p = hi * x;
        double pe = dm_fma(hi, x, -p);
        double l2 = dm_fma(lo, x, pe);
        hi = p + l2;
        lo = l2 - (hi - p);
        if (!dm_isfinite(hi)) return hi;
    }
    return hi + lo;
}

/* std::pow(double x, (double)y) restricted to what the path needs:
 *   y an exact non-negative integer <= 64 -> dm_pow_ui;
 *   y >= 2^53 (the size_t wrap of `4 - cpoints.size()`, src/PoseEstimator.cpp:336) -> limits;
 *   otherwise exp(y * log(x)) for x > 0.                                                  */
DM_FN double dm_pow(double x, double y)
{
    if (y == 0.0) return 1.0;
    if (y >= 0.0 && y <= 64.0 && dm_floor(y) == y) return dm_pow_ui(x, (uint32_t)y);
    if (x != x || y != y) return x + y;
    if (y == 0.5 && x >= 0.0) return dm_sqrt(x);      /* correctly rounded, like glibc */
    if (y >= 9007199254740992.0) {           /* huge even integer exponent */
        double a = dm_fabs(x);
        if (a == 1.0) return 1.0;
        return a < 1.0 ? 0.0 : dm_from_bits(0x7ff0000000000000ull);
    }
    if (x == 0.0) return y > 0 ? 0.0 : dm_from_bits(0x7ff0000000000000ull);
    if (x < 0.0) return dm_from_bits(0x7ff8000000000000ull);
    if (x == 1.0) return 1.0;
    return dm_exp(y * dm_log(x));
}

/* ------------------------------------------------------------------------------------ */
/* boost::math::normal pdf / cdf ratio (src/ContactModel.cpp:104-115)                    */
/* ------------------------------------------------------------------------------------ */
/* ratio = pdf(N(0,s), z) / cdf(N(0,s), z), s = sigma * correction.  With y = z / (s sqrt2),
 * t = -y, a = |t| and E = exp(-t^2) (= the pdf exponent -z^2 / (2 s^2)):
 *   pdf = E / (s sqrt(2 pi)),   cdf = erfc(t) / 2,   erfc(t) = E erfcx(a)      (t >= 0)
 *                                                      = 2 - E erfcx(a)  (t <  0)
 * so ratio = sqrt(2/pi) / (s erfcx(a)) for t >= 0 (E cancels: no exp, and no 0/0 where
 * boost underflows beyond z/s < -38), sqrt(2/pi) E / (s (2 - E erfcx(a))) otherwise.
 * Equal to boost's pdf/cdf to ~1e-15 relative; two divisions instead of three.           */
DM_FN double dm_normal_pdf_cdf_ratio(double z, double s)
{
    const double y = z / (s * 1.4142135623730951);
    const double t = -y;
    const double a = dm_fabs(t);
    const double cx = dm_erfcx_pos(a);
    if (t >= 0.0) return 0.7978845608028654 / (s * cx);
    const double E = dm_exp_negsq(a);
    return (0.7978845608028654 * E) / (s * (2.0 - E * cx));
}

/* ------------------------------------------------------------------------------------ */
/* Philox4x32-10 counter-based generator (Salmon et al., SC'11 / Random123)              */
/* ------------------------------------------------------------------------------------ */
typedef struct { uint32_t v[4]; } dm_philox_ctr;

/* a ^ b ^ c: one v_bitop3_b32 on gfx950 (truth table 0x96) instead of two v_xor_b32 */
DM_FN uint32_t dm_xor3(uint32_t a, uint32_t b, uint32_t c)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
    return a ^ b ^ c;
#endif
}

DM_FN dm_philox_ctr dm_philox4x32_10(dm_philox_ctr c, uint32_t k0, uint32_t k1)
{
    DM_UNROLL
    for (int r = 0; r < 10; ++r) {
        if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        uint64_t p0 = (uint64_t)0xD2511F53u * c.v[0];
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c.v[2];
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        dm_philox_ctr o;
        o.v[0] = dm_xor3(hi1, c.v[1], k0);
        o.v[1] = lo1;
        o.v[2] = dm_xor3(hi0, c.v[3], k1);
        o.v[3] = lo0;
        c = o;
    }
    return c;
}

/* 53-bit uniform in [0, 1) from two 32-bit words */
DM_FN double dm_u53(uint32_t a, uint32_t b)
{
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * 1.1102230246251565e-16;
}

/* Box-Muller: u1 in [0,1) mapped to (0,1] */
DM_FN void dm_box_muller(double u1, double u2, double* z0, double* z1)
{
    double r = dm_sqrt(-2.0 * dm_log(1.0 - u1));
    double s, c;
    dm_sincos(6.283185307179586 * u2, &s, &c);
    *z0 = r * c;
    *z1 = r * s;
}

/* uniform in (0, 1) from one 32-bit word: (a + 1/2) 2^-32, exact.  32-bit resolution, like
 * the reference's 31-bit minstd_rand behind boost's uniform_real / normal_distribution. */
DM_FN double dm_u32(uint32_t a) { return ((double)a + 0.5) * 2.3283064365386963e-10; }

/* sin and cos of 2 pi u for u in (0, 1): the quarter-turn reduction t = 4u - q is exact,
 * one rounding in r = t pi/2 (|r| <= pi/4), then the kernels of dm_sincos.             */
DM_FN void dm_sincos2pi(double u, double* s, double* c)
{
    const double t = u * 4.0;
    const double q = dm_floor(t + 0.5);
    const double r = (t - q) * 1.5707963267948966;
    const double sr = dm_sin_kernel(r), cr = dm_cos_kernel(r);
    dm_quadrant((int)q & 3, sr, cr, s, c);
}

/* Box-Muller tables (tools/gen_bm_tables.py: the method, the interval choice and the
 * error bounds are in its docstring) */
/* generated by tools/gen_bm_tables.py: {1/c_i, -log(1/c_i) hi, lo, 0} */
DM_CONST double dm_bm_log_tab[128][4] = {
    {1.3298701298701299, -0.28508129075172356, -6.351399668130711e-19, 0.0},
    {1.322997416020672, -0.279899932009726, -4.834062762833095e-18, 0.0},
    {1.3161953727506426, -0.2747452814210614, -3.665410036157285e-18, 0.0},
    {1.3094629156010231, -0.26961706505414207, -2.686159658510421e-17, 0.0},
    {1.3027989821882953, -0.2645150131702466, -8.166602421887088e-18, 0.0},
    {1.2962025316455696, -0.2594388601383859, -2.7423845801639452e-17, 0.0},
    {1.2896725440806045, -0.25438834435231733, -1.4339973939868338e-17, 0.0},
    {1.2832080200501252, -0.24936320814964427, -6.740267061480097e-19, 0.0},
    {1.2768079800498753, -0.24436319773293858, 1.4064713105722283e-18, 0.0},
    {1.2704714640198511, -0.23938806309282482, 1.3531467828463102e-17, 0.0},
    {1.2641975308641975, -0.23443755793296864, 1.3462500573049868e-17, 0.0},
    {1.257985257985258, -0.22951143959691278, 9.130963928926302e-18, 0.0},
    {1.2518337408312958, -0.22460946899670603, -4.873968263851468e-18, 0.0},
    {1.245742092457421, -0.2197314105432732, -1.2172989873689749e-17, 0.0},
    {1.2397094430992737, -0.21487703207847508, 6.3936369496245475e-18, 0.0},
    {1.2337349397590363, -0.21004610480880959, 1.1401416710694254e-17, 0.0},
    {1.2278177458033572, -0.20523840324070627, 6.517045487028861e-18, 0.0},
    {1.2219570405727924, -0.2004537051173701, -4.024887784647953e-18, 0.0},
    {1.2161520190023754, -0.19569179135712642, 4.194035836168105e-18, 0.0},
    {1.210401891252955, -0.1909524459932298, 1.153257055843512e-17, 0.0},
    {1.204705882352941, -0.18623545611509087, 7.239565374145492e-18, 0.0},
    {1.199063231850117, -0.18154061181088324, 1.0031622970826496e-17, 0.0},
    {1.1934731934731935, -0.1768677061114908, -1.0142708275797129e-17, 0.0},
    {1.1879350348027842, -0.17221653493575995, -9.173041762380018e-18, 0.0},
    {1.1824480369515011, -0.16758689703701793, 6.957799504672856e-18, 0.0},
    {1.1770114942528735, -0.16297859395082367, -2.968291512446388e-18, 0.0},
    {1.17162471395881, -0.15839142994391764, 2.637463471501479e-18, 0.0},
    {1.1662870159453302, -0.15382521196433638, -9.48961192244976e-18, 0.0},
    {1.1609977324263039, -0.14927974959266183, 7.432789359543407e-18, 0.0},
    {1.1557562076749435, -0.14475485499437207, 1.0071735412643571e-17, 0.0},
    {1.150561797752809, -0.14025034287326765, -7.174632062898151e-18, 0.0},
    {1.145413870246085, -0.13576603042593893, 2.0963004096866695e-18, 0.0},
    {1.1403118040089086, -0.13130173729725345, -1.920011794471695e-18, 0.0},
    {1.1352549889135255, -0.12685728553682943, -7.640536611850881e-18, 0.0},
    {1.130242825607064, -0.12243249955647377, 6.334183374683508e-18, 0.0},
    {1.1252747252747253, -0.11802720608855737, -2.7349066045479833e-18, 0.0},
    {1.1203501094091903, -0.11364123414530306, 5.870375286097418e-18, 0.0},
    {1.1154684095860568, -0.10927441497896273, 3.5628843393108066e-18, 0.0},
    {1.1106290672451193, -0.10492658204285929, -6.3947256124788025e-18, 0.0},
    {1.1058315334773219, -0.10059757095327378, 4.804056155300937e-18, 0.0},
    {1.1010752688172043, -0.09628721945215148, 4.299622091213251e-18, 0.0},
    {1.0963597430406853, -0.09199536737061052, -6.2313226384620115e-18, 0.0},
    {1.091684434968017, -0.0877218565932284, -3.1061998497496937e-18, 0.0},
    {1.0870488322717622, -0.08346653102309001, -5.556862433791088e-18, 0.0},
    {1.0824524312896406, -0.07922923654757486, -4.277690436376405e-18, 0.0},
    {1.0778947368421052, -0.07500982100486656, 2.9115176492034424e-18, 0.0},
    {1.0733752620545074, -0.07080813415116662, -5.9080686874000904e-18, 0.0},
    {1.068893528183716, -0.06662402762859244, -5.5751094781716345e-18, 0.0},
    {1.0644490644490645, -0.06245735493374666, 3.1280694702435752e-18, 0.0},
    {1.060041407867495, -0.05830797138693517, 2.070662157308864e-18, 0.0},
    {1.0556701030927835, -0.054175734102024614, 3.1245030174465517e-18, 0.0},
    {1.051334702258727, -0.05006050195691803, -9.174024604303651e-20, 0.0},
    {1.047034764826176, -0.04596213556463585, -2.5706225148512324e-19, 0.0},
    {1.0427698574338085, -0.04188049724498711, -2.283650074850234e-18, 0.0},
    {1.0385395537525355, -0.037815450996817664, 1.4251832364060072e-19, 0.0},
    {1.0343434343434343, -0.033766862470817484, 1.442127698674705e-18, 0.0},
    {1.0301810865191148, -0.029734598942879144, 1.3359261790310464e-18, 0.0},
    {1.0260521042084167, -0.025718529287989036, -8.505083404803465e-19, 0.0},
    {1.0219560878243512, -0.021718523954642903, 9.51817561415885e-19, 0.0},
    {1.0178926441351888, -0.017734454939768475, -5.192616246238567e-19, 0.0},
    {1.0138613861386139, -0.01376619576414797, -6.51170039303772e-19, 0.0},
    {1.009861932938856, -0.00981362144832467, -5.330914506885923e-19, 0.0},
    {1.005893909626719, -0.005876608488984971, 3.8610986774758214e-19, 0.0},
    {1.0, 0.0, 0.0, 0.0},
    {0.9961089494163424, 0.003898640415657309, 1.2541659038304982e-19, 0.0},
    {0.9884169884169884, 0.01165061721997525, 6.311738528333134e-19, 0.0},
    {0.9808429118773946, 0.019342962843130987, -6.612867620320467e-19, 0.0},
    {0.973384030418251, 0.026976587698202083, -1.357561021795712e-18, 0.0},
    {0.9660377358490566, 0.03455238150665973, -2.5264681161162764e-18, 0.0},
    {0.9588014981273408, 0.042071213920687044, -9.713775354759503e-20, 0.0},
    {0.9516728624535316, 0.049533935122276676, 1.664443731663614e-18, 0.0},
    {0.9446494464944649, 0.05694137640013845, 1.78594464879227e-18, 0.0},
    {0.9377289377289377, 0.06429435070539725, 3.475225966814173e-18, 0.0},
    {0.9309090909090909, 0.07159365318700882, 4.869195800165027e-19, 0.0},
    {0.924187725631769, 0.078840061707776, -4.568340554252506e-18, 0.0},
    {0.9175627240143369, 0.08603433734180316, -3.36803314523905e-18, 0.0},
    {0.9110320284697508, 0.09317722485418334, 2.8334317358750366e-18, 0.0},
    {0.9045936395759717, 0.10026945316367517, -2.822998867357873e-18, 0.0},
    {0.8982456140350877, 0.10731173578908804, -4.322456718254657e-18, 0.0},
    {0.89198606271777, 0.11430477128005863, 5.977397630760421e-18, 0.0},
    {0.8858131487889274, 0.12124924363286965, 2.6827199737801766e-18, 0.0},
    {0.8797250859106529, 0.12814582269193006, -4.109471350011548e-18, 0.0},
    {0.8737201365187713, 0.13499516453750482, 1.369660501724148e-18, 0.0},
    {0.8677966101694915, 0.1417979118602574, -1.2867304346273362e-17, 0.0},
    {0.8619528619528619, 0.1485546943231372, -1.1863378834702217e-17, 0.0},
    {0.8561872909698997, 0.15526612891112396, 1.1990886572394084e-17, 0.0},
    {0.8504983388704319, 0.16193282026931324, -1.3644842250457798e-17, 0.0},
    {0.8448844884488449, 0.16855536102980664, 1.0763132959988806e-17, 0.0},
    {0.839344262295082, 0.17513433212784915, -2.724105290158387e-18, 0.0},
    {0.8338762214983714, 0.18167030310763463, 4.954929708083542e-18, 0.0},
    {0.8284789644012945, 0.18816383241818294, 3.741953239550891e-18, 0.0},
    {0.8231511254019293, 0.19461546769967167, 1.9890959474466474e-18, 0.0},
    {0.8178913738019169, 0.2010257460605908, -4.5707808879306246e-18, 0.0},
    {0.8126984126984127, 0.2073951943460706, -5.756619770435678e-18, 0.0},
    {0.807570977917981, 0.21372432939771818, -1.2735141289933245e-17, 0.0},
    {0.8025078369905956, 0.22001365830528213, 1.1961281714072477e-18, 0.0},
    {0.7975077881619937, 0.2262636786504534, 8.337560297889984e-18, 0.0},
    {0.7925696594427245, 0.232474878743094, 6.160927890733764e-18, 0.0},
    {0.7876923076923077, 0.238647737850175, -1.6128470577184094e-18, 0.0},
    {0.7828746177370031, 0.24478272641769092, -7.47089098380464e-18, 0.0},
    {0.7781155015197568, 0.25088030628580943, -8.553911523038828e-18, 0.0},
    {0.7734138972809668, 0.2569409308975004, 7.175242481751694e-18, 0.0},
    {0.7687687687687688, 0.26296504550088134, 1.5718867588147142e-17, 0.0},
    {0.764179104477612, 0.26895308734550394, 1.0592604897911732e-17, 0.0},
    {0.7596439169139466, 0.2749054858727992, -1.402747850115579e-17, 0.0},
    {0.7551622418879056, 0.2808226629008878, -1.0950013154836128e-17, 0.0},
    {0.750733137829912, 0.2867050328039543, -2.8116608187823606e-18, 0.0},
    {0.7463556851311953, 0.29255300268637746, -5.2811179490291116e-18, 0.0},
    {0.7420289855072464, 0.2983669725517973, -1.3287151317641232e-17, 0.0},
    {0.7377521613832853, 0.3041473354672968, 7.010822479304778e-18, 0.0},
    {0.7335243553008596, 0.3098944777228647, 4.5997359765827076e-18, 0.0},
    {0.7293447293447294, 0.3156087789863033, -1.0493698520483516e-17, 0.0},
    {0.7252124645892352, 0.32129061245373425, -3.035364123413162e-18, 0.0},
    {0.7211267605633803, 0.3269403449958533, -1.5322929902901654e-17, 0.0},
    {0.7170868347338936, 0.3325583373000766, -1.8692002087134156e-17, 0.0},
    {0.713091922005571, 0.3381449440087164, -2.4651351958263637e-17, 0.0},
    {0.7091412742382271, 0.34370051385331846, -1.421331198699375e-17, 0.0},
    {0.7052341597796143, 0.3492253897852883, 4.02376954597919e-19, 0.0},
    {0.7013698630136986, 0.354719909102929, 2.198105025613807e-17, 0.0},
    {0.6975476839237057, 0.3601844035750078, 2.6812351028097144e-17, 0.0},
    {0.6937669376693767, 0.3656191995609647, -1.2762016415473489e-17, 0.0},
    {0.6900269541778976, 0.37102461812787263, -1.948933773396101e-17, 0.0},
    {0.6863270777479893, 0.376400975164253, 2.032121209009643e-17, 0.0},
    {0.6826666666666666, 0.3817485814908484, -1.9951991043846497e-17, 0.0},
    {0.6790450928381963, 0.3870677429684483, 2.5550894542318646e-17, 0.0},
    {0.6754617414248021, 0.3923587606028639, 9.493401229363408e-18, 0.0},
    {0.6719160104986877, 0.3976219306471385, -1.8770120125166398e-17, 0.0},
    {0.6684073107049608, 0.4028575447010835, 2.0735595335748982e-17, 0.0},
};
/* generated by tools/gen_bm_tables.py: {sin, cos} of 2 pi j / 256 */
DM_CONST double dm_bm_sc_tab[256][2] = {
    {0.0, 1.0},
    {0.024541228522912288, 0.9996988186962042},
    {0.049067674327418015, 0.9987954562051724},
    {0.07356456359966743, 0.9972904566786902},
    {0.0980171403295606, 0.9951847266721969},
    {0.1224106751992162, 0.99247953459871},
    {0.14673047445536175, 0.989176509964781},
    {0.17096188876030122, 0.9852776423889412},
    {0.19509032201612828, 0.9807852804032304},
    {0.2191012401568698, 0.9757021300385286},
    {0.2429801799032639, 0.970031253194544},
    {0.26671275747489837, 0.9637760657954398},
    {0.2902846772544624, 0.9569403357322088},
    {0.31368174039889146, 0.9495281805930367},
    {0.33688985339222005, 0.9415440651830208},
    {0.35989503653498817, 0.9329927988347388},
    {0.3826834323650898, 0.9238795325112867},
    {0.40524131400498986, 0.9142097557035307},
    {0.4275550934302821, 0.9039892931234433},
    {0.4496113296546066, 0.8932243011955153},
    {0.47139673682599764, 0.881921264348355},
    {0.49289819222978404, 0.8700869911087115},
    {0.5141027441932218, 0.8577286100002721},
    {0.5349976198870973, 0.8448535652497071},
    {0.5555702330196022, 0.8314696123025452},
    {0.5758081914178453, 0.8175848131515837},
    {0.5956993044924334, 0.8032075314806449},
    {0.6152315905806268, 0.7883464276266062},
    {0.6343932841636455, 0.773010453362737},
    {0.6531728429537768, 0.7572088465064846},
    {0.6715589548470184, 0.7409511253549591},
    {0.6895405447370669, 0.7242470829514669},
    {0.7071067811865476, 0.7071067811865476},
    {0.7242470829514669, 0.6895405447370669},
    {0.7409511253549591, 0.6715589548470184},
    {0.7572088465064846, 0.6531728429537768},
    {0.773010453362737, 0.6343932841636455},
    {0.7883464276266062, 0.6152315905806268},
    {0.8032075314806449, 0.5956993044924334},
    {0.8175848131515837, 0.5758081914178453},
    {0.8314696123025452, 0.5555702330196022},
    {0.8448535652497071, 0.5349976198870973},
    {0.8577286100002721, 0.5141027441932218},
    {0.8700869911087115, 0.49289819222978404},
    {0.881921264348355, 0.47139673682599764},
    {0.8932243011955153, 0.4496113296546066},
    {0.9039892931234433, 0.4275550934302821},
    {0.9142097557035307, 0.40524131400498986},
    {0.9238795325112867, 0.3826834323650898},
    {0.9329927988347388, 0.35989503653498817},
    {0.9415440651830208, 0.33688985339222005},
    {0.9495281805930367, 0.31368174039889146},
    {0.9569403357322088, 0.2902846772544624},
    {0.9637760657954398, 0.26671275747489837},
    {0.970031253194544, 0.2429801799032639},
    {0.9757021300385286, 0.2191012401568698},
    {0.9807852804032304, 0.19509032201612828},
    {0.9852776423889412, 0.17096188876030122},
    {0.989176509964781, 0.14673047445536175},
    {0.99247953459871, 0.1224106751992162},
    {0.9951847266721969, 0.0980171403295606},
    {0.9972904566786902, 0.07356456359966743},
    {0.9987954562051724, 0.049067674327418015},
    {0.9996988186962042, 0.024541228522912288},
    {1.0, 5.709968497124349e-62},
    {0.9996988186962042, -0.024541228522912288},
    {0.9987954562051724, -0.049067674327418015},
    {0.9972904566786902, -0.07356456359966743},
    {0.9951847266721969, -0.0980171403295606},
    {0.99247953459871, -0.1224106751992162},
    {0.989176509964781, -0.14673047445536175},
    {0.9852776423889412, -0.17096188876030122},
    {0.9807852804032304, -0.19509032201612828},
    {0.9757021300385286, -0.2191012401568698},
    {0.970031253194544, -0.2429801799032639},
    {0.9637760657954398, -0.26671275747489837},
    {0.9569403357322088, -0.2902846772544624},
    {0.9495281805930367, -0.31368174039889146},
    {0.9415440651830208, -0.33688985339222005},
    {0.9329927988347388, -0.35989503653498817},
    {0.9238795325112867, -0.3826834323650898},
    {0.9142097557035307, -0.40524131400498986},
    {0.9039892931234433, -0.4275550934302821},
    {0.8932243011955153, -0.4496113296546066},
    {0.881921264348355, -0.47139673682599764},
    {0.8700869911087115, -0.49289819222978404},
    {0.8577286100002721, -0.5141027441932218},
    {0.8448535652497071, -0.5349976198870973},
    {0.8314696123025452, -0.5555702330196022},
    {0.8175848131515837, -0.5758081914178453},
    {0.8032075314806449, -0.5956993044924334},
    {0.7883464276266062, -0.6152315905806268},
    {0.773010453362737, -0.6343932841636455},
    {0.7572088465064846, -0.6531728429537768},
    {0.7409511253549591, -0.6715589548470184},
    {0.7242470829514669, -0.6895405447370669},
    {0.7071067811865476, -0.7071067811865476},
    {0.6895405447370669, -0.7242470829514669},
    {0.6715589548470184, -0.7409511253549591},
    {0.6531728429537768, -0.7572088465064846},
    {0.6343932841636455, -0.773010453362737},
    {0.6152315905806268, -0.7883464276266062},
    {0.5956993044924334, -0.8032075314806449},
    {0.5758081914178453, -0.8175848131515837},
    {0.5555702330196022, -0.8314696123025452},
    {0.5349976198870973, -0.8448535652497071},
    {0.5141027441932218, -0.8577286100002721},
    {0.49289819222978404, -0.8700869911087115},
    {0.47139673682599764, -0.881921264348355},
    {0.4496113296546066, -0.8932243011955153},
    {0.4275550934302821, -0.9039892931234433},
    {0.40524131400498986, -0.9142097557035307},
    {0.3826834323650898, -0.9238795325112867},
    {0.35989503653498817, -0.9329927988347388},
    {0.33688985339222005, -0.9415440651830208},
    {0.31368174039889146, -0.9495281805930367},
    {0.2902846772544624, -0.9569403357322088},
    {0.26671275747489837, -0.9637760657954398},
    {0.2429801799032639, -0.970031253194544},
    {0.2191012401568698, -0.9757021300385286},
    {0.19509032201612828, -0.9807852804032304},
    {0.17096188876030122, -0.9852776423889412},
    {0.14673047445536175, -0.989176509964781},
    {0.1224106751992162, -0.99247953459871},
    {0.0980171403295606, -0.9951847266721969},
    {0.07356456359966743, -0.9972904566786902},
    {0.049067674327418015, -0.9987954562051724},
    {0.024541228522912288, -0.9996988186962042},
    {1.1419936994248699e-61, -1.0},
    {-0.024541228522912288, -0.9996988186962042},
    {-0.049067674327418015, -0.9987954562051724},
    {-0.07356456359966743, -0.9972904566786902},
    {-0.0980171403295606, -0.9951847266721969},
    {-0.1224106751992162, -0.99247953459871},
    {-0.14673047445536175, -0.989176509964781},
    {-0.17096188876030122, -0.9852776423889412},
    {-0.19509032201612828, -0.9807852804032304},
    {-0.2191012401568698, -0.9757021300385286},
    {-0.2429801799032639, -0.970031253194544},
    {-0.26671275747489837, -0.9637760657954398},
    {-0.2902846772544624, -0.9569403357322088},
    {-0.31368174039889146, -0.9495281805930367},
    {-0.33688985339222005, -0.9415440651830208},
    {-0.35989503653498817, -0.9329927988347388},
    {-0.3826834323650898, -0.9238795325112867},
    {-0.40524131400498986, -0.9142097557035307},
    {-0.4275550934302821, -0.9039892931234433},
    {-0.4496113296546066, -0.8932243011955153},
    {-0.47139673682599764, -0.881921264348355},
    {-0.49289819222978404, -0.8700869911087115},
    {-0.5141027441932218, -0.8577286100002721},
    {-0.5349976198870973, -0.8448535652497071},
    {-0.5555702330196022, -0.8314696123025452},
    {-0.5758081914178453, -0.8175848131515837},
    {-0.5956993044924334, -0.8032075314806449},
    {-0.6152315905806268, -0.7883464276266062},
    {-0.6343932841636455, -0.773010453362737},
    {-0.6531728429537768, -0.7572088465064846},
    {-0.6715589548470184, -0.7409511253549591},
    {-0.6895405447370669, -0.7242470829514669},
    {-0.7071067811865476, -0.7071067811865476},
    {-0.7242470829514669, -0.6895405447370669},
    {-0.7409511253549591, -0.6715589548470184},
    {-0.7572088465064846, -0.6531728429537768},
    {-0.773010453362737, -0.6343932841636455},
    {-0.7883464276266062, -0.6152315905806268},
    {-0.8032075314806449, -0.5956993044924334},
    {-0.8175848131515837, -0.5758081914178453},
    {-0.8314696123025452, -0.5555702330196022},
    {-0.8448535652497071, -0.5349976198870973},
    {-0.8577286100002721, -0.5141027441932218},
    {-0.8700869911087115, -0.49289819222978404},
    {-0.881921264348355, -0.47139673682599764},
    {-0.8932243011955153, -0.4496113296546066},
    {-0.9039892931234433, -0.4275550934302821},
    {-0.9142097557035307, -0.40524131400498986},
    {-0.9238795325112867, -0.3826834323650898},
    {-0.9329927988347388, -0.35989503653498817},
    {-0.9415440651830208, -0.33688985339222005},
    {-0.9495281805930367, -0.31368174039889146},
    {-0.9569403357322088, -0.2902846772544624},
    {-0.9637760657954398, -0.26671275747489837},
    {-0.970031253194544, -0.2429801799032639},
    {-0.9757021300385286, -0.2191012401568698},
    {-0.9807852804032304, -0.19509032201612828},
    {-0.9852776423889412, -0.17096188876030122},
    {-0.989176509964781, -0.14673047445536175},
    {-0.99247953459871, -0.1224106751992162},
    {-0.9951847266721969, -0.0980171403295606},
    {-0.9972904566786902, -0.07356456359966743},
    {-0.9987954562051724, -0.049067674327418015},
    {-0.9996988186962042, -0.024541228522912288},
    {-1.0, -1.7129905491373045e-61},
    {-0.9996988186962042, 0.024541228522912288},
    {-0.9987954562051724, 0.049067674327418015},
    {-0.9972904566786902, 0.07356456359966743},
    {-0.9951847266721969, 0.0980171403295606},
    {-0.99247953459871, 0.1224106751992162},
    {-0.989176509964781, 0.14673047445536175},
    {-0.9852776423889412, 0.17096188876030122},
    {-0.9807852804032304, 0.19509032201612828},
    {-0.9757021300385286, 0.2191012401568698},
    {-0.970031253194544, 0.2429801799032639},
    {-0.9637760657954398, 0.26671275747489837},
    {-0.9569403357322088, 0.2902846772544624},
    {-0.9495281805930367, 0.31368174039889146},
    {-0.9415440651830208, 0.33688985339222005},
    {-0.9329927988347388, 0.35989503653498817},
    {-0.9238795325112867, 0.3826834323650898},
    {-0.9142097557035307, 0.40524131400498986},
    {-0.9039892931234433, 0.4275550934302821},
    {-0.8932243011955153, 0.4496113296546066},
    {-0.881921264348355, 0.47139673682599764},
    {-0.8700869911087115, 0.49289819222978404},
    {-0.8577286100002721, 0.5141027441932218},
    {-0.8448535652497071, 0.5349976198870973},
    {-0.8314696123025452, 0.5555702330196022},
    {-0.8175848131515837, 0.5758081914178453},
    {-0.8032075314806449, 0.5956993044924334},
    {-0.7883464276266062, 0.6152315905806268},
    {-0.773010453362737, 0.6343932841636455},
    {-0.7572088465064846, 0.6531728429537768},
    {-0.7409511253549591, 0.6715589548470184},
    {-0.7242470829514669, 0.6895405447370669},
    {-0.7071067811865476, 0.7071067811865476},
    {-0.6895405447370669, 0.7242470829514669},
    {-0.6715589548470184, 0.7409511253549591},
    {-0.6531728429537768, 0.7572088465064846},
    {-0.6343932841636455, 0.773010453362737},
    {-0.6152315905806268, 0.7883464276266062},
    {-0.5956993044924334, 0.8032075314806449},
    {-0.5758081914178453, 0.8175848131515837},
    {-0.5555702330196022, 0.8314696123025452},
    {-0.5349976198870973, 0.8448535652497071},
    {-0.5141027441932218, 0.8577286100002721},
    {-0.49289819222978404, 0.8700869911087115},
    {-0.47139673682599764, 0.881921264348355},
    {-0.4496113296546066, 0.8932243011955153},
    {-0.4275550934302821, 0.9039892931234433},
    {-0.40524131400498986, 0.9142097557035307},
    {-0.3826834323650898, 0.9238795325112867},
    {-0.35989503653498817, 0.9329927988347388},
    {-0.33688985339222005, 0.9415440651830208},
    {-0.31368174039889146, 0.9495281805930367},
    {-0.2902846772544624, 0.9569403357322088},
    {-0.26671275747489837, 0.9637760657954398},
    {-0.2429801799032639, 0.970031253194544},
    {-0.2191012401568698, 0.9757021300385286},
    {-0.19509032201612828, 0.9807852804032304},
    {-0.17096188876030122, 0.9852776423889412},
    {-0.14673047445536175, 0.989176509964781},
    {-0.1224106751992162, 0.99247953459871},
    {-0.0980171403295606, 0.9951847266721969},
    {-0.07356456359966743, 0.9972904566786902},
    {-0.049067674327418015, 0.9987954562051724},
    {-0.024541228522912288, 0.9996988186962042},
};
#define DM_BM_DELTA 1.4629180792671596e-09   /* RN(2 pi 2^-32) */

/* log u of a Box-Muller uniform u in [2^-33, 1): u = 2^k z, z in [0.75, 1.5), by integer
 * operations on the high word; r = z / c_i - 1 by one fma with the tabled 1/c_i of z's
 * interval (|r| <= 1/256); log u = k ln2 + L_i + log1p(r), L_i = -log(1/c_i) tabled as hi +
 * lo, log1p(r) = r + r^2 P(r) (Taylor to r^7).  The interval holding 1 has c = 1 (L = 0,
 * r = z - 1 exact), so log u keeps its relative accuracy as u -> 1.  About 1 ulp; 21 VALU
 * instructions on gfx950 against 35 for dm_log_pos (no division).                          */
DM_FN double dm_log_bm(double u)
{
    const uint64_t b = dm_bits(u);
    const uint32_t hi = (uint32_t)(b >> 32);
    const int32_t t = (int32_t)(hi - 0x3fe80000u);              /* 0x3fe8: 0.75 */
    const int32_t k = t >> 20;                                   /* arithmetic */
    const uint32_t i = ((uint32_t)t >> 13) & 127u;
    const double z = dm_from_bits(((uint64_t)(hi - ((uint32_t)t & 0xfff00000u)) << 32) | (b & 0xffffffffull));
    const double* e = dm_bm_log_tab[i];
    const double r = dm_fma(z, e[0], -1.0);
    double p = dm_fmak(r, 1.0 / 7.0, -1.0 / 6.0);
    p = dm_fmak(p, r, 0.2);
    p = dm_fmak(p, r, -0.25);
    p = dm_fmak(p, r, 1.0 / 3.0);
    p = dm_fma_mh(p, r);
    const double l1p = dm_fma(r * r, p, r);
    const double kd = (double)k;
    const double h = kd * DM_LN2_HI + e[1];
    const double l = kd * DM_LN2_LO + e[2];
    return h + (l1p + l);
}

/* sin and cos of 2 pi (b + 1/2) 2^-32 (= dm_sincos2pi(dm_u32(b)) to about 1 ulp): the
 * angle of j = b >> 24 from the table, the rest delta = (b mod 2^24 + 1/2) 2 pi 2^-32 <
 * 2 pi / 256 by Taylor series, combined by the angle-sum formulas.                       */
DM_FN void dm_sincos2pi32(uint32_t b, double* s, double* c)
{
    const double* e = dm_bm_sc_tab[b >> 24];
    const double d = ((double)(b & 0xffffffu) + 0.5) * DM_BM_DELTA;
    const double z = d * d;
    double ps = dm_fmak(z, -1.0 / 5040.0, 1.0 / 120.0);
    ps = dm_fmak(ps, z, -1.0 / 6.0);
    const double sd = dm_fma(d * z, ps, d);
    double pc = dm_fmak(z, 1.0 / 40320.0, -1.0 / 720.0);
    pc = dm_fmak(pc, z, 1.0 / 24.0);
    pc = dm_fma_mh(pc, z);
    const double cd = dm_fma_1(pc, z);
    *s = dm_fma(e[0], cd, e[1] * sd);
    *c = dm_fma(e[1], cd, -(e[0] * sd));
}

/* generated by tools/gen_bm_tables.py: fp32 {sin, cos} of 2 pi j / 256 (each rounded once) */
DM_CONST float dm_bm_sc_tab32[256][2] = {
    {0.0f, 1.0f},
    {0.024541229009628296f, 0.99969881772995f},
    {0.049067676067352295f, 0.9987954497337341f},
    {0.0735645666718483f, 0.9972904324531555f},
    {0.0980171412229538f, 0.9951847195625305f},
    {0.12241067737340927f, 0.9924795627593994f},
    {0.1467304676771164f, 0.9891765117645264f},
    {0.1709618866443634f, 0.9852776527404785f},
    {0.19509032368659973f, 0.9807852506637573f},
    {0.21910123527050018f, 0.9757021069526672f},
    {0.24298018217086792f, 0.9700312614440918f},
    {0.2667127549648285f, 0.9637760519981384f},
    {0.290284663438797f, 0.9569403529167175f},
    {0.3136817514896393f, 0.949528157711029f},
    {0.3368898630142212f, 0.9415440559387207f},
    {0.3598950505256653f, 0.9329928159713745f},
    {0.3826834261417389f, 0.9238795042037964f},
    {0.40524131059646606f, 0.91420978307724f},
    {0.4275550842285156f, 0.903989315032959f},
    {0.4496113359928131f, 0.89322429895401f},
    {0.4713967442512512f, 0.8819212913513184f},
    {0.49289819598197937f, 0.8700869679450989f},
    {0.5141027569770813f, 0.8577286005020142f},
    {0.5349976420402527f, 0.8448535799980164f},
    {0.5555702447891235f, 0.8314695954322815f},
    {0.5758081674575806f, 0.8175848126411438f},
    {0.5956993103027344f, 0.803207516670227f},
    {0.6152315735816956f, 0.7883464097976685f},
    {0.6343932747840881f, 0.7730104327201843f},
    {0.6531728506088257f, 0.7572088241577148f},
    {0.6715589761734009f, 0.7409511208534241f},
    {0.6895405650138855f, 0.7242470979690552f},
    {0.7071067690849304f, 0.7071067690849304f},
    {0.7242470979690552f, 0.6895405650138855f},
    {0.7409511208534241f, 0.6715589761734009f},
    {0.7572088241577148f, 0.6531728506088257f},
    {0.7730104327201843f, 0.6343932747840881f},
    {0.7883464097976685f, 0.6152315735816956f},
    {0.803207516670227f, 0.5956993103027344f},
    {0.8175848126411438f, 0.5758081674575806f},
    {0.8314695954322815f, 0.5555702447891235f},
    {0.8448535799980164f, 0.5349976420402527f},
    {0.8577286005020142f, 0.5141027569770813f},
    {0.8700869679450989f, 0.49289819598197937f},
    {0.8819212913513184f, 0.4713967442512512f},
    {0.89322429895401f, 0.4496113359928131f},
    {0.903989315032959f, 0.4275550842285156f},
    {0.91420978307724f, 0.40524131059646606f},
    {0.9238795042037964f, 0.3826834261417389f},
    {0.9329928159713745f, 0.3598950505256653f},
    {0.9415440559387207f, 0.3368898630142212f},
    {0.949528157711029f, 0.3136817514896393f},
    {0.9569403529167175f, 0.290284663438797f},
    {0.9637760519981384f, 0.2667127549648285f},
    {0.9700312614440918f, 0.24298018217086792f},
    {0.9757021069526672f, 0.21910123527050018f},
    {0.9807852506637573f, 0.19509032368659973f},
    {0.9852776527404785f, 0.1709618866443634f},
    {0.9891765117645264f, 0.1467304676771164f},
    {0.9924795627593994f, 0.12241067737340927f},
    {0.9951847195625305f, 0.0980171412229538f},
    {0.9972904324531555f, 0.0735645666718483f},
    {0.9987954497337341f, 0.049067676067352295f},
    {0.99969881772995f, 0.024541229009628296f},
    {1.0f, 0.0f},
    {0.99969881772995f, -0.024541229009628296f},
    {0.9987954497337341f, -0.049067676067352295f},
    {0.9972904324531555f, -0.0735645666718483f},
    {0.9951847195625305f, -0.0980171412229538f},
    {0.9924795627593994f, -0.12241067737340927f},
    {0.9891765117645264f, -0.1467304676771164f},
    {0.9852776527404785f, -0.1709618866443634f},
    {0.9807852506637573f, -0.19509032368659973f},
    {0.9757021069526672f, -0.21910123527050018f},
    {0.9700312614440918f, -0.24298018217086792f},
    {0.9637760519981384f, -0.2667127549648285f},
    {0.9569403529167175f, -0.290284663438797f},
    {0.949528157711029f, -0.3136817514896393f},
    {0.9415440559387207f, -0.3368898630142212f},
    {0.9329928159713745f, -0.3598950505256653f},
    {0.9238795042037964f, -0.3826834261417389f},
    {0.91420978307724f, -0.40524131059646606f},
    {0.903989315032959f, -0.4275550842285156f},
    {0.89322429895401f, -0.4496113359928131f},
    {0.8819212913513184f, -0.4713967442512512f},
    {0.8700869679450989f, -0.49289819598197937f},
    {0.8577286005020142f, -0.5141027569770813f},
    {0.8448535799980164f, -0.5349976420402527f},
    {0.8314695954322815f, -0.5555702447891235f},
    {0.8175848126411438f, -0.5758081674575806f},
    {0.803207516670227f, -0.5956993103027344f},
    {0.7883464097976685f, -0.6152315735816956f},
    {0.7730104327201843f, -0.6343932747840881f},
    {0.7572088241577148f, -0.6531728506088257f},
    {0.7409511208534241f, -0.6715589761734009f},
    {0.7242470979690552f, -0.6895405650138855f},
    {0.7071067690849304f, -0.7071067690849304f},
    {0.6895405650138855f, -0.7242470979690552f},
    {0.6715589761734009f, -0.7409511208534241f},
    {0.6531728506088257f, -0.7572088241577148f},
    {0.6343932747840881f, -0.7730104327201843f},
    {0.6152315735816956f, -0.7883464097976685f},
    {0.5956993103027344f, -0.803207516670227f},
    {0.5758081674575806f, -0.8175848126411438f},
    {0.5555702447891235f, -0.8314695954322815f},
    {0.5349976420402527f, -0.8448535799980164f},
    {0.5141027569770813f, -0.8577286005020142f},
    {0.49289819598197937f, -0.8700869679450989f},
    {0.4713967442512512f, -0.8819212913513184f},
    {0.4496113359928131f, -0.89322429895401f},
    {0.4275550842285156f, -0.903989315032959f},
    {0.40524131059646606f, -0.91420978307724f},
    {0.3826834261417389f, -0.9238795042037964f},
    {0.3598950505256653f, -0.9329928159713745f},
    {0.3368898630142212f, -0.9415440559387207f},
    {0.3136817514896393f, -0.949528157711029f},
    {0.290284663438797f, -0.9569403529167175f},
    {0.2667127549648285f, -0.9637760519981384f},
    {0.24298018217086792f, -0.9700312614440918f},
    {0.21910123527050018f, -0.9757021069526672f},
    {0.19509032368659973f, -0.9807852506637573f},
    {0.1709618866443634f, -0.9852776527404785f},
    {0.1467304676771164f, -0.9891765117645264f},
    {0.12241067737340927f, -0.9924795627593994f},
    {0.0980171412229538f, -0.9951847195625305f},
    {0.0735645666718483f, -0.9972904324531555f},
    {0.049067676067352295f, -0.9987954497337341f},
    {0.024541229009628296f, -0.99969881772995f},
    {0.0f, -1.0f},
    {-0.024541229009628296f, -0.99969881772995f},
    {-0.049067676067352295f, -0.9987954497337341f},
    {-0.0735645666718483f, -0.9972904324531555f},
    {-0.0980171412229538f, -0.9951847195625305f},
    {-0.12241067737340927f, -0.9924795627593994f},
    {-0.1467304676771164f, -0.9891765117645264f},
    {-0.1709618866443634f, -0.9852776527404785f},
    {-0.19509032368659973f, -0.9807852506637573f},
    {-0.21910123527050018f, -0.9757021069526672f},
    {-0.24298018217086792f, -0.9700312614440918f},
    {-0.2667127549648285f, -0.9637760519981384f},
    {-0.290284663438797f, -0.9569403529167175f},
    {-0.3136817514896393f, -0.949528157711029f},
    {-0.3368898630142212f, -0.9415440559387207f},
    {-0.3598950505256653f, -0.9329928159713745f},
    {-0.3826834261417389f, -0.9238795042037964f},
    {-0.40524131059646606f, -0.91420978307724f},
    {-0.4275550842285156f, -0.903989315032959f},
    {-0.4496113359928131f, -0.89322429895401f},
    {-0.4713967442512512f, -0.8819212913513184f},
    {-0.49289819598197937f, -0.8700869679450989f},
    {-0.5141027569770813f, -0.8577286005020142f},
    {-0.5349976420402527f, -0.8448535799980164f},
    {-0.5555702447891235f, -0.8314695954322815f},
    {-0.5758081674575806f, -0.8175848126411438f},
    {-0.5956993103027344f, -0.803207516670227f},
    {-0.6152315735816956f, -0.7883464097976685f},
    {-0.6343932747840881f, -0.7730104327201843f},
    {-0.6531728506088257f, -0.7572088241577148f},
    {-0.6715589761734009f, -0.7409511208534241f},
    {-0.6895405650138855f, -0.7242470979690552f},
    {-0.7071067690849304f, -0.7071067690849304f},
    {-0.7242470979690552f, -0.6895405650138855f},
    {-0.7409511208534241f, -0.6715589761734009f},
    {-0.7572088241577148f, -0.6531728506088257f},
    {-0.7730104327201843f, -0.6343932747840881f},
    {-0.7883464097976685f, -0.6152315735816956f},
    {-0.803207516670227f, -0.5956993103027344f},
    {-0.8175848126411438f, -0.5758081674575806f},
    {-0.8314695954322815f, -0.5555702447891235f},
    {-0.8448535799980164f, -0.5349976420402527f},
    {-0.8577286005020142f, -0.5141027569770813f},
    {-0.8700869679450989f, -0.49289819598197937f},
    {-0.8819212913513184f, -0.4713967442512512f},
    {-0.89322429895401f, -0.4496113359928131f},
    {-0.903989315032959f, -0.4275550842285156f},
    {-0.91420978307724f, -0.40524131059646606f},
    {-0.9238795042037964f, -0.3826834261417389f},
    {-0.9329928159713745f, -0.3598950505256653f},
    {-0.9415440559387207f, -0.3368898630142212f},
    {-0.949528157711029f, -0.3136817514896393f},
    {-0.9569403529167175f, -0.290284663438797f},
    {-0.9637760519981384f, -0.2667127549648285f},
    {-0.9700312614440918f, -0.24298018217086792f},
    {-0.9757021069526672f, -0.21910123527050018f},
    {-0.9807852506637573f, -0.19509032368659973f},
    {-0.9852776527404785f, -0.1709618866443634f},
    {-0.9891765117645264f, -0.1467304676771164f},
    {-0.9924795627593994f, -0.12241067737340927f},
    {-0.9951847195625305f, -0.0980171412229538f},
    {-0.9972904324531555f, -0.0735645666718483f},
    {-0.9987954497337341f, -0.049067676067352295f},
    {-0.99969881772995f, -0.024541229009628296f},
    {-1.0f, 0.0f},
    {-0.99969881772995f, 0.024541229009628296f},
    {-0.9987954497337341f, 0.049067676067352295f},
    {-0.9972904324531555f, 0.0735645666718483f},
    {-0.9951847195625305f, 0.0980171412229538f},
    {-0.9924795627593994f, 0.12241067737340927f},
    {-0.9891765117645264f, 0.1467304676771164f},
    {-0.9852776527404785f, 0.1709618866443634f},
    {-0.9807852506637573f, 0.19509032368659973f},
    {-0.9757021069526672f, 0.21910123527050018f},
    {-0.9700312614440918f, 0.24298018217086792f},
    {-0.9637760519981384f, 0.2667127549648285f},
    {-0.9569403529167175f, 0.290284663438797f},
    {-0.949528157711029f, 0.3136817514896393f},
    {-0.9415440559387207f, 0.3368898630142212f},
    {-0.9329928159713745f, 0.3598950505256653f},
    {-0.9238795042037964f, 0.3826834261417389f},
    {-0.91420978307724f, 0.40524131059646606f},
    {-0.903989315032959f, 0.4275550842285156f},
    {-0.89322429895401f, 0.4496113359928131f},
    {-0.8819212913513184f, 0.4713967442512512f},
    {-0.8700869679450989f, 0.49289819598197937f},
    {-0.8577286005020142f, 0.5141027569770813f},
    {-0.8448535799980164f, 0.5349976420402527f},
    {-0.8314695954322815f, 0.5555702447891235f},
    {-0.8175848126411438f, 0.5758081674575806f},
    {-0.803207516670227f, 0.5956993103027344f},
    {-0.7883464097976685f, 0.6152315735816956f},
    {-0.7730104327201843f, 0.6343932747840881f},
    {-0.7572088241577148f, 0.6531728506088257f},
    {-0.7409511208534241f, 0.6715589761734009f},
    {-0.7242470979690552f, 0.6895405650138855f},
    {-0.7071067690849304f, 0.7071067690849304f},
    {-0.6895405650138855f, 0.7242470979690552f},
    {-0.6715589761734009f, 0.7409511208534241f},
    {-0.6531728506088257f, 0.7572088241577148f},
    {-0.6343932747840881f, 0.7730104327201843f},
    {-0.6152315735816956f, 0.7883464097976685f},
    {-0.5956993103027344f, 0.803207516670227f},
    {-0.5758081674575806f, 0.8175848126411438f},
    {-0.5555702447891235f, 0.8314695954322815f},
    {-0.5349976420402527f, 0.8448535799980164f},
    {-0.5141027569770813f, 0.8577286005020142f},
    {-0.49289819598197937f, 0.8700869679450989f},
    {-0.4713967442512512f, 0.8819212913513184f},
    {-0.4496113359928131f, 0.89322429895401f},
    {-0.4275550842285156f, 0.903989315032959f},
    {-0.40524131059646606f, 0.91420978307724f},
    {-0.3826834261417389f, 0.9238795042037964f},
    {-0.3598950505256653f, 0.9329928159713745f},
    {-0.3368898630142212f, 0.9415440559387207f},
    {-0.3136817514896393f, 0.949528157711029f},
    {-0.290284663438797f, 0.9569403529167175f},
    {-0.2667127549648285f, 0.9637760519981384f},
    {-0.24298018217086792f, 0.9700312614440918f},
    {-0.21910123527050018f, 0.9757021069526672f},
    {-0.19509032368659973f, 0.9807852506637573f},
    {-0.1709618866443634f, 0.9852776527404785f},
    {-0.1467304676771164f, 0.9891765117645264f},
    {-0.12241067737340927f, 0.9924795627593994f},
    {-0.0980171412229538f, 0.9951847195625305f},
    {-0.0735645666718483f, 0.9972904324531555f},
    {-0.049067676067352295f, 0.9987954497337341f},
    {-0.024541229009628296f, 0.99969881772995f},
};
#define DM_BM_DELTA_F 1.462918119976564e-09f   /* RN32(2 pi 2^-32) */

DM_FN float dm_fmaf(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

/* sin and cos of 2 pi (b + 1/2) 2^-32 in fp32 (the Box-Muller angle): the angle of j = b >> 24
 * from the fp32 table, the rest delta = (b mod 2^24 + 1/2) 2 pi 2^-32 < 2 pi / 256 by its
 * Taylor series (sin to delta^3, cos to delta^4: remainders below 2^-33 relative), combined
 * by the angle-sum formulas.  About 1 ulp of fp32; every operation is an IEEE fp32 add, mul or
 * fma, so the host and the device agree bit for bit.                                       */
DM_FN void dm_sincos2pi32f(uint32_t b, float* s, float* c)
{
    const float* e = dm_bm_sc_tab32[b >> 24];
    const float d = dm_fmaf((float)(b & 0xffffffu), DM_BM_DELTA_F, 0.5f * DM_BM_DELTA_F);
    const float z = d * d;
    const float sd = dm_fmaf(d * z, -1.0f / 6.0f, d);
    const float cd = dm_fmaf(z, dm_fmaf(z, 1.0f / 24.0f, -0.5f), 1.0f);
    *s = dm_fmaf(e[0], cd, e[1] * sd);
    *c = dm_fmaf(e[1], cd, -(e[0] * sd));
}

/* sqrt(x) correctly rounded in fp32 for a positive normal x: on the device the compiler's own
 * correctly rounded sequence (v_sqrt_f32, then the neighbour whose square brackets x) without
 * its tiny-argument scaling and zero/inf fix-up, which such an x never needs (the same bits:
 * tests/test_gpu_parity.py compares it with sqrtf on the device for all 2^32 Box-Muller
 * words); the host's sqrtf is correctly rounded.                                           */
DM_FN float dm_sqrtf_pos(float x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    const float r = __builtin_amdgcn_sqrtf(x);
    const float dn = __uint_as_float(__float_as_uint(r) - 1u), up = __uint_as_float(__float_as_uint(r) + 1u);
    float q = r;
    if (__builtin_fmaf(-dn, r, x) <= 0.0f) q = dn;
    if (__builtin_fmaf(-up, r, x) > 0.0f) q = up;
    return q;
#else
    return __builtin_sqrtf(x);
#endif
}

/* Box-Muller from two 32-bit words (the project / init draw layout): the radius
 * sqrt(-2 log u) from the fp64 log rounded to fp32 and a correctly rounded fp32 sqrt, the
 * angle's sin / cos in fp32; each normal is the exact fp64 product of the two fp32 factors
 * (24 + 24 bits).  Noise draws need no more than fp32's 2^-24 relative resolution (the
 * reference's own uniforms carry 31 bits), and fp32 arithmetic issues at twice the fp64 rate. */
DM_FN void dm_box_muller32(uint32_t a, uint32_t b, double* z0, double* z1)
{
    /* -2 log u in [4.6e-10, 45.8] for u in [2^-33, 1): positive normal in fp32 */
    const float r = dm_sqrtf_pos((float)(-2.0 * dm_log_bm(dm_u32(a))));
    float s, c;
    dm_sincos2pi32f(b, &s, &c);
    *z0 = (double)r * (double)c;
    *z1 = (double)r * (double)s;
}

/* RNG stream identifiers (Philox counter word 3, bits 24..31) */
#define DM_STREAM_PROJECT 1u
#define DM_STREAM_INIT 2u
#define DM_STREAM_HASH 3u

/* Draw block `call` of particle `gidx` for event `ev` of stream `stream`. */
DM_FN dm_philox_ctr dm_draw(uint64_t seed, uint32_t stream, uint64_t ev, uint64_t gidx, uint32_t call)
{
    dm_philox_ctr c;
    c.v[0] = (uint32_t)gidx;
    c.v[1] = (uint32_t)(gidx >> 32);
    c.v[2] = (uint32_t)ev;
    c.v[3] = (stream << 24) | ((call & 0xffu) << 16) | (uint32_t)((ev >> 32) & 0xffffu);
    return dm_philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32) ^ 0x5EED5EEDu);
}

/* ------------------------------------------------------------------------------------ */
/* minstd_rand (Park-Miller, a = 48271, m = 2^31 - 1) with jump-ahead                     */
/* ------------------------------------------------------------------------------------ */
#define DM_MINSTD_A 48271u
#define DM_MINSTD_M 2147483647u

DM_FN uint32_t dm_mulmod31(uint32_t a, uint32_t b)
{
    uint64_t p = (uint64_t)a * b;                  /* < 2^62 */
    uint64_t r = (p & DM_MINSTD_M) + (p >> 31);    /* < 2^32 */
    r = (r & DM_MINSTD_M) + (r >> 31);
    if (r >= DM_MINSTD_M) r -= DM_MINSTD_M;
    return (uint32_t)r;
}

/* boost::random::linear_congruential_engine::seed for minstd_rand */
DM_FN uint32_t dm_minstd_seed(uint64_t s)
{
    uint32_t x = (uint32_t)(s % DM_MINSTD_M);
    return x == 0 ? 1u : x;
}

DM_FN uint32_t dm_minstd_next(uint32_t x) { return dm_mulmod31(x, DM_MINSTD_A); }

/* A^n mod m by square-and-multiply */
DM_FN uint32_t dm_minstd_pow(uint64_t n)
{
    uint32_t r = 1, b = DM_MINSTD_A;
    while (n) { if (n & 1) r = dm_mulmod31(r, b); b = dm_mulmod31(b, b); n >>= 1; }
    return r;
}

/* boost::uniform_real<>(0,1) on an integral engine with min 1, max 2147483646:
 * (x - min) / (max - min + 1) * (1 - 0) + 0                                            */
DM_FN double dm_minstd_uniform(uint32_t x)
{
    return ((double)(x - 1u) / 2147483646.0) * 1.0 + 0.0;
}

/* a / b correctly rounded from y = RN(1/b), without a division (the device's fp64 division
 * is a ten-instruction sequence around a quarter-rate v_rcp_f64).  q0 = RN(a y) is within
 * 2 ulp of a/b; one correction q1 = RN(q0 + RN(a - b q0) y) makes it faithful; then
 * r1 = a - b q1 is exact (fma) and RN(q1 + r1 y) = RN(a/b) (Markstein's theorem: y within
 * half an ulp of 1/b, q1 faithful).  Used where b is a per-step constant, with
 * 0 <= a < 2^64 and 1 <= b < 2^53 (no overflow, no subnormal quotient other than 0).
 * tests/c/check_div.c checks it against the division: exhaustively for the minstd
 * uniform below, and over random and edge (a, b) for the stratified draws.             */
DM_FN double dm_div_recip(double a, double b, double y)
{
    const double q0 = a * y;
    const double q1 = dm_fma(dm_fma(-b, q0, a), y, q0);
    return dm_fma(dm_fma(-b, q1, a), y, q1);
}

#define DM_INV_MINSTD_RANGE 4.656612877414201e-10   /* RN(1 / 2147483646) = 0x1.00000004p-31 */

/* dm_minstd_uniform without the division (bit-identical for every x in [1, 2^31 - 1];
 * the result is >= +0, so "* 1.0 + 0.0" is the identity on it) */
DM_FN double dm_minstd_uniform_fast(uint32_t x)
{
    return dm_div_recip((double)(x - 1u), 2147483646.0, DM_INV_MINSTD_RANGE);
}

/* ------------------------------------------------------------------------------------ */
/* SurfaceHash pieces (host and device)                                                  */
/* ------------------------------------------------------------------------------------ */
/* Buckets<T>::bucketIndex  src/SurfaceHash.hpp:25-29 (int truncation toward zero, clamp);
 * NaN maps to bucket 0 (the reference's int cast of NaN is undefined)                    */
DM_FN int dm_bucket_index(int count, double min_val, double max_val, double value)
{
    const double v = (value - min_val) / (max_val - min_val) * count;
    if (!(v == v)) return 0;
    int idx = v >= 2147483647.0 ? 2147483647 : (v <= -2147483648.0 ? (-2147483647 - 1) : (int)v);
    int lo = idx > 0 ? idx : 0;
    return (count - 1) < lo ? (count - 1) : lo;
}

/* SurfaceParam::fromPoints  src/SurfaceHash.hpp:60-110: the normal equations of the plane
 * z = a x + b y + c solved by a pivoted LDL^T (Eigen::LDLT: the largest remaining
 * diagonal entry as pivot).  P: n points (x, y, z).                                      */
DM_FN void dm_surface_param(const double* P, uint32_t n, double* slope_x, double* slope_y)
{
    double x = 0, y = 0, z = 0, xx = 0, yy = 0, xy = 0, xz = 0, yz = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const double* p = P + 3 * i;
        x += p[0]; y += p[1]; z += p[2];
        xx += p[0] * p[0]; yy += p[1] * p[1]; xy += p[0] * p[1];
        xz += p[0] * p[2]; yz += p[1] * p[2];
    }
    double A[3][3] = {{xx, xy, x}, {xy, yy, y}, {x, y, (double)n}};
    double b[3] = {xz, yz, z};
    int perm[3] = {0, 1, 2};
    for (int k = 0; k < 3; ++k) {
        int piv = k;
        for (int i = k + 1; i < 3; ++i) if (dm_fabs(A[i][i]) > dm_fabs(A[piv][piv])) piv = i;
        if (piv != k) {
            int t = perm[k]; perm[k] = perm[piv]; perm[piv] = t;
            for (int c = 0; c < 3; ++c) { double tmp = A[k][c]; A[k][c] = A[piv][c]; A[piv][c] = tmp; }
            for (int r = 0; r < 3; ++r) { double tmp = A[r][k]; A[r][k] = A[r][piv]; A[r][piv] = tmp; }
        }
        for (int j = 0; j < k; ++j) A[k][k] -= A[k][j] * A[k][j] * A[j][j];
        for (int i = k + 1; i < 3; ++i) {
            double sum = A[i][k];
            for (int j = 0; j < k; ++j) sum -= A[i][j] * A[k][j] * A[j][j];
            A[i][k] = A[k][k] != 0.0 ? sum / A[k][k] : 0.0;
        }
    }
    double r[3] = {b[perm[0]], b[perm[1]], b[perm[2]]};
    for (int i = 0; i < 3; ++i) for (int j = 0; j < i; ++j) r[i] -= A[i][j] * r[j];
    for (int i = 0; i < 3; ++i) r[i] = A[i][i] != 0.0 ? r[i] / A[i][i] : 0.0;
    for (int i = 2; i >= 0; --i) for (int j = i + 1; j < 3; ++j) r[i] -= A[j][i] * r[j];
    double res[3];
    for (int i = 0; i < 3; ++i) res[perm[i]] = r[i];
    *slope_x = res[0];
    *slope_y = res[1];
}

/* ContactModel::lowestPointHeuristic(false)  src/ContactModel.cpp:48-79: per group the
 * lowest contact (ties: lowest index, std::sort of (z, index) pairs), ungrouped contacts
 * as they are.  pos: m yaw-compensated positions.  Returns the number of points.        */
DM_FN uint32_t dm_lowest_points(const double* pos, const int32_t* group, uint32_t m, double* out)
{
    uint32_t nlow = 0;
    int first = -1, best = -1;
    for (uint32_t i = 0; i < m; ++i) {
        if (group[i] >= 0) {
            if (first < 0) { first = (int)i; best = (int)i; }
            else if (pos[3 * i + 2] < pos[3 * best + 2]) best = (int)i;
        }
        if (first < 0) {
            out[3 * nlow] = pos[3 * i]; out[3 * nlow + 1] = pos[3 * i + 1]; out[3 * nlow + 2] = pos[3 * i + 2];
            ++nlow;
        } else if (i + 1 == m || group[i + 1] != group[i]) {
            out[3 * nlow] = pos[3 * best]; out[3 * nlow + 1] = pos[3 * best + 1]; out[3 * nlow + 2] = pos[3 * best + 2];
            ++nlow;
            first = -1;
        }
    }
    return nlow;
}

/* SurfaceHash::create  src/SurfaceHash.hpp:155-231, per (segment, cell).
 * The grid view both sides use: cell (m, n) of index n * width + m; a cell's first
 * patch mean is mean[cell_start[c] * mean_stride] (the device interleaves mean/stdev).   */
typedef struct {
    const uint32_t* cell_start;
    const float* mean;
    uint32_t mean_stride;
    uint32_t width, height;
    uint32_t bins;                       /* slopeBins */
    double scale_x, scale_y, offset_x, offset_y, inv_scale_x, inv_scale_y;
    double g2w[12];                      /* grid2world, 3x4 row-major */
} dm_hash_grid;

/* The template feet rotated for every angular segment (the reference rotates the points
 * BEFORE using them, so segment a uses a + 1 rotations, applied cumulatively) and the
 * segment's particle orientation a * 2 pi / steps + yaw_offset.  pts: steps x 4 x 2.     */
DM_FN void dm_hash_segments(uint32_t steps, const double g2w[12], double* pts, double* orient)
{
    double p[4][2] = {{0.25, 0.0}, {-0.25, 0.0}, {0.25, -0.5}, {-0.25, -0.5}};   /* base = 0.5 */
    double s, c;
    dm_sincos(2.0 * 3.141592653589793 / (double)steps, &s, &c);   /* AngleAxisd(2 pi / steps, Z) */
    const double r00 = 0.0 * 0.0 + c, r01 = 0.0 * 0.0 - s, r10 = 0.0 * 0.0 + s, r11 = 0.0 * 0.0 + c;
    /* yaw of grid2world's rotation: atan2(R10, R00) (base::getYaw), restated on the matrix */
    const double yx = __builtin_sqrt(g2w[10] * g2w[10] + g2w[9] * g2w[9]);
    const double yaw = yx > 1e-12 ? __builtin_atan2(g2w[4], g2w[0]) : 0.0;
    for (uint32_t a = 0; a < steps; ++a) {
        for (int i = 0; i < 4; ++i) {
            const double x = p[i][0], y = p[i][1];
            p[i][0] = (r00 * x + r01 * y) + 0.0 * 0.0;
            p[i][1] = (r10 * x + r11 * y) + 0.0 * 0.0;
            pts[8 * a + 2 * i] = p[i][0];
            pts[8 * a + 2 * i + 1] = p[i][1];
        }
        orient[a] = (((double)a * 2.0) * 3.141592653589793) / (double)steps + yaw;
    }
}

/* one (segment, cell) of the sweep: returns the bucket (bx * bins + by) of the particle it
 * makes, or -1 (fewer than 3 of the 4 feet on cells with patches); pose: x, y, theta, z.
 * pts: this segment's 4 rotated feet.  Cell centre = (m + 1/2) scale + offset (fromGrid);
 * a foot's cell = floor((v - offset) * (1/scale)), off-grid feet have no patch.          */
DM_FN int dm_hash_item(const dm_hash_grid* g, const double* pts, double orient, uint32_t m, uint32_t n, double* pose)
{
    const double x = ((double)m + 0.5) * g->scale_x + g->offset_x;
    const double y = ((double)n + 0.5) * g->scale_y + g->offset_y;
    const double op[4][2] = {{0.25, 0.0}, {-0.25, 0.0}, {0.25, -0.5}, {-0.25, -0.5}};
    double gp[12];
    uint32_t cnt = 0;
    double mean_z = 0.0;
    for (int i = 0; i < 4; ++i) {
        const double fm = dm_floor(((x + pts[2 * i]) - g->offset_x) * g->inv_scale_x);
        const double fn = dm_floor(((y + pts[2 * i + 1]) - g->offset_y) * g->inv_scale_y);
        if (!(fm >= 0.0 && fm < (double)g->width && fn >= 0.0 && fn < (double)g->height)) continue;
        const uint64_t cell = (uint64_t)fn * g->width + (uint64_t)fm;
        const uint32_t b = g->cell_start[cell], e = g->cell_start[cell + 1];
        if (e <= b) continue;
        const double zval = (double)g->mean[(uint64_t)b * g->mean_stride];
        mean_z += zval;
        gp[3 * cnt] = op[i][0] + 0.0;
        gp[3 * cnt + 1] = op[i][1] + 0.0;
        gp[3 * cnt + 2] = 0.0 + zval;
        ++cnt;
    }
    if (cnt < 3) return -1;
    mean_z /= (double)cnt;
    double sx, sy;
    dm_surface_param(gp, cnt, &sx, &sy);
    const int bx = dm_bucket_index((int)g->bins, -1.0, 1.0, sx);
    const int by = dm_bucket_index((int)g->bins, -1.0, 1.0, sy);
    const double* G = g->g2w;
    pose[0] = ((G[0] * x + G[1] * y) + G[2] * mean_z) + G[3];
    pose[1] = ((G[4] * x + G[5] * y) + G[6] * mean_z) + G[7];
    pose[2] = orient;
    pose[3] = (((G[8] * x + G[9] * y) + G[10] * mean_z) + G[11]) + 0.18;
    return bx * (int)g->bins + by;
}

/* inverse of a rigid 3x4 affine [R | t]: [R^T | -R^T t] (global2local -> grid2world) */
DM_FN void dm_affine_inverse(const double A[12], double out[12])
{
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) out[4 * r + c] = A[4 * c + r];
        out[4 * r + 3] = -((A[r] * A[3] + A[4 + r] * A[7]) + A[8 + r] * A[11]);
    }
}

/* glibc rand() (random_r TYPE_3: r_i = r_{i-3} + r_{i-31}, output r_i >> 1), the
 * generator behind the reference's unseeded rand() (seed 1) in SurfaceHash::sample.
 * One state per filter (the reference's is process-global).                              */
typedef struct { uint32_t r[34]; uint32_t i; uint32_t pad; } dm_libc_rand_state;

DM_FN void dm_libc_srand(dm_libc_rand_state* st, uint32_t seed)
{
    int32_t r[344];
    r[0] = (int32_t)(seed ? seed : 1u);
    for (int i = 1; i < 31; ++i) {
        const int64_t v = (16807ll * r[i - 1]) % 2147483647ll;
        r[i] = (int32_t)(v < 0 ? v + 2147483647ll : v);
    }
    for (int i = 31; i < 34; ++i) r[i] = r[i - 31];
    for (int i = 34; i < 344; ++i) r[i] = (int32_t)((uint32_t)r[i - 31] + (uint32_t)r[i - 3]);
    for (int k = 0; k < 34; ++k) st->r[k] = (uint32_t)r[310 + k];
    st->i = 0;
    st->pad = 0;
}

DM_FN int32_t dm_libc_rand(dm_libc_rand_state* st)
{
    /* ring of the last 34 values: slot i holds r_{t-34} (t = the next index) */
    const uint32_t i = st->i;
    const uint32_t v = st->r[(i + 3) % 34] + st->r[(i + 31) % 34];   /* r_{t-31} + r_{t-3} */
    st->r[i] = v;
    st->i = (i + 1) % 34;
    return (int32_t)(v >> 1);
}

/* ------------------------------------------------------------------------------------ */
/* exact fixed-point helpers (order-independent sums)                                    */
/* ------------------------------------------------------------------------------------ */
/* trunc(v * 2^shift) for the resample cumulative sum: v >= 0 finite; saturates at 2^62-1
 * (values with v * 2^shift >= 2^62).  The update path uses shift 60 (normalised weights). */
DM_FN uint64_t dm_fx_shift(double v, int shift)
{
    if (!(v > 0.0)) return 0;
    uint64_t b = dm_bits(v);
    int e = (int)(b >> 52);
    if (e == 0x7ff) return 0x3fffffffffffffffull;
    if (e == 0) return 0;
    uint64_t m = (b & 0x000fffffffffffffull) | 0x0010000000000000ull;
    int sh = e - 1075 + shift;     /* value = m * 2^(e-1075) */
    if (sh >= 10) return 0x3fffffffffffffffull;
    if (sh >= 0) return m << sh;
    if (sh <= -64) return 0;
    return m >> (-sh);
}

DM_FN uint64_t dm_fx61(double v) { return dm_fx_shift(v, 61); }

/* number of stratified draws T_k = fx(((k + U_k) / N), shift) with T_k <= c, U_k the
 * boost uniform of the (k+1)-th minstd draw after xs (the device version reads the jump
 * from tables; same values)                                                               */
DM_FN uint64_t dm_count_draws_le(uint64_t c, uint64_t N, uint32_t xs, int shift)
{
    const unsigned __int128 prod = (unsigned __int128)c * N;
    const uint64_t kstar = (uint64_t)(prod >> shift);
    const uint64_t k0 = kstar >= 1 ? kstar - 1 : 0;
    if (k0 >= N) return N;
    uint64_t cnt = k0;
    uint32_t x = dm_mulmod31(dm_minstd_pow(k0 + 1), xs);
    const double dN = (double)N;
    for (uint64_t k = k0; k <= kstar + 1 && k < N; ++k) {
        const double u = dm_minstd_uniform(x);
        const uint64_t T = dm_fx_shift(((double)k + u) / dN, shift);
        if (T <= c) cnt = k + 1;
        else break;
        x = dm_minstd_next(x);
    }
    return cnt;
}


/* trunc(v * 2^scale) as an unsigned 128-bit integer split in four 32-bit limbs.
 * v >= 0 finite.  Returns 1 if saturated (v * 2^scale >= 2^127).                        */
DM_FN int dm_fx128_limbs(double v, int scale, uint32_t limb[4])
{
    limb[0] = limb[1] = limb[2] = limb[3] = 0;
    if (!(v > 0.0)) return 0;
    uint64_t b = dm_bits(v);
    int e = (int)(b >> 52);
    uint64_t m;
    int ex;
    if (e == 0) { m = b & 0x000fffffffffffffull; ex = -1074; }
    else { m = (b & 0x000fffffffffffffull) | 0x0010000000000000ull; ex = e - 1075; }
    int sh = ex + scale;
    unsigned __int128 x;
    if (sh >= 0) {
        if (sh > 74) { limb[0] = limb[1] = limb[2] = 0xffffffffu; limb[3] = 0x7fffffffu; return 1; }
        x = (unsigned __int128)m << sh;
    } else {
        if (sh <= -64) return 0;
        x = (unsigned __int128)(m >> (-sh));
    }
    limb[0] = (uint32_t)x;
    limb[1] = (uint32_t)(x >> 32);
    limb[2] = (uint32_t)(x >> 64);
    limb[3] = (uint32_t)(x >> 96);
    return 0;
}

/* Convert an exact sum held as limb sums  S = sum_j L[j] * 2^(32 j)  (each L[j] < 2^64)
 * into the nearest double (round-half-even), scaled by 2^(-scale).  O(1): carry-propagate
 * into a 192-bit integer, take the leading 64 bits and a sticky bit.                    */
DM_FN double dm_limbs_to_double(const uint64_t L[4], int scale)
{
    uint32_t d[6];
    uint64_t carry = 0;
    for (int j = 0; j < 4; ++j) {
        uint64_t lo = (L[j] & 0xffffffffull) + carry;
        d[j] = (uint32_t)lo;
        carry = (L[j] >> 32) + (lo >> 32);
    }
    d[4] = (uint32_t)carry;
    d[5] = (uint32_t)(carry >> 32);
    const uint64_t w0 = ((uint64_t)d[1] << 32) | d[0];
    const uint64_t w1 = ((uint64_t)d[3] << 32) | d[2];
    const uint64_t w2 = ((uint64_t)d[5] << 32) | d[4];
    uint64_t hi, rest;
    int base;                                  /* bit index of hi's LSB */
    if (w2) {
        const int lz = __builtin_clzll(w2);
        hi = lz ? (w2 << lz) | (w1 >> (64 - lz)) : w2;
        rest = (lz ? (w1 << lz) : w1) | w0;
        base = 128 - lz;
    } else if (w1) {
        const int lz = __builtin_clzll(w1);
        hi = lz ? (w1 << lz) | (w0 >> (64 - lz)) : w1;
        rest = lz ? (w0 << lz) : w0;
        base = 64 - lz;
    } else if (w0) {
        const int lz = __builtin_clzll(w0);
        hi = w0 << lz;
        rest = 0;
        base = -lz;
    } else {
        return 0.0;
    }
    /* hi holds the leading 64 bits (MSB set); keep 53, round on the other 11 + sticky */
    uint64_t keep = hi >> 11;
    const uint64_t low = hi & 0x7ffull;
    const int sticky = rest != 0;
    if (low > 0x400ull || (low == 0x400ull && (sticky || (keep & 1ull)))) keep += 1;
    int e2 = base + 11;                        /* value = keep * 2^(e2) */
    if (keep == 0x0020000000000000ull) { keep >>= 1; e2 += 1; }
    return dm_ldexp((double)keep, e2 - scale);
}

/* ------------------------------------------------------------------------------------ */
/* canonical reduction order ("sum contract")                                 */
/* ------------------------------------------------------------------------------------ */
/* Per-particle doubles are summed in chunks of 64 sub-lanes x J rows of consecutive
 * global particle indices: chunk c holds [c*64*J, (c+1)*64*J); sub-lane s sums rows
 * j = 0..J-1 (index c*64*J + 64*j + s) sequentially from +0.0; the 64 sub-lane sums are
 * then combined by the xor butterfly (offsets 32,16,8,4,2,1) and the chunk total is
 * converted exactly to fixed point (dm_fx128_limbs) and summed as integers.  J depends
 * only on the GLOBAL particle count, so any sharding over GPUs gives the same bits.     */
#define DM_CHUNK_LANES 64
#define DM_FX_SCALE 112          /* fixed-point scale of a chunk total bounded by 2^10 */
/* per-particle map store: the first probe slot of a cell (multiplicative hash, 32 slots) */
DM_FN uint32_t dm_store_hash(uint32_t cell) { return (cell * 2654435761u) >> 27; }

#define DM_NBUCKETS 6            /* cpoints.size() buckets 0,1,2,3,4,>=5 (phase B)     */

/* J: rows of 64 particles per canonical summation chunk (the weighting kernel runs one chunk
 * per wave).  The chunks are sized to whole generations of the kernel's resident waves on an
 * MI355X (256 CUs x 4 SIMDs x 5 waves = ESLAM_CHUNK_WAVES): G = the generations needed at
 * <= ESLAM_CHUNK_CAP rows, J = ceil(rows / (G x waves)).  4M particles: 13 rows, 5042 chunks
 * in one generation (power-of-two rows left 8192 chunks, 1.6 generations: the second 60 %
 * full); 2M: 7 rows; up to 327 680 particles one row.  Measured (interleaved A/B,
 * profiles/r05/ab_chunk_rows.log): K1 167 -> 160 us at 4M, 96 -> 91 us at 2M.  Part of the sum
 * contract (the oracle uses the same function); ESLAM_CHUNK_CAP also bounds the packed wave
 * counts (64 J ESLAM_MAX_CONTACTS < 2^16).                                                 */
#ifndef ESLAM_CHUNK_WAVES                /* experiment builds only (changes the sum order) */
#define ESLAM_CHUNK_WAVES 5120u
#endif
#ifndef ESLAM_CHUNK_CAP
#define ESLAM_CHUNK_CAP 13u
#endif
DM_FN uint32_t dm_chunk_rows(uint64_t n_global)
{
    const uint64_t rows = (n_global + 63) / 64, per = (uint64_t)ESLAM_CHUNK_WAVES * ESLAM_CHUNK_CAP;
    const uint64_t slots = (rows <= per ? 1 : (rows + per - 1) / per) * (uint64_t)ESLAM_CHUNK_WAVES;
    const uint64_t j = (rows + slots - 1) / slots;
    return j < 1 ? 1u : (uint32_t)j;
}

/* eslam_config::sum_chunk_rows when set, else dm_chunk_rows(n_global) */
DM_FN uint32_t dm_chunk_rows_cfg(uint64_t n_global, uint32_t fixed)
{
    return fixed ? fixed : dm_chunk_rows(n_global);
}

/* exponent e >= 1 with max_w < 2^e (weight scale of the A_n / B_n accumulators) */
DM_FN int dm_weight_exp(double max_w)
{
    if (!(max_w > 0.0) || !dm_isfinite(max_w)) return 1;
    int e = (int)((dm_bits(max_w) >> 52) & 0x7ff) - 1023 + 1;   /* 2^(e-1) <= max_w < 2^e */
    return e < 1 ? 1 : e;
}

/* weightingFunction(x, alpha, beta, gamma)  src/PoseEstimator.cpp:114-128 */
DM_FN double dm_weighting_function(double x, double alpha, double beta, double gamma)
{
    if (x < alpha) return 1.0;
    if (x < beta) {
        double a = (1.0 - gamma) / (alpha - beta);
        double b = 1.0 - alpha * a;
        return a * x + b;
    }
    if (x >= beta) return gamma;
    return 0.0;
}

/* int32 of a double, saturating (NaN -> 0): the device's v_cvt_i32_f64 */
DM_FN int32_t dm_cvt_sat_i32(double x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    int32_t q;
    __asm__("v_cvt_i32_f64 %0, %1" : "=v"(q) : "v"(x));
    return q;
#else
    if (x != x) return 0;
    return x >= 2147483647.0 ? 2147483647 : (x <= -2147483648.0 ? (-2147483647 - 1) : (int32_t)x);
#endif
}

/* processMap's placement of a scan patch (sx, sy) at a particle, Translation(x, y, 0) * Rz(theta)
 * (src/EmbodiedSlamFilter.cpp:186-189), and the grid cell it lands in, for an identity
 * global2local: m = floor((co sx - sn sy + x - offset_x) / scale_x) evaluated as
 * fma(co, sx, fma(-sn, sy, bx)) * inv_scale_x with bx = x - offset_x (per particle), n likewise.
 * Returns the cell index, 0xffffffff off the grid.  The caller skips particles whose bx, by or
 * theta are not finite (no NaN reaches the conversions).                                  */
DM_FN uint32_t dm_merge_cell_mn(double bx, double by, double co, double sn, double sx, double sy, double inv_x,
                                double inv_y, uint32_t width, uint32_t height, uint32_t* mo, uint32_t* no)
{
    const int32_t m = dm_cvt_sat_i32(dm_floor(dm_fma(co, sx, dm_fma(-sn, sy, bx)) * inv_x));
    const int32_t n = dm_cvt_sat_i32(dm_floor(dm_fma(sn, sx, dm_fma(co, sy, by)) * inv_y));
    *mo = (uint32_t)m;
    *no = (uint32_t)n;
    return ((uint32_t)m < width && (uint32_t)n < height) ? (uint32_t)n * width + (uint32_t)m : 0xffffffffu;
}
/* the cell alone (the column m and row n of an on-grid cell: dm_merge_cell_mn) */
DM_FN uint32_t dm_merge_cell(double bx, double by, double co, double sn, double sx, double sy, double inv_x,
                             double inv_y, uint32_t width, uint32_t height)
{
    uint32_t m, n;
    return dm_merge_cell_mn(bx, by, co, sn, sx, sy, inv_x, inv_y, width, height, &m, &n);
}


/* ---- per-particle local maps: a window of tiles of 8 x 8 grid cells -----
 * A particle's own map covers (2 hx + 1) x (2 hy + 1) tiles centred on the tile under the
 * particle at its last map update; tile (a, b) (a = m >> 3, b = n >> 3) lives in slot
 * (a mod wx) + wx (b mod wy), so a window that moves keeps every tile it still covers in
 * place.  A page holds the tile's 64 cells (row-major, cell (m & 7) + 8 (n & 7)), each one
 * patch {mean, stdev}; a cell holds a patch iff stdev >= 0 (an empty cell stores -1).    */
#define DM_LM_TILE_BITS 3
#define DM_LM_PAGE_CELLS 64u
#define DM_LM_NONE 0xffffffffu               /* a slot with no page                           */
#define DM_LM_UNSET ((int32_t)0x80000000)    /* a map that has never been centred (empty)     */
#define DM_LM_MAX_HALF 15u                   /* at most 31 x 31 tiles per window              */
/* half-width in tiles: every cell within r metres of any cell of the centre tile lies in the
 * window (maxSensorRange, src/Configuration.hpp:107: 3 m at 0.1 m cells -> 4 tiles, 9 x 9)  */
DM_FN uint32_t dm_lm_half(double r, double scale)
{
    const double q = r / (8.0 * scale);
    if (!(q > 1.0)) return 1u;
    if (q >= (double)DM_LM_MAX_HALF) return DM_LM_MAX_HALF;
    const uint32_t h = (uint32_t)q;
    return (double)h < q ? h + 1u : h;
}
/* the centre tile of a particle at grid-local l (one axis): the tile of the cell
 * floor((l - offset) * inv_scale), saturated to int32 (callers skip non-finite positions)  */
DM_FN int32_t dm_lm_centre(double l, double off, double inv)
{
    return dm_cvt_sat_i32(dm_floor((l - off) * inv)) >> DM_LM_TILE_BITS;
}
/* tile a (>= 0) inside the window [c - h, c + h] (wrapping uint32 arithmetic: an unset centre
 * is never inside)                                                                           */
DM_FN int dm_lm_inside(uint32_t a, int32_t c, uint32_t h, uint32_t w)
{
    return (uint32_t)(a - (uint32_t)c + h) < w;
}
/* the tile of slot column sa in the window [c - h, c + h] of width w = 2 h + 1 */
DM_FN int64_t dm_lm_tile_of(uint32_t sa, int32_t c, uint32_t h, uint32_t w)
{
    const int64_t lo = (int64_t)c - (int64_t)h;
    int64_t r = ((int64_t)sa - lo) % (int64_t)w;
    if (r < 0) r += (int64_t)w;
    return lo + r;
}
/* a page cell holds a patch */
DM_FN int dm_lm_holds(float stdev) { return stdev >= 0.0f; }
/* processMap's per-cell merge of a placed scan patch (wz, var) into a cell holding (m1, s1):
 * the variance-weighted fusion when within 3 sigma (envire's MLSGrid::merge is not in the
 * reference: this rule is the build's own, parity unpinned); returns 0 when it leaves the
 * cell as it is                                                                            */
DM_FN int dm_lm_fuse(float m1f, float s1f, double wz, double var, float* mo, float* so)
{
    const double m1 = (double)m1f, s1 = (double)s1f;
    const double v1 = s1 * s1, d = wz - m1;
    if (!(d * d <= 9.0 * (v1 + var))) return 0;
    const double m = (m1 * var + wz * v1) / (v1 + var);
    const double v = (v1 * var) / (v1 + var);
    *mo = (float)m;
    *so = (float)dm_sqrt(v);
    return 1;
}

#endif /* ESLAM_DETMATH_H */
