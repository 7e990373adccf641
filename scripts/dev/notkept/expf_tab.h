#pragma once
// (float)exp((double)x) -- the spec's p = (float)exp((double)d) of ITK's S7 step -- without the full
// double exp on the common path (PC pass 0 runs one per masked voxel and iteration, in FP64 at a
// quarter of the FP32 rate).  A table-driven double evaluation: x = k ln2/64 + r (Cody-Waite, two
// constants), |r| <= ln2/128 + slack, exp(r) by its degree-5 Taylor polynomial (truncation
// < 2^-54), times 2^(j/64) (j = k mod 64, correctly rounded table) and 2^(k div 64).  Its relative
// error stays below 2^-49: within 16 double ulps of exp(x).  Rounded to float, it equals
// (float)exp((double)x) for any double exp within 1 ulp of exact unless it lies within 256 ulps of
// a float rounding midpoint (its low 29 mantissa bits near 2^28, about 2^-20 of the arguments);
// there, and outside |x| < 80, the full double exp decides.  expf_tab_check.cpp (g++, this
// directory) checks every finite float against glibc: 0 mismatches.  Measured and not kept (r4as).
#include <cmath>
#include <cstdint>
#include <cstring>

#if defined(__HIPCC__)
#define VH_EXPT_HD __host__ __device__ __forceinline__
#else
#define VH_EXPT_HD inline
#endif

#define VH_EXPT_TABLE \
    0x1.0000000000000p+0, 0x1.02c9a3e778061p+0, 0x1.059b0d3158574p+0, 0x1.0874518759bc8p+0, \
    0x1.0b5586cf9890fp+0, 0x1.0e3ec32d3d1a2p+0, 0x1.11301d0125b51p+0, 0x1.1429aaea92de0p+0, \
    0x1.172b83c7d517bp+0, 0x1.1a35beb6fcb75p+0, 0x1.1d4873168b9aap+0, 0x1.2063b88628cd6p+0, \
    0x1.2387a6e756238p+0, 0x1.26b4565e27cddp+0, 0x1.29e9df51fdee1p+0, 0x1.2d285a6e4030bp+0, \
    0x1.306fe0a31b715p+0, 0x1.33c08b26416ffp+0, 0x1.371a7373aa9cbp+0, 0x1.3a7db34e59ff7p+0, \
    0x1.3dea64c123422p+0, 0x1.4160a21f72e2ap+0, 0x1.44e086061892dp+0, 0x1.486a2b5c13cd0p+0, \
    0x1.4bfdad5362a27p+0, 0x1.4f9b2769d2ca7p+0, 0x1.5342b569d4f82p+0, 0x1.56f4736b527dap+0, \
    0x1.5ab07dd485429p+0, 0x1.5e76f15ad2148p+0, 0x1.6247eb03a5585p+0, 0x1.6623882552225p+0, \
    0x1.6a09e667f3bcdp+0, 0x1.6dfb23c651a2fp+0, 0x1.71f75e8ec5f74p+0, 0x1.75feb564267c9p+0, \
    0x1.7a11473eb0187p+0, 0x1.7e2f336cf4e62p+0, 0x1.82589994cce13p+0, 0x1.868d99b4492edp+0, \
    0x1.8ace5422aa0dbp+0, 0x1.8f1ae99157736p+0, 0x1.93737b0cdc5e5p+0, 0x1.97d829fde4e50p+0, \
    0x1.9c49182a3f090p+0, 0x1.a0c667b5de565p+0, 0x1.a5503b23e255dp+0, 0x1.a9e6b5579fdbfp+0, \
    0x1.ae89f995ad3adp+0, 0x1.b33a2b84f15fbp+0, 0x1.b7f76f2fb5e47p+0, 0x1.bcc1e904bc1d2p+0, \
    0x1.c199bdd85529cp+0, 0x1.c67f12e57d14bp+0, 0x1.cb720dcef9069p+0, 0x1.d072d4a07897cp+0, \
    0x1.d5818dcfba487p+0, 0x1.da9e603db3285p+0, 0x1.dfc97337b9b5fp+0, 0x1.e502ee78b3ff6p+0, \
    0x1.ea4afa2a490dap+0, 0x1.efa1bee615a27p+0, 0x1.f50765b6e4540p+0, 0x1.fa7c1819e90d8p+0, \

VH_EXPT_HD float vh_expf_tab(float x, const double *tab) {
    if (!(x > -80.0f && x < 80.0f)) return (float)exp((double)x);
    const float kf = rintf(x * 92.33248261689366f);   // 64 / ln2 (any nearby integer k will do)
    const int k = (int)kf;
    const double kd = (double)kf;
    double r = fma(-kd, 0x1.62e42fefa39efp-7, (double)x);   // ln2 / 64, high part
    r = fma(-kd, 0x1.abc9e3b39803fp-62, r);                 // and the rest
    double p = fma(r, 1.0 / 120.0, 1.0 / 24.0);
    p = fma(p, r, 1.0 / 6.0);
    p = fma(p, r, 0.5);
    p = fma(p, r, 1.0);
    p = fma(p, r, 1.0);
    const double y = ldexp(tab[k & 63] * p, k >> 6);   // (k >> 6: floor division, k & 63 in [0, 64))
    uint64_t bits;
    __builtin_memcpy(&bits, &y, sizeof bits);
    const int lo = (int)(bits & 0x1fffffffu);   // the double's mantissa bits below float precision
    if (abs(lo - (1 << 28)) < 256) return (float)exp((double)x);
    return (float)y;
}
