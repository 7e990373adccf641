#pragma once
// (float)exp((double)x) for |x| <= 2^-5 -- PC pass 0's p = exp(d), d the field difference of two
// consecutive iterations, is nearly always that small -- without the full double exp: the degree-6
// Taylor polynomial in double (truncation |x|^7 / 7! < 2^-47.3 relative, Horner roundings ~3 2^-53),
// within 64 double ulps of exp(x).  Rounded to float it equals (float)exp((double)x) for any double
// exp within 1 ulp of exact unless it lies within 256 ulps of a float rounding midpoint (its low
// 29 mantissa bits near 2^28: about 2^-20 of the arguments); there, and for |x| > 2^-5, the full
// double exp decides.  tests/test_expf_small.py runs this same source under g++ against glibc's
// exp; every float with |x| <= 2^-5 was checked once (0 mismatches, scripts/dev/expf_small_check.cpp).
// Plain C++ (host and device): the caller supplies its own exp for the fallback.
#include <cstdint>

template <class FullExp>
#if defined(__HIPCC__)
__host__ __device__ __forceinline__
#else
inline
#endif
float vh_expf_small(float x, FullExp full) {
    if (!(x >= -0x1p-5f && x <= 0x1p-5f)) return full(x);
    const double d = (double)x;
    double p = __builtin_fma(d, 1.0 / 720.0, 1.0 / 120.0);
    p = __builtin_fma(p, d, 1.0 / 24.0);
    p = __builtin_fma(p, d, 1.0 / 6.0);
    p = __builtin_fma(p, d, 0.5);
    p = __builtin_fma(p, d, 1.0);
    p = __builtin_fma(p, d, 1.0);
    uint64_t bits;
    __builtin_memcpy(&bits, &p, sizeof bits);
    const int lo = (int)(bits & 0x1fffffffu);   // the double's mantissa bits below float precision
    const int dm = lo - (1 << 28);
    if (dm > -256 && dm < 256) return full(x);
    return (float)p;
}

