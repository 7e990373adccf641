#pragma once
// measured and not kept (r4az: the E map's Gaussian kernel exp, no change)
#include <cstdint>

// (float)exp((double)x) for -104 < x < 88.5 without a table: x = k ln2 + r (Cody-Waite, two
// constants, |r| <= 0.347 + slack), exp(r) by its degree-12 Taylor polynomial (truncation
// < 2^-52), times 2^k; within 64 double ulps of exp(x).  Rounded to float it is the spec's value
// unless it lies near a float rounding midpoint -- the low 29 mantissa bits within 256 of 2^28 for
// a normal float result, the scaled fraction within 2^-20 of 1/2 for a subnormal one (x < -87.34)
// -- where, as outside the range, the full double exp decides.  (The E map's Gaussian kernel.)
template <class FullExp>
#if defined(__HIPCC__)
__host__ __device__ __forceinline__
#else
inline
#endif
float vh_expf_any(float x, FullExp full) {
    if (!(x > -104.0f && x < 88.5f)) return full(x);
    const float kf = __builtin_rintf(x * 1.44269504f);   // any nearby integer k will do
    const double kd = (double)kf;
    double r = __builtin_fma(-kd, 0x1.62e42fefa39efp-1, (double)x);   // ln2, high part
    r = __builtin_fma(-kd, 0x1.abc9e3b39803fp-56, r);                 // and the rest
    double p = __builtin_fma(r, 1.0 / 479001600.0, 1.0 / 39916800.0);
    p = __builtin_fma(p, r, 1.0 / 3628800.0);
    p = __builtin_fma(p, r, 1.0 / 362880.0);
    p = __builtin_fma(p, r, 1.0 / 40320.0);
    p = __builtin_fma(p, r, 1.0 / 5040.0);
    p = __builtin_fma(p, r, 1.0 / 720.0);
    p = __builtin_fma(p, r, 1.0 / 120.0);
    p = __builtin_fma(p, r, 1.0 / 24.0);
    p = __builtin_fma(p, r, 1.0 / 6.0);
    p = __builtin_fma(p, r, 0.5);
    p = __builtin_fma(p, r, 1.0);
    p = __builtin_fma(p, r, 1.0);
    const double y = __builtin_ldexp(p, (int)kf);
    bool near;
    if (y >= 0x1p-126) {
        uint64_t bits;
        __builtin_memcpy(&bits, &y, sizeof bits);
        const int dm = (int)(bits & 0x1fffffffu) - (1 << 28);
        near = dm > -256 && dm < 256;
    } else {   // a subnormal float: its spacing is 2^-149
        const double t = y * 0x1p149;
        near = __builtin_fabs((t - __builtin_floor(t)) - 0.5) < 0x1p-20;
    }
    return near ? full(x) : (float)y;
}
