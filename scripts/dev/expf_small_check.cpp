// every float x with lo <= |x| <= hi (float bit patterns, given stride): vh_expf_small(x) against
// (float)exp((double)x) with glibc's exp.  g++ -O2 -std=c++17 -ffp-contract=off -I../../vent_analysis_amd/csrc
#include "expf_small.h"
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
int main(int argc, char **argv) {
    const float lo = argc > 1 ? atof(argv[1]) : 0.0f, hi = argc > 2 ? atof(argv[2]) : 0x1p-5f;
    const long stride = argc > 3 ? atol(argv[3]) : 1;
    auto full = [](float v) { return (float)exp((double)v); };
    long n = 0, bad = 0, fb = 0;
    for (int s = 0; s < 2; ++s) {
        uint32_t a, b;
        memcpy(&a, &lo, 4);
        memcpy(&b, &hi, 4);
        for (uint64_t u = a; u <= b; u += stride) {
            const uint32_t w = (uint32_t)u | (s ? 0x80000000u : 0u);
            float x;
            memcpy(&x, &w, 4);
            const float ref = full(x);
            const float got = vh_expf_small(x, [&](float v) { ++fb; return full(v); });
            ++n;
            if (memcmp(&ref, &got, 4)) {
                if (bad < 5) printf("bad x=%a ref=%a got=%a\n", x, ref, got);
                ++bad;
            }
        }
    }
    printf("n %ld bad %ld fallbacks %ld\n", n, bad, fb);
    return bad != 0;
}
