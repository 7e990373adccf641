// every float x in [lo, hi] (both signs when lo >= 0; bit-pattern stride): vh_expf_any(x) against
// (float)exp((double)x) with glibc's exp.  g++ -O2 -std=c++17 -ffp-contract=off -I.
#include "expf_any.h"
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
int main(int argc, char **argv) {
    const float lo = atof(argv[1]), hi = atof(argv[2]);
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
            const float got = vh_expf_any(x, [&](float v) { ++fb; return full(v); });
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
