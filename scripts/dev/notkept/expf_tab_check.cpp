#include "expf_tab.h"   // g++ -O2 -std=c++17 -ffp-contract=off -I. expf_tab_check.cpp; ./a.out 0 88 1
#include <cstdio>
#include <cstdlib>
static const double TAB[64] = {VH_EXPT_TABLE};
int main(int argc, char **argv) {
    // every float in [lo, hi] with the given stride (in float bit patterns), both signs
    const float lo = atof(argv[1]), hi = atof(argv[2]);
    const long stride = atol(argv[3]);
    long n = 0, bad = 0, fb = 0;
    for (int s = 0; s < 2; ++s) {
        uint32_t a, b; float flo = lo, fhi = hi;
        memcpy(&a, &flo, 4); memcpy(&b, &fhi, 4);
        for (uint64_t u = a; u <= b; u += stride) {
            uint32_t w = (uint32_t)u | (s ? 0x80000000u : 0u);
            float x; memcpy(&x, &w, 4);
            const float ref = (float)exp((double)x), got = vh_expf_tab(x, TAB);
            ++n;
            if (memcmp(&ref, &got, 4)) { if (bad < 5) printf("bad x=%a ref=%a got=%a\n", x, ref, got); ++bad; }
        }
    }
    printf("n %ld bad %ld\n", n, bad);
    return bad != 0;
}
