// Microbenchmark: dependent latency of the float-Welford step forms on gfx950 (one wave, lane 0
// does the work; register operands, loop-invariant coefficients).  Prints cycles per step.
#include <hip/hip_runtime.h>
#include <cstdio>

#define STEPS 65536

template <int MODE>
__global__ void k_lat(double a, double b, float *out, unsigned long long *cyc) {
    double m0 = 0.3, m1 = 0.4, m2 = 0.5, m3 = 0.6;
    float f0 = 0.3f;
    const unsigned long long t0 = clock64();
    if (threadIdx.x == 0) {
#pragma unroll 16
        for (int k = 0; k < STEPS; ++k) {
            if (MODE == 0) {        // fma64 -> cvt f32 -> cvt f64
                m0 = (double)(float)fma(m0, a, b);
            } else if (MODE == 1) { // four independent chains interleaved
                m0 = (double)(float)fma(m0, a, b);
                m1 = (double)(float)fma(m1, a, b);
                m2 = (double)(float)fma(m2, a, b);
                m3 = (double)(float)fma(m3, a, b);
            } else if (MODE == 2) { // fma64 only
                m0 = fma(m0, a, b);
            } else if (MODE == 3) { // fmaf only
                f0 = fmaf(f0, (float)a, (float)b);
            } else {                // mul64 + add64 -> cvt -> cvt (unfused, as written in ITK)
                m0 = (double)(float)(m0 * a + b);
            }
        }
    }
    const unsigned long long t1 = clock64();
    if (threadIdx.x == 0) {
        out[0] = (float)(m0 + m1 + m2 + m3) + f0;
        cyc[0] = t1 - t0;
    }
}

template <int MODE>
void run(const char *name, float *dout, unsigned long long *dcyc) {
    for (int rep = 0; rep < 2; ++rep) {
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0);
        k_lat<MODE><<<1, 64>>>(0.9999, 1.0e-5, dout, dcyc);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        unsigned long long c = 0;
        hipMemcpy(&c, dcyc, 8, hipMemcpyDeviceToHost);
        printf("%-28s rep %d: %.3f ms  %.2f clock64/step  %.2f ns/step\n", name, rep, ms,
               (double)c / STEPS, ms * 1e6 / STEPS);
    }
}

int main() {
    float *dout;
    unsigned long long *dcyc;
    (void)hipMalloc(&dout, 16);
    (void)hipMalloc(&dcyc, 8);
    run<0>("fma64+cvt+cvt", dout, dcyc);
    run<1>("4 chains interleaved", dout, dcyc);
    run<2>("fma64 only", dout, dcyc);
    run<3>("fmaf only", dout, dcyc);
    run<4>("mul64+add64+cvt+cvt", dout, dcyc);
    return 0;
}
