// Microbenchmark: the product convergence chain (n4_shared.h chain_wave_mu / chain_wave_sig) on
// random d values, one workgroup per "study", 1 or 256 workgroups, n = 82k (the bench study size);
// prints ns and clock64 per step.  Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off
//   -std=c++17 -I../../include -I../../vent_analysis_amd/csrc welford_real.hip -o welford_real
#include "n4_shared.h"
#include <cstdio>
#include <vector>

__global__ void __launch_bounds__(384) k_real(const float *D, int64_t n, float *out,
                                              unsigned long long *cyc) {
    __shared__ ChainSlot slots[CH_SLOTS];
    __shared__ ChainState cs;
    chain_reset(slots, &cs);
    __syncthreads();
    const unsigned long long t0 = clock64();
    if (threadIdx.x < 64) chain_wave_mu(n, slots, &cs);
    else if (threadIdx.x < 128) chain_wave_sig(n, slots, &cs);
    else chain_wave_prod(D + blockIdx.x * n, nullptr, n, slots, &cs, (threadIdx.x >> 6) - 2, 4);
    __syncthreads();
    if (threadIdx.x == 0) {
        out[blockIdx.x] = cs.conv;
        if (blockIdx.x == 0) cyc[0] = clock64() - t0;
    }
}

int main() {
    const int64_t n = 82162;
    const int nbmax = 256;
    std::vector<float> h((size_t)n * nbmax);
    unsigned s = 12345;
    for (auto &v : h) {
        s = s * 1664525u + 1013904223u;
        v = 1e-3f * ((float)(s >> 8) / 16777216.0f - 0.5f);
    }
    float *d, *o;
    unsigned long long *c;
    (void)hipMalloc(&d, h.size() * 4);
    (void)hipMalloc(&o, nbmax * 4);
    (void)hipMalloc(&c, 8);
    (void)hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    for (int nb : {1, 256, 1, 256}) {
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        k_real<<<nb, 384>>>(d, n, o, c);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        unsigned long long cy = 0;
        float conv = 0;
        (void)hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(&conv, o, 4, hipMemcpyDeviceToHost);
        printf("blocks %3d: %.3f ms  %.2f ns/step  %.1f clock64/step  conv %.6g\n", nb, ms,
               ms * 1e6 / n, (double)cy / n, conv);
    }
    return 0;
}
