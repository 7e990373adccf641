// Exhaustive check of the PC step constants (n4_shared.h pc_rcp / pc_step) against IEEE division:
// for every k in [1, 2^25): r = RN(1/k) and c = RN((k-1)/k) computed the PC way must equal
// 1.0 / k and (k - 1.0) / k bit for bit.  Prints the mismatch counts (expect 0 0).
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I../../vent_analysis_amd/csrc recip_exact.hip -o recip_exact
#include <hip/hip_runtime.h>
#include <cstdio>
#include "n4_shared.h"

__global__ void k_check(unsigned long long *bad) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x + 1u;
    if (k >= (1u << 25)) return;
    const double kd = (double)k;
    const double r = pc_rcp(kd);
    const double A = 1.0 - r;
    const double z = A - 1.0, err = -r - z;
    const double res = fma(-kd, r, 1.0);
    const double c = A + fma(-res, r, err);
    const double r_ref = 1.0 / kd, c_ref = (kd - 1.0) / kd;
    if (__double_as_longlong(r) != __double_as_longlong(r_ref)) atomicAdd(&bad[0], 1ull);
    if (k > 1 && __double_as_longlong(c) != __double_as_longlong(c_ref)) atomicAdd(&bad[1], 1ull);
}

int main() {
    unsigned long long *d, h[2] = {0, 0};
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    hipMemset(d, 0, sizeof(h));
    k_check<<<(1u << 25) / 256, 256>>>(d);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("recip mismatches %llu  (k-1)/k mismatches %llu  over k < 2^25\n", h[0], h[1]);
    return (h[0] || h[1]) ? 2 : 0;
}
