// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the load and store widths the N4
// kernels issue (MI355X_MICROARCH.md HBM section: FETCH_SIZE is calibrated there
// only for 16-B-per-lane streaming reads, where it reports half the bytes).  Each kernel touches a
// known set of 128-B lines of a 1 GiB array (4x the 256 MiB Infinity Cache, so nothing is served
// from a warm cache) once; the counters of its dispatch divided by the bytes of the lines it touched
// give the factor for that access form.
//   mode 0  16-B loads, coalesced (the guide's calibrated case: expect FETCH = 0.5 x bytes)
//   mode 1  4-B loads, coalesced (a wave reads 256 contiguous bytes: k_n4_study's U / L0 / d loads)
//   mode 2  4-B loads, one per 128-B line (lanes 128 B apart: column walks, scattered parked p)
//   mode 3  4-B loads, lanes 32 B apart (a wave touches 16 lines, 8 B of each ... 4 B of each 32)
//   mode 4  16-B stores, coalesced
//   mode 5  4-B stores, coalesced
//   mode 6  4-B stores, one per 128-B line
// usage: fetch_calib MODE   (prints the bytes of the lines the dispatch touched)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr size_t BYTES = (size_t)1 << 30;   // 1 GiB

__global__ void ld16(const float4 *a, float *out, size_t n) {   // n float4
    float s = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.f) out[0] = s;   // keeps the loads
}
__global__ void ld4(const float *a, float *out, size_t n, size_t stride) {   // n loads, stride floats apart
    float s = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        s += a[i * stride];
    if (s == 12345.f) out[0] = s;
}
__global__ void st16(float4 *a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}
__global__ void st4(float *a, size_t n, size_t stride) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i * stride] = (float)i;
}

int main(int argc, char **argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 0;
    float *a = nullptr, *out = nullptr;
    CHK(hipMalloc(&a, BYTES));
    CHK(hipMalloc(&out, 64));
    CHK(hipMemset(a, 0, BYTES));
    CHK(hipDeviceSynchronize());
    const dim3 g(1024), b(256);
    size_t lines = 0;   // 128-B lines the dispatch touches
    switch (mode) {
        case 0: ld16<<<g, b>>>((const float4 *)a, out, BYTES / 16); lines = BYTES / 128; break;
        case 1: ld4<<<g, b>>>(a, out, BYTES / 4, 1); lines = BYTES / 128; break;
        case 2: ld4<<<g, b>>>(a, out, BYTES / 128, 32); lines = BYTES / 128; break;
        case 3: ld4<<<g, b>>>(a, out, BYTES / 32, 8); lines = BYTES / 128; break;
        case 4: st16<<<g, b>>>((float4 *)a, BYTES / 16); lines = BYTES / 128; break;
        case 5: st4<<<g, b>>>(a, BYTES / 4, 1); lines = BYTES / 128; break;
        case 6: st4<<<g, b>>>(a, BYTES / 128, 32); lines = BYTES / 128; break;
        default: printf("mode 0..6\n"); return 1;
    }
    CHK(hipGetLastError());
    CHK(hipDeviceSynchronize());
    const size_t useful = mode == 2 || mode == 6 ? lines * 4 : mode == 3 ? lines * 16 : lines * 128;
    printf("fetch_calib mode %d lines %zu line_bytes %zu useful_bytes %zu\n", mode, lines, lines * 128, useful);
    CHK(hipFree(a));
    CHK(hipFree(out));
    return 0;
}
