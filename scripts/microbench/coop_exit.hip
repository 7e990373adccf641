// Minimal reproducer for the exit-time SIGSEGV under rocprofv3: one cooperative
// launch of a trivial kernel with a grid barrier, then a normal exit.  Nothing of libventhip.so.
// build: hipcc --offload-arch=gfx950 -O2 -o coop_exit coop_exit.hip
// run:   rocprofv3 --kernel-trace --stats -d out -o run -- ./coop_exit [coop=1]
#include <hip/hip_cooperative_groups.h>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void k_grid(int *x) {
    namespace cg = cooperative_groups;
    cg::grid_group g = cg::this_grid();
    if (threadIdx.x == 0) atomicAdd(x, 1);
    g.sync();
    if (blockIdx.x == 0 && threadIdx.x == 0) x[1] = x[0];
}
__global__ void k_plain(int *x) {
    if (threadIdx.x == 0) atomicAdd(x, 1);
}

int main(int argc, char **argv) {
    const int coop = argc > 1 ? atoi(argv[1]) : 1;
    int *d = nullptr;
    if (hipMalloc(&d, 2 * sizeof(int)) != hipSuccess) return 1;
    if (hipMemset(d, 0, 2 * sizeof(int)) != hipSuccess) return 1;
    void *args[] = {&d};
    hipError_t e = coop ? hipLaunchCooperativeKernel((const void *)k_grid, dim3(64), dim3(256), args, 0, 0)
                        : hipLaunchKernel((const void *)k_plain, dim3(64), dim3(256), args, 0, 0);
    if (e != hipSuccess || hipDeviceSynchronize() != hipSuccess) return 2;
    int h[2] = {0, 0};
    if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 3;
    printf("coop=%d blocks counted %d (after barrier %d)\n", coop, h[0], h[1]);
    (void)hipFree(d);
    return 0;
}
