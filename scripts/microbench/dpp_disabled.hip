// Microtest: what a DPP read returns when its source lane is disabled by EXEC (gfx950), for
// v_mov_b32_dpp row_newbcast:0 and v_cvt_f64_f32_dpp row_newbcast:0 with lane 0 disabled.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(float *o, double *o2) {
    const int lane = threadIdx.x;
    float v = 100.0f + lane, r = -1.0f;
    double d = -1.0;
    uint64_t sv;
    asm volatile("s_mov_b64 %3, exec\n\t"
                 "s_mov_b32 exec_lo, 0xfffffffe\n\t"
                 "s_mov_b32 exec_hi, 0\n\t"
                 "s_nop 4\n\t"
                 "v_mov_b32_dpp %0, %2 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
                 "v_cvt_f64_f32_dpp %1, %2 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
                 "s_mov_b64 exec, %3\n\t"
                 : "+v"(r), "+v"(d), "+v"(v), "=&s"(sv));
    o[lane] = r;
    o2[lane] = d;
}
int main() {
    float *o; double *o2;
    (void)hipMalloc(&o, 64 * 4); (void)hipMalloc(&o2, 64 * 8);
    k<<<1, 64>>>(o, o2);
    float h[64]; double h2[64];
    (void)hipMemcpy(h, o, 256, hipMemcpyDeviceToHost);
    (void)hipMemcpy(h2, o2, 512, hipMemcpyDeviceToHost);
    for (int i : {0, 1, 2, 15, 16, 17, 31, 32, 40})
        printf("lane %2d: mov %g cvt %g\n", i, h[i], h2[i]);
    return 0;
}
