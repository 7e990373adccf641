// Microbenchmark: per-step cost of the serial float-Welford mu recurrence over 64-step blocks
// (one wave; LDS slot of (A, B) pairs written by all lanes, consumed serially), four structures:
//   0: lane 0 loop, #pragma unroll 4, LDS reads (the round-2 chain_wave_mu)
//   1: lane 0, fully unrolled 64 steps, LDS reads issued 8 steps ahead through a register ring
//   2: all lanes, (A, B) kept in the lanes' registers, step l reads lane l's pair by readlane
//   3: lane 0, fully unrolled, one b128 LDS read per step, no explicit prefetch (compiler order)
//   4: as 1, but the mu-before-step values stay in 64 registers, written as 16 b128 at block end
//   5: as 4 plus an independent second chain (the sig recurrence) interleaved in the same wave
//   6: groups of 8: the next group's 8 reads are issued before this group's 8 steps (pinned by
//      sched_barrier), mu captured in registers
//   7: explicit pipeline in inline asm: group g+1's 8 ds_read_b128 issued before group g's steps,
//      s_waitcnt lgkmcnt(N) tied to the group's registers, mu captured and written 2 x b128/group
#include <hip/hip_runtime.h>
#include <cstdio>

#define NBLK 4096

__device__ __forceinline__ void lds_order() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ double rl64(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}


// 8 ds_read_b128 of the (A, B) pairs [8 g .. 8 g + 7] at LDS byte address base
#define CH_RD8(q, base, g)                                                                          \
    asm volatile("ds_read_b128 %0, %8 offset:%9\n\t"                                              \
                 "ds_read_b128 %1, %8 offset:%10\n\t"                                             \
                 "ds_read_b128 %2, %8 offset:%11\n\t"                                             \
                 "ds_read_b128 %3, %8 offset:%12\n\t"                                             \
                 "ds_read_b128 %4, %8 offset:%13\n\t"                                             \
                 "ds_read_b128 %5, %8 offset:%14\n\t"                                             \
                 "ds_read_b128 %6, %8 offset:%15\n\t"                                             \
                 "ds_read_b128 %7, %8 offset:%16"                                                   \
                 : "=&v"(q[0]), "=&v"(q[1]), "=&v"(q[2]), "=&v"(q[3]), "=&v"(q[4]), "=&v"(q[5]),    \
                   "=&v"(q[6]), "=&v"(q[7])                                                         \
                 : "v"(base), "i"(128 * (g)), "i"(128 * (g) + 16), "i"(128 * (g) + 32),              \
                   "i"(128 * (g) + 48), "i"(128 * (g) + 64), "i"(128 * (g) + 80),                    \
                   "i"(128 * (g) + 96), "i"(128 * (g) + 112))

typedef double dbl2v __attribute__((ext_vector_type(2)));
typedef float flt4v __attribute__((ext_vector_type(4)));

template <int N>
__device__ __forceinline__ void ch_wait(dbl2v *q) {
    asm volatile("s_waitcnt lgkmcnt(%8)"
                 : "+v"(q[0]), "+v"(q[1]), "+v"(q[2]), "+v"(q[3]), "+v"(q[4]), "+v"(q[5]), "+v"(q[6]),
                   "+v"(q[7])
                 : "i"(N));
}

__device__ __forceinline__ void chain_mu_block(uint32_t base, uint32_t mbase, double &mu) {
    dbl2v qa[8], qb[8];
    CH_RD8(qa, base, 0);
#pragma unroll
    for (int g = 0; g < 8; ++g) {
        dbl2v *cur = (g & 1) ? qb : qa;
        dbl2v *nxt = (g & 1) ? qa : qb;
        if (g < 7) {
            switch (g) {   // the offsets must be immediates
            case 0: CH_RD8(nxt, base, 1); break;
            case 1: CH_RD8(nxt, base, 2); break;
            case 2: CH_RD8(nxt, base, 3); break;
            case 3: CH_RD8(nxt, base, 4); break;
            case 4: CH_RD8(nxt, base, 5); break;
            case 5: CH_RD8(nxt, base, 6); break;
            case 6: CH_RD8(nxt, base, 7); break;
            }
            if (g == 0) ch_wait<8>(cur);
            else ch_wait<10>(cur);
        } else {
            ch_wait<2>(cur);
        }
        float mr[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            mr[i] = (float)mu;
            mu = (double)(float)fma(mu, cur[i].x, cur[i].y);
        }
        const flt4v w0 = {mr[0], mr[1], mr[2], mr[3]}, w1 = {mr[4], mr[5], mr[6], mr[7]};
        asm volatile("ds_write_b128 %0, %1 offset:%3\n\tds_write_b128 %0, %2 offset:%4"
                     :
                     : "v"(mbase), "v"(w0), "v"(w1), "i"(32 * g), "i"(32 * g + 16)
                     : "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}


// one ds_read_b128 of step operands at byte offset OFF
template <int OFF>
__device__ __forceinline__ void ch_rd1(dbl2v &q, uint32_t base) {
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=&v"(q) : "v"(base), "i"(OFF) : "memory");
}
template <int N>
__device__ __forceinline__ void ch_wait1(dbl2v &q) {
    asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(q) : "i"(N) : "memory");
}
// step L of 64: wait for its operands, run it, reload the ring entry with step L + 8
template <int L>
__device__ __forceinline__ void ch_step(uint32_t base, uint32_t mbase, double &x, dbl2v *q, float *mr) {
    // LDS ops issued after step L's read: reads L+1..min(L+7, 63) and the mu writes of steps
    // m in [max(L-8, 0), L-1] with m % 4 == 3
    constexpr int RD = (L + 7 < 63 ? L + 7 : 63) - L;
    constexpr int M0 = L - 8 > 0 ? L - 8 : 0;
    constexpr int WR = (L >= 1 ? (L - 1 + 1) / 4 : 0) - (M0 >= 1 ? M0 / 4 : 0);
    constexpr int NW = RD + WR < 15 ? RD + WR : 15;
    ch_wait1<NW>(q[L & 7]);
    mr[L & 3] = (float)x;
    x = (double)(float)fma(x, q[L & 7].x, q[L & 7].y);
    if constexpr (L + 8 < 64) ch_rd1<16 * (L + 8)>(q[L & 7], base);
    if constexpr ((L & 3) == 3) {
        const flt4v w = {mr[0], mr[1], mr[2], mr[3]};
        asm volatile("ds_write_b128 %0, %1 offset:%2" : : "v"(mbase), "v"(w), "i"(4 * (L - 3)) : "memory");
    }
    if constexpr (L < 63) ch_step<L + 1>(base, mbase, x, q, mr);
}
__device__ __forceinline__ void chain_mu_ring(uint32_t base, uint32_t mbase, double &x) {
    dbl2v q[8];
    float mr[4];
    ch_rd1<0>(q[0], base); ch_rd1<16>(q[1], base); ch_rd1<32>(q[2], base); ch_rd1<48>(q[3], base);
    ch_rd1<64>(q[4], base); ch_rd1<80>(q[5], base); ch_rd1<96>(q[6], base); ch_rd1<112>(q[7], base);
    ch_step<0>(base, mbase, x, q, mr);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}


// mode 12: A_k from a global table by scalar loads (8 doubles per s_load_dwordx16), B_k as floats
// from LDS (4 per ds_read_b128); one lgkmcnt(0) wait per 8-step group, next group's loads in flight
typedef int sg16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ void s_ld16(sg16 &o, const double *p) {
    asm volatile("s_load_dwordx16 %0, %1, 0x0" : "=s"(o) : "s"(p) : "memory");
}
template <int OFF>
__device__ __forceinline__ void ds_rd2(flt4v &a, flt4v &b, uint32_t base) {
    asm volatile("ds_read_b128 %0, %2 offset:%3\n\tds_read_b128 %1, %2 offset:%4"
                 : "=&v"(a), "=&v"(b) : "v"(base), "i"(OFF), "i"(OFF + 16) : "memory");
}
__device__ __forceinline__ void wait0(sg16 &a, flt4v &b0, flt4v &b1) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(a), "+v"(b0), "+v"(b1) : : "memory");
}
template <int G>
__device__ __forceinline__ void g12(const double *At, uint32_t bbase, uint32_t mbase, double &x,
                                    sg16 &ac, flt4v &b0c, flt4v &b1c, sg16 &an, flt4v &b0n, flt4v &b1n) {
    wait0(ac, b0c, b1c);
    if constexpr (G < 7) {
        s_ld16(an, At + 8 * (G + 1));
        ds_rd2<32 * (G + 1)>(b0n, b1n, bbase);
    }
    asm volatile("" : "+v"(x));   // pins this group's steps after the next group's loads
    float mr[8];
    const float bf[8] = {b0c.x, b0c.y, b0c.z, b0c.w, b1c.x, b1c.y, b1c.z, b1c.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const double a = __longlong_as_double(((long long)ac[2 * i + 1] << 32) | (unsigned)ac[2 * i]);
        mr[i] = (float)x;
        x = (double)(float)fma(x, a, (double)bf[i]);
    }
    const flt4v w0 = {mr[0], mr[1], mr[2], mr[3]}, w1 = {mr[4], mr[5], mr[6], mr[7]};
    asm volatile("ds_write_b128 %0, %1 offset:%3\n\tds_write_b128 %0, %2 offset:%4"
                 : : "v"(mbase), "v"(w0), "v"(w1), "i"(32 * G), "i"(32 * G + 16) : "memory");
    if constexpr (G < 7) g12<G + 1>(At, bbase, mbase, x, an, b0n, b1n, ac, b0c, b1c);
}
__device__ __forceinline__ void chain_mu_smem(const double *At, uint32_t bbase, uint32_t mbase, double &x) {
    sg16 a0, a1;
    flt4v b00, b01, b10, b11;
    s_ld16(a0, At);
    ds_rd2<0>(b00, b01, bbase);
    g12<0>(At, bbase, mbase, x, a0, b00, b01, a1, b10, b11);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

template <int MODE>
__global__ void k_chain(float *out, unsigned long long *cyc, const double *__restrict__ Atab) {
    __shared__ double2 ab[64];
    __shared__ float bfs[64];
    __shared__ float mus[64];
    const int lane = threadIdx.x;
    double mu = 0.0, sig = 0.0;
    float muv = 0.0f;
    unsigned long long t0 = clock64();
    for (int blk = 0; blk < NBLK; ++blk) {
        const double kd = (double)(blk * 64 + lane + 1);
        const double r = 1.0 / kd;
        const double A = 1.0 - r, Bv = (double)(float)(1.0001 * r);
        if (MODE == 12) {
            bfs[lane] = (float)Bv;
            lds_order();
        } else if (MODE != 2 && ((MODE != 8 && MODE < 9) || MODE == 11 || blk == 0)) {
            ab[lane] = make_double2(A, Bv);
            lds_order();
        }
        if (MODE == 0) {
            if (lane == 0) {
#pragma unroll 4
                for (int l = 0; l < 64; ++l) {
                    const double2 v = ab[l];
                    mus[l] = (float)mu;
                    mu = (double)(float)fma(mu, v.x, v.y);
                }
            }
        } else if (MODE == 1) {
            if (lane == 0) {
                double2 q[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) q[i] = ab[i];
#pragma unroll
                for (int l = 0; l < 64; ++l) {
                    const double2 v = q[l & 7];
                    if (l + 8 < 64) q[l & 7] = ab[l + 8];
                    mus[l] = (float)mu;
                    mu = (double)(float)fma(mu, v.x, v.y);
                }
            }
        } else if (MODE == 2) {
#pragma unroll
            for (int l = 0; l < 64; ++l) {
                const double a = rl64(A, l), b = rl64(Bv, l);
                muv = lane == l ? (float)mu : muv;
                mu = (double)(float)fma(mu, a, b);
            }
            mus[lane] = muv;
        } else if (MODE == 3) {
            if (lane == 0) {
#pragma unroll
                for (int l = 0; l < 64; ++l) {
                    const double2 v = ab[l];
                    mus[l] = (float)mu;
                    mu = (double)(float)fma(mu, v.x, v.y);
                }
            }
        } else if (MODE == 6) {
            constexpr int G = 8;
            if (lane == 0) {
                double2 qa[G], qb[G];
                float mr[64];
#pragma unroll
                for (int i = 0; i < G; ++i) qa[i] = ab[i];
#pragma unroll
                for (int g = 0; g < 64 / G; ++g) {
                    double2 *cur = (g & 1) ? qb : qa;
                    double2 *nxt = (g & 1) ? qa : qb;
                    if (g + 1 < 64 / G) {
#pragma unroll
                        for (int i = 0; i < G; ++i) nxt[i] = ab[(g + 1) * G + i];
                    }
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int i = 0; i < G; ++i) {
                        mr[g * G + i] = (float)mu;
                        mu = (double)(float)fma(mu, cur[i].x, cur[i].y);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    reinterpret_cast<float4 *>(mus)[i] = make_float4(mr[4 * i], mr[4 * i + 1], mr[4 * i + 2], mr[4 * i + 3]);
            }
        } else if (MODE == 12) {
            if (lane == 0)
                chain_mu_smem(Atab + blk * 64, (uint32_t)(uintptr_t)&bfs[0], (uint32_t)(uintptr_t)&mus[0], mu);
        } else if (MODE == 11) {
            if (lane == 0) chain_mu_ring((uint32_t)(uintptr_t)&ab[0], (uint32_t)(uintptr_t)&mus[0], mu);
        } else if (MODE == 9 || MODE == 10) {
            if (lane == 0) {
                double2 q[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) q[i] = ab[i];
                float mr[8];
#pragma unroll
                for (int l = 0; l < 64; ++l) {
                    if (MODE == 10) mr[l & 7] = (float)mu;
                    mu = (double)(float)fma(mu, q[l & 7].x, q[l & 7].y);
                    if (MODE == 10 && (l & 7) == 7)
                        reinterpret_cast<float4 *>(mus)[l >> 3 & 15] = make_float4(mr[0] + mr[1], mr[2] + mr[3], mr[4] + mr[5], mr[6] + mr[7]);
                }
            }
        } else if (MODE == 7 || MODE == 8) {
            if (lane == 0) {
                const uint32_t base = (uint32_t)(uintptr_t)&ab[0];
                const uint32_t mbase = (uint32_t)(uintptr_t)&mus[0];
                chain_mu_block(base, mbase, mu);
            }
        } else {
            if (lane == 0) {
                double2 q[8];
                float mr[64];
#pragma unroll
                for (int i = 0; i < 8; ++i) q[i] = ab[i];
#pragma unroll
                for (int l = 0; l < 64; ++l) {
                    const double2 v = q[l & 7];
                    if (l + 8 < 64) q[l & 7] = ab[l + 8];
                    mr[l] = (float)mu;
                    mu = (double)(float)fma(mu, v.x, v.y);
                    if (MODE == 5) sig = (double)(float)fma(v.x, v.y, sig);
                }
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    reinterpret_cast<float4 *>(mus)[i] = make_float4(mr[4 * i], mr[4 * i + 1], mr[4 * i + 2], mr[4 * i + 3]);
            }
        }
        lds_order();
    }
    unsigned long long t1 = clock64();
    if (lane == 0) {
        out[0] = (float)mu + mus[5] + (float)sig;
        cyc[0] = t1 - t0;
    }
}

static const double *g_atab;
template <int MODE>
void run(const char *name, float *dout, unsigned long long *dcyc) {
    for (int rep = 0; rep < 2; ++rep) {
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        k_chain<MODE><<<1, 64>>>(dout, dcyc, g_atab);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        unsigned long long c = 0;
        float o = 0;
        (void)hipMemcpy(&c, dcyc, 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(&o, dout, 4, hipMemcpyDeviceToHost);
        printf("%-34s rep %d: %.3f ms  %.2f clock64/step  %.3f ns/step  (mu %.9g)\n", name, rep, ms,
               (double)c / (NBLK * 64.0), ms * 1e6 / (NBLK * 64.0), o);
    }
}

int main() {
    float *dout;
    unsigned long long *dcyc;
    (void)hipMalloc(&dout, 16);
    (void)hipMalloc(&dcyc, 8);
    {
        static double h[NBLK * 64];
        for (int k = 0; k < NBLK * 64; ++k) h[k] = 1.0 - 1.0 / (double)(k + 1);
        double *d;
        (void)hipMalloc(&d, sizeof(h));
        (void)hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
        g_atab = d;
    }
    run<0>("0 lane0 unroll4 (round 2)", dout, dcyc);
    run<1>("1 lane0 unroll64 + 8-deep ring", dout, dcyc);
    run<2>("2 all lanes readlane", dout, dcyc);
    run<3>("3 lane0 unroll64 plain", dout, dcyc);
    run<4>("4 ring + mu in registers", dout, dcyc);
    run<5>("5 as 4 + interleaved 2nd chain", dout, dcyc);
    run<6>("6 pinned 2x8 pipeline, mu in regs", dout, dcyc);
    run<7>("7 asm pipeline 2x8, mu 2xb128/group", dout, dcyc);
    run<8>("8 as 7, slot filled once (no fill)", dout, dcyc);
    run<9>("9 VGPR operands, no LDS in loop", dout, dcyc);
    run<10>("10 as 9 + mu capture/writes", dout, dcyc);
    run<11>("11 per-step ring read (asm), 8 deep", dout, dcyc);
    run<12>("12 A by s_load, B float LDS, 8/group", dout, dcyc);
    return 0;
}
