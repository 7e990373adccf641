// Microbenchmark: latency of ITK's float Welford recurrence (N4 convergence measure) run as a
// serial chain on one lane of a wave, inputs staged in LDS.  Prints cycles per step.
//   mu_k  = RN24(fma64(mu, A_k, B_k))      A_k = 1 - 1/k, B_k = RN24(p_k / k)
//   sig_k = RN24(fma64(s_k, C_k, sig))     s_k = RN24((p_k - mu_{k-1})^2), C_k = (k-1)/k
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define N 82000
#define BLK 64

__global__ void k_chain(const double *A, const double *B, const double *Cc, const float *P, int n,
                        int mode, float *out, unsigned long long *cyc) {
    __shared__ double sA[2][BLK], sB[2][BLK], sC[2][BLK];
    __shared__ float sP[2][BLK];
    const int lane = threadIdx.x;
    double mu = 0.0, sig = 0.0;
    unsigned long long t0 = clock64();
    int buf = 0;
    for (int k0 = 0; k0 < n; k0 += BLK) {
        if (k0 + lane < n) {
            sA[buf][lane] = A[k0 + lane];
            sB[buf][lane] = B[k0 + lane];
            sC[buf][lane] = Cc[k0 + lane];
            sP[buf][lane] = P[k0 + lane];
        }
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) {
            const int m = min(BLK, n - k0);
            if (mode == 0) {
#pragma unroll 8
                for (int j = 0; j < m; ++j) mu = (double)(float)fma(mu, sA[buf][j], sB[buf][j]);
            } else {
#pragma unroll 8
                for (int j = 0; j < m; ++j) {
                    const float muf = (float)mu;
                    const float dd = sP[buf][j] - muf;
                    const float s = dd * dd;
                    sig = (double)(float)fma((double)s, sC[buf][j], sig);
                    mu = (double)(float)fma(mu, sA[buf][j], sB[buf][j]);
                }
            }
        }
        buf ^= 1;
    }
    unsigned long long t1 = clock64();
    if (lane == 0) {
        out[0] = (float)mu;
        out[1] = (float)sig;
        cyc[0] = t1 - t0;
    }
}

int main() {
    std::vector<double> A(N), B(N), C(N);
    std::vector<float> P(N);
    for (int k = 1; k <= N; ++k) {
        const float p = 1.0f + 1e-3f * (float)((k * 7919) % 1000 - 500) / 500.0f;
        P[k - 1] = p;
        A[k - 1] = 1.0 - 1.0 / (double)k;
        B[k - 1] = (double)(p / (float)k);
        C[k - 1] = (double)(k - 1) / (double)k;
    }
    double *dA, *dB, *dC;
    float *dP, *dout;
    unsigned long long *dcyc;
    hipMalloc(&dA, 8 * N); hipMalloc(&dB, 8 * N); hipMalloc(&dC, 8 * N); hipMalloc(&dP, 4 * N);
    hipMalloc(&dout, 8); hipMalloc(&dcyc, 8);
    hipMemcpy(dA, A.data(), 8 * N, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), 8 * N, hipMemcpyHostToDevice);
    hipMemcpy(dC, C.data(), 8 * N, hipMemcpyHostToDevice);
    hipMemcpy(dP, P.data(), 4 * N, hipMemcpyHostToDevice);
    for (int mode = 0; mode < 2; ++mode)
        for (int rep = 0; rep < 3; ++rep) {
            hipEvent_t e0, e1;
            hipEventCreate(&e0); hipEventCreate(&e1);
            hipEventRecord(e0);
            k_chain<<<1, 64>>>(dA, dB, dC, dP, N, mode, dout, dcyc);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            unsigned long long cyc = 0;
            float o[2];
            hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost);
            hipMemcpy(o, dout, 8, hipMemcpyDeviceToHost);
            printf("mode %d rep %d: %.3f ms, %.1f cycles/step (clock64), mu %.9g sig %.9g\n", mode, rep,
                   ms, (double)cyc / N, o[0], o[1]);
        }
    return 0;
}
