// recon.hip -- TWIX raw k-space reconstruction on gfx950 (Vent_Analysis.process_RAW,
// Vent_Analysis.py:532-540):
//   for k: raw_HPvent[:, :, k] = fftshift(fft2(fftshift(raw_K[:, :, k])))     complex128
//   raw_HPvent = np.transpose(raw_HPvent, (1, 0, 2))[:, ::-1, :]
// The 2-D transform is separable: along each axis v -> fftshift(fft(fftshift(v))).  Two kernels,
// one per axis, each a batch of 1-D lines staged in LDS:
//   k_recon_rows  lines along axis 1 (cols) of one row b0 and a run of slices: the (col, slice) plane
//                 of a row is contiguous, so the block's load and store are dense; out Y[b0][a1][k]
//   k_recon_cols  lines along axis 0 (rows) of a run of consecutive (col, slice) columns: every row
//                 contributes one contiguous run; the store applies the transpose and the row flip,
//                 out[a1][n0 - 1 - a0][k]
// The 1-D FFT is a mixed-radix Stockham autosort (radices 4, 2, 3, 5, 7, then any remaining prime by
// its direct DFT) on double2 in LDS, ping-ponging between two buffers; twiddles come from an exact
// table tw[t] = exp(-2 pi i t / n) (host long double) indexed by integer products mod n.  The
// fftshifts are index maps on the load (x[b] -> slot (b + n/2) mod n) and the store (out[a] =
// Y[(a - n/2) mod n]).  Accuracy: O(eps log n) like numpy's pocketfft (tests: <= 1e-12 of the slice's
// largest value).
#include <cmath>
#include <vector>

#include "vh_internal.h"

#define RC_TPB 256
#define RC_MAXST 40
#define RC_LDS (64 * 1024)       // two line buffers per block, default budget
#define RC_LDS_MAX (160 * 1024)

struct RcPlan {
    int n, h, nst;
    int R[RC_MAXST];
};

static RcPlan rc_plan(int n) {
    RcPlan p{};
    p.n = n;
    p.h = n / 2;
    int m = n;
    auto take = [&](int r) {
        while (m % r == 0 && m > 1) {
            if (p.nst >= RC_MAXST) throw VhError{VH_ERR_ARG, "recon: too many FFT stages"};
            p.R[p.nst++] = r;
            m /= r;
        }
    };
    take(4);
    take(2);
    take(3);
    take(5);
    take(7);
    int r = 11;
    while (m > 1) {   // any remaining prime factor: direct DFT stages
        take(r);
        r += 2;
    }
    return p;
}

// one radix-R pass of a line (Stockham, sub-transform size Ns): butterfly j of n / R
template <int R>
__device__ __forceinline__ void rc_bfly(const double2 *src, double2 *dst, int n, int Ns, int j,
                                        const double2 *tw) {
    const int nr = n / R, js = j % Ns, step = n / (Ns * R);
    double2 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const double2 x = src[j + r * nr];
        const double2 w = tw[(int)(((int64_t)js * r * step) % n)];
        v[r] = make_double2(x.x * w.x - x.y * w.y, x.x * w.y + x.y * w.x);
    }
    const int od = (j / Ns) * Ns * R + js;
#pragma unroll
    for (int q = 0; q < R; ++q) {
        double re = 0.0, im = 0.0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const double2 w = tw[((r * q) % R) * nr];
            re += v[r].x * w.x - v[r].y * w.y;
            im += v[r].x * w.y + v[r].y * w.x;
        }
        dst[od + q * Ns] = make_double2(re, im);
    }
}
// any other (prime) radix: the direct DFT of the R inputs, read from LDS per output
__device__ void rc_bfly_any(const double2 *src, double2 *dst, int n, int R, int Ns, int j,
                            const double2 *tw) {
    const int nr = n / R, js = j % Ns, step = n / (Ns * R);
    const int od = (j / Ns) * Ns * R + js;
    for (int q = 0; q < R; ++q) {
        double re = 0.0, im = 0.0;
        for (int r = 0; r < R; ++r) {
            const double2 x = src[j + r * nr];
            const double2 w1 = tw[(int)(((int64_t)js * r * step) % n)];
            const double2 xw = make_double2(x.x * w1.x - x.y * w1.y, x.x * w1.y + x.y * w1.x);
            const double2 w = tw[((r * q) % R) * nr];
            re += xw.x * w.x - xw.y * w.y;
            im += xw.x * w.y + xw.y * w.x;
        }
        dst[od + q * Ns] = make_double2(re, im);
    }
}

// nl lines of length n, line l at a[l n ..]; returns the buffer holding the transforms
__device__ double2 *rc_fft_lines(double2 *a, double2 *b, int nl, const RcPlan &pl,
                                 const double2 *tw) {
    const int n = pl.n;
    int Ns = 1;
    for (int s = 0; s < pl.nst; ++s) {
        const int R = pl.R[s], nr = n / R, work = nl * nr;
        for (int idx = threadIdx.x; idx < work; idx += RC_TPB) {
            const int l = idx / nr, j = idx - l * nr;
            const double2 *src = a + (size_t)l * n;
            double2 *dst = b + (size_t)l * n;
            switch (R) {
                case 4: rc_bfly<4>(src, dst, n, Ns, j, tw); break;
                case 2: rc_bfly<2>(src, dst, n, Ns, j, tw); break;
                case 3: rc_bfly<3>(src, dst, n, Ns, j, tw); break;
                case 5: rc_bfly<5>(src, dst, n, Ns, j, tw); break;
                case 7: rc_bfly<7>(src, dst, n, Ns, j, tw); break;
                default: rc_bfly_any(src, dst, n, R, Ns, j, tw); break;
            }
        }
        __syncthreads();
        double2 *t = a;
        a = b;
        b = t;
        Ns *= R;
    }
    return a;
}

__device__ __forceinline__ int rc_mod(int v, int n) {
    v %= n;
    return v < 0 ? v + n : v;
}

// lines along axis 1: block (b0, slices [k0, k0 + kc))
__global__ void __launch_bounds__(RC_TPB) k_recon_rows(const double2 *X, double2 *Y, int n0, int n1, int nz,
                                                       int kc, RcPlan pl, const double2 *tw) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double2 *a = reinterpret_cast<double2 *>(smem), *b = a + (size_t)kc * n1;
    const int b0 = blockIdx.x, k0 = blockIdx.y * kc, nk = min(kc, nz - k0);
    const double2 *src = X + (size_t)b0 * n1 * nz;
    for (int e = threadIdx.x; e < n1 * nk; e += RC_TPB) {   // (col, slice) pairs, slice fastest
        const int c = e / nk, k = e - c * nk;
        a[(size_t)k * n1 + rc_mod(c + pl.h, n1)] = src[(size_t)c * nz + k0 + k];   // fftshift
    }
    __syncthreads();
    const double2 *o = rc_fft_lines(a, b, nk, pl, tw);
    double2 *dst = Y + (size_t)b0 * n1 * nz;
    for (int e = threadIdx.x; e < n1 * nk; e += RC_TPB) {
        const int c = e / nk, k = e - c * nk;
        dst[(size_t)c * nz + k0 + k] = o[(size_t)k * n1 + rc_mod(c - pl.h, n1)];   // fftshift
    }
}

// lines along axis 0: block = columns [c0, c0 + cc) of the (col, slice) plane; output transposed
// and flipped: out[a1][n0 - 1 - a0][k]
__global__ void __launch_bounds__(RC_TPB) k_recon_cols(const double2 *Y, double2 *out, int n0, int n1, int nz,
                                                       int cc, RcPlan pl, const double2 *tw) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double2 *a = reinterpret_cast<double2 *>(smem), *b = a + (size_t)cc * n0;
    const int64_t CZ = (int64_t)n1 * nz;
    const int64_t c0 = (int64_t)blockIdx.x * cc;
    const int nc = (int)min<int64_t>(cc, CZ - c0);
    for (int e = threadIdx.x; e < n0 * nc; e += RC_TPB) {   // row-major: each row's run is contiguous
        const int r = e / nc, c = e - r * nc;
        a[(size_t)c * n0 + rc_mod(r + pl.h, n0)] = Y[(size_t)r * CZ + c0 + c];
    }
    __syncthreads();
    const double2 *o = rc_fft_lines(a, b, nc, pl, tw);
    for (int e = threadIdx.x; e < n0 * nc; e += RC_TPB) {
        const int r = e / nc, c = e - r * nc;   // r = a0
        const int64_t col = c0 + c, a1 = col / nz, k = col - a1 * nz;
        out[((size_t)a1 * n0 + (n0 - 1 - r)) * nz + k] = o[(size_t)c * n0 + rc_mod(r - pl.h, n0)];
    }
}

static std::vector<double2> rc_twiddles(int n) {
    std::vector<double2> t(n);
    const long double two_pi = 6.283185307179586476925286766559005768L;
    for (int i = 0; i < n; ++i) {
        const long double ang = two_pi * (long double)i / (long double)n;
        t[i] = make_double2((double)cosl(ang), -(double)sinl(ang));
    }
    return t;
}

// lines of length n per block within the LDS budget (two ping-pong buffers of double2)
static int rc_lines(int n, int want, int *lds) {
    int nl = std::max(1, std::min(want, RC_LDS / (32 * n)));
    const size_t bytes = (size_t)32 * n * nl;
    if (bytes > RC_LDS_MAX) throw VhError{VH_ERR_ARG, "recon: a line longer than 5120 points"};
    *lds = (int)bytes;
    return nl;
}

void vh_recon_run(hipStream_t st, const double2 *d_in, double2 *d_tmp, double2 *d_out, double2 *d_tw0,
                  double2 *d_tw1, int64_t n0, int64_t n1, int64_t nz) {
    const RcPlan p0 = rc_plan((int)n0), p1 = rc_plan((int)n1);
    const std::vector<double2> t0 = rc_twiddles((int)n0), t1 = rc_twiddles((int)n1);
    HIP_TRY(hipMemcpyAsync(d_tw0, t0.data(), sizeof(double2) * n0, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(d_tw1, t1.data(), sizeof(double2) * n1, hipMemcpyHostToDevice, st));
    int lds1 = 0, lds0 = 0;
    const int kc = rc_lines((int)n1, (int)nz, &lds1);
    vh_set_max_lds((const void *)k_recon_rows, RC_LDS_MAX);
    vh_set_max_lds((const void *)k_recon_cols, RC_LDS_MAX);
    k_recon_rows<<<dim3((unsigned)n0, (unsigned)((nz + kc - 1) / kc)), RC_TPB, lds1, st>>>(
        d_in, d_tmp, (int)n0, (int)n1, (int)nz, kc, p1, d_tw1);
    VH_CHECK_LAUNCH();
    const int64_t CZ = n1 * nz;
    const int cc = rc_lines((int)n0, (int)std::min<int64_t>(CZ, 64), &lds0);
    k_recon_cols<<<(unsigned)((CZ + cc - 1) / cc), RC_TPB, lds0, st>>>(d_tmp, d_out, (int)n0, (int)n1,
                                                                       (int)nz, cc, p0, d_tw0);
    VH_CHECK_LAUNCH();
}
