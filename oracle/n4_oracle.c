/* ORACLE -- test infrastructure only.  CPU restatement of N4 bias-field correction as the
 * reference calls it: sitk.N4BiasFieldCorrectionImageFilter().Execute(image, mask) with every
 * SimpleITK 2.3.1 default (Vent_Analysis.py:316-334; algorithm: SURVEY.md Appendix A).  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * PARITY UNPINNED against SimpleITK: neither SimpleITK nor ITK source is available offline
 * (SURVEY.md §8c), so the algorithm is restated from SURVEY Appendix A and pinned by the build's
 * known-answer tests (tests/test_n4_oracle.py).
 *
 * Two precision modes over one algorithm:
 *
 *  mode 0 "build spec" (n4_oracle): the arithmetic libventhip.so performs, operation for
 *    operation, so the GPU drivers (n4_study.hip, n4.hip) and this file produce bit-identical
 *    U = L0 - B after every iteration.  Every reduction whose order could change a rounding is
 *    either an exact integer sum or follows a fixed, documented order:
 *      S1  L0 = (float)log((double)I) at mask == 1, I > 0; 0 for non-positive masked voxels
 *          (ITK takes log of the whole image and replaces -inf/NaN by 0).
 *      S2  bin range in raster order with ITK's `if (u > max) max = u; else if (u < min) min = u;`.
 *      S3  Parzen histogram: c = (u - min) / slope, i = floor(c), o = c - i; a voxel with
 *          i == bins-1 and o > 0 adds nothing (ITK's else-if); a1 = trunc(o * 2^24),
 *          a0 = 2^24 - a1 are added to bins i, i+1 as integers (exact, order-free).
 *      S4  512-point Wiener deconvolution / E(u) map in double (radix-2 DIT, host twiddles).
 *      S5  B-spline fit (Lee-Wolberg-Shin, single level, cubic), separable and item-ordered:
 *          items are (64-column tile of the (col, slice) plane) x (64-row slot).  Per item and
 *          column, each control row's partial is an fma chain over the item's masked rows in row
 *          order; it is contracted over the tile's slices (fma chain, slice order) and cols (fma
 *          chain, col order); each (item, control point) result enters the lattice numerator as a
 *          128-bit fixed-point integer (trunc(|v| 2^80), two's complement): exact and order-free.
 *          Numerator weights wx^3/sum wx^2 (rows), wy^3, wz^3 with p = r * (1/sum wy^2 * 1/sum wz^2);
 *          denominator weights w^2 with p = 1.  phi = (float)(num / den), lattice += phi.
 *      S6  evaluation: P1 = sum_k wz lat (double), T = (float) sum_j wy P1 (double), B = float
 *          sum_i wx T (4 products, left to right); U = L0 - B.
 *      S7  convergence (conv_mode 0): ITK's float convergence measure over d = B_old - B_new in
 *          raster order, RealType = float throughout -- the counter N too (N += 1.0 is exact up to
 *          2^24 and then frozen) -- with ITK's separate double roundings of every right-hand side
 *          (conv_welford below).  conv_mode 1 (S7x): the exact coefficient of variation from
 *          sum d', sum d'^2 in double, d' = expm1c(d).
 *      S8  level change: exact cubic subdivision (spans doubled per axis), axis by axis.
 *      S9  output: B at every voxel per S6, I / (float)exp((double)B).
 *
 *  mode 1 "itk float" (n4_oracle_itk): a restatement of ITK's own float (RealType) arithmetic,
 *    single-threaded: logf, float histogram summed in raster order, float fit accumulation in
 *    raster order over the 64 tensor weights, float lattice collapse, float Welford convergence,
 *    I / expf(B).  Used only to quantify the distance of the build's precision choices from an
 *    ITK-like float pipeline; never compared bit-for-bit with the GPU.
 *
 * Geometry: numpy (R, C, Z) C-order == ITK raster order (x = slice axis fastest), spacing 1,
 * origin 0 (GetImageFromArray, Vent_Analysis.py:322-327).  Lattices are [i over R][j over C][k over Z].
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int32_t n_levels;
    int32_t max_iters[8];
    float conv_threshold;
    int32_t ncp[3];
    int32_t spline_order;
    int32_t n_bins;
    float wiener_noise;
    float fwhm;
    int32_t conv_mode;   /* 0: ITK float Welford (S7), 1: exact CoV in double (S7x) */
} n4o_params;

#define FFT_P 512
#define TILE 64      /* columns per item (one wave on the GPU) */
#define SLOT 64      /* rows per item */
#define HFIX 16777216.0   /* 2^24: histogram weight unit */

typedef __int128 i128;

static float expf_cr(float x) { return (float)exp((double)x); }

/* S7: expm1 of a float difference of fields */
static float expm1c(float x)
{
    if (fabsf(x) < 0.0625f)
        return x + x * x * (0.5f + x * (0.16666667f + x * (0.041666668f + x * 0.008333334f)));
    return (float)expm1((double)x);
}

/* ---- per-axis B-spline tables (n4.hip vh_axis_tables) --------------------------------------- */
static float bspline_eps(int max_spans)
{
    float eps = 100.0f * FLT_EPSILON;
    while ((float)max_spans == (float)max_spans - eps) eps *= 10.0f;
    return eps;
}

typedef struct {
    int n, ncp;
    int32_t *base;     /* [n] */
    float *w;          /* [n][4] */
    double *isw2;      /* [n] 1 / sum w^2 */
    int32_t *klo, *khi;/* [ncp] first / last index whose support holds control point k */
} axis_t;

static void axis_build(axis_t *a, int n, int ncp, float eps)
{
    a->n = n;
    a->ncp = ncp;
    a->base = malloc(sizeof(int32_t) * n);
    a->w = malloc(sizeof(float) * 4 * n);
    a->isw2 = malloc(sizeof(double) * n);
    a->klo = malloc(sizeof(int32_t) * ncp);
    a->khi = malloc(sizeof(int32_t) * ncp);
    const int spans = ncp - 3;
    const float scale = (float)spans / (float)(n - 1);
    for (int idx = 0; idx < n; ++idx) {
        volatile float pv = (float)idx * scale;
        float p = pv;
        if (fabsf(p - (float)spans) <= eps) p = (float)spans - eps;
        if (p < 0.0f) p = 0.0f;
        const int b = (int)p;
        const float f = p - (float)b;
        const double d = (double)f;
        const double d2 = d * d, d3 = d2 * d;
        const float w0 = (float)((1.0 - d) * (1.0 - d) * (1.0 - d) / 6.0);
        const float w1 = (float)((3.0 * d3 - 6.0 * d2 + 4.0) / 6.0);
        const float w2 = (float)((-3.0 * d3 + 3.0 * d2 + 3.0 * d + 1.0) / 6.0);
        const float w3 = (float)(d3 / 6.0);
        a->base[idx] = b;
        a->w[4 * idx + 0] = w0; a->w[4 * idx + 1] = w1; a->w[4 * idx + 2] = w2; a->w[4 * idx + 3] = w3;
        const double sw2 = (double)w0 * w0 + (double)w1 * w1 + (double)w2 * w2 + (double)w3 * w3;
        a->isw2[idx] = 1.0 / sw2;
    }
    for (int k = 0; k < ncp; ++k) {
        int lo = n, hi = -1;
        for (int idx = 0; idx < n; ++idx)
            if (a->base[idx] <= k && k <= a->base[idx] + 3) {
                if (idx < lo) lo = idx;
                if (idx > hi) hi = idx;
            }
        a->klo[k] = lo;
        a->khi[k] = hi;
    }
}

static void axis_free(axis_t *a)
{
    free(a->base); free(a->w); free(a->isw2); free(a->klo); free(a->khi);
}

/* w(idx, k)^P as double, 0 outside the support (wpow<P> of n4_study.hip) */
static double wpow_at(const axis_t *a, int idx, int k, int P)
{
    const int d = k - a->base[idx];
    if (d < 0 || d > 3) return 0.0;
    const double v = (double)a->w[4 * idx + d];
    return P == 3 ? v * v * v : v * v;
}

/* ---- FFT / E map (S4) --------------------------------------------------------------------- */
typedef struct { double re, im; } cpx;

static void fft_inplace(cpx *x, const cpx *tw, int inverse)
{
    const int P = FFT_P;
    for (int i = 1, j = 0; i < P; ++i) {
        int bit = P >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) { cpx t = x[i]; x[i] = x[j]; x[j] = t; }
    }
    for (int len = 2; len <= P; len <<= 1) {
        const int half = len >> 1, step = P / len;
        for (int s = 0; s < P; s += len)
            for (int j = 0; j < half; ++j) {
                cpx w = tw[j * step];
                if (inverse) w.im = -w.im;
                cpx b = x[s + j + half];
                cpx t = {w.re * b.re - w.im * b.im, w.re * b.im + w.im * b.re};
                cpx a = x[s + j];
                x[s + j].re = a.re + t.re; x[s + j].im = a.im + t.im;
                x[s + j + half].re = a.re - t.re; x[s + j + half].im = a.im - t.im;
            }
    }
}

static void make_twiddles(cpx *tw)
{
    for (int k = 0; k < FFT_P / 2; ++k) {
        double a = 2.0 * M_PI * (double)k / (double)FFT_P;
        tw[k].re = cos(a);
        tw[k].im = -sin(a);
    }
}

/* E(u|v) map of ITK SharpenImage (Appendix A.3 steps 4-8) from the histogram series hv[bins]. */
static void emap(const double *hv, int bins, float binMin, float slope, float fwhm, float noise,
                 const cpx *tw, float *E)
{
    const int P = FFT_P;
    const int off = (P - bins) / 2;
    cpx V[FFT_P], F[FFT_P], U[FFT_P], num[FFT_P], den[FFT_P];
    memset(V, 0, sizeof V);
    memset(F, 0, sizeof F);
    for (int n = 0; n < bins; ++n) V[n + off].re = hv[n];
    fft_inplace(V, tw, 0);
    const float sFWHM = fwhm / slope;
    const float ef = (float)(4.0 * log(2.0) / (double)(sFWHM * sFWHM));
    const float sf = (float)(2.0 * sqrt(log(2.0) / M_PI) / (double)sFWHM);
    F[0].re = (double)sf;
    for (int n = 1; n <= P / 2; ++n) {
        float nf = (float)n;
        double v = (double)(sf * expf_cr(-(nf * nf) * ef));
        F[n].re = v;
        F[P - n].re = v;
    }
    F[P / 2].re = (double)sf * exp(-0.25 * (double)((float)P * (float)P) * (double)ef);
    fft_inplace(F, tw, 0);  /* Ff */
    for (int n = 0; n < P; ++n) {
        const double a = F[n].re, b = F[n].im;
        const double g = a / ((a * a - (-b) * b) + (double)noise);  /* Re(conj(Ff)/(|Ff|^2+noise)) */
        U[n].re = V[n].re * g;
        U[n].im = V[n].im * g;
    }
    fft_inplace(U, tw, 1);
    for (int n = 0; n < P; ++n) {
        U[n].re = U[n].re > 0.0 ? U[n].re : 0.0;
        U[n].im = 0.0;
        const float c = binMin + ((float)n - (float)off) * slope;
        num[n].re = (double)c * U[n].re;
        num[n].im = 0.0;
        den[n] = U[n];
    }
    fft_inplace(num, tw, 0);
    fft_inplace(den, tw, 0);
    for (int n = 0; n < P; ++n) {
        const double a = F[n].re, b = F[n].im;
        cpx x = num[n];
        num[n].re = x.re * a - x.im * b; num[n].im = x.re * b + x.im * a;
        x = den[n];
        den[n].re = x.re * a - x.im * b; den[n].im = x.re * b + x.im * a;
    }
    fft_inplace(num, tw, 1);
    fft_inplace(den, tw, 1);
    for (int n = 0; n < bins; ++n) {
        const double d = den[n + off].re;
        E[n] = d != 0.0 ? (float)(num[n + off].re / d) : 0.0f;
    }
}

/* S3 sharpen value (n4_shared.h sharpen_value) */
static float sharpen(float u, float bmin, float slope, const float *E, int bins)
{
    const float cidx = (u - bmin) / slope;
    const int idx = (cidx >= 0.0f && cidx < (float)bins) ? (int)floorf(cidx) : bins;
    if (idx < bins - 1) return E[idx] + (E[idx + 1] - E[idx]) * (cidx - (float)idx);
    return E[bins - 1];
}

/* ---- lattice subdivision along one axis (S8) ------------------------------------------------ */
static void refine_axis(const float *in, float *out, const int *dims, int axis)
{
    int od[3] = {dims[0], dims[1], dims[2]};
    od[axis] = 2 * dims[axis] - 3;
    for (int a = 0; a < od[0]; ++a)
        for (int b = 0; b < od[1]; ++b)
            for (int c = 0; c < od[2]; ++c) {
                int o[3] = {a, b, c};
                int m = o[axis], j = m >> 1;
                int s0[3] = {a, b, c}, s1[3] = {a, b, c}, s2[3] = {a, b, c};
                s0[axis] = j; s1[axis] = j + 1; s2[axis] = j + 2;
#define IDX(s) (((size_t)(s)[0] * dims[1] + (s)[1]) * dims[2] + (s)[2])
                double v;
                if ((m & 1) == 0) v = ((double)in[IDX(s0)] + (double)in[IDX(s1)]) * 0.5;
                else v = ((double)in[IDX(s0)] + 6.0 * (double)in[IDX(s1)] + (double)in[IDX(s2)]) * 0.125;
#undef IDX
                out[((size_t)a * od[1] + b) * od[2] + c] = (float)v;
            }
}

static void refine(float *lat, float *tmp, float *tmp2, int *ncp)
{
    int d0[3] = {ncp[0], ncp[1], ncp[2]};
    refine_axis(lat, tmp, d0, 0);
    int d1[3] = {2 * ncp[0] - 3, ncp[1], ncp[2]};
    refine_axis(tmp, tmp2, d1, 1);
    int d2[3] = {2 * ncp[0] - 3, 2 * ncp[1] - 3, ncp[2]};
    refine_axis(tmp2, lat, d2, 2);
    ncp[0] = 2 * ncp[0] - 3; ncp[1] = 2 * ncp[1] - 3; ncp[2] = 2 * ncp[2] - 3;
}

/* ---- 128-bit fixed point (n4_study.hip fix128_add / fix128_get) ---------------------------- */
static i128 fix128(double v)
{
    const double s = fabs(v) * 65536.0;
    const double fh = floor(s);
    const uint64_t h = (uint64_t)fh;
    const double r = s - fh;
    const uint64_t l = (uint64_t)(r * 18446744073709551616.0);
    const i128 m = (i128)(((unsigned __int128)h << 64) | l);
    return v < 0.0 ? -m : m;
}

static double fix128_get(i128 s)
{
    const unsigned __int128 u = (unsigned __int128)s;
    const uint64_t lo = (uint64_t)u;
    const int64_t hi = (int64_t)(uint64_t)(u >> 64);
    return (double)hi * (1.0 / 65536.0) + (double)lo * 8.271806125530277e-25;
}

/* ---- S5: item-ordered separable fit ---------------------------------------------------------
 * P = 3: numerator, p(x, c) = (double)r * isyz(c), row weights WX = (wx^3) * isw2x
 * P = 2: denominator, p = 1, row weights WX = wx^2
 * acc[] += fix128 of every (item, control point) contribution. */
typedef struct {
    int64_t R, C, Z, CZ;
    const uint8_t *mask;
    const axis_t *ax, *ay, *az;
} geom_t;

static void fit_items(const geom_t *g, int P, const float *rval, i128 *acc)
{
    const int64_t R = g->R, Z = g->Z, CZ = g->CZ;
    const axis_t *ax = g->ax, *ay = g->ay, *az = g->az;
    const int ncx = ax->ncp, ncy = ay->ncp, ncz = az->ncp;
    double *Q = malloc(sizeof(double) * (size_t)ncx * TILE);
    double *S = malloc(sizeof(double) * (size_t)ncx * (size_t)(Z + 2 * TILE) * ncz);
    double *WX = malloc(sizeof(double) * 4 * R);
    for (int64_t x = 0; x < R; ++x)
        for (int a = 0; a < 4; ++a) {
            const double v = (double)ax->w[4 * x + a];
            WX[4 * x + a] = P == 3 ? (v * v * v) * ax->isw2[x] : v * v;
        }
    const int64_t ntiles = (CZ + TILE - 1) / TILE, nslots = (R + SLOT - 1) / SLOT;
    for (int64_t t = 0; t < ntiles; ++t) {
        const int64_t c0 = t * TILE, c1 = (c0 + TILE < CZ ? c0 + TILE : CZ) - 1;
        const int y0 = (int)(c0 / Z), y1 = (int)(c1 / Z), z0 = (int)(c0 % Z), z1 = (int)(c1 % Z);
        const int ny = y1 - y0 + 1;
        const int klo = az->base[y0 == y1 ? z0 : 0];
        const int KT = az->base[y0 == y1 ? z1 : Z - 1] + 4 - klo;
        const int jlo = ay->base[y0], JT = ay->base[y1] + 4 - jlo;
        for (int64_t s = 0; s < nslots; ++s) {
            const int64_t x0 = s * SLOT, x1 = (x0 + SLOT < R ? x0 + SLOT : R) - 1;
            int64_t xs = -1, xe = -1;
            for (int64_t x = x0; x <= x1; ++x)
                for (int64_t c = c0; c <= c1; ++c)
                    if (g->mask[x * CZ + c] == 1) {
                        if (xs < 0) xs = x;
                        xe = x;
                        break;
                    }
            if (xs < 0) continue;
            const int i0 = ax->base[xs], i1 = ax->base[xe] + 3;
            memset(Q, 0, sizeof(double) * (size_t)ncx * TILE);
            for (int64_t c = c0; c <= c1; ++c) {
                const int l = (int)(c - c0);
                const int y = (int)(c / Z), z = (int)(c % Z);
                const double isyz = ay->isw2[y] * az->isw2[z];
                for (int64_t x = xs; x <= xe; ++x) {
                    const int64_t v = x * CZ + c;
                    if (g->mask[v] != 1) continue;
                    const double p = P == 3 ? (double)rval[v] * isyz : 1.0;
                    const int bx = ax->base[x];
                    for (int a = 0; a < 4; ++a)
                        Q[(size_t)(bx + a) * TILE + l] = fma(WX[4 * x + a], p, Q[(size_t)(bx + a) * TILE + l]);
                }
            }
            for (int i = i0; i <= i1; ++i) {
                /* stage 1: S[yy][k] over the tile's slices of col y0 + yy */
                for (int yy = 0; yy < ny; ++yy) {
                    const int yv = y0 + yy;
                    const int zlo = yv == y0 ? z0 : 0, zhi = yv == y1 ? z1 : (int)Z - 1;
                    for (int kk = 0; kk < KT; ++kk) {
                        const int k = klo + kk;
                        const int zs = zlo > az->klo[k] ? zlo : az->klo[k];
                        const int ze = zhi < az->khi[k] ? zhi : az->khi[k];
                        double o = 0.0;
                        for (int z = zs; z <= ze; ++z)
                            o = fma(wpow_at(az, z, k, P), Q[(size_t)i * TILE + (yv * Z - c0) + z], o);
                        S[(size_t)yy * KT + kk] = o;
                    }
                }
                /* stage 2: over the tile's cols, into the fixed-point lattice */
                for (int jj = 0; jj < JT; ++jj) {
                    const int j = jlo + jj;
                    for (int kk = 0; kk < KT; ++kk) {
                        const int k = klo + kk;
                        double a = 0.0;
                        for (int yy = 0; yy < ny; ++yy) {
                            const int d = j - ay->base[y0 + yy];
                            if (d < 0 || d > 3) continue;
                            a = fma(wpow_at(ay, y0 + yy, j, P), S[(size_t)yy * KT + kk], a);
                        }
                        if (a != 0.0) acc[((size_t)i * ncy + j) * ncz + k] += fix128(a);
                    }
                }
            }
        }
    }
    free(Q); free(S); free(WX);
}

/* ---- S6 / S9: separable evaluation ---------------------------------------------------------- */
/* P1[i][j][z] for the current lattice */
static void eval_P1(const float *lat, const axis_t *az, int ncx, int ncy, int64_t Z, double *P1)
{
    const int ncz = az->ncp;
    for (int ij = 0; ij < ncx * ncy; ++ij)
        for (int64_t z = 0; z < Z; ++z) {
            const float *w = az->w + 4 * z;
            const float *l = lat + (size_t)ij * ncz + az->base[z];
            P1[(size_t)ij * Z + z] = (double)w[0] * (double)l[0] + (double)w[1] * (double)l[1] +
                                     (double)w[2] * (double)l[2] + (double)w[3] * (double)l[3];
        }
}

/* T[col][i] for every column */
static void eval_T(const double *P1, const axis_t *ay, int ncx, int64_t C, int64_t Z, float *T)
{
    const int ncy = ay->ncp;
    for (int64_t y = 0; y < C; ++y) {
        const float *w = ay->w + 4 * y;
        const int by = ay->base[y];
        for (int64_t z = 0; z < Z; ++z)
            for (int i = 0; i < ncx; ++i) {
                const double *r = P1 + ((size_t)i * ncy + by) * Z + z;
                T[((size_t)y * Z + z) * ncx + i] =
                    (float)((double)w[0] * r[0] + (double)w[1] * r[Z] + (double)w[2] * r[2 * Z] +
                            (double)w[3] * r[3 * Z]);
            }
    }
}

static inline float eval_B(const float *T, const axis_t *ax, int ncx, int64_t x, int64_t col)
{
    const float *w = ax->w + 4 * x;
    const float *t = T + (size_t)col * ncx + ax->base[x];
    return ((w[0] * t[0] + w[1] * t[1]) + w[2] * t[2]) + w[3] * t[3];
}

/* ---- S7: convergence of one iteration from d = B_old - B_new at the masked voxels in raster order.
 * ITK (itkN4BiasFieldCorrectionImageFilter CalculateConvergenceMeasurement, RealType = float):
 *   RealType pixel = std::exp(d); N += 1.0;
 *   if (N > 1.0) sigma = sigma + sqr(pixel - mu) * (N - 1.0) / N;
 *   mu = mu * (1.0 - 1.0 / N) + pixel / N;
 *   sigma = std::sqrt(sigma / (N - 1.0)); return sigma / mu;
 * with float state (mu, sigma, N) and the double literals promoting each right-hand side to double,
 * evaluated left to right with a rounding after every operation:
 *   N   <- (float)(N + 1.0)                       exact below 2^24; 2^24 + 1 rounds back to 2^24
 *   sig <- (float)(sig + RN(RN(sqr(p - mu) * (N - 1)) / N))   (the product is exact: 24 x 24 bits)
 *   mu  <- (float)(RN(mu * RN(1 - RN(1 / N))) + (double)(p / N))   (p / N a float division)
 * p = (float)exp((double)d) (correctly rounded).  The state is a serial float recurrence (the float
 * running mean drifts): it must be evaluated in raster order.  This is exactly the S7 of the ITK-float
 * restatement n4_oracle_itk below (which takes expf instead). */
static float conv_welford(const float *d, int64_t n)
{
    float mu = 0.0f, sig = 0.0f, N = 0.0f;
    for (int64_t k = 1; k <= n; ++k) {
        const float p = expf_cr(d[k - 1]);
        N = (float)((double)N + 1.0);
        const double Nd = (double)N;
        if (Nd > 1.0) {
            const float q = p - mu;
            sig = (float)((double)sig + ((double)(q * q) * (Nd - 1.0)) / Nd);
        }
        mu = (float)((double)mu * (1.0 - 1.0 / Nd) + (double)(p / N));
    }
    const float s = (float)sqrt((double)sig / ((double)N - 1.0));
    return s / mu;
}

/* S7 alone (tests/test_n4_oracle.py) */
float n4o_conv_welford(const float *d, int64_t n) { return conv_welford(d, n); }

/* (1 - 2^-24)^m rounded down by 2^-40 (n4_shared.h pc_accum_factor, the same expression) */
static double pc_accum_factor(double m) { return exp(m * log1p(-0x1p-24)) * (1.0 - 0x1p-40); }

/* The lower bound of the float sig that PC's certified decision uses (vent_analysis_amd/csrc/
 * n4_shared.h pcw_run, after stage 0): nb blocks of consecutive steps, block j's float sum
 * B_j = fma(q, q, B_j) of q = (float)(p - mu) along the exact mu trajectory, weighted by
 * 1 - 1/min(k0_j, 2^24), summed in double in block order, times (1 - 2^-24)^(n + L + 8)
 * (pc_accum_factor: the float accumulation of n positive terms keeps at least that fraction of
 * their exact sum; round 6, before: the linear 1 - (n + L + 8) 2^-24, negative past 2^24).  Returns the
 * true float sig of the recurrence in *sig and the bound in *lo (tests/test_n4_oracle.py checks
 * lo <= sig on oracle d sequences). */
void n4o_pc_sig_bound(const float *d, int64_t n, int nb, double *lo, float *sig_out, float *mu_out)
{
    float mu = 0.0f, sig = 0.0f, N = 0.0f;
    const int64_t L = n / nb, rem = n % nb;
    double tot = 0.0;
    int64_t k = 1;
    for (int j = 0; j < nb; ++j) {
        const int64_t len = L + (j < rem ? 1 : 0), k0 = k;
        float B = 0.0f;
        for (int64_t s = 0; s < len; ++s, ++k) {
            const float p = expf_cr(d[k - 1]);
            N = (float)((double)N + 1.0);
            const double Nd = (double)N;
            if (Nd > 1.0) {
                const float q = p - mu;
                B = fmaf(q, q, B);
                sig = (float)((double)sig + ((double)(q * q) * (Nd - 1.0)) / Nd);
            }
            mu = (float)((double)mu * (1.0 - 1.0 / Nd) + (double)(p / N));
        }
        if (k0 > 1) tot += (double)B * (1.0 - 1.0 / fmin((double)k0, 16777216.0));
    }
    *lo = tot * pc_accum_factor((double)n + (double)L + 8.0);
    *sig_out = sig;
    *mu_out = mu;
}

/* The early certified decision (n4_shared.h pcw_run, PC_PRE): the same bound from the exact running
 * mean, block by block as the GPU forms it (nb blocks, float reciprocals, the same margins).  Returns
 * lo (a lower bound of ITK's float sig), muhi (an upper bound of its float mean) and ok (every p in
 * (0.5, 1.9), where the bound holds); *dmax_out = max over k of |mu_k - m_k| / D_k, the float mean's
 * observed distance from the exact one over the bound D_k = 2^-25 M (k + 3) (1 + 2^-20) (must be
 * <= 1), M = max p (1 + 2^-24 (n + 3)) (1 + 2^-20) >= every |mu_i|, |p_i| (the code's cD (k + 3)).
 * Also ITK's float (mu, sig) for the check.  Test infrastructure (tests/test_n4_oracle.py). */
void n4o_pc_pre_bound(const float *d, int64_t n, int nb, double *lo_out, float *muhi_out, int *ok_out,
                      double *dmax_out, float *sig_out, float *mu_out)
{
    const int64_t L = n / nb, rem = n % nb;
    float *p = (float *)malloc(sizeof(float) * (size_t)(n > 0 ? n : 1));
    int ok = 1;
    float pmax = 0.0f;
    for (int64_t k = 0; k < n; ++k) {
        p[k] = expf_cr(d[k]);
        if (!(p[k] < 1.9f && p[k] > 0.5f)) ok = 0;
        if (p[k] > pmax) pmax = p[k];
    }
    const double Mx = (double)pmax * (1.0 + 0x1p-24 * ((double)n + 3.0)) * (1.0 + 0x1p-20);
    const double cD = 0x1p-25 * Mx * (1.0 + 0x1p-20);
    /* ITK's float recurrence and the observed drift from the exact running mean */
    float mu = 0.0f, sig = 0.0f, N = 0.0f;
    double P = 0.0, dmax = 0.0;
    for (int64_t k = 1; k <= n; ++k) {
        const float pk = p[k - 1];
        N = (float)((double)N + 1.0);
        const double Nd = (double)N;
        if (Nd > 1.0) {
            const float q = pk - mu;
            sig = (float)((double)sig + ((double)(q * q) * (Nd - 1.0)) / Nd);
        }
        mu = (float)((double)mu * (1.0 - 1.0 / Nd) + (double)(pk / N));
        P += (double)pk - 1.0;
        const double mk = 1.0 + P / (double)k;
        const double r = fabs((double)mu - mk) / (cD * ((double)k + 3.0));
        if (r > dmax) dmax = r;
    }
    /* the GPU's bound: blocks of L (+1) steps, exact prefix of (p - 1), float reciprocals */
    double tot = 0.0, Pk = 0.0;
    int64_t k = 1;
    for (int j = 0; j < nb; ++j) {
        const int64_t len = L + (j < rem ? 1 : 0), k0 = k;
        double acc = 0.0;
        for (int64_t s = 0; s < len; ++s, ++k) {
            const double pd = (double)p[k - 1];
            if (k >= 2) {
                const double r = (double)(1.0f / (float)(k - 1));
                const double m = fma(Pk, r, 1.0);
                const double eps = fabs(m - 1.0) * 0x1p-21 + 0x1p-50;
                const double a = fabs(pd - m) - cD * (double)(k + 2) - eps;
                if (a > 0.0) acc = fma(a, a, acc);
            }
            Pk += pd - 1.0;
        }
        tot += acc * (1.0 - 1.0 / fmax((double)k0, 2.0));
    }
    *lo_out = tot * pc_accum_factor((double)n + 8.0);
    const double mn = 1.0 + Pk / (double)n;
    const double hi = mn + cD * ((double)n + 3.0) + fabs(mn - 1.0) * 0x1p-50 + 0x1p-50;
    float f = (float)hi;
    if ((double)f < hi) f = nextafterf(f, INFINITY);
    *muhi_out = f;
    *ok_out = ok;
    *dmax_out = dmax;
    *sig_out = sig;
    *mu_out = mu;
    free(p);
}

/* S7x (conv_mode 1): the coefficient of variation ITK intends, evaluated exactly enough that
 * order does not matter: d' = expm1c(d), CoV from sum d', sum d'^2 in double */
static double conv_exact(const float *d, int64_t n)
{
    double sd = 0.0, sd2 = 0.0;
    for (int64_t k = 0; k < n; ++k) {
        const double e = (double)expm1c(d[k]);
        sd += e;
        sd2 = fma(e, e, sd2);
    }
    const double N = (double)n;
    const double mu = 1.0 + sd / N;
    double var = (sd2 - sd * sd / N) / (N - 1.0);
    if (var < 0.0) var = 0.0;
    return sqrt(var) / mu;
}

/* ---- driver: mode 0 (build spec) ------------------------------------------------------------ */
int n4_oracle(const float *I, const uint8_t *mask, int64_t R, int64_t C, int64_t Z,
              const n4o_params *prm, float *out, int32_t *iters_out, float *conv_out)
{
    if (prm->spline_order != 3 || prm->n_levels < 1 || prm->n_levels > 8 || prm->n_bins < 2 ||
        prm->n_bins > FFT_P / 2 || R < 2 || C < 2 || Z < 2)
        return 1;
    const int64_t V = R * C * Z, CZ = C * Z;
    const int bins = prm->n_bins;
    float *L0 = calloc((size_t)V, sizeof(float));
    float *B = calloc((size_t)V, sizeof(float));
    float *rv = calloc((size_t)V, sizeof(float));
    float *dr = calloc((size_t)V, sizeof(float));
    int ncp[3] = {prm->ncp[0], prm->ncp[1], prm->ncp[2]};
    int mx = ncp[0] > ncp[1] ? ncp[0] : ncp[1];
    mx = mx > ncp[2] ? mx : ncp[2];
    const int maxcp = 3 + (mx - 3) * (1 << (prm->n_levels - 1));
    const size_t latmax = (size_t)maxcp * maxcp * maxcp;
    float *lat = calloc(latmax, sizeof(float));
    float *tmp = calloc(latmax, sizeof(float));
    float *tmp2 = calloc(latmax, sizeof(float));
    i128 *num = calloc(latmax, sizeof(i128));
    i128 *denf = calloc(latmax, sizeof(i128));
    double *P1 = calloc((size_t)maxcp * maxcp * Z, sizeof(double));
    float *T = calloc((size_t)CZ * maxcp, sizeof(float));
    uint64_t *H = malloc(sizeof(uint64_t) * bins);
    double *hv = malloc(sizeof(double) * bins);
    float *E = malloc(sizeof(float) * bins);
    cpx tw[FFT_P / 2];
    make_twiddles(tw);
    axis_t ax = {0}, ay = {0}, az = {0};
    int have_axes = 0;
    int64_t nmask = 0;
    for (int64_t v = 0; v < V; ++v)
        if (mask[v] == 1) {
            L0[v] = I[v] > 0.0f ? (float)log((double)I[v]) : 0.0f;
            ++nmask;
        }
    int rc = 0;
    if (nmask < 2) { rc = 3; goto done; }

    for (int level = 0; level < prm->n_levels; ++level) {
        if (have_axes) { axis_free(&ax); axis_free(&ay); axis_free(&az); }
        int ms = ncp[0] > ncp[1] ? ncp[0] : ncp[1];
        ms = ms > ncp[2] ? ms : ncp[2];
        const float eps = bspline_eps(ms - 3);
        axis_build(&ax, (int)R, ncp[0], eps);
        axis_build(&ay, (int)C, ncp[1], eps);
        axis_build(&az, (int)Z, ncp[2], eps);
        have_axes = 1;
        const geom_t g = {R, C, Z, CZ, mask, &ax, &ay, &az};
        const size_t nl = (size_t)ncp[0] * ncp[1] * ncp[2];
        memset(denf, 0, nl * sizeof(i128));
        fit_items(&g, 2, NULL, denf);
        int it = 0;
        double conv = INFINITY;
        while (it++ < prm->max_iters[level] && conv > (double)prm->conv_threshold) {
            /* --- S2 bin range (raster order, ITK's else-if) --- */
            float bmax = -FLT_MAX, bmin = FLT_MAX;
            for (int64_t v = 0; v < V; ++v) {
                if (mask[v] != 1) continue;
                const float u = L0[v] - B[v];
                if (u > bmax) bmax = u;
                else if (u < bmin) bmin = u;
            }
            const float slope = (bmax - bmin) / (float)(bins - 1);
            /* --- S3 Parzen histogram --- */
            memset(H, 0, sizeof(uint64_t) * bins);
            for (int64_t v = 0; v < V; ++v) {
                if (mask[v] != 1) continue;
                const float u = L0[v] - B[v];
                const float cidx = (u - bmin) / slope;
                if (!(cidx >= 0.0f) || !(cidx < (float)bins)) continue;
                const int idx = (int)floorf(cidx);
                const float o = cidx - (float)idx;
                if (idx == bins - 1 && o > 0.0f) continue;
                const uint64_t a1 = (uint64_t)(uint32_t)(o * 16777216.0f);
                H[idx] += (uint64_t)16777216 - a1;
                if (a1) H[idx + 1] += a1;
            }
            for (int n = 0; n < bins; ++n) hv[n] = (double)H[n] * (1.0 / HFIX);
            emap(hv, bins, bmin, slope, prm->fwhm, prm->wiener_noise, tw, E);
            /* --- S5 sharpen, residual, fit --- */
            for (int64_t v = 0; v < V; ++v) {
                if (mask[v] != 1) continue;
                const float u = L0[v] - B[v];
                rv[v] = u - sharpen(u, bmin, slope, E, bins);
            }
            memset(num, 0, nl * sizeof(i128));
            fit_items(&g, 3, rv, num);
            for (size_t c = 0; c < nl; ++c) {
                const double d = fix128_get(denf[c]);
                const float phi = d != 0.0 ? (float)(fix128_get(num[c]) / d) : 0.0f;
                lat[c] = lat[c] + phi;
            }
            /* --- S6 evaluate at masked voxels, S7 convergence --- */
            eval_P1(lat, &az, ncp[0], ncp[1], Z, P1);
            eval_T(P1, &ay, ncp[0], C, Z, T);
            int64_t k = 0;
            for (int64_t x = 0; x < R; ++x)
                for (int64_t col = 0; col < CZ; ++col) {
                    const int64_t v = x * CZ + col;
                    if (mask[v] != 1) continue;
                    const float bn = eval_B(T, &ax, ncp[0], x, col);
                    dr[k++] = B[v] - bn;
                    B[v] = bn;
                }
            {   /* dev hook: append each iteration's raster-ordered d to $N4_DUMP_D (scripts/dev) */
                const char *dump = getenv("N4_DUMP_D");
                if (dump) {
                    FILE *f = fopen(dump, "ab");
                    if (f) { fwrite(&nmask, sizeof nmask, 1, f); fwrite(dr, sizeof(float), (size_t)nmask, f); fclose(f); }
                }
            }
            conv = prm->conv_mode == 1 ? conv_exact(dr, nmask) : (double)conv_welford(dr, nmask);
        }
        iters_out[level] = it - 1;
        if (conv_out) conv_out[level] = (float)conv;
        if (level < prm->n_levels - 1) refine(lat, tmp, tmp2, ncp);
    }
    /* --- S9 final field at every voxel (the last level's tables and lattice), output --- */
    eval_P1(lat, &az, ncp[0], ncp[1], Z, P1);
    eval_T(P1, &ay, ncp[0], C, Z, T);
    for (int64_t x = 0; x < R; ++x)
        for (int64_t col = 0; col < CZ; ++col) {
            const int64_t v = x * CZ + col;
            out[v] = I[v] / expf_cr(eval_B(T, &ax, ncp[0], x, col));
        }
done:
    if (have_axes) { axis_free(&ax); axis_free(&ay); axis_free(&az); }
    free(L0); free(B); free(rv); free(dr); free(lat); free(tmp); free(tmp2); free(num); free(denf);
    free(P1); free(T); free(H); free(hv); free(E);
    return rc;
}

/* ---- driver: mode 1 (ITK float arithmetic, raster order, one thread) ------------------------ */
/* lattice collapse in float along x (rows) first, then y, then z -- ITK's
 * BSplineControlPointImageFilter collapses from the last image dimension (numpy axis 0) down */
static float itk_eval(const float *lat, const axis_t *ax, const axis_t *ay, const axis_t *az,
                      int64_t x, int64_t y, int64_t z)
{
    const int ncy = ay->ncp, ncz = az->ncp;
    float cy[4][4];
    for (int b = 0; b < 4; ++b)
        for (int c = 0; c < 4; ++c) {
            float s = 0.0f;
            for (int a = 0; a < 4; ++a)
                s += ax->w[4 * x + a] * lat[((size_t)(ax->base[x] + a) * ncy + ay->base[y] + b) * ncz + az->base[z] + c];
            cy[b][c] = s;
        }
    float cz[4];
    for (int c = 0; c < 4; ++c) {
        float s = 0.0f;
        for (int b = 0; b < 4; ++b) s += ay->w[4 * y + b] * cy[b][c];
        cz[c] = s;
    }
    float s = 0.0f;
    for (int c = 0; c < 4; ++c) s += az->w[4 * z + c] * cz[c];
    return s;
}

/* spec: ablation mask -- bit k replaces ITK's float form of stage Sk by the build spec's (S1 log,
 * S3 histogram, S5 fit, S6 evaluation, S7 exp, S9 output), so scripts/n4_itk_distance.py can tell
 * which stage puts the spec where it is relative to ITK's float arithmetic (0 = pure ITK-float). */
#define ABL(k) ((spec >> (k)) & 1)
int n4_oracle_itk(const float *I, const uint8_t *mask, int64_t R, int64_t C, int64_t Z,
                  const n4o_params *prm, int nonpos_raw, int nthreads, int spec, float *out,
                  int32_t *iters_out, float *conv_out)
{
    /* nthreads > 1: ITK's BSplineScatteredDataPointSetToImageFilter splits the points into
     * contiguous ranges, one float delta/omega lattice per thread, summed in thread order */
    if (nthreads < 1) nthreads = 1;
    if (prm->spline_order != 3 || prm->n_levels < 1 || prm->n_levels > 8 || prm->n_bins < 2 ||
        prm->n_bins > FFT_P / 2 || R < 2 || C < 2 || Z < 2)
        return 1;
    const int64_t V = R * C * Z, CZ = C * Z;
    const int bins = prm->n_bins;
    float *L0 = calloc((size_t)V, sizeof(float));
    float *B = calloc((size_t)V, sizeof(float));
    float *rv = calloc((size_t)V, sizeof(float));
    int ncp[3] = {prm->ncp[0], prm->ncp[1], prm->ncp[2]};
    int mx = ncp[0] > ncp[1] ? ncp[0] : ncp[1];
    mx = mx > ncp[2] ? mx : ncp[2];
    const int maxcp = 3 + (mx - 3) * (1 << (prm->n_levels - 1));
    const size_t latmax = (size_t)maxcp * maxcp * maxcp;
    float *lat = calloc(latmax, sizeof(float));
    float *tmp = calloc(latmax, sizeof(float));
    float *tmp2 = calloc(latmax, sizeof(float));
    float *delta = calloc(latmax * (size_t)(nthreads < 1 ? 1 : nthreads), sizeof(float));
    float *omega = calloc(latmax * (size_t)(nthreads < 1 ? 1 : nthreads), sizeof(float));
    i128 *num = calloc(latmax, sizeof(i128));
    i128 *denf = calloc(latmax, sizeof(i128));
    double *P1 = calloc((size_t)maxcp * maxcp * Z, sizeof(double));
    float *T = calloc((size_t)CZ * maxcp, sizeof(float));
    float *H = malloc(sizeof(float) * bins);
    uint64_t *Hi = malloc(sizeof(uint64_t) * bins);
    double *hv = malloc(sizeof(double) * bins);
    float *E = malloc(sizeof(float) * bins);
    cpx tw[FFT_P / 2];
    make_twiddles(tw);
    axis_t ax = {0}, ay = {0}, az = {0};
    int have_axes = 0;
    int64_t nmask = 0;
    for (int64_t v = 0; v < V; ++v)
        if (mask[v] == 1) {
            L0[v] = I[v] > 0.0f ? (ABL(1) ? (float)log((double)I[v]) : logf(I[v]))
                                : (nonpos_raw ? I[v] : 0.0f);
            ++nmask;
        }
    int rc = 0;
    if (nmask < 2) { rc = 3; goto done; }
    for (int level = 0; level < prm->n_levels; ++level) {
        if (have_axes) { axis_free(&ax); axis_free(&ay); axis_free(&az); }
        int ms = ncp[0] > ncp[1] ? ncp[0] : ncp[1];
        ms = ms > ncp[2] ? ms : ncp[2];
        const float eps = bspline_eps(ms - 3);
        axis_build(&ax, (int)R, ncp[0], eps);
        axis_build(&ay, (int)C, ncp[1], eps);
        axis_build(&az, (int)Z, ncp[2], eps);
        have_axes = 1;
        const size_t nl = (size_t)ncp[0] * ncp[1] * ncp[2];
        const geom_t g = {R, C, Z, CZ, mask, &ax, &ay, &az};
        if (ABL(5)) {
            memset(denf, 0, nl * sizeof(i128));
            fit_items(&g, 2, NULL, denf);
        }
        int it = 0;
        float conv = INFINITY;
        while (it++ < prm->max_iters[level] && conv > prm->conv_threshold) {
            float bmax = -FLT_MAX, bmin = FLT_MAX;
            for (int64_t v = 0; v < V; ++v) {
                if (mask[v] != 1) continue;
                const float u = L0[v] - B[v];
                if (u > bmax) bmax = u;
                else if (u < bmin) bmin = u;
            }
            const float slope = (bmax - bmin) / (float)(bins - 1);
            if (ABL(3)) {   /* S3 spec: exact packed integer weights */
                memset(Hi, 0, sizeof(uint64_t) * bins);
                for (int64_t v = 0; v < V; ++v) {
                    if (mask[v] != 1) continue;
                    const float cidx = ((L0[v] - B[v]) - bmin) / slope;
                    if (!(cidx >= 0.0f) || !(cidx < (float)bins)) continue;
                    const int idx = (int)floorf(cidx);
                    const float o = cidx - (float)idx;
                    if (idx == bins - 1 && o > 0.0f) continue;
                    const uint64_t a1 = (uint64_t)(uint32_t)(o * 16777216.0f);
                    Hi[idx] += (uint64_t)16777216 - a1;
                    if (a1) Hi[idx + 1] += a1;
                }
                for (int n = 0; n < bins; ++n) hv[n] = (double)Hi[n] * (1.0 / HFIX);
            } else {
                for (int n = 0; n < bins; ++n) H[n] = 0.0f;
                for (int64_t v = 0; v < V; ++v) {
                    if (mask[v] != 1) continue;
                    const float cidx = ((L0[v] - B[v]) - bmin) / slope;
                    const int idx = (int)floorf(cidx);
                    const float o = cidx - (float)idx;
                    if (o == 0.0f) {
                        if (idx >= 0 && idx < bins) H[idx] += 1.0f;
                    } else if (idx >= 0 && idx < bins - 1) {
                        H[idx] += 1.0f - o;
                        H[idx + 1] += o;
                    }
                }
                for (int n = 0; n < bins; ++n) hv[n] = (double)H[n];
            }
            emap(hv, bins, bmin, slope, prm->fwhm, prm->wiener_noise, tw, E);
            if (ABL(5)) {   /* S5 spec: item-ordered separable fit, fixed point */
                for (int64_t v = 0; v < V; ++v) {
                    if (mask[v] != 1) continue;
                    const float u = L0[v] - B[v];
                    rv[v] = u - sharpen(u, bmin, slope, E, bins);
                }
                memset(num, 0, nl * sizeof(i128));
                fit_items(&g, 3, rv, num);
                for (size_t c = 0; c < nl; ++c) {
                    const double d = fix128_get(denf[c]);
                    lat[c] += d != 0.0 ? (float)(fix128_get(num[c]) / d) : 0.0f;
                }
            } else {
                memset(delta, 0, nl * nthreads * sizeof(float));
                memset(omega, 0, nl * nthreads * sizeof(float));
                int64_t pt = 0;
                for (int64_t x = 0; x < R; ++x)
                    for (int64_t y = 0; y < C; ++y)
                        for (int64_t z = 0; z < Z; ++z) {
                            const int64_t v = (x * C + y) * Z + z;
                            if (mask[v] != 1) continue;
                            const float u = L0[v] - B[v];
                            const float r = u - sharpen(u, bmin, slope, E, bins);
                            const size_t th = (size_t)((pt++ * nthreads) / nmask) * nl;
                            float w2s = 0.0f;
                            for (int a = 0; a < 4; ++a)
                                for (int b = 0; b < 4; ++b)
                                    for (int c = 0; c < 4; ++c) {
                                        const float w = ax.w[4 * x + a] * ay.w[4 * y + b] * az.w[4 * z + c];
                                        w2s += w * w;
                                    }
                            for (int a = 0; a < 4; ++a)
                                for (int b = 0; b < 4; ++b)
                                    for (int c = 0; c < 4; ++c) {
                                        const float w = ax.w[4 * x + a] * ay.w[4 * y + b] * az.w[4 * z + c];
                                        const size_t e = ((size_t)(ax.base[x] + a) * ncp[1] + ay.base[y] + b) * ncp[2] + az.base[z] + c;
                                        const float wc = w * w;
                                        delta[th + e] += wc * (w * r / w2s);
                                        omega[th + e] += wc;
                                    }
                        }
                for (int q = 1; q < nthreads; ++q)
                    for (size_t c = 0; c < nl; ++c) {
                        delta[c] += delta[q * nl + c];
                        omega[c] += omega[q * nl + c];
                    }
                for (size_t c = 0; c < nl; ++c) lat[c] += omega[c] != 0.0f ? delta[c] / omega[c] : 0.0f;
            }
            if (ABL(6)) {
                eval_P1(lat, &az, ncp[0], ncp[1], Z, P1);
                eval_T(P1, &ay, ncp[0], C, Z, T);
            }
            float N = 0.0f, mu = 0.0f, sig = 0.0f;   /* RealType; literals 1.0 are double */
            for (int64_t x = 0; x < R; ++x)
                for (int64_t y = 0; y < C; ++y)
                    for (int64_t z = 0; z < Z; ++z) {
                        const int64_t v = (x * C + y) * Z + z;
                        if (mask[v] != 1) continue;
                        const float bn = ABL(6) ? eval_B(T, &ax, ncp[0], x, y * Z + z) : itk_eval(lat, &ax, &ay, &az, x, y, z);
                        const float p = ABL(7) ? expf_cr(B[v] - bn) : expf(B[v] - bn);
                        N = (float)((double)N + 1.0);
                        if ((double)N > 1.0) {
                            const float q = p - mu;
                            sig = (float)((double)sig + ((double)(q * q) * ((double)N - 1.0)) / (double)N);
                        }
                        mu = (float)((double)mu * (1.0 - 1.0 / (double)N) + (double)(p / N));
                        B[v] = bn;
                    }
            sig = (float)sqrt((double)sig / ((double)N - 1.0));
            conv = sig / mu;
        }
        iters_out[level] = it - 1;
        if (conv_out) conv_out[level] = conv;
        if (level < prm->n_levels - 1) refine(lat, tmp, tmp2, ncp);
    }
    if (ABL(6)) {
        eval_P1(lat, &az, ncp[0], ncp[1], Z, P1);
        eval_T(P1, &ay, ncp[0], C, Z, T);
    }
    for (int64_t x = 0; x < R; ++x)
        for (int64_t y = 0; y < C; ++y)
            for (int64_t z = 0; z < Z; ++z) {
                const int64_t v = (x * C + y) * Z + z;
                const float bb = ABL(6) ? eval_B(T, &ax, ncp[0], x, y * Z + z) : itk_eval(lat, &ax, &ay, &az, x, y, z);
                out[v] = I[v] / (ABL(9) ? expf_cr(bb) : expf(bb));
            }
done:
    if (have_axes) { axis_free(&ax); axis_free(&ay); axis_free(&az); }
    free(L0); free(B); free(rv); free(lat); free(tmp); free(tmp2); free(delta); free(omega);
    free(num); free(denf); free(P1); free(T); free(H); free(Hi); free(hv); free(E);
    return rc;
}
#undef ABL

/* ---- lemma check (tests/test_n4_oracle.py): the exact sig step of the GPU's PC (n4_shared.h pc_div)
 * takes RN(Q / N) as Markstein's correction RN(y + r (Q - N y)), y = RN(Q r), r = RN(1 / N), for
 * Q = sqr(p - mu) (N - 1) (exact in double).  Returns the number of cases, out of `count`
 * pseudo-random (q2 float, N integer in [2, 2^24]) pairs and the edge N values, whose corrected
 * quotient differs from the IEEE division. */
static uint64_t xs64(uint64_t *s) { *s ^= *s << 13; *s ^= *s >> 7; *s ^= *s << 17; return *s; }
int64_t markstein_check(int64_t count, uint64_t seed)
{
    uint64_t st = seed ? seed : 88172645463325252ull;
    int64_t bad = 0;
    for (int64_t i = 0; i < count; ++i) {
        const uint64_t u = xs64(&st);
        double N;
        switch (i & 7) {
        case 0: N = (double)(1u << (1 + (u >> 59) % 24)); break;                 /* powers of two */
        case 1: N = (double)(1u << (1 + (u >> 59) % 24)) - 1.0; break;
        case 2: N = (double)((1u << (1 + (u >> 59) % 23)) + 1u); break;
        case 3: N = 16777216.0 - (double)(u >> 60); break;                         /* near 2^24 */
        default: N = 2.0 + (double)(u % 16777215u); break;
        }
        if (N < 2.0) N = 2.0;
        const uint32_t bits = (uint32_t)(xs64(&st) >> 32);
        const int ex = (int)(xs64(&st) % 80) - 70;
        const float q2 = ldexpf(1.0f + (float)(bits & 0x7fffff) * 0x1p-23f, ex);
        const double Q = (double)q2 * (N - 1.0);
        const double r = 1.0 / N;
        const double y = Q * r;
        const double e = fma(-N, y, Q);
        const double t = fma(e, r, y);
        if (t != Q / N) ++bad;
    }
    return bad;
}
