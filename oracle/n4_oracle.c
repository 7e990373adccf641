/* ORACLE -- test infrastructure only.  CPU restatement of N4 bias-field correction as the
 * reference calls it: sitk.N4BiasFieldCorrectionImageFilter().Execute(image, mask) with every
 * SimpleITK 2.3.1 default (Vent_Analysis.py:316-334).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.
 *
 * PARITY UNPINNED against SimpleITK: neither SimpleITK nor ITK source is available offline
 * (SURVEY.md §8c), so this file restates the ITK 5.3 algorithm from SURVEY Appendix A and is pinned
 * only by the build's known-answer tests (tests/test_n4_oracle.py).  The GPU path is checked
 * against it within tolerance.
 *
 * Geometry: numpy (R, C, Z) C-order == ITK raster order (x = slice axis fastest), spacing 1,
 * origin 0 (GetImageFromArray, Vent_Analysis.py:322-327).  The B-spline lattice is stored
 * [i over R][j over C][k over Z].
 *
 * Spec points (A.3) and the precision choices this build makes (same on CPU and GPU):
 *  - log input: L0 = (float)log((double)I) for mask==1 (MaskLabel 1) and I > 0, else 0 (?).
 *  - bin range: ITK's raster scan `if (p > max) max = p; else if (p < min) min = p;` -- the first
 *    masked pixel, and every later new maximum, never update the minimum.  Reproduced exactly.
 *  - triangular Parzen histogram, 200 bins; weights accumulated in unsigned 64-bit fixed point
 *    (2^-32 units; ITK sums in float) so CPU and GPU histograms are bit-identical.
 *  - 512-point zero-padded Wiener deconvolution and E(u|v) mapping in double, radix-2 FFT with
 *    host-computed twiddles; Gaussian taps use (float)exp((double)x) in place of expf.
 *  - B-spline fit (single level, cubic, Lee-Wolberg-Shin): num += w^2 (w r / sum w^2),
 *    den += w^2 over the 64 tensor weights, in double; phi = num/den (0 where den == 0);
 *    lattice += (float)phi.  Parametric coordinate p = idx * (spans / (n-1)) in float, clamped to
 *    spans - eps at the far end (ITK BSplineEpsilon = 100 FLT_EPSILON, x10 until representable).
 *  - evaluation: sum of the 64 weighted control points in double, rounded to float.
 *  - convergence: CoV of exp(B_old - B_new) over masked voxels, Welford recurrence in double.
 *  - level change: exact cubic B-spline subdivision (spans doubled per axis), axis by axis.
 *  - output: I / (float)exp((double)B) at every voxel.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
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
} n4o_params;

#define FFT_P 512

static float expf_cr(float x) { return (float)exp((double)x); }

/* ---- per-axis B-spline tables ------------------------------------------------------------- */
static float bspline_eps(int max_spans)
{
    float eps = 100.0f * FLT_EPSILON;
    while ((float)max_spans == (float)max_spans - eps) eps *= 10.0f;
    return eps;
}

static void axis_tables(int n, int ncp, float eps, int32_t *base, float *w, double *sw2)
{
    const int spans = ncp - 3;
    const float scale = (float)spans / (float)(n - 1);
    for (int idx = 0; idx < n; ++idx) {
        float p = (float)idx * scale;
        if (fabsf(p - (float)spans) <= eps) p = (float)spans - eps;
        if (p < 0.0f) p = 0.0f;
        int b = (int)p;
        float f = p - (float)b;
        double d = (double)f;
        double d2 = d * d, d3 = d2 * d;
        float w0 = (float)((1.0 - d) * (1.0 - d) * (1.0 - d) / 6.0);
        float w1 = (float)((3.0 * d3 - 6.0 * d2 + 4.0) / 6.0);
        float w2 = (float)((-3.0 * d3 + 3.0 * d2 + 3.0 * d + 1.0) / 6.0);
        float w3 = (float)(d3 / 6.0);
        base[idx] = b;
        w[4 * idx + 0] = w0; w[4 * idx + 1] = w1; w[4 * idx + 2] = w2; w[4 * idx + 3] = w3;
        sw2[idx] = (double)w0 * w0 + (double)w1 * w1 + (double)w2 * w2 + (double)w3 * w3;
    }
}

/* ---- FFT ---------------------------------------------------------------------------------- */
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

/* E(u|v) map of ITK SharpenImage (Appendix A.3 steps 4-8), from the fixed-point histogram. */
static void emap(const uint64_t *hfix, int bins, float binMin, float slope, float fwhm,
                 float noise, const cpx *tw, float *E)
{
    const int P = FFT_P;
    const int off = (P - bins) / 2;
    cpx V[FFT_P], F[FFT_P], U[FFT_P], num[FFT_P], den[FFT_P];
    memset(V, 0, sizeof V);
    memset(F, 0, sizeof F);
    for (int n = 0; n < bins; ++n) V[n + off].re = (double)hfix[n] * (1.0 / 4294967296.0);
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

/* ---- lattice subdivision along one axis ---------------------------------------------------- */
static void refine_axis(const float *in, float *out, const int *dims, int axis)
{
    /* in dims d[0..2]; out has d[axis] -> 2*d[axis]-3 */
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

/* ---- driver -------------------------------------------------------------------------------- */
int n4_oracle(const float *I, const uint8_t *mask, int64_t R, int64_t C, int64_t Z,
              const n4o_params *prm, float *out, int32_t *iters_out, float *conv_out)
{
    if (prm->spline_order != 3 || prm->n_levels < 1 || prm->n_levels > 8 || prm->n_bins < 2 ||
        prm->n_bins > FFT_P / 2 || R < 2 || C < 2 || Z < 2)
        return 1;
    const int64_t V = R * C * Z;
    const int bins = prm->n_bins;
    float *L0 = calloc((size_t)V, sizeof(float));
    float *B = calloc((size_t)V, sizeof(float));
    float *Bn = calloc((size_t)V, sizeof(float));
    int ncp[3] = {prm->ncp[0], prm->ncp[1], prm->ncp[2]};
    const int maxcp = 3 + ((ncp[0] > ncp[1] ? (ncp[0] > ncp[2] ? ncp[0] : ncp[2]) : (ncp[1] > ncp[2] ? ncp[1] : ncp[2])) - 3) * (1 << (prm->n_levels - 1));
    const size_t latmax = (size_t)maxcp * maxcp * maxcp;
    float *lat = calloc(latmax, sizeof(float));
    float *tmp = calloc(latmax, sizeof(float));
    float *tmp2 = calloc(latmax, sizeof(float));
    double *num = calloc(latmax, sizeof(double));
    double *den = calloc(latmax, sizeof(double));
    int32_t *bx = malloc(sizeof(int32_t) * R), *by = malloc(sizeof(int32_t) * C), *bz = malloc(sizeof(int32_t) * Z);
    float *wx = malloc(sizeof(float) * 4 * R), *wy = malloc(sizeof(float) * 4 * C), *wz = malloc(sizeof(float) * 4 * Z);
    double *sx = malloc(sizeof(double) * R), *sy = malloc(sizeof(double) * C), *sz = malloc(sizeof(double) * Z);
    uint64_t *H = malloc(sizeof(uint64_t) * bins);
    float *E = malloc(sizeof(float) * bins);
    cpx tw[FFT_P / 2];
    make_twiddles(tw);
    int64_t nmask = 0;
    for (int64_t v = 0; v < V; ++v)
        if (mask[v] == 1) {
            L0[v] = I[v] > 0.0f ? (float)log((double)I[v]) : 0.0f;
            ++nmask;
        }
    int rc = 0;
    if (nmask < 2) { rc = 3; goto done; }

    for (int level = 0; level < prm->n_levels; ++level) {
        int ms = ncp[0] > ncp[1] ? ncp[0] : ncp[1];
        ms = ms > ncp[2] ? ms : ncp[2];
        const float eps = bspline_eps(ms - 3);
        axis_tables((int)R, ncp[0], eps, bx, wx, sx);
        axis_tables((int)C, ncp[1], eps, by, wy, sy);
        axis_tables((int)Z, ncp[2], eps, bz, wz, sz);
        const size_t nl = (size_t)ncp[0] * ncp[1] * ncp[2];
        /* den depends only on the mask and this level's weights */
        memset(den, 0, nl * sizeof(double));
        for (int64_t x = 0; x < R; ++x)
            for (int64_t y = 0; y < C; ++y)
                for (int64_t z = 0; z < Z; ++z) {
                    if (mask[(x * C + y) * Z + z] != 1) continue;
                    for (int a = 0; a < 4; ++a)
                        for (int b = 0; b < 4; ++b)
                            for (int c = 0; c < 4; ++c) {
                                double w = (double)wx[4 * x + a] * (double)wy[4 * y + b] * (double)wz[4 * z + c];
                                den[((size_t)(bx[x] + a) * ncp[1] + (by[y] + b)) * ncp[2] + (bz[z] + c)] += w * w;
                            }
                }
        int it = 0;
        double conv = INFINITY;
        while (it++ < prm->max_iters[level] && conv > (double)prm->conv_threshold) {
            /* --- bin range with ITK's else-if quirk (raster order) --- */
            float bmax = -FLT_MAX, bmin = FLT_MAX;
            for (int64_t v = 0; v < V; ++v) {
                if (mask[v] != 1) continue;
                const float u = L0[v] - B[v];
                if (u > bmax) bmax = u;
                else if (u < bmin) bmin = u;
            }
            const float slope = (bmax - bmin) / (float)(bins - 1);
            /* --- Parzen histogram (fixed point) --- */
            memset(H, 0, sizeof(uint64_t) * bins);
            for (int64_t v = 0; v < V; ++v) {
                if (mask[v] != 1) continue;
                const float u = L0[v] - B[v];
                const float cidx = (u - bmin) / slope;
                if (!(cidx >= 0.0f)) continue;
                const int idx = (int)floorf(cidx);
                const float o = cidx - (float)idx;
                if (o == 0.0f) {
                    if (idx < bins) H[idx] += (uint64_t)1 << 32;
                } else if (idx < bins - 1) {
                    H[idx] += (uint64_t)((double)(1.0f - o) * 4294967296.0);
                    H[idx + 1] += (uint64_t)((double)o * 4294967296.0);
                }
            }
            emap(H, bins, bmin, slope, prm->fwhm, prm->wiener_noise, tw, E);
            /* --- sharpen, residual, B-spline fit --- */
            memset(num, 0, nl * sizeof(double));
            for (int64_t x = 0; x < R; ++x)
                for (int64_t y = 0; y < C; ++y)
                    for (int64_t z = 0; z < Z; ++z) {
                        const int64_t v = (x * C + y) * Z + z;
                        if (mask[v] != 1) continue;
                        const float u = L0[v] - B[v];
                        const float cidx = (u - bmin) / slope;
                        float S;
                        const int idx = cidx >= 0.0f ? (int)floorf(cidx) : bins;
                        if (idx < bins - 1) S = E[idx] + (E[idx + 1] - E[idx]) * (cidx - (float)idx);
                        else S = E[bins - 1];
                        const float r = u - S;
                        const double q = (double)r / (sx[x] * sy[y] * sz[z]);
                        for (int a = 0; a < 4; ++a)
                            for (int b = 0; b < 4; ++b)
                                for (int c = 0; c < 4; ++c) {
                                    double w = (double)wx[4 * x + a] * (double)wy[4 * y + b] * (double)wz[4 * z + c];
                                    num[((size_t)(bx[x] + a) * ncp[1] + (by[y] + b)) * ncp[2] + (bz[z] + c)] += w * w * w * q;
                                }
                    }
            for (size_t c = 0; c < nl; ++c) {
                const float phi = den[c] != 0.0 ? (float)(num[c] / den[c]) : 0.0f;
                lat[c] = lat[c] + phi;
            }
            /* --- evaluate at masked voxels, convergence --- */
            double N = 0.0, mu = 0.0, sig = 0.0;
            for (int64_t x = 0; x < R; ++x)
                for (int64_t y = 0; y < C; ++y)
                    for (int64_t z = 0; z < Z; ++z) {
                        const int64_t v = (x * C + y) * Z + z;
                        if (mask[v] != 1) continue;
                        double acc = 0.0;
                        for (int a = 0; a < 4; ++a)
                            for (int b = 0; b < 4; ++b)
                                for (int c = 0; c < 4; ++c) {
                                    double w = (double)wx[4 * x + a] * (double)wy[4 * y + b] * (double)wz[4 * z + c];
                                    acc += w * (double)lat[((size_t)(bx[x] + a) * ncp[1] + (by[y] + b)) * ncp[2] + (bz[z] + c)];
                                }
                        Bn[v] = (float)acc;
                        const double p = exp((double)B[v] - (double)Bn[v]);
                        N += 1.0;
                        if (N > 1.0) sig += (p - mu) * (p - mu) * (N - 1.0) / N;
                        mu = mu * (1.0 - 1.0 / N) + p / N;
                    }
            conv = sqrt(sig / (N - 1.0)) / mu;
            for (int64_t v = 0; v < V; ++v)
                if (mask[v] == 1) B[v] = Bn[v];
        }
        iters_out[level] = it - 1;
        if (conv_out) conv_out[level] = (float)conv;
        if (level < prm->n_levels - 1) {
            int d0[3] = {ncp[0], ncp[1], ncp[2]};
            refine_axis(lat, tmp, d0, 0);
            int d1[3] = {2 * ncp[0] - 3, ncp[1], ncp[2]};
            refine_axis(tmp, tmp2, d1, 1);
            int d2[3] = {2 * ncp[0] - 3, 2 * ncp[1] - 3, ncp[2]};
            refine_axis(tmp2, lat, d2, 2);
            ncp[0] = 2 * ncp[0] - 3; ncp[1] = 2 * ncp[1] - 3; ncp[2] = 2 * ncp[2] - 3;
        }
    }
    /* --- final field at every voxel, output --- */
    for (int64_t x = 0; x < R; ++x)
        for (int64_t y = 0; y < C; ++y)
            for (int64_t z = 0; z < Z; ++z) {
                const int64_t v = (x * C + y) * Z + z;
                double acc = 0.0;
                for (int a = 0; a < 4; ++a)
                    for (int b = 0; b < 4; ++b)
                        for (int c = 0; c < 4; ++c) {
                            double w = (double)wx[4 * x + a] * (double)wy[4 * y + b] * (double)wz[4 * z + c];
                            acc += w * (double)lat[((size_t)(bx[x] + a) * ncp[1] + (by[y] + b)) * ncp[2] + (bz[z] + c)];
                        }
                out[v] = I[v] / expf_cr((float)acc);
            }
done:
    free(L0); free(B); free(Bn); free(lat); free(tmp); free(tmp2); free(num); free(den);
    free(bx); free(by); free(bz); free(wx); free(wy); free(wz); free(sx); free(sy); free(sz);
    free(H); free(E);
    return rc;
}
