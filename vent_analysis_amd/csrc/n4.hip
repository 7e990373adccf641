// n4.hip -- N4 bias-field correction on gfx950, batched over volumes
// (replaces sitk.N4BiasFieldCorrectionImageFilter().Execute(image, mask), Vent_Analysis.py:316-334;
// algorithm restated in SURVEY.md Appendix A; CPU twin: oracle/n4_oracle.c, same spec).
//
// Per volume state lives in HBM: L0 (log input) and B (log bias) at masked voxels, the control
// lattice (<= 11^3 floats at the default 4 levels) and small per-iteration scratch.  Every voxel
// pass is a "column sweep": one thread per (col, slice) column walking the rows inside the
// column's masked range, so a wave reads 64 consecutive floats per row (coalesced) and the B-spline
// row weights are wave-uniform.  The cubic tensor-product fit and evaluation are SEPARABLE:
//   num[i][j][k] = sum_x wx(x,i)^3 sum_y wy(y,j)^3 sum_z wz(z,k)^3 q(x,y,z)     (q = r / sum w^2)
//   B(x,y,z)     = sum_i wx(x,i) sum_j wy(y,j) sum_z wz(z,k) phi[i][j][k]
// so each voxel costs ~4 double FMAs per pass instead of the 64 tensor terms (the row axis is
// contracted in registers by a sliding 4-wide window, the other two axes per volume in a small
// contraction kernel).  Reductions are deterministic: integer atomics (fixed-point histogram,
// min/max keys) or fixed-order per-block partials (convergence sums).
//
// Per iteration (one launch each, all volumes of the batch in one grid; converged volumes exit):
//   ctrl -> exact_min (rare) -> hist -> emap -> fit -> contract -> eval
#include <cfloat>
#include <climits>
#include <cstring>

#include "vh_internal.h"

struct DevAxis {
    const int32_t *base;
    const float *w;
    const double *sw2;
    const double *isw2;   // 1 / sw2
    int32_t n, ncp;
};
struct DevLevel {
    DevAxis ax[3];
};

struct FitTile {
    int yb, zb;        // tile extent
    int nty, ntz;      // tiles per volume along cols / slices
};

__host__ __device__ inline FitTile fit_tile(int64_t C, int64_t Z) {
    FitTile t;
    t.zb = (int)(Z < VH_TPB ? Z : VH_TPB);
    t.yb = VH_TPB / t.zb;
    if (t.yb > C) t.yb = (int)C;
    t.nty = (int)((C + t.yb - 1) / t.yb);
    t.ntz = (int)((Z + t.zb - 1) / t.zb);
    return t;
}

#define LN2 0.69314718055994530942
#define PI_D 3.14159265358979323846

// ---------------------------------------------------------------------------------------------
// host: per-level axis tables (identical expressions to oracle/n4_oracle.c axis_tables)
// ---------------------------------------------------------------------------------------------
float vh_bspline_eps(int max_spans) {
    float eps = 100.0f * FLT_EPSILON;
    while ((float)max_spans == (float)max_spans - eps) eps *= 10.0f;
    return eps;
}

void vh_axis_tables(int n, int ncp, float eps, AxisTab &t) {
    t.n = n;
    t.ncp = ncp;
    t.base.resize(n);
    t.w.resize(4 * (size_t)n);
    t.sw2.resize(n);
    const int spans = ncp - 3;
    const float scale = (float)spans / (float)(n - 1);
    for (int idx = 0; idx < n; ++idx) {
        volatile float pv = (float)idx * scale;   // volatile: keep float rounding points exact
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
        t.base[idx] = b;
        t.w[4 * idx + 0] = w0;
        t.w[4 * idx + 1] = w1;
        t.w[4 * idx + 2] = w2;
        t.w[4 * idx + 3] = w3;
        t.sw2[idx] = (double)w0 * w0 + (double)w1 * w1 + (double)w2 * w2 + (double)w3 * w3;
    }
}

static bool same_params(const vh_n4_params &a, const vh_n4_params &b) {
    if (a.n_levels != b.n_levels || a.spline_order != b.spline_order || a.n_bins != b.n_bins)
        return false;
    for (int i = 0; i < 3; ++i)
        if (a.ncp[i] != b.ncp[i]) return false;
    return true;
}

static int level_ncp(const vh_n4_params &p, int level, int axis) {
    int n = p.ncp[axis];
    for (int l = 0; l < level; ++l) n = 2 * n - 3;
    return n;
}

void vh_n4_prepare_tables(vh_batch *b, const vh_n4_params &prm) {
    if (b->tabs_valid && same_params(b->tab_prm, prm)) return;
    const int64_t dims[3] = {b->R, b->C, b->Z};
    std::vector<uint8_t> blob;
    b->tab_off.assign((size_t)prm.n_levels * 3 * 4, 0);
    auto push = [&](const void *p, size_t bytes) {
        size_t off = (blob.size() + 15) & ~(size_t)15;
        blob.resize(off + bytes);
        std::memcpy(blob.data() + off, p, bytes);
        return off;
    };
    for (int L = 0; L < prm.n_levels; ++L) {
        int ms = 0;
        for (int a = 0; a < 3; ++a) ms = std::max(ms, level_ncp(prm, L, a));
        const float eps = vh_bspline_eps(ms - 3);
        for (int a = 0; a < 3; ++a) {
            AxisTab t;
            vh_axis_tables((int)dims[a], level_ncp(prm, L, a), eps, t);
            std::vector<double> inv(t.sw2.size());
            for (size_t i = 0; i < inv.size(); ++i) inv[i] = 1.0 / t.sw2[i];
            b->tab_off[(L * 3 + a) * 4 + 0] = push(t.base.data(), t.base.size() * 4);
            b->tab_off[(L * 3 + a) * 4 + 1] = push(t.w.data(), t.w.size() * 4);
            b->tab_off[(L * 3 + a) * 4 + 2] = push(t.sw2.data(), t.sw2.size() * 8);
            b->tab_off[(L * 3 + a) * 4 + 3] = push(inv.data(), inv.size() * 8);
        }
    }
    if (b->d_tabs) HIP_TRY(hipFree(b->d_tabs));
    b->d_tabs = nullptr;
    HIP_TRY(hipMalloc(&b->d_tabs, blob.size()));
    HIP_TRY(hipMemcpy(b->d_tabs, blob.data(), blob.size(), hipMemcpyHostToDevice));
    if (!b->d_twiddle) {
        std::vector<double2> tw(VH_FFT_P / 2);
        for (int k = 0; k < VH_FFT_P / 2; ++k) {
            const double a = 2.0 * M_PI * (double)k / (double)VH_FFT_P;
            tw[k].x = cos(a);
            tw[k].y = -sin(a);
        }
        HIP_TRY(hipMalloc(&b->d_twiddle, sizeof(double2) * tw.size()));
        HIP_TRY(hipMemcpy(b->d_twiddle, tw.data(), sizeof(double2) * tw.size(),
                          hipMemcpyHostToDevice));
    }
    b->tab_prm = prm;
    b->tabs_valid = true;
}

static DevLevel dev_level(const vh_batch *b, const vh_n4_params &prm, int L) {
    DevLevel lv;
    const int64_t dims[3] = {b->R, b->C, b->Z};
    const uint8_t *base = (const uint8_t *)b->d_tabs;
    for (int a = 0; a < 3; ++a) {
        lv.ax[a].base = (const int32_t *)(base + b->tab_off[(L * 3 + a) * 4 + 0]);
        lv.ax[a].w = (const float *)(base + b->tab_off[(L * 3 + a) * 4 + 1]);
        lv.ax[a].sw2 = (const double *)(base + b->tab_off[(L * 3 + a) * 4 + 2]);
        lv.ax[a].isw2 = (const double *)(base + b->tab_off[(L * 3 + a) * 4 + 3]);
        lv.ax[a].n = (int32_t)dims[a];
        lv.ax[a].ncp = level_ncp(prm, L, a);
    }
    return lv;
}

void vh_ensure_n4_workspace(vh_batch *b, const vh_n4_params &prm) {
    const int L = prm.n_levels - 1;
    const int64_t cx = level_ncp(prm, L, 0), cy = level_ncp(prm, L, 1), cz = level_ncp(prm, L, 2);
    const int64_t lat = cx * cy * cz;
    const int64_t q2 = cx * cy * b->Z;
    if (b->d_L0 == nullptr) {
        HIP_TRY(hipMalloc(&b->d_L0, sizeof(float) * b->nb * b->V));
        HIP_TRY(hipMalloc(&b->d_B, sizeof(float) * b->nb * b->V));
        HIP_TRY(hipMalloc(&b->d_hist, sizeof(uint64_t) * b->nb * VH_MAX_BINS));
        HIP_TRY(hipMalloc(&b->d_E, sizeof(float) * b->nb * VH_MAX_BINS));
        HIP_TRY(hipMalloc(&b->d_st, sizeof(N4State) * b->nb));
        HIP_TRY(hipMalloc(&b->d_nactive, sizeof(int32_t) * 8 * 1024));
    }
    if (lat > b->lat_cap) {
        if (b->d_lat) HIP_TRY(hipFree(b->d_lat));
        if (b->d_num) HIP_TRY(hipFree(b->d_num));
        if (b->d_den) HIP_TRY(hipFree(b->d_den));
        HIP_TRY(hipMalloc(&b->d_lat, sizeof(float) * 3 * b->nb * lat));   // lattice + 2 scratch
        HIP_TRY(hipMalloc(&b->d_num, sizeof(double) * b->nb * lat));
        HIP_TRY(hipMalloc(&b->d_den, sizeof(double) * b->nb * lat));
        b->lat_cap = lat;
    }
    if (cx > 64) throw VhError{VH_ERR_ARG, "N4 lattice too fine: > 64 control points along rows"};
    const FitTile ft = fit_tile(b->C, b->Z);
    const int64_t fp = (int64_t)ft.nty * ft.ntz * lat;   // per-volume tile slabs
    if (fp > b->q1_cap) {
        if (b->d_fitpart) HIP_TRY(hipFree(b->d_fitpart));
        HIP_TRY(hipMalloc(&b->d_fitpart, sizeof(double) * b->nb * fp));
        b->q1_cap = fp;
    }
    if (q2 > b->q2_cap) {
        if (b->d_P1) HIP_TRY(hipFree(b->d_P1));
        HIP_TRY(hipMalloc(&b->d_P1, sizeof(double) * b->nb * q2));
        b->q2_cap = q2;
    }
    vh_n4_prepare_tables(b, prm);
}

// ---------------------------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float sharpen_value(float u, float bmin, float slope, const float *E,
                                               int bins) {
    const float cidx = (u - bmin) / slope;
    const int idx = (cidx >= 0.0f && cidx < (float)bins) ? (int)floorf(cidx) : bins;
    if (idx < bins - 1) return E[idx] + (E[idx + 1] - E[idx]) * (cidx - (float)idx);
    return E[bins - 1];
}

template <typename T>
__device__ __forceinline__ T block_sum_fixed(T v, T *s_red) {
    // wave shuffle tree, then waves in order: deterministic
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = v;
    __syncthreads();
    T r = 0;
    if (threadIdx.x == 0)
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) r += s_red[w];
    return r;
}

__device__ __forceinline__ double conv_from_parts(const double *part, int64_t nparts, int64_t b,
                                                  double N) {
    double sd = 0.0, sd2 = 0.0;
    for (int64_t p = 0; p < nparts; ++p) {
        sd += part[(b * nparts + p) * 2];
        sd2 += part[(b * nparts + p) * 2 + 1];
    }
    // CoV of p = exp(B_old - B_new) over masked voxels, with d = p - 1 (no cancellation)
    const double mu = 1.0 + sd / N;
    double var = (sd2 - sd * sd / N) / (N - 1.0);
    if (var < 0.0) var = 0.0;
    return sqrt(var) / mu;
}

// ---------------------------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------------------------
__global__ void k_n4_state_init(N4State *st, int64_t nb) {
    const int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (b >= nb) return;
    N4State s{};
    s.umax_key = 0u;
    s.umin_key = 0xffffffffu;
    s.active = 0;
    st[b] = s;
}

// ---------------------------------------------------------------------------------------------
// column-sweep scaffolding.  A lane owns one (col, slice) column; the wave walks the UNION of its
// lanes' masked row ranges in aligned chunks of 8 rows (row index wave-uniform, so the B-spline
// row weights are scalar loads), each lane predicating on its column's mask==1 row bitmap.  All 8
// rows' loads of a chunk are issued before any is used (memory-level parallelism).
// ---------------------------------------------------------------------------------------------
#define SW_CHUNK 8

struct ColSweep {
    int64_t col;      // column index in the volume (valid iff col < CZ)
    bool valid;
    int wlo, whi;     // wave-uniform row range (wlo > whi: nothing to do)
};

__device__ __forceinline__ ColSweep col_sweep_begin(const int32_t *colrange, int64_t b,
                                                    int64_t CZ, int64_t R) {
    ColSweep s;
    s.col = blockIdx.x * (int64_t)VH_TPB + threadIdx.x;
    s.valid = s.col < CZ;
    int lo = (int)R, hi = -1;
    if (s.valid) {
        lo = colrange[(b * CZ + s.col) * 2];
        hi = colrange[(b * CZ + s.col) * 2 + 1];
    }
    for (int off = 32; off > 0; off >>= 1) {
        lo = min(lo, __shfl_xor(lo, off, 64));
        hi = max(hi, __shfl_xor(hi, off, 64));
    }
    s.wlo = __builtin_amdgcn_readfirstlane(lo);
    s.whi = __builtin_amdgcn_readfirstlane(hi);
    return s;
}

__device__ __forceinline__ uint32_t chunk_bits(const uint32_t *colbits, const ColSweep &s,
                                               int64_t b, int64_t nw, int64_t CZ, int x0) {
    if (!s.valid) return 0u;
    const uint32_t w = colbits[(b * nw + (x0 >> 5)) * CZ + s.col];
    return (w >> (x0 & 31)) & 0xffu;
}

// L0 = log(I) at mask == 1 (non-positive -> 0), B = 0, U = L0 and the first U range.
__global__ void __launch_bounds__(VH_TPB) k_n4_init(const float *__restrict__ I,
                                                   const uint32_t *__restrict__ colbits,
                                                   const int32_t *colrange,
                                                   const VolScalars *sc, int64_t R, int64_t CZ,
                                                   int64_t V, float *L0, float *B, float *U,
                                                   N4State *st) {
    __shared__ uint32_t s_max, s_min;
    const int64_t b = blockIdx.y;
    if (threadIdx.x == 0) { s_max = 0u; s_min = 0xffffffffu; }
    __syncthreads();
    const ColSweep cs = col_sweep_begin(colrange, b, CZ, R);
    const int64_t nw = (R + 31) >> 5;
    const int64_t first = sc[b].first_masked;
    uint32_t kmax = 0u, kmin = 0xffffffffu;
    for (int x0 = cs.wlo & ~(SW_CHUNK - 1); x0 <= cs.whi; x0 += SW_CHUNK) {
        const uint32_t m8 = chunk_bits(colbits, cs, b, nw, CZ, x0);
        float a[SW_CHUNK];
#pragma unroll
        for (int k = 0; k < SW_CHUNK; ++k)
            a[k] = (m8 >> k) & 1u ? I[b * V + (int64_t)(x0 + k) * CZ + cs.col] : 0.0f;
#pragma unroll
        for (int k = 0; k < SW_CHUNK; ++k) {
            if (!((m8 >> k) & 1u)) continue;
            const int64_t r = (int64_t)(x0 + k) * CZ + cs.col, v = b * V + r;
            const float l = a[k] > 0.0f ? (float)log((double)a[k]) : 0.0f;
            L0[v] = l;
            B[v] = 0.0f;
            U[v] = l;
            const uint32_t key = f2key(l);
            kmax = key > kmax ? key : kmax;
            if (r == first) st[b].u_first = l;
            else kmin = key < kmin ? key : kmin;
        }
    }
    if (kmax) atomicMax(&s_max, kmax);
    if (kmin != 0xffffffffu) atomicMin(&s_min, kmin);
    __syncthreads();
    if (threadIdx.x == 0) {
        if (s_max) atomicMax(&st[b].umax_key, s_max);
        if (s_min != 0xffffffffu) atomicMin(&st[b].umin_key, s_min);
    }
}

// Iteration control: convergence of the previous iteration, the while-condition of ITK's loop,
// bin range (common case of the else-if quirk), histogram reset.
__global__ void k_n4_ctrl(N4State *st, const double *part, int64_t nparts, const VolScalars *sc,
                          int level, int it, float thresh, int bins, int64_t nb,
                          uint64_t *hist, int32_t *nactive) {
    const int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (b >= nb) return;
    N4State &s = st[b];
    if (it == 0) {
        s.active = 1;
        s.iters = 0;
        s.conv = INFINITY;
    } else if (s.active) {
        const double conv = conv_from_parts(part, nparts, b, (double)sc[b].n_mask1);
        s.conv = conv;
        if (!(conv > (double)thresh)) {
            s.active = 0;
            s.iters_level[level] = s.iters;
            s.conv_level[level] = (float)conv;
        }
    }
    if (!s.active) return;
    s.iters += 1;
    const float bmax = key2f(s.umax_key);
    const float umin = s.umin_key == 0xffffffffu ? FLT_MAX : key2f(s.umin_key);
    s.bin_max = bmax;
    if (umin <= s.u_first) {
        s.need_exact_min = 0;
        s.bin_min = umin;
        s.slope = (bmax - umin) / (float)(bins - 1);
    } else {
        s.need_exact_min = 1;   // k_n4_exact_min computes bin_min and slope
    }
    s.umax_key = 0u;
    s.umin_key = 0xffffffffu;
    for (int i = 0; i < VH_MAX_BINS; ++i) hist[b * VH_MAX_BINS + i] = 0ull;
    atomicAdd(nactive, 1);
}

__global__ void k_n4_level_end(N4State *st, const double *part, int64_t nparts,
                               const VolScalars *sc, int level, int64_t nb) {
    const int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (b >= nb) return;
    N4State &s = st[b];
    if (s.active) {
        const double conv = conv_from_parts(part, nparts, b, (double)sc[b].n_mask1);
        s.conv = conv;
        s.iters_level[level] = s.iters;
        s.conv_level[level] = (float)conv;
        s.active = 0;
    }
}

// Exact ITK bin minimum when the first masked pixel is the strict minimum: min over the pixels
// that are not running maxima in raster order (chunked prefix-max scan).  One block per volume.
__global__ void __launch_bounds__(VH_TPB) k_n4_exact_min(const float *__restrict__ U,
                                                        const uint8_t *__restrict__ mask,
                                                        int64_t V, int bins, N4State *st) {
    __shared__ float s_cmax[VH_TPB];
    __shared__ float s_min[VH_TPB];
    const int64_t b = blockIdx.x;
    if (!st[b].active || !st[b].need_exact_min) return;
    const int t = threadIdx.x;
    const int64_t per = (V + VH_TPB - 1) / VH_TPB;
    const int64_t s0 = t * per, e0 = s0 + per < V ? s0 + per : V;
    float cmax = -FLT_MAX;
    for (int64_t r = s0; r < e0; ++r)
        if (mask[b * V + r] == 1) {
            const float u = U[b * V + r];
            cmax = u > cmax ? u : cmax;
        }
    s_cmax[t] = cmax;
    __syncthreads();
    if (t == 0) {
        float run = -FLT_MAX;
        for (int i = 0; i < VH_TPB; ++i) { const float v = s_cmax[i]; s_cmax[i] = run; run = v > run ? v : run; }
    }
    __syncthreads();
    float run = s_cmax[t], mn = FLT_MAX;
    for (int64_t r = s0; r < e0; ++r)
        if (mask[b * V + r] == 1) {
            const float u = U[b * V + r];
            if (u > run) run = u;
            else if (u < mn) mn = u;
        }
    s_min[t] = mn;
    __syncthreads();
    if (t == 0) {
        float m = FLT_MAX;
        for (int i = 0; i < VH_TPB; ++i) m = s_min[i] < m ? s_min[i] : m;
        st[b].bin_min = m;
        st[b].slope = (st[b].bin_max - m) / (float)(bins - 1);
    }
}

// Triangular Parzen histogram of U at mask == 1, unsigned 64-bit fixed point (2^-32 units).
// Neighbouring rows of a column fall in the same bin most of the time: each lane keeps a run
// (bin, two weights) in registers and only touches LDS when the bin changes.
__global__ void __launch_bounds__(VH_TPB) k_n4_hist(const float *__restrict__ U,
                                                   const uint32_t *__restrict__ colbits,
                                                   const int32_t *colrange, int64_t R,
                                                   int64_t CZ, int64_t V, int bins,
                                                   const N4State *st, uint64_t *hist) {
    __shared__ unsigned long long H[VH_MAX_BINS];
    const int64_t b = blockIdx.y;
    if (!st[b].active) return;
    for (int i = threadIdx.x; i < VH_MAX_BINS; i += VH_TPB) H[i] = 0ull;
    __syncthreads();
    const float bmin = st[b].bin_min, slope = st[b].slope;
    const ColSweep cs = col_sweep_begin(colrange, b, CZ, R);
    const int64_t nw = (R + 31) >> 5;
    int cur = -1;
    unsigned long long w0 = 0ull, w1 = 0ull;
    for (int x0 = cs.wlo & ~(SW_CHUNK - 1); x0 <= cs.whi; x0 += SW_CHUNK) {
        const uint32_t m8 = chunk_bits(colbits, cs, b, nw, CZ, x0);
        float u[SW_CHUNK];
#pragma unroll
        for (int k = 0; k < SW_CHUNK; ++k)
            u[k] = (m8 >> k) & 1u ? U[b * V + (int64_t)(x0 + k) * CZ + cs.col] : 0.0f;
#pragma unroll
        for (int k = 0; k < SW_CHUNK; ++k) {
            if (!((m8 >> k) & 1u)) continue;
            const float cidx = (u[k] - bmin) / slope;
            if (!(cidx >= 0.0f) || !(cidx < (float)bins)) continue;
            const int idx = (int)floorf(cidx);
            const float o = cidx - (float)idx;
            unsigned long long a0, a1 = 0ull;
            if (o == 0.0f) {
                a0 = 1ull << 32;
            } else if (idx < bins - 1) {
                a0 = (unsigned long long)((double)(1.0f - o) * 4294967296.0);
                a1 = (unsigned long long)((double)o * 4294967296.0);
            } else {
                continue;
            }
            if (idx != cur) {
                if (cur >= 0) {
                    if (w0) atomicAdd(&H[cur], w0);
                    if (w1) atomicAdd(&H[cur + 1], w1);
                }
                cur = idx;
                w0 = 0ull;
                w1 = 0ull;
            }
            w0 += a0;
            w1 += a1;
        }
    }
    if (cur >= 0) {
        if (w0) atomicAdd(&H[cur], w0);
        if (w1) atomicAdd(&H[cur + 1], w1);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < bins; i += VH_TPB)
        if (H[i]) atomicAdd((unsigned long long *)&hist[b * VH_MAX_BINS + i], H[i]);
}

// 512-point radix-2 FFT in LDS, 256 threads (one butterfly each per stage); same butterfly and
// twiddle indexing as oracle/n4_oracle.c fft_inplace.
__device__ void lds_fft(double2 *x, double2 *tmp, const double2 *tw, bool inverse) {
    const int P = VH_FFT_P;
    const int t = threadIdx.x;
    for (int i = t; i < P; i += VH_TPB) tmp[i] = x[i];
    __syncthreads();
    for (int i = t; i < P; i += VH_TPB) {
        const int r = (int)(__brev((unsigned)i) >> (32 - 9));
        x[r] = tmp[i];
    }
    __syncthreads();
    for (int len = 2; len <= P; len <<= 1) {
        const int half = len >> 1, step = P / len;
        const int g = t / half, j = t % half;
        const int i0 = g * len + j, i1 = i0 + half;
        double2 w = tw[j * step];
        if (inverse) w.y = -w.y;
        const double2 bb = x[i1];
        const double tr = w.x * bb.x - w.y * bb.y, ti = w.x * bb.y + w.y * bb.x;
        const double2 a = x[i0];
        x[i0] = make_double2(a.x + tr, a.y + ti);
        x[i1] = make_double2(a.x - tr, a.y - ti);
        __syncthreads();
    }
}

__device__ __forceinline__ float expf_cr(float x) { return (float)exp((double)x); }

// E(u|v) map (Wiener deconvolution of the histogram by the bias Gaussian), one block per volume.
__global__ void __launch_bounds__(VH_TPB) k_n4_emap(const uint64_t *hist, const double2 *tw,
                                                   int bins, float fwhm, float noise,
                                                   const N4State *st, float *Eout) {
    __shared__ double2 V[VH_FFT_P], F[VH_FFT_P], U[VH_FFT_P], NUM[VH_FFT_P], DEN[VH_FFT_P],
        TMP[VH_FFT_P];
    const int64_t b = blockIdx.x;
    if (!st[b].active) return;
    const int P = VH_FFT_P, off = (P - bins) / 2;
    const int t = threadIdx.x;
    const float binMin = st[b].bin_min, slope = st[b].slope;
    for (int n = t; n < P; n += VH_TPB) {
        const int h = n - off;
        V[n] = make_double2(h >= 0 && h < bins ? (double)hist[b * VH_MAX_BINS + h] * (1.0 / 4294967296.0) : 0.0, 0.0);
        F[n] = make_double2(0.0, 0.0);
    }
    __syncthreads();
    const float sFWHM = fwhm / slope;
    const float ef = (float)(4.0 * LN2 / (double)(sFWHM * sFWHM));
    const float sf = (float)(2.0 * sqrt(LN2 / PI_D) / (double)sFWHM);
    for (int n = t; n <= P / 2; n += VH_TPB) {
        if (n == 0) {
            F[0].x = (double)sf;
        } else if (n == P / 2) {
            F[n].x = (double)sf * exp(-0.25 * (double)((float)P * (float)P) * (double)ef);
        } else {
            const float nf = (float)n;
            const double v = (double)(sf * expf_cr(-(nf * nf) * ef));
            F[n].x = v;
            F[P - n].x = v;
        }
    }
    __syncthreads();
    lds_fft(V, TMP, tw, false);
    lds_fft(F, TMP, tw, false);
    for (int n = t; n < P; n += VH_TPB) {
        const double a = F[n].x, bb = F[n].y;
        const double g = a / ((a * a - (-bb) * bb) + (double)noise);
        U[n] = make_double2(V[n].x * g, V[n].y * g);
    }
    __syncthreads();
    lds_fft(U, TMP, tw, true);
    for (int n = t; n < P; n += VH_TPB) {
        const double ur = U[n].x > 0.0 ? U[n].x : 0.0;
        U[n] = make_double2(ur, 0.0);
        const float c = binMin + ((float)n - (float)off) * slope;
        NUM[n] = make_double2((double)c * ur, 0.0);
        DEN[n] = make_double2(ur, 0.0);
    }
    __syncthreads();
    lds_fft(NUM, TMP, tw, false);
    lds_fft(DEN, TMP, tw, false);
    for (int n = t; n < P; n += VH_TPB) {
        const double a = F[n].x, bb = F[n].y;
        double2 x = NUM[n];
        NUM[n] = make_double2(x.x * a - x.y * bb, x.x * bb + x.y * a);
        x = DEN[n];
        DEN[n] = make_double2(x.x * a - x.y * bb, x.x * bb + x.y * a);
    }
    __syncthreads();
    lds_fft(NUM, TMP, tw, true);
    lds_fft(DEN, TMP, tw, true);
    for (int n = t; n < bins; n += VH_TPB) {
        const double d = DEN[n + off].x;
        Eout[b * VH_MAX_BINS + n] = d != 0.0 ? (float)(NUM[n + off].x / d) : 0.0f;
    }
}

// ---------------------------------------------------------------------------------------------
// Fit sweep with in-block contraction.  A block owns a tile of YB cols x ZB slices (YB*ZB <= 256
// columns, one per thread); after the row sweep (same sliding window as k_n4_fitsweep) every
// thread holds Q1[i] of its column in LDS, and the block contracts its tile over cols and slices:
//   Pn[i][j][k] = sum_{y in tile} sum_{z in tile} wy(y,j)^p wz(z,k)^p Q1[i][y][z]
// for the lattice rows j / slices k its tile touches.  Only that small slab goes to HBM; the
// contract kernel adds the slabs of a volume's tiles in tile order (deterministic).
// p = 3 (MODE 0, numerator) or 2 (MODE 1, denominator).
// ---------------------------------------------------------------------------------------------
template <int MODE>
__global__ void __launch_bounds__(VH_TPB) k_n4_fitblock(const float *__restrict__ U,
                                                       const uint32_t *__restrict__ colbits,
                                                       const int32_t *colrange, int64_t R,
                                                       int64_t C, int64_t Z, int64_t V, int bins,
                                                       const N4State *st, const float *E,
                                                       DevLevel lv, int64_t slab, double *part) {
    extern __shared__ __attribute__((aligned(16))) double sQ1[];   // [ncx][VH_TPB]
    __shared__ float sE[VH_MAX_BINS];
    const int64_t b = blockIdx.y;
    if (MODE == 0 && !st[b].active) return;
    const FitTile ft = fit_tile(C, Z);
    const int tile = blockIdx.x;
    const int ty0 = (tile / ft.ntz) * ft.yb, tz0 = (tile % ft.ntz) * ft.zb;
    const int ny = (int)(C - ty0 < ft.yb ? C - ty0 : ft.yb);
    const int nz = (int)(Z - tz0 < ft.zb ? Z - tz0 : ft.zb);
    const int tid = threadIdx.x;
    const int ly = tid / ft.zb, lz = tid % ft.zb;
    const bool mine = ly < ny && lz < nz;
    const int64_t CZ = C * Z;
    const DevAxis ax = lv.ax[0], ay = lv.ax[1], az = lv.ax[2];
    const int ncx = ax.ncp;
    for (int i = 0; i < ncx; ++i) sQ1[i * VH_TPB + tid] = 0.0;
    if (MODE == 0)
        for (int i = tid; i < bins; i += VH_TPB) sE[i] = E[b * VH_MAX_BINS + i];
    // ---- row sweep of this thread's column (wave-uniform chunked rows) ----
    ColSweep cs;
    cs.col = (int64_t)(ty0 + ly) * Z + (tz0 + lz);
    cs.valid = mine;
    {
        int lo = (int)R, hi = -1;
        if (mine) {
            lo = colrange[(b * CZ + cs.col) * 2];
            hi = colrange[(b * CZ + cs.col) * 2 + 1];
        }
        for (int off = 32; off > 0; off >>= 1) {
            lo = min(lo, __shfl_xor(lo, off, 64));
            hi = max(hi, __shfl_xor(hi, off, 64));
        }
        cs.wlo = __builtin_amdgcn_readfirstlane(lo);
        cs.whi = __builtin_amdgcn_readfirstlane(hi);
    }
    __syncthreads();
    if (cs.wlo <= cs.whi) {
        const int64_t nw = (R + 31) >> 5;
        float bmin = 0.0f, slope = 1.0f;
        if (MODE == 0) {
            bmin = st[b].bin_min;
            slope = st[b].slope;
        }
        double isyz = 1.0;
        if (mine) isyz = ay.isw2[ty0 + ly] * az.isw2[tz0 + lz];
        const int xs = cs.wlo & ~(SW_CHUNK - 1);
        int wb = ax.base[xs];
        double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
        for (int x0 = xs; x0 <= cs.whi; x0 += SW_CHUNK) {
            const uint32_t m8 = chunk_bits(colbits, cs, b, nw, CZ, x0);
            float u[SW_CHUNK];
            if (MODE == 0) {
#pragma unroll
                for (int k = 0; k < SW_CHUNK; ++k)
                    u[k] = (m8 >> k) & 1u ? U[b * V + (int64_t)(x0 + k) * CZ + cs.col] : 0.0f;
            }
#pragma unroll
            for (int k = 0; k < SW_CHUNK; ++k) {
                const int x = x0 + k;
                if (x >= R) break;
                const int bx = ax.base[x];
                while (wb < bx) {
                    sQ1[wb * VH_TPB + tid] = a0;
                    a0 = a1; a1 = a2; a2 = a3; a3 = 0.0;
                    ++wb;
                }
                if (!((m8 >> k) & 1u)) continue;
                const float4 w = *reinterpret_cast<const float4 *>(ax.w + 4 * x);
                const double w0 = w.x, w1 = w.y, w2 = w.z, w3 = w.w;
                if (MODE == 0) {
                    const float r = u[k] - sharpen_value(u[k], bmin, slope, sE, bins);
                    const double q = ((double)r * ax.isw2[x]) * isyz;
                    a0 += (w0 * w0 * w0) * q;
                    a1 += (w1 * w1 * w1) * q;
                    a2 += (w2 * w2 * w2) * q;
                    a3 += (w3 * w3 * w3) * q;
                } else {
                    a0 += w0 * w0;
                    a1 += w1 * w1;
                    a2 += w2 * w2;
                    a3 += w3 * w3;
                }
            }
        }
        sQ1[wb * VH_TPB + tid] = a0;
        if (wb + 1 < ncx) sQ1[(wb + 1) * VH_TPB + tid] = a1;
        if (wb + 2 < ncx) sQ1[(wb + 2) * VH_TPB + tid] = a2;
        if (wb + 3 < ncx) sQ1[(wb + 3) * VH_TPB + tid] = a3;
    }
    __syncthreads();
    // ---- contract the tile over cols and slices ----
    const int jlo = ay.base[ty0], jhi = ay.base[ty0 + ny - 1] + 3;
    const int klo = az.base[tz0], khi = az.base[tz0 + nz - 1] + 3;
    const int JT = jhi - jlo + 1, KT = khi - klo + 1;
    double *out = part + (b * (int64_t)(ft.nty * ft.ntz) + tile) * slab;
    for (int e = tid; e < ncx * JT * KT; e += VH_TPB) {
        const int i = e / (JT * KT), jj = (e / KT) % JT, kk = e % KT;
        const int j = jlo + jj, kq = klo + kk;
        double acc = 0.0;
        for (int yy = 0; yy < ny; ++yy) {
            const int cy = j - ay.base[ty0 + yy];
            if (cy < 0 || cy > 3) continue;
            const double wyv = ay.w[4 * (ty0 + yy) + cy];
            const double wyp = MODE == 0 ? wyv * wyv * wyv : wyv * wyv;
            double accz = 0.0;
            for (int zz = 0; zz < nz; ++zz) {
                const int cz = kq - az.base[tz0 + zz];
                if (cz < 0 || cz > 3) continue;
                const double wzv = az.w[4 * (tz0 + zz) + cz];
                const double wzp = MODE == 0 ? wzv * wzv * wzv : wzv * wzv;
                accz += wzp * sQ1[i * VH_TPB + yy * ft.zb + zz];
            }
            acc += wyp * accz;
        }
        out[e] = acc;
    }
}

// Sum the tile slabs of each volume (tile order), then MODE 1: den; MODE 0: phi = num/den,
// lattice += phi, P1[i][j][z] = sum_k wz(z,k) lat[i][j][k] for the eval sweep.  One block/volume.
template <int MODE>
__global__ void __launch_bounds__(VH_TPB) k_n4_tilesum(const double *part, int64_t slab,
                                                      float *lat, double *den, double *P1,
                                                      int64_t C, int64_t Z, int64_t lat_cap,
                                                      int64_t q2_cap, const N4State *st,
                                                      DevLevel lv) {
    const int64_t b = blockIdx.x;
    if (MODE == 0 && !st[b].active) return;
    const FitTile ft = fit_tile(C, Z);
    const int ntiles = ft.nty * ft.ntz;
    const DevAxis ay = lv.ax[1], az = lv.ax[2];
    const int ncx = lv.ax[0].ncp, ncy = ay.ncp, ncz = az.ncp;
    float *L = lat + b * lat_cap;
    double *D = den + b * lat_cap;
    for (int e = threadIdx.x; e < ncx * ncy * ncz; e += VH_TPB) {
        const int i = e / (ncy * ncz), j = (e / ncz) % ncy, kq = e % ncz;
        double acc = 0.0;
        for (int tile = 0; tile < ntiles; ++tile) {
            const int ty0 = (tile / ft.ntz) * ft.yb, tz0 = (tile % ft.ntz) * ft.zb;
            const int ny = (int)(C - ty0 < ft.yb ? C - ty0 : ft.yb);
            const int nz = (int)(Z - tz0 < ft.zb ? Z - tz0 : ft.zb);
            const int jlo = ay.base[ty0], jhi = ay.base[ty0 + ny - 1] + 3;
            const int klo = az.base[tz0], khi = az.base[tz0 + nz - 1] + 3;
            if (j < jlo || j > jhi || kq < klo || kq > khi) continue;
            const int JT = jhi - jlo + 1, KT = khi - klo + 1;
            acc += part[(b * (int64_t)ntiles + tile) * slab + (i * JT + (j - jlo)) * KT + (kq - klo)];
        }
        if (MODE == 1) {
            D[e] = acc;
        } else {
            const double d = D[e];
            const float phi = d != 0.0 ? (float)(acc / d) : 0.0f;
            L[e] = L[e] + phi;
        }
    }
    if (MODE == 0) {
        __syncthreads();
        double *p1 = P1 + b * q2_cap;
        for (int64_t e = threadIdx.x; e < (int64_t)ncx * ncy * Z; e += VH_TPB) {
            const int64_t ij = e / Z, z = e % Z;
            const int bz = az.base[z];
            const float4 w = *reinterpret_cast<const float4 *>(az.w + 4 * z);
            const float *l = L + ij * ncz + bz;
            p1[e] = (double)w.x * (double)l[0] + (double)w.y * (double)l[1] +
                    (double)w.z * (double)l[2] + (double)w.w * (double)l[3];
        }
    }
}

// T(i) = sum_j wy(y,j) P1[i][j][z] for one column
__device__ __forceinline__ double col_T(const double *p1, int i, int ncy, int64_t Z, int by,
                                        float4 wy, int64_t z) {
    const double *r = p1 + ((int64_t)i * ncy + by) * Z + z;
    return (double)wy.x * r[0] + (double)wy.y * r[Z] + (double)wy.z * r[2 * Z] + (double)wy.w * r[3 * Z];
}

// Evaluate the new field at masked voxels, convergence partials, U = L0 - B and its range for the
// next iteration.
__global__ void __launch_bounds__(VH_TPB) k_n4_eval(const float *__restrict__ L0, float *B,
                                                   float *U, const uint32_t *__restrict__ colbits,
                                                   const int32_t *colrange, const VolScalars *sc,
                                                   int64_t R, int64_t C, int64_t Z, int64_t V,
                                                   int64_t q2_cap, const double *P1,
                                                   DevLevel lv, N4State *st, int64_t nparts,
                                                   double *part) {
    __shared__ double s_red[VH_TPB / 64];
    __shared__ uint32_t s_max, s_min;
    const int64_t b = blockIdx.y;
    if (!st[b].active) return;
    if (threadIdx.x == 0) { s_max = 0u; s_min = 0xffffffffu; }
    const int64_t CZ = C * Z;
    const ColSweep cs = col_sweep_begin(colrange, b, CZ, R);
    const int64_t nw = (R + 31) >> 5;
    double sd = 0.0, sd2 = 0.0;
    uint32_t kmax = 0u, kmin = 0xffffffffu;
    if (cs.wlo <= cs.whi) {
        const int64_t y = cs.valid ? cs.col / Z : 0, z = cs.valid ? cs.col % Z : 0;
        const int ncy = lv.ax[1].ncp;
        const int by = lv.ax[1].base[y];
        const float4 wy = *reinterpret_cast<const float4 *>(lv.ax[1].w + 4 * y);
        const double *p1 = P1 + b * q2_cap;
        const DevAxis ax = lv.ax[0];
        const int64_t first = sc[b].first_masked;
        const int xs = cs.wlo & ~(SW_CHUNK - 1);
        int wb = ax.base[xs];
        // window of T(i), i = wb..wb+3 (double contraction, float value like the lattice)
        float t0 = (float)col_T(p1, wb, ncy, Z, by, wy, z), t1 = (float)col_T(p1, wb + 1, ncy, Z, by, wy, z);
        float t2 = (float)col_T(p1, wb + 2, ncy, Z, by, wy, z), t3 = (float)col_T(p1, wb + 3, ncy, Z, by, wy, z);
        for (int x0 = xs; x0 <= cs.whi; x0 += SW_CHUNK) {
            const uint32_t m8 = chunk_bits(colbits, cs, b, nw, CZ, x0);
            float l0[SW_CHUNK], bo[SW_CHUNK];
#pragma unroll
            for (int k = 0; k < SW_CHUNK; ++k) {
                const bool on = (m8 >> k) & 1u;
                const int64_t v = b * V + (int64_t)(x0 + k) * CZ + cs.col;
                l0[k] = on ? L0[v] : 0.0f;
                bo[k] = on ? B[v] : 0.0f;
            }
#pragma unroll
            for (int k = 0; k < SW_CHUNK; ++k) {
                const int x = x0 + k;
                if (x >= R) break;
                const int bx = ax.base[x];
                while (wb < bx) {
                    ++wb;
                    t0 = t1; t1 = t2; t2 = t3;
                    t3 = (float)col_T(p1, wb + 3, ncy, Z, by, wy, z);
                }
                if (!((m8 >> k) & 1u)) continue;
                const float4 w = *reinterpret_cast<const float4 *>(ax.w + 4 * x);
                const float bn = ((w.x * t0 + w.y * t1) + w.z * t2) + w.w * t3;
                const double d = (double)expm1f(bo[k] - bn);   // p - 1, p = exp(B_old - B_new)
                sd += d;
                sd2 += d * d;
                const int64_t r = (int64_t)x * CZ + cs.col, v = b * V + r;
                B[v] = bn;
                const float u = l0[k] - bn;
                U[v] = u;
                const uint32_t key = f2key(u);
                kmax = key > kmax ? key : kmax;
                if (r == first) st[b].u_first = u;
                else kmin = key < kmin ? key : kmin;
            }
        }
    }
    __syncthreads();
    if (kmax) atomicMax(&s_max, kmax);
    if (kmin != 0xffffffffu) atomicMin(&s_min, kmin);
    const double tsd = block_sum_fixed(sd, s_red);
    __syncthreads();
    const double tsd2 = block_sum_fixed(sd2, s_red);
    if (threadIdx.x == 0) {
        part[(b * nparts + blockIdx.x) * 2] = tsd;
        part[(b * nparts + blockIdx.x) * 2 + 1] = tsd2;
        if (s_max) atomicMax(&st[b].umax_key, s_max);
        if (s_min != 0xffffffffu) atomicMin(&st[b].umin_key, s_min);
    }
}

// Exact cubic B-spline subdivision (spans doubled on every axis), axis by axis, one block/volume.
__device__ void refine_axis_dev(const float *in, float *out, int d0, int d1, int d2, int axis) {
    int od[3] = {d0, d1, d2};
    const int dims[3] = {d0, d1, d2};
    od[axis] = 2 * dims[axis] - 3;
    const int total = od[0] * od[1] * od[2];
    for (int e = threadIdx.x; e < total; e += VH_TPB) {
        const int a = e / (od[1] * od[2]), bq = (e / od[2]) % od[1], c = e % od[2];
        int o[3] = {a, bq, c};
        const int m = o[axis], j = m >> 1;
        int s0[3] = {a, bq, c}, s1[3] = {a, bq, c}, s2[3] = {a, bq, c};
        s0[axis] = j; s1[axis] = j + 1; s2[axis] = j + 2;
        auto IDX = [&](const int *s) { return ((size_t)s[0] * dims[1] + s[1]) * dims[2] + s[2]; };
        double v;
        if ((m & 1) == 0) v = ((double)in[IDX(s0)] + (double)in[IDX(s1)]) * 0.5;
        else v = ((double)in[IDX(s0)] + 6.0 * (double)in[IDX(s1)] + (double)in[IDX(s2)]) * 0.125;
        out[e] = (float)v;
    }
}

__global__ void __launch_bounds__(VH_TPB) k_n4_refine(float *lat, int64_t lat_cap, int64_t nb,
                                                     int n0, int n1, int n2) {
    const int64_t b = blockIdx.x;
    float *L = lat + b * lat_cap;
    float *T1 = lat + (nb + b) * lat_cap;
    float *T2 = lat + (2 * nb + b) * lat_cap;
    refine_axis_dev(L, T1, n0, n1, n2, 0);
    __syncthreads();
    refine_axis_dev(T1, T2, 2 * n0 - 3, n1, n2, 1);
    __syncthreads();
    refine_axis_dev(T2, L, 2 * n0 - 3, 2 * n1 - 3, n2, 2);
}

// Final field at every voxel and the corrected image I / exp(B).
__global__ void __launch_bounds__(VH_TPB) k_n4_final(const float *__restrict__ I, float *out,
                                                    int64_t R, int64_t C, int64_t Z, int64_t V,
                                                    int64_t q2_cap, const double *P1,
                                                    DevLevel lv) {
    const int64_t b = blockIdx.y;
    const int64_t CZ = C * Z;
    const int64_t col = blockIdx.x * (int64_t)VH_TPB + threadIdx.x;
    if (col >= CZ) return;
    const int64_t y = col / Z, z = col % Z;
    const int ncy = lv.ax[1].ncp;
    const int by = lv.ax[1].base[y];
    const float4 wy = *reinterpret_cast<const float4 *>(lv.ax[1].w + 4 * y);
    const double *p1 = P1 + b * q2_cap;
    const DevAxis ax = lv.ax[0];
    int wb = ax.base[0];
    double t0 = col_T(p1, wb, ncy, Z, by, wy, z), t1 = col_T(p1, wb + 1, ncy, Z, by, wy, z);
    double t2 = col_T(p1, wb + 2, ncy, Z, by, wy, z), t3 = col_T(p1, wb + 3, ncy, Z, by, wy, z);
    for (int64_t x = 0; x < R; ++x) {
        const int bx = ax.base[x];
        while (wb < bx) {
            ++wb;
            t0 = t1; t1 = t2; t2 = t3;
            t3 = col_T(p1, wb + 3, ncy, Z, by, wy, z);
        }
        const float4 w = *reinterpret_cast<const float4 *>(ax.w + 4 * x);
        const float bn = (float)((double)w.x * t0 + (double)w.y * t1 + (double)w.z * t2 + (double)w.w * t3);
        const int64_t v = b * V + x * CZ + col;
        out[v] = I[v] / (float)exp((double)bn);
    }
}

// ---------------------------------------------------------------------------------------------
// host driver
// ---------------------------------------------------------------------------------------------
void vh_launch_n4(vh_batch *b, const vh_n4_params &prm) {
    hipStream_t st = b->ctx->stream;
    vh_ensure_n4_workspace(b, prm);
    const dim3 cg = col_grid(b);
    const int64_t nparts = cg.x;
    const int bins = prm.n_bins;
    const double masked_bytes = (double)b->V;   // refined per kernel below
    (void)masked_bytes;
    float *U = b->d_n4;   // U = L0 - B lives in the output buffer until k_n4_final overwrites it
    HIP_TRY(hipMemsetAsync(b->d_lat, 0, sizeof(float) * b->nb * b->lat_cap, st));
    k_n4_state_init<<<(unsigned)((b->nb + 255) / 256), 256, 0, st>>>(b->d_st, b->nb);
    VH_CHECK_LAUNCH();
    int total_iters = 0;
    for (int L = 0; L < prm.n_levels; ++L) total_iters += prm.max_iters[L];
    HIP_TRY(hipMemsetAsync(b->d_nactive, 0, sizeof(int32_t) * (total_iters + 1), st));
    {
        ScopedKTimer tm(b, "n4_init", 0.0);
        k_n4_init<<<cg, VH_TPB, 0, st>>>(b->d_hp, b->d_colbits, b->d_colrange, b->d_sc, b->R,
                                         b->CZ, b->V, b->d_L0, b->d_B, U, b->d_st);
        VH_CHECK_LAUNCH();
    }
    const int LOOK = 3;
    std::vector<hipEvent_t> evs;
    int32_t *hflag = b->ctx->h_pinned;
    int gi = 0;   // global iteration slot
    for (int L = 0; L < prm.n_levels; ++L) {
        const DevLevel lv = dev_level(b, prm, L);
        const FitTile ftile = fit_tile(b->C, b->Z);
        const dim3 fg((unsigned)(ftile.nty * ftile.ntz), (unsigned)b->nb);
        const size_t fit_lds = sizeof(double) * (size_t)lv.ax[0].ncp * VH_TPB;
        {
            ScopedKTimer tm(b, "n4_den", 0.0);
            k_n4_fitblock<1><<<fg, VH_TPB, fit_lds, st>>>(U, b->d_colbits, b->d_colrange, b->R,
                                                          b->C, b->Z, b->V, bins, b->d_st, b->d_E,
                                                          lv, b->lat_cap, b->d_fitpart);
            VH_CHECK_LAUNCH();
            k_n4_tilesum<1><<<(unsigned)b->nb, VH_TPB, 0, st>>>(b->d_fitpart, b->lat_cap, b->d_lat,
                                                                b->d_den, b->d_P1, b->C, b->Z,
                                                                b->lat_cap, b->q2_cap, b->d_st, lv);
            VH_CHECK_LAUNCH();
        }
        const int level_start = (int)evs.size();
        for (int it = 0; it < prm.max_iters[L]; ++it, ++gi) {
            k_n4_ctrl<<<(unsigned)((b->nb + 255) / 256), 256, 0, st>>>(
                b->d_st, b->d_part, nparts, b->d_sc, L, it, prm.conv_threshold, bins, b->nb,
                b->d_hist, b->d_nactive + gi);
            VH_CHECK_LAUNCH();
            HIP_TRY(hipMemcpyAsync(hflag + (gi % 1024), b->d_nactive + gi, sizeof(int32_t),
                                   hipMemcpyDeviceToHost, st));
            hipEvent_t ev;
            HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            HIP_TRY(hipEventRecord(ev, st));
            evs.push_back(ev);
            k_n4_exact_min<<<(unsigned)b->nb, VH_TPB, 0, st>>>(U, b->d_mask, b->V, bins,
                                                               b->d_st);
            VH_CHECK_LAUNCH();
            {
                ScopedKTimer tm(b, "n4_hist", 0.0);
                k_n4_hist<<<cg, VH_TPB, 0, st>>>(U, b->d_colbits, b->d_colrange, b->R, b->CZ,
                                                 b->V, bins, b->d_st, b->d_hist);
                VH_CHECK_LAUNCH();
            }
            k_n4_emap<<<(unsigned)b->nb, VH_TPB, 0, st>>>(b->d_hist, b->d_twiddle, bins, prm.fwhm,
                                                           prm.wiener_noise, b->d_st, b->d_E);
            VH_CHECK_LAUNCH();
            {
                ScopedKTimer tm(b, "n4_fit", 0.0);
                k_n4_fitblock<0><<<fg, VH_TPB, fit_lds, st>>>(U, b->d_colbits, b->d_colrange,
                                                              b->R, b->C, b->Z, b->V, bins,
                                                              b->d_st, b->d_E, lv, b->lat_cap,
                                                              b->d_fitpart);
                VH_CHECK_LAUNCH();
            }
            {
                ScopedKTimer tm(b, "n4_contract", 0.0);
                k_n4_tilesum<0><<<(unsigned)b->nb, VH_TPB, 0, st>>>(
                    b->d_fitpart, b->lat_cap, b->d_lat, b->d_den, b->d_P1, b->C, b->Z, b->lat_cap,
                    b->q2_cap, b->d_st, lv);
                VH_CHECK_LAUNCH();
            }
            {
                ScopedKTimer tm(b, "n4_eval", 0.0);
                k_n4_eval<<<cg, VH_TPB, 0, st>>>(b->d_L0, b->d_B, U, b->d_colbits,
                                                 b->d_colrange, b->d_sc, b->R, b->C, b->Z, b->V,
                                                 b->q2_cap, b->d_P1, lv, b->d_st, nparts,
                                                 b->d_part);
                VH_CHECK_LAUNCH();
            }
            const int k = (int)evs.size() - 1 - LOOK;
            if (k >= level_start) {
                HIP_TRY(hipEventSynchronize(evs[k]));
                if (hflag[(gi - LOOK) % 1024] == 0) { ++gi; break; }
            }
        }
        k_n4_level_end<<<(unsigned)((b->nb + 255) / 256), 256, 0, st>>>(b->d_st, b->d_part,
                                                                         nparts, b->d_sc, L, b->nb);
        VH_CHECK_LAUNCH();
        if (L < prm.n_levels - 1) {
            k_n4_refine<<<(unsigned)b->nb, VH_TPB, 0, st>>>(b->d_lat, b->lat_cap, b->nb,
                                                            lv.ax[0].ncp, lv.ax[1].ncp,
                                                            lv.ax[2].ncp);
            VH_CHECK_LAUNCH();
        }
    }
    {
        const DevLevel lv = dev_level(b, prm, prm.n_levels - 1);
        ScopedKTimer tm(b, "n4_final", 9.0 * (double)b->V);
        k_n4_final<<<cg, VH_TPB, 0, st>>>(b->d_hp, b->d_n4, b->R, b->C, b->Z, b->V, b->q2_cap,
                                          b->d_P1, lv);
        VH_CHECK_LAUNCH();
    }
    for (auto e : evs) HIP_TRY(hipEventDestroy(e));
}
