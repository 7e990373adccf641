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
#include <algorithm>
#include <cfloat>
#include <climits>
#include <cstring>

#include <hip/hip_cooperative_groups.h>

#include "n4_shared.h"

#define SEG_R 16    // rows per wave segment
#define N4_CH 4096  // compact voxels per chunk (flat sweeps: 256 threads x 16)
#define N4_VPT (N4_CH / VH_TPB)
#define HIST_COPIES 8   // LDS histogram copies (neighbouring lanes share bins)
#define FIT_WAVES 4     // fit items per block (one per wave)
#ifndef FIT_GS
#define FIT_GS FIT_G    // the sweep fit's rows per load group (fit_item FG)
#endif
#ifndef FIT_WPE
#define FIT_WPE 1       // the sweep fit's minimum waves per SIMD (launch bound; 1: no register cap)
#endif

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

int vh_level_ncp(const vh_n4_params &p, int level, int axis) {
    int n = p.ncp[axis];
    for (int l = 0; l < level; ++l) n = 2 * n - 3;
    return n;
}

void vh_n4_prepare_tables(vh_batch *b, const vh_n4_params &prm) {
    if (b->tabs_valid && same_params(b->tab_prm, prm)) return;
    const int64_t dims[3] = {b->R, b->C, b->Z};
    std::vector<uint8_t> blob;
    b->tab_off.assign((size_t)prm.n_levels * 3 * 8, 0);
    auto push = [&](const void *p, size_t bytes) {
        size_t off = (blob.size() + 15) & ~(size_t)15;
        blob.resize(off + bytes);
        std::memcpy(blob.data() + off, p, bytes);
        return off;
    };
    for (int L = 0; L < prm.n_levels; ++L) {
        int ms = 0;
        for (int a = 0; a < 3; ++a) ms = std::max(ms, vh_level_ncp(prm, L, a));
        const float eps = vh_bspline_eps(ms - 3);
        for (int a = 0; a < 3; ++a) {
            AxisTab t;
            vh_axis_tables((int)dims[a], vh_level_ncp(prm, L, a), eps, t);
            std::vector<double> inv(t.sw2.size()), w2(t.w.size()), w3(t.w.size()), w3i(t.w.size());
            for (size_t i = 0; i < inv.size(); ++i) inv[i] = 1.0 / t.sw2[i];
            for (size_t i = 0; i < w2.size(); ++i) {
                const double w = t.w[i];
                w2[i] = w * w;
                w3[i] = w * w * w;
                w3i[i] = w3[i] * inv[i / 4];   // S5 numerator row weight: w^3 / sum w^2
            }
            b->tab_off[(L * 3 + a) * 8 + 0] = push(t.base.data(), t.base.size() * 4);
            b->tab_off[(L * 3 + a) * 8 + 1] = push(t.w.data(), t.w.size() * 4);
            b->tab_off[(L * 3 + a) * 8 + 2] = push(t.sw2.data(), t.sw2.size() * 8);
            b->tab_off[(L * 3 + a) * 8 + 3] = push(inv.data(), inv.size() * 8);
            b->tab_off[(L * 3 + a) * 8 + 4] = push(w2.data(), w2.size() * 8);
            b->tab_off[(L * 3 + a) * 8 + 5] = push(w3.data(), w3.size() * 8);
            b->tab_off[(L * 3 + a) * 8 + 7] = push(w3i.data(), w3i.size() * 8);
            // control point k -> the index range whose 4-wide support contains k
            std::vector<int32_t> kr(2 * (size_t)t.ncp);
            for (int k = 0; k < t.ncp; ++k) {
                int lo = t.n, hi = -1;
                for (int idx = 0; idx < t.n; ++idx)
                    if (t.base[idx] <= k && k <= t.base[idx] + 3) {
                        lo = std::min(lo, idx);
                        hi = std::max(hi, idx);
                    }
                kr[2 * k] = lo;
                kr[2 * k + 1] = hi;
            }
            b->tab_off[(L * 3 + a) * 8 + 6] = push(kr.data(), kr.size() * 4);
        }
    }
    // per level: row-span starts of the row axis and the dense slice weights (S5 stage 1)
    b->lvx_off.assign((size_t)prm.n_levels * 3, 0);
    for (int L = 0; L < prm.n_levels; ++L) {
        const float eps = vh_bspline_eps(std::max({vh_level_ncp(prm, L, 0), vh_level_ncp(prm, L, 1),
                                                   vh_level_ncp(prm, L, 2)}) - 3);
        AxisTab tx, tz;
        vh_axis_tables((int)b->R, vh_level_ncp(prm, L, 0), eps, tx);
        vh_axis_tables((int)b->Z, vh_level_ncp(prm, L, 2), eps, tz);
        const int ncx = tx.ncp, ncz = tz.ncp;
        std::vector<int32_t> xst((size_t)ncx - 2);
        for (int i = 0; i <= ncx - 3; ++i) {
            int x = 0;
            while (x < b->R && tx.base[x] < i) ++x;
            xst[i] = i == ncx - 3 ? (int32_t)b->R : x;
        }
        std::vector<double> wk3((size_t)ncz * b->Z), wk2((size_t)ncz * b->Z);
        for (int k = 0; k < ncz; ++k)
            for (int64_t z = 0; z < b->Z; ++z) {
                const int d = k - tz.base[z];
                const bool in = d >= 0 && d <= 3;
                const double w = in ? (double)tz.w[4 * z + d] : 0.0;
                wk3[(size_t)k * b->Z + z] = in ? w * w * w : 0.0;
                wk2[(size_t)k * b->Z + z] = in ? w * w : 0.0;
            }
        b->lvx_off[L * 3 + 0] = push(xst.data(), xst.size() * 4);
        b->lvx_off[L * 3 + 1] = push(wk3.data(), wk3.size() * 8);
        b->lvx_off[L * 3 + 2] = push(wk2.data(), wk2.size() * 8);
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

DevLevel vh_dev_level(const vh_batch *b, const vh_n4_params &prm, int L) {
    DevLevel lv;
    const int64_t dims[3] = {b->R, b->C, b->Z};
    const uint8_t *base = (const uint8_t *)b->d_tabs;
    for (int a = 0; a < 3; ++a) {
        lv.ax[a].base = (const int32_t *)(base + b->tab_off[(L * 3 + a) * 8 + 0]);
        lv.ax[a].w = (const float *)(base + b->tab_off[(L * 3 + a) * 8 + 1]);
        lv.ax[a].sw2 = (const double *)(base + b->tab_off[(L * 3 + a) * 8 + 2]);
        lv.ax[a].isw2 = (const double *)(base + b->tab_off[(L * 3 + a) * 8 + 3]);
        lv.ax[a].w2 = (const double *)(base + b->tab_off[(L * 3 + a) * 8 + 4]);
        lv.ax[a].w3 = (const double *)(base + b->tab_off[(L * 3 + a) * 8 + 5]);
        lv.ax[a].krange = (const int2 *)(base + b->tab_off[(L * 3 + a) * 8 + 6]);
        lv.ax[a].w3i = (const double *)(base + b->tab_off[(L * 3 + a) * 8 + 7]);
        lv.ax[a].n = (int32_t)dims[a];
        lv.ax[a].ncp = vh_level_ncp(prm, L, a);
    }
    lv.xst = (const int32_t *)(base + b->lvx_off[L * 3 + 0]);
    lv.wk3 = (const double *)(base + b->lvx_off[L * 3 + 1]);
    lv.wk2 = (const double *)(base + b->lvx_off[L * 3 + 2]);
    return lv;
}

void vh_ensure_n4_workspace(vh_batch *b, const vh_n4_params &prm) {
    const int L = prm.n_levels - 1;
    const int64_t cx = vh_level_ncp(prm, L, 0), cy = vh_level_ncp(prm, L, 1), cz = vh_level_ncp(prm, L, 2);
    const int64_t lat = cx * cy * cz;
    const int64_t q2 = cx * cy * b->Z;
    if (b->V >= (int64_t)1 << 29) throw VhError{VH_ERR_ARG, "N4: volume too large (>= 2^29 voxels)"};
    b->rsh = 1;   // compact voxel index = (row << rsh) | column
    while (((int64_t)1 << b->rsh) < b->CZ) ++b->rsh;
    if (b->R >= ((int64_t)1 << (31 - b->rsh))) throw VhError{VH_ERR_ARG, "N4: rows x columns too large for the packed voxel index"};
    if (b->d_L0 == nullptr) {
        b->VS = (b->V + 63) & ~(int64_t)63;   // compact-array stride: 256-byte aligned volumes
        const int64_t nch = b->nb * ((b->VS + N4_CH - 1) / N4_CH);
        HIP_TRY(hipMalloc(&b->d_L0, sizeof(float) * b->nb * b->VS));
        // U and D three times: the study driver speculates up to two iterations past the last
        // decided one (rings of 3); the sweep driver keeps PC's p values in D's second third
        HIP_TRY(hipMalloc(&b->d_U, sizeof(float) * 3 * b->nb * b->VS));
        HIP_TRY(hipMalloc(&b->d_D, sizeof(float) * 3 * b->nb * b->VS));
        HIP_TRY(hipMalloc(&b->d_perm, sizeof(int32_t) * b->nb * b->VS));
        HIP_TRY(hipMalloc(&b->d_ridx, sizeof(int32_t) * b->nb * b->VS));
        HIP_TRY(hipMalloc(&b->d_cp, sizeof(int32_t) * (b->nb + 1)));
        HIP_TRY(hipMalloc(&b->d_cvol, sizeof(int32_t) * nch));
        HIP_TRY(hipMalloc(&b->d_hpart, sizeof(uint64_t) * nch * VH_MAX_BINS));
        HIP_TRY(hipMalloc(&b->d_cpart, sizeof(double) * 2 * nch));
        HIP_TRY(hipMalloc(&b->d_E, sizeof(float) * b->nb * VH_MAX_BINS));
        HIP_TRY(hipMalloc(&b->d_st, sizeof(N4State) * b->nb));
        HIP_TRY(hipMalloc(&b->d_nactive, sizeof(int32_t) * 8 * 1024));
    }
    if (lat > b->lat_cap) {
        if (b->d_lat) HIP_TRY(hipFree(b->d_lat));
        if (b->d_numfix) HIP_TRY(hipFree(b->d_numfix));
        if (b->d_den) HIP_TRY(hipFree(b->d_den));
        HIP_TRY(hipMalloc(&b->d_lat, sizeof(float) * 3 * b->nb * lat));   // lattice + 2 scratch
        HIP_TRY(hipMalloc(&b->d_numfix, sizeof(uint64_t) * 2 * b->nb * lat));
        HIP_TRY(hipMalloc(&b->d_den, sizeof(double) * b->nb * lat));
        b->lat_cap = lat;
    }
    if (cx > 64) throw VhError{VH_ERR_ARG, "N4 lattice too fine: > 64 control points along rows"};
    const int64_t ntiles = (b->CZ + TILE_W - 1) / TILE_W;
    if (b->d_rowstart == nullptr || b->n4_tiles != ntiles) {
        if (b->d_rowstart) HIP_TRY(hipFree(b->d_rowstart));
        if (b->d_rowmask) HIP_TRY(hipFree(b->d_rowmask));
        if (b->d_rrank) HIP_TRY(hipFree(b->d_rrank));
        HIP_TRY(hipMalloc(&b->d_rowstart, sizeof(int32_t) * b->nb * ntiles * b->R));
        HIP_TRY(hipMalloc(&b->d_rowmask, sizeof(uint64_t) * b->nb * ntiles * b->R));
        HIP_TRY(hipMalloc(&b->d_rrank, sizeof(int32_t) * b->nb * ntiles * b->R));
        b->n4_tiles = ntiles;
    }
    if (cx * b->CZ > b->t_cap) {
        if (b->d_T) HIP_TRY(hipFree(b->d_T));
        HIP_TRY(hipMalloc(&b->d_T, sizeof(float) * 2 * b->nb * cx * b->CZ));
        b->t_cap = cx * b->CZ;
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

// Convergence measure from the eval partials (one slot per chunk of the volume), reduced by one
// wave in a fixed order (lane l sums slots l, l+64, ...; then a shuffle tree): deterministic.
__device__ __forceinline__ double conv_from_parts(const double *part, const int32_t *cp, int64_t b,
                                                  double N) {
    const int lane = threadIdx.x & 63;
    double sd = 0.0, sd2 = 0.0;
    for (int64_t p = cp[b] + lane; p < cp[b + 1]; p += 64) {
        sd += part[p * 2];
        sd2 += part[p * 2 + 1];
    }
    for (int off = 32; off > 0; off >>= 1) {
        sd += __shfl_down(sd, off, 64);
        sd2 += __shfl_down(sd2, off, 64);
    }
    sd = __shfl(sd, 0, 64);
    sd2 = __shfl(sd2, 0, 64);
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
    s.tlast = 0;
    st[b] = s;
}

// ---------------------------------------------------------------------------------------------
// Compact N4 state.  The mask==1 voxels of a volume are stored in "tile-row" order: column tiles
// of 64 consecutive (col, slice) columns -- one wave, one lane per column -- then rows, then the
// set lanes of that row in lane order.  rs[b][tile][x] is the start of (tile, row x); a lane's
// slot is rs + mbcnt(ballot(its bit)).  A wave processes one tile x 16-row segment: 16 coalesced
// loads per array in flight, only masked bytes move, one memory round trip per wave.
// ---------------------------------------------------------------------------------------------

__device__ __forceinline__ __amdgpu_buffer_rsrc_t vol_rsrc(const float *base, int64_t V) {
    return __builtin_amdgcn_make_buffer_rsrc((void *)base, 0, (int)(V * 4), 0x00020000);
}
__device__ __forceinline__ float bload(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, 0, 0));
}
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t r, uint32_t voff, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, (int)voff, 0, 0);
}

struct Seg {
    int64_t col;      // this lane's column
    int tile, x0;     // wave-uniform tile and first row
    uint32_t m;       // this lane's mask==1 bits for rows x0..x0+15
    uint32_t off[SEG_R];   // byte offsets into the volume's compact arrays (VH_OOB when unset)
};

// one wave = (tile, 16-row segment); x0 multiple of 16 so the bits sit in one 32-row word
__device__ __forceinline__ void seg_begin(Seg &s, const uint32_t *colbits, const int32_t *rs,
                                          int64_t b, int64_t R, int64_t CZ, int64_t ntiles,
                                          int tile, int x0) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (R + 31) >> 5;
    s.tile = tile;
    s.x0 = x0;
    s.col = (int64_t)tile * TILE_W + lane;
    s.m = 0u;
    if (s.col < CZ && x0 < R) s.m = (colbits[(b * nw + (x0 >> 5)) * CZ + s.col] >> (x0 & 31)) & 0xffffu;
    const int32_t *r = rs + (b * ntiles + tile) * R;
#pragma unroll
    for (int k = 0; k < SEG_R; ++k) {
        const bool on = (s.m >> k) & 1u;
        const uint64_t bal = __ballot(on);
        const int32_t rk = x0 + k < R ? r[x0 + k] : 0;   // wave-uniform guard: ragged last segment
        s.off[k] = on ? (uint32_t)((rk + lanes_below(bal)) * 4) : VH_OOB;
    }
}

// per (volume, tile, row): number of mask==1 lanes (pass 1 of the compact offsets) and the lane
// mask itself (the volume-resident driver walks tile rows from it)
__global__ void __launch_bounds__(64) k_n4_rowcount(const uint32_t *colbits, int64_t R,
                                                   int64_t CZ, int64_t ntiles, int32_t *rs,
                                                   uint64_t *rowmask) {
    const int64_t b = blockIdx.y;
    const int tile = blockIdx.x;
    const int64_t col = (int64_t)tile * TILE_W + threadIdx.x;
    const int64_t nw = (R + 31) >> 5;
    int32_t *out = rs + (b * ntiles + tile) * R;
    uint64_t *rm = rowmask + (b * ntiles + tile) * R;
    // 4 bitmap words' loads in flight (unconditional at a clamped column), then per word 32 row
    // ballots, row k's mask kept by lane k, and lanes 0..31 store their rows together (lane 0
    // storing every row after its ballot took 58 us per batch)
    const int lane = threadIdx.x;
    const int64_t cl = col < CZ ? col : CZ - 1;
    for (int64_t w0 = 0; w0 < nw; w0 += 4) {
        uint32_t bits[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t v = colbits[(b * nw + (w0 + q < nw ? w0 + q : nw - 1)) * CZ + cl];
            bits[q] = col < CZ ? v : 0u;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t w = w0 + q;
            if (w >= nw) break;   // wave-uniform
            uint64_t mine = 0ull;
#pragma unroll
            for (int k = 0; k < 32; ++k) {
                const uint64_t bal = __ballot((bits[q] >> k) & 1u);
                mine = lane == k ? bal : mine;
            }
            const int64_t x = w * 32 + lane;
            if (lane < 32 && x < R) {
                out[x] = __popcll(mine);
                rm[x] = mine;
            }
        }
    }
}

// exclusive scan of VH_TPB partials in LDS by one wave (integers: exact in any order)
__device__ __forceinline__ void excl_scan_parts(int64_t *s_part) {
    const int t = threadIdx.x;
    if (t < 64) {
        int64_t v[VH_TPB / 64], tot = 0;
#pragma unroll
        for (int q = 0; q < VH_TPB / 64; ++q) { v[q] = s_part[t * (VH_TPB / 64) + q]; tot += v[q]; }
        int64_t inc = tot;
        for (int off = 1; off < 64; off <<= 1) {
            const int64_t o = __shfl_up(inc, off, 64);
            if (t >= off) inc += o;
        }
        int64_t run = inc - tot;
#pragma unroll
        for (int q = 0; q < VH_TPB / 64; ++q) { s_part[t * (VH_TPB / 64) + q] = run; run += v[q]; }
    }
}
#define RSB 16   // loads per batch, all in flight (unconditional, clamped index): a loop of guarded
                 // loads waits for each one in turn (k_n4_rowscan + k_n4_rrank took 0.1 ms per batch)

// pass 2: exclusive scan over (tile, row) in tile-major order, one block per volume
__global__ void __launch_bounds__(VH_TPB) k_n4_rowscan(int32_t *rs, int64_t n) {
    __shared__ int64_t s_part[VH_TPB];
    const int64_t b = blockIdx.x;
    int32_t *a = rs + b * n;
    const int t = threadIdx.x;
    const int64_t per = (n + VH_TPB - 1) / VH_TPB;
    const int64_t s0 = t * per < n ? t * per : n, e0 = s0 + per < n ? s0 + per : n;
    int64_t acc = 0;
    for (int64_t i0 = s0; i0 < e0; i0 += RSB) {
        int32_t v[RSB];
#pragma unroll
        for (int q = 0; q < RSB; ++q) v[q] = a[i0 + q < e0 ? i0 + q : s0];
#pragma unroll
        for (int q = 0; q < RSB; ++q) acc += i0 + q < e0 ? v[q] : 0;
    }
    s_part[t] = acc;
    __syncthreads();
    excl_scan_parts(s_part);
    __syncthreads();
    int64_t run = s_part[t];
    for (int64_t i0 = s0; i0 < e0; i0 += RSB) {
        int32_t v[RSB];
#pragma unroll
        for (int q = 0; q < RSB; ++q) v[q] = a[i0 + q < e0 ? i0 + q : s0];
#pragma unroll
        for (int q = 0; q < RSB; ++q)
            if (i0 + q < e0) { a[i0 + q] = (int32_t)run; run += v[q]; }
    }
}

// ---- the same two scans for large volumes, over the whole GPU (config 5: the one-workgroup forms
// above took 3.5 + 3.9 ms of a 154 ms study) -------------------------------------------------------
#define RS_CH 4096   // entries per chunk of the flat row-start scan (16 per thread)
__device__ __forceinline__ int32_t block_excl_scan_i32(int32_t v, int32_t *s_w, int32_t &total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int32_t inc = v;
    for (int off = 1; off < 64; off <<= 1) {
        const int32_t y = __shfl_up(inc, off, 64);
        if (lane >= off) inc += y;
    }
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    int32_t base = 0;
    total = 0;
    for (int q = 0; q < VH_TPB / 64; ++q) {
        if (q < w) base += s_w[q];
        total += s_w[q];
    }
    return base + inc - v;
}
// pass 1: chunk sums
__global__ void __launch_bounds__(VH_TPB) k_n4_rowscan_parts(const int32_t *rs, int64_t n, int32_t *parts,
                                                            int64_t ncs) {
    __shared__ int32_t s_w[VH_TPB / 64];
    const int64_t b = blockIdx.y, c0 = (int64_t)blockIdx.x * RS_CH;
    const int32_t *a = rs + b * n;
    int32_t acc = 0;
    for (int64_t i = c0 + threadIdx.x; i < n && i < c0 + RS_CH; i += VH_TPB) acc += a[i];
    int32_t tot;
    (void)block_excl_scan_i32(acc, s_w, tot);
    if (threadIdx.x == 0) parts[b * ncs + blockIdx.x] = tot;
}
// pass 2: exclusive scan of the chunk sums of each volume (in place)
__global__ void __launch_bounds__(VH_TPB) k_n4_rowscan_top(int32_t *parts, int64_t ncs) {
    __shared__ int32_t s_w[VH_TPB / 64];
    int32_t *p = parts + blockIdx.x * ncs;
    int32_t carry = 0;
    for (int64_t c0 = 0; c0 < ncs; c0 += VH_TPB) {
        const int64_t i = c0 + threadIdx.x;
        const int32_t v = i < ncs ? p[i] : 0;
        int32_t tot;
        const int32_t ex = block_excl_scan_i32(v, s_w, tot);
        if (i < ncs) p[i] = carry + ex;
        carry += tot;
        __syncthreads();
    }
}
// pass 3: each chunk's exclusive scan (16 consecutive entries per thread) plus its offset, in place
__global__ void __launch_bounds__(VH_TPB) k_n4_rowscan_apply(int32_t *rs, int64_t n, const int32_t *parts,
                                                            int64_t ncs) {
    __shared__ int32_t s_w[VH_TPB / 64];
    const int64_t b = blockIdx.y, c0 = (int64_t)blockIdx.x * RS_CH;
    int32_t *a = rs + b * n;
    const int64_t i0 = c0 + (int64_t)threadIdx.x * (RS_CH / VH_TPB);
    int32_t v[RS_CH / VH_TPB];
    int32_t acc = 0;
#pragma unroll
    for (int q = 0; q < RS_CH / VH_TPB; ++q) {
        v[q] = i0 + q < n ? a[i0 + q] : 0;
        acc += v[q];
    }
    int32_t tot;
    int32_t run = parts[b * ncs + blockIdx.x] + block_excl_scan_i32(acc, s_w, tot);
#pragma unroll
    for (int q = 0; q < RS_CH / VH_TPB; ++q)
        if (i0 + q < n) {
            a[i0 + q] = run;
            run += v[q];
        }
}
// raster ranks, pass 1: per (chunk of 64 tiles, volume) and row, the running count over the chunk's
// tiles (local) and the chunk's total per row (rows across threads: coalesced)
#define RR_CH 64
__global__ void __launch_bounds__(VH_TPB) k_n4_rr_chunk(const uint64_t *rowmask, int64_t R, int64_t ntiles,
                                                       int32_t *rrank, int32_t *ctot, int64_t nrc) {
    const int64_t b = blockIdx.y, t0 = (int64_t)blockIdx.x * RR_CH;
    const int64_t t1 = t0 + RR_CH < ntiles ? t0 + RR_CH : ntiles;
    const uint64_t *rm = rowmask + b * ntiles * R;
    int32_t *rr = rrank + b * ntiles * R;
    for (int64_t x = threadIdx.x; x < R; x += VH_TPB) {
        int32_t run = 0;
        for (int64_t t = t0; t < t1; ++t) {
            rr[t * R + x] = run;
            run += __popcll(rm[t * R + x]);
        }
        ctot[(b * (nrc + 1) + blockIdx.x) * R + x] = run;
    }
}
// pass 2 (one block per volume): per row, exclusive prefix over the chunks (in place); the row
// totals' exclusive prefix over the rows into the extra chunk row nrc
__global__ void __launch_bounds__(VH_TPB) k_n4_rr_top(int32_t *ctot, int64_t R, int64_t nrc) {
    __shared__ int32_t s_w[VH_TPB / 64];
    int32_t *c = ctot + blockIdx.x * (nrc + 1) * R;
    int32_t carry = 0;
    for (int64_t x0 = 0; x0 < R; x0 += VH_TPB) {
        const int64_t x = x0 + threadIdx.x;
        int32_t run = 0;
        if (x < R)
            for (int64_t q = 0; q < nrc; ++q) {
                const int32_t v = c[q * R + x];
                c[q * R + x] = run;
                run += v;
            }
        int32_t tot;
        const int32_t ex = block_excl_scan_i32(x < R ? run : 0, s_w, tot);
        if (x < R) c[nrc * R + x] = carry + ex;
        carry += tot;
        __syncthreads();
    }
}
// pass 3: the chunk offset and the row base added to every (tile, row)
__global__ void __launch_bounds__(VH_TPB) k_n4_rr_apply(int64_t R, int64_t ntiles, int32_t *rrank,
                                                       const int32_t *ctot, int64_t nrc) {
    const int64_t b = blockIdx.y, t0 = (int64_t)blockIdx.x * RR_CH;
    const int64_t t1 = t0 + RR_CH < ntiles ? t0 + RR_CH : ntiles;
    const int32_t *c = ctot + b * (nrc + 1) * R;
    int32_t *rr = rrank + b * ntiles * R;
    for (int64_t x = threadIdx.x; x < R; x += VH_TPB) {
        const int32_t off = c[blockIdx.x * R + x] + c[nrc * R + x];
        for (int64_t t = t0; t < t1; ++t) rr[t * R + x] += off;
    }
}

// Raster rank of the first masked voxel of every (tile, row): masked voxels before row x plus
// those of row x in tiles before t -- the position of the voxel in ITK's raster-order scans (the
// convergence recurrence S7).  One block per volume; dynamic LDS holds the R row totals.
__global__ void __launch_bounds__(VH_TPB) k_n4_rrank(const uint64_t *rowmask, const int32_t *rowstart,
                                                    int64_t R, int64_t ntiles, int64_t VS,
                                                    int32_t *rrank, int32_t *perm) {
    extern __shared__ int32_t s_rowtot[];   // [R]
    __shared__ int64_t s_part[VH_TPB];
    const int64_t b = blockIdx.x;
    const uint64_t *rm = rowmask + b * ntiles * R;
    int32_t *rr = rrank + b * ntiles * R;
    for (int64_t x = threadIdx.x; x < R; x += VH_TPB) {   // row totals
        int32_t run = 0;
        for (int64_t t0 = 0; t0 < ntiles; t0 += RSB) {
            uint64_t m[RSB];
#pragma unroll
            for (int q = 0; q < RSB; ++q) m[q] = rm[(t0 + q < ntiles ? t0 + q : 0) * R + x];
#pragma unroll
            for (int q = 0; q < RSB; ++q) run += t0 + q < ntiles ? __popcll(m[q]) : 0;
        }
        s_rowtot[x] = run;
    }
    __syncthreads();
    const int t = threadIdx.x;
    const int64_t per = (R + VH_TPB - 1) / VH_TPB;
    const int64_t s0 = t * per < R ? t * per : R, e0 = s0 + per < R ? s0 + per : R;
    int64_t acc = 0;
    for (int64_t i = s0; i < e0; ++i) acc += s_rowtot[i];
    s_part[t] = acc;
    __syncthreads();
    excl_scan_parts(s_part);
    __syncthreads();
    int32_t run = (int32_t)s_part[t];
    for (int64_t i = s0; i < e0; ++i) { const int32_t v = s_rowtot[i]; s_rowtot[i] = run; run += v; }
    __syncthreads();
    // raster rank of each (tile, row)'s first masked voxel = masked voxels of the rows before x
    // plus those of row x in the tiles before; perm (raster rank -> compact index, the sweep
    // driver's convergence walk) is scattered by k_n4_perm over the whole GPU (one workgroup here
    // took 22 ms at 512^3)
    for (int64_t x = threadIdx.x; x < R; x += VH_TPB) {
        int32_t r = s_rowtot[x];
        for (int64_t t0 = 0; t0 < ntiles; t0 += RSB) {
            uint64_t m[RSB];
#pragma unroll
            for (int q = 0; q < RSB; ++q) m[q] = rm[(t0 + q < ntiles ? t0 + q : 0) * R + x];
#pragma unroll
            for (int q = 0; q < RSB; ++q)
                if (t0 + q < ntiles) { rr[(t0 + q) * R + x] = r; r += __popcll(m[q]); }
        }
    }
}

// One stage of a 32 x 32 bit-matrix transpose (element (i, j) = bit j of A[i]): rows k and k + J
// (k with bit J clear) swap the J-bit blocks above / below the diagonal.
template <int J>
__device__ __forceinline__ void bit_swap_stage(uint32_t (&A)[32], uint32_t m) {
#pragma unroll
    for (int k0 = 0; k0 < 32; k0 += 2 * J)
#pragma unroll
        for (int k = k0; k < k0 + J; ++k) {
            const uint32_t tt = ((A[k] >> J) ^ A[k + J]) & m;
            A[k] ^= tt << J;
            A[k + J] ^= tt;
        }
}

// k_n4_rowcount + k_n4_rowscan + k_n4_rrank in one workgroup of 1024 threads per volume, for
// volumes with nrs = tiles x R <= RP_MAX_NRS.  Each thread takes 16 columns of one bitmap word
// (32 rows) and transposes them into 32 16-bit row pieces (a bit-matrix transpose: ~400 bit
// operations instead of 32 ballots and their 64-bit selects per word): the quarter (c % 64) / 16 of
// the (tile, row) lane masks, stored as 16-bit pieces of the u64 rowmask, and their popcounts added
// into the (tile, row) counts in LDS.  Then from that LDS copy: raster ranks (row totals, their scan,
// each row's running count over the tiles) and the compact offsets (the exclusive scan in tile-major
// order).  Integers only: the same values as the three kernels.
#define RP_MAX_NRS 16384
#define RP_MAX_R 4096
#define RP_TPB 1024
__global__ void __launch_bounds__(RP_TPB) k_n4_rowprep(const uint32_t *colbits, int64_t R, int64_t CZ,
                                                      int64_t ntiles, int32_t *rs, uint64_t *rowmask,
                                                      int32_t *rrank) {
    extern __shared__ int32_t s_dyn[];   // [nrs] counts, then [R] row totals -> row bases
    __shared__ int64_t s_part[RP_TPB];
    const int64_t b = blockIdx.x, nrs = ntiles * R;
    const int64_t nw = (R + 31) >> 5;
    int32_t *s_cnt = s_dyn, *s_row = s_dyn + nrs;
    const int t = threadIdx.x;
    for (int64_t i = t; i < nrs; i += RP_TPB) s_cnt[i] = 0;
    __syncthreads();
    const int64_t nq = ntiles * 4;   // 16-column groups, the last tile's past CZ included (zeros)
    uint16_t *rm16 = reinterpret_cast<uint16_t *>(rowmask + b * nrs);
    for (int64_t item = t; item < nw * nq; item += RP_TPB) {
        const int64_t w = item / nq, g = item - w * nq, c0 = g * 16;
        const uint32_t *src = colbits + (b * nw + w) * CZ;
        uint32_t A[32];
#pragma unroll
        for (int i = 0; i < 16; ++i) {   // unconditional at a clamped column: the 16 loads in flight
            const int64_t c = c0 + i;
            const uint32_t v = src[c < CZ ? c : CZ - 1];
            const uint32_t x = c < CZ ? v : 0u;
            A[i] = x & 0xFFFFu;
            A[i + 16] = x >> 16;
        }
        bit_swap_stage<8>(A, 0x00FF00FFu);   // (the first stage, J = 16, was the split above)
        bit_swap_stage<4>(A, 0x0F0F0F0Fu);
        bit_swap_stage<2>(A, 0x33333333u);
        bit_swap_stage<1>(A, 0x55555555u);
        // A[k] bit i: column c0 + i at row 32 w + k
        const int64_t tile = g >> 2, x0 = w * 32;
        uint16_t *dst = rm16 + (tile * R + x0) * 4 + (g & 3);
        int32_t *cnt = s_cnt + tile * R + x0;
#pragma unroll
        for (int k = 0; k < 32; ++k)
            if (x0 + k < R) {
                dst[4 * k] = (uint16_t)A[k];
                if (A[k]) atomicAdd(&cnt[k], __popc(A[k]));
            }
    }
    __syncthreads();
    for (int64_t x = t; x < R; x += RP_TPB) {   // row totals over the tiles
        int32_t run = 0;
        for (int64_t tt = 0; tt < ntiles; ++tt) run += s_cnt[tt * R + x];
        s_row[x] = run;
    }
    __syncthreads();
    auto block_excl = [&](int32_t *a, int64_t n, int32_t *out_g) {
        // exclusive scan of a[0, n) in place (thread chunks, then one wave over the partials); with
        // out_g the scanned values go to global memory instead (a keeps the counts)
        const int64_t per = (n + RP_TPB - 1) / RP_TPB;
        const int64_t s0 = t * per < n ? t * per : n, e0 = s0 + per < n ? s0 + per : n;
        int64_t acc = 0;
        for (int64_t i = s0; i < e0; ++i) acc += a[i];
        s_part[t] = acc;
        __syncthreads();
        if (t < 64) {
            int64_t v[RP_TPB / 64], tot = 0;
#pragma unroll
            for (int q = 0; q < RP_TPB / 64; ++q) { v[q] = s_part[t * (RP_TPB / 64) + q]; tot += v[q]; }
            int64_t inc = tot;
            for (int off = 1; off < 64; off <<= 1) {
                const int64_t o = __shfl_up(inc, off, 64);
                if (t >= off) inc += o;
            }
            int64_t run = inc - tot;
#pragma unroll
            for (int q = 0; q < RP_TPB / 64; ++q) { s_part[t * (RP_TPB / 64) + q] = run; run += v[q]; }
        }
        __syncthreads();
        int32_t run = (int32_t)s_part[t];
        for (int64_t i = s0; i < e0; ++i) {
            const int32_t v = a[i];
            if (out_g) out_g[i] = run; else a[i] = run;
            run += v;
        }
        __syncthreads();
    };
    block_excl(s_row, R, nullptr);   // row bases: masked voxels of the rows before
    int32_t *rr = rrank + b * nrs;
    for (int64_t x = t; x < R; x += RP_TPB) {   // raster rank of each (tile, row)'s first masked voxel
        int32_t r = s_row[x];
        for (int64_t tt = 0; tt < ntiles; ++tt) { rr[tt * R + x] = r; r += s_cnt[tt * R + x]; }
    }
    block_excl(s_cnt, nrs, rs + b * nrs);   // compact offsets, tile-major
}

// perm[raster rank] = compact index: one wave per (tile, row), one lane per column of the tile
__global__ void __launch_bounds__(VH_TPB) k_n4_perm(const uint64_t *rowmask, const int32_t *rowstart,
                                                   const int32_t *rrank, int64_t R, int64_t ntiles,
                                                   int64_t VS, int32_t *perm) {
    const int64_t b = blockIdx.y;
    const int64_t e = (int64_t)blockIdx.x * (VH_TPB / 64) + (threadIdx.x >> 6);   // tile * R + row
    if (e >= ntiles * R) return;
    const int lane = threadIdx.x & 63;
    const int64_t o = b * ntiles * R + e;
    const uint64_t m = rowmask[o];
    if (!((m >> lane) & 1ull)) return;
    const int32_t i = __popcll(m & ((1ull << lane) - 1ull));
    perm[b * VS + rrank[o] + i] = rowstart[o] + i;
}

// L0 = log(I) at mask == 1 (non-positive -> 0), U = L0 (B = 0), ridx = (row << rsh) | column
// (compact, volume stride VS) and the first U range.  grid (ceil(tiles/4), segments, volumes), 4 tile-waves/block.
__global__ void __launch_bounds__(VH_TPB) k_n4_init(const float *__restrict__ I,
                                                   const uint32_t *__restrict__ colbits,
                                                   const int32_t *rs, const VolScalars *sc,
                                                   int64_t R, int64_t CZ, int64_t V, int64_t VS,
                                                   int64_t ntiles, float *L0, float *U,
                                                   int32_t *ridx, int rsh, N4State *st) {
    const int64_t b = blockIdx.z;
    const int tile = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tile >= ntiles) return;
    Seg s;
    seg_begin(s, colbits, rs, b, R, CZ, ntiles, tile, blockIdx.y * SEG_R);
    const __amdgpu_buffer_rsrc_t rL = vol_rsrc(L0 + b * VS, VS), rU = vol_rsrc(U + b * VS, VS),
                                 rR = vol_rsrc((const float *)(ridx + b * VS), VS);
    const int64_t first = sc[b].first_masked;
    uint32_t kmax = 0u, kmin = 0xffffffffu;
#pragma unroll
    for (int k = 0; k < SEG_R; ++k) {
        if (!((s.m >> k) & 1u)) continue;
        const int64_t r = (int64_t)(s.x0 + k) * CZ + s.col;
        const float a = I[b * V + r];
        const float l = a > 0.0f ? (float)log((double)a) : 0.0f;
        bstore(rL, s.off[k], l);
        bstore(rU, s.off[k], l);
        bstore(rR, s.off[k], __int_as_float(((s.x0 + k) << rsh) | (int)s.col));
        const uint32_t key = f2key(l);
        kmax = key > kmax ? key : kmax;
        if (r == first) st[b].u_first = l;
        else kmin = key < kmin ? key : kmin;
    }
    kmax = wave_max_u32(kmax);
    kmin = wave_min_u32(kmin);
    if ((threadIdx.x & 63) == 0) {
        if (kmax) atomicMax(&st[b].umax_key, kmax);
        if (kmin != 0xffffffffu) atomicMin(&st[b].umin_key, kmin);
    }
}

// Chunk table: volume b's compact voxels split into chunks of N4_CH; cp = exclusive prefix of the
// chunk counts, cvol[c] = owning volume.  One block.
__global__ void __launch_bounds__(VH_TPB) k_n4_chunks(const VolScalars *sc, int64_t nb,
                                                     int32_t *cp, int32_t *cvol) {
    __shared__ int32_t s_part[VH_TPB];
    const int t = threadIdx.x;
    const int64_t per = (nb + VH_TPB - 1) / VH_TPB;
    const int64_t s0 = t * per < nb ? t * per : nb, e0 = s0 + per < nb ? s0 + per : nb;
    int32_t acc = 0;
    for (int64_t b = s0; b < e0; ++b) acc += (int32_t)((sc[b].n_mask1 + N4_CH - 1) / N4_CH);
    s_part[t] = acc;
    __syncthreads();
    if (t == 0) {
        int32_t run = 0;
        for (int i = 0; i < VH_TPB; ++i) { const int32_t v = s_part[i]; s_part[i] = run; run += v; }
        cp[nb] = run;
    }
    __syncthreads();
    int32_t run = s_part[t];
    for (int64_t b = s0; b < e0; ++b) {
        const int32_t n = (int32_t)((sc[b].n_mask1 + N4_CH - 1) / N4_CH);
        cp[b] = run;
        for (int32_t c = 0; c < n; ++c) cvol[run + c] = (int32_t)b;
        run += n;
    }
}

// Exact ITK bin minimum when the first masked pixel is the strict minimum: min over the pixels
// that are not running maxima in raster order (chunked prefix-max scan over rows).  Rare path;
// each thread walks whole rows, tracking compact offsets incrementally.
__device__ __forceinline__ void exact_row_scan(const float *Uv, const uint32_t *colbits,
                                               const int32_t *rs, int64_t b, int64_t R, int64_t CZ,
                                               int64_t ntiles, int64_t x, float &run, float &mn,
                                               bool track_min) {
    const int64_t nw = (R + 31) >> 5;
    int64_t off = 0;
    for (int64_t col = 0; col < CZ; ++col) {
        if ((col & (TILE_W - 1)) == 0) off = rs[(b * ntiles + col / TILE_W) * R + x];
        if (!((colbits[(b * nw + (x >> 5)) * CZ + col] >> (x & 31)) & 1u)) continue;
        const float u = Uv[off++];
        if (u > run) run = u;
        else if (track_min && u < mn) mn = u;
    }
}

__device__ float exact_min_block(const float *Uv, const uint32_t *colbits, const int32_t *rs,
                                 int64_t b, int64_t R, int64_t CZ, int64_t ntiles) {
    __shared__ float s_cmax[VH_TPB];
    __shared__ float s_min[VH_TPB];
    const int t = threadIdx.x;
    const int64_t per = (R + VH_TPB - 1) / VH_TPB;
    const int64_t s0 = t * per < R ? t * per : R, e0 = s0 + per < R ? s0 + per : R;
    float cmax = -FLT_MAX, dummy = FLT_MAX;
    for (int64_t x = s0; x < e0; ++x) exact_row_scan(Uv, colbits, rs, b, R, CZ, ntiles, x, cmax, dummy, false);
    s_cmax[t] = cmax;
    __syncthreads();
    if (t == 0) {
        float run = -FLT_MAX;
        for (int i = 0; i < VH_TPB; ++i) { const float v = s_cmax[i]; s_cmax[i] = run; run = v > run ? v : run; }
    }
    __syncthreads();
    float run = s_cmax[t], mn = FLT_MAX;
    for (int64_t x = s0; x < e0; ++x) exact_row_scan(Uv, colbits, rs, b, R, CZ, ntiles, x, run, mn, true);
    s_min[t] = mn;
    __syncthreads();
    float m = FLT_MAX;
    if (t == 0)
        for (int i = 0; i < VH_TPB; ++i) m = s_min[i] < m ? s_min[i] : m;
    return m;
}

// Iteration control: convergence of the previous iteration, the while-condition of ITK's loop,
// bin range (the else-if quirk: common case directly, the exact raster scan when the first masked
// pixel is the strict minimum).  One block per volume.
__global__ void __launch_bounds__(VH_TPB) k_n4_ctrl(N4State *st, const double *part,
                                                   const int32_t *cp, const VolScalars *sc,
                                                   int conv_mode, int level, int it, float thresh,
                                                   int bins,
                                                   int64_t vol0, int32_t *nactive, const float *U,
                                                   const uint32_t *colbits, const int32_t *rs,
                                                   int64_t R, int64_t CZ, int64_t VS,
                                                   int64_t ntiles) {
    __shared__ int s_exact;
    __shared__ float s_bmax;
    const int64_t b = vol0 + blockIdx.x;
    const bool was_active = st[b].active;
    double conv = 0.0;
    if (conv_mode == 0) conv = (double)st[b].conv_w;
    else if (threadIdx.x < 64 && it > 0 && was_active)
        conv = conv_from_parts(part, cp, b, (double)sc[b].n_mask1);
    if (threadIdx.x == 0) {
        N4State &s = st[b];
        s_exact = 0;
        if (it == 0) {
            s.active = 1;
            s.iters = 0;
            s.conv = INFINITY;
        } else if (was_active) {
            s.tlast ^= 1;   // the previous iteration's eval used the other T buffer as "new"
            s.conv = conv;
            const bool go = conv_mode == 0 ? st[b].conv_w > thresh : conv > (double)thresh;
            if (!go) {
                s.active = 0;
                s.iters_level[level] = s.iters;
                s.conv_level[level] = (float)conv;
            }
        }
        if (s.active) {
            s.iters += 1;
            const float bmax = key2f(s.umax_key);
            const float umin = s.umin_key == 0xffffffffu ? FLT_MAX : key2f(s.umin_key);
            s.bin_max = bmax;
            if (umin <= s.u_first) {
                s.bin_min = umin;
                s.slope = (bmax - umin) / (float)(bins - 1);
            } else {
                s_exact = 1;
                s_bmax = bmax;
            }
            s.umax_key = 0u;
            s.umin_key = 0xffffffffu;
            atomicAdd(nactive, 1);
        }
    }
    __syncthreads();
    if (!s_exact) return;
    const float m = exact_min_block(U + b * VS, colbits, rs, b, R, CZ, ntiles);
    if (threadIdx.x == 0) {
        st[b].bin_min = m;
        st[b].slope = (s_bmax - m) / (float)(bins - 1);
    }
}

__global__ void __launch_bounds__(64) k_n4_level_end(N4State *st, const double *part,
                                                    const int32_t *cp, const VolScalars *sc,
                                                    int conv_mode, int level, int64_t vol0) {
    const int64_t b = vol0 + blockIdx.x;
    N4State &s = st[b];
    if (!s.active) return;
    const double conv = conv_mode == 0 ? (double)s.conv_w
                                       : conv_from_parts(part, cp, b, (double)sc[b].n_mask1);
    if (threadIdx.x != 0) return;
    s.tlast ^= 1;
    s.conv = conv;
    s.iters_level[level] = s.iters;
    s.conv_level[level] = (float)conv;
    s.active = 0;
}

// Packed Parzen histogram of U at mask == 1 (S3, hist_pack: count << 44 | sum of o-weights in
// 2^-24 units).  One block per chunk of N4_CH compact voxels (< 2^20 values: the packed words stay
// exact), LDS copies, then the block writes its chunk's packed histogram; k_n4_emap unpacks and adds
// a volume's chunks (integer sums: order-free).
__global__ void __launch_bounds__(VH_TPB) k_n4_hist(const float *__restrict__ U, const int32_t *cp,
                                                   const int32_t *cvol, const VolScalars *sc,
                                                   int64_t VS, int bins, const N4State *st,
                                                   uint64_t *hpart, int32_t c0) {
    __shared__ unsigned long long Hc[HIST_COPIES * VH_MAX_BINS];   // lane & 7 picks a copy
    const int32_t c = c0 + blockIdx.x;
    const int64_t b = cvol[c];
    if (!st[b].active) return;
    for (int i = threadIdx.x; i < HIST_COPIES * VH_MAX_BINS; i += VH_TPB) Hc[i] = 0ull;
    unsigned long long *H = Hc + (threadIdx.x & (HIST_COPIES - 1)) * VH_MAX_BINS;
    const int64_t j0 = (int64_t)(c - cp[b]) * N4_CH;
    const int64_t n = sc[b].n_mask1 - j0 < N4_CH ? sc[b].n_mask1 - j0 : N4_CH;
    const int t0 = threadIdx.x * N4_VPT;
    const float *src = U + b * VS + j0 + t0;
    float u[N4_VPT];
    if (t0 + N4_VPT <= n) {
#pragma unroll
        for (int q = 0; q < N4_VPT / 4; ++q) {
            const float4 v = reinterpret_cast<const float4 *>(src)[q];
            u[4 * q] = v.x; u[4 * q + 1] = v.y; u[4 * q + 2] = v.z; u[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < N4_VPT; ++k) u[k] = t0 + k < n ? src[k] : __int_as_float(0x7fc00000);
    }
    __syncthreads();
    const float bmin = st[b].bin_min;
    const double rinv = 1.0 / (double)st[b].slope;
#pragma unroll
    for (int k = 0; k < N4_VPT; ++k) {
        int idx;
        const unsigned long long w = hist_pack(u[k], bmin, rinv, bins, idx);
        if (w) atomicAdd(&H[idx], w);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < bins; i += VH_TPB) {
        unsigned long long cnt = 0ull, os = 0ull;
#pragma unroll
        for (int q = 0; q < HIST_COPIES; ++q) {
            const unsigned long long w = Hc[q * VH_MAX_BINS + i];
            cnt += hist_count(w);
            os += hist_osum(w);
        }
        hpart[(int64_t)c * VH_MAX_BINS + i] = (cnt << HIST_CSHIFT) | os;   // < 4096 values: exact
    }
}

// 512-point radix-2 FFT in LDS, 256 threads (one butterfly each per stage); same butterfly and
// twiddle indexing as oracle/n4_oracle.c fft_inplace.  Twiddles come from LDS; lds_fft2 runs two
// independent transforms through the same stages (half the barriers, identical arithmetic).
__device__ __forceinline__ void fft_bitrev(double2 *x, double2 *tmp) {
    for (int i = threadIdx.x; i < VH_FFT_P; i += VH_TPB) tmp[i] = x[i];
    __syncthreads();
    for (int i = threadIdx.x; i < VH_FFT_P; i += VH_TPB) x[(int)(__brev((unsigned)i) >> (32 - 9))] = tmp[i];
}

__device__ __forceinline__ void fft_butterfly(double2 *x, double2 w, int i0, int i1) {
    const double2 bb = x[i1];
    const double tr = w.x * bb.x - w.y * bb.y, ti = w.x * bb.y + w.y * bb.x;
    const double2 a = x[i0];
    x[i0] = make_double2(a.x + tr, a.y + ti);
    x[i1] = make_double2(a.x - tr, a.y - ti);
}

__device__ void lds_fft(double2 *x, double2 *tmp, const double2 *tw, bool inverse) {
    fft_bitrev(x, tmp);
    __syncthreads();
    const int t = threadIdx.x;
    for (int len = 2; len <= VH_FFT_P; len <<= 1) {
        const int half = len >> 1, step = VH_FFT_P / len;
        const int g = t / half, j = t % half;
        double2 w = tw[j * step];
        if (inverse) w.y = -w.y;
        fft_butterfly(x, w, g * len + j, g * len + j + half);
        __syncthreads();
    }
}

__device__ void lds_fft2(double2 *x, double2 *y, double2 *tx, double2 *ty, const double2 *tw,
                         bool inverse) {
    fft_bitrev(x, tx);
    fft_bitrev(y, ty);
    __syncthreads();
    const int t = threadIdx.x;
    for (int len = 2; len <= VH_FFT_P; len <<= 1) {
        const int half = len >> 1, step = VH_FFT_P / len;
        const int g = t / half, j = t % half;
        double2 w = tw[j * step];
        if (inverse) w.y = -w.y;
        fft_butterfly(x, w, g * len + j, g * len + j + half);
        fft_butterfly(y, w, g * len + j, g * len + j + half);
        __syncthreads();
    }
}


// Slice sums of a study's chunk histograms for studies with many chunks (a 512^3 study has ~7k:
// one emap block summing them alone took ~0.4 ms per iteration).  Block (s, b) adds chunks
// ca + s*per .. of study b per bin, counts and o-weight sums apart (integer sums: exact, order-free);
// k_n4_emap then adds the N4_HSL slices.
#define N4_HSL 64
__global__ void __launch_bounds__(VH_TPB) k_n4_hred(const uint64_t *hpart, const int32_t *cp,
                                                   const N4State *st, int bins, uint64_t *hred,
                                                   int64_t vol0) {
    const int64_t b = vol0 + blockIdx.y;
    if (!st[b].active) return;
    const int32_t ca = cp[b], ce = cp[b + 1];
    const int32_t per = (ce - ca + N4_HSL - 1) / N4_HSL, c0 = ca + (int32_t)blockIdx.x * per,
                  c1 = min(ce, c0 + per);
    uint64_t *out = hred + ((int64_t)blockIdx.y * N4_HSL + blockIdx.x) * 2 * VH_MAX_BINS;
    for (int h = threadIdx.x; h < bins; h += VH_TPB) {
        uint64_t cs = 0ull, os = 0ull;
#pragma unroll 8
        for (int32_t c = c0; c < c1; ++c) {
            const uint64_t w = hpart[(int64_t)c * VH_MAX_BINS + h];
            cs += hist_count(w);
            os += hist_osum(w);
        }
        out[h] = cs;
        out[VH_MAX_BINS + h] = os;
    }
}

// E(u|v) map (Wiener deconvolution of the histogram by the bias Gaussian), one block per volume.
__global__ void __launch_bounds__(VH_TPB) k_n4_emap(const uint64_t *hpart, const int32_t *cp,
                                                   const double2 *tw, int bins, float fwhm,
                                                   float noise, const N4State *st, float *Eout,
                                                   int64_t vol0, const uint64_t *hred,
                                                   const int32_t *nactive, int32_t *hflag) {
    __shared__ double2 V[VH_FFT_P], F[VH_FFT_P], U[VH_FFT_P], NUM[VH_FFT_P], DEN[VH_FFT_P],
        TMP[VH_FFT_P], TMP2[VH_FFT_P], TW[VH_FFT_P / 2];
    // the iteration's active count (k_n4_ctrl's atomic sum) into the host's page-locked flag: the
    // host reads it after the event behind this launch (a 4-byte D2H ran as a 10 us blit kernel)
    if (blockIdx.x == 0 && threadIdx.x == 0) *hflag = *nactive;
    const int64_t b = vol0 + blockIdx.x;
    if (!st[b].active) return;
    const int P = VH_FFT_P, off = (P - bins) / 2;
    const int t = threadIdx.x;
    const float binMin = st[b].bin_min, slope = st[b].slope;
    for (int n = t; n < P / 2; n += VH_TPB) TW[n] = tw[n];
    const int32_t ca = cp[b], ce = cp[b + 1];
    {   // the chunks' packed histograms summed per bin: thread (slice, bin) sums the counts and the
        // o-weight sums of a slice of the chunks (integer sums: order-free, exact), TMP / TMP2 hold
        // the partials (a 512^3 study has ~7k chunks: two loads per chunk per value took 2.4 ms)
        static_assert(VH_TPB % 256 == 0 && VH_TPB <= 1024 && VH_MAX_BINS <= 256, "slices of 256 bins");
        constexpr int NSL = VH_TPB / 256;
        uint64_t *const pc = reinterpret_cast<uint64_t *>(TMP), *const po = reinterpret_cast<uint64_t *>(TMP2);
        const int h = t & 255, sl = t >> 8;
        const int32_t per = (ce - ca + NSL - 1) / NSL, c0 = ca + sl * per, c1 = min(ce, c0 + per);
        uint64_t cs = 0ull, os = 0ull;
        if (hred) {   // k_n4_hred's slices of this study
            const uint64_t *r = hred + (int64_t)blockIdx.x * N4_HSL * 2 * VH_MAX_BINS;
            if (h < bins && sl == 0)
#pragma unroll 8
                for (int q = 0; q < N4_HSL; ++q) {
                    cs += r[(int64_t)q * 2 * VH_MAX_BINS + h];
                    os += r[(int64_t)q * 2 * VH_MAX_BINS + VH_MAX_BINS + h];
                }
        } else if (h < bins) {
#pragma unroll 8
            for (int32_t c = c0; c < c1; ++c) {
                const uint64_t w = hpart[(int64_t)c * VH_MAX_BINS + h];
                cs += hist_count(w);
                os += hist_osum(w);
            }
        }
        pc[sl * 256 + h] = cs;
        po[sl * 256 + h] = os;
    }
    __syncthreads();
    uint64_t hsv[(VH_FFT_P + VH_TPB - 1) / VH_TPB];
    {
        const uint64_t *const pc = reinterpret_cast<const uint64_t *>(TMP), *const po = reinterpret_cast<const uint64_t *>(TMP2);
        int q = 0;
        for (int n = t; n < P; n += VH_TPB, ++q) {
            const int h = n - off;
            uint64_t hs = 0ull;   // S3 unpacking: (count << 24) - osum of bin h, + osum of bin h - 1
            if (h >= 0 && h < bins)
                for (int sl = 0; sl < VH_TPB / 256; ++sl) {
                    hs += (pc[sl * 256 + h] << 24) - po[sl * 256 + h];
                    if (h > 0) hs += po[sl * 256 + h - 1];
                }
            hsv[q] = hs;
        }
    }
    __syncthreads();   // TMP / TMP2 are the FFT's scratch from here on
    {
        int q = 0;
        for (int n = t; n < P; n += VH_TPB, ++q) {
            V[n] = make_double2((double)hsv[q] * (1.0 / 16777216.0), 0.0);
            F[n] = make_double2(0.0, 0.0);
        }
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
            const double v = (double)(sf * expf_cr_tail(-(nf * nf) * ef));
            F[n].x = v;
            F[P - n].x = v;
        }
    }
    __syncthreads();
    lds_fft2(V, F, TMP, TMP2, TW, false);
    for (int n = t; n < P; n += VH_TPB) {
        const double a = F[n].x, bb = F[n].y;
        const double g = a / ((a * a - (-bb) * bb) + (double)noise);
        U[n] = make_double2(V[n].x * g, V[n].y * g);
    }
    __syncthreads();
    lds_fft(U, TMP, TW, true);
    for (int n = t; n < P; n += VH_TPB) {
        const double ur = U[n].x > 0.0 ? U[n].x : 0.0;
        U[n] = make_double2(ur, 0.0);
        const float c = binMin + ((float)n - (float)off) * slope;
        NUM[n] = make_double2((double)c * ur, 0.0);
        DEN[n] = make_double2(ur, 0.0);
    }
    __syncthreads();
    lds_fft2(NUM, DEN, TMP, TMP2, TW, false);
    for (int n = t; n < P; n += VH_TPB) {
        const double a = F[n].x, bb = F[n].y;
        double2 x = NUM[n];
        NUM[n] = make_double2(x.x * a - x.y * bb, x.x * bb + x.y * a);
        x = DEN[n];
        DEN[n] = make_double2(x.x * a - x.y * bb, x.x * bb + x.y * a);
    }
    __syncthreads();
    lds_fft2(NUM, DEN, TMP, TMP2, TW, true);
    for (int n = t; n < bins; n += VH_TPB) {
        const double d = DEN[n + off].x;
        Eout[b * VH_MAX_BINS + n] = d != 0.0 ? (float)(NUM[n + off].x / d) : 0.0f;
    }
}

// ---------------------------------------------------------------------------------------------
// S5 fit, item-ordered (n4_shared.h fit_item, the same code the volume-resident driver runs): a wave
// owns one (64-column tile, 64-row slot) item of one volume; the finished control rows of its tile
// are contracted over slices and cols and added to the volume's lattice numerator as 128-bit
// fixed-point integers with global atomics (order-free).  Tables are read from global memory.
// grid (ceil(items / FIT_WAVES), volumes); dynamic LDS: per wave a ring of nbmax rows + the
// stage-1 output buffer, then E.
// ---------------------------------------------------------------------------------------------
template <int MODE>
__global__ void __launch_bounds__(FIT_WAVES * 64, FIT_WPE) k_n4_fit_items(
    const float *__restrict__ U, const int32_t *rs, const uint64_t *rmask, const VolScalars *sc,
    int R, int C, int Z, int64_t VS, int ntiles, int nslots, int bins, const N4State *st,
    const float *E, DevLevel lv, int rowcap, int nbmax, unsigned long long *numfix,
    int64_t lat_cap, int64_t vol0) {
    extern __shared__ __attribute__((aligned(16))) double fsm[];
    __shared__ float sE[VH_MAX_BINS];
    const int64_t b = vol0 + blockIdx.y;
    if (MODE == 0 && !st[b].active) return;
    const int wv = threadIdx.x >> 6;
    const int nitems = ntiles * nslots;
    if (MODE == 0)
        for (int i = threadIdx.x; i < bins; i += FIT_WAVES * 64) sE[i] = E[b * VH_MAX_BINS + i];
    __syncthreads();
    const int item = blockIdx.x * FIT_WAVES + wv;
    if (item >= nitems) return;
    const int CZ = C * Z;
    const int64_t tb = b * (int64_t)ntiles * R;
    Item it;
    if (!item_begin(it, rmask + tb, rs + tb, nullptr, R, C, Z, CZ, nslots, item)) return;
    TabV T;
    T.wx = reinterpret_cast<const float4 *>(lv.ax[0].w);
    T.wy = reinterpret_cast<const float4 *>(lv.ax[1].w);
    T.wz = reinterpret_cast<const float4 *>(lv.ax[2].w);
    T.ix = lv.ax[0].isw2;
    T.iy = lv.ax[1].isw2;
    T.iz = lv.ax[2].isw2;
    T.bx = lv.ax[0].base;
    T.by = lv.ax[1].base;
    T.bz = lv.ax[2].base;
    T.krz = lv.ax[2].krange;
    T.xst = lv.xst;
    FitRing rg;
    rg.q = fsm + (size_t)wv * 2 * nbmax * rowcap;
    rg.sx = rg.q + (size_t)nbmax * rowcap;
    rg.rowcap = rowcap;
    rg.nr = 0;
    const int ncy = lv.ax[1].ncp, ncz = lv.ax[2].ncp;
    unsigned long long *nf = numfix + 2 * b * lat_cap;
    const int64_t n = sc[b].n_mask1;
    if (MODE == 0) {
        const float bmin = st[b].bin_min;
        const double rinv = 1.0 / (double)st[b].slope;
        fit_item<0, false, FIT_GS>(it, T, lv.wk3, reinterpret_cast<const double2 *>(lv.ax[0].w3i), ncy, ncz, Z,
                    bins, U + b * VS, n, sE, bmin, rinv, rg, nbmax, nf);
    } else {
        fit_item<1, false, FIT_GS>(it, T, lv.wk2, reinterpret_cast<const double2 *>(lv.ax[0].w2), ncy, ncz, Z,
                    bins, U + b * VS, n, sE, 0.0f, 1.0, rg, nbmax, nf);
    }
}

// clear the numerator of active volumes before a fit
template <int MODE>
__global__ void __launch_bounds__(VH_TPB) k_n4_fit_clear(unsigned long long *numfix, int64_t lat_cap,
                                                        int64_t nlat, const N4State *st, int64_t vol0) {
    const int64_t b = vol0 + blockIdx.y;
    if (MODE == 0 && !st[b].active) return;
    const int64_t e = blockIdx.x * (int64_t)VH_TPB + threadIdx.x;
    if (e < 2 * nlat) numfix[2 * b * lat_cap + e] = 0ull;
}

// MODE 1: den = fixed-point sum; MODE 0: phi = num / den (0 where den == 0), lattice += phi (S5).
// The fixed-point accumulators are zeroed once read, so the next fit starts from zero without a
// clearing launch (k_n4_fit_clear runs once per level, before the denominators' fit).
template <int MODE>
__global__ void __launch_bounds__(VH_TPB) k_n4_latupd(unsigned long long *numfix, float *lat,
                                                     double *den, int64_t lat_cap, int64_t nlat,
                                                     const N4State *st, int64_t vol0) {
    const int64_t b = vol0 + blockIdx.x;
    if (MODE == 0 && !st[b].active) return;
    const int64_t e = blockIdx.y * (int64_t)VH_TPB + threadIdx.x;
    if (e >= nlat) return;
    unsigned long long *nf = numfix + 2 * (b * lat_cap + e);
    const double v = fix128_get(nf, nf + 1);
    nf[0] = 0ull;
    nf[1] = 0ull;
    if (MODE == 1) {
        den[b * lat_cap + e] = v;
    } else {
        const double d = den[b * lat_cap + e];
        const float phi = d != 0.0 ? (float)(v / d) : 0.0f;
        lat[b * lat_cap + e] += phi;
    }
}

// P1[i][j][z] = sum_k wz(z,k) lat[i][j][k] for the eval sweep.  grid (volumes, chunks of 256).
__global__ void __launch_bounds__(VH_TPB) k_n4_P1(const float *lat, int64_t lat_cap, double *P1,
                                                 int64_t q2_cap, int64_t Z, const N4State *st,
                                                 DevLevel lv, int64_t vol0) {
    const int64_t b = vol0 + blockIdx.x;
    if (!st[b].active) return;
    const DevAxis az = lv.ax[2];
    const int ncx = lv.ax[0].ncp, ncy = lv.ax[1].ncp, ncz = az.ncp;
    const int64_t e = blockIdx.y * (int64_t)VH_TPB + threadIdx.x;
    if (e >= (int64_t)ncx * ncy * Z) return;
    const int64_t ij = e / Z, z = e % Z;
    const int bz = az.base[z];
    const float4 w = *reinterpret_cast<const float4 *>(az.w + 4 * z);
    const float *l = lat + b * lat_cap + ij * ncz + bz;
    P1[b * q2_cap + e] = (double)w.x * (double)l[0] + (double)w.y * (double)l[1] +
                         (double)w.z * (double)l[2] + (double)w.w * (double)l[3];
}

// T(i) = sum_j wy(y,j) P1[i][j][z] for one column
__device__ __forceinline__ double col_T(const double *p1, int i, int ncy, int64_t Z, int by,
                                        float4 wy, int64_t z) {
    const double *r = p1 + ((int64_t)i * ncy + by) * Z + z;
    return (double)wy.x * r[0] + (double)wy.y * r[Z] + (double)wy.z * r[2 * Z] + (double)wy.w * r[3 * Z];
}

// Per-column contraction of the lattice for the eval sweep: T[i][col] (float).
__global__ void __launch_bounds__(VH_TPB) k_n4_T(const double *P1, int64_t q2_cap, int64_t C,
                                                int64_t Z, DevLevel lv, const N4State *st,
                                                float *T, int64_t tbuf, int64_t tcap, int64_t vol0) {
    const int64_t b = vol0 + blockIdx.y;
    if (!st[b].active) return;
    // one thread per (column, control row): a thread walking its column's ncx rows waited for
    // each row's loads in turn (18 us per launch at config 2)
    const int64_t CZ = C * Z;
    const int ncx = lv.ax[0].ncp;
    const int64_t e = blockIdx.x * (int64_t)VH_TPB + threadIdx.x;
    if (e >= CZ * ncx) return;
    const int64_t col = e / ncx;
    const int i = (int)(e - col * ncx);
    const int64_t y = col / Z, z = col % Z;
    const int ncy = lv.ax[1].ncp;
    const int by = lv.ax[1].base[y];
    const float4 wy = *reinterpret_cast<const float4 *>(lv.ax[1].w + 4 * y);
    const double *p1 = P1 + b * q2_cap;
    float *t = T + (st[b].tlast ^ 1) * tbuf + b * tcap;   // [col][ncx]: one 16-B load per voxel
    t[e] = (float)col_T(p1, i, ncy, Z, by, wy, z);
}

// Evaluate the new field at masked voxels: B_new and U = L0 - B_new (compact), the convergence
// partial sums of exp(B_old - B_new) - 1 (one slot per chunk, fixed-order block reduction) and the
// U range for the next iteration.  B is never stored: B_old is re-evaluated from the previous
// field's column tables (the other T buffer, with that field's level tables `lvo` -- the same
// float expression the previous eval computed, so the values are identical), which trades 8 B of
// HBM per voxel for one more 16-byte load from the L2-resident tables.  One block per chunk,
// lane-consecutive voxels; row weights from LDS.  bo_mode 0: B_old = 0 (first iteration).
__global__ void __launch_bounds__(VH_TPB) k_n4_eval(const float *__restrict__ L0, float *U,
                                                   const int32_t *__restrict__ ridx,
                                                   const int32_t *cp, const int32_t *cvol,
                                                   const VolScalars *sc, int64_t R, int64_t CZ,
                                                   int64_t VS, int rsh, const float *T,
                                                   int64_t tbuf, int64_t tcap, DevLevel lv,
                                                   DevLevel lvo, int bo_mode, N4State *st,
                                                   double *part, int32_t c0, int conv_mode,
                                                   float *D) {
    extern __shared__ __attribute__((aligned(16))) float4 sW[];   // [R] new, [R] old, then bases
    __shared__ double s_sd[VH_TPB / 64], s_sd2[VH_TPB / 64];
    __shared__ uint32_t s_max[VH_TPB / 64], s_min[VH_TPB / 64];
    const int32_t c = c0 + blockIdx.x;
    const int64_t b = cvol[c];
    if (!st[b].active) return;
    float4 *sWo = sW + R;
    int *sB = reinterpret_cast<int *>(sW + 2 * R);
    int *sBo = sB + R;
    const int ncx = lv.ax[0].ncp, ncxo = lvo.ax[0].ncp;
    for (int x = threadIdx.x; x < R; x += VH_TPB) {
        sW[x] = *reinterpret_cast<const float4 *>(lv.ax[0].w + 4 * x);
        sB[x] = lv.ax[0].base[x];
        sWo[x] = *reinterpret_cast<const float4 *>(lvo.ax[0].w + 4 * x);
        sBo[x] = lvo.ax[0].base[x];
    }
    const int64_t j0 = (int64_t)(c - cp[b]) * N4_CH;
    const int n = (int)(sc[b].n_mask1 - j0 < N4_CH ? sc[b].n_mask1 - j0 : N4_CH);
    const int64_t f = sc[b].first_masked;   // packed like ridx
    const int first = f < 0 ? -1 : (int)(((f / CZ) << rsh) | (f % CZ));
    const float *Lb = L0 + b * VS + j0;
    float *Ub = U + b * VS + j0;
    float *Db = D + b * VS + j0;
    const int32_t *Rb = ridx + b * VS + j0;
    const int tl = st[b].tlast;
    const __amdgpu_buffer_rsrc_t rTn = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(T + (tl ^ 1) * tbuf + b * tcap), 0, (int)(tcap * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t rTo = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(T + tl * tbuf + b * tcap), 0, (int)(tcap * 4), 0x00020000);
    int rr[N4_VPT];
    float la[N4_VPT];
#pragma unroll
    for (int k = 0; k < N4_VPT; ++k) {
        const int j = threadIdx.x + k * VH_TPB;
        const bool ok = j < n;
        rr[k] = ok ? Rb[j] : -1;
        la[k] = ok ? Lb[j] : 0.0f;
    }
    __syncthreads();
    double sd = 0.0, sd2 = 0.0;
    uint32_t kmax = 0u, kmin = 0xffffffffu;
    const int cmask = (1 << rsh) - 1;
#pragma unroll
    for (int h = 0; h < N4_VPT; h += 4) {
        float4 tn[4], to[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int r = rr[h + k];
            const int x = r < 0 ? 0 : r >> rsh;
            const int64_t col = r & cmask;
            const uint32_t on = r < 0 ? VH_OOB : (uint32_t)((col * ncx + sB[x]) * 4);
            const uint32_t oo = (r < 0 || !bo_mode) ? VH_OOB : (uint32_t)((col * ncxo + sBo[x]) * 4);
            const auto vn = __builtin_amdgcn_raw_buffer_load_b128(rTn, (int)on, 0, 0);
            const auto vo = __builtin_amdgcn_raw_buffer_load_b128(rTo, (int)oo, 0, 0);
            tn[k] = make_float4(__uint_as_float(vn[0]), __uint_as_float(vn[1]),
                                __uint_as_float(vn[2]), __uint_as_float(vn[3]));
            to[k] = make_float4(__uint_as_float(vo[0]), __uint_as_float(vo[1]),
                                __uint_as_float(vo[2]), __uint_as_float(vo[3]));
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int r = rr[h + k];
            if (r < 0) continue;
            const int x = r >> rsh;
            const int j = threadIdx.x + (h + k) * VH_TPB;
            const float4 w = sW[x], t = tn[k];
            const float bn = ((w.x * t.x + w.y * t.y) + w.z * t.z) + w.w * t.w;
            float bo = 0.0f;
            if (bo_mode) {
                const float4 wo = sWo[x], q = to[k];
                bo = ((wo.x * q.x + wo.y * q.y) + wo.z * q.z) + wo.w * q.w;
            }
            const float u = la[h + k] - bn;
            Ub[j] = u;
            if (conv_mode == 0) {   // S7 input: the field difference, compact order (like U)
                Db[j] = bo - bn;
            } else {                // S7x
                const double d = (double)expm1c(bo - bn);
                sd += d;
                sd2 = fma(d, d, sd2);
            }
            const uint32_t key = f2key(u);
            kmax = key > kmax ? key : kmax;
            if (r == first) st[b].u_first = u;
            else kmin = key < kmin ? key : kmin;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        sd += __shfl_down(sd, off, 64);
        sd2 += __shfl_down(sd2, off, 64);
    }
    kmax = wave_max_u32(kmax);
    kmin = wave_min_u32(kmin);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s_sd[w] = sd;
        s_sd2[w] = sd2;
        s_max[w] = kmax;
        s_min[w] = kmin;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double a = 0.0, a2 = 0.0;
        uint32_t mx = 0u, mn = 0xffffffffu;
        for (int i = 0; i < VH_TPB / 64; ++i) {
            a += s_sd[i];
            a2 += s_sd2[i];
            mx = s_max[i] > mx ? s_max[i] : mx;
            mn = s_min[i] < mn ? s_min[i] : mn;
        }
        part[(int64_t)c * 2] = a;
        part[(int64_t)c * 2 + 1] = a2;
        if (mx) atomicMax(&st[b].umax_key, mx);
        if (mn != 0xffffffffu) atomicMin(&st[b].umin_key, mn);
    }
}

// S7: ITK's float Welford convergence of the last eval of each active volume (two waves per
// volume: n4_shared.h chain_wave_mu / chain_wave_sig fed by chain_wave_prod, over the field
// differences read in raster order through the volume's raster -> compact permutation).
#define WF_PROD 4   // producer waves of k_n4_welford
#define WF_TPB (64 * chain_waves(WF_PROD))
__global__ void __launch_bounds__(WF_TPB) k_n4_welford(const float *D, const int32_t *perm,
                                                                  int64_t VS, const VolScalars *sc,
                                                                  N4State *st, int64_t vol0) {
    __shared__ ChainSlot slots[CH_SLOTS];
    __shared__ ChainState cs;
    const int64_t b = vol0 + blockIdx.x;
    if (!st[b].active) return;
    chain_reset(slots, &cs);
    __syncthreads();
    const int64_t n = sc[b].n_mask1;
    const int w = threadIdx.x >> 6, pid = chain_prod_id(w);
    if (w == 0) chain_wave_mu(n, slots, &cs);
    else if (w == 1) chain_wave_sig(n, slots, &cs);
    else if (pid >= 0 && pid < WF_PROD)
        chain_wave_prod(D + b * VS, perm + b * VS, n, slots, &cs, pid, WF_PROD);
    __syncthreads();
    if (threadIdx.x == 0) st[b].conv_w = cs.conv;
}

// S7 by guess and verify (n4_shared.h pcw_run): one 1024-thread workgroup per active volume, one
// chain block per thread.  d is read through the raster -> compact permutation in pass 0; P (the
// p values in block layout) lives in the second half of the D buffer.  For a large study this
// replaces the serial chain's n dependent steps (~30 cycles each) by ~13 parallel rounds.
__global__ void __launch_bounds__(PC_TPB) k_n4_pcw(const float *D, const int32_t *perm, float *Pbuf,
                                                   int64_t VS, const VolScalars *sc, N4State *st,
                                                   int64_t vol0, float skip_thresh) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int64_t b = vol0 + blockIdx.x;
    if (!st[b].active) return;
    PcShared<PC_TPB> &S = *reinterpret_cast<PcShared<PC_TPB> *>(smem);
    __shared__ ChainState ch;
    const float *const Db = D + b * VS;
    const int32_t *const pb = perm + b * VS;
    // D[b] (compact d) is free once pass 0 has read it: PCX's stored increments.  skip_thresh:
    // the certified "above the threshold" decision of pcw_run (0 at the level's last iteration)
    // early decision (PC_PRE): a level's first call, then as long as it keeps deciding
    pcw_run<PC_TPB>([=](int64_t r) { return Db[pb[r]]; }, Pbuf + b * VS, sc[b].n_mask1, S, ch, 1,
            reinterpret_cast<double *>(const_cast<float *>(Db)), (int)(VS / 2), skip_thresh, nullptr,
            false, st[b].iters == 1 || st[b].pc_pre != 0);
    if (threadIdx.x == 0) {
        st[b].conv_w = ch.conv;
        st[b].pc_pre = S.xdone == 4 * 1 + 1;
        st[b].conv_bound = S.xdone == 4 * 1 + 1 || S.xdone == 4 * 1 + 3;   // decided on bounds
    }
}

// S7 by guess and verify over the whole GPU, for one large study (the sweep driver with a single
// volume, e.g. BASELINE config 5): a cooperative grid of G 1024-thread workgroups, one chain block per
// thread (NB = 1024 G blocks of n / NB steps).  The per-block state lives in global memory (struct of
// arrays); the affine transition maps are scanned in three levels (wave shuffles, the workgroup's
// waves in LDS, the workgroups' aggregates after a grid barrier).  Two grid barriers per round.
struct PcgArgs {
    const float *D;
    const int32_t *perm;
    float *P;                        // p in block layout: step s of block j at s NB + j
    const VolScalars *sc;
    N4State *st;
    int64_t b;
    float *gmu, *gsig, *emu, *esig, *gmu_o, *emu_o;   // [NB]
    double *s1, *s2;                                   // [NB] pass-0 sums
    double *agA, *agB, *agS;                           // [G] workgroup aggregates
    int *agF;                                          // [G] first failing transition of a workgroup
};
struct PcgLds {
    double wA[PC_TPB / 64], wB[PC_TPB / 64], wS[PC_TPB / 64];
    int wF[PC_TPB / 64];
    double pB, pS;   // the workgroups before this one, applied to delta = 0
    int first;
};
// Exclusive grid-wide composition of the maps (a, b) (and sums bs) in block order, applied to 0:
// dm, ds.  *first (in: this thread's failing flag) -> the smallest failing block index of the grid
// (NB when none).  Contains one grid barrier.
__device__ void pcg_scan(const PcgArgs &A, PcgLds &L, cooperative_groups::grid_group &grid, double a,
                         double b, double bs, bool fail, double &dm, double &ds, int &first) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, G = gridDim.x;
    const int NB = G * PC_TPB;
    double Aw = a, Bw = b, Sw = bs;
    for (int off = 1; off < 64; off <<= 1) {
        const double ya = __shfl_up(Aw, off, 64), yb = __shfl_up(Bw, off, 64), ys = __shfl_up(Sw, off, 64);
        if (lane >= off) {
            Bw = Aw * yb + Bw;
            Aw = Aw * ya;
            Sw = ys + Sw;
        }
    }
    const uint64_t bal = __ballot(fail);
    if (lane == 63) {
        L.wA[w] = Aw;
        L.wB[w] = Bw;
        L.wS[w] = Sw;
    }
    if (lane == 0) L.wF[w] = bal ? (int)(blockIdx.x * PC_TPB + w * 64 + __ffsll((unsigned long long)bal) - 1) : NB;
    double ea = __shfl_up(Aw, 1, 64), eb = __shfl_up(Bw, 1, 64), es = __shfl_up(Sw, 1, 64);
    if (lane == 0) {
        ea = 1.0;
        eb = 0.0;
        es = 0.0;
    }
    __syncthreads();
    if (threadIdx.x == 0) {   // this workgroup's aggregate
        double At = 1.0, Bt = 0.0, St = 0.0;
        int f = NB;
        for (int v = 0; v < PC_TPB / 64; ++v) {
            Bt = L.wA[v] * Bt + L.wB[v];
            At = At * L.wA[v];
            St = St + L.wS[v];
            f = min(f, L.wF[v]);
        }
        A.agA[blockIdx.x] = At;
        A.agB[blockIdx.x] = Bt;
        A.agS[blockIdx.x] = St;
        A.agF[blockIdx.x] = f;
    }
    grid.sync();
    if (w == 0) {   // the workgroups before this one (ordered: lane l folds [per l, per l + per)), and
        // the grid's first failure; any grid size (per = ceil(G / 64) aggregates per lane)
        double Al = 1.0, Bl = 0.0, Sl = 0.0;
        int f = NB;
        const int per = (G + 63) / 64;
        for (int i = 0; i < per; ++i) {
            const int u = per * lane + i;
            if (u < G) {
                f = min(f, A.agF[u]);
                if (u < (int)blockIdx.x) {
                    const double au = A.agA[u];
                    Bl = au * Bl + A.agB[u];
                    Al = Al * au;
                    Sl = Sl + A.agS[u];
                }
            }
        }
        for (int off = 1; off < 64; off <<= 1) {
            const double ya = __shfl_up(Al, off, 64), yb = __shfl_up(Bl, off, 64), ys = __shfl_up(Sl, off, 64);
            if (lane >= off) {
                Bl = Al * yb + Bl;
                Al = Al * ya;
                Sl = ys + Sl;
            }
            f = min(f, __shfl_xor(f, off, 64));
        }
        if (lane == 63) {
            L.pB = Bl;
            L.pS = Sl;
            L.first = f;
        }
    }
    __syncthreads();
    double x = L.pB, xs = L.pS;
    for (int v = 0; v < w; ++v) {
        x = L.wA[v] * x + L.wB[v];
        xs = xs + L.wS[v];
    }
    dm = ea * x + eb;
    ds = xs + es;
    first = L.first;
}

__global__ void __launch_bounds__(PC_TPB) k_n4_pcg(PcgArgs A) {
    namespace cg = cooperative_groups;
    cg::grid_group grid = cg::this_grid();
    if (!A.st[A.b].active) return;   // uniform over the grid
    __shared__ PcgLds L;
    const int64_t n = A.sc[A.b].n_mask1;
    const int NB = gridDim.x * PC_TPB;
    const PcMap m = pc_map(n, NB);
    const uint32_t j = blockIdx.x * PC_TPB + threadIdx.x, len = pc_len(m, j), k0 = pc_k0(m, j);
    const int nbe = m.L ? NB : (int)m.rem;
    const float *const Db = A.D + A.b * 0;   // D, perm, P are this volume's (host offsets)
    // pass 0: p = exp(d) in block layout, block sums
    double s1 = 0.0, s2 = 0.0;
    for (uint32_t s0 = 0; s0 < len; s0 += 8) {
        int32_t pi[8];
#pragma unroll
        for (int i = 0; i < 8; ++i)   // clamped, unconditional: the loads stay in flight together
            pi[i] = A.perm[k0 - 1u + (s0 + i < len ? s0 + i : len - 1u)];
        float v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = Db[pi[i]];
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (s0 + i < len) {
                const float p = expf_crs(v[i]);
                A.P[(size_t)(s0 + i) * NB + j] = p;
                const double e = (double)p - 1.0;
                s1 += e;
                s2 = fma(e, e, s2);
            }
    }
    double dm, ds;
    int first;
    pcg_scan(A, L, grid, 1.0, s1, s2, false, dm, ds, first);   // exclusive sums: dm = S1, ds = S2
    {
        const double K = (double)(k0 - 1u);
        float g = 0.0f, gs = 0.0f;
        if (K > 0.0) {
            g = (float)(1.0 + dm / K);
            const double v = ds - dm * (dm / K);
            gs = (float)(v > 0.0 ? v : 0.0);
        }
        A.gmu[j] = g;
        A.gsig[j] = gs;
    }
    grid.sync();
    float lg = __int_as_float(0x7fc00000), ls = lg, le = 0.0f, les = 0.0f;
    bool done = false;
    int round = 0;
#ifdef PCG_PROF
    const unsigned long long pc0 = wall_clock64();
    int ra = 0;
#endif
    for (int phase = 0; phase < 2 && !done; ++phase) {
#ifdef PCG_PROF
        if (phase == 1) ra = round;
#endif
        const int cap = phase == 0 ? PC_AMAX : PC_RMAX;
        for (int r = 0; r < cap; ++r, ++round) {
            const float g = A.gmu[j], gs = A.gsig[j];
            float mu = g, sig = gs;
            if (phase == 1) {
                pc_block<0>(A.P, j, len, k0, mu, sig, NB);
            } else {
                const bool same = __float_as_uint(g) == __float_as_uint(lg) && __float_as_uint(gs) == __float_as_uint(ls);
                if (__ballot(!same) != 0ull && !same) {
                    pc_block_apx<0>(A.P, j, len, k0, mu, sig, (uint32_t)NB, (m.L + 1u) * (uint32_t)NB);
                    lg = g;
                    ls = gs;
                    le = mu;
                    les = sig;
                }
                mu = le;
                sig = les;
            }
            // the transition j -> j + 1 (as pcw_update)
            double a = 1.0, bm = 0.0, bsv = 0.0;
            bool mm = false;
            if ((int)j < nbe - 1) {
                const float gn = A.gmu[j + 1], gsn = A.gsig[j + 1];
                mm = __float_as_uint(mu) != __float_as_uint(gn) || __float_as_uint(sig) != __float_as_uint(gsn);
                bm = (double)mu - (double)gn;
                bsv = (double)sig - (double)gsn;
                const uint32_t k1 = k0 + len - 1u;
                float af = (float)(k0 - 1u) * __builtin_amdgcn_rcpf((float)k1);
                const float go = A.gmu_o[j], eo = A.emu_o[j];
                if (round > 0 && g != go) {
                    const float sl = (mu - eo) * __builtin_amdgcn_rcpf(g - go);
                    if (sl >= 0.0f && sl <= 1.0f) af = sl;
                }
                a = (double)af;
                A.gmu_o[j] = g;
                A.emu_o[j] = mu;
            }
            A.emu[j] = mu;
            A.esig[j] = sig;
            pcg_scan(A, L, grid, a, bm, bsv, mm, dm, ds, first);
            if (first == NB) {   // every block end matched its successor's guess
                if (phase == 0) break;   // phase A's fixed point (sig steps uncertified): verify it exactly
                if (j == (uint32_t)(nbe - 1)) A.st[A.b].conv_w = itk_conv(mu, sig, n);
                done = true;
                break;
            }
            if (r == cap - 1) break;   // phase A cap: on to the exact rounds; phase B cap: serial below
            if ((int)j < nbe - 1) {
                A.gmu[j + 1] = dm == 0.0 ? mu : (float)((double)mu + a * dm);
                A.gsig[j + 1] = ds == 0.0 ? sig : (float)((double)sig + ds);
            }
            grid.sync();
        }
        if (phase == 0 && !done) grid.sync();   // the last phase-A ends, then exact rounds
    }
#ifdef PCG_PROF
    if (j == 0)
        printf("PCG_PROF n %lld G %d L %u roundsA %d roundsB %d done %d wall %llu\n", (long long)n, (int)gridDim.x,
               m.L, ra, round - ra, (int)done, wall_clock64() - pc0);
#endif
    if (!done && j == 0) {   // round cap: serial from the first failing transition (ends are exact up to it)
        float mu = A.emu[first], sig = A.esig[first];
        for (int jb = first + 1; jb < nbe; ++jb) {
            const uint32_t l = pc_len(m, jb);
            double kd = (double)pc_k0(m, jb);
            for (uint32_t s = 0; s < l; ++s, kd += 1.0) pc_step(kd, A.P[(size_t)s * NB + jb], mu, sig);
        }
        A.st[A.b].conv_w = itk_conv(mu, sig, n);
    }
}

__global__ void __launch_bounds__(PC_TPB) k_n4_pcg2(Pcg2Args A) {
    namespace cg = cooperative_groups;
    cg::grid_group grid = cg::this_grid();
    __shared__ Pcg2Lds L;
    __shared__ float T0[PCG_G0 * (PC_TPB + 8)];   // pass 0's transpose (pcg2_body)
    kst_begin(A.kst);   // profiling: this launch's span (stamped timer)
    if (A.st[A.b].active) {   // uniform over the grid
        // pass 0's loads: the perm loads of a group issued together, then the d loads they address
        const float *const D = A.D;
        const int32_t *const perm = A.perm;
        pcg2_body(A, L, grid, [=](int64_t r) { return D[perm[r]]; },
                  A.t0 ? T0 : nullptr);
    }
    kst_end(A.kst);
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
                                                     int n0, int n1, int n2, int64_t vol0) {
    const int64_t b = vol0 + blockIdx.x;
    float *L = lat + b * lat_cap;
    float *T1 = lat + (nb + b) * lat_cap;
    float *T2 = lat + (2 * nb + b) * lat_cap;
    refine_axis_dev(L, T1, n0, n1, n2, 0);
    __syncthreads();
    refine_axis_dev(T1, T2, 2 * n0 - 3, n1, n2, 1);
    __syncthreads();
    refine_axis_dev(T2, L, 2 * n0 - 3, 2 * n1 - 3, n2, 2);
}

#ifndef NF_PF
#define NF_PF 16   // k_n4_final: image rows in flight per lane (8, 16 or 32)
#endif
// Final field at every voxel and the corrected image I / exp(B), in 32-row slabs (one bitmap word)
// with one column per lane.  With keys != nullptr it also emits the VDP chain's sort keys of the
// mask == 1 voxels (coalesced: a wave is 64 columns, a row's masked lanes are contiguous),
// replacing the separate masked gather for volumes whose mask is binary (n_mask == n_mask1); and
// it accumulates calculate_SNR's partial sums from the image it streams (k_snr's arithmetic).
__global__ void __launch_bounds__(VH_TPB) k_n4_final(const float *__restrict__ I, float *out,
                                                    int64_t R, int64_t C, int64_t Z, int64_t V,
                                                    int64_t ncb, int64_t q2_cap, const double *P1,
                                                    DevLevel lv, const uint32_t *colbits,
                                                    const uint32_t *colbnz, const int64_t *colstart,
                                                    const VolScalars *sc, uint32_t *keys, SnrBox sb) {
    __shared__ uint32_t s_rows[2];
    __shared__ double s_red[4][VH_TPB / 64];
    __shared__ float4 s_w[VH_SLAB];   // the slab's row weights and lattice bases: uniform per row,
    __shared__ int s_base[VH_SLAB];   // read from LDS instead of a global load + wait per voxel
    const int64_t b = blockIdx.y;
    const int64_t CZ = C * Z;
    const int64_t sl = blockIdx.x / ncb;
    const int64_t col = (blockIdx.x % ncb) * VH_TPB + threadIdx.x;
    const int64_t x0 = sl * VH_SLAB;
    const int nr = (int)(R - x0 < VH_SLAB ? R - x0 : VH_SLAB);
    const VolScalars s = sc[b];
    const DevAxis ax = lv.ax[0];
    if ((int)threadIdx.x < nr) {
        s_w[threadIdx.x] = *reinterpret_cast<const float4 *>(ax.w + 4 * (x0 + threadIdx.x));
        s_base[threadIdx.x] = ax.base[x0 + threadIdx.x];
    }
    snr_slab_rows(sb, s, b, R, x0, nr, s_rows);
    __syncthreads();
    const bool act = col < CZ;
    const int64_t nw = (R + 31) >> 5;
    const bool emit = keys != nullptr;   // block-uniform
    // keys of the mask != 0 voxels (k_gather's set; for a binary mask the N4 label's): the wave's 64
    // columns own one contiguous run of k_gather's column compaction, slab by slab; the sort needs
    // the values only, so they are stored row by row across the wave
    int64_t kpos = 0;
    if (emit) {
        int before = 0;   // this column's keys in the earlier slabs
        if (act)
            for (int64_t w = 0; w < sl; ++w) before += __popc(colbnz[(b * nw + w) * CZ + col]);
        for (int off = 32; off > 0; off >>= 1) before += __shfl_xor(before, off, 64);
        if (act) kpos = b * V + colstart[b * CZ + (col & ~(int64_t)63)] + before;
    }
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    if (act) {
        const int64_t y = (uint32_t)col / (uint32_t)Z, z = col - y * Z;
        const int ncy = lv.ax[1].ncp;
        const int by = lv.ax[1].base[y];
        const float4 wy = *reinterpret_cast<const float4 *>(lv.ax[1].w + 4 * y);
        const double *p1 = P1 + b * q2_cap;
        const uint32_t sig = colbnz[(b * nw + sl) * CZ + col];
        const uint32_t noise = snr_col_noise(sb, s, b, Z, col, s_rows);
        snr_count(acc, noise);
        int wb = s_base[0];
        // S9: the final field per S6 (float T window, float row sum), I / (float)exp((double)B)
        float t0 = (float)col_T(p1, wb, ncy, Z, by, wy, z), t1 = (float)col_T(p1, wb + 1, ncy, Z, by, wy, z);
        float t2 = (float)col_T(p1, wb + 2, ncy, Z, by, wy, z), t3 = (float)col_T(p1, wb + 3, ncy, Z, by, wy, z);
        const float *src = I + b * V + x0 * CZ + col;
        float *dst = out + b * V + x0 * CZ + col;
        // the image loads of NF_PF rows are issued together, ahead of the field, exp and stores of
        // their rows (the row walk of one column is otherwise a dependent load -> exp -> store
        // chain); row weights and bases come from LDS 8 rows at a time
#pragma unroll
        for (int f0 = 0; f0 < VH_SLAB; f0 += NF_PF) {
            if (f0 >= nr) break;
            float iv[NF_PF];
#pragma unroll
            for (int k = 0; k < NF_PF; ++k) iv[k] = f0 + k < nr ? src[(int64_t)(f0 + k) * CZ] : 0.0f;
#pragma unroll
            for (int g0 = 0; g0 < NF_PF; g0 += 8) {
                const int i0 = f0 + g0;
                if (i0 >= nr) break;
                float4 wv[8];
                int bv[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) {   // the group's LDS reads together, one wait
                    wv[k] = s_w[(i0 + k) & (VH_SLAB - 1)];
                    bv[k] = s_base[(i0 + k) & (VH_SLAB - 1)];
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const int i = i0 + k;
                    if (i >= nr) break;
                    const int bx = bv[k];
                    while (wb < bx) {
                        ++wb;
                        t0 = t1; t1 = t2; t2 = t3;
                        t3 = (float)col_T(p1, wb + 3, ncy, Z, by, wy, z);
                    }
                    const float4 w = wv[k];
                    const float bn = ((w.x * t0 + w.y * t1) + w.z * t2) + w.w * t3;
                    const float x = iv[g0 + k];
                    const float o = x / expf_cr(bn);
                    dst[(int64_t)i * CZ] = o;
                    snr_add(acc, x, (sig >> i) & 1u, (noise >> i) & 1u);
                    if (emit) {
                        const bool on = (sig >> i) & 1u;
                        const uint64_t bal = __ballot(on);
                        if (on) keys[kpos + lanes_below(bal)] = f2key(o);
                        kpos += __popcll(bal);
                    }
                }
            }
        }
    }
    snr_block_write(acc, s_red, sb.part + (b * sb.nparts + blockIdx.x) * 4);
}

// ---------------------------------------------------------------------------------------------
// host driver
// ---------------------------------------------------------------------------------------------
// One sub-batch [vol0, vol0 + ns): the whole multi-level loop.  Flat sweeps run over the chunk
// range [cp[vol0], cp[vol0 + ns]); converged volumes' blocks exit at once.
// Doubles of one fit ring row for level L: >= 64 and >= the largest tile's stage-1 output count.
static int fit_rowcap(const vh_batch *b, const vh_n4_params &prm, int L) {
    const int Z = (int)b->Z;
    AxisTab tz;
    const float eps = vh_bspline_eps(std::max({vh_level_ncp(prm, L, 0), vh_level_ncp(prm, L, 1),
                                               vh_level_ncp(prm, L, 2)}) - 3);
    vh_axis_tables(Z, vh_level_ncp(prm, L, 2), eps, tz);
    int cap = 64;
    for (int64_t c0 = 0; c0 < b->CZ; c0 += TILE_W) {
        const int64_t c1 = std::min(c0 + TILE_W, b->CZ) - 1;
        const int y0 = (int)(c0 / Z), y1 = (int)(c1 / Z), z0 = (int)(c0 % Z), z1 = (int)(c1 % Z);
        const int klo = tz.base[y0 == y1 ? z0 : 0];
        const int KT = tz.base[y0 == y1 ? z1 : Z - 1] + 4 - klo;
        cap = std::max(cap, (y1 - y0 + 1) * KT);
    }
    return cap;
}

// VH_N4_TRACE (diagnostics): per iteration, hashes of volume vol0's U and D and its conv_w
static void n4_trace(vh_batch *b, int64_t vol0, int L, int it) {
    HIP_TRY(hipStreamSynchronize(b->stream));
    VolScalars sc;
    N4State s;
    HIP_TRY(hipMemcpy(&sc, b->d_sc + vol0, sizeof(sc), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(&s, b->d_st + vol0, sizeof(s), hipMemcpyDeviceToHost));
    const int64_t n = sc.n_mask1;
    std::vector<uint32_t> h((size_t)n);
    auto fnv = [&](const float *dp) {
        HIP_TRY(hipMemcpy(h.data(), dp + vol0 * b->VS, 4 * (size_t)n, hipMemcpyDeviceToHost));
        uint64_t x = 1469598103934665603ull;
        for (int64_t i = 0; i < n; ++i) x = (x ^ h[(size_t)i]) * 1099511628211ull;
        return x;
    };
    const uint64_t hu = fnv(b->d_U), hd = fnv(b->d_D);
    fprintf(stderr, "N4TRACE L%d it%d active %d U %016llx D %016llx conv_w %.9g%s\n", L, it, s.active,
            (unsigned long long)hu, (unsigned long long)hd, s.conv_w,
            s.conv_bound ? " (certified bound: decided above the threshold, not ITK's value)" : "");
}

// One sub-batch [vol0, vol0 + ns): the whole multi-level loop.  Flat sweeps run over the chunk
// range [cp[vol0], cp[vol0 + ns]); converged volumes' blocks exit at once.
static void n4_subbatch(vh_batch *b, const vh_n4_params &prm, int64_t vol0, int64_t ns,
                        const std::vector<int32_t> &hcp) {
    hipStream_t st = b->stream;
    const int64_t ntiles = b->n4_tiles;
    const int32_t ch0 = hcp[vol0], nch = hcp[vol0 + ns] - hcp[vol0];
    const int rsh = b->rsh;
    const int bins = prm.n_bins;
    const int cm = prm.conv_mode;
    const int LOOK = 3;
    const int nslots = (int)((b->R + SLOT_R - 1) / SLOT_R);
    const int nitems = (int)ntiles * nslots;
    const dim3 fg((unsigned)((nitems + FIT_WAVES - 1) / FIT_WAVES), (unsigned)ns);
    float *U = b->d_U;
    std::vector<hipEvent_t> evs;
    std::vector<int> ev_slot;   // iteration slot (d_nactive / h_flags index) behind each event
    if (!b->h_flags) HIP_TRY(hipHostMalloc((void **)&b->h_flags, sizeof(int32_t) * 1024));
    volatile int32_t *hflag = b->h_flags;   // written by k_n4_emap through its device mapping
    int32_t *dflag = nullptr;
    HIP_TRY(hipHostGetDevicePointer((void **)&dflag, b->h_flags, 0));
    // studies with many chunks: their chunk histograms are summed in slices first (k_n4_hred)
    int32_t max_ch = 0;
    for (int64_t v = vol0; v < vol0 + ns; ++v) max_ch = std::max(max_ch, hcp[v + 1] - hcp[v]);
    uint64_t *hred = nullptr;
    if (max_ch >= 4 * N4_HSL) {
        const size_t need = sizeof(uint64_t) * (size_t)ns * N4_HSL * 2 * VH_MAX_BINS;
        if (need > b->hred_cap) {
            if (b->d_hred) HIP_TRY(hipFree(b->d_hred));
            b->d_hred = nullptr;
            b->hred_cap = 0;
            HIP_TRY(hipMalloc(&b->d_hred, need));
            b->hred_cap = need;
        }
        hred = b->d_hred;
    }
    int total_iters = 0;
    for (int L = 0; L < prm.n_levels; ++L) total_iters += prm.max_iters[L];
    HIP_TRY(hipMemsetAsync(b->d_nactive, 0, sizeof(int32_t) * (total_iters + 1), st));
    int gi = 0;   // iteration slot within this sub-batch
    try {
        for (int L = 0; L < prm.n_levels; ++L) {
            const DevLevel lv = vh_dev_level(b, prm, L);
            const int ncx = lv.ax[0].ncp;
            const int rowcap = fit_rowcap(b, prm, L);
            const size_t fit_lds = sizeof(double) * FIT_WAVES * 2 * FIT_NB * (size_t)rowcap;
            if (fit_lds > 150 * 1024)
                throw VhError{VH_ERR_ARG, "N4 fit: tile contraction rows exceed the LDS budget"};
            vh_set_max_lds((const void *)k_n4_fit_items<0>, 150 * 1024);
            vh_set_max_lds((const void *)k_n4_fit_items<1>, 150 * 1024);
            const int64_t nlat = (int64_t)ncx * lv.ax[1].ncp * lv.ax[2].ncp;
            const dim3 lg((unsigned)ns, (unsigned)((nlat + VH_TPB - 1) / VH_TPB));
            const dim3 zg((unsigned)((2 * nlat + VH_TPB - 1) / VH_TPB), (unsigned)ns);
            const dim3 pg((unsigned)ns, (unsigned)((nlat / lv.ax[2].ncp * b->Z + VH_TPB - 1) / VH_TPB));
            {
                ScopedKTimer tm(b, "n4_den", 0.0);
                k_n4_fit_clear<1><<<zg, VH_TPB, 0, st>>>(b->d_numfix, b->lat_cap, nlat, b->d_st, vol0);
                VH_CHECK_LAUNCH();
                k_n4_fit_items<1><<<fg, FIT_WAVES * 64, fit_lds, st>>>(
                    U, b->d_rowstart, b->d_rowmask, b->d_sc, (int)b->R, (int)b->C, (int)b->Z, b->VS,
                    (int)ntiles, nslots, bins, b->d_st, b->d_E, lv, rowcap, FIT_NB, b->d_numfix,
                    b->lat_cap, vol0);
                VH_CHECK_LAUNCH();
                k_n4_latupd<1><<<lg, VH_TPB, 0, st>>>(b->d_numfix, b->d_lat, b->d_den, b->lat_cap,
                                                      nlat, b->d_st, vol0);
                VH_CHECK_LAUNCH();
            }
            const int level_start = (int)evs.size();
            // S7: PC (k_n4_pcw) unless VH_N4_SERIAL_CHAIN selects the serial chain (A/B runs)
            const bool pc = getenv("VH_N4_SERIAL_CHAIN") == nullptr;
            // a launch of one large volume: the grid form (k_n4_pcg) over up to one workgroup per CU,
            // ~64+ steps per chain block (VH_N4_PCG=0 keeps the one-workgroup form)
            int pcg_grid = 0;
            PcgArgs pcg_args{};
            Pcg2Args pcg2_args{};
            // VH_PCG_V=1: the round-4 grid PC (two grid barriers per round, no stage 0 / decision)
            const bool pcg_v1 = getenv("VH_PCG_V") && atoi(getenv("VH_PCG_V")) == 1;
            if (cm == 0 && pc && ns == 1 && b->V >= ((int64_t)1 << 20) &&
                !(getenv("VH_N4_PCG") && atoi(getenv("VH_N4_PCG")) == 0)) {
                int dev = 0, ncu = 0, per = 0;
                HIP_TRY(hipGetDevice(&dev));
                HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
                // the occupancy of the kernel actually launched (k_n4_pcg2 unless VH_PCG_V=1: other
                // LDS and register use); a cooperative launch larger than fits would fail
                HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(
                    &per, pcg_v1 ? (const void *)k_n4_pcg : (const void *)k_n4_pcg2, PC_TPB, 0));
                if (per < 1) throw VhError{VH_ERR_ARG, "N4 grid PC: no workgroup fits on a CU"};
                // ~1/4 of V masked, VH_PCG_STEPS (default 16) steps per chain block (config 2: 64 -> 16
                // steps: n4_pcg 14.4 -> 10.3 ms per study; config 5 is at one workgroup per CU anyway)
                const int64_t spb = getenv("VH_PCG_STEPS") ? std::max(1, atoi(getenv("VH_PCG_STEPS"))) : 16;
                const int64_t want = (b->V / 4 + PC_TPB * spb - 1) / (PC_TPB * spb);
                // at most one workgroup per CU whatever the occupancy API says: it can report one
                // block per CU too many, and the cooperative launch accepts an over-size grid
                // whose grid barrier would then never complete (MI355X_MICROARCH.md, correctness)
                pcg_grid = (int)std::max<int64_t>(1, std::min<int64_t>(want, (int64_t)std::min(per, 1) * ncu));
                const int64_t NB = (int64_t)pcg_grid * PC_TPB;
                const size_t need = NB * (6 * sizeof(float) + 2 * sizeof(double)) +
                                    (size_t)pcg_grid * (3 * sizeof(double) + sizeof(int)) + 256 +
                                    2 * (size_t)pcg_grid * sizeof(PcgWg) + 2 * (size_t)NB * sizeof(float) + 256;
                if ((int64_t)need > b->pcg_cap) {
                    if (b->d_pcg) HIP_TRY(hipFree(b->d_pcg));
                    b->d_pcg = nullptr;
                    b->pcg_cap = 0;
                    HIP_TRY(hipMalloc(&b->d_pcg, need));
                    b->pcg_cap = (int64_t)need;
                }
                char *w = (char *)b->d_pcg;
                pcg_args.s1 = (double *)w; w += NB * sizeof(double);
                pcg_args.s2 = (double *)w; w += NB * sizeof(double);
                pcg_args.agA = (double *)w; w += pcg_grid * sizeof(double);
                pcg_args.agB = (double *)w; w += pcg_grid * sizeof(double);
                pcg_args.agS = (double *)w; w += pcg_grid * sizeof(double);
                float **fa[6] = {&pcg_args.gmu, &pcg_args.gsig, &pcg_args.emu, &pcg_args.esig,
                                 &pcg_args.gmu_o, &pcg_args.emu_o};
                for (int q = 0; q < 6; ++q) { *fa[q] = (float *)w; w += NB * sizeof(float); }
                pcg_args.agF = (int *)w; w += pcg_grid * sizeof(int);
                pcg_args.sc = b->d_sc;
                pcg_args.st = b->d_st;
                w = (char *)(((uintptr_t)w + 255) & ~(uintptr_t)255);
                pcg2_args.wg = (PcgWg *)w; w += 2 * (size_t)pcg_grid * sizeof(PcgWg);
                pcg2_args.E = (float *)w;
                pcg2_args.sc = b->d_sc;
                // VH_PCG_T0=0: pass 0 reads each thread's own block (the round-5 form, A/B runs)
                pcg2_args.t0 = !(getenv("VH_PCG_T0") && atoi(getenv("VH_PCG_T0")) == 0);
                pcg2_args.st = b->d_st;
            }
            for (int it = 0; it < prm.max_iters[L]; ++it, ++gi) {
                k_n4_ctrl<<<(unsigned)ns, VH_TPB, 0, st>>>(
                    b->d_st, b->d_cpart, b->d_cp, b->d_sc, cm, L, it, prm.conv_threshold, bins, vol0,
                    b->d_nactive + gi, U, b->d_colbits, b->d_rowstart, b->R, b->CZ, b->VS, ntiles);
                VH_CHECK_LAUNCH();
                if (nch > 0) {
                    ScopedKTimer tm(b, "n4_hist", 0.0);
                    k_n4_hist<<<(unsigned)nch, VH_TPB, 0, st>>>(U, b->d_cp, b->d_cvol, b->d_sc, b->VS,
                                                                bins, b->d_st, b->d_hpart, ch0);
                    VH_CHECK_LAUNCH();
                }
                if (hred) {
                    k_n4_hred<<<dim3(N4_HSL, (unsigned)ns), VH_TPB, 0, st>>>(b->d_hpart, b->d_cp, b->d_st,
                                                                             bins, hred, vol0);
                    VH_CHECK_LAUNCH();
                }
                k_n4_emap<<<(unsigned)ns, VH_TPB, 0, st>>>(b->d_hpart, b->d_cp, b->d_twiddle, bins,
                                                           prm.fwhm, prm.wiener_noise, b->d_st,
                                                           b->d_E, vol0, hred, b->d_nactive + gi,
                                                           dflag + (gi % 1024));
                VH_CHECK_LAUNCH();
                {
                    hipEvent_t ev;
                    HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
                    evs.push_back(ev);
                    ev_slot.push_back(gi);
                    HIP_TRY(hipEventRecord(ev, st));
                }
                {
                    ScopedKTimer tm(b, "n4_fit", 0.0);
                    k_n4_fit_items<0><<<fg, FIT_WAVES * 64, fit_lds, st>>>(
                        U, b->d_rowstart, b->d_rowmask, b->d_sc, (int)b->R, (int)b->C, (int)b->Z,
                        b->VS, (int)ntiles, nslots, bins, b->d_st, b->d_E, lv, rowcap, FIT_NB,
                        b->d_numfix, b->lat_cap, vol0);
                    VH_CHECK_LAUNCH();
                }
                {
                    ScopedKTimer tm(b, "n4_contract", 0.0);
                    k_n4_latupd<0><<<lg, VH_TPB, 0, st>>>(b->d_numfix, b->d_lat, b->d_den, b->lat_cap,
                                                          nlat, b->d_st, vol0);
                    VH_CHECK_LAUNCH();
                    k_n4_P1<<<pg, VH_TPB, 0, st>>>(b->d_lat, b->lat_cap, b->d_P1, b->q2_cap, b->Z,
                                                   b->d_st, lv, vol0);
                    VH_CHECK_LAUNCH();
                    k_n4_T<<<dim3((unsigned)((b->CZ * ncx + VH_TPB - 1) / VH_TPB), (unsigned)ns), VH_TPB, 0, st>>>(b->d_P1, b->q2_cap, b->C, b->Z, lv, b->d_st,
                                                  b->d_T, b->nb * b->t_cap, b->t_cap, vol0);
                    VH_CHECK_LAUNCH();
                }
                if (nch > 0) {
                    ScopedKTimer tm(b, "n4_eval", 0.0);
                    const DevLevel lvo = (it == 0 && L > 0) ? vh_dev_level(b, prm, L - 1) : lv;
                    const int bo_mode = (it == 0 && L == 0) ? 0 : 1;
                    k_n4_eval<<<(unsigned)nch, VH_TPB, (size_t)b->R * 40, st>>>(
                        b->d_L0, U, b->d_ridx, b->d_cp, b->d_cvol, b->d_sc, b->R, b->CZ, b->VS, rsh,
                        b->d_T, b->nb * b->t_cap, b->t_cap, lv, lvo, bo_mode, b->d_st, b->d_cpart,
                        ch0, cm, b->d_D);
                    VH_CHECK_LAUNCH();
                }
                if (cm == 0 && !pc) {
                    ScopedKTimer tm(b, "n4_welford", 0.0);
                    k_n4_welford<<<(unsigned)ns, WF_TPB, 0, st>>>(b->d_D, b->d_perm, b->VS, b->d_sc,
                                                               b->d_st, vol0);
                    VH_CHECK_LAUNCH();
                } else if (cm == 0 && pcg_grid > 0 && !pcg_v1) {   // one large study: PC over the GPU
                    ScopedKTimer tm(b, "n4_pcg", 0.0, true);   // stamped: a cooperative launch
                    Pcg2Args A = pcg2_args;
                    A.kst = tm.stamp();
                    A.b = vol0;
                    A.D = b->d_D + vol0 * b->VS;
                    A.perm = b->d_perm + vol0 * b->VS;
                    A.P = b->d_D + (b->nb + vol0) * b->VS;
                    A.skip_thresh = it + 1 < prm.max_iters[L] ? prm.conv_threshold : 0.0f;
                    void *args[] = {&A};
                    HIP_TRY(hipLaunchCooperativeKernel((const void *)k_n4_pcg2, dim3((unsigned)pcg_grid),
                                                       dim3(PC_TPB), args, 0, st));
                } else if (cm == 0 && pcg_grid > 0) {
                    ScopedKTimer tm(b, "n4_pcg", 0.0);
                    PcgArgs A = pcg_args;
                    A.b = vol0;
                    A.D = b->d_D + vol0 * b->VS;
                    A.perm = b->d_perm + vol0 * b->VS;
                    A.P = b->d_D + (b->nb + vol0) * b->VS;
                    void *args[] = {&A};
                    HIP_TRY(hipLaunchCooperativeKernel((const void *)k_n4_pcg, dim3((unsigned)pcg_grid),
                                                       dim3(PC_TPB), args, 0, st));
                } else if (cm == 0) {
                    ScopedKTimer tm(b, "n4_pcw", 0.0);
                    vh_set_max_lds((const void *)k_n4_pcw, (int)pcw_lds_bytes<PC_TPB>());
                    k_n4_pcw<<<(unsigned)ns, PC_TPB, pcw_lds_bytes<PC_TPB>(), st>>>(
                        b->d_D, b->d_perm, b->d_D + b->nb * b->VS, b->VS, b->d_sc, b->d_st, vol0,
                        it + 1 < prm.max_iters[L] ? prm.conv_threshold : 0.0f);
                    VH_CHECK_LAUNCH();
                }
                if (getenv("VH_N4_TRACE")) n4_trace(b, vol0, L, it);
                const int k = (int)evs.size() - 1 - LOOK;
                if (k >= level_start) {
                    HIP_TRY(hipEventSynchronize(evs[k]));
                    // the flag the event covers (slots skip one per early exit: gi != event index)
                    if (hflag[ev_slot[k] % 1024] == 0) { ++gi; break; }
                }
            }
            k_n4_level_end<<<(unsigned)ns, 64, 0, st>>>(b->d_st, b->d_cpart, b->d_cp, b->d_sc, cm, L,
                                                        vol0);
            VH_CHECK_LAUNCH();
            if (L < prm.n_levels - 1) {
                k_n4_refine<<<(unsigned)ns, VH_TPB, 0, st>>>(b->d_lat, b->lat_cap, b->nb,
                                                             lv.ax[0].ncp, lv.ax[1].ncp,
                                                             lv.ax[2].ncp, vol0);
                VH_CHECK_LAUNCH();
            }
        }
    } catch (...) {
        for (auto e : evs) (void)hipEventDestroy(e);
        throw;
    }
    for (auto e : evs) HIP_TRY(hipEventDestroy(e));
}

void vh_launch_n4(vh_batch *b, const vh_n4_params &prm) {
    hipStream_t st = b->stream;
    vh_ensure_n4_workspace(b, prm);
    const int64_t ntiles = b->n4_tiles;
    HIP_TRY(hipMemsetAsync(b->d_lat, 0, sizeof(float) * b->nb * b->lat_cap, st));
    k_n4_state_init<<<(unsigned)((b->nb + 255) / 256), 256, 0, st>>>(b->d_st, b->nb);
    VH_CHECK_LAUNCH();
    // driver: volume-resident (one workgroup per study) when the batch has studies for the CUs
    // and a study's state fits in LDS, else per-iteration sweeps over the whole batch
    int mode = b->n4_mode;
    if (const char *e = getenv("VH_N4_MODE")) mode = atoi(e);
    size_t study_lds = 0;
    const bool fits = vh_n4_study_eligible(b, prm, &study_lds);
    if (getenv("VH_N4_DEBUG"))
        fprintf(stderr, "N4 study driver: %s, %zu B LDS\n", fits ? "eligible" : "not eligible", study_lds);
    if (mode == 2 && !fits) throw VhError{VH_ERR_ARG, "n4_mode=2: study state exceeds the LDS budget"};
    // the grid form (one study over G workgroups, one cooperative launch per study): a batch of one
    // study (the class's calls, configs 2 and 5 when their state fits); VH_N4_GRID=0 keeps the sweeps
    size_t grid_lds = 0;
    const bool gfits = (mode == 3 || (mode == 0 && b->nb == 1)) && vh_n4_studyg_eligible(b, prm, &grid_lds) &&
                       !(getenv("VH_N4_GRID") && atoi(getenv("VH_N4_GRID")) == 0);
    if (mode == 3 && !gfits) throw VhError{VH_ERR_ARG, "n4_mode=3: study state exceeds the grid form's LDS budget"};
    const bool use_grid = mode == 3 || (mode == 0 && b->nb == 1 && gfits);
    b->n4_used_study = mode == 2 || (mode == 0 && fits && b->nb >= 16) || use_grid;
    {
        ScopedKTimer tm(b, "n4_init", 0.0);
        const int64_t nrs = ntiles * b->R;
        const bool prep = nrs <= RP_MAX_NRS && b->R <= RP_MAX_R && !getenv("VH_ROWPREP_OLD");
        if (prep) {   // masks, counts, raster ranks and offsets in one launch per volume
            k_n4_rowprep<<<(unsigned)b->nb, RP_TPB, sizeof(int32_t) * (size_t)(nrs + b->R), st>>>(
                b->d_colbits, b->R, b->CZ, ntiles, b->d_rowstart, b->d_rowmask, b->d_rrank);
            VH_CHECK_LAUNCH();
        } else {
            k_n4_rowcount<<<dim3((unsigned)ntiles, (unsigned)b->nb), 64, 0, st>>>(
                b->d_colbits, b->R, b->CZ, ntiles, b->d_rowstart, b->d_rowmask);
            VH_CHECK_LAUNCH();
        }
        if (prep) {
        } else if (nrs <= ((int64_t)1 << 16)) {   // small volumes (the bench): one workgroup per volume
            k_n4_rowscan<<<(unsigned)b->nb, VH_TPB, 0, st>>>(b->d_rowstart, nrs);
            VH_CHECK_LAUNCH();
            if (b->R > 16384) throw VhError{VH_ERR_ARG, "N4: more than 16384 rows"};
            k_n4_rrank<<<(unsigned)b->nb, VH_TPB, sizeof(int32_t) * (size_t)b->R, st>>>(
                b->d_rowmask, b->d_rowstart, b->R, ntiles, b->VS, b->d_rrank, b->d_perm);
            VH_CHECK_LAUNCH();
        } else {   // large volumes: chunked scans over the GPU
            const int64_t ncs = (nrs + RS_CH - 1) / RS_CH, nrc = (ntiles + RR_CH - 1) / RR_CH;
            const int64_t need = b->nb * std::max(ncs, (nrc + 1) * b->R);
            if (need > b->iscan_cap) {
                if (b->d_iscan) HIP_TRY(hipFree(b->d_iscan));
                b->d_iscan = nullptr;
                b->iscan_cap = 0;
                HIP_TRY(hipMalloc(&b->d_iscan, sizeof(int32_t) * need));
                b->iscan_cap = need;
            }
            const dim3 gs((unsigned)ncs, (unsigned)b->nb), gr((unsigned)nrc, (unsigned)b->nb);
            k_n4_rowscan_parts<<<gs, VH_TPB, 0, st>>>(b->d_rowstart, nrs, b->d_iscan, ncs);
            VH_CHECK_LAUNCH();
            k_n4_rowscan_top<<<(unsigned)b->nb, VH_TPB, 0, st>>>(b->d_iscan, ncs);
            VH_CHECK_LAUNCH();
            k_n4_rowscan_apply<<<gs, VH_TPB, 0, st>>>(b->d_rowstart, nrs, b->d_iscan, ncs);
            VH_CHECK_LAUNCH();
            k_n4_rr_chunk<<<gr, VH_TPB, 0, st>>>(b->d_rowmask, b->R, ntiles, b->d_rrank, b->d_iscan, nrc);
            VH_CHECK_LAUNCH();
            k_n4_rr_top<<<(unsigned)b->nb, VH_TPB, 0, st>>>(b->d_iscan, b->R, nrc);
            VH_CHECK_LAUNCH();
            k_n4_rr_apply<<<gr, VH_TPB, 0, st>>>(b->R, ntiles, b->d_rrank, b->d_iscan, nrc);
            VH_CHECK_LAUNCH();
        }
        if (!b->n4_used_study) {   // raster rank -> compact index: the sweep driver's S7 walk only
            // (the study kernel writes d at its raster rank itself; 0.155 ms of the bench step)
            const int64_t pairs = ntiles * b->R;
            k_n4_perm<<<dim3((unsigned)((pairs + VH_TPB / 64 - 1) / (VH_TPB / 64)), (unsigned)b->nb), VH_TPB, 0, st>>>(
                b->d_rowmask, b->d_rowstart, b->d_rrank, b->R, ntiles, b->VS, b->d_perm);
            VH_CHECK_LAUNCH();
        }
    }
    if (!b->n4_used_study) {   // the study kernel computes L0 / U itself
        ScopedKTimer tm(b, "n4_init", 0.0);
        const dim3 sg((unsigned)((ntiles + 3) / 4), (unsigned)((b->R + SEG_R - 1) / SEG_R),
                      (unsigned)b->nb);
        k_n4_init<<<sg, VH_TPB, 0, st>>>(b->d_hp, b->d_colbits, b->d_rowstart, b->d_sc, b->R, b->CZ,
                                         b->V, b->VS, ntiles, b->d_L0, b->d_U, b->d_ridx,
                                         b->rsh, b->d_st);
        VH_CHECK_LAUNCH();
    }
    if (use_grid) {
        vh_launch_n4_studyg(b, prm);
    } else if (b->n4_used_study) {
        vh_launch_n4_study(b, prm);
    } else {
        std::vector<int32_t> hcp(b->nb + 1);
        k_n4_chunks<<<1, VH_TPB, 0, st>>>(b->d_sc, b->nb, b->d_cp, b->d_cvol);
        VH_CHECK_LAUNCH();
        HIP_TRY(hipMemcpyAsync(hcp.data(), b->d_cp, sizeof(int32_t) * (b->nb + 1),
                               hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        int64_t sb = b->n4_subbatch > 0 ? b->n4_subbatch : b->nb;
        if (const char *e = getenv("VH_N4_SUBBATCH")) {
            const long v = atol(e);
            if (v > 0) sb = v;
        }
        if (sb > b->nb) sb = b->nb;
        for (int64_t v0 = 0; v0 < b->nb; v0 += sb)
            n4_subbatch(b, prm, v0, std::min(sb, b->nb - v0), hcp);
    }
    {
        const DevLevel lv = vh_dev_level(b, prm, prm.n_levels - 1);
        ScopedKTimer tm(b, "n4_final", 9.0 * (double)b->V);
        const SnrBox sbox{b->d_rowany, b->d_sliceany, b->d_snrpart, b->slab_blocks};
        k_n4_final<<<slab_grid(b), VH_TPB, 0, st>>>(b->d_hp, b->d_n4, b->R, b->C, b->Z, b->V,
                                                    b->part_blocks, b->q2_cap, b->d_P1, lv,
                                                    b->d_colbits, b->d_colbnz, b->d_colstart,
                                                    b->d_sc, b->d_keys0, sbox);
        b->keys_fused = true;   // the VDP chain's gather is not needed
        b->snr_fused = true;    // and the SNR partials of the input image are done
        VH_CHECK_LAUNCH();
    }
}

