// n4_study.hip -- volume-resident N4 bias-field correction on gfx950: ONE workgroup (1024 threads,
// 16 waves) per study runs the whole multi-level iteration loop of
// sitk.N4BiasFieldCorrectionImageFilter (Vent_Analysis.py:316-334; CPU twin
// oracle/n4_oracle.c) in a single launch.  Between sweeps the study's small state -- B-spline
// lattice, fit denominators, the z-contracted lattices P1 (current and previous field), level
// tables, histogram, FFT buffers, E(u) map -- never leaves LDS, so an iteration costs three
// streaming passes over the compact masked voxels and workgroup barriers, with no kernel launches,
// no grid-wide dependencies and no host round trips.  A batch of >= one study per CU fills the
// chip (256 studies on 256 CUs); per-study work is a fixed 16 B per masked voxel per iteration.
//
// Per iteration (all inside the workgroup):
//   ctrl  convergence of the previous field, ITK's while-condition, bin range (+ the exact raster
//         minimum when the first masked voxel is the strict minimum)
//   hist  flat pass over compact U: triangular Parzen histogram, u64 fixed point, 8 LDS copies
//   emap  512-point radix-2 FFT Wiener deconvolution in LDS (two transforms per stage)
//   fit   column walk: a wave owns one (64-column tile, 64-row slot) item; each lane one column,
//         the row axis contracted in registers by a sliding 4-wide window (fixed row order, f64);
//         each finished control row i is contracted over the tile's slices and cols in the wave
//         and added to the lattice numerator with 128-bit fixed-point LDS atomics (order-free)
//   lat   phi = num / den, lattice += phi, P1 = lattice contracted over slices (f64)
//   eval  column walk again: per lane the column's T(i) window for the new and the previous
//         field (same float expressions as n4.hip's k_n4_T / k_n4_eval, so B_old is the previous
//         B_new exactly), U = L0 - B_new stored, convergence sums per item (summed in item order)
// Work items are taken from an LDS counter; every reduction is either integer (order-free) or
// per item in a fixed order, so results are deterministic.
#include <algorithm>
#include <cfloat>
#include <cstring>

#include "n4_shared.h"

#define ST_TPB 1024
#define ST_WAVES (ST_TPB / 64)
#define ST_G 8         // rows per lane with loads in flight together
#define ST_HC 8        // LDS histogram copies
#define ST_MAX_LDS (160 * 1024)

// ST_PROF builds (scripts/dev): block 0 prints shader cycles per phase at the end of the launch
#ifdef ST_PROF
#define ST_MARK(k) do { if (threadIdx.x == 0) { const unsigned long long _c = clock64(); \
    st_prof[k] += _c - st_t0; st_t0 = _c; } } while (0)
#else
#define ST_MARK(k) do { } while (0)
#endif

struct StudyLevels {
    DevLevel lv[VH_MAX_LEVELS];
    int32_t max_iters[VH_MAX_LEVELS];
};

struct StudyArgs {
    const float *I;     // HPvent [nb][R][C][Z] (the init pass computes L0 = log I here)
    int64_t V;
    float *L0;
    float *U;
    const int32_t *rs;
    const uint64_t *rmask;
    const VolScalars *sc;
    N4State *st;
    double *P1out;
    int64_t q2cap;
    const double2 *tw;
    int64_t VS;
    int32_t R, C, Z, CZ, ntiles, nslots, nitems;
    int32_t nlev, bins;
    float thresh, fwhm, noise;
    const StudyLevels *lvs;   // device copy: per-level tables and iteration caps
    // dynamic-LDS carve (byte offsets)
    int32_t o_E, o_tab0, o_tab1, o_lat, o_den, o_P10, o_P11, o_ipart, o_misc, o_scr, o_wave, o_order;
    int32_t s_cap;   // doubles of a wave's ring row (>= 64, >= ny * KT)
    int32_t nb_ring; // ring rows per wave (<= ST_NB)
    int32_t o_wx;    // row weights^P of the current level: Wx[2][R][4] doubles (p = 3, p = 2)
    int32_t o_wk;    // dense slice weights Wk[2][ncz][Z] (p = 3, p = 2) of the current level
    int32_t kcap;    // krange entries per table set
    int64_t vol0;
};

struct StudyMisc {
    int32_t item_ctr, stop, exact, pad;
    uint32_t umax_key, umin_key, umin2_key;   // max; min over all but the 1st / 1st and 2nd voxel
    float u_first, u_second, u_third, bin_min, slope, bmax;
    int32_t rx[3], rc[3];    // (row, column) of the first three masked voxels in raster order (-1: none)
    double sd, sd2, conv;
    int32_t nc[2][3];
};

// One level's axis tables staged in LDS.
struct TabV {
    float4 *wx, *wy, *wz;
    double *ix, *iy, *iz;
    int32_t *bx, *by, *bz;
    int2 *krz;
    int32_t *xst;   // [ncx - 2]: first row x with bx[x] >= i (xst[ncx - 3] = R)
};

__host__ __device__ inline size_t study_tab_bytes(int R, int C, int Z, int kcap) {
    return (((size_t)28 * (R + C + Z) + 12 * (size_t)kcap + 16) + 15) & ~(size_t)15;
}

__device__ __forceinline__ TabV tab_view(char *p, int R, int C, int Z, int kcap) {
    TabV t;
    t.wx = (float4 *)p; p += 16 * (size_t)R;
    t.wy = (float4 *)p; p += 16 * (size_t)C;
    t.wz = (float4 *)p; p += 16 * (size_t)Z;
    t.ix = (double *)p; p += 8 * (size_t)R;
    t.iy = (double *)p; p += 8 * (size_t)C;
    t.iz = (double *)p; p += 8 * (size_t)Z;
    t.bx = (int32_t *)p; p += 4 * (size_t)R;
    t.by = (int32_t *)p; p += 4 * (size_t)C;
    t.bz = (int32_t *)p; p += 4 * (size_t)Z;
    t.krz = (int2 *)(((uintptr_t)p + 7) & ~(uintptr_t)7);
    t.xst = (int32_t *)(t.krz + kcap);
    return t;
}

__device__ void load_tables(const TabV &t, const DevLevel &lv, int R, int C, int Z) {
    for (int x = threadIdx.x; x < R; x += ST_TPB) {
        t.wx[x] = *reinterpret_cast<const float4 *>(lv.ax[0].w + 4 * x);
        t.ix[x] = lv.ax[0].isw2[x];
        t.bx[x] = lv.ax[0].base[x];
    }
    for (int y = threadIdx.x; y < C; y += ST_TPB) {
        t.wy[y] = *reinterpret_cast<const float4 *>(lv.ax[1].w + 4 * y);
        t.iy[y] = lv.ax[1].isw2[y];
        t.by[y] = lv.ax[1].base[y];
    }
    for (int z = threadIdx.x; z < Z; z += ST_TPB) {
        t.wz[z] = *reinterpret_cast<const float4 *>(lv.ax[2].w + 4 * z);
        t.iz[z] = lv.ax[2].isw2[z];
        t.bz[z] = lv.ax[2].base[z];
    }
    for (int k = threadIdx.x; k < lv.ax[2].ncp; k += ST_TPB) t.krz[k] = lv.ax[2].krange[k];
    const int ncx = lv.ax[0].ncp;
    for (int i = threadIdx.x; i <= ncx - 3; i += ST_TPB) {   // spans of the row axis
        int x = 0;
        while (x < R && lv.ax[0].base[x] < i) ++x;
        t.xst[i] = i == ncx - 3 ? R : x;
    }
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t st_rsrc(const float *base, int64_t n) {
    return __builtin_amdgcn_make_buffer_rsrc((void *)base, 0, (int)(n * 4), 0x00020000);
}
__device__ __forceinline__ float st_load(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, 0, 0));
}
__device__ __forceinline__ void st_store(__amdgpu_buffer_rsrc_t r, uint32_t voff, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, (int)voff, 0, 0);
}
// c / slope as IEEE float division, evaluated as (double)c * (1 / (double)slope) rounded once to
// float.  The double product is within 2^-52 (relative) of the exact quotient, and a quotient of
// two floats is never closer than 2^-49 (relative) to a float rounding midpoint, so the rounding
// lands on the correctly rounded quotient: bit-equal to c / slope (also checked on 4e8 random
// pairs), including 0, inf and NaN cases, at a quarter of the instructions.
__device__ __forceinline__ float div_r(float c, double rinv) { return (float)((double)c * rinv); }

// sharpen_value / parzen_bin (n4_shared.h) with the bin division in div_r form
__device__ __forceinline__ float sharpen_r(float u, float bmin, double rinv, const float *E, int bins) {
    const float cidx = div_r(u - bmin, rinv);
    const int idx = (cidx >= 0.0f && cidx < (float)bins) ? (int)floorf(cidx) : bins;
    if (idx < bins - 1) return E[idx] + (E[idx + 1] - E[idx]) * (cidx - (float)idx);
    return E[bins - 1];
}
__device__ __forceinline__ bool parzen_bin_r(float u, float bmin, double rinv, int bins, int &idx,
                                             unsigned long long &a0, unsigned long long &a1) {
    const float cidx = div_r(u - bmin, rinv);
    if (!(cidx >= 0.0f) || !(cidx < (float)bins)) return false;
    idx = (int)floorf(cidx);
    const float o = cidx - (float)idx;
    a1 = 0ull;
    if (o == 0.0f) {
        a0 = 1ull << 32;
    } else if (idx < bins - 1) {
        const float om = 1.0f - o;
        a0 = om == 1.0f ? (1ull << 32) : (unsigned long long)(uint32_t)((double)om * 4294967296.0);
        a1 = (unsigned long long)(uint32_t)((double)o * 4294967296.0);
    } else {
        return false;
    }
    return true;
}

// parzen_bin_r without branches: idx in [0, bins - 1], zero weights where parzen_bin adds nothing
__device__ __forceinline__ void parzen_bin_bf(float u, float bmin, double rinv, int bins, int &idx,
                                              unsigned long long &a0, unsigned long long &a1) {
    const float cidx = div_r(u - bmin, rinv);
    const bool in = cidx >= 0.0f && cidx < (float)bins;   // false for NaN
    const float cf = in ? floorf(cidx) : 0.0f;
    const float o = in ? cidx - cf : 0.0f;
    const bool zero = o == 0.0f, inner = (int)cf < bins - 1;
    const float om = 1.0f - o;
    // x * 2^32 is exact in float (power-of-two scale, < 2^32): the f32 -> u32 truncation equals
    // the double-path truncation of n4_shared.h parzen_bin
    const unsigned long long w0 =
        (zero || om == 1.0f) ? (1ull << 32) : (unsigned long long)(uint32_t)(om * 4294967296.0f);
    a0 = in && (zero || inner) ? w0 : 0ull;
    a1 = in && !zero && inner ? (unsigned long long)(uint32_t)(o * 4294967296.0f) : 0ull;
    idx = (int)cf;
}

__device__ __forceinline__ float wsel(float4 w, int d) {
    return d == 0 ? w.x : d == 1 ? w.y : d == 2 ? w.z : w.w;
}
template <int P>
__device__ __forceinline__ double wpow(float w) {
    const double d = (double)w;
    return P == 3 ? d * d * d : d * d;
}

// ---------------------------------------------------------------------------------------------
// work item = (64-column tile, 64-row slot): the wave's view of its rows
// ---------------------------------------------------------------------------------------------
struct Item {
    int tile, x0, xs, xe;     // wave-uniform: tile, slot's first row, first / last non-empty row
    uint64_t mreg;            // lane l: mask == 1 lanes of row x0 + l
    int rsreg;                // lane l: compact offset of row x0 + l
    int col, y, z;            // this lane's column
    bool colok;
    // tile geometry (uniform)
    int c0, y0, y1, z0, z1, ny;
};

__device__ __forceinline__ bool item_begin(Item &it, const StudyArgs &a, int64_t b, int item) {
    const int lane = threadIdx.x & 63;
    it.tile = item / a.nslots;
    it.x0 = (item % a.nslots) * 64;
    const int64_t rbase = ((int64_t)b * a.ntiles + it.tile) * a.R;
    const int xr = it.x0 + lane;
    it.mreg = xr < a.R ? a.rmask[rbase + xr] : 0ull;
    it.rsreg = xr < a.R ? a.rs[rbase + xr] : 0;
    const uint64_t nzb = __ballot(it.mreg != 0ull);
    if (nzb == 0ull) return false;
    it.xs = it.x0 + __builtin_ctzll(nzb);
    it.xe = it.x0 + 63 - __builtin_clzll(nzb);
    it.col = it.tile * TILE_W + lane;
    it.colok = it.col < a.CZ;
    it.y = it.colok ? it.col / a.Z : 0;
    it.z = it.colok ? it.col % a.Z : 0;
    it.c0 = it.tile * TILE_W;
    const int c1 = min(it.c0 + TILE_W, a.CZ) - 1;
    it.y0 = it.c0 / a.Z;
    it.y1 = c1 / a.Z;
    it.z0 = it.c0 % a.Z;
    it.z1 = c1 % a.Z;
    it.ny = it.y1 - it.y0 + 1;
    return true;
}

// Compact byte offset of (row x, this lane) or VH_OOB when the voxel is not in the mask; x is
// wave-uniform and inside the item's slot.
__device__ __forceinline__ uint32_t item_off(const Item &it, int x, bool valid) {
    const int lane = threadIdx.x & 63;
    const int xl = x - it.x0;
    const uint32_t mlo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)it.mreg, xl);
    const uint32_t mhi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(it.mreg >> 32), xl);
    const uint64_t m = ((uint64_t)mhi << 32) | mlo;
    const int r0 = __builtin_amdgcn_readlane(it.rsreg, xl);
    const bool on = valid && ((m >> lane) & 1ull);
    return on ? (uint32_t)(r0 + lanes_below(m)) * 4u : VH_OOB;
}

// Exact, order-free accumulation of doubles with a huge dynamic range: 128-bit two's-complement
// fixed point in units of 2^-80 (|v| < 2^37), kept as (lo u64, hi i64) and added with integer LDS
// atomics, the low word's carry detected from the value the atomic returns.  A 64-bit 2^-32 grid
// is too coarse here: the tile slabs are already contracted over cols and slices, and edge control
// points collect products of three cubed weights (den ~ 1e-12 and below).
__device__ __forceinline__ void fix128_add(unsigned long long *lo, unsigned long long *hi, double v) {
    const double s = fabs(v) * 65536.0;            // |v| * 2^16, exact
    const double fh = floor(s);
    unsigned long long h = (unsigned long long)fh; // s < 2^53
    const double r = s - fh;                       // fractional bits of s: [0, 1), exact
    unsigned long long l = (unsigned long long)(r * 18446744073709551616.0);   // < 2^64
    if (v < 0.0) {                                 // two's-complement negation of (h, l)
        l = ~l + 1ull;
        h = ~h + (l == 0ull ? 1ull : 0ull);
    }
    const unsigned long long old = atomicAdd(lo, l);
    const unsigned long long carry = old + l < old ? 1ull : 0ull;
    atomicAdd(hi, h + carry);
}
__device__ __forceinline__ double fix128_get(const unsigned long long *lo, const unsigned long long *hi) {
    return (double)(long long)*hi * (1.0 / 65536.0) + (double)*lo * 8.271806125530277e-25;   // 2^-80
}

// ---------------------------------------------------------------------------------------------
// fit: contraction of finished control rows of the item's tile (wave-collective).  A wave keeps
// up to ST_NB finished rows Q[r][lane] (control rows i0 .. i0+nr-1) in its LDS ring and contracts
// them together, so the dependent LDS chains of the contraction are paid once per batch:
//   S[r][y][k]    = sum_{z of row y in the tile} Wk[k][z] Q[r][(y, z)]     (Wk = wz(z, k)^P, dense)
//   num[i0+r][j][k] += sum_y wy(y, j)^P S[r][y][k]                        (128-bit fixed point)
// S overwrites Q in place (all reads of a batch finish before its writes).
// ---------------------------------------------------------------------------------------------
#define ST_NB 4        // finished control rows per contraction batch
#define ST_SO 4        // stage-1 outputs per lane per batch (nr * ny * KT <= 64 * ST_SO)

struct FitRing {
    double *q;        // [ST_NB][rowcap] this wave's rows
    int rowcap;       // doubles per row (>= 64, >= ny * KT)
    int nbmax;        // rows per batch for this geometry
    int nr, i0;       // rows held, control row of row 0
};

template <int P>
__device__ void fit_contract(FitRing &rg, const Item &it, const TabV &T, const double *Wk, int ncy,
                             int ncz, int Z, unsigned long long *numfix) {
    const int nr = rg.nr;
    if (nr == 0) return;
    const int lane = threadIdx.x & 63;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int klo = T.bz[it.y0 == it.y1 ? it.z0 : 0];
    const int KT = T.bz[it.y0 == it.y1 ? it.z1 : Z - 1] + 4 - klo;
    const int nyk = it.ny * KT;
    // the ST_SO outputs of a lane are independent fma chains over their slices: walk them in
    // lockstep (step s of every chain together) so the LDS latency of one chain hides behind the
    // others; each chain still adds its terms in slice order, so the sums are unchanged
    double outv[ST_SO];
    const double *qp[ST_SO], *wp[ST_SO];
    int len[ST_SO];
    int maxlen = 0;
#pragma unroll
    for (int q = 0; q < ST_SO; ++q) {
        outv[q] = 0.0;
        len[q] = 0;
        qp[q] = rg.q;
        wp[q] = Wk;
        const int o = lane + 64 * q;
        if (o >= nr * nyk) continue;
        const int r = o / nyk, yk = o % nyk;
        const int yy = yk / KT, k = klo + yk % KT, yv = it.y0 + yy;
        const int zlo = yv == it.y0 ? it.z0 : 0, zhi = yv == it.y1 ? it.z1 : Z - 1;
        const int2 kr = T.krz[k];
        const int zs = max(zlo, kr.x), ze = min(zhi, kr.y);
        qp[q] = rg.q + r * rg.rowcap + (yv * Z - it.c0) + zs;
        wp[q] = Wk + k * Z + zs;
        len[q] = max(ze - zs + 1, 0);
        maxlen = max(maxlen, len[q]);
    }
#pragma unroll 1
    for (int s = 0; s < maxlen; ++s) {
#pragma unroll
        for (int q = 0; q < ST_SO; ++q) {
            const int ss = min(s, max(len[q] - 1, 0));   // in-range read for finished chains
            const double v = fma(wp[q][ss], qp[q][ss], outv[q]);
            outv[q] = s < len[q] ? v : outv[q];
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int q = 0; q < ST_SO; ++q) {
        const int o = lane + 64 * q;
        if (o < nr * nyk) rg.q[(o / nyk) * rg.rowcap + o % nyk] = outv[q];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int jlo = T.by[it.y0];
    const int JT = T.by[it.y1] + 4 - jlo;
    const int njk = JT * KT;
    for (int o = lane; o < nr * njk; o += 64) {
        const int r = o / njk, jk = o % njk;
        const int j = jlo + jk / KT, kk = jk % KT, k = klo + kk;
        const double *sr = rg.q + r * rg.rowcap;
        double acc = 0.0;
        for (int yy = 0; yy < it.ny; ++yy) {
            const int d = j - T.by[it.y0 + yy];
            if (d < 0 || d > 3) continue;
            acc = fma(wpow<P>(wsel(T.wy[it.y0 + yy], d)), sr[yy * KT + kk], acc);
        }
        if (acc != 0.0) {
            const int64_t e = ((int64_t)(rg.i0 + r) * ncy + j) * ncz + k;
            fix128_add(numfix + 2 * e, numfix + 2 * e + 1, acc);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    rg.nr = 0;
}

// control row i (this lane's value v) is finished: into the ring, contract when the batch is full
template <int P>
__device__ __forceinline__ void fit_push(FitRing &rg, double v, int i, const Item &it,
                                         const TabV &T, const double *Wk, int ncy, int ncz, int Z,
                                         unsigned long long *numfix) {
    if (rg.nr == 0) rg.i0 = i;
    rg.q[rg.nr * rg.rowcap + (threadIdx.x & 63)] = v;
    if (++rg.nr == rg.nbmax) fit_contract<P>(rg, it, T, Wk, ncy, ncz, Z, numfix);
}

// MODE 0: numerator (w^3, q = (u - sharpen(u)) / (sum wx^2 sum wy^2 sum wz^2));
// MODE 1: denominator (w^2, q = 1).
template <int MODE>
__device__ void fit_item(const StudyArgs &a, const Item &it, const TabV &T, const double *Wk,
                         const double2 *Wx, int ncy, int ncz, const float *Ub, int64_t n,
                         const float *sE, float bmin, double rinv, FitRing &rg,
                         unsigned long long *numfix) {
    constexpr int P = MODE == 0 ? 3 : 2;
    const __amdgpu_buffer_rsrc_t rU = st_rsrc(Ub, n);
    const double isyz = MODE == 0 ? T.iy[it.y] * T.iz[it.z] : 1.0;
    int wb = T.bx[it.xs];
    double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0, acc3 = 0.0;
    int x = it.xs, tail = 0;
    {   // rows per batch: the stage-1 outputs of a batch must fit the lanes' ST_SO slots
        const int klo = T.bz[it.y0 == it.y1 ? it.z0 : 0];
        const int KT = T.bz[it.y0 == it.y1 ? it.z1 : a.Z - 1] + 4 - klo;
        rg.nbmax = max(1, min(a.nb_ring, 64 * ST_SO / (it.ny * KT)));
        rg.nr = 0;
    }
#pragma unroll 1
    for (;;) {
        if (x <= it.xe) {   // rows of control span wb: the window does not move
            const int rb = min(it.xe, T.xst[wb + 1] - 1);
#pragma unroll 1
            for (int xb = x; xb <= rb; xb += ST_G) {
                uint32_t offs[ST_G];
                float u[ST_G];
#pragma unroll
                for (int g = 0; g < ST_G; ++g) {
                    const int xg = xb + g;
                    offs[g] = item_off(it, xg <= rb ? xg : rb, xg <= rb);
                    if (MODE == 0) u[g] = st_load(rU, offs[g]);
                }
#pragma unroll
                for (int g = 0; g < ST_G; ++g) {
                    if (offs[g] == VH_OOB) continue;
                    const int xg = xb + g;
                    const double2 wa = Wx[2 * xg], wc = Wx[2 * xg + 1];   // wx(x, 0..3)^P
                    if (MODE == 0) {
                        const float rv = u[g] - sharpen_r(u[g], bmin, rinv, sE, a.bins);
                        const double q = ((double)rv * T.ix[xg]) * isyz;
                        acc0 += wa.x * q;
                        acc1 += wa.y * q;
                        acc2 += wc.x * q;
                        acc3 += wc.y * q;
                    } else {
                        acc0 += wa.x;
                        acc1 += wa.y;
                        acc2 += wc.x;
                        acc3 += wc.y;
                    }
                }
            }
            x = rb + 1 > x ? rb + 1 : x;
        }
        fit_push<P>(rg, acc0, wb, it, T, Wk, ncy, ncz, a.Z, numfix);   // control row wb is done
        acc0 = acc1; acc1 = acc2; acc2 = acc3; acc3 = 0.0;
        ++wb;
        if (x > it.xe && ++tail == 4) break;
    }
    fit_contract<P>(rg, it, T, Wk, ncy, ncz, a.Z, numfix);
}

// ---------------------------------------------------------------------------------------------
// U range for the next histogram.  ITK scans in raster order with
//   if (u > max) max = u; else if (u < min) min = u;
// so the minimum skips every "record" voxel (strictly above all earlier ones).  The records that
// can matter form the strictly increasing run u1 < u2 < ... < uK at the start of the raster order
// (a later record is above a non-record voxel), so min = min over voxels after that run.  The
// sweeps track min over all voxels but the 1st (K = 1) and but the 1st and 2nd (K = 2) together
// with u1, u2, u3; a run of 3 or more falls back to the exact raster scan.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ bool item_has(const Item &it, int x, int col) {
    return x >= it.xs && x <= it.xe && col >= it.c0 && col < it.c0 + TILE_W;
}
__device__ __forceinline__ void range_special(StudyMisc &M, int x, int col, float u, float &umin,
                                              float &umin2) {
    if (x == M.rx[0] && col == M.rc[0]) {
        M.u_first = u;
        return;
    }
    umin = fminf(umin, u);
    if (x == M.rx[1] && col == M.rc[1]) {
        M.u_second = u;
        return;
    }
    umin2 = fminf(umin2, u);
    if (x == M.rx[2] && col == M.rc[2]) M.u_third = u;
}
__device__ __forceinline__ void range_commit(StudyMisc &M, float umax, float umin, float umin2) {
    uint32_t kmax = umax == -FLT_MAX ? 0u : f2key(umax);
    uint32_t kmin = umin == FLT_MAX ? 0xffffffffu : f2key(umin);
    uint32_t kmin2 = umin2 == FLT_MAX ? 0xffffffffu : f2key(umin2);
    kmax = wave_max_u32(kmax);
    kmin = wave_min_u32(kmin);
    kmin2 = wave_min_u32(kmin2);
    if ((threadIdx.x & 63) == 0) {
        if (kmax) atomicMax(&M.umax_key, kmax);
        if (kmin != 0xffffffffu) atomicMin(&M.umin_key, kmin);
        if (kmin2 != 0xffffffffu) atomicMin(&M.umin2_key, kmin2);
    }
}

// Init + range of the initial field over one item: L0 = log(I) at mask == 1 (k_n4_init's
// expression; non-positive -> 0), U = L0 (B = 0), same range bookkeeping as the eval.  Replaces the
// separate k_n4_init sweep in this driver (the volume-resident kernel reads I directly).
__device__ void init_item(const StudyArgs &a, int64_t b, const Item &it, float *Lb, float *Ub,
                          int64_t n, StudyMisc &M) {
    const __amdgpu_buffer_rsrc_t rL = st_rsrc(Lb, n), rU = st_rsrc(Ub, n);
    const float *Ib = a.I + b * a.V + it.col;
    float umax = -FLT_MAX, umin = FLT_MAX, umin2 = FLT_MAX;
    const bool has_rv = item_has(it, M.rx[0], M.rc[0]) || item_has(it, M.rx[1], M.rc[1]) ||
                        item_has(it, M.rx[2], M.rc[2]);
#pragma unroll 1
    for (int xb = it.xs; xb <= it.xe; xb += ST_G) {
        uint32_t offs[ST_G];
        float iv[ST_G];
#pragma unroll
        for (int g = 0; g < ST_G; ++g) {   // the group's image loads together
            const int xg = xb + g;
            offs[g] = item_off(it, xg <= it.xe ? xg : it.xe, xg <= it.xe);
            iv[g] = offs[g] != VH_OOB ? Ib[(int64_t)xg * a.CZ] : 0.0f;
        }
#pragma unroll
        for (int g = 0; g < ST_G; ++g) {
            if (offs[g] == VH_OOB) continue;
            const float l = iv[g] > 0.0f ? (float)log((double)iv[g]) : 0.0f;
            st_store(rL, offs[g], l);
            st_store(rU, offs[g], l);
            umax = fmaxf(umax, l);
            if (has_rv) {
                range_special(M, xb + g, it.col, l, umin, umin2);
            } else {
                umin = fminf(umin, l);
                umin2 = fminf(umin2, l);
            }
        }
    }
    range_commit(M, umax, umin, umin2);
}

// U range of the initial field (U = L0) over one item, same bookkeeping as the eval
__device__ void range_item(const Item &it, const float *Ub, int64_t n, StudyMisc &M) {
    const __amdgpu_buffer_rsrc_t rU = st_rsrc(Ub, n);
    float umax = -FLT_MAX, umin = FLT_MAX, umin2 = FLT_MAX;
    const bool has_rv = item_has(it, M.rx[0], M.rc[0]) || item_has(it, M.rx[1], M.rc[1]) ||
                        item_has(it, M.rx[2], M.rc[2]);
#pragma unroll 1
    for (int x = it.xs; x <= it.xe; ++x) {
        const uint32_t off = item_off(it, x, true);
        if (off == VH_OOB) continue;
        const float u = st_load(rU, off);
        umax = fmaxf(umax, u);
        if (has_rv) {
            range_special(M, x, it.col, u, umin, umin2);
        } else {
            umin = fminf(umin, u);
            umin2 = fminf(umin2, u);
        }
    }
    range_commit(M, umax, umin, umin2);
}

// wave 0: the first three masked voxels in raster order (row, then column)
__device__ void find_first3(const StudyArgs &a, int64_t b, int64_t first, StudyMisc &M) {
    const int lane = threadIdx.x & 63;
    int found = 0;
    if (lane == 0)
        for (int q = 0; q < 3; ++q) M.rx[q] = M.rc[q] = -1;
    if (first < 0) return;
    const int fx = (int)(first / a.CZ), fcol = (int)(first % a.CZ);
    for (int x = fx; x < a.R && found < 3; ++x)
        for (int t0 = x == fx ? fcol / TILE_W : 0; t0 < a.ntiles && found < 3; t0 += 64) {
            const int t = t0 + lane;
            uint64_t m = t < a.ntiles ? a.rmask[((int64_t)b * a.ntiles + t) * a.R + x] : 0ull;
            if (x == fx && t < fcol / TILE_W) m = 0ull;
            if (x == fx && t == fcol / TILE_W) m &= ~((2ull << (fcol % TILE_W)) - 1ull) | (1ull << (fcol % TILE_W));
            uint64_t nz = __ballot(m != 0ull);
            while (nz && found < 3) {
                const int l = __builtin_ctzll(nz);
                nz &= nz - 1;
                const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)m, l);
                const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(m >> 32), l);
                uint64_t mm = ((uint64_t)hi << 32) | lo;
                while (mm && found < 3) {
                    const int bit = __builtin_ctzll(mm);
                    mm &= mm - 1;
                    if (lane == 0) {
                        M.rx[found] = x;
                        M.rc[found] = (t0 + l) * TILE_W + bit;
                    }
                    ++found;
                }
            }
        }
}

// expm1f for the convergence terms: the argument (B_old - B_new) is small after the first
// iteration of a level, where a degree-5 Taylor polynomial is within float rounding of expm1f
__device__ __forceinline__ float expm1_small(float x) {
    if (fabsf(x) < 0.0625f)
        return x + x * x * (0.5f + x * (0.16666667f + x * (0.041666668f + x * 0.008333334f)));
    return expm1f(x);
}

// T(i) of this lane's column: the lattice contracted over slices (P1) then cols, rounded to float
// (identical expression to n4.hip col_T + k_n4_T)
__device__ __forceinline__ float col_T_lds(const double *P1, int i, int ncy, int Z, int by,
                                           float4 wy, int z) {
    const double *r = P1 + ((int64_t)i * ncy + by) * Z + z;
    return (float)((double)wy.x * r[0] + (double)wy.y * r[Z] + (double)wy.z * r[2 * Z] +
                   (double)wy.w * r[3 * Z]);
}

// eval: B_new, U = L0 - B_new, convergence sums of exp(B_old - B_new) - 1, U range.  SAME: the
// previous field uses this level's tables (every iteration but the first of levels > 0), so both
// T windows move together at the row-span boundaries; otherwise rows are taken one at a time.
template <bool SAME>
__device__ void eval_item(const StudyArgs &a, const Item &it, int item, const TabV &Tn,
                          const TabV &To, int ncyn, int ncyo, const double *P1n, const double *P1o,
                          bool bo_mode, const float *Lb, float *Ub, int64_t n, int64_t first,
                          double *ipart, StudyMisc &M) {
    const __amdgpu_buffer_rsrc_t rL = st_rsrc(Lb, n), rU = st_rsrc(Ub, n);
    const int Z = a.Z;
    const float4 wyn = it.colok ? Tn.wy[it.y] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 wyo = it.colok ? To.wy[it.y] : make_float4(0.f, 0.f, 0.f, 0.f);
    const int byn = Tn.by[it.y], byo = To.by[it.y];
    int wbn = Tn.bx[it.xs], wbo = To.bx[it.xs];
    float tn0 = col_T_lds(P1n, wbn, ncyn, Z, byn, wyn, it.z);
    float tn1 = col_T_lds(P1n, wbn + 1, ncyn, Z, byn, wyn, it.z);
    float tn2 = col_T_lds(P1n, wbn + 2, ncyn, Z, byn, wyn, it.z);
    float tn3 = col_T_lds(P1n, wbn + 3, ncyn, Z, byn, wyn, it.z);
    float to0 = 0.f, to1 = 0.f, to2 = 0.f, to3 = 0.f;
    if (bo_mode) {
        to0 = col_T_lds(P1o, wbo, ncyo, Z, byo, wyo, it.z);
        to1 = col_T_lds(P1o, wbo + 1, ncyo, Z, byo, wyo, it.z);
        to2 = col_T_lds(P1o, wbo + 2, ncyo, Z, byo, wyo, it.z);
        to3 = col_T_lds(P1o, wbo + 3, ncyo, Z, byo, wyo, it.z);
    }
    double sd = 0.0, sd2 = 0.0;
    float umax = -FLT_MAX, umin = FLT_MAX, umin2 = FLT_MAX;
    // the study's first three masked voxels (ITK's bin-range rule) only matter in their items
    const bool has_rv = item_has(it, M.rx[0], M.rc[0]) || item_has(it, M.rx[1], M.rc[1]) ||
                        item_has(it, M.rx[2], M.rc[2]);
    auto voxel = [&](uint32_t off, float la, int x) {
        const float4 w = Tn.wx[x];
        const float bn = ((w.x * tn0 + w.y * tn1) + w.z * tn2) + w.w * tn3;
        float bo = 0.0f;
        if (bo_mode) {
            const float4 wo = SAME ? w : To.wx[x];
            bo = ((wo.x * to0 + wo.y * to1) + wo.z * to2) + wo.w * to3;
        }
        const float u = la - bn;
        st_store(rU, off, u);
        const double d = (double)expm1_small(bo - bn);   // p - 1, p = exp(B_old - B_new)
        sd += d;
        sd2 = fma(d, d, sd2);
        umax = fmaxf(umax, u);
        if (has_rv) {
            range_special(M, x, it.col, u, umin, umin2);
        } else {
            umin = fminf(umin, u);
            umin2 = fminf(umin2, u);
        }
    };
    if (SAME) {
        int x = it.xs;
#pragma unroll 1
        for (;;) {
            const int rb = min(it.xe, Tn.xst[wbn + 1] - 1);
#pragma unroll 1
            for (int xb = x; xb <= rb; xb += ST_G) {
                uint32_t offs[ST_G];
                float la[ST_G];
#pragma unroll
                for (int g = 0; g < ST_G; ++g) {
                    const int xg = xb + g;
                    offs[g] = item_off(it, xg <= rb ? xg : rb, xg <= rb);
                    la[g] = st_load(rL, offs[g]);
                }
#pragma unroll
                for (int g = 0; g < ST_G; ++g)
                    if (offs[g] != VH_OOB) voxel(offs[g], la[g], xb + g);
            }
            x = rb + 1 > x ? rb + 1 : x;
            if (x > it.xe) break;
            ++wbn;   // next span: both windows move one control row
            tn0 = tn1; tn1 = tn2; tn2 = tn3;
            tn3 = col_T_lds(P1n, wbn + 3, ncyn, Z, byn, wyn, it.z);
            if (bo_mode) {
                ++wbo;
                to0 = to1; to1 = to2; to2 = to3;
                to3 = col_T_lds(P1o, wbo + 3, ncyo, Z, byo, wyo, it.z);
            }
        }
    } else {
#pragma unroll 1
        for (int x = it.xs; x <= it.xe; ++x) {
            const int bxn = Tn.bx[x];
            while (bxn > wbn) {
                ++wbn;
                tn0 = tn1; tn1 = tn2; tn2 = tn3;
                tn3 = col_T_lds(P1n, wbn + 3, ncyn, Z, byn, wyn, it.z);
            }
            const int bxo = To.bx[x];
            while (bxo > wbo) {
                ++wbo;
                to0 = to1; to1 = to2; to2 = to3;
                to3 = col_T_lds(P1o, wbo + 3, ncyo, Z, byo, wyo, it.z);
            }
            const uint32_t off = item_off(it, x, true);
            if (off != VH_OOB) voxel(off, st_load(rL, off), x);
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        sd += __shfl_down(sd, off, 64);
        sd2 += __shfl_down(sd2, off, 64);
    }
    range_commit(M, umax, umin, umin2);
    if ((threadIdx.x & 63) == 0) {
        ipart[2 * item] = sd;
        ipart[2 * item + 1] = sd2;
    }
}

// ---------------------------------------------------------------------------------------------
// FFT (512-point radix-2 DIT, same butterflies and twiddle indexing as oracle/n4_oracle.c) by ONE
// wave in place in LDS.  The points sit at padded slots fpad(i) (one spare slot per 8), so the
// strided passes below hit distinct LDS banks.  Only wave-local ordering is needed (a wave's LDS
// operations complete in issue order; the fences keep the compiler from moving them).
// ---------------------------------------------------------------------------------------------
#define ST_FFT_N (VH_FFT_P + VH_FFT_P / 8)   // padded slots of one transform
__device__ __forceinline__ int fpad(int i) { return i + (i >> 3); }

struct FftId {
    __device__ double2 operator()(int, double2 v) const { return v; }
};

__device__ __forceinline__ void wave_lds_order() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The 9 stages run as 3 register passes of 3: in pass p a lane owns the 8 points
// base + m * 8^p (m < 8), which the stages of half-length 8^p, 2 * 8^p, 4 * 8^p pair only among
// themselves.  Pass 0 gathers in bit-reversed order (all loads of the wave issue before its
// stores) through pro(i, v); pass 2 stores epi(i, v) -- the elementwise steps around a transform
// ride on its first and last pass.
template <class Pro, class Epi>
__device__ __forceinline__ void wave_fft_lds(double2 *x, const double2 *tw, bool inverse, const Pro &pro,
                             const Epi &epi) {
    const int lane = threadIdx.x & 63;
#pragma unroll 1
    for (int p = 0; p < 3; ++p) {
        const int stride = 1 << (3 * p);
        const int base = (lane / stride) * 8 * stride + lane % stride;
        double2 v[8];
        if (p == 0) {
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const int src = (int)(__brev((unsigned)(base + m)) >> (32 - 9));
                v[m] = pro(src, x[fpad(src)]);
            }
        } else {
#pragma unroll
            for (int m = 0; m < 8; ++m) v[m] = x[fpad(base + m * stride)];
        }
#pragma unroll
        for (int s = 0; s < 3; ++s) {
            const int half = stride << s, step = VH_FFT_P / (2 * half);
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                if (m & (1 << s)) continue;
                const int j = stride * (m & ((1 << s) - 1)) + lane % stride;   // (base + m stride) % half
                const double2 w = tw[j * step];
                const double wy = inverse ? -w.y : w.y;
                const double2 a = v[m], bb = v[m + (1 << s)];
                const double tr = w.x * bb.x - wy * bb.y, ti = w.x * bb.y + wy * bb.x;
                v[m] = make_double2(a.x + tr, a.y + ti);
                v[m + (1 << s)] = make_double2(a.x - tr, a.y - ti);
            }
        }
        if (p == 2) {
#pragma unroll
            for (int m = 0; m < 8; ++m) v[m] = epi(base + m * stride, v[m]);
        }
#pragma unroll
        for (int m = 0; m < 8; ++m) x[fpad(base + m * stride)] = v[m];
        wave_lds_order();
    }
}

// ---------------------------------------------------------------------------------------------
// exact ITK bin minimum (rare): min over the voxels that are not running maxima in raster order
// ---------------------------------------------------------------------------------------------
__device__ void exact_row(const StudyArgs &a, int64_t b, const float *Ub, int x, float &run,
                          float &mn, bool track_min) {
    for (int tile = 0; tile < a.ntiles; ++tile) {
        const int64_t e = ((int64_t)b * a.ntiles + tile) * a.R + x;
        uint64_t m = a.rmask[e];
        int off = a.rs[e];
        while (m) {
            const float u = Ub[off++];
            m &= m - 1;
            if (u > run) run = u;
            else if (track_min && u < mn) mn = u;
        }
    }
}

__device__ float exact_min_study(const StudyArgs &a, int64_t b, const float *Ub, float *s_cmax,
                                 float *s_min) {
    const int t = threadIdx.x;
    const int per = (a.R + ST_TPB - 1) / ST_TPB;
    const int s0 = min(t * per, a.R), e0 = min(s0 + per, a.R);
    float cmax = -FLT_MAX, dummy = FLT_MAX;
    for (int x = s0; x < e0; ++x) exact_row(a, b, Ub, x, cmax, dummy, false);
    s_cmax[t] = cmax;
    __syncthreads();
    if (t == 0) {
        float run = -FLT_MAX;
        for (int i = 0; i < ST_TPB; ++i) { const float v = s_cmax[i]; s_cmax[i] = run; run = v > run ? v : run; }
    }
    __syncthreads();
    float run = s_cmax[t], mn = FLT_MAX;
    for (int x = s0; x < e0; ++x) exact_row(a, b, Ub, x, run, mn, true);
    s_min[t] = mn;
    __syncthreads();
    float m = FLT_MAX;
    if (t == 0)
        for (int i = 0; i < ST_TPB; ++i) m = s_min[i] < m ? s_min[i] : m;
    return m;
}

__device__ __forceinline__ double conv_of(double sd, double sd2, double N) {
    const double mu = 1.0 + sd / N;
    double var = (sd2 - sd * sd / N) / (N - 1.0);
    if (var < 0.0) var = 0.0;
    return sqrt(var) / mu;
}

__device__ void refine_axis_st(const float *in, float *out, int d0, int d1, int d2, int axis) {
    int od[3] = {d0, d1, d2};
    const int dims[3] = {d0, d1, d2};
    od[axis] = 2 * dims[axis] - 3;
    const int total = od[0] * od[1] * od[2];
    for (int e = threadIdx.x; e < total; e += ST_TPB) {
        const int a0 = e / (od[1] * od[2]), a1 = (e / od[2]) % od[1], a2 = e % od[2];
        int s0[3] = {a0, a1, a2}, s1[3] = {a0, a1, a2}, s2[3] = {a0, a1, a2};
        const int m = s0[axis], j = m >> 1;
        s0[axis] = j; s1[axis] = j + 1; s2[axis] = j + 2;
        auto IDX = [&](const int *s) { return ((size_t)s[0] * dims[1] + s[1]) * dims[2] + s[2]; };
        double v;
        if ((m & 1) == 0) v = ((double)in[IDX(s0)] + (double)in[IDX(s1)]) * 0.5;
        else v = ((double)in[IDX(s0)] + 6.0 * (double)in[IDX(s1)] + (double)in[IDX(s2)]) * 0.125;
        out[e] = (float)v;
    }
}

// ---------------------------------------------------------------------------------------------
// the kernel: one workgroup per study
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(ST_TPB) k_n4_study(StudyArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int64_t b = a.vol0 + blockIdx.x;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    StudyMisc &M = *reinterpret_cast<StudyMisc *>(smem + a.o_misc);
    float *sE = reinterpret_cast<float *>(smem + a.o_E);
    float *lat = reinterpret_cast<float *>(smem + a.o_lat);
    double *den = reinterpret_cast<double *>(smem + a.o_den);
    double *const P1b0 = reinterpret_cast<double *>(smem + a.o_P10);
    double *const P1b1 = reinterpret_cast<double *>(smem + a.o_P11);
    double *ipart = reinterpret_cast<double *>(smem + a.o_ipart);
    int32_t *ordr = reinterpret_cast<int32_t *>(smem + a.o_order);
    char *scr = smem + a.o_scr;

    const int64_t n = a.sc[b].n_mask1;
    N4State *stb = a.st + b;
    const DevLevel &lvl = a.lvs->lv[a.nlev - 1];
    const int p1last = lvl.ax[0].ncp * lvl.ax[1].ncp * a.Z;
    if (n < 2) {   // no fit: zero field (output = input), no iterations
        for (int e = t; e < p1last; e += ST_TPB) a.P1out[b * a.q2cap + e] = 0.0;
        if (t < VH_MAX_LEVELS) {
            stb->iters_level[t] = 0;
            stb->conv_level[t] = 0.0f;
        }
        return;
    }
    float *Lb = a.L0 + b * a.VS;
    float *Ub = a.U + b * a.VS;
    const int64_t fm = a.sc[b].first_masked;
    // fit / eval scratch: lattice numerator (fixed point), then per-wave Q / S rows
    unsigned long long *numfix = reinterpret_cast<unsigned long long *>(scr);
    FitRing ring;
    ring.q = reinterpret_cast<double *>(scr + a.o_wave) + (size_t)wv * a.nb_ring * a.s_cap;
    ring.rowcap = a.s_cap;
    ring.nr = 0;
    double *const Wk3 = reinterpret_cast<double *>(smem + a.o_wk);
    // emap scratch: V (= U = NUM), F, DEN, twiddles, then the histogram copies
    double2 *V = reinterpret_cast<double2 *>(scr), *F = V + ST_FFT_N, *DEN = F + ST_FFT_N;
    double2 *TW = DEN + ST_FFT_N;
    unsigned long long *Hc = reinterpret_cast<unsigned long long *>(TW + VH_FFT_P / 2);
    const int bins = a.bins;

    if (t == 0) {
        M.umax_key = 0u;
        M.umin_key = M.umin2_key = 0xffffffffu;
        M.u_first = M.u_second = M.u_third = 0.0f;
        M.item_ctr = 0;
    }
    if (wv == 0) find_first3(a, b, fm, M);
    {   // item schedule: items by row count, largest first (ties by index), so the dynamic item
        // queue of every pass ends on small items; the item order of every reduction is unchanged
        int32_t *isz = reinterpret_cast<int32_t *>(scr);
        for (int item = wv; item < a.nitems; item += ST_WAVES) {
            Item it;
            const bool any = item_begin(it, a, b, item);
            if (lane == 0) isz[item] = any ? it.xe - it.xs + 1 : 0;
        }
        __syncthreads();
        for (int i = t; i < a.nitems; i += ST_TPB) {
            const int si = isz[i];
            int rank = 0;
            for (int j = 0; j < a.nitems; ++j) {
                const int sj = isz[j];
                rank += (sj > si || (sj == si && j < i)) ? 1 : 0;
            }
            ordr[rank] = i;
        }
    }
    __syncthreads();
    for (;;) {   // range of the initial field U = L0
        int item = 0;
        if (lane == 0) item = atomicAdd(&M.item_ctr, 1);
        item = __shfl(item, 0, 64);
        if (item >= a.nitems) break;
        item = ordr[item];   // largest items first
        Item it;
        if (!item_begin(it, a, b, item)) continue;
        init_item(a, b, it, Lb, Ub, n, M);
    }
    {
        const DevLevel &l0 = a.lvs->lv[0];
        const int nl0 = l0.ax[0].ncp * l0.ax[1].ncp * l0.ax[2].ncp;
        for (int e = t; e < nl0; e += ST_TPB) lat[e] = 0.0f;
    }
    int cur = 0;   // P1b[cur] holds the last evaluated field
#ifdef ST_PROF
    unsigned long long st_prof[13] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, st_t0 = clock64();
    const unsigned long long st_w0 = wall_clock64(), st_c0 = clock64();
#endif
    for (int L = 0; L < a.nlev; ++L) {
        const DevLevel &lv = a.lvs->lv[L];
        const TabV T = tab_view(smem + ((L & 1) ? a.o_tab1 : a.o_tab0), a.R, a.C, a.Z, a.kcap);
        const int ncx = lv.ax[0].ncp, ncy = lv.ax[1].ncp, ncz = lv.ax[2].ncp;
        const int nlat = ncx * ncy * ncz;
        load_tables(T, lv, a.R, a.C, a.Z);
        if (t == 0) {
            M.nc[L & 1][0] = ncx;
            M.nc[L & 1][1] = ncy;
            M.nc[L & 1][2] = ncz;
        }
        double *const Wk2 = Wk3 + (size_t)ncz * a.Z;
        for (int e = t; e < ncz * a.Z; e += ST_TPB) {   // dense slice weights of this level
            const int k = e / a.Z, z = e % a.Z;
            const float4 w = *reinterpret_cast<const float4 *>(lv.ax[2].w + 4 * z);
            const int d = k - lv.ax[2].base[z];
            const bool in = d >= 0 && d <= 3;
            Wk3[e] = in ? wpow<3>(wsel(w, d)) : 0.0;
            Wk2[e] = in ? wpow<2>(wsel(w, d)) : 0.0;
        }
        double2 *const Wx3 = reinterpret_cast<double2 *>(smem + a.o_wx), *const Wx2 = Wx3 + 2 * a.R;
        for (int x = t; x < a.R; x += ST_TPB) {   // row weights^P of this level (wave-uniform reads)
            const float4 w = *reinterpret_cast<const float4 *>(lv.ax[0].w + 4 * x);
            Wx3[2 * x] = make_double2(wpow<3>(w.x), wpow<3>(w.y));
            Wx3[2 * x + 1] = make_double2(wpow<3>(w.z), wpow<3>(w.w));
            Wx2[2 * x] = make_double2(wpow<2>(w.x), wpow<2>(w.y));
            Wx2[2 * x + 1] = make_double2(wpow<2>(w.z), wpow<2>(w.w));
        }
        // ---- denominator of this level: sum of w^2 over the mask ----
        for (int e = t; e < 2 * nlat; e += ST_TPB) numfix[e] = 0ull;
        if (t == 0) M.item_ctr = 0;
        __syncthreads();
        for (;;) {
            int item = 0;
            if (lane == 0) item = atomicAdd(&M.item_ctr, 1);
            item = __shfl(item, 0, 64);
            if (item >= a.nitems) break;
        item = ordr[item];   // largest items first
            Item it;
            if (!item_begin(it, a, b, item)) continue;
            fit_item<1>(a, it, T, Wk2, Wx2, ncy, ncz, Ub, n, sE, 0.0f, 1.0, ring, numfix);
        }
        __syncthreads();
        ST_MARK(0);
        for (int e = t; e < nlat; e += ST_TPB) den[e] = fix128_get(numfix + 2 * e, numfix + 2 * e + 1);
        // ---- iterations ----
        int itn = 0;
        for (;;) {
            __syncthreads();
            ST_MARK(7);
            if (t == 0) {
                M.stop = 0;
                M.exact = 0;
                if (itn > 0) {
                    const double conv = conv_of(M.sd, M.sd2, (double)n);
                    M.conv = conv;
                    if (!(conv > (double)a.thresh) || itn >= a.lvs->max_iters[L]) M.stop = 1;
                }
                if (!M.stop) {
                    const float bmax = key2f(M.umax_key);
                    const float umin = M.umin_key == 0xffffffffu ? FLT_MAX : key2f(M.umin_key);
                    const float umin2 = M.umin2_key == 0xffffffffu ? FLT_MAX : key2f(M.umin2_key);
                    M.bmax = bmax;
                    if (umin <= M.u_first) {                       // u1 is not the strict minimum
                        M.bin_min = umin;
                        M.slope = (bmax - umin) / (float)(bins - 1);
                    } else if (M.rx[2] >= 0 && !(M.u_third > M.u_second)) {   // run u1 < u2 >= u3
                        M.bin_min = umin2;
                        M.slope = (bmax - umin2) / (float)(bins - 1);
                    } else {
                        M.exact = 1;
                    }
                    M.umax_key = 0u;
                    M.umin_key = M.umin2_key = 0xffffffffu;
                }
            }
            __syncthreads();
            ST_MARK(1);
            if (M.stop) break;
            if (M.exact) {
                float *s_cmax = reinterpret_cast<float *>(scr);
                const float m = exact_min_study(a, b, Ub, s_cmax, s_cmax + ST_TPB);
                if (t == 0) {
                    M.bin_min = m;
                    M.slope = (M.bmax - m) / (float)(bins - 1);
                }
                __syncthreads();
            }
            ST_MARK(1);
            ++itn;
            const float bmin = M.bin_min, slope = M.slope;
            const double rinv = 1.0 / (double)slope;   // div_r form of the bin division
            // ---- hist ----
            for (int i = t; i < ST_HC * VH_MAX_BINS; i += ST_TPB) Hc[i] = 0ull;
            __syncthreads();
            {
                unsigned long long *H = Hc + (lane & (ST_HC - 1)) * VH_MAX_BINS;
                for (int64_t j0 = (int64_t)t * 16; j0 < n; j0 += (int64_t)ST_TPB * 16) {
                    float u[16];
                    if (j0 + 16 <= n) {
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const float4 v = reinterpret_cast<const float4 *>(Ub + j0)[q];
                            u[4 * q] = v.x; u[4 * q + 1] = v.y; u[4 * q + 2] = v.z; u[4 * q + 3] = v.w;
                        }
                    } else {
#pragma unroll
                        for (int k = 0; k < 16; ++k) u[k] = j0 + k < n ? Ub[j0 + k] : __int_as_float(0x7fc00000);
                    }
                    // branch-free: every value does its two adds (zero weights for values that
                    // add nothing) -- no divergent run bookkeeping
#pragma unroll
                    for (int k = 0; k < 16; ++k) {
                        int idx;
                        unsigned long long a0, a1;
                        parzen_bin_bf(u[k], bmin, rinv, bins, idx, a0, a1);
                        atomicAdd(&H[idx], a0);
                        atomicAdd(&H[min(idx + 1, bins - 1)], a1);
                    }
                }
            }
            __syncthreads();
            ST_MARK(2);
            // ---- emap (same arithmetic as n4.hip k_n4_emap) ----
            {
                const int P = VH_FFT_P, off = (P - bins) / 2;
                const float sFWHM = a.fwhm / slope;
                const float ef = (float)(4.0 * LN2 / (double)(sFWHM * sFWHM));
                const float sf = (float)(2.0 * sqrt(LN2 / PI_D) / (double)sFWHM);
                static_assert(VH_FFT_P / 2 <= ST_TPB, "one twiddle per thread");
                const double2 twv = t < P / 2 ? a.tw[t] : make_double2(0.0, 0.0);   // in flight
                for (int i = t; i < P; i += ST_TPB) {   // histogram series and Gaussian kernel
                    const int h = i - off;
                    unsigned long long s = 0ull;
                    if (h >= 0 && h < bins)
                        for (int q = 0; q < ST_HC; ++q) s += Hc[q * VH_MAX_BINS + h];
                    V[fpad(i)] = make_double2((double)s * (1.0 / 4294967296.0), 0.0);
                    double fx;
                    if (i == 0) {
                        fx = (double)sf;
                    } else if (i == P / 2) {
                        fx = (double)sf * exp(-0.25 * (double)((float)P * (float)P) * (double)ef);
                    } else {
                        const float nf = (float)(i < P / 2 ? i : P - i);
                        fx = (double)(sf * expf_cr(-(nf * nf) * ef));
                    }
                    F[fpad(i)] = make_double2(fx, 0.0);
                }
                if (t < P / 2) TW[t] = twv;
                __syncthreads();
                ST_MARK(9);
                if (wv < 2) wave_fft_lds(wv ? F : V, TW, false, FftId(), FftId());
                __syncthreads();
                ST_MARK(10);
                if (wv == 0) {   // Wiener filter (first pass), inverse, clamp and the moment series (last pass)
                    const double noise = (double)a.noise;
                    wave_fft_lds(V, TW, true,
                        [=](int i, double2 v) {
                            const double2 f = F[fpad(i)];
                            const double fa = f.x, fb = f.y;
                            const double g = fa / ((fa * fa - (-fb) * fb) + noise);
                            return make_double2(v.x * g, v.y * g);
                        },
                        [=](int i, double2 v) {
                            const double ur = v.x > 0.0 ? v.x : 0.0;
                            const float c = bmin + ((float)i - (float)off) * slope;
                            DEN[fpad(i)] = make_double2(ur, 0.0);
                            return make_double2((double)c * ur, 0.0);
                        });
                }
                __syncthreads();
                ST_MARK(11);
                if (wv < 2) {   // each series: forward, times the kernel's transform (last pass), inverse
                    double2 *x = wv ? DEN : V;
                    wave_fft_lds(x, TW, false, FftId(), [=](int i, double2 v) {
                        const double2 f = F[fpad(i)];
                        const double fa = f.x, fb = f.y;
                        return make_double2(v.x * fa - v.y * fb, v.x * fb + v.y * fa);
                    });
                    wave_fft_lds(x, TW, true, FftId(), FftId());
                }
                __syncthreads();
                ST_MARK(12);
                for (int i = t; i < bins; i += ST_TPB) {
                    const double d = DEN[fpad(i + off)].x;
                    sE[i] = d != 0.0 ? (float)(V[fpad(i + off)].x / d) : 0.0f;
                }
                __syncthreads();
            }
            ST_MARK(3);
            // ---- fit ----
            for (int e = t; e < 2 * nlat; e += ST_TPB) numfix[e] = 0ull;
            if (t == 0) M.item_ctr = 0;
            __syncthreads();
            for (;;) {
                int item = 0;
                if (lane == 0) item = atomicAdd(&M.item_ctr, 1);
                item = __shfl(item, 0, 64);
                if (item >= a.nitems) break;
        item = ordr[item];   // largest items first
                Item it;
                if (!item_begin(it, a, b, item)) continue;
                fit_item<0>(a, it, T, Wk3, Wx3, ncy, ncz, Ub, n, sE, bmin, rinv, ring, numfix);
            }
            __syncthreads();
            ST_MARK(4);
            // ---- lattice update (k_n4_tilesum<0>) and P1 (k_n4_P1) ----
            for (int e = t; e < nlat; e += ST_TPB) {
                const double d = den[e];
                const double num = fix128_get(numfix + 2 * e, numfix + 2 * e + 1);
                const float phi = d != 0.0 ? (float)(num / d) : 0.0f;
                lat[e] += phi;
            }
            __syncthreads();
            double *P1n = cur ? P1b0 : P1b1;
            double *P1o = cur ? P1b1 : P1b0;
            for (int e = t; e < ncx * ncy * a.Z; e += ST_TPB) {
                const int ij = e / a.Z, z = e % a.Z;
                const float4 w = T.wz[z];
                const float *l = lat + ij * ncz + T.bz[z];
                P1n[e] = (double)w.x * (double)l[0] + (double)w.y * (double)l[1] +
                         (double)w.z * (double)l[2] + (double)w.w * (double)l[3];
            }
            if (t == 0) M.item_ctr = 0;
            __syncthreads();
            ST_MARK(5);
            // ---- eval ----
            {
                const bool first_of_level = itn == 1;
                const bool bo_mode = !(L == 0 && first_of_level);
                const int so = (first_of_level && L > 0) ? ((L - 1) & 1) : (L & 1);
                const TabV To = tab_view(smem + (so ? a.o_tab1 : a.o_tab0), a.R, a.C, a.Z, a.kcap);
                const int ncyo = M.nc[so][1];
                for (;;) {
                    int item = 0;
                    if (lane == 0) item = atomicAdd(&M.item_ctr, 1);
                    item = __shfl(item, 0, 64);
                    if (item >= a.nitems) break;
        item = ordr[item];   // largest items first
                    Item it;
                    if (!item_begin(it, a, b, item)) {
                        if (lane == 0) { ipart[2 * item] = 0.0; ipart[2 * item + 1] = 0.0; }
                        continue;
                    }
                    if (so == (L & 1))
                        eval_item<true>(a, it, item, T, To, ncy, ncyo, P1n, P1o, bo_mode, Lb, Ub,
                                        n, fm, ipart, M);
                    else
                        eval_item<false>(a, it, item, T, To, ncy, ncyo, P1n, P1o, bo_mode, Lb, Ub,
                                         n, fm, ipart, M);
                }
            }
            __syncthreads();
            ST_MARK(6);
            if (wv == 0) {   // item partials in item order: deterministic
                double sd = 0.0, sd2 = 0.0;
                for (int i = lane; i < a.nitems; i += 64) {
                    sd += ipart[2 * i];
                    sd2 += ipart[2 * i + 1];
                }
                for (int off = 32; off > 0; off >>= 1) {
                    sd += __shfl_down(sd, off, 64);
                    sd2 += __shfl_down(sd2, off, 64);
                }
                if (lane == 0) {
                    M.sd = sd;
                    M.sd2 = sd2;
                }
            }
            cur ^= 1;
        }
        if (t == 0) {
            stb->iters_level[L] = itn;
            stb->conv_level[L] = (float)M.conv;
        }
        if (L < a.nlev - 1) {   // exact subdivision of the lattice for the next level
            const int nl_max = lvl.ax[0].ncp * lvl.ax[1].ncp * lvl.ax[2].ncp;
            float *T1 = reinterpret_cast<float *>(scr), *T2 = T1 + nl_max;
            refine_axis_st(lat, T1, ncx, ncy, ncz, 0);
            __syncthreads();
            refine_axis_st(T1, T2, 2 * ncx - 3, ncy, ncz, 1);
            __syncthreads();
            refine_axis_st(T2, lat, 2 * ncx - 3, 2 * ncy - 3, ncz, 2);
            __syncthreads();
        }
        ST_MARK(8);
    }
#ifdef ST_PROF
    if (t == 0) stb->conv_level[3] = (float)(wall_clock64() - st_w0) * 0.01f;   // us
    if (t == 0 && blockIdx.x == 0)
        printf("ST_BLK %d wall %llu %llu cycles %llu xcc %u\n", (int)blockIdx.x, st_w0, wall_clock64(),
               clock64() - st_c0, __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11)));
    if (t == 0 && blockIdx.x == 0)
        printf("ST_PROF den %llu ctrl %llu hist %llu emap %llu fit %llu latP1 %llu eval %llu loop %llu "
               "refine %llu | emap: init %llu fwd %llu wiener %llu conv %llu sE %llu\n", st_prof[0],
               st_prof[1], st_prof[2], st_prof[3], st_prof[4], st_prof[5], st_prof[6], st_prof[7],
               st_prof[8], st_prof[9], st_prof[10], st_prof[11], st_prof[12], st_prof[3]);
#endif
    // final field's P1 for k_n4_final
    const double *P1f = cur ? P1b1 : P1b0;
    for (int e = t; e < p1last; e += ST_TPB) a.P1out[b * a.q2cap + e] = P1f[e];
    if (t == 0) {
        stb->conv = M.conv;
        stb->active = 0;
    }
}

// ---------------------------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------------------------
struct StudyLayout {
    size_t bytes;
    StudyArgs a;
};

static bool study_layout(const vh_batch *b, const vh_n4_params &prm, StudyLayout &out) {
    StudyArgs &a = out.a;
    std::memset(&a, 0, sizeof(a));
    const int R = (int)b->R, C = (int)b->C, Z = (int)b->Z;
    int kcap = 0, nlat_max = 0, p1_max = 0, s_cap = 0;
    for (int L = 0; L < prm.n_levels; ++L) {
        const int ncx = vh_level_ncp(prm, L, 0), ncy = vh_level_ncp(prm, L, 1), ncz = vh_level_ncp(prm, L, 2);
        kcap = std::max({kcap, ncz, ncx});
        nlat_max = std::max(nlat_max, ncx * ncy * ncz);
        p1_max = std::max(p1_max, ncx * ncy * Z);
        AxisTab tz;
        const float eps = vh_bspline_eps(std::max({ncx, ncy, ncz}) - 3);
        vh_axis_tables(Z, ncz, eps, tz);
        for (int64_t c0 = 0; c0 < b->CZ; c0 += TILE_W) {
            const int64_t c1 = std::min(c0 + TILE_W, b->CZ) - 1;
            const int y0 = (int)(c0 / Z), y1 = (int)(c1 / Z);
            const int z0 = (int)(c0 % Z), z1 = (int)(c1 % Z);
            const int klo = tz.base[y0 == y1 ? z0 : 0];
            const int KT = tz.base[y0 == y1 ? z1 : Z - 1] + 4 - klo;
            s_cap = std::max(s_cap, (y1 - y0 + 1) * KT);
        }
    }
    // refinement temporaries: two lattices of the next level (<= 8x the current)
    const size_t refine = 2 * sizeof(float) * (size_t)nlat_max + 64;
    const size_t emap = sizeof(double2) * (3 * ST_FFT_N + VH_FFT_P / 2) +
                        sizeof(unsigned long long) * ST_HC * VH_MAX_BINS;
    const bool geom_ok = s_cap <= 64 * ST_SO;   // one ring row's stage-1 outputs fit the lanes
    s_cap = std::max(s_cap, 64);
    // ring rows per wave: up to ST_NB within ~40 KB for all waves
    const int nb_ring = std::max(1, std::min(ST_NB, (int)(40960 / (ST_WAVES * 8 * (size_t)s_cap))));
    const size_t fit_num = 2 * sizeof(unsigned long long) * (size_t)nlat_max;
    const size_t fit = ((fit_num + 15) & ~(size_t)15) + sizeof(double) * ST_WAVES * nb_ring * (size_t)s_cap;
    const size_t exact = sizeof(float) * 2 * ST_TPB;
    const size_t scr = std::max({refine, emap, fit, exact});
    auto A = [](size_t v) { return (v + 15) & ~(size_t)15; };
    size_t o = 0;
    a.o_E = (int32_t)o; o += A(sizeof(float) * VH_MAX_BINS);
    const size_t tb = study_tab_bytes(R, C, Z, kcap);
    a.o_tab0 = (int32_t)o; o += tb;
    a.o_tab1 = (int32_t)o; o += tb;
    a.o_lat = (int32_t)o; o += A(sizeof(float) * nlat_max);
    a.o_den = (int32_t)o; o += A(sizeof(double) * nlat_max);
    a.o_P10 = (int32_t)o; o += A(sizeof(double) * p1_max);
    a.o_P11 = (int32_t)o; o += A(sizeof(double) * p1_max);
    const int64_t nslots = (b->R + 63) / 64;
    const int64_t nitems = b->n4_tiles * nslots;
    a.o_ipart = (int32_t)o; o += A(sizeof(double) * 2 * (size_t)nitems);
    a.o_order = (int32_t)o; o += A(sizeof(int32_t) * (size_t)nitems);
    a.o_misc = (int32_t)o; o += A(sizeof(StudyMisc));
    a.o_wk = (int32_t)o; o += A(2 * sizeof(double) * (size_t)kcap * Z);
    a.o_wx = (int32_t)o; o += A(2 * 4 * sizeof(double) * (size_t)R);
    a.o_scr = (int32_t)o; o += A(scr);
    a.o_wave = (int32_t)((fit_num + 15) & ~(size_t)15);   // ring offset inside the scratch
    a.s_cap = s_cap;
    a.nb_ring = nb_ring;
    a.kcap = kcap;
    a.nslots = (int32_t)nslots;
    a.nitems = (int32_t)nitems;
    out.bytes = o;
    return geom_ok && o <= ST_MAX_LDS && prm.n_levels <= VH_MAX_LEVELS && b->V < ((int64_t)1 << 29);
}

bool vh_n4_study_eligible(const vh_batch *b, const vh_n4_params &prm, size_t *lds_bytes) {
    if (b->n4_tiles == 0) return false;
    StudyLayout L;
    const bool ok = study_layout(b, prm, L);
    if (lds_bytes) *lds_bytes = L.bytes;
    return ok;
}

void vh_launch_n4_study(vh_batch *b, const vh_n4_params &prm) {
    StudyLayout Ly;
    if (!study_layout(b, prm, Ly)) throw VhError{VH_ERR_ARG, "N4 study kernel: LDS budget exceeded"};
    StudyArgs a = Ly.a;
    a.I = b->d_hp;
    a.V = b->V;
    a.L0 = b->d_L0;
    a.U = b->d_U;
    a.rs = b->d_rowstart;
    a.rmask = b->d_rowmask;
    a.sc = b->d_sc;
    a.st = b->d_st;
    a.P1out = b->d_P1;
    a.q2cap = b->q2_cap;
    a.tw = b->d_twiddle;
    a.VS = b->VS;
    a.R = (int32_t)b->R;
    a.C = (int32_t)b->C;
    a.Z = (int32_t)b->Z;
    a.CZ = (int32_t)b->CZ;
    a.ntiles = (int32_t)b->n4_tiles;
    a.nlev = prm.n_levels;
    a.bins = prm.n_bins;
    a.thresh = prm.conv_threshold;
    a.fwhm = prm.fwhm;
    a.noise = prm.wiener_noise;
    StudyLevels h{};
    for (int L = 0; L < prm.n_levels; ++L) {
        h.max_iters[L] = prm.max_iters[L];
        h.lv[L] = vh_dev_level(b, prm, L);
    }
    if (!b->d_study_lv) HIP_TRY(hipMalloc(&b->d_study_lv, sizeof(StudyLevels)));
    HIP_TRY(hipMemcpyAsync(b->d_study_lv, &h, sizeof(StudyLevels), hipMemcpyHostToDevice,
                           b->ctx->stream));
    a.lvs = (const StudyLevels *)b->d_study_lv;
    a.vol0 = 0;
    static bool attr_set = false;
    if (!attr_set) {
        HIP_TRY(hipFuncSetAttribute((const void *)k_n4_study,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, ST_MAX_LDS));
        attr_set = true;
    }
    ScopedKTimer tm(b, "n4_study", 0.0);
    k_n4_study<<<(unsigned)b->nb, ST_TPB, Ly.bytes, b->ctx->stream>>>(a);
    VH_CHECK_LAUNCH();
}
