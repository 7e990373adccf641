// Declarations and device code shared by the two N4 drivers: n4.hip (per-iteration sweeps over
// the whole batch) and n4_study.hip (one workgroup per study, the whole level/iteration loop in
// one launch).  Both drivers evaluate the N4 build spec (oracle/n4_oracle.c header, S1-S9)
// operation for operation, so U = L0 - B is bit-identical between them and the CPU oracle after
// every iteration.
#pragma once
#include "vh_internal.h"
#include "expf_small.h"
#include <cfloat>
#include <hip/hip_cooperative_groups.h>

struct DevAxis {
    const int32_t *base;
    const float *w;
    const double *sw2;
    const double *isw2;   // 1 / sum w^2
    const double *w2;     // [n][4] w^2 (double)
    const double *w3;     // [n][4] w^3 (double)
    const double *w3i;    // [n][4] w^3 * isw2 (row axis: the fit's numerator row weights, S5)
    const int2 *krange;   // [ncp] first / last index whose support contains control point k
    int32_t n, ncp;
};
struct DevLevel {
    DevAxis ax[3];
    const int32_t *xst;   // [ncx - 2]: first row x with base[x] >= i (xst[ncx - 3] = R)
    const double *wk3;    // [ncz][Z] dense slice weights w^3 (0 outside the support)
    const double *wk2;    // [ncz][Z] w^2
};

#define TILE_W 64   // columns per compact tile / fit item (one wave)
#define SLOT_R 64   // rows per fit item
#define VH_OOB 0x80000000u
#define N4_FIX 4294967296.0    // 2^32
#define N4_MAGIC 6755399441055744.0   // 1.5 * 2^52: x + MAGIC rounds x to an integer (|x| < 2^51)
#define HIST_UNIT 16777216.0f   // 2^24: Parzen weight unit (S3)
#define HIST_CSHIFT 44          // packed histogram word: count << 44 | sum of o-weights
#define LN2 0.69314718055994530942
#define PI_D 3.14159265358979323846

int vh_level_ncp(const vh_n4_params &p, int level, int axis);
DevLevel vh_dev_level(const vh_batch *b, const vh_n4_params &prm, int L);

// N4 driver selection (vh_run_opts.n4_mode)
bool vh_n4_study_eligible(const vh_batch *b, const vh_n4_params &prm, size_t *lds_bytes);
void vh_launch_n4_study(vh_batch *b, const vh_n4_params &prm);
bool vh_n4_studyg_eligible(const vh_batch *b, const vh_n4_params &prm, size_t *lds_bytes);
void vh_launch_n4_studyg(vh_batch *b, const vh_n4_params &prm);

// ---- small device helpers ----------------------------------------------------------------------
__device__ __forceinline__ int lanes_below(uint64_t m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    for (int off = 32; off > 0; off >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, off, 64));
    return v;
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    for (int off = 32; off > 0; off >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, off, 64));
    return v;
}
__device__ __forceinline__ void wave_lds_order() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// correctly rounded float exp through double (S1/S7/S9)
__device__ __forceinline__ float expf_cr(float x) { return (float)exp((double)x); }
// the same floats, by a short double polynomial when |x| <= 2^-5 (expf_small.h; PC pass 0)
__device__ __forceinline__ float expf_crs(float x) {
    return vh_expf_small(x, [](float v) { return expf_cr(v); });
}
// the Wiener kernel's Gaussian tail: (float)exp((double)x) is +0 for every float x < -104
// (e^-104 < 2^-150, half the smallest float denormal), and the double exp of such an argument
// took ~30 k cycles a step in the E map (ST_PROF r4e: thread 300's exp 0.96 M cycles per study)
__device__ __forceinline__ float expf_cr_tail(float x) { return x < -104.0f ? 0.0f : expf_cr(x); }

// S7x (conv_mode 1): expm1 of a float field difference
__device__ __forceinline__ float expm1c(float x) {
    if (fabsf(x) < 0.0625f)
        return x + x * x * (0.5f + x * (0.16666667f + x * (0.041666668f + x * 0.008333334f)));
    return (float)expm1((double)x);
}

// c / slope as IEEE float division, evaluated as (double)c * (1 / (double)slope) rounded once to
// float.  The double product is within 2^-52 (relative) of the exact quotient, and a quotient of
// two floats is never closer than 2^-49 (relative) to a float rounding midpoint, so the rounding
// lands on the correctly rounded quotient: bit-equal to c / slope.
__device__ __forceinline__ float div_r(float c, double rinv) { return (float)((double)c * rinv); }

// S3 sharpen value E(u)
__device__ __forceinline__ float sharpen_r(float u, float bmin, double rinv, const float *E, int bins,
                                           float fbins, float elast) {
    const float cidx = div_r(u - bmin, rinv);
    const int idx = (cidx >= 0.0f && cidx < fbins) ? (int)floorf(cidx) : bins;
    // branch-free (a divergent branch here split the fit's row groups): both table reads always
    // happen, at a clamped index when the value takes the last bin's E (= elast, fbins = bins)
    const bool in = idx < bins - 1;
    const int j = in ? idx : bins - 2;
    const float e0 = E[j], e1 = E[j + 1];
    float lin = e0 + (e1 - e0) * (cidx - (float)idx);
    __asm__ volatile("" : "+v"(lin));   // keeps the select a select (not a branch round the reads)
    return in ? lin : elast;
}

// S3 Parzen histogram contribution of one U value, packed as (1 << 44) | trunc(o * 2^24) on bin
// idx; 0 (and idx = 0) when the value adds nothing (outside [0, bins), NaN padding, or the last bin
// with o > 0 -- ITK's else-if).  Bin b of the histogram is then
//   H[b] = count[b] * 2^24 - osum[b] + osum[b - 1]      (2^-24 units, exact integers)
// i.e. the value adds 2^24 - a1 to bin idx and a1 to bin idx + 1.  One 64-bit add per value; a
// packed bin stays exact for < 2^20 values.
__device__ __forceinline__ unsigned long long hist_pack(float u, float bmin, double rinv, int bins,
                                                        int &idx) {
    const float cidx = div_r(u - bmin, rinv);
    const bool in = cidx >= 0.0f && cidx < (float)bins;   // false for NaN
    const float cf = in ? floorf(cidx) : 0.0f;
    const float o = in ? cidx - cf : 0.0f;
    idx = (int)cf;
    const bool keep = in && !(idx == bins - 1 && o > 0.0f);
    const uint32_t a1 = (uint32_t)(o * HIST_UNIT);   // o * 2^24 is exact in float
    return keep ? ((1ull << HIST_CSHIFT) | (unsigned long long)a1) : 0ull;
}
__device__ __forceinline__ unsigned long long hist_count(unsigned long long w) { return w >> HIST_CSHIFT; }
__device__ __forceinline__ unsigned long long hist_osum(unsigned long long w) {
    return w & ((1ull << HIST_CSHIFT) - 1ull);
}

// ---- 128-bit fixed point -------------------------------------------------------------------------
// Exact, order-free accumulation of doubles with a huge dynamic range: trunc(|v| 2^80) as a 128-bit
// two's-complement integer, kept as (lo u64, hi i64) and added with integer atomics (LDS or global),
// the low word's carry detected from the value the atomic returns.
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

__device__ __forceinline__ float wsel(float4 w, int d) {
    return d == 0 ? w.x : d == 1 ? w.y : d == 2 ? w.z : w.w;
}
template <int P>
__device__ __forceinline__ double wpow(float w) {
    const double d = (double)w;
    return P == 3 ? d * d * d : d * d;
}

// ---- one level's axis tables as the fit / eval read them (LDS in n4_study, global in n4) ------
struct TabV {
    const float4 *wx, *wy, *wz;
    const double *ix, *iy, *iz;
    const int32_t *bx, *by, *bz;
    const int2 *krz;
    const int32_t *xst;   // [ncx - 2]
};

// ---------------------------------------------------------------------------------------------
// work item = (64-column tile, 64-row slot) of one study: the wave's view of its rows
// ---------------------------------------------------------------------------------------------
// a wave-uniform value moved to an SGPR (values read from LDS or shuffled are VGPRs to the
// compiler; row loops indexed by them then pay a readfirstlane + wait states per row)
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ float uni(float v) { return __int_as_float(uni(__float_as_int(v))); }
__device__ __forceinline__ double uni(double v) {
    const long long b = __double_as_longlong(v);
    return __longlong_as_double(((long long)(uint32_t)uni((int)(b >> 32)) << 32) | (uint32_t)uni((int)b));
}

struct Item {
    int tile, x0, xs, xe;     // wave-uniform: tile, slot's first row, first / last non-empty row
    uint64_t mreg;            // lane l: mask == 1 lanes of row x0 + l
    int rsreg;                // lane l: compact offset of row x0 + l
    int rrreg;                // lane l: raster rank of the first masked voxel of (tile, row x0 + l)
    int col, y, z;            // this lane's column
    bool colok;
    int c0, y0, y1, z0, z1, ny;   // tile geometry (uniform)
};

// rowmask / rowstart / rrank: [tiles][R] arrays of this study
__device__ __forceinline__ bool item_begin(Item &it, const uint64_t *rowmask, const int32_t *rowstart,
                                           const int32_t *rrank, int R, int C, int Z, int CZ,
                                           int nslots, int item) {
    const int lane = threadIdx.x & 63;
    item = uni(item);
    it.tile = item / nslots;
    it.x0 = (item % nslots) * SLOT_R;
    const int64_t rbase = (int64_t)it.tile * R;
    const int xr = it.x0 + lane;
    it.mreg = xr < R ? rowmask[rbase + xr] : 0ull;
    it.rsreg = xr < R ? rowstart[rbase + xr] : 0;
    it.rrreg = (rrank && xr < R) ? rrank[rbase + xr] : 0;
    const uint64_t nzb = __ballot(it.mreg != 0ull);
    if (nzb == 0ull) return false;
    it.xs = it.x0 + __builtin_ctzll(nzb);
    it.xe = it.x0 + 63 - __builtin_clzll(nzb);
    it.col = it.tile * TILE_W + lane;
    it.colok = it.col < CZ;
    it.y = it.colok ? it.col / Z : 0;
    it.z = it.colok ? it.col % Z : 0;
    it.c0 = it.tile * TILE_W;
    const int c1 = min(it.c0 + TILE_W, CZ) - 1;
    it.y0 = it.c0 / Z;
    it.y1 = c1 / Z;
    it.z0 = it.c0 % Z;
    it.z1 = c1 % Z;
    it.ny = it.y1 - it.y0 + 1;
    (void)C;
    return true;
}

// Compact byte offset of (row x, this lane) or VH_OOB when the voxel is not in the mask; x is
// wave-uniform and inside the item's slot.  With rr != nullptr also the voxel's raster rank (index
// among the study's masked voxels in raster order: the order of ITK's convergence scan).
__device__ __forceinline__ uint32_t item_off(const Item &it, int x, bool valid, int *rr = nullptr) {
    const int xl = x - it.x0;
    const uint32_t mlo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)it.mreg, xl);
    const uint32_t mhi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(it.mreg >> 32), xl);
    const uint64_t m = ((uint64_t)mhi << 32) | mlo;
    const int r0 = __builtin_amdgcn_readlane(it.rsreg, xl);
    // lane's own bit from two lane counts (bits 0..lane minus bits below lane): no per-lane
    // (1 << lane) mask pair to keep in VGPRs across the row loops
    const int below = lanes_below(m);
    const bool on = valid && lanes_below(m >> 1) + (int)(m & 1ull) != below;
    if (rr) *rr = __builtin_amdgcn_readlane(it.rrreg, xl) + below;
    return on ? (uint32_t)(r0 + below) * 4u : VH_OOB;
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

// ---------------------------------------------------------------------------------------------
// S5 fit: contraction of finished control rows of the item's tile (wave-collective).  A wave keeps
// up to nbmax finished rows Q[r][lane] (control rows i0 .. i0+nr-1) in its LDS ring and contracts
// them together:
//   S[r][y][k]    = fma chain over the tile's slices z of col y (ascending): Wk[k][z] Q[r][(y, z)]
//   num[i0+r][j][k] += fix128( fma chain over the tile's cols y (ascending): wy(y, j)^P S[r][y][k] )
// In place (S overwrites Q) when the batch's stage-1 outputs fit the lanes' FIT_SO slots (all reads
// of a batch finish before its writes); otherwise into the separate buffer Sx, in chunks.
// ---------------------------------------------------------------------------------------------
#define FIT_NB 4        // finished control rows per contraction batch (max)
#define FIT_SO 4        // stage-1 outputs per lane per chunk
#ifndef FIT_G
#define FIT_G 6         // rows per lane with loads in flight together (r4bf / r4bg: 4 / 5 / 6 / 7 / 8 / 12 -> 17.97 / 18.00 / 17.89 / 18.15 / 18.27 / 22.2 ms isolated)
#endif

struct FitRing {
    double *q;        // [nbmax][rowcap] this wave's rows
    double *sx;       // separate stage-1 output buffer ([nbmax][rowcap]) or nullptr (in place)
    int rowcap;       // doubles per row (>= 64, >= ny * KT)
    int nbmax;        // rows per batch for this geometry
    int nr, i0;       // rows held, control row of row 0
};

// INPLACE (n4_study): one chunk, S overwrites Q; otherwise (n4) chunks into the separate rg.sx.
template <int P, bool INPLACE>
__device__ void fit_contract(FitRing &rg, const Item &it, const TabV &T, const double *Wk, int ncy,
                             int ncz, int Z, unsigned long long *numfix) {
    const int nr = rg.nr;
    if (nr == 0) return;
    const int lane = threadIdx.x & 63;
    wave_lds_order();
    const int klo = T.bz[it.y0 == it.y1 ? it.z0 : 0];
    const int KT = T.bz[it.y0 == it.y1 ? it.z1 : Z - 1] + 4 - klo;
    const int nyk = it.ny * KT;
    double *S = INPLACE ? rg.q : rg.sx;
    for (int o0 = 0; o0 < nr * nyk; o0 += 64 * FIT_SO) {
        // the FIT_SO outputs of a lane are independent fma chains over their slices: walk them in
        // lockstep (step s of every chain together) so the LDS latency of one chain hides behind
        // the others; each chain still adds its terms in slice order
        double outv[FIT_SO];
        const double *qp[FIT_SO], *wp[FIT_SO];
        int len[FIT_SO];
        int maxlen = 0;
#pragma unroll
        for (int q = 0; q < FIT_SO; ++q) {
            outv[q] = 0.0;
            len[q] = 0;
            qp[q] = rg.q;
            wp[q] = Wk;
            const int o = o0 + lane + 64 * q;
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
#ifndef FIT_SUNROLL
#define FIT_SUNROLL 4   // slice steps per trip: the next steps' LDS reads issued together (r4ay: 18.44 -> 18.39 ms)
#endif
#pragma unroll FIT_SUNROLL
        for (int s = 0; s < maxlen; ++s) {
#pragma unroll
            for (int q = 0; q < FIT_SO; ++q) {
                const int ss = min(s, max(len[q] - 1, 0));   // in-range read for finished chains
                const double v = fma(wp[q][ss], qp[q][ss], outv[q]);
                outv[q] = s < len[q] ? v : outv[q];
            }
        }
        if (INPLACE) wave_lds_order();   // in place: every read of the batch before any write
#pragma unroll
        for (int q = 0; q < FIT_SO; ++q) {
            const int o = o0 + lane + 64 * q;
            if (o < nr * nyk) S[(o / nyk) * rg.rowcap + o % nyk] = outv[q];
        }
        if (INPLACE) break;   // nbmax keeps a batch within one chunk
    }
    wave_lds_order();
    const int jlo = T.by[it.y0];
    const int JT = T.by[it.y1] + 4 - jlo;
    const int njk = JT * KT;
    for (int o = lane; o < nr * njk; o += 64) {
        const int r = o / njk, jk = o % njk;
        const int j = jlo + jk / KT, kk = jk % KT, k = klo + kk;
        const double *sr = S + r * rg.rowcap;
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
    wave_lds_order();
    rg.nr = 0;
}

// control row i (this lane's value v) is finished: into the ring, contract when the batch is full
template <int P, bool INPLACE>
__device__ __forceinline__ void fit_push(FitRing &rg, double v, int i, const Item &it,
                                         const TabV &T, const double *Wk, int ncy, int ncz, int Z,
                                         unsigned long long *numfix) {
    if (rg.nr == 0) rg.i0 = i;
    rg.q[rg.nr * rg.rowcap + (threadIdx.x & 63)] = v;
    if (++rg.nr == rg.nbmax) fit_contract<P, INPLACE>(rg, it, T, Wk, ncy, ncz, Z, numfix);
}

// rows per contraction batch for this item's geometry
template <bool INPLACE>
__device__ __forceinline__ void fit_ring_begin(FitRing &rg, const Item &it, const TabV &T, int Z,
                                               int nb_ring) {
    const int klo = T.bz[it.y0 == it.y1 ? it.z0 : 0];
    const int KT = T.bz[it.y0 == it.y1 ? it.z1 : Z - 1] + 4 - klo;
    rg.nbmax = INPLACE ? max(1, min(nb_ring, 64 * FIT_SO / (it.ny * KT))) : nb_ring;
    rg.nr = 0;
}

// One item's fit (S5).  MODE 0: numerator, row weights Wx = wx^3 / sum wx^2 (double2 pairs
// [2x], [2x+1]), p = (double)(u - sharpen(u)) * (1/sum wy^2 * 1/sum wz^2); MODE 1: denominator,
// Wx = wx^2, p = 1.  Each control row's column partial is an fma chain over the item's rows in
// row order: acc_a = fma(Wx(x, a), p(x), acc_a) for the window's four control rows.
template <int MODE, bool INPLACE, int FG = FIT_G>
__device__ void fit_item(const Item &it, const TabV &T, const double *Wk, const double2 *Wx,
                         int ncy, int ncz, int Z, int bins, const float *Ub, int64_t n,
                         const float *sE, float bmin, double rinv, FitRing &rg, int nb_ring,
                         unsigned long long *numfix, unsigned long long *fprof = nullptr) {
    // fprof (profiling builds): lane 0 adds the cycles of the row loops / pushes / contraction
    unsigned long long fpc = fprof ? clock64() : 0ull;
    auto fpm = [&](int k) {
        if (fprof && (threadIdx.x & 63) == 0) {
            const unsigned long long c = clock64();
            fprof[k] += c - fpc;
            fpc = c;
        }
    };
    constexpr int P = MODE == 0 ? 3 : 2;
    const __amdgpu_buffer_rsrc_t rU = st_rsrc(Ub, n);
    bmin = uni(bmin);   // SGPRs: as VGPRs they were spilled and reloaded once per voxel
    rinv = uni(rinv);
    const float fbins = uni((float)bins), elast = MODE == 0 ? uni(sE[bins - 1]) : 0.0f;
    const double isyz = MODE == 0 ? T.iy[it.y] * T.iz[it.z] : 1.0;
    int wb = uni(T.bx[it.xs]);
    double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0, acc3 = 0.0;
    int x = it.xs, tail = 0;
    fit_ring_begin<INPLACE>(rg, it, T, Z, nb_ring);
#pragma unroll 1
    for (;;) {
        if (x <= it.xe) {   // rows of control span wb: the window does not move
            const int rb = uni(min(it.xe, T.xst[wb + 1] - 1));
            // groups of FG rows, two per trip: the next group's U loads are in flight while this
            // group's rows are added (the chains still take the rows in order)
            uint32_t oA[FG], oB[FG];
            float uA[FG], uB[FG];
            auto issue = [&](int xb, uint32_t (&o)[FG], float (&u)[FG]) {
#pragma unroll
                for (int g = 0; g < FG; ++g) {
                    const int xg = xb + g;
                    o[g] = item_off(it, xg <= rb ? xg : rb, xg <= rb);
#ifdef AB_FIT_NOLOAD   // A/B builds only (fixed iteration counts): the fit without its U loads
                    if (MODE == 0) u[g] = 0.5f + 0.01f * (float)g;
#else
                    if (MODE == 0) u[g] = st_load(rU, o[g]);
#endif
                }
            };
            auto run = [&](int xb, const uint32_t (&o)[FG], const float (&u)[FG]) {
#pragma unroll
                for (int g = 0; g < FG; ++g) {
                    // branch-free: a masked-out lane / row past the span adds exact zeros (its U load
                    // returned 0, so every operand is finite) -- see eval_item for why
                    const bool on = o[g] != VH_OOB;
                    const int xg = xb + g <= rb ? xb + g : rb;
                    const double2 wa = Wx[2 * xg], wc = Wx[2 * xg + 1];
                    if (MODE == 0) {
                        const float rv = u[g] - sharpen_r(u[g], bmin, rinv, sE, bins, fbins, elast);
                        const double p = on ? (double)rv * isyz : 0.0;
                        acc0 = fma(wa.x, p, acc0);
                        acc1 = fma(wa.y, p, acc1);
                        acc2 = fma(wc.x, p, acc2);
                        acc3 = fma(wc.y, p, acc3);
                    } else {
                        acc0 += on ? wa.x : 0.0;
                        acc1 += on ? wa.y : 0.0;
                        acc2 += on ? wc.x : 0.0;
                        acc3 += on ? wc.y : 0.0;
                    }
                }
            };
            if (x <= rb) {
                issue(x, oA, uA);
#pragma unroll 1
                for (int xb = x;; xb += 2 * FG) {
                    // the next group is issued unconditionally (rows past rb load nothing): a branch
                    // round the issue makes its loads maybe-pending at the join
                    issue(xb + FG, oB, uB);
                    run(xb, oA, uA);
                    if (xb + FG > rb) break;
                    issue(xb + 2 * FG, oA, uA);
                    run(xb + FG, oB, uB);
                    if (xb + 2 * FG > rb) break;
                }
            }
            x = rb + 1 > x ? rb + 1 : x;
        }
        fpm(0);
        fit_push<P, INPLACE>(rg, acc0, wb, it, T, Wk, ncy, ncz, Z, numfix);   // control row wb is done
        fpm(1);
        acc0 = acc1; acc1 = acc2; acc2 = acc3; acc3 = 0.0;
        ++wb;
        if (x > it.xe && ++tail == 4) break;
    }
    fit_contract<P, INPLACE>(rg, it, T, Wk, ncy, ncz, Z, numfix);
    fpm(2);
    if (fprof && (threadIdx.x & 63) == 0) fprof[3] += 1;
}

// ---------------------------------------------------------------------------------------------
// U range for the next histogram (S2).  ITK scans in raster order with
//   if (u > max) max = u; else if (u < min) min = u;
// so the minimum skips every "record" voxel (strictly above all earlier ones).  Let u1 < ... < uK be
// the strictly increasing run at the start of the raster order (u(K+1) <= uK).  Every later record
// lies above uK >= u(K+1), a non-record, so it never is the minimum: ITK's minimum is the minimum
// over all voxels but the run.  The sweeps keep the maximum and the three smallest values (a
// multiset) per lane; the run is read back from the first masked voxels and taken out of the
// triple; the exact raster scan is left for a run that outlasts the voxels read back or that
// swallows the whole triple.
// ---------------------------------------------------------------------------------------------
struct Range3 {
    float mx, m1, m2, m3;   // max; three smallest, m1 <= m2 <= m3
};
__device__ __forceinline__ void r3_init(Range3 &r) {
    r.mx = -FLT_MAX;
    r.m1 = r.m2 = r.m3 = FLT_MAX;
}
// insert u into the sorted triple (med3 keeps the three smallest of the multiset)
__device__ __forceinline__ void r3_ins(Range3 &r, float u) {
    r.m3 = __builtin_amdgcn_fmed3f(r.m2, r.m3, u);
    r.m2 = __builtin_amdgcn_fmed3f(r.m1, r.m2, u);
    r.m1 = fminf(r.m1, u);
}
__device__ __forceinline__ void r3_add(Range3 &r, float u) {
    r.mx = fmaxf(r.mx, u);
    r3_ins(r, u);
}
__device__ __forceinline__ void r3_merge(Range3 &r, const Range3 &o) {
    r.mx = fmaxf(r.mx, o.mx);
    r3_ins(r, o.m1);
    r3_ins(r, o.m2);
    r3_ins(r, o.m3);
}
__device__ __forceinline__ Range3 r3_wave(Range3 r) {
    for (int off = 32; off > 0; off >>= 1) {
        Range3 o;
        o.mx = __shfl_xor(r.mx, off, 64);
        o.m1 = __shfl_xor(r.m1, off, 64);
        o.m2 = __shfl_xor(r.m2, off, 64);
        o.m3 = __shfl_xor(r.m3, off, 64);
        r3_merge(r, o);
    }
    return r;
}
// ITK's bin minimum from the merged range and the first masked voxels' values (u[0..nfirst)).
// Returns false when the exact raster scan is needed.
__device__ __forceinline__ bool r3_bin_min(const Range3 &r, const float *u, int nfirst, float &bmin) {
    if (nfirst < 3) return false;
    int K = 1;
    while (K < nfirst && u[K] > u[K - 1]) ++K;
    if (K == nfirst || !(u[K] <= u[K - 1])) return false;   // run may go on / NaN ends it
    const float m[3] = {r.m1, r.m2, r.m3};
    int j = 0;   // multiset difference of two ascending lists: triple minus run
    for (int i = 0; i < 3; ++i) {
        while (j < K && u[j] < m[i]) ++j;
        if (j < K && u[j] == m[i]) { ++j; continue; }
        bmin = m[i];
        return true;
    }
    return false;
}

// ---------------------------------------------------------------------------------------------
// S7 convergence (conv_mode 0): ITK's convergence measure (itkN4BiasFieldCorrectionImageFilter
// CalculateConvergenceMeasurement, RealType = float) over the masked voxels in raster order,
// d_k = B_old - B_new:
//   N += 1.0                                   float counter: exact up to 2^24, then frozen (itk_Nd)
//   p = (float)exp((double)d)
//   sig <- (float)((double)sig + ((double)sqr(p - mu) * (N - 1.0)) / N)      (N > 1)
//   mu  <- (float)((double)mu * (1.0 - 1.0 / N) + (double)(p / N))           (p / N: float division)
//   conv = (float)sqrt((double)sig / (N - 1.0)) / mu
// every right-hand side in double with ITK's separate roundings (oracle/n4_oracle.c conv_welford).
// The state is a serial float recurrence (the float running mean drifts) that must be evaluated in
// raster order.  It is run either by PC (guess and verify, below: the default) or by this serial
// chain (ST_PC 0 / VH_N4_SERIAL_CHAIN, A/B and the equivalence test): waves of one workgroup over a
// ring of 64-step blocks:
//   producers (several waves): per block, all lanes compute p, a = RN(1 - RN(1/N)),
//     b = RN_f(p / N) and N into the block's LDS slot;
//   wave A (mu): the 64 steps mu <- (float)(RN(mu a) + b), systolic (chain_sys64), recording mu
//     before each step for wave B;
//   wave B (sig): lanes form t = RN(RN(sqr(p - mu_prev) (N - 1)) / N) in parallel (the product is
//     exact: 24 x 24 bits), then the 64 steps sig <- (float)(sig + t), systolic.
// ---------------------------------------------------------------------------------------------
#define ITK_NMAX 16777216.0   // 2^24: float N += 1.0 stops growing there (2^24 + 1 rounds to 2^24)
// The certified decisions' accumulation factor (round 6): a float running sum of m positive terms,
// each step rounded once (relative error <= 2^-24 of that step's sum), keeps at least (1 - 2^-24)^m
// of their exact sum -- s_m = sum_k t_k prod_{j >= k} (1 + delta_j) >= (1 - 2^-24)^m sum_k t_k --
// rounded down here by a 2^-40 margin (exp / log1p are within a few double ulps).  By Bernoulli it
// is >= the linear form 1 - m 2^-24 the decisions used before, and unlike that form it stays
// positive for m > 2^24 (config 5's 28 M-voxel iterations, where the linear form was < 0).
__host__ __device__ inline double pc_accum_factor(double m) {
    return exp(m * log1p(-0x1p-24)) * (1.0 - 0x1p-40);
}
__device__ __forceinline__ double itk_Nd(double k) { return fmin(k, ITK_NMAX); }
// the measure from the final state after n steps
__device__ __forceinline__ float itk_conv(float mu, float sig, int64_t n) {
    const float sd = (float)sqrt((double)sig / (itk_Nd((double)n) - 1.0));
    return sd / mu;
}

#ifndef CH_SLOTS
#define CH_SLOTS 16
#endif
struct ChainSlot {
    double2 ab[64];    // (RN(1 - RN(1/N)), RN_f(p / N)) for wave A; (1, 0) past the end (a no-op step)
    double nd[64];     // N of the step (double)
    float p[64];
    float mu[64];      // mu before step k
    int ready;         // block + 1 once a producer has filled the slot for that block
    int pad[3];
};
#ifndef CH_PRIO
#define CH_PRIO 3
#endif
// Wave roles by SIMD.  A workgroup's waves are dealt to the CU's 4 SIMDs round-robin (wave w on
// SIMD w % 4), and a producer's VALU instruction in flight on wave A's SIMD delays A's next
// dependent step however A is prioritised.  So wave 0 (A) and wave 1 (B) keep SIMDs 0 and 1 to
// themselves and the producers are the waves on SIMDs 2 and 3.  Producer index of wave w, or -1.
__device__ __forceinline__ int chain_prod_id(int w) { return (w & 3) >= 2 ? (w >> 2) * 2 + (w & 1) : -1; }
// waves a workgroup needs for np producers
constexpr int chain_waves(int np) { return 4 * ((np + 1) / 2); }
struct ChainState {
    int a_done, b_done, c_done;   // blocks finished by wave A / wave B / the producer
    float mu, conv;
#ifdef CH_PROF
    unsigned long long wait[3], total[3];   // cycles polling / in the loop: A, B, producer
#endif
};
#ifdef CH_PROF
#define CH_T0() const unsigned long long _ch_t0 = clock64()
#define CH_WAIT(w, loop) do { const unsigned long long _t = clock64(); loop; w += clock64() - _t; } while (0)
#define CH_DONE(i, w) do { if ((threadIdx.x & 63) == 0) { cs->wait[i] = w; cs->total[i] = clock64() - _ch_t0; } } while (0)
#else
#define CH_T0() do { } while (0)
#define CH_WAIT(w, loop) do { (void)(w); loop; } while (0)
#define CH_DONE(i, w) do { (void)(w); } while (0)
#endif

// Counter hand-off between waves of one workgroup through LDS only.  LDS executes a wave's DS
// instructions in order, so a counter written after the data (and read before it) needs no
// hardware fence -- only a compiler barrier.  (A workgroup-scope atomic release would also wait
// for this wave's outstanding global loads, vmcnt(0): it serialised the producer's prefetch.)
// (Relaxed atomics rather than volatile: a volatile access through a generic pointer stays a flat
// access, which counts against vmcnt too.)
__device__ __forceinline__ int lds_load_acq(int *p) {
    const int v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    asm volatile("" ::: "memory");
    return v;
}
__device__ __forceinline__ void lds_store_rel(int *p, int v) {
    asm volatile("" ::: "memory");
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Producer wave: per block of 64 steps, all lanes compute p = (float)exp((double)d), the mu step
// constants (a, b) and N into the block's LDS slot, up to CH_SLOTS blocks ahead of wave B.  The n
// d values are in raster order: Dr[k] (perm == nullptr), else Dr[perm[k]].  np producer waves
// share the blocks round-robin (producer pid takes blk = pid mod np); each prefetches its next
// block's d (and perm entries two blocks ahead) while it processes the current one.
template <int NS = CH_SLOTS>
__device__ void chain_wave_prod(const float *Dr, const int32_t *perm, int64_t n, ChainSlot *slots,
                                ChainState *cs, int pid, int np) {
    const int lane = threadIdx.x & 63;
    const int64_t nblk = (n + 63) / 64;
    int64_t blk = pid;
    auto ld_perm = [&](int64_t b) -> int32_t {
        const int64_t j = b * 64 + lane;
        return perm && j < n ? perm[j] : 0;
    };
    auto ld_d = [&](int64_t b, int32_t pj) -> float {
        const int64_t j = b * 64 + lane;
        return j < n ? Dr[perm ? (int64_t)pj : j] : 0.0f;
    };
    int32_t p1 = ld_perm(blk + np);
    float dnext = ld_d(blk, ld_perm(blk));
    int bseen = 0;   // last b_done read: slots of blocks < bseen + NS are free
    unsigned long long wt = 0;
    CH_T0();
    for (; blk < nblk; blk += np) {
        ChainSlot &S = slots[blk % NS];
        const int64_t j = blk * 64 + lane;
        const float d = dnext;
        dnext = ld_d(blk + np, p1);
        p1 = ld_perm(blk + 2 * np);
        const bool ok = j < n;
        const float p = expf_crs(d);
        const double N = itk_Nd((double)(j + 1));
        const double r = 1.0 / N;
        const double2 ab = ok ? make_double2(1.0 - r, (double)(float)((double)p * r))   // p / N, div_r form
                              : make_double2(1.0, 0.0);
        if (blk >= NS + bseen)
            CH_WAIT(wt, while ((bseen = lds_load_acq(&cs->b_done)) <= (int)(blk - NS)) __builtin_amdgcn_s_sleep(1));
        S.ab[lane] = ab;
        S.nd[lane] = N;
        S.p[lane] = p;
        wave_lds_order();
        if (lane == 0) lds_store_rel(&S.ready, (int)(blk + 1));
    }
    if (pid == 0) CH_DONE(2, wt);
}

// Before a chain: every slot's ready flag cleared (a flag left from the previous chain could name
// the same block).  Threads (or lanes, tid = lane) [0, NS), then a barrier / the go signal.
template <int NS = CH_SLOTS>
__device__ __forceinline__ void chain_reset(ChainSlot *slots, ChainState *cs, int tid = threadIdx.x) {
    if (tid < NS) slots[tid].ready = 0;
    if (tid == 0) {
        cs->a_done = 0;
        cs->b_done = 0;
        cs->c_done = 0;
    }
}

// ---- the 64 serial steps of one block, systolic ------------------------------------------------
// Lane j holds step j's constants (one LDS read of the block by all lanes).  Every tick all lanes
// take the float x of lane j - 1 (DPP wave_shr:1; lane 0, which has no source lane, keeps the
// carried-in x) and apply their own step.  After tick t lanes 0..t hold the chain's values and keep
// them (their inputs no longer change), so after 64 ticks lane j holds x after step j, and the
// shifted copy holds x before it.  No LDS access on the chain.
// MU: x <- (float)(RN(x q0) + q1) (mul, add: ITK's two roundings); SIG: x <- (float)(x + q1) (q0
// is 1, or 0 with q1 = 0 for a no-op step: fma(q1, q0, x) is then the plain sum).  xin is
// wave-uniform; returns lane 63's x (wave-uniform); rec = x before the lane's step.
template <bool MU>
__device__ __forceinline__ float chain_sys64(double q0, double q1, float xin, float &rec) {
    float xf = xin, xs = xin;
    double x;
    if (MU)
        asm volatile(".rept 64\n\t"
                     "s_nop 1\n\t"   // VALU write -> DPP read: 2 wait states
                     "v_mov_b32_dpp %1, %0 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"
                     "v_cvt_f64_f32 %2, %1\n\t"
                     "v_mul_f64 %2, %2, %3\n\t"
                     "v_add_f64 %2, %2, %4\n\t"
                     "v_cvt_f32_f64 %0, %2\n\t"
                     ".endr"
                     : "+v"(xf), "+v"(xs), "=&v"(x)
                     : "v"(q0), "v"(q1));
    else
        asm volatile(".rept 64\n\t"
                     "s_nop 1\n\t"
                     "v_mov_b32_dpp %1, %0 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"
                     "v_cvt_f64_f32 %2, %1\n\t"
                     "v_fma_f64 %2, %4, %3, %2\n\t"
                     "v_cvt_f32_f64 %0, %2\n\t"
                     ".endr"
                     : "+v"(xf), "+v"(xs), "=&v"(x)
                     : "v"(q0), "v"(q1));
    rec = xs;
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xf), 63));
}
// ---- S7 by guess and verify ("PC") ------------------------------------------------------------
// The recurrence is serial, but one step is cheap to *check*: given the float state before a step,
// the state after it is a pure function of that state and the step's inputs.  So the n steps are cut
// into NL consecutive blocks, one per lane; every lane runs its block from a GUESS of the state at
// the block's start, and the guesses are exact iff every block's computed end equals the next
// block's guess (block 0 starts from the exact (0, 0)).  That check is the termination test, so the
// result is the serial recurrence bit for bit whatever the guesses were; the guesses only decide how
// many rounds it takes.  Between rounds the block ends propagate into new guesses through an affine
// model of each block's map (delta_{j+1} = a_j delta_j + (end_j - guess_{j+1}); a = 1 for sig, whose
// float steps add the same rounded increment anywhere inside a binade; for mu the secant of the
// block's map from the previous round, clamped to [0, 1], else the linear model (k0 - 1) / k1 of the
// running mean).  A block whose predecessor matched gets the predecessor's end exactly (delta = 0),
// so the exact prefix grows every round; after PC_RMAX rounds the rest runs serially from the
// first mismatch.  Measured on the bench studies' d sequences: 6 - 21 rounds (scripts/dev/pc_sim.c).
//
// Step arithmetic is that of the serial chain (chain_wave_prod / _mu / _sig, ITK's roundings) with
// the two divisions replaced by exact equivalents: r = RN(1/N) by rcp and two Newton steps
// (pc_rcp, checked bit-exact against IEEE division for every N < 2^25 by
// scripts/microbench/recip_exact.hip), and RN(Q / N) by Markstein's correction y + r (Q - N y)
// from y = RN(Q r) (pc_div: y is faithful and r correctly rounded, so the corrected quotient is
// the correctly rounded one; tests/test_n4_oracle.py checks it against IEEE division).
//
// Layout of the step inputs: block j holds steps [k0_j, k0_j + len_j) (1-based), len_j = L + (j < rem),
// L = n / NL, rem = n % NL; step s of block j lives at s NL + j, so one wave-wide load reads 64
// consecutive floats.  pc_addr maps a raster rank (0-based step index) to that position; the map is
// a bijection of [0, n).
#ifndef PC_RMAX
#define PC_RMAX 48
#endif
struct PcMap {
    uint32_t L, rem, big;   // big = rem (L + 1): raster ranks below it are in the long blocks
    double rL, rL1;         // 1 / L, 1 / (L + 1)
};
__device__ __forceinline__ PcMap pc_map(int64_t n, int NL) {
    PcMap m;
    m.L = (uint32_t)(n / NL);
    m.rem = (uint32_t)(n % NL);
    m.big = m.rem * (m.L + 1);
    m.rL = m.L ? 1.0 / (double)m.L : 0.0;
    m.rL1 = 1.0 / (double)(m.L + 1);
    return m;
}
__device__ __forceinline__ uint32_t pc_udiv(uint32_t r, uint32_t d, double rd) {
    uint32_t q = (uint32_t)((double)r * rd);
    if ((uint64_t)q * d > r) --q;
    else if ((uint64_t)(q + 1) * d <= r) ++q;
    return q;
}
template <int NL>
__device__ __forceinline__ uint32_t pc_addr(uint32_t r, const PcMap &m) {
    uint32_t j, s;
    if (r < m.big) {
        j = pc_udiv(r, m.L + 1, m.rL1);
        s = r - j * (m.L + 1);
    } else {
        const uint32_t r2 = r - m.big, j2 = pc_udiv(r2, m.L, m.rL);
        j = m.rem + j2;
        s = r2 - j2 * m.L;
    }
    return s * NL + j;
}
__device__ __forceinline__ uint32_t pc_len(const PcMap &m, uint32_t j) { return m.L + (j < m.rem ? 1u : 0u); }
__device__ __forceinline__ uint32_t pc_k0(const PcMap &m, uint32_t j) { return j * m.L + min(j, m.rem) + 1u; }

// RN(1 / N) for an integer N < 2^25: rcp, then two Newton steps with exact fma residuals
__device__ __forceinline__ double pc_rcp(double kd) {
    double y = __builtin_amdgcn_rcp(kd);
    double e = fma(-kd, y, 1.0);
    y = fma(y, e, y);
    e = fma(-kd, y, 1.0);
    return fma(y, e, y);
}
// RN(Q / N) from r = RN(1 / N) (Markstein): y = RN(Q r) is within an ulp of Q / N, the residual
// Q - N y is exact by fma, and RN(y + r (Q - N y)) is the correctly rounded quotient
__device__ __forceinline__ double pc_div(double Q, double N, double r) {
    const double y = Q * r;
    const double e = fma(-N, y, Q);
    return fma(e, r, y);
}
// the constants of step k (kd = k, N = itk_Nd(k)): A = RN(1 - RN(1/N)) and B = RN_f(p / N) as
// chain_wave_prod forms them (div_r form, r = RN(1/N)), and N, r for sig's RN(Q / N)
struct PcK {
    double A, B, N, r;
};
__device__ __forceinline__ PcK pc_consts(double kd, float p) {
    PcK q;
    q.N = itk_Nd(kd);
    q.r = pc_rcp(q.N);
    q.A = 1.0 - q.r;
    q.B = (double)(float)((double)p * q.r);
    return q;
}
// one step on the float state (mu, sig) with ITK's roundings; sig is untouched at k = 1 (N > 1);
// the sig product sqr(p - mu) (N - 1) is exact in double (24-bit by at most 24-bit integers)
__device__ __forceinline__ void pc_apply(const PcK &q, float p, bool first, float &mu, float &sig) {
    if (!first) {
        const float d = p - mu;
        sig = (float)__dadd_rn((double)sig, pc_div((double)(d * d) * (q.N - 1.0), q.N, q.r));
    }
    mu = (float)__dadd_rn(__dmul_rn((double)mu, q.A), q.B);
}
__device__ __forceinline__ void pc_step(double kd, float p, float &mu, float &sig) {
    pc_apply(pc_consts(kd, p), p, kd == 1.0, mu, sig);
}
// a lane's block: len steps from k0 over the inputs at P[s NL + j].  Groups of 8 steps without
// guards (the constants of the 8 steps are independent of the state, so they overlap the two
// 8-step chains), the next group's loads in flight; the tail step by step.
template <int NL>
__device__ __forceinline__ void pc_block(const float *P, uint32_t j, uint32_t len, uint32_t k0,
                                         float &mu, float &sig, uint32_t nl = NL) {
    float cur[8], nxt[8];
    // unconditional loads at clamped steps (a guarded load waited for itself before the next issued);
    // the values past the block's end are never used
    // (an empty block reads P[0], which every non-empty call has written: past a tiny study's block
    // layout P[j] could lie beyond the buffer)
    const uint32_t lc = len ? len - 1u : 0u, jc = len ? j : 0u;
#pragma unroll
    for (int i = 0; i < 8; ++i) cur[i] = P[(size_t)((uint32_t)i < len ? (uint32_t)i : lc) * nl + jc];
    double kd = (double)k0;
    uint32_t s0 = 0;
    for (; s0 + 8 <= len; s0 += 8) {
#pragma unroll
        for (int i = 0; i < 8; ++i) nxt[i] = P[(size_t)(s0 + 8 + i < len ? s0 + 8 + i : lc) * nl + jc];
        PcK q[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) q[i] = pc_consts(kd + (double)i, cur[i]);
        const bool first = kd == 1.0;
        pc_apply(q[0], cur[0], first, mu, sig);
#pragma unroll
        for (int i = 1; i < 8; ++i) pc_apply(q[i], cur[i], false, mu, sig);
        kd += 8.0;
#pragma unroll
        for (int i = 0; i < 8; ++i) cur[i] = nxt[i];
    }
#pragma unroll
    for (int i = 0; i < 7; ++i)
        if (s0 + i < len) {
            pc_step(kd, cur[i], mu, sig);
            kd += 1.0;
        }
}

// 32 bytes, 16-aligned: the compiler merges neighbouring fields into b64 / b128 LDS accesses, and a
// b128 access at an address that is only 8-aligned stores the wrong bytes (seen with a 24-byte
// block: the pass-0 sums came back as garbage).
struct alignas(16) PcBlk {
    float gmu, gsig;     // guess of the state at the block start
    float emu, esig;     // the block's computed end
    float gmu_o, emu_o;  // the previous round's guess and end (secant of the mu map)
    float sp0, sp1;      // pass 0 only: (s1, s2) below
};
// LDS through an address_space(3) pointer: pcw_run is not inlined, so its LDS pointers are generic
// and every access compiled to a flat_load / flat_store, which counts in vmcnt: waiting for one
// waited for every global load in flight too (pass 0's prefetch).  A C-style cast to address space
// 3 gives ds_read / ds_write (lgkmcnt only).
typedef __attribute__((address_space(3))) float lds_f32;
__device__ __forceinline__ float lds_ld(const float *p) { return *(const lds_f32 *)p; }
__device__ __forceinline__ void lds_st(float *p, float v) { *(lds_f32 *)p = v; }
// any object in LDS (PcShared fields) read / written through an address-space-3 pointer
// (the host compilation pass of these device functions has no address spaces: plain accesses there)
template <class T> __device__ __forceinline__ T lget(const T &r) {
#if __HIP_DEVICE_COMPILE__
    return *(const __attribute__((address_space(3))) T *)&r;
#else
    return r;
#endif
}
template <class T> __device__ __forceinline__ void lset(T &r, const T &v) {
#if __HIP_DEVICE_COMPILE__
    *(__attribute__((address_space(3))) T *)&r = v;
#else
    r = v;
#endif
}
template <int NL>
struct PcShared {
    PcBlk b[NL];
    int done, fallback, first_bad, rounds;   // done / fallback: the request number they refer to
    float mu, sig;
    int bar_cnt, bar_gen;
    // all-wave update (pcw_*): per-wave aggregates of the block transitions
    double agA[NL / 64], agB[NL / 64], agS[NL / 64];
    int agFirst[NL / 64];
    // exact sig after stage 0 (pcx_*): t-slot allocator, result tag, walks taken
    int xslots, xdone, xwalks, xslow;
    int nfrz;   // pcw_run calls closed by the frozen serial (diagnostics; reset per call)
    int nfr;    // stage 0 at its cap: blocks past the frontier certified frozen at their guesses
#ifdef PC_PROF
    int pchg[32], pwav[32];   // stage-0 rounds: blocks whose start changed, waves that ran
    unsigned long long xwcyc, xscyc;   // PCX scan: cycles in walks, whole scan
#endif
    // pass 0: per block, the float starts m for which every step of the block leaves mu at m
    // (pc_mu_serial_frozen; empty for blocks before step PC_FRZ_K0)
    float4 fz[NL];   // (lo, hi) for starts in (0.5, 1], (lo, hi) for starts in (1, 2)
    // pass-0 block sums of p - 1 and (p - 1)^2 (double, 16-aligned pair over gmu_o .. sp1: those
    // fields are written by round 0 before they are next read)
    __device__ double &s1(int j) { return *reinterpret_cast<double *>(&b[j].gmu_o); }
    __device__ double &s2(int j) { return *reinterpret_cast<double *>(&b[j].sp0); }
};

// Initial guesses from the running mean / variance sum in double (one wave, PB = NL / 64 blocks per
// lane, fixed-order scan).
template <int NL>
__device__ void pc_guess(PcShared<NL> &S, const PcMap &m) {
    constexpr int PB = NL / 64;
    const int lane = threadIdx.x & 63;
    double l1[PB], l2[PB], t1 = 0.0, t2 = 0.0;
#pragma unroll
    for (int i = 0; i < PB; ++i) {
        l1[i] = t1;
        l2[i] = t2;
        t1 += S.s1(lane * PB + i);
        t2 += S.s2(lane * PB + i);
    }
    double x1 = t1, x2 = t2;   // inclusive scan of the lane totals
    for (int off = 1; off < 64; off <<= 1) {
        const double y1 = __shfl_up(x1, off, 64), y2 = __shfl_up(x2, off, 64);
        if (lane >= off) {
            x1 = y1 + x1;
            x2 = y2 + x2;
        }
    }
    double e1 = __shfl_up(x1, 1, 64), e2 = __shfl_up(x2, 1, 64);
    if (lane == 0) e1 = e2 = 0.0;
#pragma unroll
    for (int i = 0; i < PB; ++i) {
        const uint32_t jb = lane * PB + i;
        const double K = (double)(pc_k0(m, jb) - 1u);
        const double S1 = e1 + l1[i], S2 = e2 + l2[i];
        float g = 0.0f, gs = 0.0f;
        if (K > 0.0) {
            g = (float)(1.0 + S1 / K);
            const double v = S2 - S1 * (S1 / K);
            gs = (float)(v > 0.0 ? v : 0.0);
        }
        S.b[jb].gmu = g;
        S.b[jb].gsig = gs;
    }
}

// Check and update after a round (one wave).  Sets S.done (every block end matched: S.mu / S.sig
// hold the result) or S.fallback (round cap: S.first_bad = the first transition that failed), else
// writes the next guesses.
template <int NL>
__device__ void pc_update(PcShared<NL> &S, const PcMap &m, int round, int req) {
    constexpr int PB = NL / 64;
    const int lane = threadIdx.x & 63;
    const int nbe = m.L ? NL : (int)m.rem;   // non-empty blocks
    double am[PB], bm[PB], bs[PB];
    float em[PB], es[PB];
    bool mism = false;
    int firstm = PB;
#pragma unroll
    for (int i = 0; i < PB; ++i) {
        const int jb = lane * PB + i;
        am[i] = 1.0;
        bm[i] = bs[i] = 0.0;
        em[i] = es[i] = 0.0f;
        if (jb < nbe - 1) {
            const PcBlk B = S.b[jb];
            const float gn = S.b[jb + 1].gmu, gsn = S.b[jb + 1].gsig;
            em[i] = B.emu;
            es[i] = B.esig;
            const bool mm = __float_as_uint(B.emu) != __float_as_uint(gn) ||
                            __float_as_uint(B.esig) != __float_as_uint(gsn);
            if (mm && firstm == PB) firstm = i;
            mism |= mm;
            bm[i] = (double)B.emu - (double)gn;
            bs[i] = (double)B.esig - (double)gsn;
            const uint32_t k0 = pc_k0(m, jb), k1 = k0 + pc_len(m, jb) - 1u;
            double a = (double)(k0 - 1u) / (double)k1;
            if (round > 0 && B.gmu != B.gmu_o) {
                const double sl = ((double)B.emu - (double)B.emu_o) / ((double)B.gmu - (double)B.gmu_o);
                if (sl >= 0.0 && sl <= 1.0) a = sl;
            }
            am[i] = a;
            S.b[jb].gmu_o = B.gmu;   // this round's guess and end, for the next round's secant
            S.b[jb].emu_o = B.emu;
        }
    }
    const uint64_t bal = __ballot(mism);
    if (bal == 0ull) {
        if (lane == 0) {
            S.mu = S.b[nbe - 1].emu;
            S.sig = S.b[nbe - 1].esig;
            S.rounds = round + 1;
            S.done = req;
        }
        return;
    }
    if (round + 1 >= PC_RMAX) {
        const int fl = __ffsll((unsigned long long)bal) - 1;
        if (lane == fl) {
            S.first_bad = lane * PB + firstm;
            S.rounds = round + 1;
            S.fallback = req;
        }
        return;
    }
    double Am = 1.0, Bm = 0.0, Bs = 0.0;   // the lane's transitions composed
#pragma unroll
    for (int i = 0; i < PB; ++i) {
        Bm = am[i] * Bm + bm[i];
        Am = am[i] * Am;
        Bs = Bs + bs[i];
    }
    for (int off = 1; off < 64; off <<= 1) {
        const double ya = __shfl_up(Am, off, 64), yb = __shfl_up(Bm, off, 64), ys = __shfl_up(Bs, off, 64);
        if (lane >= off) {
            Bm = Am * yb + Bm;
            Am = Am * ya;
            Bs = ys + Bs;
        }
    }
    double dm = __shfl_up(Bm, 1, 64), ds = __shfl_up(Bs, 1, 64);
    if (lane == 0) dm = ds = 0.0;
#pragma unroll
    for (int i = 0; i < PB; ++i) {
        const int jb = lane * PB + i;
        if (jb < nbe - 1) {
            S.b[jb + 1].gmu = dm == 0.0 ? em[i] : (float)((double)em[i] + am[i] * dm);
            S.b[jb + 1].gsig = ds == 0.0 ? es[i] : (float)((double)es[i] + ds);
            dm = am[i] * dm + bm[i];
            ds = ds + bs[i];
        }
    }
}

// Serial remainder after the round cap (one lane): blocks first_bad + 1 .. nbe - 1 from the exact
// end of block first_bad.
template <int NL>
__device__ void pc_serial(PcShared<NL> &S, const PcMap &m, const float *P) {
    const int nbe = m.L ? NL : (int)m.rem;
    const int f = S.first_bad;
    float mu = S.b[f].emu, sig = S.b[f].esig;
    for (int jb = f + 1; jb < nbe; ++jb) {
        const uint32_t len = pc_len(m, jb);
        double kd = (double)pc_k0(m, jb);
        for (uint32_t s = 0; s < len; ++s, kd += 1.0) pc_step(kd, P[(size_t)s * NL + jb], mu, sig);
    }
    S.mu = mu;
    S.sig = sig;
}

// ---- frozen mu (stage 0 at its round cap) -------------------------------------------------------
// Near convergence p = exp(d) ~ 1 and, past N ~ 2e4, most steps' increment (p - mu) / N is below
// half an ulp: ITK's float mu stops moving for whole blocks (r4u: 782 of 1024 blocks in an
// iteration of seed 1).  The frozen value sits thousands of ulps from the double running mean that
// seeds PC's guesses, a frozen block maps any nearby start to itself, so wrong guesses pass the
// continuity check and only the exact frontier corrects them, a few blocks per round: stage 0 and
// stage 1 hit their caps and the exact rounds end in the serial fallback (the 32 slowest of 256
// studies were exactly those with such an iteration).  Certified freeze: with mu' =
// RN_f(RN_d(m A) + B) = m + (p - m) / N + E, |E| <= 2^-23 / N + 7e-16 (A = RN(1 - RN(1/N)),
// B = RN_f(p RN(1/N)), m, p < 2), a start m with |p - m| <= N h stays at m when h + |E| is below
// half the float spacing on both sides of m: h = 0.99 2^-25 for m in (0.5, 1] (spacing 2^-24, and
// 2^-25 below 1.0), h = 0.99 2^-24 for m in (1, 2) (spacing 2^-23).  Pass 0 intersects those
// intervals over each block for both h (steps from PC_FRZ_K0 on, where |E| < 3e-11, far inside the
// 1 % margin), rounded inward to floats.  Checked on the CPU against the exact trajectories of the
// frozen iterations (every certified block's end equals its start; 734 of 1024 blocks certified in
// the worst one).
#define PC_FRZ_H1 (0x1p-25 * 0.99)
#define PC_FRZ_H2 (0x1p-24 * 0.99)
#define PC_FRZ_K0 4096u
__device__ __forceinline__ float f_up(double x) {
    float f = (float)x;
    if ((double)f < x) f = __uint_as_float(f >= 0.0f ? __float_as_uint(f) + 1u : __float_as_uint(f) - 1u);
    return f;
}
__device__ __forceinline__ float f_dn(double x) {
    float f = (float)x;
    if ((double)f > x) f = __uint_as_float(f > 0.0f ? __float_as_uint(f) - 1u : __float_as_uint(f) + 1u);
    return f;
}
__device__ __forceinline__ double readlane_d(double v, int l) {
    const long long x = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)x, l), hi = __builtin_amdgcn_readlane((int)(x >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (long long)(uint32_t)lo);
}
__device__ __forceinline__ bool pc_frozen(float4 z, float m) {
    return m > 0.5f && m < 2.0f && (m <= 1.0f ? (z.x <= m && m <= z.y) : (z.z <= m && m <= z.w));
}
// One wave: the exact mu at every block start past the frontier S.first_bad, skipping certified
// frozen blocks in O(1) and running the others step by step (lane l forms step s0 + l's constants,
// the chain reads them across lanes; the same exact step as pc_apply), at most PC_FRZ_RUN of them.
// Returns true when it reached the last block: stage 0's next round then matches everywhere and
// PCX gives sig.  Otherwise the exact starts it set stay as guesses and stage 1 goes on.
#ifndef PC_AMAX0
#define PC_AMAX0 28   // stage 0's round cap, where the frozen serial takes over (r4ba / r4bb: 20 / 24 / 28 / 40 / 56 -> 18.72 / 18.42 / 18.34 / 18.43 / 18.51 ms with the drift-seeded guesses)
#endif
#ifndef PC_FRZ_RUN
#define PC_FRZ_RUN 96   // blocks run step by step (~10 k cycles each) before handing back to the rounds
#endif
template <int NL>
__device__ bool pc_mu_serial_frozen(PcShared<NL> &S, const PcMap &m, const float *P) {
    const int lane = threadIdx.x & 63;
    const int nbe = m.L ? NL : (int)m.rem;
    const int f = S.first_bad;
    float mu = S.b[f].emu;   // block f's start was exact, so is its end
    int run = 0;
    for (int jb = f + 1; jb < nbe; ++jb) {
        if (lane == 0) S.b[jb].gmu = mu;
        if (pc_frozen(S.fz[jb], mu)) continue;   // end = start
        if (++run > PC_FRZ_RUN) return false;
        const uint32_t len = pc_len(m, jb), k0 = pc_k0(m, jb);
        for (uint32_t s0 = 0; s0 < len; s0 += 64) {
            const uint32_t s = s0 + (uint32_t)lane;
            double A = 1.0, B = 0.0;
            if (s < len) {
                const PcK q = pc_consts((double)(k0 + s), P[(size_t)s * NL + jb]);
                A = q.A;
                B = q.B;
            }
            const int cnt = (int)min(64u, len - s0);
            for (int i = 0; i < cnt; ++i)
                mu = (float)__dadd_rn(__dmul_rn((double)mu, readlane_d(A, i)), readlane_d(B, i));
        }
    }
    return true;
}

// ---- PC phase A: certified float steps --------------------------------------------------------
// The same recurrence with float-float step constants: r ~ r0 + rl (r0 = rcp(k), rl from the exact
// residual 1 - k r0), p/k ~ B = fma(p, r0, p rl), c ~ ch + cl.  mu: t = B - mu (r0 + rl) (two fmas)
// is within E of the exact increment (E = 2^-22 (|t1| + |t|) + 2^-46 |mu| bounds the roundings, the
// float-float error and the double rounding of the exact step), and the step's result is CERTIFIED
// when mu + (t - E) and mu + (t + E) round to the same float: the exact step then gives that float.
// Otherwise (a few steps per study and iteration) the lane takes the exact double step.  sig:
// y = RN(sig + q^2 ch), its rounding error rho, w = rho + q^2 cl, sig' = RN(y + w) (uncertified:
// equal to the exact step unless sig + q^2 c lies within ~2^-24 ulp of a tie).  Phase A iterates
// these rounds to their own fixed point; phase B (exact rounds) then verifies it, usually in one
// round (scripts/dev/pc_sim.c: 12 A + 1.2 B rounds on the bench studies, against 13 exact rounds).
// consts of one step for phase A
struct PcKf {
    float r0, rl, B, ch, cl;
};
__device__ __forceinline__ PcKf pc_kf(float k, float p) {
    PcKf q;
    q.r0 = __builtin_amdgcn_rcpf(k);
    q.rl = q.r0 * fmaf(-k, q.r0, 1.0f);
    q.B = fmaf(p, q.r0, p * q.rl);
    q.ch = 1.0f - q.r0;
    q.cl = ((-q.r0) - (q.ch - 1.0f)) - q.rl;
    return q;
}
// the same constants for two steps at once (packed FP32: v_pk_fma / v_pk_mul / v_pk_add issue two
// lanes' worth per instruction; identical roundings to pc_kf)
typedef float pc_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void pc_kf2(pc_f2 k, pc_f2 p, PcKf &qa, PcKf &qb) {
    const pc_f2 r0 = {__builtin_amdgcn_rcpf(k.x), __builtin_amdgcn_rcpf(k.y)};
    const pc_f2 rl = r0 * __builtin_elementwise_fma(-k, r0, (pc_f2)1.0f);
    const pc_f2 B = __builtin_elementwise_fma(p, r0, p * rl);
    const pc_f2 ch = 1.0f - r0;
    const pc_f2 cl = ((-r0) - (ch - 1.0f)) - rl;
    qa = PcKf{r0.x, rl.x, B.x, ch.x, cl.x};
    qb = PcKf{r0.y, rl.y, B.y, ch.y, cl.y};
}
// one phase-A step; returns false when the mu step is not certified (the state is then approximate)
// e0 >= r0 2^-40 + 2^-44 >= 2^-22 |mu rl| + 2^-46 |mu| for mu < 4 (one bound per block: r0 <= 1/k0)
template <bool SIG = true>
__device__ __forceinline__ bool pc_apx_step(const PcKf &q, float e0, float p, bool first, float &mu, float &sig) {
    if (!SIG && !first) {   // mu alone: sig carries sum (p - mu)^2 along the block (PCX's binade estimate)
        const float dq = p - mu;
        sig = fmaf(dq, dq, sig);
    }
    if (SIG && !first) {
        const float d = p - mu, q2 = d * d;
        const float y = fmaf(q2, q.ch, sig);
        const float rho = fmaf(q2, q.ch, sig - y);
        sig = y + fmaf(q2, q.cl, rho);
    }
    // E = 2^-21 |t| + e0 bounds 2^-22 (|t1| + |t|) + 2^-46 |mu| (|t1| <= |t| + |mu rl|, |rl| <=
    // 2^-23 r0); e0 assumes |mu| < 4 (p = exp(d) of a smooth field difference, mu a running mean of
    // them): a larger mu only makes a step uncertified-but-wrong, which phase B then corrects
    const float t1 = fmaf(-mu, q.r0, q.B);
    const float t = fmaf(-mu, q.rl, t1);
    const float E = fmaf(fabsf(t), 0x1p-21f, e0);
    const pc_f2 y2 = (pc_f2)mu + ((pc_f2)t + (pc_f2){-E, E});   // both ends in two packed adds
    const bool ok = y2.x == y2.y;
    mu = y2.x;   // = RN(mu + t) whenever ok
    return ok;
}
// a lane's block in phase A: groups of 8 steps without guards; a group with an uncertified step is
// redone with the exact steps (rare: the wave branches only when one of its lanes needs it)
// SIG = false: the mu recurrence alone (mu never reads sig); sig returns sum (p - mu)^2 over the
// block (approximate: the exact redo and tail steps add their sig increments instead)
// P is read through a buffer resource of np floats (np = (L + 1) nl, the block layout's extent): the
// step rows are loaded unguarded with the row offset in an SGPR (soffset), and rows past a block's
// end (or past np) cost nothing but a load whose value is never used (0 beyond np)
// one group of 8 phase-A steps from N = kf (the float counter); a group with an uncertified step is
// redone with the exact steps.  CLAMP: some step of the block may pass 2^24 (ITK's frozen counter).
// PART: only the first cnt (< 8) steps (a block's tail; lanes differ by at most one step there)
template <bool SIG, bool CLAMP, bool PART = false>
__device__ __forceinline__ void pc_apx_group(const float (&c)[8], float kf, float e0, float &mu, float &sig,
                                             int cnt = 8) {
    PcKf q[8];
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
        pc_f2 kk = kf + (pc_f2){(float)i, (float)(i + 1)};
        if (CLAMP) kk = __builtin_elementwise_min(kk, (pc_f2)(float)ITK_NMAX);
        pc_kf2(kk, (pc_f2){c[i], c[i + 1]}, q[i], q[i + 1]);
    }
    const float mu0 = mu, sig0 = sig;
    bool ok = !PART || cnt > 0 ? pc_apx_step<SIG>(q[0], e0, c[0], kf == 1.0f, mu, sig) : true;
#pragma unroll
    for (int i = 1; i < 8; ++i)
        if (!PART || i < cnt) ok &= pc_apx_step<SIG>(q[i], e0, c[i], false, mu, sig);
    if (!ok) {   // redo the group exactly
        mu = mu0;
        sig = sig0;
        double kd = (double)kf;
#pragma unroll 1
        for (int i = 0; i < (PART ? cnt : 8); ++i, kd += 1.0) pc_step(kd, c[i], mu, sig);
    }
}
// a lane's block in phase A: groups of 8 steps without guards, two groups per trip (the loads of
// one group in flight while the other computes, no register rotation); the tail by exact steps.
// SIG = false: the mu recurrence alone (mu never reads sig); sig returns sum (p - mu)^2 over the
// block (approximate: the exact redo and tail steps add their sig increments instead)
// P is read through a buffer resource of np floats (np = (L + 1) nl, the block layout's extent): the
// step rows are loaded unguarded with the row offset in an SGPR (soffset), and rows past a block's
// end (or past np) cost nothing but a load whose value is never used (0 beyond np)
template <bool SIG, bool CLAMP>
__device__ __forceinline__ void pc_block_apx_t(const __amdgpu_buffer_rsrc_t rs, int voff, int rstride,
                                               uint32_t len, uint32_t k0, float &mu, float &sig) {
    auto ld = [&](uint32_t s) {
        return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, voff, (int)s * rstride, 0));
    };
    // after the loop s0 differs between lanes whose lengths straddle a 16-step boundary: the row
    // offset goes in the lane's voffset there (an SGPR soffset would need a waterfall)
    auto ldv = [&](uint32_t s) {
        return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, voff + (int)s * rstride, 0, 0));
    };
    auto adv = [](float kf) { return CLAMP ? fminf(kf + 8.0f, (float)ITK_NMAX) : kf + 8.0f; };
    float a[8], b[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = ld((uint32_t)i);
    // N of the group's first step: min(k, 2^24), exact in float (ITK's frozen float counter)
    float kf = CLAMP ? fminf((float)k0, (float)ITK_NMAX) : (float)k0;
    const float e0 = fmaf(__builtin_amdgcn_rcpf(kf), 0x1p-39f, 0x1p-44f);   // covers every step's r0
    uint32_t s0 = 0;
    for (; s0 + 16 <= len; s0 += 16) {
#pragma unroll
        for (int i = 0; i < 8; ++i) b[i] = ld(s0 + 8 + (uint32_t)i);
        pc_apx_group<SIG, CLAMP>(a, kf, e0, mu, sig);
        kf = adv(kf);
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = ld(s0 + 16 + (uint32_t)i);
        pc_apx_group<SIG, CLAMP>(b, kf, e0, mu, sig);
        kf = adv(kf);
    }
    if (s0 + 8 <= len) {
#pragma unroll
        for (int i = 0; i < 8; ++i) b[i] = ldv(s0 + 8 + (uint32_t)i);
        pc_apx_group<SIG, CLAMP>(a, kf, e0, mu, sig);
        kf = adv(kf);
        s0 += 8;
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = b[i];
    }
    if (s0 < len) pc_apx_group<SIG, CLAMP, true>(a, kf, e0, mu, sig, (int)(len - s0));   // the tail
}
template <int NL, bool SIG = true>
__device__ __forceinline__ void pc_block_apx(const float *P, uint32_t j, uint32_t len, uint32_t k0,
                                             float &mu, float &sig, uint32_t nl, uint32_t np) {
    if (!SIG) sig = 0.0f;
    // P, nl and np are uniform (one study per workgroup / grid): scalar registers, no waterfall
    const uint64_t pa = (uint64_t)P;
    const uint32_t plo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)pa),
                   phi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(pa >> 32));
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(((uint64_t)phi << 32) | plo), 0, __builtin_amdgcn_readfirstlane((int)(np * 4u)), 0x00020000);
    const int voff = (int)(j * 4u), rstride = __builtin_amdgcn_readfirstlane((int)(nl * 4u));
    if ((uint64_t)k0 + len <= (uint64_t)ITK_NMAX) pc_block_apx_t<SIG, false>(rs, voff, rstride, len, k0, mu, sig);
    else pc_block_apx_t<SIG, true>(rs, voff, rstride, len, k0, mu, sig);
}

// ---- all-wave PC helpers (NL = threads of the workgroup, one block per thread) -----------------
// Affine transition maps T_j: delta -> a delta + b composed in block order: a wave-level inclusive
// scan (shuffles), per-wave aggregates in LDS, then each wave composes the aggregates before it.
// Fixed order, so deterministic; exact zeros stay exact zeros (the property the convergence proof
// uses: a block whose predecessors all matched gets the exact predecessor end).
// a double from the DPP source lane (CTRL / RMASK as __builtin_amdgcn_update_dpp); lanes with no
// source, or in rows the mask leaves out, get `id`
template <int CTRL, int RMASK>
__device__ __forceinline__ double dpp_d(double v, double id) {
    const long long x = __double_as_longlong(v), y = __double_as_longlong(id);
    const int lo = __builtin_amdgcn_update_dpp((int)y, (int)x, CTRL, RMASK, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(y >> 32), (int)(x >> 32), CTRL, RMASK, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (long long)(uint32_t)lo);
}
// one Hillis-Steele step of the affine scan: (A, B) <- (A, B) o (lane source's (A, B)); Bs sums
template <int CTRL, int RMASK>
__device__ __forceinline__ void aff_step(double &A, double &B, double &Bs) {
    const double ya = dpp_d<CTRL, RMASK>(A, 1.0), yb = dpp_d<CTRL, RMASK>(B, 0.0), ys = dpp_d<CTRL, RMASK>(Bs, 0.0);
    B = A * yb + B;
    A = A * ya;
    Bs = ys + Bs;
}
// Exclusive affine scan over the workgroup's NL threads.  One barrier in the middle (the wave
// aggregates published by lane 63), none at the end: two calls back to back need a __syncthreads()
// between them, or a fast wave's second-call aggregate store races a slow wave's first-call read.
template <int NL>
__device__ __forceinline__ void pcw_scan(PcShared<NL> &S, double a, double b, double bs, double &dm,
                                         double &ds) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double A = a, B = b, Bs = bs;
    // inclusive wave scan with DPP (row shifts, then the row broadcasts of gfx9): VALU moves instead
    // of 36 dependent ds_bpermute round trips
    aff_step<0x111, 0xf>(A, B, Bs);   // row_shr:1
    aff_step<0x112, 0xf>(A, B, Bs);   // row_shr:2
    aff_step<0x114, 0xf>(A, B, Bs);   // row_shr:4
    aff_step<0x118, 0xf>(A, B, Bs);   // row_shr:8
    aff_step<0x142, 0xa>(A, B, Bs);   // row_bcast:15 -> rows 1, 3
    aff_step<0x143, 0xc>(A, B, Bs);   // row_bcast:31 -> rows 2, 3
    if (lane == 63) {
        lset(S.agA[w], A);
        lset(S.agB[w], B);
        lset(S.agS[w], Bs);
    }
    const double ea = dpp_d<0x138, 0xf>(A, 1.0), eb = dpp_d<0x138, 0xf>(B, 0.0),   // wave_shr:1
                 es = dpp_d<0x138, 0xf>(Bs, 0.0);
    __syncthreads();
    // the waves before this one: lanes v < w hold wave v's aggregate, scanned across the row (NL / 64
    // <= 16 waves: one row), lane w - 1 has their composition applied to delta = 0
    static_assert(NL / 64 <= 16, "one DPP row of wave aggregates");
    double gA = 1.0, gB = 0.0, gS = 0.0;
    if (lane < w) {
        gA = lget(S.agA[lane]);
        gB = lget(S.agB[lane]);
        gS = lget(S.agS[lane]);
    }
    aff_step<0x111, 0xf>(gA, gB, gS);
    aff_step<0x112, 0xf>(gA, gB, gS);
    aff_step<0x114, 0xf>(gA, gB, gS);
    aff_step<0x118, 0xf>(gA, gB, gS);
    double pb = 0.0, ps = 0.0;
    if (w > 0) {
        pb = __shfl(gB, w - 1, 64);
        ps = __shfl(gS, w - 1, 64);
    }
    dm = ea * pb + eb;
    ds = ps + es;
}

// initial guesses (all threads): running mean / variance sum in double from the pass-0 block sums
// gd: the double running mean at the block start; dr: the float trajectory's offset from it at the
// previous call (PC_DRIFT), 0 without one
template <int NL>
__device__ void pcw_guess(PcShared<NL> &S, const PcMap &m, double &gd, float dr = 0.0f) {
    const uint32_t j = threadIdx.x;
    double dm, ds;
    pcw_scan<NL>(S, 1.0, S.s1(j), S.s2(j), dm, ds);   // exclusive sums of s1 (dm) and s2 (ds)
    const double K = (double)(pc_k0(m, j) - 1u);
    float g = 0.0f, gs = 0.0f;
    gd = 0.0;
    if (K > 0.0) {
        gd = 1.0 + dm / K;
        g = (float)(gd + (double)dr);
        const double v = ds - dm * (dm / K);
        gs = (float)(v > 0.0 ? v : 0.0);
    }
    lset(S.b[j].gmu, g);
    lset(S.b[j].gsig, gs);
}

// Check and update after a round (all threads).  S.done = req when every block end matched (S.mu /
// S.sig hold the result); at the round cap (cap_fallback) S.fallback = req and S.first_bad = the
// first failing transition; else the next guesses.  Ends with the caller's barrier.
template <int NL>
__device__ void pcw_update(PcShared<NL> &S, const PcMap &m, int round, int req, bool at_cap,
                           bool cap_fallback, bool use_sig = true) {
    const int j = threadIdx.x, lane = j & 63, w = j >> 6;
    const int nbe = m.L ? NL : (int)m.rem;
    double a = 1.0, bm = 0.0, bs = 0.0;
    float em = 0.0f, es = 0.0f;
    bool mm = false;
    if (j < nbe - 1) {
        const PcBlk B = lget(S.b[j]);
        const float gn = lget(S.b[j + 1].gmu), gsn = lget(S.b[j + 1].gsig);
        em = B.emu;
        es = B.esig;
        mm = __float_as_uint(B.emu) != __float_as_uint(gn) ||
             (use_sig && __float_as_uint(B.esig) != __float_as_uint(gsn));
        bm = (double)B.emu - (double)gn;
        bs = use_sig ? (double)B.esig - (double)gsn : 0.0;
        const uint32_t k0 = pc_k0(m, j), k1 = k0 + pc_len(m, j) - 1u;
        // model slopes (deterministic float arithmetic; they only steer the guesses)
        float af = (float)(k0 - 1u) * __builtin_amdgcn_rcpf((float)k1);
        if (round > 0 && B.gmu != B.gmu_o) {
            const float sl = (B.emu - B.emu_o) * __builtin_amdgcn_rcpf(B.gmu - B.gmu_o);
            if (sl >= 0.0f && sl <= 1.0f) af = sl;
        }
        a = (double)af;
        lset(S.b[j].gmu_o, B.gmu);
        lset(S.b[j].emu_o, B.emu);
    }
    const uint64_t bal = __ballot(mm);
    if (lane == 0) lset(S.agFirst[w], bal ? w * 64 + __ffsll((unsigned long long)bal) - 1 : NL);
    double dm, ds;
    pcw_scan<NL>(S, a, bm, bs, dm, ds);   // its barrier also publishes agFirst
    int first = NL;
    for (int v = 0; v < NL / 64; ++v) first = min(first, lget(S.agFirst[v]));
    if (first == NL) {
        if (j == 0) {
            S.mu = S.b[nbe - 1].emu;
            S.sig = S.b[nbe - 1].esig;
            S.rounds = round + 1;
            S.done = req;
        }
        return;
    }
    if (at_cap) {
        if (j == 0 && cap_fallback) {
            S.first_bad = first;
            S.rounds = round + 1;
            S.fallback = req;
        }
        return;
    }
    if (j < nbe - 1) {
        lset(S.b[j + 1].gmu, dm == 0.0 ? em : (float)((double)em + a * dm));
        if (use_sig) lset(S.b[j + 1].gsig, ds == 0.0 ? es : (float)((double)es + ds));
    }
}

// ---- exact sig after stage 0 ("PCX") --------------------------------------------------------------
// Once stage 0 has made every block's mu start exact, sig needs no rounds: with mu exact, every
// step's increment t_k = RN(RN(sqr(p - mu) (N - 1)) / N) is a known double, and sig is the float
// accumulation sig <- (float)(sig + t_k), non-decreasing.  Inside one binade [2^e, 2^(e+1)) that
// accumulation is an integer sum: sig + t rounds first to the double grid 2^(e-52) and then to the
// float grid 2^(e-23), both anchored on sig's own grid, so a step adds
//   c_k(e) = RN(RN(t 2^(52-e)) / 2^29)    whole float ulps (ties to even: a remainder of exactly
// 2^28 depends on sig's last bit -- flagged), independent of sig as long as sig + t stays below
// 2^(e+1).  So:
//   estimate (all threads): sig at every block start from the prefix over the blocks of
//     sum (p - mu)^2 along stage 0's last trajectories (within ~1e-4 of the float sig; the pass-0
//     variance guess misses the float mean's drift, up to a factor 2.2);
//   T pass (all threads): each block runs its steps from its stage-0 start with the exact mu step
//     (verifying stage 0: its end must be the next block's start) and forms t_k.  A block whose
//     estimated start and end lie in one binade e sums c_k(e); a block whose estimate crosses a
//     binade (with a 2^-10 margin), block 0 and the last block store their t_k in tbuf instead;
//   scan (one wave): from sig = 0, runs of blocks that stay in the current binade are integer prefix
//     sums (64 blocks per step, DPP scan); a crossing block is walked from its exact start over its
//     stored t_k, again as integer prefix sums in the current binade up to the step that crosses or
//     holds a tie, which is evaluated exactly as one float step.
// Every step is the spec's step evaluated exactly, so the result is the serial recurrence bit for bit
// (no verification round needed).  A block the estimate misplaced is walked by recomputing its mu
// trajectory (systolic); stage 0 not verified falls back to the stage-1 / exact rounds below.
// scripts/dev/pc_sim2.c (GPX=1) emulates this on oracle d sequences: ~20 walks per iteration, all
// predicted, every result exact.
struct PcX {                 // overlays (gmu_o, emu_o, sp0, sp1) once stage 0 is over
    int32_t c;               // sum of c_k(e) over the block (saturated at 2^30)
    int32_t e;               // binade of the block's estimated start (-200: none)
    int32_t flags;           // bit 0: tie inside; bit 1: candidate (t_k stored)
    int32_t slot;            // tbuf slot of a candidate, -1 when none
};
#define PCX_TIEF 1
#define PCX_CANDF 2
template <int NL>
__device__ __forceinline__ PcX &pcx_of(PcShared<NL> &S, int j) {
    return *reinterpret_cast<PcX *>(&S.b[j].gmu_o);
}
// binade e of a positive normal float (2^e <= f < 2^(e+1)); -200 for 0, subnormals, inf / NaN
__device__ __forceinline__ int pcx_binade(float f) {
    const int be = (__float_as_int(f) >> 23) & 0xff;
    return (f > 0.0f && be > 0 && be < 255) ? be - 127 : -200;
}
// c(e) of one increment: t 2^(52 - e) rounded to an integer (the double grid), then to whole floats
// (2^29 double ulps, ties flagged)
__device__ __forceinline__ double pcx_c(double t, int e, bool &tie) {
    const double Y = rint(ldexp(t, 52 - e));
    const double hi = floor(Y * 0x1p-29);
    const double rem = fma(-hi, 0x1p29, Y);
    tie = rem == 0x1p28;
    return hi + (rem > 0x1p28 ? 1.0 : 0.0);
}
// inclusive prefix sum over the wave's 64 lanes (int32), DPP row shifts and row broadcasts (gfx9)
__device__ __forceinline__ int pcx_iscan(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);   // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);   // row_bcast:31 -> rows 2, 3
    return v;
}

// T pass: this thread's block from its stage-0 start (S.b[j].gmu) with exact steps; sest / snext =
// the sig estimate at its start / end
template <int NL>
__device__ void pcx_tpass(PcShared<NL> &S, const PcMap &m, const float *P, uint32_t j, uint32_t len,
                          uint32_t k0, double sest, double snext, double *tbuf, int tcap) {
    const int nbe = m.L ? NL : (int)m.rem;
    const int e = pcx_binade((float)sest);
    const bool cand = (int)j == 0 || (int)j >= nbe - 1 || e < -125 ||
                      e != pcx_binade((float)(snext * (1.0 + 0x1p-10))) ||
                      e != pcx_binade((float)(sest * (1.0 - 0x1p-10)));
    int slot = -1;
    if (cand && (int)j < nbe) {
        const int sl = atomicAdd(&S.xslots, 1);
        if ((sl + 1) * (int)(m.L + 1) <= tcap) slot = sl;
    }
    double C = 0.0;
    bool tie = false;
    float mu = S.b[j].gmu;
    double kd = (double)k0;
    double *const tb = tbuf + (size_t)(slot >= 0 ? slot : 0) * (m.L + 1);
    for (uint32_t s0 = 0; s0 < len; s0 += 8) {
        float pv[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) pv[i] = P[(size_t)(s0 + i < len ? s0 + i : len - 1u) * NL + j];   // (clamped: unused past len)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (s0 + i >= len) break;
            const PcK q = pc_consts(kd, pv[i]);
            double t = 0.0;
            if (kd != 1.0) {
                const float d = pv[i] - mu;
                t = pc_div((double)(d * d) * (q.N - 1.0), q.N, q.r);
            }
            if (slot >= 0) {
                tb[s0 + i] = t;
            } else if (!cand) {
                bool ti;
                C += pcx_c(t, e, ti);
                tie |= ti;
            }
            mu = (float)__dadd_rn(__dmul_rn((double)mu, q.A), q.B);
            kd += 1.0;
        }
    }
    S.b[j].emu = mu;
    PcX &x = pcx_of(S, j);
    x.c = (int32_t)fmin(C, 1073741824.0);
    x.e = e;
    x.flags = (tie ? PCX_TIEF : 0) | (cand ? PCX_CANDF : 0);
    x.slot = slot;
}

// Walk block j from its exact start s over its stored increments t (tb[0 .. len)): per 64-step piece,
// integer prefix sums in the current binade up to the first step that crosses (or comes within an ulp
// of) the binade's end or holds a tie; that step is one exact float step; repeat.
// t0 / t1: the first two pieces, loaded ahead by the caller (global latency off the serial path)
__device__ float pcx_walk_t(const double *tb, uint32_t len, float s, double t0, double t1) {
    const int lane = threadIdx.x & 63;
    for (uint32_t s0 = 0; s0 < len; s0 += 64) {
        const bool in = s0 + lane < len;
        const double t = !in ? 0.0 : s0 == 0 ? t0 : s0 == 64 ? t1 : tb[s0 + lane];
        int from = 0;   // lanes below are done
        while (from < 64) {
            const int e = pcx_binade(s);
            bool tie = false;
            double c = 0.0;
            if (e >= -125 && in && lane >= from) c = pcx_c(t, e, tie);
            const bool big = c >= 0x1p23;   // one step past a whole binade: crosses
            const int pre = pcx_iscan((in && lane >= from && !big) ? (int)c : 0);
            const double ulp = ldexp(1.0, e - 23), lim = ldexp(1.0, e + 1) - ulp;
            const double val = (double)s + (double)pre * ulp;
            const bool bad = in && lane >= from && (e < -125 || tie || big || !(val < lim));
            const uint64_t bb = __ballot(bad);
            if (!bb) {   // the rest of the piece stays in the binade
                s = (float)__shfl(val, 63, 64);
                break;
            }
            const int f = (int)__builtin_ctzll(bb);   // exact step f from the value before it
            const double before = f > from ? __shfl(val, f - 1, 64) : (double)s;
            const double tf = __shfl(t, f, 64);
            s = (float)((double)(float)before + tf);
            from = f + 1;
        }
    }
    return s;
}

// Walk block j exactly without stored increments (a block the estimate did not flag): the wave
// recomputes the block's mu trajectory (systolic) and t_k, then the sig steps (systolic)
template <int NL>
__device__ float pcx_walk_mu(const PcShared<NL> &S, const PcMap &m, const float *P, int j, float s) {
    const int lane = threadIdx.x & 63;
    const uint32_t len = pc_len(m, (uint32_t)j), k0 = pc_k0(m, (uint32_t)j);
    float mu = S.b[j].gmu;
    for (uint32_t s0 = 0; s0 < len; s0 += 64) {
        const bool in = s0 + lane < len;
        const float p = in ? P[(size_t)(s0 + lane) * NL + j] : 1.0f;
        const double kd = (double)(k0 + s0 + lane);
        const PcK q = pc_consts(kd, p);
        float mprev;   // mu before this lane's step
        mu = chain_sys64<true>(in ? q.A : 1.0, in ? q.B : 0.0, mu, mprev);
        double t = 0.0;
        if (in && kd != 1.0) {
            const float d = p - mprev;
            t = pc_div((double)(d * d) * (q.N - 1.0), q.N, q.r);
        }
        float rec;
        s = chain_sys64<false>(in ? 1.0 : 0.0, t, s, rec);
    }
    return s;
}

// The scan (wave 0).  Returns false when stage 0 is not verified (the caller falls back).
template <int NL>
__device__ bool pcx_scan(PcShared<NL> &S, const PcMap &m, const float *P, const double *tbuf, float &sig_out,
                         int &walks, int &slow) {
    const int lane = threadIdx.x & 63;
    const int nbe = m.L ? NL : (int)m.rem;
    bool bad = false;   // stage 0 verified: every block's exact end is its successor's start
    for (int j = lane; j < nbe - 1; j += 64)
        bad |= __float_as_uint(S.b[j].emu) != __float_as_uint(S.b[j + 1].gmu);
    if (__ballot(bad)) return false;
    float s = 0.0f;   // exact sig at the start of block j
    int j = 0;
    walks = slow = 0;
    // the next candidate block at or after `from` and its first two pieces of t, loaded ahead
    int nxt = -1;
    double pf0 = 0.0, pf1 = 0.0;
    auto prefetch = [&](int from) {
        nxt = nbe;
        for (int c0 = from; c0 < nbe; c0 += 64) {
            const bool cnd = c0 + lane < nbe && (pcx_of(S, c0 + lane).flags & PCX_CANDF);
            const uint64_t bl = __ballot(cnd);
            if (bl) {
                nxt = c0 + (int)__builtin_ctzll(bl);
                break;
            }
        }
        if (nxt < nbe) {
            const PcX x = pcx_of(S, nxt);
            const uint32_t len = pc_len(m, (uint32_t)nxt);
            const double *tb = tbuf + (size_t)(x.slot >= 0 ? x.slot : 0) * (m.L + 1);
            pf0 = (x.slot >= 0 && (uint32_t)lane < len) ? tb[lane] : 0.0;
            pf1 = (x.slot >= 0 && (uint32_t)lane + 64 < len) ? tb[lane + 64] : 0.0;
        }
    };
    prefetch(0);
    while (j < nbe) {
        const int jj = j + lane;
        const bool have = jj < nbe;
        const int e = pcx_binade(s);   // wave-uniform
        bool ok = false;
        int inc = 0;
        if (have && e >= -125) {
            const PcX x = pcx_of(S, jj);
            ok = x.flags == 0 && x.e == e && x.c < (1 << 23);
            inc = ok ? x.c : 0;
        }
        const int pre = pcx_iscan(inc);
        const double ulp = ldexp(1.0, e - 23), lim = ldexp(1.0, e + 1) - ulp;
        const double end = (double)s + (double)pre * ulp;
        ok = ok && end < lim;
        const uint64_t fail = ~__ballot(ok || !have);
        const int first = fail ? (int)__builtin_ctzll(fail) : 64;   // first block that cannot be summed
        if (first > 0) {   // blocks j .. j + first - 1 stay in the binade: exact integer sums
            const int last = min(first, nbe - j) - 1;
            s = (float)__shfl(end, last, 64);
            j += last + 1;
            continue;
        }
        const PcX x = pcx_of(S, j);   // block j: walked exactly
#ifdef PC_PROF
        const unsigned long long cw0 = clock64();
#endif
        if ((x.flags & PCX_CANDF) && x.slot >= 0) {
            const double a0 = j == nxt ? pf0 : 0.0, a1 = j == nxt ? pf1 : 0.0;
            const bool mine = j == nxt;
            if (mine) prefetch(j + 1);   // the next candidate's loads fly during this walk
            const double *tb = tbuf + (size_t)x.slot * (m.L + 1);
            const uint32_t len = pc_len(m, (uint32_t)j);
            s = mine ? pcx_walk_t(tb, len, s, a0, a1)
                     : pcx_walk_t(tb, len, s, (uint32_t)lane < len ? tb[lane] : 0.0,
                                  (uint32_t)lane + 64 < len ? tb[lane + 64] : 0.0);
        } else {
            s = pcx_walk_mu<NL>(S, m, P, j, s);
            ++slow;
        }
#ifdef PC_PROF
        if (lane == 0) S.xwcyc += clock64() - cw0;
#endif
        ++walks;
        ++j;
    }
    sig_out = s;
    return true;
}

#define PC_TPB 1024
// The recurrence of one iteration on a whole NL-thread workgroup (one block per thread), shared by
// the study kernel (ST_PC 2) and the sweep driver (k_n4_pcw).  ld(r) returns d at raster rank r
// (the study's raster-ordered stores, or the sweep's compact d through the raster permutation);
// pass 0 reads each block's run of it, writes
// p = exp(d) into P in block layout (one wave-wide load per step afterwards) and the block sums;
// then phase A (certified float rounds) and phase B (exact rounds, the verification); after
// PC_RMAX exact rounds the rest runs serially from the first failing block.  ch.conv = result.
#ifndef PC_APASS
#define PC_APASS 2   // phase-A stages; 1 = mu alone, then straight to the exact rounds (measured 7.56k
                     // against 8.02k vol/s: sig then takes several of the dearer exact rounds)
#endif
// the done / fallback tags are 4 req + stage: phase-A stages 0 .. PC_APASS - 1, phase B 2
static_assert(PC_APASS >= 1 && PC_APASS <= 2, "PC_APASS: 1 or 2 phase-A stages (tag 2 is phase B's)");
#ifndef PC_AMAX
#define PC_AMAX 40
#endif
#ifndef PC_XSIG
#define PC_XSIG 1   // exact sig after stage 0 (PCX above); 0: stage 1 and the exact rounds always
#endif
// PEXP: ld returns p = expf_cr(d) already (the study kernel's eval stored it, ST_EVAL_EXP)
// pass 0's transpose groups: PC_G0 steps of every block per two barriers (LDS: PC_G0 (NL + 8) floats
// over the PcShared area, so the area is the larger of the two)
#ifndef PC_G0
#define PC_G0 8
#endif
#ifndef PC_EXPS
#define PC_EXPS 1   // pass 0's exp by expf_crs (the same floats; r4ax: 18.62 -> 18.44 ms per isolated launch)
#endif
#ifndef PC_S12F
#define PC_S12F 1   // the guesses' block sums in float (r4ar: 18.87 vs 18.93 ms per isolated launch)
#endif
#ifndef PC_PRE
#define PC_PRE 1    // early certified decision from the exact running mean (pcw_run, round 5)
#endif
#ifndef PC_P0CLAMP
#define PC_P0CLAMP 1   // pass 0's loads unconditional at clamped indices (round 6)
#endif
#ifndef PC_INLINE
#define PC_INLINE 0    // 1: pcw_run inlined (LDS through ds_* instead of flat; A/B builds)
#endif
template <int NL>
__host__ __device__ constexpr size_t pcw_lds_bytes() {
    return sizeof(PcShared<NL>) > sizeof(float) * PC_G0 * (NL + 8) ? sizeof(PcShared<NL>)
                                                                    : sizeof(float) * PC_G0 * (NL + 8);
}
#if PC_INLINE
#define PCW_INL __forceinline__
#else
#define PCW_INL __attribute__((noinline))
#endif
template <int NL, bool PEXP = false, class LoadD>
__device__ PCW_INL void pcw_run(LoadD ld, float *P, int64_t n, PcShared<NL> &S,
                                                  ChainState &ch, int req, double *tbuf, int tcap,
                                                  float skip_thresh = 0.0f, float *drift = nullptr,
                                                  bool drift_in = false, bool try_pre = false) {
    const int tid = threadIdx.x;
    const PcMap m = pc_map(n, NL);
    const uint32_t j = (uint32_t)tid, len = pc_len(m, j), k0 = pc_k0(m, j);
    // the previous call's offsets of the exact block starts from the double running mean (the float
    // mean's drift changes little from one iteration to the next): added to this call's guesses
    const float dr = drift && drift_in ? drift[j] : 0.0f;
#ifdef PC_PROF
    const unsigned long long c0 = clock64();
    unsigned long long c1 = 0, c2 = 0;
    int ra = 0;
#endif
    // pass 0: p = exp(d) from raster order into block layout (P[s NL + j]) and the block sums.  A
    // block's d values are consecutive in raster order, so one thread reading its own block touched
    // 64 cache lines per wave-wide load; instead the workgroup loads each group of PC_G0 steps of
    // all blocks together (8 lanes per block: 32-byte runs) and transposes it through LDS (the
    // PcShared area, rewritten after this pass; rows padded by 8 floats against bank conflicts).
    constexpr int G0 = PC_G0, TS = NL + 8;
    static_assert(sizeof(float) * G0 * TS <= pcw_lds_bytes<NL>(), "pass-0 transpose buffer");
    float *const T0 = reinterpret_cast<float *>(&S);
    const uint32_t lmax = m.L + (m.rem ? 1u : 0u);
    // s1 = sum of (p - 1) in double: exact wherever the early decision uses it (it requires every p
    // in (0.5, 1.9): then p - 1 is a multiple of 2^-24 with |p - 1| < 0.9, so it and every partial
    // sum of n < 2^24 of them are integers times 2^-24 below 2^24 in size -- at most 48 significant
    // bits, within a double's 53, so any order of the sums is exact); s2 seeds the guesses
    double s1 = 0.0;
#if PC_S12F   // the guesses' block sums: they only seed the rounds (the result is exact either way)
    float s2 = 0.0f;
#else
    double s2 = 0.0;
#endif
    // certified-frozen start intervals: the block's p range; the bound N h is taken at the block's
    // first step, where N is smallest (N = min(k, NMAX) never decreases), so [max p - N0 h,
    // min p + N0 h] lies inside every step's [p - N h, p + N h] -- the intersection the
    // certification needs, at 2 float ops per step instead of 10 double ones
    float pmax = -__int_as_float(0x7f800000), pmin = __int_as_float(0x7f800000);
    // thread tid loads step i = tid % G0 of blocks tid / G0 + (NL / G0) q; the next group's
    // loads are in flight while this group's exp runs
    float v[G0];
    auto fetch = [&](uint32_t g0) {
#if PC_P0CLAMP
        // unconditional loads at a clamped index, the select after them (round 6): the guarded form
        // `in ? ld(...) : 0` compiled to an exec-masked branch per load whose s_waitcnt vmcnt(0)
        // waited for each load before the next issued -- the group's 8 loads one round trip at a
        // time (scripts/dev/isa_serial_loads.py)
#pragma unroll
        for (int q = 0; q < G0; ++q) {   // (the value of a step past the block's end: never read)
            const uint32_t jb = (uint32_t)tid / G0 + (uint32_t)(NL / G0) * q, i = (uint32_t)tid % G0;
            const uint32_t lb = pc_len(m, jb), ii = g0 + i;
            const int64_t r = lb ? (int64_t)(pc_k0(m, jb) - 1u + (ii < lb ? ii : lb - 1u)) : 0;
            v[q] = ld(r < n ? r : (n > 0 ? n - 1 : 0));
        }
#else
#pragma unroll
        for (int q = 0; q < G0; ++q) {
            const uint32_t jb = (uint32_t)tid / G0 + (uint32_t)(NL / G0) * q, i = (uint32_t)tid % G0;
            v[q] = g0 + i < pc_len(m, jb) ? ld((int64_t)(pc_k0(m, jb) - 1u + g0 + i)) : 0.0f;
        }
#endif
    };
    // (n == 0: no load at all -- the clamped index 0 would read a permutation entry of an empty
    // study, r6y's illegal address)
    if (lmax) fetch(0);
#ifdef PC_PROF
    unsigned long long p0t[4] = {0, 0, 0, 0}, p0c = clock64();
#define P0M(k) do { const unsigned long long _c = clock64(); p0t[k] += _c - p0c; p0c = _c; } while (0)
#else
#define P0M(k) do { } while (0)
#endif
    for (uint32_t g0 = 0; g0 < lmax; g0 += G0) {
#pragma unroll
        for (int q = 0; q < G0; ++q)
            lds_st(T0 + (tid % G0) * TS + tid / G0 + (NL / G0) * q, v[q]);
        P0M(0);   // (profiling) the group's loads arrived and went to LDS
        __syncthreads();
        P0M(1);   // first barrier
        if (g0 + G0 < lmax) fetch(g0 + G0);
        float tv[G0];   // this group's steps of this thread's block, from LDS (ds_read: lgkmcnt only)
#pragma unroll
        for (int i = 0; i < G0; ++i) tv[i] = lds_ld(T0 + i * TS + j);
#pragma unroll
        for (int i = 0; i < G0; ++i)
            if (g0 + i < len) {
#ifdef AB_P0_FASTEXP   // A/B probe only (results not the spec's): pass 0 without the double exp
                const float p = PEXP ? tv[i] : __expf(tv[i]);
#else
                const float p = PEXP ? tv[i] : PC_EXPS ? expf_crs(tv[i]) : expf_cr(tv[i]);
#endif
                P[(size_t)(g0 + i) * NL + j] = p;
                s1 += (double)p - 1.0;
#if PC_S12F
                const float e = p - 1.0f;
                s2 = fmaf(e, e, s2);
#else
                const double e = (double)p - 1.0;
                s2 = fma(e, e, s2);
#endif
                pmax = fmaxf(pmax, p);
                pmin = fminf(pmin, p);
            }
        P0M(2);   // exp, stores and sums
        __syncthreads();
        P0M(3);   // second barrier
    }
#undef P0M
#ifdef PC_PROF
    if (blockIdx.x == 0 && tid == 0)
        printf("PCW_P0 loads %llu bar1 %llu work %llu bar2 %llu\n", p0t[0], p0t[1], p0t[2], p0t[3]);
#endif
    if (tid == 0) {   // flags from an earlier call (or other phases' use of this LDS) must not match
        S.done = 0;
        S.fallback = 0;
        S.xdone = 0;
        S.nfrz = 0;
        S.nfr = 0;
        S.xslots = 0;   // (the early decision's max p before PCX takes the field over)
    }
#ifdef PC_PROF
    if (tid < 32) S.pchg[tid] = S.pwav[tid] = 0;
#endif
    S.s1(j) = (double)s1;
    S.s2(j) = (double)s2;
    {   // empty intervals (lo = +inf) before PC_FRZ_K0 or where the block's p spread is too wide
        const bool ok = k0 >= PC_FRZ_K0 && len > 0u;
        const double nd = itk_Nd((double)k0), nh1 = nd * PC_FRZ_H1, nh2 = nd * PC_FRZ_H2;
        const double fa1 = (double)pmax - nh1, fb1 = (double)pmin + nh1;
        const double fa2 = (double)pmax - nh2, fb2 = (double)pmin + nh2;
        const float inf = __int_as_float(0x7f800000);
        S.fz[j] = make_float4(ok && fa1 <= fb1 ? f_up(fa1) : inf, ok && fa1 <= fb1 ? f_dn(fb1) : -inf,
                              ok && fa2 <= fb2 ? f_up(fa2) : inf, ok && fa2 <= fb2 ? f_dn(fb2) : -inf);
    }
    __syncthreads();
    bool pre = false;   // decided from the exact running mean: no rounds at all (below)
#if PC_PRE
    if (try_pre && skip_thresh > 0.0f && n > 1 && n < ((int64_t)1 << 24)) {
        // Early certified decision (round 5).  The float mean's distance from the exact running mean
        // m_k is bounded without running the recurrence: a step's rounding errors (float division p/N,
        // the double products, the final float rounding) are at most 2^-24 (|mu_k| + |p_k| / k)(1 +
        // 2^-26), and the recurrence damps older errors by (1 - 1/k), so |mu_k - m_k| <= sum_i
        // |delta_i| i / k <= D_k = 2^-25 M (k + 3)(1 + 2^-20) with M >= |mu_i|, |p_i| for every i
        // (below; every p in (0.5, 1.9), which also keeps the sums of p - 1 exact).  Then |q_k| >= (|p_k - m_(k-1)| - D_(k-1))(1 - 2^-24), and
        // with the bounds of the certified decision below (t_k >= q^2 (1 - 1/N)(1 - 2^-24)(1 -
        // 2^-52)^2, S >= (1 - 2^-24)^n sum t_k) lo = sum over blocks of (1 - 1/max(k0, 2)) sum_k
        // max(0, |p_k - m_(k-1)| - D_(k-1) - eps_k)^2 (1 - 2^-24)^(n + 8) bounds ITK's float sig
        // from below, and mu_n <= m_n + D_n.  ITK's measure is monotone in both, so a measure above
        // the threshold at (RD(lo), RU(m_n + D_n)) proves the iteration goes on.  It decides the
        // iterations whose measure is well above the threshold (about a quarter on the bench
        // studies), without a single round; the caller tries it only where the previous measure
        // was (try_pre).  m_(k-1) = 1 + P_(k-1) / (k - 1) from the exact prefix P of (p - 1), the
        // quotient by a float reciprocal: eps_k = |m - 1| 2^-21 + 2^-50 covers its error.
        double dmx, nbad;
        const bool okb = len == 0u || (pmax < 1.9f && pmin > 0.5f);
        if (len > 0u) atomicMax(&S.xslots, __float_as_int(pmax));   // positive floats order as ints
        pcw_scan<NL>(S, 1.0, S.s1(j), okb ? 0.0 : 1.0, dmx, nbad);   // exact prefix of (p - 1); its
        // barrier also completes the max: M = max p (the exact mean and, within D, the float mean
        // never exceed it)
        // (|mu_i| <= max p + D_i: M = max p / (1 - 2^-25 (n + 3)(1 + 2^-20)) <= max p (1 + 2^-24 (n + 3)))
        const double Mx = (double)__int_as_float(S.xslots) * (1.0 + 0x1p-24 * ((double)n + 3.0)) * (1.0 + 0x1p-20);
        double Pk = dmx, acc = 0.0;
        const double cD = 0x1p-25 * Mx * (1.0 + 0x1p-20);   // D_k = cD (k + 3)
        for (uint32_t s0 = 0; s0 < len; s0 += 8) {   // 8 loads in flight (unconditional, clamped)
            float pv[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) pv[q] = P[(size_t)(s0 + q < len ? s0 + q : len - 1u) * NL + j];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const uint32_t k = k0 + s0 + (uint32_t)q;   // 1-based step index of this value
                const double p = (double)pv[q];
                const bool in = s0 + (uint32_t)q < len;
                if (in && k >= 2u) {
                    const double r = (double)__frcp_rn((float)(k - 1u));
                    const double mk = fma(Pk, r, 1.0);
                    const double eps = fabs(mk - 1.0) * 0x1p-21 + 0x1p-50;
                    const double a = fabs(p - mk) - cD * (double)(k + 2u) - eps;
                    acc = a > 0.0 ? fma(a, a, acc) : acc;
                }
                Pk += in ? p - 1.0 : 0.0;
            }
        }
        const double wown = acc * (1.0 - 1.0 / fmax((double)k0, 2.0));
        double wpre, unused;
        // the first scan's wave aggregates may still be being read by a slower wave (pcw_scan ends
        // without a barrier): the second scan's lane-63 stores must wait for every wave
        __syncthreads();
        pcw_scan<NL>(S, 1.0, wown, 0.0, wpre, unused);
        if (tid == NL - 1) {
            const double f = pc_accum_factor((double)n + 8.0);
            const double lo = (wpre + wown) * f;
            const bool allok = nbad + (okb ? 0.0 : 1.0) == 0.0;   // every block's p in (0.5, 1.9)
            float sl = (float)lo;
            if ((double)sl > lo && sl > 0.0f) sl = __uint_as_float(__float_as_uint(sl) - 1u);
            const double Pn = dmx + s1;                     // exact sum of (p - 1) over all n steps
            const double mn = 1.0 + Pn / (double)n;         // m_n (one double division)
            const float muh = f_up(mn + cD * ((double)n + 3.0) + fabs(mn - 1.0) * 0x1p-50 + 0x1p-50);
            if (allok && lo > 0.0 && itk_conv(muh, sl, n) > skip_thresh) {
                S.mu = muh;
                S.sig = sl;
                S.rounds = 0;
                S.xdone = 4 * req + 1;
            }
        }
        __syncthreads();
        pre = S.xdone == 4 * req + 1;
    }
#endif
    double gd = 0.0;
    if (!pre) pcw_guess<NL>(S, m, gd, dr);
    __syncthreads();
#ifdef PC_PROF
    c1 = clock64();
#endif
    int round = 0;
    // phase A: certified float rounds to their fixed point, first on mu alone (mu never reads sig:
    // a third fewer instructions per step), then on both.  A thread whose start did not change
    // keeps its end; a wave whose threads all kept theirs skips the round.
#ifdef PC_PROF
    unsigned long long cblk = 0, cst[2] = {0, 0}, cbs[2] = {0, 0};
    int rst[2] = {0, 0};
#endif
    bool xs = pre;   // sig finished exactly by PCX (or decided early): no stage 1, no exact rounds
    for (int pass = 0; pass < PC_APASS && !pre; ++pass) {
        if (pass == 1 && PC_XSIG && S.done == 4 * req) {   // stage 0 reached its fixed point
#ifdef PC_PROF
            const unsigned long long cx0 = clock64();
#endif
            const bool real = j < (uint32_t)(m.L ? NL : m.rem);
            const double own = real ? (double)S.b[j].esig : 0.0;   // stage 0's sum (p - mu)^2
            // the same sums weighted by the smallest (N - 1) / N of the block: their total bounds
            // the float sig from below (the certified decision below)
            const double wown = (real && k0 > 1u) ? own * (1.0 - 1.0 / fmin((double)k0, ITK_NMAX)) : 0.0;
            double sest, wpre;   // sig estimate at the block start: the prefix of those sums
            pcw_scan<NL>(S, 1.0, own, wown, sest, wpre);
            // Certified decision (skip_thresh > 0: this iteration's measure is only compared with the
            // threshold, never reported): with mu exact after stage 0, every float sig step is
            // t_k = RN(RN(RN_f(q q) (N - 1)) / N) >= q^2 (1 - 1/N)(1 - 2^-24)(1 - 2^-52)^2, the float
            // accumulation keeps S >= (1 - 2^-24)^n sum t_k, and a block's stage-0 float sum B of
            // fma(q, q, .) over its <= L + 1 steps has sum q^2 >= B (1 - 2^-24)^(L + 1).  So
            // S >= lo = (sum of the weighted B) (1 - 2^-24)^(n + L + 8) (pc_accum_factor), and since ITK's measure
            // sqrt(S / (N - 1)) / mu is monotone in S under round-to-nearest, a measure above the
            // threshold at sig = RD(lo) proves the true one is above it too: the iteration goes on
            // and the exact sig (PCX below) is not needed.  Otherwise, or when the measure is the
            // level's reported one (skip_thresh = 0), PCX computes it exactly.
            if (tid == NL - 1 && skip_thresh > 0.0f) {
                const double f = pc_accum_factor((double)n + (double)m.L + 8.0);
                const double lo = (wpre + wown) * f;
                float sl = (float)lo;
                if ((double)sl > lo && sl > 0.0f) sl = __uint_as_float(__float_as_uint(sl) - 1u);
                const int nbe = m.L ? NL : (int)m.rem;
                const float mue = S.b[nbe - 1].emu;   // (one float up: a margin that costs nothing)
                const float muh = __uint_as_float(__float_as_uint(mue) + 1u);
                if (lo > 0.0 && mue > 0.0f && itk_conv(muh, sl, n) > skip_thresh) {
                    S.mu = mue;
                    S.sig = sl;
                    S.rounds = round + 1;
                    S.xdone = 4 * req + 3;
                }
            }
            if (tid == 0) S.xslots = 0;
            __syncthreads();
            if (S.xdone == 4 * req + 3) {   // decided: no PCX, no exact rounds
                xs = true;
                break;
            }
#ifdef PC_PROF
            const unsigned long long cxt = clock64();
#endif
            pcx_tpass<NL>(S, m, P, j, len, k0, sest, sest + own, tbuf, tcap);
            __syncthreads();
#ifdef PC_PROF
            cbs[1] = clock64() - cxt;   // T pass (reported as stage1 blocks)
#endif
            if (tid < 64) {
#ifdef PC_PROF
                if (tid == 0) S.xwcyc = 0;
                const unsigned long long csc = clock64();
#endif
                float sg = 0.0f;
                int w = 0, slow = 0;
                const bool ok = pcx_scan<NL>(S, m, P, tbuf, sg, w, slow);
                if (tid == 0) {
                    const int nbe = m.L ? NL : (int)m.rem;
                    if (ok) {
                        S.mu = S.b[nbe - 1].emu;
                        S.sig = sg;
                        S.rounds = round + 1;
                        S.xdone = 4 * req + 3;
                    }
                    S.xwalks = ok ? w : -1;
                    S.xslow = slow;
#ifdef PC_PROF
                    S.xscyc = clock64() - csc;
#endif
                }
            }
            __syncthreads();
#ifdef PC_PROF
            cst[1] = clock64() - cx0;
#endif
            if (S.xdone == 4 * req + 3) {
                xs = true;
                break;
            }
        }
#ifdef PC_PROF
        const unsigned long long cs0 = clock64(), cb0 = cblk;
#endif
        // done / fallback flags carry a tag per call and stage (no reset between stages: a wave
        // still reading the flag of the stage before must not see it cleared)
        const int tag = 4 * req + pass;
        float lg = __int_as_float(0x7fc00000), ls = lg, le = 0.0f, les = 0.0f;
        int amax = pass == 0 ? PC_AMAX0 : PC_AMAX;
        bool frz = false;   // stage 0 closed by pc_mu_serial_frozen (one more round to confirm)
        for (int ra0 = 0; ra0 < amax; ++ra0, ++round) {
#ifdef PC_PROF
            const unsigned long long cq = clock64();
#endif
            const float g = lget(S.b[j].gmu), gs = lget(S.b[j].gsig);
            const bool same = __float_as_uint(g) == __float_as_uint(lg) && __float_as_uint(gs) == __float_as_uint(ls);
#ifdef PC_PROF
            if (pass == 0 && ra0 < 32 && (tid & 63) == 0) {
                const uint64_t bq = __ballot(!same);
                atomicAdd(&S.pchg[ra0], __popcll(bq));
                atomicAdd(&S.pwav[ra0], bq != 0ull);
            }
#endif
            if (__ballot(!same) != 0ull && !same) {
                float mu = g, sig = gs;
                if (pass == 0) pc_block_apx<NL, false>(P, j, len, k0, mu, sig, NL, (m.L + 1u) * NL);
                else pc_block_apx<NL, true>(P, j, len, k0, mu, sig, NL, (m.L + 1u) * NL);
                lg = g;
                ls = gs;
                le = mu;
                les = sig;
            }
            lset(S.b[j].emu, le);
            lset(S.b[j].esig, les);
            __syncthreads();
#ifdef PC_PROF
            cblk += clock64() - cq;
#endif
            // stage 0 at its cap also reports its frontier (first_bad) and sets fallback = tag
            pcw_update<NL>(S, m, round, tag, ra0 == amax - 1, pass == 0 && !frz, pass == 1);
            __syncthreads();
#ifdef PC_PROF
            rst[pass]++;
#endif
            if (S.done == tag) break;
            if (pass == 0 && !frz && S.fallback == tag) {
                // the frozen serial from the frontier; when it stops at its budget, its exact starts
                // stay as guesses and stage 1's rounds go on as before
                frz = true;
                if (tid < 64) {
                    const bool all = pc_mu_serial_frozen<NL>(S, m, P);
                    if (tid == 0) {
                        S.nfr = all ? 1 : 0;
                        S.nfrz += all ? 1 : 100;
                    }
                }
                __syncthreads();
                if (S.nfr) amax = ra0 + 2;   // every start past the frontier is exact now
            }
        }
#ifdef PC_PROF
        cst[pass] = clock64() - cs0;
        cbs[pass] = cblk - cb0;
#endif
    }
#ifdef PC_PROF
    ra = round + 1;
    c2 = clock64();
#endif
    // phase B: exact rounds (the verification; usually one)
    const int tagb = 4 * req + 2;
    for (int rb = 0; rb < PC_RMAX && !xs; ++rb) {
        ++round;
        float mu = S.b[j].gmu, sig = S.b[j].gsig;
        pc_block<NL>(P, j, len, k0, mu, sig);
        S.b[j].emu = mu;
        S.b[j].esig = sig;
        __syncthreads();
        pcw_update<NL>(S, m, round, tagb, rb == PC_RMAX - 1, true);
        __syncthreads();
        if (S.done == tagb) break;
        if (S.fallback == tagb) {
            if (tid == 0) pc_serial<NL>(S, m, P);
            __syncthreads();
            break;
        }
    }
    // stage 0 reached its fixed point (xs): the block starts are the exact float trajectory's
    // (a study's first call, which reads no drift, always writes one: 0 when stage 0 stopped short,
    // so a later call never starts from another batch's or an unset value -- ADVICE r4)
    if (drift && !pre && (xs || !drift_in)) drift[j] = xs ? (float)((double)S.b[j].gmu - gd) : 0.0f;
    if (drift && pre && !drift_in) drift[j] = 0.0f;   // (an early decision finds no block starts)
    if (tid == 0) {
        ch.mu = S.mu;
        ch.conv = itk_conv(S.mu, S.sig, n);
#ifdef PC_PROF
        if (blockIdx.x == 0)
            printf("PCW_PROF n %lld roundsA %d roundsB %d fallback %d pass0 %llu A %llu (blocks %llu) B %llu"
                   " | stage0 %d rounds %llu cyc (blocks %llu) stage1 %d rounds %llu cyc (blocks %llu) xsig %d walks %d\n",
                   (long long)n, ra, S.rounds - ra + 0, S.fallback == tagb, c1 - c0, c2 - c1, cblk, clock64() - c2,
                   rst[0], cst[0], cbs[0], rst[1], cst[1], cbs[1], (int)xs, S.xwalks * 1000 + S.xslow);
        if (blockIdx.x == 0)
            for (int r = 0; r < rst[0] && r < 32; ++r) printf("PCW_RND %d chg %d waves %d\n", r, S.pchg[r], S.pwav[r]);
        if (blockIdx.x == 0 && xs) printf("PCW_X scan %llu walks %llu\n", S.xscyc, S.xwcyc);
#endif
    }
}


// wave A: the mu recurrence, block by block as the producers fill them.
template <int NS = CH_SLOTS>
__device__ void chain_wave_mu(int64_t n, ChainSlot *slots, ChainState *cs) {
    const int lane = threadIdx.x & 63;
    const int64_t nblk = (n + 63) / 64;
    unsigned long long wt = 0;
    __builtin_amdgcn_s_setprio(CH_PRIO);   // the serial waves win issue arbitration on their SIMD
    CH_T0();
    float muf = 0.0f;
    for (int64_t blk = 0; blk < nblk; ++blk) {
        ChainSlot &S = slots[blk % NS];
        CH_WAIT(wt, while (lds_load_acq(&S.ready) != (int)(blk + 1)) __builtin_amdgcn_s_sleep(1));
        const double2 q = S.ab[lane];
        float rec;
        muf = chain_sys64<true>(q.x, q.y, muf, rec);
        S.mu[lane] = rec;
        wave_lds_order();
        if (lane == 0) {
            if (blk == nblk - 1) cs->mu = muf;   // published by the release below
            lds_store_rel(&cs->a_done, (int)(blk + 1));
        }
    }
    CH_DONE(0, wt);
    __builtin_amdgcn_s_setprio(0);
}

// wave B.  Returns conv in cs->conv.
template <int NS = CH_SLOTS>
__device__ void chain_wave_sig(int64_t n, ChainSlot *slots, ChainState *cs) {
    const int lane = threadIdx.x & 63;
    float sig = 0.0f;
    const int64_t nblk = (n + 63) / 64;
    unsigned long long wt = 0;
    __builtin_amdgcn_s_setprio(CH_PRIO);
    CH_T0();
    for (int64_t blk = 0; blk < nblk; ++blk) {
        ChainSlot &S = slots[blk % NS];
        const int64_t j = blk * 64 + lane;
        CH_WAIT(wt, while (lds_load_acq(&cs->a_done) <= (int)blk) __builtin_amdgcn_s_sleep(1));
        const float q = S.p[lane] - S.mu[lane];
        const double N = S.nd[lane];
        const double t = ((double)(q * q) * (N - 1.0)) / N;   // IEEE double division
        // k = 1 adds nothing (ITK's N > 1 test), nor do the steps past the end: (0, 0) is a no-op
        const bool ok = j < n && j > 0;
        float rec;
        sig = chain_sys64<false>(ok ? 1.0 : 0.0, ok ? t : 0.0, sig, rec);
        (void)rec;
        wave_lds_order();
        if (lane == 0) lds_store_rel(&cs->b_done, (int)(blk + 1));
    }
    CH_DONE(1, wt);
    __builtin_amdgcn_s_setprio(0);
    if (lane == 0) {
        while (lds_load_acq(&cs->a_done) < (int)nblk) __builtin_amdgcn_s_sleep(1);
        cs->conv = itk_conv(cs->mu, sig, n);
    }
}

// ---- grid PC, one grid barrier per round (round 5) ----------------------------------------------
// k_n4_pcg2: the study kernel's stage structure (pcw_run) over a cooperative grid.
//   stage 0: certified float rounds on mu alone to their fixed point (mu never reads sig), each
//            block also summing (p - mu)^2 along its trajectory;
//   decision: below the level's iteration cap, the measure is only compared with the threshold:
//            with mu exact, the weighted stage-0 sums bound ITK's float sig from below (pcw_run's
//            certified decision), and a bound above the threshold ends the call -- most iterations;
//   stage 1 + phase B: otherwise certified rounds on (mu, sig) from the exact mu starts and the
//            stage-0 prefix as sig guesses, then exact rounds (the verification), as k_n4_pcg.
// One grid barrier per round instead of two: a block's map T_j(x) = a_j x + b_j needs b_j =
// e_j - g_{j+1}, and g_{j+1} of a workgroup's last block lives in the next workgroup.  So each
// workgroup composes its maps with its last block's b left out and publishes, before the barrier,
// that aggregate, its first block's guesses and its last block's ends; after the barrier every
// workgroup adds the boundary terms itself (b = e_last(v) - g_first(v + 1)) while composing the
// aggregates before it, finds the first mismatch (local ones and boundaries) and sets its own blocks'
// next guesses g_j + delta_j -- no second barrier to publish guesses.  The records are double
// buffered by round parity: a workgroup writes round r + 2's record only after every workgroup
// passed barrier r + 1, i.e. finished reading round r's.
struct PcgWg {
    double A, B, S;         // the workgroup's composed maps (last block's b left out) / sig-channel sum
    float gfirst, gsfirst;  // its first block's guesses this round
    float elast, eslast;    // its last block's ends this round
    int F;                  // first local mismatch (global block index), NB when none
    float enbe;             // the end of block nbe - 1 when this workgroup holds it
};
struct Pcg2Args {
    const float *D;
    const int32_t *perm;
    float *P;
    const VolScalars *sc;
    N4State *st;
    int64_t b;
    PcgWg *wg;              // [2][G]
    float *E;               // [2][NB] every block's ends (the serial fallback)
    float skip_thresh;      // > 0: the measure is only compared with it (certified decision allowed)
    // the grid study form: the round records as tagged granules [2][G][PCG_GW] (no grid barrier per
    // round; zeroed before the launch), and the tag base of this call (tags base + scan + 1); null:
    // records through A.wg and a grid barrier (k_n4_pcg2)
    unsigned long long *gran;
    uint32_t tag0;
    int32_t t0;             // k_n4_pcg2: pass 0 through the LDS transpose (pcg2_body's T0)
    unsigned long long *kst;   // profiling: the launch's stamped-timer slot (kst_begin / kst_end), or null
};
// A round record as PCG_GW tagged granules (cdna_hip_programming.md Guideline 16, R2: the data is the
// flag): each 32-bit word of the record in an 8-byte {tag, word} granule written by ONE relaxed
// agent-scope atomic store (sc1) and read by sc1 loads until every tag is the round's.  A workgroup
// publishes round r + 1 only after reading every round-r record, so the parity double buffer is
// never overwritten under a reader (as with the barrier form).
#define PCG_GW 12
__device__ __forceinline__ void pcg_publish(unsigned long long *g, const PcgWg &r, uint32_t tag) {
    const uint64_t a = (uint64_t)__double_as_longlong(r.A), bb = (uint64_t)__double_as_longlong(r.B),
                   s = (uint64_t)__double_as_longlong(r.S);
    const uint32_t v[PCG_GW] = {(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)bb, (uint32_t)(bb >> 32),
                                (uint32_t)s, (uint32_t)(s >> 32), __float_as_uint(r.gfirst),
                                __float_as_uint(r.gsfirst), __float_as_uint(r.elast),
                                __float_as_uint(r.eslast), (uint32_t)r.F, __float_as_uint(r.enbe)};
#pragma unroll
    for (int k = 0; k < PCG_GW; ++k)
        __hip_atomic_store(g + k, ((unsigned long long)tag << 32) | v[k], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
// true when every granule of the record carries the tag; the record in r
__device__ __forceinline__ bool pcg_fetch(const unsigned long long *g, uint32_t tag, PcgWg &r) {
    uint32_t v[PCG_GW];
    bool ok = true;
#pragma unroll
    for (int k = 0; k < PCG_GW; ++k) {
        const unsigned long long x = __hip_atomic_load(g + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok &= (uint32_t)(x >> 32) == tag;
        v[k] = (uint32_t)x;
    }
    r.A = __longlong_as_double((long long)(((uint64_t)v[1] << 32) | v[0]));
    r.B = __longlong_as_double((long long)(((uint64_t)v[3] << 32) | v[2]));
    r.S = __longlong_as_double((long long)(((uint64_t)v[5] << 32) | v[4]));
    r.gfirst = __uint_as_float(v[6]);
    r.gsfirst = __uint_as_float(v[7]);
    r.elast = __uint_as_float(v[8]);
    r.eslast = __uint_as_float(v[9]);
    r.F = (int)v[10];
    r.enbe = __uint_as_float(v[11]);
    return ok;
}
struct Pcg2Lds {
    double wA[PC_TPB / 64], wB[PC_TPB / 64], wS[PC_TPB / 64];
    int wF[PC_TPB / 64];
    float gg[PC_TPB], gsg[PC_TPB];   // this round's guesses of the workgroup's blocks
    float elast, eslast, enbe;
    double pB, pS, tot;     // the workgroups before this one applied to 0; the grid's S total
    float mue;              // the end of the last non-empty block
    int first;
    double xA[PC_TPB / 64], xB[PC_TPB / 64], xS[PC_TPB / 64];   // waves before wave w composed
};
// The round's scan (one grid barrier).  Per thread: the map (a, b) and sig channel bs of its block
// (b, bs of a workgroup's last block are ignored: its boundary terms are added after the barrier),
// its mismatch flag (likewise), its guesses g, gs and ends e, es.  sum_mode: the S channel is a plain
// sum (stage 0: the decision sums), no boundary term.  Out: dm, ds = the exclusive compositions at
// this block applied to 0; first = the grid's first mismatching transition (NB when none).
__device__ void pcg2_scan(const Pcg2Args &A, Pcg2Lds &L, cooperative_groups::grid_group &grid, int parity,
                          int nbe, double a, double b, double bs, bool mm, float g, float gs, float e, float es,
                          bool sum_mode, double &dm, double &ds, int &first, uint32_t tag = 0u) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, G = gridDim.x;
    const int NB = G * PC_TPB;
    const bool last = t == PC_TPB - 1;
    if (t == 0) lset(L.enbe, 0.0f);
    __syncthreads();
    if ((int)(blockIdx.x * PC_TPB + t) == nbe - 1) lset(L.enbe, e);
    if (last) {
        b = 0.0;
        if (!sum_mode) bs = 0.0;
        mm = false;
        lset(L.elast, e);
        lset(L.eslast, es);
    }
    double Aw = a, Bw = b, Sw = bs;
    aff_step<0x111, 0xf>(Aw, Bw, Sw);
    aff_step<0x112, 0xf>(Aw, Bw, Sw);
    aff_step<0x114, 0xf>(Aw, Bw, Sw);
    aff_step<0x118, 0xf>(Aw, Bw, Sw);
    aff_step<0x142, 0xa>(Aw, Bw, Sw);
    aff_step<0x143, 0xc>(Aw, Bw, Sw);
    const uint64_t bal = __ballot(mm);
    if (lane == 63) {
        lset(L.wA[w], Aw);
        lset(L.wB[w], Bw);
        lset(L.wS[w], Sw);
    }
    if (lane == 0) lset(L.wF[w], bal ? (int)(blockIdx.x * PC_TPB + w * 64 + __ffsll((unsigned long long)bal) - 1) : NB);
    const double ea = dpp_d<0x138, 0xf>(Aw, 1.0), eb = dpp_d<0x138, 0xf>(Bw, 0.0), es_ = dpp_d<0x138, 0xf>(Sw, 0.0);
    __syncthreads();
    PcgWg *const rec = A.wg + (size_t)parity * G;
    constexpr int NW = PC_TPB / 64;
    static_assert(NW <= 16, "the wave aggregates in one DPP row");
    if (w == 0) {   // the wave aggregates scanned on lanes 0..NW-1 (one DPP row, 4 steps instead of a
        // 16-step serial loop on thread 0 and up to 15 steps on every thread): lane v holds waves
        // 0..v composed -- the workgroup's aggregate on lane NW-1, wave v+1's prefix on lane v
        double A2 = 1.0, B2 = 0.0, S2 = 0.0;
        int f2 = NB;
        if (lane < NW) {
            A2 = lget(L.wA[lane]);
            B2 = lget(L.wB[lane]);
            S2 = lget(L.wS[lane]);
            f2 = lget(L.wF[lane]);
        }
        aff_step<0x111, 0xf>(A2, B2, S2);   // row_shr:1
        aff_step<0x112, 0xf>(A2, B2, S2);   // row_shr:2
        aff_step<0x114, 0xf>(A2, B2, S2);   // row_shr:4
        aff_step<0x118, 0xf>(A2, B2, S2);   // row_shr:8
        if (lane < NW - 1) {
            lset(L.xA[lane + 1], A2);
            lset(L.xB[lane + 1], B2);
            lset(L.xS[lane + 1], S2);
        }
        if (lane == 0) {
            lset(L.xA[0], 1.0);
            lset(L.xB[0], 0.0);
            lset(L.xS[0], 0.0);
        }
        for (int off = 1; off < NW; off <<= 1) f2 = min(f2, __shfl_xor(f2, off, 64));
        const double At = __shfl(A2, NW - 1, 64), Bt = __shfl(B2, NW - 1, 64), St = __shfl(S2, NW - 1, 64);
        const int f = __shfl(f2, 0, 64);
        if (lane == 0) {
        PcgWg r;
        r.A = At;
        r.B = Bt;
        r.S = St;
        r.F = f;
        r.enbe = lget(L.enbe);
        r.gfirst = g;
        r.gsfirst = gs;
        r.elast = lget(L.elast);
        r.eslast = lget(L.eslast);
        if (A.gran) pcg_publish(A.gran + ((size_t)parity * G + blockIdx.x) * PCG_GW, r, tag);
        else rec[blockIdx.x] = r;
        }
    }
    unsigned long long *const gr = A.gran ? A.gran + (size_t)parity * G * PCG_GW : nullptr;
    if (!A.gran) grid.sync();
    if (w == 0 && gr) {   // wait until every record this lane reads carries the round's tag (bounded:
        // a missing record would be a bug; the rounds' result is then unusable but nothing hangs)
        const int per = (G + 63) / 64;
        for (uint32_t spin = 0;; ++spin) {
            bool ok = true;
            for (int i = 0; i < per; ++i) {
                const int u = per * lane + i;
                PcgWg q;
                if (u < G) ok &= pcg_fetch(gr + (size_t)u * PCG_GW, tag, q);
                if ((u + 1) * PC_TPB < nbe) ok &= pcg_fetch(gr + (size_t)(u + 1) * PCG_GW, tag, q);
            }
            if (__all(ok) || spin > (1u << 24)) break;
            __builtin_amdgcn_s_sleep(1);
        }
    }
    auto recv = [&](int u) {
        PcgWg q;
        if (gr) pcg_fetch(gr + (size_t)u * PCG_GW, tag, q);
        else q = rec[u];
        return q;
    };
    if (w == 0) {   // lane l folds workgroups [per l, per l + per) in order: those before this one
        // into the prefix (with their boundary terms), all of them into the S total and the first
        // mismatch
        double Al = 1.0, Bl = 0.0, Sl = 0.0, Tl = 0.0;
        int f = NB;
        float mue = 0.0f;
        const int per = (G + 63) / 64;
        for (int i = 0; i < per; ++i) {
            const int u = per * lane + i;
            if (u < G) {
                const PcgWg r = recv(u);
                const int jl = (u + 1) * PC_TPB - 1;   // the boundary transition jl -> jl + 1
                double bb = 0.0, bs2 = 0.0;
                if (jl < nbe - 1) {
                    const PcgWg rn = recv(u + 1);
                    bb = (double)r.elast - (double)rn.gfirst;
                    if (!sum_mode) bs2 = (double)r.eslast - (double)rn.gsfirst;
                    const bool bm = __float_as_uint(r.elast) != __float_as_uint(rn.gfirst) ||
                                    (!sum_mode && __float_as_uint(r.eslast) != __float_as_uint(rn.gsfirst));
                    if (bm) f = min(f, jl);
                }
                if (jl >= nbe - 1 && jl - PC_TPB < nbe - 1) mue = r.enbe;   // holds block nbe - 1
                f = min(f, r.F);
                Tl += r.S + bs2;
                if (u < (int)blockIdx.x) {
                    Bl = r.A * Bl + (r.B + bb);
                    Al = Al * r.A;
                    Sl = Sl + (r.S + bs2);
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
        for (int off = 32; off > 0; off >>= 1) Tl += __shfl_down(Tl, off, 64);   // fixed tree
        const uint64_t hm = __ballot(mue != 0.0f);
        const float me = hm ? __shfl(mue, __ffsll((unsigned long long)hm) - 1, 64) : 0.0f;
        if (lane == 63) {
            lset(L.pB, Bl);
            lset(L.pS, Sl);
            lset(L.first, f);
        }
        if (lane == 0) {
            lset(L.tot, Tl);
            lset(L.mue, me);
        }
    }
    __syncthreads();
    // the waves before this one applied to the workgroups before this one (the guesses only steer the
    // rounds: the composed form rounds differently from the serial fold, the result is exact either way)
    const double x = lget(L.xA[w]) * lget(L.pB) + lget(L.xB[w]), xs = lget(L.pS) + lget(L.xS[w]);
    dm = ea * x + eb;
    ds = xs + es_;
    first = lget(L.first);
}

// The grid PC's whole call over the launch's grid (every workgroup of it, PC_TPB threads each):
// pass 0 reads d through ld(raster rank) (k_n4_pcg2: the raster -> compact permutation; the grid
// study kernel: d stored in raster order); the result goes to A.st[A.b].conv_w / conv_bound, written
// by one thread -- the caller's next grid barrier publishes it.
// Pass 0's loads transposed through LDS (T0: PCG_G0 x (PC_TPB + 8) floats, or null): a thread's block
// is ~n / NB consecutive raster steps, so one thread reading its own block made every wave-wide
// load touch 64 lines (config 5: 107 steps per block, two such gathers per step through the
// permutation); instead the workgroup loads each group of PCG_G0 steps of all its blocks together
// (PCG_G0 lanes per block: 32-byte runs) and transposes it through LDS, as pcw_run's pass 0 does.
#define PCG_G0 8
template <class LoadD>
__device__ void pcg2_body(const Pcg2Args &A, Pcg2Lds &L, cooperative_groups::grid_group &grid, LoadD ld,
                          float *T0 = nullptr) {
    const int64_t n = A.sc[A.b].n_mask1;
    const int NB = gridDim.x * PC_TPB;
    const PcMap m = pc_map(n, NB);
    const int t = threadIdx.x;
    const uint32_t j = blockIdx.x * PC_TPB + t, len = pc_len(m, j), k0 = pc_k0(m, j);
    const int nbe = m.L ? NB : (int)m.rem;
    const uint32_t np = (m.L + 1u) * (uint32_t)NB;
    // pass 0: p = exp(d) in block layout, block sums (they seed the mu guesses)
    double s1 = 0.0, s2 = 0.0;
    if (T0) {
        constexpr int G0 = PCG_G0, TS = PC_TPB + 8;
        const uint32_t lmax = m.L + (m.rem ? 1u : 0u);
        float v[G0];
        // thread t loads step t % G0 of the workgroup's blocks t / G0 + (PC_TPB / G0) q, at a clamped
        // index (unconditional: the group's loads stay in flight together)
        auto fetch = [&](uint32_t g0) {
#pragma unroll
            for (int q = 0; q < G0; ++q) {
                const uint32_t jb = blockIdx.x * PC_TPB + (uint32_t)t / G0 + (uint32_t)(PC_TPB / G0) * q;
                const uint32_t lb = pc_len(m, jb), i = g0 + (uint32_t)t % G0;
                const int64_t r = lb ? (int64_t)(pc_k0(m, jb) - 1u + (i < lb ? i : lb - 1u)) : 0;
                v[q] = ld(r < n ? r : (n > 0 ? n - 1 : 0));
            }
        };
        if (lmax) fetch(0);
        for (uint32_t g0 = 0; g0 < lmax; g0 += G0) {
#pragma unroll
            for (int q = 0; q < G0; ++q) T0[(t % G0) * TS + t / G0 + (PC_TPB / G0) * q] = v[q];
            __syncthreads();
            if (g0 + G0 < lmax) fetch(g0 + G0);   // the next group's loads in flight during this one's exp
#pragma unroll
            for (int i = 0; i < G0; ++i)
                if (g0 + i < len) {
                    const float p = expf_crs(T0[i * TS + t]);
                    A.P[(size_t)(g0 + i) * NB + j] = p;
                    const double e = (double)p - 1.0;
                    s1 += e;
                    s2 = fma(e, e, s2);
                }
            __syncthreads();
        }
    }
    for (uint32_t s0 = 0; !T0 && s0 < len; s0 += 8) {
        float v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i)   // clamped, unconditional: the loads stay in flight together
            v[i] = ld((int64_t)(k0 - 1u + (s0 + i < len ? s0 + i : len - 1u)));
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
    int parity = 0, first = NB;
    double dm, ds;
    // the guesses: exclusive sums of s1 (dm) through the same scan in sum mode (no maps: a = 1, b = 0)
    uint32_t nscan = 0;   // the grid form's record tags: A.tag0 + the scan's index (1-based)
    pcg2_scan(A, L, grid, parity, nbe, 1.0, 0.0, s1, false, 0.0f, 0.0f, 0.0f, 0.0f, true, dm, ds, first,
              A.gran ? A.tag0 + (++nscan) : 0u);
    parity ^= 1;
    float g = 0.0f, gs = 0.0f;
    {
        const double K = (double)(k0 - 1u);
        if (K > 0.0) g = (float)(1.0 + ds / K);   // ds = the sum of p - 1 over the steps before the block
    }
    // stage 0: mu alone
    float lg = __int_as_float(0x7fc00000), le = 0.0f, lsum = 0.0f, go = 0.0f, eo = 0.0f;
    bool have_o = false, s0done = false;
    int round = 0;
    for (int r = 0; r < PC_AMAX; ++r, ++round) {
        lset(L.gg[t], g);
        const bool same = __float_as_uint(g) == __float_as_uint(lg);
        if (__ballot(!same) != 0ull && !same) {
            float mu = g, sq = 0.0f;
            pc_block_apx<0, false>(A.P, j, len, k0, mu, sq, (uint32_t)NB, np);
            lg = g;
            le = mu;
            lsum = sq;
        }
        __syncthreads();
        double a = 1.0, bm = 0.0;
        bool mm = false;
        if ((int)j < nbe - 1 && t < PC_TPB - 1) {
            const float gn = lget(L.gg[t + 1]);
            mm = __float_as_uint(le) != __float_as_uint(gn);
            bm = (double)le - (double)gn;
        }
        if ((int)j < nbe - 1) {
            const uint32_t k1 = k0 + len - 1u;
            float af = (float)(k0 - 1u) * __builtin_amdgcn_rcpf((float)k1);
            if (have_o && g != go) {
                const float sl = (le - eo) * __builtin_amdgcn_rcpf(g - go);
                if (sl >= 0.0f && sl <= 1.0f) af = sl;
            }
            a = (double)af;
        }
        go = g;
        eo = le;
        have_o = true;
        // the decision sums: the block's stage-0 sum weighted by the smallest (N - 1) / N of the block
        const double wown = ((int)j < nbe && k0 > 1u) ? (double)lsum * (1.0 - 1.0 / fmin((double)k0, ITK_NMAX)) : 0.0;
        pcg2_scan(A, L, grid, parity, nbe, a, bm, wown, mm, g, 0.0f, le, 0.0f, true, dm, ds, first,
                  A.gran ? A.tag0 + (++nscan) : 0u);
        parity ^= 1;
        if (first == NB) {
            s0done = true;
            break;
        }
        g = dm == 0.0 ? g : (float)((double)g + dm);
    }
    if (s0done && A.skip_thresh > 0.0f) {   // certified decision (pcw_run; uniform over the grid)
        const double f = pc_accum_factor((double)n + (double)m.L + 8.0);
        const double lo = lget(L.tot) * f;
        float sl = (float)lo;
        if ((double)sl > lo && sl > 0.0f) sl = __uint_as_float(__float_as_uint(sl) - 1u);
        const float mue = lget(L.mue);
        const float muh = __uint_as_float(__float_as_uint(mue) + 1u);
        if (lo > 0.0 && mue > 0.0f && itk_conv(muh, sl, n) > A.skip_thresh) {
            if (j == 0) {
                A.st[A.b].conv_w = itk_conv(muh, sl, n);
                A.st[A.b].conv_bound = 1;   // a bound, not ITK's float measure (threshold test only)
            }
#ifdef PCG_PROF
            if (j == 0) printf("PCG2 n %lld G %d L %u stage0 %d decided\n", (long long)n, (int)gridDim.x, m.L, round + 1);
#endif
            return;
        }
    }
    // stage 1 (mu, sig) from the stage-0 guesses (exact mu starts when stage 0 converged) and the
    // prefix of the stage-0 sums as sig guesses, then exact rounds
    gs = (float)(ds > 0.0 ? ds : 0.0);
    if (!s0done) gs = 0.0f;
    float ls = __int_as_float(0x7fc00000), les = 0.0f;
    lg = __int_as_float(0x7fc00000);
    have_o = false;
    bool done = false;
    const int rs1 = round;
    (void)rs1;
    for (int phase = 0; phase < 2 && !done; ++phase) {
        const int cap = phase == 0 ? PC_AMAX : PC_RMAX;
        for (int r = 0; r < cap; ++r, ++round) {
            lset(L.gg[t], g);
            lset(L.gsg[t], gs);
            float mu = g, sig = gs;
            if (phase == 1) {
                pc_block<0>(A.P, j, len, k0, mu, sig, NB);
                le = mu;
                les = sig;
            } else {
                const bool same = __float_as_uint(g) == __float_as_uint(lg) && __float_as_uint(gs) == __float_as_uint(ls);
                if (__ballot(!same) != 0ull && !same) {
                    pc_block_apx<0>(A.P, j, len, k0, mu, sig, (uint32_t)NB, np);
                    lg = g;
                    ls = gs;
                    le = mu;
                    les = sig;
                }
            }
            __syncthreads();
            double a = 1.0, bm = 0.0, bsv = 0.0;
            bool mm = false;
            if ((int)j < nbe - 1 && t < PC_TPB - 1) {
                const float gn = lget(L.gg[t + 1]), gsn = lget(L.gsg[t + 1]);
                mm = __float_as_uint(le) != __float_as_uint(gn) || __float_as_uint(les) != __float_as_uint(gsn);
                bm = (double)le - (double)gn;
                bsv = (double)les - (double)gsn;
            }
            if ((int)j < nbe - 1) {
                const uint32_t k1 = k0 + len - 1u;
                float af = (float)(k0 - 1u) * __builtin_amdgcn_rcpf((float)k1);
                if (have_o && g != go) {
                    const float sl = (le - eo) * __builtin_amdgcn_rcpf(g - go);
                    if (sl >= 0.0f && sl <= 1.0f) af = sl;
                }
                a = (double)af;
            }
            go = g;
            eo = le;
            have_o = true;
            pcg2_scan(A, L, grid, parity, nbe, a, bm, bsv, mm, g, gs, le, les, false, dm, ds, first,
                      A.gran ? A.tag0 + (++nscan) : 0u);
            parity ^= 1;
            if (first == NB) {
                if (phase == 0) break;   // stage 1's fixed point (sig steps uncertified): verify it exactly
                if (j == (uint32_t)(nbe - 1)) {
                    A.st[A.b].conv_w = itk_conv(le, les, n);
                    A.st[A.b].conv_bound = 0;
                }
                done = true;
                break;
            }
            if (r == cap - 1) break;
            g = dm == 0.0 ? g : (float)((double)g + dm);
            gs = ds == 0.0 ? gs : (float)((double)gs + ds);
        }
    }
#ifdef PCG_PROF
    if (j == 0) printf("PCG2 n %lld G %d L %u stage0 %d stage1+B %d done %d\n", (long long)n, (int)gridDim.x, m.L,
                       rs1 + 1, round - rs1, (int)done);
#endif
    if (!done) {   // round cap: serial from the first failing transition (ends exact up to it); its
        // predecessors' ends are in the published records only at workgroup edges, so the grid
        // publishes every end first
        float *const E = A.E;
        E[j] = le;
        E[(size_t)NB + j] = les;
        grid.sync();
        if (j == 0) {
            float mu = E[first], sig = E[(size_t)NB + first];
            for (int jb = first + 1; jb < nbe; ++jb) {
                const uint32_t l = pc_len(m, jb);
                double kd = (double)pc_k0(m, jb);
                for (uint32_t s = 0; s < l; ++s, kd += 1.0) pc_step(kd, A.P[(size_t)s * NB + jb], mu, sig);
            }
            A.st[A.b].conv_w = itk_conv(mu, sig, n);
            A.st[A.b].conv_bound = 0;
        }
    }
}

