// n4_study.hip -- volume-resident N4 bias-field correction on gfx950: ONE workgroup (1024 threads,
// 16 waves; ST_TPB=512 builds: 8 waves, two studies per CU) per study runs the whole multi-level
// iteration loop of
// sitk.N4BiasFieldCorrectionImageFilter (Vent_Analysis.py:316-334; build spec
// S1-S9 in oracle/n4_oracle.c, which this kernel matches bit for bit) in a single launch.  Between
// sweeps the study's small state -- B-spline lattice, level tables, histogram, FFT buffers, E(u)
// map, the new field's z-contracted lattice P1 -- stays in LDS (70 KB at 128x128x24); the fit
// denominators and the per-column T windows of the last two fields (the old field's B at every
// voxel is rebuilt from them) sit in small per-study global buffers that stay in L2.  An
// iteration costs three streaming passes over the compact masked voxels, workgroup barriers and
// (conv_mode 0) the convergence recurrence, with no kernel launches, no grid-wide dependencies and
// no host round trips.  A batch of >= one study per CU fills the chip.
//
// Per iteration (all inside the workgroup):
//   ctrl  convergence of the previous iteration, ITK's while-condition, bin range (S2: max and the
//         three smallest U per item, merged; ITK's else-if minimum from the first masked voxels)
//   hist  flat pass over compact U: packed Parzen histogram (S3), one 64-bit LDS add per value
//   emap  512-point radix-2 FFT Wiener deconvolution in LDS (S4)
//   fit   column walk: a wave owns one (64-column tile, 64-row slot) item; each lane one column,
//         the row axis contracted in registers by a sliding 4-wide window (S5), finished control
//         rows contracted over the tile's slices and cols, 128-bit fixed-point LDS atomics
//   lat   phi = num / den, lattice += phi, P1 = lattice contracted over slices (S6)
//   eval  column walk again: B_new from the column's T window (from P1, stored for the next
//         iteration), B_old from the stored window of the previous field, U = L0 - B_new, the field
//         difference d written in raster order (conv_mode 0) or the exact-CoV sums (conv_mode 1)
//   conv  (conv_mode 0) ITK's float Welford recurrence over d in raster order (S7) by guess and
//         verify on all waves (n4_shared.h PC)
// Work items are taken from an LDS counter; every reduction is either integer (order-free) or in
// a fixed order, so results are deterministic.
//
// Round 4: 153 -> 70 KB of LDS per study (P1 pair, denominators and the second table set out of
// LDS, 4 histogram copies in the emap's DEN buffer) at unchanged speed, so that ST_TPB=512 builds
// fit two studies per CU.  Measured: two 512-thread studies on a CU
// take 1.37x as long as one alone, 1.46x the CU's throughput -- but one alone takes 1.26x as long
// as a 1024-thread study (128 VGPRs and half the waves for the latency-bound fit and eval walks),
// and 256-study batches do not keep both slots fed (the next batch's short kernels wait for CUs
// that two studies fill), so 1024 threads stay the default.  The serial-chain variant of S7 (chain
// waves beside the compute waves, 46-54 ms per bench step against PC's 33 ms) is gone.
#include <algorithm>
#include <cfloat>
#include <cstring>

#include "n4_shared.h"

#ifndef ST_TPB
#define ST_TPB 1024
#endif
#define ST_WAVES (ST_TPB / 64)
#define ST_HC 4        // LDS histogram copies (in the emap's DEN buffer, free until the Wiener pass)
#define ST_NFIRST 16   // first masked voxels (raster order) tracked for the bin minimum (n4_shared.h r3_bin_min)
#define ST_MAX_LDS (160 * 1024)
#ifndef PC_DRIFT
#define PC_DRIFT 1   // PC's first guesses carry the previous iteration's drift (pcw_run; r4at: 18.89 -> 18.63 ms)
#endif
#ifndef ST_EVAL_EXP
#define ST_EVAL_EXP 0   // 1: eval stores p = expf_cr(d) for PC (its pass 0 then skips the exp)
#endif
// 1024 only: the round-4 512-thread build (two studies per CU) no longer
// converges since the round-5/6 PC changes (r6t: every level runs 50 iterations) and is not kept up
static_assert(ST_TPB == 1024, "pcw_run takes the whole workgroup (one block per thread)");
constexpr int ST_NB = 2;   // U buffers: the last computed field's and the one being computed

// ST_PROF builds (scripts/dev/phase_ab.sh): block 0 prints shader cycles per phase at the end
#ifdef ST_PROF
#define ST_MARK(k) do { if (t == st_pt) { const unsigned long long _c = clock64(); \
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
    float *D;           // [nb][VS] B_old - B_new in raster order of the masked voxels (conv_mode 0)
    const int32_t *rs;
    const uint64_t *rmask;
    const int32_t *rrs;
    const VolScalars *sc;
    const int32_t *order;   // workgroup -> study (largest first; null: identity)
    N4State *st;
    double *P1out;
    int64_t q2cap;
    const double2 *tw;
    int64_t VS;
    int32_t R, C, Z, CZ, ntiles, nslots, nitems;
    int32_t nlev, bins, conv_mode;
    float thresh, fwhm, noise;
    const StudyLevels *lvs;   // device copy: per-level tables and iteration caps
    // dynamic-LDS carve (byte offsets)
    int32_t o_E, o_tab, o_lat, o_ipart, o_rpart, o_misc, o_scr, o_wave, o_order;
    int64_t half;              // U buffers: the second at + half floats (D: PC's p values there)
    int32_t s_cap;   // doubles of a wave's ring row (>= 64, >= ny * KT)
    int32_t nb_ring; // ring rows per wave (<= FIT_NB)
    int32_t o_wx;    // row weights of the current level: Wx[2][R][4] doubles (w^3/sum w^2, w^2)
    int32_t o_wk;    // dense slice weights Wk[2][ncz][Z] (w^3, w^2) of the current level
    int32_t kcap;    // krange entries per table set
    int64_t vol0;
    double *den;     // [nb][lat_cap] fit denominators of the current level
    int64_t lat_cap;
    float *Tg;       // [nb][2][tcap] T(i, col) of the last two fields, col fastest (stride CZ)
    float *pcdrift;  // [nb][ST_TPB] PC: the last call's block-start offsets (PC_DRIFT), or null
    int64_t tcap;
};

struct StudyMisc {
    int32_t item_ctr, stop, exact, nfirst;
    int32_t foff[ST_NFIRST];   // compact offsets of the first masked voxels in raster order
    int32_t rx[ST_NFIRST], rc[ST_NFIRST];   // their (row, column)
    float fu[ST_NFIRST];   // their values in the current field (ctrl wave)
    float bin_min, slope, bmax, pad;
#ifdef ST_PROF
    unsigned long long fprof[4];   // wave of thread st_pt: fit rows / push / contract / items
    unsigned long long sprof[4];   // emap series of thread 300 (h in range): total, hist sums, kernel exp, twiddle
#endif
    double sd, sd2, conv;
    ChainState ch;             // PC's result (conv of the last iteration)
    int32_t itn, uin;          // iterations of the level, U buffer of the last field
    int32_t pc_rounds, pc_fb;  // S7 by PC: rounds and serial fallbacks over all iterations
    int32_t pc_pre;            // the last call decided early (PC_PRE): try again on the next one
};

// One level's axis tables staged in LDS.
struct TabW {
    float4 *wx, *wy, *wz;
    double *ix, *iy, *iz;
    int32_t *bx, *by, *bz;
    int2 *krz;
    int32_t *xst;   // [ncx - 2]: first row x with bx[x] >= i (xst[ncx - 3] = R)
};

__host__ __device__ inline size_t study_tab_bytes(int R, int C, int Z, int kcap) {
    return (((size_t)28 * (R + C + Z) + 12 * (size_t)kcap + 16) + 15) & ~(size_t)15;
}

__device__ __forceinline__ TabW tab_w(char *p, int R, int C, int Z, int kcap) {
    TabW t;
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
__device__ __forceinline__ TabV tab_view(char *p, int R, int C, int Z, int kcap) {
    const TabW w = tab_w(p, R, C, Z, kcap);
    TabV t;
    t.wx = w.wx; t.wy = w.wy; t.wz = w.wz;
    t.ix = w.ix; t.iy = w.iy; t.iz = w.iz;
    t.bx = w.bx; t.by = w.by; t.bz = w.bz;
    t.krz = w.krz;
    t.xst = w.xst;
    return t;
}

__device__ void load_tables(const TabW &t, const DevLevel &lv, int R, int C, int Z) {
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
    for (int i = threadIdx.x; i <= lv.ax[0].ncp - 3; i += ST_TPB) t.xst[i] = lv.xst[i];
}

__device__ __forceinline__ bool study_item(Item &it, const StudyArgs &a, int64_t b, int item) {
    const int64_t tb = b * (int64_t)a.ntiles * a.R;
    return item_begin(it, a.rmask + tb, a.rs + tb, a.rrs + tb, a.R, a.C, a.Z, a.CZ, a.nslots, item);
}

__device__ __forceinline__ void rpart_store(float4 *rpart, int item, const Range3 &r) {
    if ((threadIdx.x & 63) == 0) rpart[item] = make_float4(r.mx, r.m1, r.m2, r.m3);
}

// Init + range of the initial field over one item: L0 = (float)log((double)I) at mask == 1 (S1;
// non-positive -> 0), U = L0 (B = 0).
__device__ void init_item(const StudyArgs &a, int64_t b, const Item &it, int item, float *Lb,
                          float *Ub, int64_t n, float4 *rpart) {
    const __amdgpu_buffer_rsrc_t rL = st_rsrc(Lb, n), rU = st_rsrc(Ub, n);
    const float *Ib = a.I + b * a.V + it.col;
    Range3 rg;
    r3_init(rg);
#pragma unroll 1
    for (int xb = it.xs; xb <= it.xe; xb += FIT_G) {
        uint32_t offs[FIT_G];
        float iv[FIT_G];
#pragma unroll
        for (int g = 0; g < FIT_G; ++g) {   // the group's image loads together
            const int xg = xb + g;
            offs[g] = item_off(it, xg <= it.xe ? xg : it.xe, xg <= it.xe);
            iv[g] = offs[g] != VH_OOB ? Ib[(int64_t)xg * a.CZ] : 0.0f;
        }
#pragma unroll
        for (int g = 0; g < FIT_G; ++g) {
            if (offs[g] == VH_OOB) continue;
            const float l = iv[g] > 0.0f ? (float)log((double)iv[g]) : 0.0f;
            st_store(rL, offs[g], l);
            st_store(rU, offs[g], l);
            r3_add(rg, l);
        }
    }
    rpart_store(rpart, item, r3_wave(rg));
}

// wave 0: the first ST_NFIRST masked voxels in raster order (row, then column) and their compact offsets
__device__ void find_first(const StudyArgs &a, int64_t b, int64_t first, StudyMisc &M) {
    const int lane = threadIdx.x & 63;
    int found = 0;
    if (lane == 0) {
        for (int q = 0; q < ST_NFIRST; ++q) M.rx[q] = M.rc[q] = M.foff[q] = -1;
        M.nfirst = 0;
    }
    if (first < 0) return;
    const int64_t tb = b * (int64_t)a.ntiles * a.R;
    const int fx = (int)(first / a.CZ), fcol = (int)(first % a.CZ);
    for (int x = fx; x < a.R && found < ST_NFIRST; ++x)
        for (int t0 = x == fx ? fcol / TILE_W : 0; t0 < a.ntiles && found < ST_NFIRST; t0 += 64) {
            const int t = t0 + lane;
            uint64_t m = t < a.ntiles ? a.rmask[tb + (int64_t)t * a.R + x] : 0ull;
            if (x == fx && t < fcol / TILE_W) m = 0ull;
            if (x == fx && t == fcol / TILE_W) m &= ~((2ull << (fcol % TILE_W)) - 1ull) | (1ull << (fcol % TILE_W));
            uint64_t nz = __ballot(m != 0ull);
            while (nz && found < ST_NFIRST) {
                const int l = __builtin_ctzll(nz);
                nz &= nz - 1;
                const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)m, l);
                const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(m >> 32), l);
                uint64_t mm = ((uint64_t)hi << 32) | lo;
                while (mm && found < ST_NFIRST) {
                    const int bit = __builtin_ctzll(mm);
                    mm &= mm - 1;
                    if (lane == 0) {
                        const int tt = t0 + l;
                        const int64_t e = tb + (int64_t)tt * a.R + x;
                        const uint64_t full = a.rmask[e];
                        M.rx[found] = x;
                        M.rc[found] = tt * TILE_W + bit;
                        M.foff[found] = a.rs[e] + __popcll(full & ((1ull << bit) - 1ull));
                        M.nfirst = found + 1;
                    }
                    ++found;
                }
            }
        }
}

// T(i) of this lane's column: the lattice contracted over slices (P1) then cols, rounded to float
// (S6; identical expression to n4.hip col_T / k_n4_T)
__device__ __forceinline__ float col_T_lds(const double *P1, int i, int ncy, int Z, int by,
                                           float4 wy, int z) {
    const double *r = P1 + ((int64_t)i * ncy + by) * Z + z;
    return (float)((double)wy.x * r[0] + (double)wy.y * r[Z] + (double)wy.z * r[2 * Z] +
                   (double)wy.w * r[3 * Z]);
}

// eval: B_new, U = L0 - B_new, the field difference d = B_old - B_new (conv_mode 0: stored at the
// voxel's raster rank; conv_mode 1: exact-CoV sums), U range.  The lane's column T window of the
// new field comes from P1 in LDS and is stored to Tgn (the next iteration's old window, the same
// control rows: the walk is the same); the old field's window is loaded from Tgo (written by the
// previous iteration's eval with the tables of its level: the same floats a P1 of the old field
// would give).  SAME: the previous field uses this level's tables (every
// iteration but the first of levels > 0), so both windows move together at the row-span
// boundaries (the old window's next row is loaded one span ahead); otherwise rows are taken one
// at a time (To: the previous level's row tables, in global memory).
template <bool SAME, int CM>
__device__ void eval_item(const Item &it, int item, int Z, int CZ, const TabV &Tn, const TabV &To,
                          int ncxn, int ncyn, int ncxo, const double *P1n, float *Tgn, const float *Tgo,
                          bool bo_mode, const float *Lb, float *Ub, float *Db, int64_t n,
                          double *ipart, float4 *rpart, const PcMap &pm) {
    const __amdgpu_buffer_rsrc_t rL = st_rsrc(Lb, n), rU = st_rsrc(Ub, n), rD = st_rsrc(Db, n);
    const float4 wyn = it.colok ? Tn.wy[it.y] : make_float4(0.f, 0.f, 0.f, 0.f);
    const int byn = Tn.by[it.y];
    // T(i, col) at byte offset 4 (i CZ + col) of a buffer resource: 32-bit offsets (no 64-bit
    // address pairs to keep live), a masked-off lane's store dropped and its load 0 by the range check
    const __amdgpu_buffer_rsrc_t rTn = st_rsrc(Tgn, (int64_t)ncxn * CZ), rTo = st_rsrc(Tgo, (int64_t)ncxo * CZ);
    const uint32_t cb = (uint32_t)it.col * 4u, rsz = (uint32_t)uni(CZ * 4);
    int wbn = uni(Tn.bx[it.xs]), wbo = uni(To.bx[it.xs]);
    auto tnew = [&](int i) {
        const float v = col_T_lds(P1n, i, ncyn, Z, byn, wyn, it.z);
        st_store(rTn, it.colok ? cb + (uint32_t)i * rsz : VH_OOB, v);
        return v;
    };
    auto told = [&](int i) { return st_load(rTo, it.colok ? cb + (uint32_t)i * rsz : VH_OOB); };
    float tn0 = tnew(wbn), tn1 = tnew(wbn + 1), tn2 = tnew(wbn + 2), tn3 = tnew(wbn + 3);
    float to0 = 0.f, to1 = 0.f, to2 = 0.f, to3 = 0.f, to4 = 0.f;
    if (bo_mode) {
        to0 = told(wbo);
        to1 = told(wbo + 1);
        to2 = told(wbo + 2);
        to3 = told(wbo + 3);
        if (SAME) to4 = told(wbo + 4);   // (past the last control row: 0 from the range check)
    }
    double sd = 0.0, sd2 = 0.0;
    Range3 rg;
    r3_init(rg);
    // one voxel; off / roff are VH_OOB for a masked-out lane or a row past the span: its stores are
    // dropped by the buffer range check and its values are replaced by neutral ones (the current max /
    // third smallest for the range, 0 for the sums), so the row groups below run without branches (a branch per voxel
    // made every load of the group a maybe-pending one at the joins, and the waits for them undid
    // the next group's prefetch)
    auto voxel = [&](uint32_t off, uint32_t roff, float la, int x) {
        const bool on = off != VH_OOB;
        const float4 w = Tn.wx[x];
        const float bn = ((w.x * tn0 + w.y * tn1) + w.z * tn2) + w.w * tn3;
        float bo = 0.0f;
        if (bo_mode) {
            const float4 wo = SAME ? w : To.wx[x];
            bo = ((wo.x * to0 + wo.y * to1) + wo.z * to2) + wo.w * to3;
        }
        const float u = la - bn;
#ifndef AB_EVAL_NOSTORE   // A/B builds only: the phase without its U / d stores
        st_store(rU, off, u);
#endif
        if (CM == 0) {
#ifndef AB_EVAL_NOSTORE
            st_store(rD, roff, ST_EVAL_EXP ? expf_cr(bo - bn) : bo - bn);
#else
            if (bo - bn == 12345.0f) st_store(rD, roff, u);
#endif
        } else {
            const double d = on ? (double)expm1c(bo - bn) : 0.0;
            sd += d;
            sd2 = fma(d, d, sd2);
        }
        const float um = on ? u : rg.mx, un = on ? u : rg.m3;   // neutral: max(mx, mx), ins(m3)
        rg.mx = fmaxf(rg.mx, um);
        r3_ins(rg, un);
    };
    if (SAME) {
        int x = it.xs;
#pragma unroll 1
        for (;;) {
            const int rb = uni(min(it.xe, Tn.xst[wbn + 1] - 1));
            // groups of FIT_G rows, two per trip: the next group's L0 loads are in flight while
            // this group's voxels are evaluated (the span's rows only: the window moves after it)
            uint32_t oA[FIT_G], oB[FIT_G];
            int rA[FIT_G], rB[FIT_G];
            float lA[FIT_G], lB[FIT_G];
            auto issue = [&](int xb, uint32_t (&o)[FIT_G], int (&r)[FIT_G], float (&l)[FIT_G]) {
#pragma unroll
                for (int g = 0; g < FIT_G; ++g) {
                    const int xg = xb + g;
                    int rr = 0;
                    o[g] = item_off(it, xg <= rb ? xg : rb, xg <= rb, CM == 0 ? &rr : nullptr);
                    r[g] = o[g] == VH_OOB ? (int)VH_OOB : rr * 4;
#ifdef AB_EVAL_NOLOAD   // A/B builds only (fixed iteration counts): the phase without its L0 loads
                    l[g] = 1.0f + (float)g;
#else
                    l[g] = st_load(rL, o[g]);
#endif
                }
            };
            auto run = [&](int xb, const uint32_t (&o)[FIT_G], const int (&r)[FIT_G], const float (&l)[FIT_G]) {
#pragma unroll
                for (int g = 0; g < FIT_G; ++g)
                    voxel(o[g], CM == 0 ? (uint32_t)r[g] : VH_OOB, l[g], xb + g <= rb ? xb + g : rb);
            };
            if (x <= rb) {
                issue(x, oA, rA, lA);
#pragma unroll 1
                for (int xb = x;; xb += 2 * FIT_G) {
                    issue(xb + FIT_G, oB, rB, lB);   // unconditional, as in fit_item
                    run(xb, oA, rA, lA);
                    if (xb + FIT_G > rb) break;
                    issue(xb + 2 * FIT_G, oA, rA, lA);
                    run(xb + FIT_G, oB, rB, lB);
                    if (xb + 2 * FIT_G > rb) break;
                }
            }
            x = rb + 1 > x ? rb + 1 : x;
            if (x > it.xe) break;
            ++wbn;   // next span: both windows move one control row
            tn0 = tn1; tn1 = tn2; tn2 = tn3;
            tn3 = tnew(wbn + 3);
            if (bo_mode) {
                ++wbo;
                to0 = to1; to1 = to2; to2 = to3; to3 = to4;
                to4 = told(wbo + 4);
            }
        }
    } else {
#pragma unroll 1
        for (int x = it.xs; x <= it.xe; ++x) {
            const int bxn = uni(Tn.bx[x]);
            while (bxn > wbn) {
                ++wbn;
                tn0 = tn1; tn1 = tn2; tn2 = tn3;
                tn3 = tnew(wbn + 3);
            }
            const int bxo = uni(To.bx[x]);
            while (bo_mode && bxo > wbo) {
                ++wbo;
                to0 = to1; to1 = to2; to2 = to3;
                to3 = told(wbo + 3);
            }
            int rr = 0;
            const uint32_t off = item_off(it, x, true, CM == 0 ? &rr : nullptr);
            if (off != VH_OOB) voxel(off, (uint32_t)rr * 4u, st_load(rL, off), x);
        }
    }
    if (CM != 0) {
        for (int off = 32; off > 0; off >>= 1) {
            sd += __shfl_down(sd, off, 64);
            sd2 += __shfl_down(sd2, off, 64);
        }
        if ((threadIdx.x & 63) == 0) {
            ipart[2 * item] = sd;
            ipart[2 * item + 1] = sd2;
        }
    }
    rpart_store(rpart, item, r3_wave(rg));
}

// ---------------------------------------------------------------------------------------------
// FFT (512-point radix-2 DIT, same butterflies and twiddle indexing as oracle/n4_oracle.c) by ONE
// wave in place in LDS.  The points sit at padded slots fpad(i) (one spare slot per 8), so the
// strided passes below hit distinct LDS banks.  Only wave-local ordering is needed.
// ---------------------------------------------------------------------------------------------
#define ST_FFT_N (VH_FFT_P + VH_FFT_P / 8)   // padded slots of one transform
#ifndef ST_WPAR
// E-map: the pointwise steps between the FFTs run on all threads, as passes of their own (3: the
// Wiener filter, the clamp / moment series and the kernel product; 2: not the product; 1: only the
// filter; 0: all inside the one- or two-wave FFTs' first / last passes, round 4).  Bit-identical
// arithmetic; 3 is 5 % faster on the study kernel (DESIGN_LOG.md round 5).
#define ST_WPAR 3
#endif
__device__ __forceinline__ int fpad(int i) { return i + (i >> 3); }

struct FftId {
    __device__ double2 operator()(int, double2 v) const { return v; }
};

// The 9 stages run as 3 register passes of 3: in pass p a lane owns the 8 points
// base + m * 8^p (m < 8), which the stages of half-length 8^p, 2 * 8^p, 4 * 8^p pair only among
// themselves.  Pass 0 gathers in bit-reversed order through pro(i, v); pass 2 stores epi(i, v).
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
                const int j = stride * (m & ((1 << s) - 1)) + lane % stride;
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

// The workgroup's barrier (the phases below were once shared with a subset of the waves)
struct Grp {
    int t, n, w, nw;   // thread / threads, wave / waves of the group
};
__device__ __forceinline__ void gsync(const Grp &, StudyMisc &) { __syncthreads(); }

__device__ float exact_min_study(const StudyArgs &a, int64_t b, const float *Ub, float *s_cmax,
                                 float *s_min, const Grp &g, StudyMisc &M) {
    const int t = g.t;
    const int per = (a.R + g.n - 1) / g.n;
    const int s0 = min(t * per, a.R), e0 = min(s0 + per, a.R);
    float cmax = -FLT_MAX, dummy = FLT_MAX;
    for (int x = s0; x < e0; ++x) exact_row(a, b, Ub, x, cmax, dummy, false);
    s_cmax[t] = cmax;
    gsync(g, M);
    if (t == 0) {
        float run = -FLT_MAX;
        for (int i = 0; i < g.n; ++i) { const float v = s_cmax[i]; s_cmax[i] = run; run = v > run ? v : run; }
    }
    gsync(g, M);
    float run = s_cmax[t], mn = FLT_MAX;
    for (int x = s0; x < e0; ++x) exact_row(a, b, Ub, x, run, mn, true);
    s_min[t] = mn;
    gsync(g, M);
    float m = FLT_MAX;
    if (t == 0)
        for (int i = 0; i < g.n; ++i) m = s_min[i] < m ? s_min[i] : m;
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

// take the next item of the current pass (largest first)
__device__ __forceinline__ int next_item(StudyMisc &M, const int32_t *ordr, int nitems) {
    int item = 0;
    if ((threadIdx.x & 63) == 0) item = atomicAdd(&M.item_ctr, 1);
    item = uni(__shfl(item, 0, 64));
    return item >= nitems ? -1 : uni(ordr[item]);
}

// ---------------------------------------------------------------------------------------------
// the kernel: one workgroup per study
// ---------------------------------------------------------------------------------------------
// 4 waves per SIMD (<= 128 VGPRs): one 1024-thread workgroup or two 512-thread ones per CU
__global__ void __launch_bounds__(ST_TPB, 4) k_n4_study(StudyArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int64_t b = a.vol0 + (a.order ? a.order[blockIdx.x] : (int32_t)blockIdx.x);
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    StudyMisc &M = *reinterpret_cast<StudyMisc *>(smem + a.o_misc);
    float *sE = reinterpret_cast<float *>(smem + a.o_E);
    float *lat = reinterpret_cast<float *>(smem + a.o_lat);
    double *ipart = reinterpret_cast<double *>(smem + a.o_ipart);
    float4 *const rpart0 = reinterpret_cast<float4 *>(smem + a.o_rpart);   // [2][nitems]: per U buffer
    int32_t *ordr = reinterpret_cast<int32_t *>(smem + a.o_order);
    char *scr = smem + a.o_scr;

    const int64_t n = a.sc[b].n_mask1;
    N4State *stb = a.st + b;
    if (t == 0) {   // per-study durations and placement (vh_batch_study_times, VH_STUDY_TRACE)
        stb->t_start = wall_clock64();
        stb->hw_id = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID: cu / sh / se
        stb->xcc_id = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // HW_REG_XCC_ID
    }
    const DevLevel &lvl = a.lvs->lv[a.nlev - 1];
    const int p1last = lvl.ax[0].ncp * lvl.ax[1].ncp * a.Z;
    if (n < 2) {   // no fit: zero field (output = input), no iterations
        for (int e = t; e < p1last; e += ST_TPB) a.P1out[b * a.q2cap + e] = 0.0;
        if (t < VH_MAX_LEVELS) {
            stb->iters_level[t] = 0;
            stb->conv_level[t] = 0.0f;
        }
        if (t == 0) stb->t_end = wall_clock64();
        return;
    }
    Grp g;
    g.w = wv;
    g.nw = ST_WAVES;
    g.t = t;
    g.n = ST_TPB;
    float *Lb = a.L0 + b * a.VS;
    const int64_t fm = a.sc[b].first_masked;
    // fit scratch: lattice numerator (fixed point), then per-wave Q / S rows; from the lattice
    // update to the end of eval: the new field's P1
    unsigned long long *numfix = reinterpret_cast<unsigned long long *>(scr);
    double *const P1 = reinterpret_cast<double *>(scr);
    double *const den = a.den + b * a.lat_cap;          // this level's fit denominators
    float *const Tg0 = a.Tg + (size_t)b * 2 * a.tcap;   // T windows of the last two fields
    FitRing ring;
    ring.q = reinterpret_cast<double *>(scr + a.o_wave) + (size_t)g.w * a.nb_ring * a.s_cap;
    ring.sx = nullptr;
    ring.rowcap = a.s_cap;
    ring.nr = 0;
    double *const Wk3 = reinterpret_cast<double *>(smem + a.o_wk);
    // emap scratch: V (= U = NUM), F, DEN, twiddles; the histogram copies in DEN (read by the
    // series loop, which writes V and F; DEN is written after it)
    double2 *V = reinterpret_cast<double2 *>(scr), *F = V + ST_FFT_N, *DEN = F + ST_FFT_N;
    double2 *TW = DEN + ST_FFT_N;
    unsigned long long *Hc = reinterpret_cast<unsigned long long *>(DEN);
    static_assert(sizeof(unsigned long long) * ST_HC * VH_MAX_BINS <= sizeof(double2) * ST_FFT_N,
                  "histogram copies fit the DEN buffer");
    const PcMap pm = pc_map(n, 256);   // (eval_item's PC layout argument: unused here)
    const int bins = a.bins;
#ifdef ST_PROF
    const int st_pt = 0;   // the thread that keeps the marks
#endif

    if (t == 0) {
        M.item_ctr = 0;
        M.uin = 0;
        M.pc_rounds = 0;
        M.pc_fb = 0;
        M.pc_pre = 0;
    }
    if (wv == 0) find_first(a, b, fm, M);
    {   // item schedule: items by row count, largest first (ties by index), so the dynamic item
        // queue of every pass ends on small items; the item order of every reduction is unchanged
        int32_t *isz = reinterpret_cast<int32_t *>(scr);
        for (int item = wv; item < a.nitems; item += ST_WAVES) {
            Item it;
            const bool any = study_item(it, a, b, item);
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
    for (;;) {   // L0, U = L0 (U buffer 0) and its range
        const int item = next_item(M, ordr, a.nitems);
        if (item < 0) break;
        Item it;
        if (!study_item(it, a, b, item)) {
            if (lane == 0) rpart0[item] = make_float4(-FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX);
            continue;
        }
        init_item(a, b, it, item, Lb, a.U + b * a.VS, n, rpart0);
    }
    // every wave must have left the init queue before thread 0 resets the item counter for the
    // denominator pass (a late wave would otherwise take den-pass items)
    __syncthreads();
    {
        const DevLevel &l0 = a.lvs->lv[0];
        const int nl0 = l0.ax[0].ncp * l0.ax[1].ncp * l0.ax[2].ncp;
        for (int e = t; e < nl0; e += ST_TPB) lat[e] = 0.0f;
    }
#ifdef ST_PROF
    unsigned long long st_prof[18] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, st_t0 = clock64();
    if (t == 0) M.fprof[0] = M.fprof[1] = M.fprof[2] = M.fprof[3] = 0ull;
    if (t == 0) M.sprof[0] = M.sprof[1] = M.sprof[2] = M.sprof[3] = 0ull;
#endif
    int tpar = 0;   // Tg buffer of the last computed field's T windows
    for (int L = 0; L < a.nlev; ++L) {
        const DevLevel &lv = a.lvs->lv[L];
        char *tabp = smem + a.o_tab;
        load_tables(tab_w(tabp, a.R, a.C, a.Z, a.kcap), lv, a.R, a.C, a.Z);
        const TabV T = tab_view(tabp, a.R, a.C, a.Z, a.kcap);
        const int ncx = lv.ax[0].ncp, ncy = lv.ax[1].ncp, ncz = lv.ax[2].ncp;
        const int nlat = ncx * ncy * ncz;
        double *const Wk2 = Wk3 + (size_t)ncz * a.Z;
        for (int e = t; e < ncz * a.Z; e += ST_TPB) {   // dense slice weights of this level
            Wk3[e] = lv.wk3[e];
            Wk2[e] = lv.wk2[e];
        }
        double2 *const Wx3 = reinterpret_cast<double2 *>(smem + a.o_wx), *const Wx2 = Wx3 + 2 * a.R;
        for (int x = t; x < a.R; x += ST_TPB) {   // row weights of this level (wave-uniform reads)
            const double2 *w3 = reinterpret_cast<const double2 *>(lv.ax[0].w3i + 4 * x);
            const double2 *w2 = reinterpret_cast<const double2 *>(lv.ax[0].w2 + 4 * x);
            Wx3[2 * x] = w3[0];
            Wx3[2 * x + 1] = w3[1];
            Wx2[2 * x] = w2[0];
            Wx2[2 * x + 1] = w2[1];
        }
        // ---- denominator of this level: sum of w^2 over the mask (the compute waves' rings) ----
        for (int e = t; e < 2 * nlat; e += ST_TPB) numfix[e] = 0ull;
        if (t == 0) M.item_ctr = 0;
        __syncthreads();
        {
            const int uin = M.uin;
            float *const Ub = a.U + uin * a.half + b * a.VS;
            for (;;) {
                const int item = next_item(M, ordr, a.nitems);
                if (item < 0) break;
                Item it;
                if (!study_item(it, a, b, item)) continue;
                fit_item<1, true>(it, T, Wk2, Wx2, ncy, ncz, a.Z, bins, Ub, n, sE, 0.0f, 1.0, ring,
                                  a.nb_ring, numfix);
            }
        }
        __syncthreads();
        ST_MARK(0);
        for (int e = t; e < nlat; e += ST_TPB) den[e] = fix128_get(numfix + 2 * e, numfix + 2 * e + 1);
        {
            // ---- the iterations ----
            int itn = 0;       // iterations computed in this level
            int uin = M.uin;   // U buffer (and its rpart row) of the last computed iteration
            for (;;) {
                gsync(g, M);
                ST_MARK(10);
                float *const Ub = a.U + uin * a.half + b * a.VS;
                const float4 *const rp_in = rpart0 + uin * a.nitems;
                if (g.w == 0) {   // ctrl: ITK's while-condition (at the cap, or conv_mode 1), bin range
                    Range3 r;
                    r3_init(r);
                    for (int i = lane; i < a.nitems; i += 64) {
                        const float4 p = rp_in[i];
                        Range3 o;
                        o.mx = p.x; o.m1 = p.y; o.m2 = p.z; o.m3 = p.w;
                        r3_merge(r, o);
                    }
                    r = r3_wave(r);
                    if (lane < M.nfirst) M.fu[lane] = Ub[M.foff[lane]];   // the run's values
                    wave_lds_order();
                    if (lane == 0) {
                        M.stop = 0;
                        M.exact = 0;
                        if (itn > 0) {
                            if (a.conv_mode == 1) M.conv = conv_of(M.sd, M.sd2, (double)n);
                            if (!(M.conv > (double)a.thresh) || itn >= a.lvs->max_iters[L]) M.stop = 1;
                        }
                        if (!M.stop) {
                            float bmin;
                            M.bmax = r.mx;
                            if (r3_bin_min(r, M.fu, M.nfirst, bmin)) {
                                M.bin_min = bmin;
                                M.slope = (r.mx - bmin) / (float)(bins - 1);
                            } else {
                                M.exact = 1;
                            }
                        }
                    }
                }
                gsync(g, M);
                ST_MARK(1);
                if (M.stop) break;
                if (M.exact) {
                    float *s_cmax = reinterpret_cast<float *>(scr);
                    const float m = exact_min_study(a, b, Ub, s_cmax, s_cmax + g.n, g, M);
                    if (g.t == 0) {
                        M.bin_min = m;
                        M.slope = (M.bmax - m) / (float)(bins - 1);
                    }
                    gsync(g, M);
                }
                const int itk = itn + 1;   // the iteration computed now
                ST_MARK(9);
                const float bmin = M.bin_min, slope = M.slope;
                const double rinv = 1.0 / (double)slope;   // div_r form of the bin division
                // ---- hist (S3): one packed 64-bit add per value ----
                for (int i = g.t; i < ST_HC * VH_MAX_BINS; i += g.n) Hc[i] = 0ull;
                gsync(g, M);
                {
                    unsigned long long *H = Hc + (lane & (ST_HC - 1)) * VH_MAX_BINS;
                    for (int64_t j0 = (int64_t)g.t * 16; j0 < n; j0 += (int64_t)g.n * 16) {
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
#pragma unroll
                        for (int k = 0; k < 16; ++k) {
                            int idx;
                            const unsigned long long w = hist_pack(u[k], bmin, rinv, bins, idx);
                            atomicAdd(&H[idx], w);
                        }
                    }
                }
                gsync(g, M);
                ST_MARK(2);
                // ---- emap (same arithmetic as n4.hip k_n4_emap and the oracle) ----
                {
                    const int P = VH_FFT_P, off = (P - bins) / 2;
                    const float sFWHM = a.fwhm / slope;
                    const float ef = (float)(4.0 * LN2 / (double)(sFWHM * sFWHM));
                    const float sf = (float)(2.0 * sqrt(LN2 / PI_D) / (double)sFWHM);
                    // one twiddle per thread: P / 2 <= g.n
#ifdef ST_PROF
                    const unsigned long long sp0 = clock64();
#endif
                    const double2 twv = g.t < P / 2 ? a.tw[g.t] : make_double2(0.0, 0.0);   // in flight
                    for (int i = g.t; i < P; i += g.n) {   // histogram series and Gaussian kernel
                        const int h = i - off;
                        unsigned long long s = 0ull;
                        if (h >= 0 && h < bins)
                            for (int q = 0; q < ST_HC; ++q) {
                                const unsigned long long w = Hc[q * VH_MAX_BINS + h];
                                s += (hist_count(w) << 24) - hist_osum(w);
                                if (h > 0) s += hist_osum(Hc[q * VH_MAX_BINS + h - 1]);
                            }
                        V[fpad(i)] = make_double2((double)s * (1.0 / 16777216.0), 0.0);
#ifdef ST_PROF
                        const unsigned long long sp1 = clock64();
                        if (g.t == 300) M.sprof[1] += sp1 - sp0;
#endif
                        double fx;
                        if (i == 0) {
                            fx = (double)sf;
                        } else if (i == P / 2) {
                            fx = (double)sf * exp(-0.25 * (double)((float)P * (float)P) * (double)ef);
                        } else {
                            const float nf = (float)(i < P / 2 ? i : P - i);
                            fx = (double)(sf * expf_cr_tail(-(nf * nf) * ef));
                        }
                        F[fpad(i)] = make_double2(fx, 0.0);
#ifdef ST_PROF
                        if (g.t == 300) M.sprof[2] += clock64() - sp1;
#endif
                    }
#ifdef ST_PROF
                    const unsigned long long sp2 = clock64();
#endif
                    if (g.t < P / 2) TW[g.t] = twv;
#ifdef ST_PROF
                    if (g.t == 300) M.sprof[0] += clock64() - sp0;
                    if (g.t == 200) M.sprof[3] += clock64() - sp2;
#endif
                    gsync(g, M);
                    ST_MARK(11);
                    if (g.w < 2) wave_fft_lds(g.w ? F : V, TW, false, FftId(), FftId());
                    gsync(g, M);
                    ST_MARK(12);
                    const auto wpost = [=](int i, double2 v) {   // clamp; the moment series' points
                        const double ur = v.x > 0.0 ? v.x : 0.0;
                        const float c = bmin + ((float)i - (float)off) * slope;
                        DEN[fpad(i)] = make_double2(ur, 0.0);
                        return make_double2((double)c * ur, 0.0);
                    };
#if ST_WPAR
                    // Wiener filter on every thread (the divisions would otherwise run 8 deep on
                    // one wave); the same per-point arithmetic as the gather-side form below
                    for (int i = g.t; i < P; i += g.n) {
                        const double2 f = F[fpad(i)], v = V[fpad(i)];
                        const double fa = f.x, fb = f.y;
                        const double gg = fa / ((fa * fa - (-fb) * fb) + (double)a.noise);
                        V[fpad(i)] = make_double2(v.x * gg, v.y * gg);
                    }
                    gsync(g, M);
                    ST_MARK(16);
#if ST_WPAR >= 2
                    if (g.w == 0) wave_fft_lds(V, TW, true, FftId(), FftId());   // inverse
                    ST_MARK(17);
                    gsync(g, M);
                    for (int i = g.t; i < P; i += g.n) V[fpad(i)] = wpost(i, V[fpad(i)]);
#else
                    if (g.w == 0) wave_fft_lds(V, TW, true, FftId(), wpost);   // inverse, clamp, series
                    ST_MARK(17);
#endif
#else
                    if (g.w == 0) {   // Wiener filter (first pass), inverse, clamp and the moment series (last pass)
                        const double noise = (double)a.noise;
                        wave_fft_lds(V, TW, true,
                            [=](int i, double2 v) {
                                const double2 f = F[fpad(i)];
                                const double fa = f.x, fb = f.y;
                                const double gg = fa / ((fa * fa - (-fb) * fb) + noise);
                                return make_double2(v.x * gg, v.y * gg);
                            }, wpost);
                    }
#endif
                    gsync(g, M);
                    ST_MARK(13);
                    const auto kmul = [=](int i, double2 v) {   // times the kernel's transform
                        const double2 f = F[fpad(i)];
                        const double fa = f.x, fb = f.y;
                        return make_double2(v.x * fa - v.y * fb, v.x * fb + v.y * fa);
                    };
#if ST_WPAR >= 3
                    // each series: forward; the product on every thread; inverse
                    if (g.w < 2) wave_fft_lds(g.w ? DEN : V, TW, false, FftId(), FftId());
                    gsync(g, M);
                    for (int e = g.t; e < 2 * P; e += g.n) {
                        double2 *const x = e < P ? V : DEN;
                        const int i = e < P ? e : e - P;
                        x[fpad(i)] = kmul(i, x[fpad(i)]);
                    }
                    gsync(g, M);
                    if (g.w < 2) wave_fft_lds(g.w ? DEN : V, TW, true, FftId(), FftId());
#else
                    if (g.w < 2) {   // each series: forward, times the kernel's transform (last pass), inverse
                        double2 *x = g.w ? DEN : V;
                        wave_fft_lds(x, TW, false, FftId(), kmul);
                        wave_fft_lds(x, TW, true, FftId(), FftId());
                    }
#endif
                    gsync(g, M);
                    ST_MARK(14);
                    for (int i = g.t; i < bins; i += g.n) {
                        const double d = DEN[fpad(i + off)].x;
                        sE[i] = d != 0.0 ? (float)(V[fpad(i + off)].x / d) : 0.0f;
                    }
                    gsync(g, M);
                }
                ST_MARK(3);
                // ---- fit ----
                for (int e = g.t; e < 2 * nlat; e += g.n) numfix[e] = 0ull;
                if (g.t == 0) M.item_ctr = 0;
                gsync(g, M);
                for (;;) {
                    const int item = next_item(M, ordr, a.nitems);
                    if (item < 0) break;
                    Item it;
                    if (!study_item(it, a, b, item)) continue;
                    fit_item<0, true>(it, T, Wk3, Wx3, ncy, ncz, a.Z, bins, Ub, n, sE, bmin, rinv, ring,
                                      a.nb_ring, numfix
#ifdef ST_PROF
                                      , (t >> 6) == (st_pt >> 6) ? M.fprof : nullptr
#endif
                                      );
                }
                gsync(g, M);
                ST_MARK(4);
                // ---- lattice update and P1 (in the fit scratch, free from here to the end of eval) ----
                for (int e = g.t; e < nlat; e += g.n) {
                    const double d = den[e];
                    const double num = fix128_get(numfix + 2 * e, numfix + 2 * e + 1);
                    const float phi = d != 0.0 ? (float)(num / d) : 0.0f;
                    lat[e] += phi;
                }
                gsync(g, M);
                for (int e = g.t; e < ncx * ncy * a.Z; e += g.n) {
                    const int ij = e / a.Z, z = e % a.Z;
                    const float4 w = T.wz[z];
                    const float *l = lat + ij * ncz + T.bz[z];
                    P1[e] = (double)w.x * (double)l[0] + (double)w.y * (double)l[1] +
                            (double)w.z * (double)l[2] + (double)w.w * (double)l[3];
                }
                if (g.t == 0) M.item_ctr = 0;
                gsync(g, M);
                ST_MARK(5);
                // ---- eval: U into the other buffer, d into D, this field's T windows into Tg ----
                {
                    const int uo = (uin + 1) % ST_NB;
                    float *const Uo = a.U + uo * a.half + b * a.VS;
                    float *const Dw = a.D + b * a.VS;
                    float4 *const rp_out = rpart0 + uo * a.nitems;
                    const bool first_of_level = itk == 1;
                    const bool bo_mode = !(L == 0 && first_of_level);
                    const bool same = !(first_of_level && L > 0);
                    TabV To = T;   // first iteration of a level > 0: the old field's row tables
                    int ncxo = ncx;
                    if (!same) {
                        const DevLevel &lo = a.lvs->lv[L - 1];
                        To.wx = reinterpret_cast<const float4 *>(lo.ax[0].w);
                        To.bx = lo.ax[0].base;
                        ncxo = lo.ax[0].ncp;
                    }
                    float *const Tgn = Tg0 + (size_t)(tpar ^ 1) * a.tcap;
                    const float *const Tgo = Tg0 + (size_t)tpar * a.tcap;
                    for (;;) {
                        const int item = next_item(M, ordr, a.nitems);
                        if (item < 0) break;
                        Item it;
                        if (!study_item(it, a, b, item)) {
                            if (lane == 0) {
                                ipart[2 * item] = 0.0;
                                ipart[2 * item + 1] = 0.0;
                                rp_out[item] = make_float4(-FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX);
                            }
                            continue;
                        }
#define ST_EVAL(S, CM) eval_item<S, CM>(it, item, a.Z, a.CZ, T, To, ncx, ncy, ncxo, P1, Tgn, Tgo, bo_mode, \
                                        Lb, Uo, Dw, n, ipart, rp_out, pm)
                        if (a.conv_mode == 0) {
                            if (same) ST_EVAL(true, 0);
                            else ST_EVAL(false, 0);
                        } else {
                            if (same) ST_EVAL(true, 1);
                            else ST_EVAL(false, 1);
                        }
#undef ST_EVAL
                    }
                }
                gsync(g, M);
                ST_MARK(6);
                if (a.conv_mode == 0) {   // S7 on the whole workgroup by guess and verify
                    PcShared<ST_TPB> &PW = *reinterpret_cast<PcShared<ST_TPB> *>(smem + a.o_scr);
                    const float *const Dr = a.D + b * a.VS;
                    // the raster d buffer is free once pass 0 has read it: PCX's stored increments
                    // below the iteration cap this iteration's measure only decides whether the
                    // level goes on: PC may certify "above the threshold" without the exact sig
                    pcw_run<ST_TPB, ST_EVAL_EXP>([=](int64_t r) { return Dr[r]; }, a.D + a.half + b * a.VS, n, PW, M.ch, itk,
                            reinterpret_cast<double *>(a.D + b * a.VS), (int)(a.VS / 2),
                            itk < a.lvs->max_iters[L] ? a.thresh : 0.0f,
                            a.pcdrift ? a.pcdrift + (size_t)b * ST_TPB : nullptr, !(L == 0 && itk == 1),
                            itk == 1 || M.pc_pre != 0);   // early decision: a level's first call, then while it decides
                    if (t == 0) {
                        M.pc_pre = PW.xdone == 4 * itk + 1;
                        M.conv = (double)M.ch.conv;
                        M.pc_rounds += PW.rounds;
                        // serial fallbacks of the exact rounds (units), frozen-serial stage-0 closes (thousands)
                        M.pc_fb += (PW.fallback == 4 * itk + 2 ? 1 : 0) + 1000 * PW.nfrz;
                    }
                } else if (g.w == 0) {   // S7x: item partials in item order
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
                ST_MARK(7);
                tpar ^= 1;
                uin = (uin + 1) % ST_NB;
                itn = itk;
            }
            if (g.t == 0) {
                M.itn = itn;
                M.uin = uin;
            }
        }
        __syncthreads();
        ST_MARK(8);
        if (t == 0) {
            stb->iters_level[L] = M.itn;
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
    }
#ifdef ST_PROF
    // ST_PROF_B: the study whose phase cycles are printed (one study: a printf in every workgroup
    // made the instrumented kernel ~50x slower)
#ifndef ST_PROF_B
#define ST_PROF_B 0
#endif
    if (t == st_pt && b == ST_PROF_B) {
        int its = 0;   // (st_pt is thread 0, the writer of iters_level)
        for (int q = 0; q < a.nlev; ++q) its += stb->iters_level[q];
        printf("ST_PROF b %d n %lld its %d den %llu ctrl %llu hist %llu emap %llu fit %llu latP1 %llu eval %llu "
               "wait %llu level %llu exact %llu top %llu | emap: series %llu fwd %llu filter %llu conv %llu div %llu"
               " (filter: wiener %llu fft %llu sync %llu)\n",
               ST_PROF_B, (long long)n, its, st_prof[0], st_prof[1], st_prof[2],
               st_prof[3] + st_prof[11] + st_prof[12] + st_prof[13] + st_prof[14],
               st_prof[4], st_prof[5], st_prof[6], st_prof[7], st_prof[8], st_prof[9], st_prof[10],
               st_prof[11], st_prof[12], st_prof[13] + st_prof[16] + st_prof[17], st_prof[14], st_prof[3],
               st_prof[16], st_prof[17], st_prof[13]);
        printf("ST_PROF fit: rows %llu push %llu contract %llu items %llu | series thread 300: total %llu "
               "hist %llu kernel-exp %llu; thread 200 twiddle %llu\n", M.fprof[0], M.fprof[1],
               M.fprof[2], M.fprof[3], M.sprof[0], M.sprof[1], M.sprof[2], M.sprof[3]);
    }
#endif
    {   // final field's P1 for k_n4_final, from the lattice (the last level's tables are loaded)
        const TabV T = tab_view(smem + a.o_tab, a.R, a.C, a.Z, a.kcap);
        const int ncz = lvl.ax[2].ncp;
        for (int e = t; e < p1last; e += ST_TPB) {
            const int ij = e / a.Z, z = e % a.Z;
            const float4 w = T.wz[z];
            const float *l = lat + ij * ncz + T.bz[z];
            a.P1out[b * a.q2cap + e] = (double)w.x * (double)l[0] + (double)w.y * (double)l[1] +
                                       (double)w.z * (double)l[2] + (double)w.w * (double)l[3];
        }
    }
    if (t == 0) {
        stb->conv = M.conv;
        stb->active = 0;
        stb->pc_rounds = M.pc_rounds;
        stb->pc_fallbacks = M.pc_fb;
        stb->t_end = wall_clock64();
    }
}

// =============================================================================================
// Grid form (round 6): ONE study over G cooperating workgroups (k_n4_studyg, a cooperative launch)
// =============================================================================================
// The per-iteration sweep launches of the sweep driver (~10 per iteration, plus the host's flag
// reads) carried one large study (config 2, 256x256x24; the class's one-study calls): its kernels
// were short and the launches, gaps and host round trips set the time.  Here the whole multi-level
// loop of one study runs in one launch, as k_n4_study does for a batch, with the study's items
// dealt over G workgroups.  Every workgroup keeps its own copy of the small state in LDS (tables,
// lattice, E map, P1) and computes it redundantly from the same integer sums, so the copies stay
// identical; only order-free integer sums cross workgroups:
//   hist  each workgroup's packed LDS histogram of its slice of compact U, unpacked into counts and
//         o-weight sums and added to the global sums of this iteration's parity (integer atomics)
//   fit   each workgroup's 128-bit fixed-point LDS numerators added to the global numerators of
//         this iteration's parity (carry-correct 64-bit atomics, fix128_flush)
//   range each workgroup's Range3 of its items (a plain record per workgroup; merging is order-free)
//   S7    the grid PC (n4_shared.h pcg2_body) over all G x 1024 threads, d read in raster order
// with a grid barrier after hist, fit, eval and S7 (and the PC's own rounds).  A buffer of one
// parity is zeroed (each workgroup its slice) two barriers after its last read, so no pass needs a
// clearing launch.  Results are bit-identical to k_n4_study / the oracle: the same per-item code,
// the same item-order reductions (the exact CoV sums go through global memory in item order).
struct StudyGrid {
    unsigned long long *hsum;  // [2 parity][2][VH_MAX_BINS]: bin counts, then o-weight sums
    unsigned long long *nsum;  // [3][2 * lat_cap]: fixed-point numerators by parity; [2]: denominators
    float4 *rrec;              // [ST_NB][G]: each workgroup's Range3 of U buffer u
    double *ipart;             // [nitems][2]: exact-CoV item sums (conv_mode 1)
    Pcg2Args pc;               // the grid PC: P, wg, E (this study's scratch), sc, st, b
};

// 128-bit fixed-point partial (l, h) added to a global accumulator (fix128_add's carry rule)
__device__ __forceinline__ void fix128_flush(unsigned long long *glo, unsigned long long *ghi,
                                             unsigned long long l, unsigned long long h) {
    if (l == 0ull && h == 0ull) return;
    const unsigned long long old = atomicAdd(glo, l);
    const unsigned long long carry = old + l < old ? 1ull : 0ull;
    atomicAdd(ghi, h + carry);
}

// The c-th item of workgroup r in the largest-first order: items dealt in snake order (round q
// forward when q is even, backward when odd), so every workgroup's share has about the same rows
__device__ __forceinline__ int owned_item(int c, int r, int G, int nitems) {
    const int pos = (c & 1) ? G - 1 - r : r;
    const int k = c * G + pos;
    return k < nitems ? k : -1;
}
__device__ __forceinline__ int next_item_g(StudyMisc &M, const int32_t *ordr, int nitems, int r, int G) {
    int c = 0;
    if ((threadIdx.x & 63) == 0) c = atomicAdd(&M.item_ctr, 1);
    c = uni(__shfl(c, 0, 64));
    const int k = owned_item(c, r, G, nitems);
    return k < 0 ? -1 : uni(ordr[k]);
}

// wave 0: this workgroup's items' Range3 merged, as record rrec[u][r]
__device__ void publish_range(const StudyGrid &g, const float4 *rp, const int32_t *ordr, int nitems, int u,
                              int r, int G) {
    if (threadIdx.x >= 64) return;
    const int lane = threadIdx.x;
    Range3 rg;
    r3_init(rg);
    for (int c = lane;; c += 64) {
        const int k = owned_item(c, r, G, nitems);
        if (k < 0) break;
        const float4 p = rp[ordr[k]];
        Range3 o;
        o.mx = p.x; o.m1 = p.y; o.m2 = p.z; o.m3 = p.w;
        r3_merge(rg, o);
    }
    rg = r3_wave(rg);
    if (lane == 0) g.rrec[(size_t)u * G + r] = make_float4(rg.mx, rg.m1, rg.m2, rg.m3);
}

// STG_PROF builds: workgroup 0 prints the device wall-clock ticks (100 MHz) spent per phase
#ifdef STG_PROF
#define STG_MARK(k) do { if (r == 0 && t == 0) { const uint64_t _c = wall_clock64(); stg_p[k] += _c - stg_t0; stg_t0 = _c; } } while (0)
#else
#define STG_MARK(k) do { } while (0)
#endif
__global__ void __launch_bounds__(ST_TPB, 4) k_n4_studyg(StudyArgs a, StudyGrid gd) {
    namespace cg = cooperative_groups;
    cg::grid_group grid = cg::this_grid();
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ Pcg2Lds PL;
    const int64_t b = a.vol0;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int r = blockIdx.x, G = gridDim.x;
    StudyMisc &M = *reinterpret_cast<StudyMisc *>(smem + a.o_misc);
    float *sE = reinterpret_cast<float *>(smem + a.o_E);
    float *lat = reinterpret_cast<float *>(smem + a.o_lat);
    float4 *const rpart0 = reinterpret_cast<float4 *>(smem + a.o_rpart);   // [2][nitems] (own items)
    int32_t *ordr = reinterpret_cast<int32_t *>(smem + a.o_order);
    char *scr = smem + a.o_scr;

    const int64_t n = a.sc[b].n_mask1;
    N4State *stb = a.st + b;
    kst_begin(gd.pc.kst);   // profiling: this launch's span (stamped timer)
    if (r == 0 && t == 0) {
        stb->t_start = wall_clock64();
        stb->hw_id = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        stb->xcc_id = __builtin_amdgcn_s_getreg((15 << 11) | 20);
    }
    const DevLevel &lvl = a.lvs->lv[a.nlev - 1];
    const int p1last = lvl.ax[0].ncp * lvl.ax[1].ncp * a.Z;
    if (n < 2) {   // no fit: zero field, no iterations (uniform over the grid)
        if (r == 0) {
            for (int e = t; e < p1last; e += ST_TPB) a.P1out[b * a.q2cap + e] = 0.0;
            if (t < VH_MAX_LEVELS) {
                stb->iters_level[t] = 0;
                stb->conv_level[t] = 0.0f;
            }
            if (t == 0) stb->t_end = wall_clock64();
        }
        kst_end(gd.pc.kst);
        return;
    }
    Grp g;
    g.w = wv;
    g.nw = ST_WAVES;
    g.t = t;
    g.n = ST_TPB;
    float *Lb = a.L0 + b * a.VS;
    const int64_t fm = a.sc[b].first_masked;
    unsigned long long *numfix = reinterpret_cast<unsigned long long *>(scr);
    double *const P1 = reinterpret_cast<double *>(scr);
    float *const Tg0 = a.Tg + (size_t)b * 2 * a.tcap;
    FitRing ring;
    ring.q = reinterpret_cast<double *>(scr + a.o_wave) + (size_t)g.w * a.nb_ring * a.s_cap;
    ring.sx = nullptr;
    ring.rowcap = a.s_cap;
    ring.nr = 0;
    double *const Wk3 = reinterpret_cast<double *>(smem + a.o_wk);
    double2 *V = reinterpret_cast<double2 *>(scr), *F = V + ST_FFT_N, *DEN = F + ST_FFT_N;
    double2 *TW = DEN + ST_FFT_N;
    unsigned long long *Hc = reinterpret_cast<unsigned long long *>(DEN);
    const PcMap pm = pc_map(n, 256);
    const int bins = a.bins;
    unsigned long long *const NSd = gd.nsum + (size_t)2 * 2 * a.lat_cap;   // denominators

    if (t == 0) {
        M.item_ctr = 0;
        M.uin = 0;
    }
    if (wv == 0) find_first(a, b, fm, M);
    {   // the largest-first item order (every workgroup computes the same one)
        int32_t *isz = reinterpret_cast<int32_t *>(scr);
        for (int item = wv; item < a.nitems; item += ST_WAVES) {
            Item it;
            const bool any = study_item(it, a, b, item);
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
    for (;;) {   // L0, U = L0 (U buffer 0) and its range, this workgroup's items
        const int item = next_item_g(M, ordr, a.nitems, r, G);
        if (item < 0) break;
        Item it;
        if (!study_item(it, a, b, item)) {
            if (lane == 0) rpart0[item] = make_float4(-FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX);
            continue;
        }
        init_item(a, b, it, item, Lb, a.U + b * a.VS, n, rpart0);
    }
    __syncthreads();
    publish_range(gd, rpart0, ordr, a.nitems, 0, r, G);
    {
        const DevLevel &l0 = a.lvs->lv[0];
        const int nl0 = l0.ax[0].ncp * l0.ax[1].ncp * l0.ax[2].ncp;
        for (int e = t; e < nl0; e += ST_TPB) lat[e] = 0.0f;
    }
    int tpar = 0;   // Tg buffer of the last computed field's T windows
    int gi = 0;     // iterations computed so far (all levels): the parity of the global sums
#ifdef STG_PROF
    uint64_t stg_p[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, stg_t0 = wall_clock64();
#endif
    for (int L = 0; L < a.nlev; ++L) {
        const DevLevel &lv = a.lvs->lv[L];
        char *tabp = smem + a.o_tab;
        load_tables(tab_w(tabp, a.R, a.C, a.Z, a.kcap), lv, a.R, a.C, a.Z);
        const TabV T = tab_view(tabp, a.R, a.C, a.Z, a.kcap);
        const int ncx = lv.ax[0].ncp, ncy = lv.ax[1].ncp, ncz = lv.ax[2].ncp;
        const int nlat = ncx * ncy * ncz;
        double *const Wk2 = Wk3 + (size_t)ncz * a.Z;
        for (int e = t; e < ncz * a.Z; e += ST_TPB) {
            Wk3[e] = lv.wk3[e];
            Wk2[e] = lv.wk2[e];
        }
        double2 *const Wx3 = reinterpret_cast<double2 *>(smem + a.o_wx), *const Wx2 = Wx3 + 2 * a.R;
        for (int x = t; x < a.R; x += ST_TPB) {
            const double2 *w3 = reinterpret_cast<const double2 *>(lv.ax[0].w3i + 4 * x);
            const double2 *w2 = reinterpret_cast<const double2 *>(lv.ax[0].w2 + 4 * x);
            Wx3[2 * x] = w3[0];
            Wx3[2 * x + 1] = w3[1];
            Wx2[2 * x] = w2[0];
            Wx2[2 * x + 1] = w2[1];
        }
        // ---- denominators of this level: the previous level's are read by nobody any more (every
        // workgroup passed the last iteration's barriers); level 0's were zeroed by the host ----
        if (L > 0) {
            for (int e = r * ST_TPB + t; e < 2 * nlat; e += G * ST_TPB) NSd[e] = 0ull;
            grid.sync();
        }
        for (int e = t; e < 2 * nlat; e += ST_TPB) numfix[e] = 0ull;
        if (t == 0) M.item_ctr = 0;
        __syncthreads();
        {
            float *const Ub = a.U + M.uin * a.half + b * a.VS;
            for (;;) {
                const int item = next_item_g(M, ordr, a.nitems, r, G);
                if (item < 0) break;
                Item it;
                if (!study_item(it, a, b, item)) continue;
                fit_item<1, true>(it, T, Wk2, Wx2, ncy, ncz, a.Z, bins, Ub, n, sE, 0.0f, 1.0, ring,
                                  a.nb_ring, numfix);
            }
        }
        __syncthreads();
        for (int e = t; e < nlat; e += ST_TPB) fix128_flush(NSd + 2 * e, NSd + 2 * e + 1, numfix[2 * e], numfix[2 * e + 1]);
        grid.sync();
        STG_MARK(7);
        {
            int itn = 0;
            int uin = M.uin;
            for (;;) {
                float *const Ub = a.U + uin * a.half + b * a.VS;
                const int p = gi & 1;
                unsigned long long *const HS = gd.hsum + (size_t)p * 2 * VH_MAX_BINS;
                unsigned long long *const HSo = gd.hsum + (size_t)(p ^ 1) * 2 * VH_MAX_BINS;
                unsigned long long *const NS = gd.nsum + (size_t)p * 2 * a.lat_cap;
                unsigned long long *const NSo = gd.nsum + (size_t)(p ^ 1) * 2 * a.lat_cap;
                if (g.w == 0) {   // ctrl (every workgroup, the same decision): the grid's records
                    Range3 rr;
                    r3_init(rr);
                    for (int i = lane; i < G; i += 64) {
                        const float4 q = gd.rrec[(size_t)uin * G + i];
                        Range3 o;
                        o.mx = q.x; o.m1 = q.y; o.m2 = q.z; o.m3 = q.w;
                        r3_merge(rr, o);
                    }
                    rr = r3_wave(rr);
                    if (lane < M.nfirst) M.fu[lane] = Ub[M.foff[lane]];
                    double sd = 0.0, sd2 = 0.0;   // S7x: the item sums in item order (k_n4_study's order)
                    if (a.conv_mode == 1 && itn > 0) {
                        for (int i = lane; i < a.nitems; i += 64) {
                            sd += gd.ipart[2 * i];
                            sd2 += gd.ipart[2 * i + 1];
                        }
                        for (int off = 32; off > 0; off >>= 1) {
                            sd += __shfl_down(sd, off, 64);
                            sd2 += __shfl_down(sd2, off, 64);
                        }
                    }
                    wave_lds_order();
                    if (lane == 0) {
                        M.stop = 0;
                        M.exact = 0;
                        if (itn > 0) {
                            M.conv = a.conv_mode == 1 ? conv_of(sd, sd2, (double)n) : (double)stb->conv_w;
                            if (!(M.conv > (double)a.thresh) || itn >= a.lvs->max_iters[L]) M.stop = 1;
                        }
                        if (!M.stop) {
                            float bmin;
                            M.bmax = rr.mx;
                            if (r3_bin_min(rr, M.fu, M.nfirst, bmin)) {
                                M.bin_min = bmin;
                                M.slope = (rr.mx - bmin) / (float)(bins - 1);
                            } else {
                                M.exact = 1;
                            }
                        }
                    }
                }
                __syncthreads();
                STG_MARK(0);
                if (M.stop) break;
                if (M.exact) {   // rare: every workgroup scans the study itself
                    float *s_cmax = reinterpret_cast<float *>(scr);
                    const float m = exact_min_study(a, b, Ub, s_cmax, s_cmax + g.n, g, M);
                    if (g.t == 0) {
                        M.bin_min = m;
                        M.slope = (M.bmax - m) / (float)(bins - 1);
                    }
                    __syncthreads();
                }
                const int itk = itn + 1;
                const float bmin = M.bin_min, slope = M.slope;
                const double rinv = 1.0 / (double)slope;
                // ---- hist (S3): this workgroup's slice of compact U, then the grid's integer sums ----
                for (int i = g.t; i < ST_HC * VH_MAX_BINS; i += g.n) Hc[i] = 0ull;
                __syncthreads();
                {
                    unsigned long long *H = Hc + (lane & (ST_HC - 1)) * VH_MAX_BINS;
                    const int64_t hchunk = ((n + G - 1) / G + 15) / 16 * 16;   // (16-aligned slices)
                    const int64_t h0 = (int64_t)r * hchunk, h1 = min(n, h0 + hchunk);
                    for (int64_t j0 = h0 + (int64_t)g.t * 16; j0 < h1; j0 += (int64_t)g.n * 16) {
                        float u[16];
                        if (j0 + 16 <= h1) {
#pragma unroll
                            for (int q = 0; q < 4; ++q) {
                                const float4 v = reinterpret_cast<const float4 *>(Ub + j0)[q];
                                u[4 * q] = v.x; u[4 * q + 1] = v.y; u[4 * q + 2] = v.z; u[4 * q + 3] = v.w;
                            }
                        } else {
#pragma unroll
                            for (int k = 0; k < 16; ++k) u[k] = j0 + k < h1 ? Ub[j0 + k] : __int_as_float(0x7fc00000);
                        }
#pragma unroll
                        for (int k = 0; k < 16; ++k) {
                            int idx;
                            const unsigned long long w = hist_pack(u[k], bmin, rinv, bins, idx);
                            atomicAdd(&H[idx], w);
                        }
                    }
                }
                __syncthreads();
                for (int h = t; h < bins; h += ST_TPB) {
                    unsigned long long cs = 0ull, os = 0ull;
#pragma unroll
                    for (int q = 0; q < ST_HC; ++q) {
                        const unsigned long long w = Hc[q * VH_MAX_BINS + h];
                        cs += hist_count(w);
                        os += hist_osum(w);
                    }
                    if (cs) atomicAdd(HS + h, cs);
                    if (os) atomicAdd(HS + VH_MAX_BINS + h, os);
                }
                STG_MARK(1);
                grid.sync();
                STG_MARK(8);
                // the other parity's sums were last read by the previous iteration's E map
                for (int e = r * ST_TPB + t; e < 2 * VH_MAX_BINS; e += G * ST_TPB) HSo[e] = 0ull;
                // ---- emap (k_n4_study's arithmetic on the grid's sums) ----
                {
                    const int P = VH_FFT_P, off = (P - bins) / 2;
                    const float sFWHM = a.fwhm / slope;
                    const float ef = (float)(4.0 * LN2 / (double)(sFWHM * sFWHM));
                    const float sf = (float)(2.0 * sqrt(LN2 / PI_D) / (double)sFWHM);
                    const double2 twv = g.t < P / 2 ? a.tw[g.t] : make_double2(0.0, 0.0);
                    for (int i = g.t; i < P; i += g.n) {
                        const int h = i - off;
                        unsigned long long s = 0ull;
                        if (h >= 0 && h < bins) {
                            s = (HS[h] << 24) - HS[VH_MAX_BINS + h];
                            if (h > 0) s += HS[VH_MAX_BINS + h - 1];
                        }
                        V[fpad(i)] = make_double2((double)s * (1.0 / 16777216.0), 0.0);
                        double fx;
                        if (i == 0) {
                            fx = (double)sf;
                        } else if (i == P / 2) {
                            fx = (double)sf * exp(-0.25 * (double)((float)P * (float)P) * (double)ef);
                        } else {
                            const float nf = (float)(i < P / 2 ? i : P - i);
                            fx = (double)(sf * expf_cr_tail(-(nf * nf) * ef));
                        }
                        F[fpad(i)] = make_double2(fx, 0.0);
                    }
                    if (g.t < P / 2) TW[g.t] = twv;
                    __syncthreads();
                    if (g.w < 2) wave_fft_lds(g.w ? F : V, TW, false, FftId(), FftId());
                    __syncthreads();
                    for (int i = g.t; i < P; i += g.n) {
                        const double2 f = F[fpad(i)], v = V[fpad(i)];
                        const double fa = f.x, fb = f.y;
                        const double gg = fa / ((fa * fa - (-fb) * fb) + (double)a.noise);
                        V[fpad(i)] = make_double2(v.x * gg, v.y * gg);
                    }
                    __syncthreads();
                    if (g.w == 0) wave_fft_lds(V, TW, true, FftId(), FftId());
                    __syncthreads();
                    for (int i = g.t; i < P; i += g.n) {
                        const double ur = V[fpad(i)].x > 0.0 ? V[fpad(i)].x : 0.0;
                        const float c = bmin + ((float)i - (float)off) * slope;
                        DEN[fpad(i)] = make_double2(ur, 0.0);
                        V[fpad(i)] = make_double2((double)c * ur, 0.0);
                    }
                    __syncthreads();
                    if (g.w < 2) wave_fft_lds(g.w ? DEN : V, TW, false, FftId(), FftId());
                    __syncthreads();
                    for (int e = g.t; e < 2 * P; e += g.n) {
                        double2 *const x = e < P ? V : DEN;
                        const int i = e < P ? e : e - P;
                        const double2 f = F[fpad(i)], v = x[fpad(i)];
                        x[fpad(i)] = make_double2(v.x * f.x - v.y * f.y, v.x * f.y + v.y * f.x);
                    }
                    __syncthreads();
                    if (g.w < 2) wave_fft_lds(g.w ? DEN : V, TW, true, FftId(), FftId());
                    __syncthreads();
                    for (int i = g.t; i < bins; i += g.n) {
                        const double d = DEN[fpad(i + off)].x;
                        sE[i] = d != 0.0 ? (float)(V[fpad(i + off)].x / d) : 0.0f;
                    }
                    __syncthreads();
                }
                STG_MARK(2);
                // ---- fit: this workgroup's items into LDS, then into the grid's numerators ----
                for (int e = g.t; e < 2 * nlat; e += g.n) numfix[e] = 0ull;
                if (g.t == 0) M.item_ctr = 0;
                __syncthreads();
                for (;;) {
                    const int item = next_item_g(M, ordr, a.nitems, r, G);
                    if (item < 0) break;
                    Item it;
                    if (!study_item(it, a, b, item)) continue;
                    fit_item<0, true>(it, T, Wk3, Wx3, ncy, ncz, a.Z, bins, Ub, n, sE, bmin, rinv, ring,
                                      a.nb_ring, numfix);
                }
                __syncthreads();
                for (int e = t; e < nlat; e += ST_TPB)
                    fix128_flush(NS + 2 * e, NS + 2 * e + 1, numfix[2 * e], numfix[2 * e + 1]);
                STG_MARK(3);
                grid.sync();
                STG_MARK(8);
                // ---- lattice update and P1 (each workgroup its own copy, from the grid's sums) ----
                for (int e = g.t; e < nlat; e += g.n) {
                    const double d = fix128_get(NSd + 2 * e, NSd + 2 * e + 1);
                    const double num = fix128_get(NS + 2 * e, NS + 2 * e + 1);
                    const float phi = d != 0.0 ? (float)(num / d) : 0.0f;
                    lat[e] += phi;
                }
                // the other parity's numerators were last read by the previous iteration's update
                for (int e = r * ST_TPB + t; e < 2 * nlat; e += G * ST_TPB) NSo[e] = 0ull;
                __syncthreads();
                for (int e = g.t; e < ncx * ncy * a.Z; e += g.n) {
                    const int ij = e / a.Z, z = e % a.Z;
                    const float4 w = T.wz[z];
                    const float *l = lat + ij * ncz + T.bz[z];
                    P1[e] = (double)w.x * (double)l[0] + (double)w.y * (double)l[1] +
                            (double)w.z * (double)l[2] + (double)w.w * (double)l[3];
                }
                if (g.t == 0) M.item_ctr = 0;
                __syncthreads();
                STG_MARK(4);
                // ---- eval: this workgroup's items; U into the other buffer, d in raster order ----
                const int uo = (uin + 1) % ST_NB;
                {
                    float *const Uo = a.U + uo * a.half + b * a.VS;
                    float *const Dw = a.D + b * a.VS;
                    float4 *const rp_out = rpart0 + uo * a.nitems;
                    const bool first_of_level = itk == 1;
                    const bool bo_mode = !(L == 0 && first_of_level);
                    const bool same = !(first_of_level && L > 0);
                    TabV To = T;
                    int ncxo = ncx;
                    if (!same) {
                        const DevLevel &lo = a.lvs->lv[L - 1];
                        To.wx = reinterpret_cast<const float4 *>(lo.ax[0].w);
                        To.bx = lo.ax[0].base;
                        ncxo = lo.ax[0].ncp;
                    }
                    float *const Tgn = Tg0 + (size_t)(tpar ^ 1) * a.tcap;
                    const float *const Tgo = Tg0 + (size_t)tpar * a.tcap;
                    for (;;) {
                        const int item = next_item_g(M, ordr, a.nitems, r, G);
                        if (item < 0) break;
                        Item it;
                        if (!study_item(it, a, b, item)) {
                            if (lane == 0) {
                                gd.ipart[2 * item] = 0.0;
                                gd.ipart[2 * item + 1] = 0.0;
                                rp_out[item] = make_float4(-FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX);
                            }
                            continue;
                        }
#define STG_EVAL(S, CM) eval_item<S, CM>(it, item, a.Z, a.CZ, T, To, ncx, ncy, ncxo, P1, Tgn, Tgo, bo_mode, \
                                         Lb, Uo, Dw, n, gd.ipart, rp_out, pm)
                        if (a.conv_mode == 0) {
                            if (same) STG_EVAL(true, 0);
                            else STG_EVAL(false, 0);
                        } else {
                            if (same) STG_EVAL(true, 1);
                            else STG_EVAL(false, 1);
                        }
#undef STG_EVAL
                    }
                    __syncthreads();
                    publish_range(gd, rpart0 + uo * a.nitems, ordr, a.nitems, uo, r, G);
                }
                STG_MARK(5);
                grid.sync();
                STG_MARK(8);
                if (a.conv_mode == 0) {   // S7: the grid PC over every workgroup, d in raster order
                    Pcg2Args A = gd.pc;
                    A.skip_thresh = itk < a.lvs->max_iters[L] ? a.thresh : 0.0f;
                    A.tag0 = (uint32_t)gi << 12;   // < 4096 scans per call (stage caps 40 + 40 + 48 rounds)
                    const float *const Dr = a.D + b * a.VS;
                    pcg2_body(A, PL, grid, [=](int64_t q) { return Dr[q]; });
                    grid.sync();   // conv_w (one thread's store) to every workgroup
                }
                STG_MARK(6);
                tpar ^= 1;
                uin = uo;
                itn = itk;
                ++gi;
            }
            if (g.t == 0) {
                M.itn = itn;
                M.uin = uin;
            }
        }
        __syncthreads();
        if (r == 0 && t == 0) {
            stb->iters_level[L] = M.itn;
            stb->conv_level[L] = (float)M.conv;
        }
        if (L < a.nlev - 1) {   // exact subdivision of the lattice for the next level (every copy)
            const int nl_max = lvl.ax[0].ncp * lvl.ax[1].ncp * lvl.ax[2].ncp;
            float *T1 = reinterpret_cast<float *>(scr), *T2 = T1 + nl_max;
            refine_axis_st(lat, T1, ncx, ncy, ncz, 0);
            __syncthreads();
            refine_axis_st(T1, T2, 2 * ncx - 3, ncy, ncz, 1);
            __syncthreads();
            refine_axis_st(T2, lat, 2 * ncx - 3, 2 * ncy - 3, ncz, 2);
            __syncthreads();
        }
    }
#ifdef STG_PROF
    STG_MARK(7);
    if (r == 0 && t == 0)
        printf("STG_PROF G %d n %lld its %d ticks(10ns): ctrl %llu hist %llu emap %llu fit %llu lat %llu eval %llu "
               "pc %llu level %llu barriers(hist/fit/eval) %llu\n", G, (long long)n, gi,
               (unsigned long long)stg_p[0], (unsigned long long)stg_p[1], (unsigned long long)stg_p[2],
               (unsigned long long)stg_p[3], (unsigned long long)stg_p[4], (unsigned long long)stg_p[5],
               (unsigned long long)stg_p[6], (unsigned long long)stg_p[7], (unsigned long long)stg_p[8]);
#endif
    if (r == 0) {   // final field's P1 for k_n4_final
        const TabV T = tab_view(smem + a.o_tab, a.R, a.C, a.Z, a.kcap);
        const int ncz = lvl.ax[2].ncp;
        for (int e = t; e < p1last; e += ST_TPB) {
            const int ij = e / a.Z, z = e % a.Z;
            const float4 w = T.wz[z];
            const float *l = lat + ij * ncz + T.bz[z];
            a.P1out[b * a.q2cap + e] = (double)w.x * (double)l[0] + (double)w.y * (double)l[1] +
                                       (double)w.z * (double)l[2] + (double)w.w * (double)l[3];
        }
        if (t == 0) {
            stb->conv = M.conv;
            stb->active = 0;
            stb->t_end = wall_clock64();
        }
    }
    kst_end(gd.pc.kst);
}

// Workgroup -> study, the largest study (most mask == 1 voxels, the best a-priori proxy of its
// cost) first, ties by index: the dispatcher starts workgroups in order, so when the CUs are
// shared with another batch's launch (batches in flight) the long studies start first and the
// launch's tail is its short studies.  One workgroup, rank by counting (nb <= 4096).
// The counts are staged in LDS first (each thread reading all nb counts from global memory, one
// load after another, took 26 us).
__global__ void __launch_bounds__(1024) k_study_order(const VolScalars *sc, int64_t nb, int32_t *order) {
    __shared__ int64_t s_n[4096];
    for (int64_t i = threadIdx.x; i < nb; i += blockDim.x) s_n[i] = sc[i].n_mask1;
    __syncthreads();
    for (int64_t i = threadIdx.x; i < nb; i += blockDim.x) {
        const int64_t ni = s_n[i];
        int32_t r = 0;
        for (int64_t j = 0; j < nb; ++j) {
            const int64_t nj = s_n[j];
            r += (nj > ni) || (nj == ni && j < i);
        }
        order[r] = (int32_t)i;
    }
}

// ---------------------------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------------------------
struct StudyLayout {
    size_t bytes;
    StudyArgs a;
};

// grid = true: the grid form's per-workgroup layout (k_n4_studyg): no item partials of the exact CoV
// in LDS (they go to global memory), no PC area (the grid PC's LDS is static), the budget less that
// static area, and the packed-histogram bound per workgroup (<= V / G values) instead of per study.
static bool study_layout(const vh_batch *b, const vh_n4_params &prm, StudyLayout &out, bool grid = false,
                         int G = 1) {
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
    const size_t emap = sizeof(double2) * (3 * ST_FFT_N + VH_FFT_P / 2);   // (histogram copies in DEN)
    const bool geom_ok = s_cap <= 64 * FIT_SO;   // one ring row's stage-1 outputs fit the lanes
    s_cap = std::max(s_cap, 64);
    const int fit_waves = ST_WAVES;
    // ring rows per wave: up to FIT_NB within ~32 KB
    const int nb_ring = std::max(1, std::min(FIT_NB, (int)(32768 / (fit_waves * 8 * (size_t)s_cap))));
    const size_t fit_num = 2 * sizeof(unsigned long long) * (size_t)nlat_max;
    const size_t fit = ((fit_num + 15) & ~(size_t)15) + sizeof(double) * fit_waves * nb_ring * (size_t)s_cap;
    const size_t exact = sizeof(float) * 2 * ST_TPB;
    const size_t pcs = prm.conv_mode == 0 && !grid ? pcw_lds_bytes<ST_TPB>() : 0;
    const size_t p1 = sizeof(double) * (size_t)p1_max;   // the new field's P1, lattice update to eval
    const size_t scr = std::max({refine, emap, fit, exact, pcs, p1});
    auto A = [](size_t v) { return (v + 15) & ~(size_t)15; };
    size_t o = 0;
    a.o_E = (int32_t)o; o += A(sizeof(float) * VH_MAX_BINS);
    const size_t tb = study_tab_bytes(R, C, Z, kcap);
    a.o_tab = (int32_t)o; o += tb;
    a.o_lat = (int32_t)o; o += A(sizeof(float) * nlat_max);
    const int64_t nslots = (b->R + SLOT_R - 1) / SLOT_R;
    const int64_t nitems = b->n4_tiles * nslots;
    a.o_ipart = (int32_t)o; o += grid ? 0 : A(sizeof(double) * 2 * (size_t)nitems);
    a.o_rpart = (int32_t)o; o += A(sizeof(float4) * ST_NB * (size_t)nitems);
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
    // packed histogram bins stay exact below 2^20 values per workgroup (hist_pack)
    if (grid)
        return geom_ok && o + sizeof(Pcg2Lds) <= ST_MAX_LDS && prm.n_levels <= VH_MAX_LEVELS &&
               (b->V + G - 1) / G + 16 < ((int64_t)1 << 20);
    return geom_ok && o <= ST_MAX_LDS && prm.n_levels <= VH_MAX_LEVELS && b->V < ((int64_t)1 << 20);
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
    a.D = b->d_D;
    a.half = b->nb * b->VS;   // second U / D buffers (vh_ensure_n4_workspace)
    a.rs = b->d_rowstart;
    a.rmask = b->d_rowmask;
    a.rrs = b->d_rrank;
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
    a.conv_mode = prm.conv_mode;
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
                           b->stream));
    a.lvs = (const StudyLevels *)b->d_study_lv;
    a.vol0 = 0;
    a.order = nullptr;
    if (b->nb > 1 && b->nb <= 4096) {
        if (!b->d_study_order) HIP_TRY(hipMalloc(&b->d_study_order, sizeof(int32_t) * b->nb));
        k_study_order<<<1, 1024, 0, b->stream>>>(b->d_sc, b->nb, b->d_study_order);
        VH_CHECK_LAUNCH();
        a.order = b->d_study_order;
    }
    // global state of the study: the fit denominators and the two T-window buffers (the sweep
    // driver's d_den / d_T, vh_ensure_n4_workspace)
    {
        const int Lf = prm.n_levels - 1;
        const int64_t cx = vh_level_ncp(prm, Lf, 0);
        const int64_t nl = cx * vh_level_ncp(prm, Lf, 1) * vh_level_ncp(prm, Lf, 2);
        if (!b->d_den || !b->d_T || b->lat_cap < nl || b->t_cap < cx * b->CZ)
            throw VhError{VH_ERR_ARG, "N4 study kernel: workspace not prepared"};
    }
    a.den = b->d_den;
    a.lat_cap = b->lat_cap;
    a.Tg = b->d_T;
    a.tcap = b->t_cap;
    a.pcdrift = nullptr;
    if (PC_DRIFT) {
        if (!b->d_pcdrift) {
            HIP_TRY(hipMalloc(&b->d_pcdrift, sizeof(float) * ST_TPB * b->nb));
            HIP_TRY(hipMemsetAsync(b->d_pcdrift, 0, sizeof(float) * ST_TPB * b->nb, b->stream));
        }
        a.pcdrift = b->d_pcdrift;
    }
    vh_set_max_lds((const void *)k_n4_study, ST_MAX_LDS);
    size_t lds = Ly.bytes;
    if (const char *e = getenv("VH_ST_MIN_LDS"))   // A/B runs: more LDS than needed, fewer studies per CU
        lds = std::max(lds, std::min((size_t)atoll(e), (size_t)ST_MAX_LDS));
    ScopedKTimer tm(b, "n4_study", 0.0);
    hipStream_t ks = b->stream;
    if (b->st_n4) {   // VH_PRIO: the study kernel on the batch's low-priority stream, in order
        HIP_TRY(hipEventRecord(b->ev_n4_pre, b->stream));
        HIP_TRY(hipStreamWaitEvent(b->st_n4, b->ev_n4_pre, 0));
        ks = b->st_n4;
    }
    k_n4_study<<<(unsigned)b->nb, ST_TPB, lds, ks>>>(a);
    VH_CHECK_LAUNCH();
    if (b->st_n4) {
        HIP_TRY(hipEventRecord(b->ev_n4_post, b->st_n4));
        HIP_TRY(hipStreamWaitEvent(b->stream, b->ev_n4_post, 0));
    }
}

// ---- grid form (k_n4_studyg): one study per cooperative launch of G workgroups ----
// G: about one item per wave (items / 16 workgroups), at most one workgroup per CU (the cooperative
// launch needs the whole grid resident), at least V / 2^20 (the per-workgroup packed histogram).
// VH_STG_G overrides (A/B runs).
static int studyg_workgroups(const vh_batch *b, int nitems) {
    int dev = 0, ncu = 0, per = 0;
    HIP_TRY(hipGetDevice(&dev));
    HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void *)k_n4_studyg, ST_TPB, 0));
    int G = (nitems + ST_WAVES - 1) / ST_WAVES;
    if (const char *e = getenv("VH_STG_G")) G = atoi(e);
    G = std::max<int>(G, (int)((b->V >> 20) + 1));
    // one workgroup per CU at most whatever the occupancy query says (it can report one too many,
    // and a cooperative grid that does not fit would never pass its first barrier)
    G = std::min(G, ncu * std::min(std::max(per, 1), 1));
    return std::max(G, 1);
}

bool vh_n4_studyg_eligible(const vh_batch *b, const vh_n4_params &prm, size_t *lds_bytes) {
    if (b->n4_tiles == 0) return false;
    StudyLayout L0;
    study_layout(b, prm, L0);   // (item count)
    const int G = studyg_workgroups(b, L0.a.nitems);
    StudyLayout L;
    const bool ok = study_layout(b, prm, L, true, G);
    if (lds_bytes) *lds_bytes = L.bytes;
    return ok;
}

void vh_launch_n4_studyg(vh_batch *b, const vh_n4_params &prm) {
    StudyLayout L0;
    study_layout(b, prm, L0);
    const int G = studyg_workgroups(b, L0.a.nitems);
    StudyLayout Ly;
    if (!study_layout(b, prm, Ly, true, G)) throw VhError{VH_ERR_ARG, "N4 grid study kernel: LDS budget exceeded"};
    StudyArgs a = Ly.a;
    a.I = b->d_hp;
    a.V = b->V;
    a.L0 = b->d_L0;
    a.U = b->d_U;
    a.D = b->d_D;
    a.half = b->nb * b->VS;
    a.rs = b->d_rowstart;
    a.rmask = b->d_rowmask;
    a.rrs = b->d_rrank;
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
    a.conv_mode = prm.conv_mode;
    a.thresh = prm.conv_threshold;
    a.fwhm = prm.fwhm;
    a.noise = prm.wiener_noise;
    StudyLevels h{};
    for (int L = 0; L < prm.n_levels; ++L) {
        h.max_iters[L] = prm.max_iters[L];
        h.lv[L] = vh_dev_level(b, prm, L);
    }
    if (!b->d_study_lv) HIP_TRY(hipMalloc(&b->d_study_lv, sizeof(StudyLevels)));
    HIP_TRY(hipMemcpyAsync(b->d_study_lv, &h, sizeof(StudyLevels), hipMemcpyHostToDevice, b->stream));
    a.lvs = (const StudyLevels *)b->d_study_lv;
    a.order = nullptr;
    {
        const int Lf = prm.n_levels - 1;
        const int64_t cx = vh_level_ncp(prm, Lf, 0);
        const int64_t nl = cx * vh_level_ncp(prm, Lf, 1) * vh_level_ncp(prm, Lf, 2);
        if (!b->d_den || !b->d_T || b->lat_cap < nl || b->t_cap < cx * b->CZ)
            throw VhError{VH_ERR_ARG, "N4 grid study kernel: workspace not prepared"};
    }
    a.den = b->d_den;
    a.lat_cap = b->lat_cap;
    a.Tg = b->d_T;
    a.tcap = b->t_cap;
    a.pcdrift = nullptr;
    // per-launch global state: the sums of both parities and the denominators (zeroed here), the
    // range records, the exact-CoV item sums, the grid PC's records / ends / p values
    const int64_t NB = (int64_t)G * PC_TPB;
    auto A256 = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const size_t b_h = A256(sizeof(unsigned long long) * 2 * 2 * VH_MAX_BINS);
    const size_t b_n = A256(sizeof(unsigned long long) * 3 * 2 * (size_t)b->lat_cap);
    const size_t b_r = A256(sizeof(float4) * ST_NB * (size_t)G);
    const size_t b_i = A256(sizeof(double) * 2 * (size_t)std::max<int32_t>(a.nitems, 1));
    const size_t b_w = A256(sizeof(PcgWg) * 2 * (size_t)G);
    const size_t b_g = A256(sizeof(unsigned long long) * 2 * PCG_GW * (size_t)G);   // (zeroed)
    const size_t b_e = A256(sizeof(float) * 2 * (size_t)NB);
    const size_t b_p = A256(sizeof(float) * ((size_t)b->VS + (size_t)NB));   // (L + 1) NB <= n + NB
    const size_t need = b_h + b_n + b_g + b_r + b_i + b_w + b_e + b_p;
    if ((int64_t)need > b->stg_cap) {
        if (b->d_stg) HIP_TRY(hipFree(b->d_stg));
        b->d_stg = nullptr;
        b->stg_cap = 0;
        HIP_TRY(hipMalloc(&b->d_stg, need));
        b->stg_cap = (int64_t)need;
    }
    vh_set_max_lds((const void *)k_n4_studyg, (int)(ST_MAX_LDS - sizeof(Pcg2Lds)));
    for (int64_t v = 0; v < b->nb; ++v) {   // one study per launch (the class and configs 2 / 5: one)
        ScopedKTimer tm(b, "n4_study", 0.0, true);   // stamped: a cooperative launch
        char *w = (char *)b->d_stg;
        StudyGrid gd{};
        gd.hsum = (unsigned long long *)w; w += b_h;
        gd.nsum = (unsigned long long *)w; w += b_n;
        // VH_STG_GRAN=1: the rounds' records as tagged granules instead of through a grid barrier
        // (measured slower, r6e: S7 4.22 vs 3.87 ms per config-2 study; kept for A/B runs)
        gd.pc.gran = (getenv("VH_STG_GRAN") && atoi(getenv("VH_STG_GRAN")) == 1)
                         ? (unsigned long long *)w : nullptr;
        w += b_g;
        gd.pc.tag0 = 0u;
        gd.rrec = (float4 *)w; w += b_r;
        gd.ipart = (double *)w; w += b_i;
        gd.pc.wg = (PcgWg *)w; w += b_w;
        gd.pc.E = (float *)w; w += b_e;
        gd.pc.P = (float *)w;
        gd.pc.D = nullptr;
        gd.pc.perm = nullptr;
        gd.pc.sc = b->d_sc;
        gd.pc.st = b->d_st;
        gd.pc.b = v;
        gd.pc.skip_thresh = 0.0f;
        gd.pc.kst = tm.stamp();
        HIP_TRY(hipMemsetAsync(b->d_stg, 0, b_h + b_n + b_g, b->stream));
        StudyArgs av = a;
        av.vol0 = v;
        void *args[] = {&av, &gd};
        HIP_TRY(hipLaunchCooperativeKernel((const void *)k_n4_studyg, dim3((unsigned)G), dim3(ST_TPB), args,
                                           Ly.bytes, b->stream));
    }
}
