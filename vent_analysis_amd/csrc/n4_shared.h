// Declarations shared by the two N4 drivers: n4.hip (per-iteration sweeps over the whole batch)
// and n4_study.hip (one workgroup per study, the whole level/iteration loop in one launch).
#pragma once
#include "vh_internal.h"

struct DevAxis {
    const int32_t *base;
    const float *w;
    const double *sw2;
    const double *isw2;   // 1 / sw2
    const double *w2;     // [n][4] w^2 (double)
    const double *w3;     // [n][4] w^3 (double)
    const int2 *krange;   // [ncp] first / last index whose support contains control point k
    int32_t n, ncp;
};
struct DevLevel {
    DevAxis ax[3];
    // per 128-column fit tile: {y0, y1, z0, z1} (first/last column's col and slice), then
    // {jlo, JT, klo, KT} (lattice cols / slices the tile's slab covers)
    const int4 *tiles;
    const int2 *jt;   // per lattice col j: first / last tile whose slab covers j
};

#define TILE_W 64   // columns per compact tile (one wave)
#define VH_OOB 0x80000000u
#define N4_FIX 4294967296.0    // 2^32: fixed-point scale of the fit contractions
#define N4_MAGIC 6755399441055744.0   // 1.5 * 2^52: x + MAGIC rounds x to an integer (|x| < 2^51)
#define LN2 0.69314718055994530942
#define PI_D 3.14159265358979323846

int vh_level_ncp(const vh_n4_params &p, int level, int axis);
DevLevel vh_dev_level(const vh_batch *b, const vh_n4_params &prm, int L);

// N4 driver selection (vh_run_opts.n4_mode)
bool vh_n4_study_eligible(const vh_batch *b, const vh_n4_params &prm, size_t *lds_bytes);
void vh_launch_n4_study(vh_batch *b, const vh_n4_params &prm);

// ---- device helpers shared by both drivers ----------------------------------------------------
__device__ __forceinline__ float sharpen_value(float u, float bmin, float slope, const float *E,
                                               int bins) {
    const float cidx = (u - bmin) / slope;
    const int idx = (cidx >= 0.0f && cidx < (float)bins) ? (int)floorf(cidx) : bins;
    if (idx < bins - 1) return E[idx] + (E[idx + 1] - E[idx]) * (cidx - (float)idx);
    return E[bins - 1];
}

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

__device__ __forceinline__ float expf_cr(float x) { return (float)exp((double)x); }

// Histogram bin weights of one U value (triangular Parzen, u64 fixed point 2^-32); same
// expressions as oracle/n4_oracle.c.  Returns false when the value adds nothing.
__device__ __forceinline__ bool parzen_bin(float u, float bmin, float slope, int bins, int &idx,
                                           unsigned long long &a0, unsigned long long &a1) {
    const float cidx = (u - bmin) / slope;   // NaN (padding) fails both range tests
    if (!(cidx >= 0.0f) || !(cidx < (float)bins)) return false;
    idx = (int)floorf(cidx);
    const float o = cidx - (float)idx;
    a1 = 0ull;
    if (o == 0.0f) {
        a0 = 1ull << 32;
    } else if (idx < bins - 1) {
        // both products are < 2^32 (o in (0, 1)), so the single-instruction f64 -> u32
        // conversion truncates exactly like the u64 one; 1 - o rounds to 1 only for tiny o
        const float om = 1.0f - o;
        a0 = om == 1.0f ? (1ull << 32) : (unsigned long long)(uint32_t)((double)om * 4294967296.0);
        a1 = (unsigned long long)(uint32_t)((double)o * 4294967296.0);
    } else {
        return false;
    }
    return true;
}
