// vdp.hip -- post-N4 VDP chain on gfx950 (Vent_Analysis.calculate_VDP, Vent_Analysis.py:239-263),
// calculateBorder (:225-231) and calculate_SNR (:337-357), over a batch of volumes.
//
// Layout: volume b at [b][R][C][Z] (numpy C order, slice axis fastest).  A "column" is one
// (col, slice) pair; column sweeps put one thread per column and walk the rows, so consecutive
// lanes touch consecutive bytes for every row (coalesced).
#include <cfloat>
#include <climits>

#include "vh_internal.h"

// =============================================================================================
// mask statistics (once per batch): per-column masked row range + count, row/col/slice "any"
// flags for calculate_SNR's box (Vent_Analysis.py:344-347), masked counts, first mask==1 voxel.
// =============================================================================================
__global__ void k_init_scalars(VolScalars *sc, int64_t nb) {
    int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (b >= nb) return;
    VolScalars s{};
    s.first_masked = INT64_MAX;
    sc[b] = s;
}

// One pass over the mask in 32-row slabs (one bitmap word) x 4 columns per lane (a 32-bit load
// per row: 256 B per wave).  Writes the slab's bitmap words of mask == 1 (N4 label) and mask != 0
// (VDP / SNR mask), the row "any" flags, and per volume the masked counts and the first mask == 1
// voxel (atomics on integers: order-free).  The four bytes of a row word are tested together (SWAR:
// bit 7 of each byte) and gathered 8 rows at a time before they are spread into the column words.
// k_mask_cols then derives each column's masked row range and count from the mask != 0 words;
// the column / slice flags come from those counts in k_mask_finish (one byte store per masked column
// and slab into a volume's one or two flag lines made this kernel 3x slower than its loads).
template <int CPL, bool VEC>
__global__ void __launch_bounds__(VH_TPB) k_mask_stats(const uint8_t *__restrict__ mask, int64_t R,
                                                      int64_t C, int64_t Z, int64_t V, int64_t ncb,
                                                      uint32_t *colbits, uint32_t *colbnz,
                                                      uint8_t *rowany, VolScalars *sc) {
    constexpr int NW4 = CPL / 4;   // 32-bit words of a lane's row (VEC: one 4- or 16-byte load)
    __shared__ uint32_t s_row;
    __shared__ unsigned long long s_n, s_n1, s_first;
    const int64_t b = blockIdx.y;
    const int64_t CZ = C * Z;
    const int64_t sl = blockIdx.x / ncb;
    const int64_t c0 = ((blockIdx.x % ncb) * VH_TPB + threadIdx.x) * CPL;
    const int64_t x0 = sl * VH_SLAB;
    const int nr = (int)(R - x0 < VH_SLAB ? R - x0 : VH_SLAB);
    if (threadIdx.x == 0) { s_row = 0u; s_n = 0; s_n1 = 0; s_first = ULLONG_MAX; }
    __syncthreads();
    uint32_t w1[CPL], wn[CPL];
#pragma unroll
    for (int q = 0; q < CPL; ++q) { w1[q] = 0u; wn[q] = 0u; }
    const int nc = c0 < CZ ? (int)(CZ - c0 < CPL ? CZ - c0 : CPL) : 0;
    if (nc) {
        const uint8_t *m = mask + b * V + x0 * CZ + c0;
        uint32_t mv[VH_SLAB][NW4];   // the slab's 32 row loads all in flight
#pragma unroll
        for (int k = 0; k < VH_SLAB; ++k) {
#pragma unroll
            for (int j = 0; j < NW4; ++j) mv[k][j] = 0u;
            if (k < nr) {
                const uint8_t *p = m + (int64_t)k * CZ;
                if (VEC) {
                    if (NW4 == 4) {
                        const uint4 u = *reinterpret_cast<const uint4 *>(p);
                        mv[k][0] = u.x; mv[k][NW4 > 1 ? 1 : 0] = u.y;
                        mv[k][NW4 > 2 ? 2 : 0] = u.z; mv[k][NW4 > 3 ? 3 : 0] = u.w;
                    } else {
                        mv[k][0] = *reinterpret_cast<const uint32_t *>(p);
                    }
                } else {
                    for (int q = 0; q < nc; ++q) mv[k][0] |= (uint32_t)p[q] << (8 * q);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < NW4; ++j) {
#pragma unroll
            for (int g = 0; g < VH_SLAB / 8; ++g) {
                uint32_t a1 = 0u, an = 0u;   // byte q, bit r: row 8g + r of column 4j + q
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    uint32_t x = mv[8 * g + r][j];
                    asm volatile("" : "+v"(x));   // keeps the word a word (else the byte tests become i8 vectors: 14x the code, scratch)
                    const uint32_t y = x ^ 0x01010101u;
                    const uint32_t nz = (((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
                    const uint32_t ne1 = (((y & 0x7f7f7f7fu) + 0x7f7f7f7fu) | y) & 0x80808080u;
                    an |= (nz >> 7) << r;
                    a1 |= ((ne1 ^ 0x80808080u) >> 7) << r;
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    wn[4 * j + q] |= ((an >> (8 * q)) & 0xFFu) << (8 * g);
                    w1[4 * j + q] |= ((a1 >> (8 * q)) & 0xFFu) << (8 * g);
                }
            }
        }
        const int64_t nw = (R + 31) >> 5;
        uint32_t *cb = colbits + (b * nw + sl) * CZ + c0, *cn = colbnz + (b * nw + sl) * CZ + c0;
        if (VEC) {
#pragma unroll
            for (int j = 0; j < NW4; ++j) {
                *reinterpret_cast<uint4 *>(cb + 4 * j) = make_uint4(w1[4 * j], w1[4 * j + 1], w1[4 * j + 2], w1[4 * j + 3]);
                *reinterpret_cast<uint4 *>(cn + 4 * j) = make_uint4(wn[4 * j], wn[4 * j + 1], wn[4 * j + 2], wn[4 * j + 3]);
            }
        } else {
            for (int q = 0; q < nc; ++q) { cb[q] = w1[q]; cn[q] = wn[q]; }
        }
    }
    unsigned long long n = 0, n1 = 0, first = ULLONG_MAX;
    uint32_t rows = 0u;
#pragma unroll
    for (int q = 0; q < CPL; ++q) {   // words past nc are 0
        n += (unsigned)__popc(wn[q]);
        n1 += (unsigned)__popc(w1[q]);
        rows |= wn[q];
        if (w1[q]) {
            const unsigned long long idx =
                (unsigned long long)((x0 + __builtin_ctz(w1[q])) * CZ + c0 + q);
            if (idx < first) first = idx;
        }
    }
    if (rows) atomicOr(&s_row, rows);
    if (n) atomicAdd(&s_n, n);
    if (n1) atomicAdd(&s_n1, n1);
    if (first != ULLONG_MAX) atomicMin(&s_first, first);
    __syncthreads();
    if ((int)threadIdx.x < nr && ((s_row >> threadIdx.x) & 1u)) rowany[b * R + x0 + threadIdx.x] = 1;
    if (threadIdx.x == 0) {
        if (s_n) atomicAdd((unsigned long long *)&sc[b].n_mask, s_n);
        if (s_n1) atomicAdd((unsigned long long *)&sc[b].n_mask1, s_n1);
        if (s_first != ULLONG_MAX) atomicMin((unsigned long long *)&sc[b].first_masked, s_first);
    }
}

// each column's masked (mask != 0) row range [lo, hi] (lo = R, hi = -1 when empty) and count; the
// column's bitmap words load 8 at a time (clamped index: all in flight)
__global__ void __launch_bounds__(VH_TPB) k_mask_cols(const uint32_t *colbnz, int64_t R, int64_t CZ,
                                                     int32_t *colrange, int32_t *colcount) {
    const int64_t b = blockIdx.y;
    const int64_t col = blockIdx.x * (int64_t)VH_TPB + threadIdx.x;
    if (col >= CZ) return;
    const int64_t nw = (R + 31) >> 5;
    int32_t lo = (int32_t)R, hi = -1, n = 0;
    for (int64_t w0 = 0; w0 < nw; w0 += 8) {
        uint32_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = colbnz[(b * nw + (w0 + k < nw ? w0 + k : nw - 1)) * CZ + col];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t x = w0 + k < nw ? v[k] : 0u;
            if (!x) continue;
            n += __popc(x);
            if (lo == (int32_t)R) lo = (int32_t)((w0 + k) * 32 + __builtin_ctz(x));
            hi = (int32_t)((w0 + k) * 32 + 31 - __builtin_clz(x));
        }
    }
    colrange[(b * CZ + col) * 2] = lo;
    colrange[(b * CZ + col) * 2 + 1] = hi;
    colcount[b * CZ + col] = n;
}

// exclusive prefix of the per-column masked counts (compaction offsets for the sort keys), the
// column / slice flags from the counts and the SNR box parameters.  One block per volume; the
// counts stream through LDS in tiles of MF_TILE (coalesced loads, all in flight; each thread scans
// 16 consecutive counts; coalesced colstart stores).  Flags go to LDS bitmaps when C, Z <= 32768,
// else straight to the global flag arrays.
#define MF_TILE (VH_TPB * 16)
#define MF_FLAGW 1024
__device__ __forceinline__ int64_t mf_block_excl(int64_t v, int64_t *s_w, int64_t &total) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    int64_t inc = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int64_t o = __shfl_up(inc, off, 64);
        if (lane >= off) inc += o;
    }
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    int64_t pre = 0;
    total = 0;
#pragma unroll
    for (int q = 0; q < VH_TPB / 64; ++q) {
        const int64_t x = s_w[q];
        if (q < w) pre += x;
        total += x;
    }
    __syncthreads();
    return pre + inc - v;
}

__global__ void __launch_bounds__(VH_TPB) k_mask_finish(const int32_t *colcount, int64_t *colstart,
                                                       const uint8_t *rowany, uint8_t *colany,
                                                       uint8_t *sliceany, int64_t R,
                                                       int64_t C, int64_t Z, VolScalars *sc) {
    __shared__ int32_t s_cnt[MF_TILE];
    __shared__ int64_t s_ex[MF_TILE];
    __shared__ int64_t s_w[VH_TPB / 64];
    __shared__ uint32_t s_cf[MF_FLAGW], s_sf[MF_FLAGW];
    __shared__ int32_t s_cmin, s_cmax, s_rowe, s_slie, s_rlo, s_rhi;
    const int64_t b = blockIdx.x;
    const int64_t CZ = C * Z;
    const int t = threadIdx.x;
    const bool lf = C <= 32 * MF_FLAGW && Z <= 32 * MF_FLAGW;
    for (int i = t; i < MF_FLAGW; i += VH_TPB) { s_cf[i] = 0u; s_sf[i] = 0u; }
    if (t == 0) { s_cmin = INT_MAX; s_cmax = 0; s_rowe = 0; s_slie = 0; s_rlo = INT_MAX; s_rhi = -1; }
    __syncthreads();
    const int32_t *cc = colcount + b * CZ;
    int64_t base = 0;
    for (int64_t c0 = 0; c0 < CZ; c0 += MF_TILE) {
        int32_t v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int64_t i = c0 + k * VH_TPB + t;
            v[k] = cc[i < CZ ? i : CZ - 1];
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int64_t i = c0 + k * VH_TPB + t;
            const int32_t x = i < CZ ? v[k] : 0;
            s_cnt[k * VH_TPB + t] = x;
            if (x) {   // 32-bit division (CZ < 2^31, check_dims)
                const uint32_t y = (uint32_t)i / (uint32_t)Z, z = (uint32_t)i - y * (uint32_t)Z;
                if (lf) {
                    atomicOr(&s_cf[y >> 5], 1u << (y & 31));
                    atomicOr(&s_sf[z >> 5], 1u << (z & 31));
                } else {
                    colany[b * C + y] = 1;
                    sliceany[b * Z + z] = 1;
                }
            }
        }
        __syncthreads();
        int32_t own[16];
        int64_t acc = 0;
#pragma unroll
        for (int q = 0; q < 16; ++q) { own[q] = s_cnt[16 * t + q]; acc += own[q]; }
        int64_t tot;
        int64_t run = base + mf_block_excl(acc, s_w, tot);
#pragma unroll
        for (int q = 0; q < 16; ++q) { s_ex[16 * t + q] = run; run += own[q]; }
        __syncthreads();
        const int64_t cn = CZ - c0 < MF_TILE ? CZ - c0 : MF_TILE;
        for (int k = t; k < cn; k += VH_TPB) colstart[b * CZ + c0 + k] = s_ex[k];
        base += tot;
        __syncthreads();
    }
    if (lf) {
        for (int64_t wi = t; wi < (C + 31) / 32; wi += VH_TPB) {
            const uint32_t x = s_cf[wi], xm = wi == 0 ? x & ~1u : x;   // column 0 counts for cmax only
            if (xm) atomicMin(&s_cmin, (int32_t)(wi * 32 + __builtin_ctz(xm)));
            if (x) atomicMax(&s_cmax, (int32_t)(wi * 32 + 31 - __builtin_clz(x)));
        }
        for (int64_t z = t; z < Z; z += VH_TPB) {
            const uint8_t f = (uint8_t)((s_sf[z >> 5] >> (z & 31)) & 1u);
            sliceany[b * Z + z] = f;
            if (!f) s_slie = 1;
        }
    } else {
        for (int64_t c = t; c < C; c += VH_TPB)
            if (colany[b * C + c]) {
                if (c > 0) atomicMin(&s_cmin, (int32_t)c);
                atomicMax(&s_cmax, (int32_t)c);
            }
        for (int64_t z = t; z < Z; z += VH_TPB)
            if (!sliceany[b * Z + z]) s_slie = 1;
    }
    for (int64_t r = t; r < R; r += VH_TPB) {
        if (!rowany[b * R + r]) s_rowe = 1;
        else {
            atomicMin(&s_rlo, (int32_t)r);
            atomicMax(&s_rhi, (int32_t)r);
        }
    }
    __syncthreads();
    if (t == 0) {
        sc[b].cmin = s_cmin;
        sc[b].cmax = s_cmax;
        sc[b].any_row_empty = s_rowe;
        sc[b].any_slice_empty = s_slie;
        sc[b].snr_ok = s_cmin != INT_MAX;
        sc[b].row_lo = s_rlo;
        sc[b].row_hi = s_rhi;
    }
}

void vh_launch_mask_stats(vh_batch *b) {
    hipStream_t st = b->stream;
    b->snr_fused = false;
    HIP_TRY(hipMemsetAsync(b->d_rowany, 0, b->nb * b->R, st));
    HIP_TRY(hipMemsetAsync(b->d_colany, 0, b->nb * b->C, st));
    HIP_TRY(hipMemsetAsync(b->d_sliceany, 0, b->nb * b->Z, st));
    k_init_scalars<<<(unsigned)((b->nb + 255) / 256), 256, 0, st>>>(b->d_sc, b->nb);
    VH_CHECK_LAUNCH();
    {
        ScopedKTimer tm(b, "mask_stats", (double)b->V);
        // 16 columns per lane (16-byte row loads) when CZ % 16 == 0, else 4 (4-byte or byte loads)
        const int cpl = (b->CZ & 15) == 0 ? 16 : 4;
        const int64_t ncb = (b->CZ + cpl * VH_TPB - 1) / (cpl * VH_TPB);
        const dim3 grid((unsigned)(ncb * ((b->R + VH_SLAB - 1) / VH_SLAB)), (unsigned)b->nb);
        auto fn = cpl == 16 ? k_mask_stats<16, true> : (b->CZ & 3) == 0 ? k_mask_stats<4, true> : k_mask_stats<4, false>;
        fn<<<grid, VH_TPB, 0, st>>>(b->d_mask, b->R, b->C, b->Z, b->V, ncb, b->d_colbits,
                                    b->d_colbnz, b->d_rowany, b->d_sc);
        VH_CHECK_LAUNCH();
        k_mask_cols<<<col_grid(b), VH_TPB, 0, st>>>(b->d_colbnz, b->R, b->CZ, b->d_colrange,
                                                   b->d_colcount);
        VH_CHECK_LAUNCH();
    }
    k_mask_finish<<<(unsigned)b->nb, VH_TPB, 0, st>>>(b->d_colcount, b->d_colstart, b->d_rowany,
                                                      b->d_colany, b->d_sliceany, b->R, b->C,
                                                      b->Z, b->d_sc);
    VH_CHECK_LAUNCH();
}

// =============================================================================================
// masked gather -> sortable uint32 keys, compacted column by column (order is irrelevant: sorted
// next; only the multiset matters, Vent_Analysis.py:245).
// =============================================================================================
__global__ void __launch_bounds__(VH_TPB) k_gather(const float *__restrict__ n4,
                                                  const uint8_t *__restrict__ mask,
                                                  const int32_t *colrange, const int64_t *colstart,
                                                  int64_t CZ, int64_t V, const VolScalars *sc,
                                                  int skip_binary, uint32_t *keys) {
    const int64_t b = blockIdx.y;
    if (skip_binary && sc[b].n_mask == sc[b].n_mask1) return;   // keys written by k_n4_final
    const int64_t col = blockIdx.x * (int64_t)VH_TPB + threadIdx.x;
    if (col >= CZ) return;
    const int32_t lo = colrange[(b * CZ + col) * 2], hi = colrange[(b * CZ + col) * 2 + 1];
    int64_t pos = b * V + colstart[b * CZ + col];
    const float *p = n4 + b * V + col;
    const uint8_t *m = mask + b * V + col;
    for (int64_t x0 = lo; x0 <= hi; x0 += 8) {   // 8 rows of mask and value loads in flight
        uint8_t mk[8];
        float v[8];
        // unconditional loads at a clamped row (a guarded load compiles to a branch that waits for
        // it: the mask-then-value chain took 0.55 ms per batch)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int64_t x = x0 + k <= hi ? x0 + k : hi;
            mk[k] = m[x * CZ];
            v[k] = p[x * CZ];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) mk[k] = x0 + k <= hi ? mk[k] : 0;
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (mk[k]) keys[pos++] = f2key(v[k]);
    }
}

// =============================================================================================
// Stable LSD radix sort (4 x 8-bit digits) of each volume's masked keys, ONE workgroup (1024
// threads) per volume: a volume's keys
// (~330 KB at 128x128x24) stay in L2 / MALL, the four digit histograms come from one read pass
// (digit counts do not depend on order), and each pass ranks chunks of VS_CHUNK keys in order
// (wave ballots within a wave, wave prefixes per digit across waves, running digit offsets
// across chunks) -- one launch for the whole sort instead of 12, all volumes in parallel.
// =============================================================================================
#define VS_TPB 1024
#define VS_WAVES (VS_TPB / 64)
#ifndef VS_KPT
#define VS_KPT 12   // keys per lane per chunk (8: 0.51 ms per bench step, 16: 0.47, r4c; with the LDS lane-set
                    // ranking 12: 0.320-0.322 against 16: 0.331-0.335 ms and no VGPR spills, r6an)
#endif
#define VS_CHUNK (VS_TPB * VS_KPT)

// peers of this lane's digit among the wave's valid lanes (8 ballots)
__device__ __forceinline__ uint64_t vs_peers(uint32_t d, bool valid) {
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int bit = 0; bit < 8; ++bit) {
        const uint64_t bb = __ballot(valid && ((d >> bit) & 1u));
        peers &= ((d >> bit) & 1u) ? bb : ~bb;
    }
    return peers;
}

#ifndef VS_MATCH_LDS
#define VS_MATCH_LDS 1
#endif
// the same set through a per-wave LDS table of 64-bit lane sets (3 LDS instructions instead of 8
// ballots and their 64-bit merges): every lane ORs its bit into its digit's entry, reads the entry
// back and clears it.  A wave's LDS instructions execute in order, so the read sees the whole row's
// ORs and the next row's ORs see the clear; invalid lanes use the spare entry 256.
__device__ __forceinline__ uint64_t vs_peers_lds(unsigned long long *m, uint32_t d, bool valid, int lane) {
    unsigned long long *e = m + (valid ? d : 256u);
    __hip_atomic_fetch_or(e, 1ull << lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    const uint64_t p = __hip_atomic_load(e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    __hip_atomic_store(e, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    return valid ? p : 0ull;
}
#if VS_MATCH_LDS
#define VS_PEERS(d, valid) vs_peers_lds(&s_match[w][0], d, valid, lane)
#define VS_MATCH_DECL __shared__ unsigned long long s_match[VS_WAVES][257]
#define VS_MATCH_INIT for (int i_ = lane; i_ < 257; i_ += 64) s_match[w][i_] = 0ull
#else
#define VS_PEERS(d, valid) vs_peers(d, valid)
#define VS_MATCH_DECL
#define VS_MATCH_INIT
#endif

__global__ void __launch_bounds__(VS_TPB) k_sort_vol(uint32_t *__restrict__ k0,
                                                    uint32_t *__restrict__ k1,
                                                    const VolScalars *sc, int64_t V) {
    __shared__ uint32_t s_hist[4][256];      // digit counts -> digit bases
    __shared__ uint32_t s_wc[VS_WAVES][256]; // per-wave digit counts -> per-wave digit offsets
    __shared__ uint32_t s_run[256];          // keys of each digit placed by earlier chunks
    __shared__ uint32_t s_tot[256], s_cst[256], s_wsum[4];   // chunk digit totals / starts
    __shared__ uint32_t s_stage[VS_CHUNK + 1];   // the chunk in digit order (+ a slot for invalid keys)
    __shared__ uint32_t s_off[256];              // digit d's output position minus its chunk-local start
    VS_MATCH_DECL;
    const int64_t b = blockIdx.x;
    const int64_t n = sc[b].n_mask;
    if (n <= 1) return;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int i = t; i < 4 * 256; i += VS_TPB) (&s_hist[0][0])[i] = 0u;
    VS_MATCH_INIT;
    __syncthreads();
    uint32_t *kin = k0 + b * V, *kout = k1 + b * V;
#ifdef VS_PROF
    uint64_t vp[7] = {0, 0, 0, 0, 0, 0, 0}, vrank[4] = {0, 0, 0, 0};
    uint32_t vor = 0u, vfirst = n > 0 ? k0[b * V] : 0u;
    uint64_t vq = wall_clock64();
#define VS_STAMP(k) do { if (t == 0) { const uint64_t x_ = wall_clock64(); vp[k] += x_ - vq; vq = x_; } } while (0)
#else
#define VS_STAMP(k) do { } while (0)
#endif
    // ---- the four digit histograms (one add per row when a row shares its digit); each wave
    // loads VS_KPT rows of 64 keys at a time, so one memory round trip covers 8 rows ----
    for (int64_t i0 = (int64_t)w * (VS_KPT * 64); i0 < n; i0 += (int64_t)VS_TPB * VS_KPT) {
        uint32_t kr[VS_KPT];
#pragma unroll
        for (int r = 0; r < VS_KPT; ++r) {
            const int64_t i = i0 + r * 64 + lane;
            kr[r] = i < n ? kin[i] : 0u;
        }
#pragma unroll
        for (int r = 0; r < VS_KPT; ++r) {
            const bool valid = i0 + r * 64 + lane < n;
#ifdef VS_PROF
            if (valid) vor |= kr[r] ^ vfirst;
#endif
            // valid lanes are a prefix of the row, so lane 0's key stands for the row when any is
            // valid.  Digits 0 and 1 nearly always differ inside a row: plain adds, no test.  Digit
            // 3 nearly always agrees: one row test and one add of the row's count; digit 2 takes
            // the same test and either path.  (Round 6: four shuffle-and-vote tests per row, one
            // per digit, made this pass the sort's costliest after the ranking.)
            const uint32_t kk = kr[r];
            const uint64_t vmask = __ballot(valid);
            const uint32_t k0r = (uint32_t)__builtin_amdgcn_readfirstlane((int)kk);
            const uint32_t cnt = (uint32_t)__popcll(vmask);
            if (valid) {
                atomicAdd(&s_hist[0][kk & 255u], 1u);
                atomicAdd(&s_hist[1][(kk >> 8) & 255u], 1u);
            }
            const bool same3 = __ballot(valid && (kk >> 24) != (k0r >> 24)) == 0ull;
            const bool same2 = __ballot(valid && ((kk >> 16) & 255u) != ((k0r >> 16) & 255u)) == 0ull;
            if (same3) {
                if (lane == 0 && cnt) atomicAdd(&s_hist[3][k0r >> 24], cnt);
            } else if (valid) {
                atomicAdd(&s_hist[3][kk >> 24], 1u);
            }
            if (same2) {
                if (lane == 0 && cnt) atomicAdd(&s_hist[2][(k0r >> 16) & 255u], cnt);
            } else if (valid) {
                atomicAdd(&s_hist[2][(kk >> 16) & 255u], 1u);
            }
        }
    }
    __syncthreads();
    VS_STAMP(0);
    if (t < 4) {   // exclusive scan per digit position
        uint32_t run = 0;
        for (int d = 0; d < 256; ++d) { const uint32_t v = s_hist[t][d]; s_hist[t][d] = run; run += v; }
    }
    __syncthreads();
    for (int p = 0; p < 4; ++p) {
        const int shift = 8 * p;
        if (t < 256) s_run[t] = 0u;
        for (int64_t c0 = 0; c0 < n; c0 += VS_CHUNK) {
            for (int d = lane; d < 256; d += 64) s_wc[w][d] = 0u;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            uint32_t key[VS_KPT], rank[VS_KPT];
#pragma unroll
            for (int r = 0; r < VS_KPT; ++r) {   // all loads first: the ranking below is fenced
                const int64_t idx = c0 + (int64_t)w * (VS_KPT * 64) + r * 64 + lane;
                key[r] = idx < n ? kin[idx] : 0u;
            }
#ifdef VS_PROF
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            VS_STAMP(6);
#endif
#pragma unroll
            for (int r = 0; r < VS_KPT; ++r) {   // wave w owns keys [c0 + 64 VS_KPT w, c0 + 64 VS_KPT (w + 1))
                const int64_t idx = c0 + (int64_t)w * (VS_KPT * 64) + r * 64 + lane;
                const bool valid = idx < n;
                const uint32_t kk = key[r];
                const uint32_t d = (kk >> shift) & 255u;
                // a row that shares one digit (typical of high digits) needs no match ballots (lane
                // 0 is valid whenever any lane is: valid lanes are a prefix of the row)
                const uint32_t d0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)d);
                const uint64_t peers = __all(!valid || d == d0) ? __ballot(valid) : VS_PEERS(d, valid);
                const uint32_t below = (uint32_t)__popcll(peers & lt);
                // the digit group's leader reserves its slots with a returning LDS add (a wave's
                // LDS atomics complete in issue order, so rows stay ordered) and hands the base
                // to its peers
                uint32_t base = 0u;
                if (valid && below == 0) base = atomicAdd(&s_wc[w][d], (uint32_t)__popcll(peers));
                const int leader = peers ? __builtin_ctzll(peers) : lane;
                base = (uint32_t)__shfl((int)base, leader, 64);
                key[r] = kk;
                rank[r] = valid ? base + below : 0xffffffffu;
            }
            __syncthreads();
#ifdef VS_PROF
            if (t == 0) { const uint64_t x_ = wall_clock64(); vrank[p] += x_ - vq; }
#endif
            VS_STAMP(1);
            if (t < 256) {   // digit t: chunk-local wave prefixes and chunk total, then a scan of
                             // the totals over digits (wave shuffles + wave sums)
                uint32_t tot = 0;
                uint32_t wcv[VS_WAVES];
#pragma unroll
                for (int ww = 0; ww < VS_WAVES; ++ww) wcv[ww] = s_wc[ww][t];   // loads together
#pragma unroll
                for (int ww = 0; ww < VS_WAVES; ++ww) { s_wc[ww][t] = tot; tot += wcv[ww]; }
                uint32_t inc = tot;
                for (int off = 1; off < 64; off <<= 1) {
                    const uint32_t o = __shfl_up(inc, off, 64);
                    if (lane >= off) inc += o;
                }
                if (lane == 63) s_wsum[w] = inc;
                s_tot[t] = tot;
                s_cst[t] = inc - tot;   // exclusive within this wave of digits
            }
            __syncthreads();
            VS_STAMP(2);
            if (t < 256) {
                uint32_t pre = 0;
                for (int ww = 0; ww < w; ++ww) pre += s_wsum[ww];
                s_cst[t] += pre;        // chunk-local start of digit t
                s_off[t] = s_hist[p][t] + s_run[t] - s_cst[t];
            }
            __syncthreads();
            VS_STAMP(3);
            // stage at the chunk-local sorted position; branch-free (an invalid key goes to the spare
            // slot), so the rows' LDS reads issue together instead of one row's after another's
#pragma unroll
            for (int r = 0; r < VS_KPT; ++r) {
                const uint32_t d = (key[r] >> shift) & 255u;
                rank[r] = rank[r] == 0xffffffffu ? (uint32_t)VS_CHUNK : s_cst[d] + s_wc[w][d] + rank[r];
            }
#pragma unroll
            for (int r = 0; r < VS_KPT; ++r) s_stage[rank[r]] = key[r];
            __syncthreads();
            VS_STAMP(4);
            // write out in staged order: equal digits are consecutive, so are their targets
            const int cn = (int)(n - c0 < VS_CHUNK ? n - c0 : VS_CHUNK);
            for (int q = t; q < cn; q += VS_TPB) {
                const uint32_t kk = s_stage[q];
                kout[s_off[(kk >> shift) & 255u] + (uint32_t)q] = kk;
            }
            __syncthreads();
            VS_STAMP(5);
            if (t < 256) s_run[t] += s_tot[t];
        }
        uint32_t *tmp = kin; kin = kout; kout = tmp;
        __syncthreads();   // this pass's stores before the next pass's loads (same workgroup)
    }
#ifdef VS_PROF
    if (t == 0 && b < 4)
        printf("VSPROF b=%d n=%ld hist=%lu load=%lu rank=%lu scan=%lu pre=%lu stage=%lu write=%lu rank/pass %lu %lu %lu %lu varbits(t0) %08x\n", (int)b,
               (long)n, (unsigned long)vp[0], (unsigned long)vp[6], (unsigned long)vp[1], (unsigned long)vp[2],
               (unsigned long)vp[3], (unsigned long)vp[4], (unsigned long)vp[5], (unsigned long)vrank[0],
               (unsigned long)vrank[1], (unsigned long)vrank[2], (unsigned long)vrank[3], vor);
#endif
#undef VS_STAMP
}

// ---------------------------------------------------------------------------------------------
// The same stable LSD sort over the whole GPU for ONE large volume (config 5: ~28 M keys, where the
// one-workgroup sort took 118 ms).  Per 8-bit pass: k_sortg_count (one workgroup per VSG_CHUNK-key chunk:
// the chunk's digit counts), k_sortg_offsets (one workgroup: per digit, the exclusive prefix over
// chunks in chunk order plus the digit's base), k_sortg_scatter (one workgroup per chunk: the
// chunk ranked exactly as k_sort_vol ranks it, written at its chunk's digit offsets).  Chunk c of
// every pass holds keys [VSG_CHUNK c, VSG_CHUNK (c + 1)), so the order of equal digits is the input order:
// stable, and the result is the same array k_sort_vol produces.
// ---------------------------------------------------------------------------------------------
// the grid sort keeps 16 keys per lane per chunk: with k_sort_vol's 12 its per-digit chunk offsets
// (k_sortg_offsets, one workgroup, serial over the chunks) took config 5's sort 1.18 -> 1.38 ms (r6ao)
#define VSG_KPT 16
#define VSG_CHUNK (VS_TPB * VSG_KPT)
__global__ void __launch_bounds__(VS_TPB) k_sortg_count(const uint32_t *__restrict__ kin,
                                                       const VolScalars *sc, int64_t b, int shift,
                                                       uint32_t *cnt) {
    __shared__ uint32_t s_c[256];
    const int64_t n = sc[b].n_mask;
    const int64_t c0 = (int64_t)blockIdx.x * VSG_CHUNK;
    if (n <= 1 || c0 >= n) return;
    const int t = threadIdx.x;
    if (t < 256) s_c[t] = 0u;
    __syncthreads();
    uint32_t kr[VSG_KPT];
#pragma unroll
    for (int r = 0; r < VSG_KPT; ++r) {
        const int64_t i = c0 + (int64_t)r * VS_TPB + t;
        kr[r] = i < n ? kin[i] : 0u;
    }
#pragma unroll
    for (int r = 0; r < VSG_KPT; ++r)
        if (c0 + (int64_t)r * VS_TPB + t < n) atomicAdd(&s_c[(kr[r] >> shift) & 255u], 1u);
    __syncthreads();
    if (t < 256) cnt[(int64_t)blockIdx.x * 256 + t] = s_c[t];
}

__global__ void __launch_bounds__(VS_TPB) k_sortg_offsets(uint32_t *cnt, const VolScalars *sc,
                                                         int64_t b) {
    // thread (q, d): digit d = t & 255 over the q-th quarter of the chunks; cnt -> offsets in place
    __shared__ uint32_t s_q[4][256];
    __shared__ uint32_t s_base[256];
    const int64_t n = sc[b].n_mask;
    if (n <= 1) return;
    const int64_t nch = (n + VSG_CHUNK - 1) / VSG_CHUNK;
    const int t = threadIdx.x, d = t & 255, q = t >> 8;
    const int64_t per = (nch + 3) / 4, lo = min(nch, q * per), hi = min(nch, lo + per);
    uint32_t sum = 0;
    for (int64_t c = lo; c < hi; ++c) sum += cnt[c * 256 + d];
    s_q[q][d] = sum;
    __syncthreads();
    if (t < 256) {   // digit totals, bases by a serial scan over digits (256 adds)
        uint32_t tot = s_q[0][t] + s_q[1][t] + s_q[2][t] + s_q[3][t];
        s_base[t] = tot;
    }
    __syncthreads();
    if (t == 0) {
        uint32_t run = 0;
        for (int dd = 0; dd < 256; ++dd) { const uint32_t v = s_base[dd]; s_base[dd] = run; run += v; }
    }
    __syncthreads();
    uint32_t run = s_base[d];
    for (int qq = 0; qq < q; ++qq) run += s_q[qq][d];
    for (int64_t c = lo; c < hi; ++c) {
        const uint32_t v = cnt[c * 256 + d];
        cnt[c * 256 + d] = run;
        run += v;
    }
}

__global__ void __launch_bounds__(VS_TPB) k_sortg_scatter(const uint32_t *__restrict__ kin,
                                                         uint32_t *__restrict__ kout,
                                                         const uint32_t *off, const VolScalars *sc,
                                                         int64_t b, int shift) {
    __shared__ uint32_t s_wc[VS_WAVES][256];
    __shared__ uint32_t s_tot[256], s_cst[256], s_wsum[4], s_off[256];
    __shared__ uint32_t s_stage[VSG_CHUNK];
    VS_MATCH_DECL;
    const int64_t n = sc[b].n_mask;
    const int64_t c0 = (int64_t)blockIdx.x * VSG_CHUNK;
    if (n <= 1 || c0 >= n) return;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int d = lane; d < 256; d += 64) s_wc[w][d] = 0u;
    if (t < 256) s_off[t] = off[(int64_t)blockIdx.x * 256 + t];
    VS_MATCH_INIT;
    __syncthreads();
    uint32_t key[VSG_KPT], rank[VSG_KPT];
#pragma unroll
    for (int r = 0; r < VSG_KPT; ++r) {
        const int64_t idx = c0 + (int64_t)w * (VSG_KPT * 64) + r * 64 + lane;
        key[r] = idx < n ? kin[idx] : 0u;
    }
#pragma unroll
    for (int r = 0; r < VSG_KPT; ++r) {   // as k_sort_vol: wave w owns keys [c0 + 64 VSG_KPT w, c0 + 64 VSG_KPT (w + 1))
        const int64_t idx = c0 + (int64_t)w * (VSG_KPT * 64) + r * 64 + lane;
        const bool valid = idx < n;
        const uint32_t kk = key[r];
        const uint32_t d = (kk >> shift) & 255u;
        const uint32_t d0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)d);   // (valid lanes: a prefix)
        const uint64_t peers = __all(!valid || d == d0) ? __ballot(valid) : VS_PEERS(d, valid);
        const uint32_t below = (uint32_t)__popcll(peers & lt);
        uint32_t base = 0u;
        if (valid && below == 0) base = atomicAdd(&s_wc[w][d], (uint32_t)__popcll(peers));
        const int leader = peers ? __builtin_ctzll(peers) : lane;
        base = (uint32_t)__shfl((int)base, leader, 64);
        rank[r] = valid ? base + below : 0xffffffffu;
    }
    __syncthreads();
    if (t < 256) {
        uint32_t tot = 0;
        uint32_t wcv[VS_WAVES];
#pragma unroll
        for (int ww = 0; ww < VS_WAVES; ++ww) wcv[ww] = s_wc[ww][t];
#pragma unroll
        for (int ww = 0; ww < VS_WAVES; ++ww) { s_wc[ww][t] = tot; tot += wcv[ww]; }
        uint32_t inc = tot;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t v = __shfl_up(inc, o, 64);
            if (lane >= o) inc += v;
        }
        if (lane == 63) s_wsum[w] = inc;
        s_tot[t] = tot;
        s_cst[t] = inc - tot;
    }
    __syncthreads();
    if (t < 256) {
        uint32_t pre = 0;
        for (int ww = 0; ww < w; ++ww) pre += s_wsum[ww];
        s_cst[t] += pre;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < VSG_KPT; ++r) {
        if (rank[r] == 0xffffffffu) continue;
        const uint32_t d = (key[r] >> shift) & 255u;
        s_stage[s_cst[d] + s_wc[w][d] + rank[r]] = key[r];
    }
    __syncthreads();
    const int cn = (int)(n - c0 < VSG_CHUNK ? n - c0 : VSG_CHUNK);
    for (int q = t; q < cn; q += VS_TPB) {
        const uint32_t kk = s_stage[q];
        const uint32_t d = (kk >> shift) & 255u;
        kout[s_off[d] + ((uint32_t)q - s_cst[d])] = kk;
    }
}

// =============================================================================================
// mean anchor (Vent_Analysis.py:246): np.mean of the sorted float32 list is
//   float32( float64( serial float32 sum over 8192-chunks of numpy pairwise_sum(chunk) ) / n ).
// One wave per chunk evaluates numpy's pairwise recursion exactly (k_chunk_sums: leaves of <= 128
// values on 8 lanes each, then the tree's left + right combines), then one thread per volume adds
// the chunk sums in order (pairwise_sum's leaf: 8 stride-8 accumulators combined as
// ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), then the n % 8 tail; fewer than 8 values: a plain loop).  p99 (Vent_Analysis.py:255) is the order
// statistic sorted[int(n * 0.99)].
// =============================================================================================
#define PW_MAX_LEAVES 64   // 8192 / 128

// A partial chunk's pairwise tree (numpy's split n2 = n/2 - (n/2) % 8 down to leaves of <= 128)
// built level by level by the whole wave in LDS (no per-lane stack: a dynamically indexed private
// array lives in scratch memory, and the one-lane recursion walk plus its replay took ~0.25 ms of a
// step), the leaves summed 8 lanes each, then the internal nodes combined bottom-up, left + right.
#define PW_NODES 256   // nodes of one chunk's tree (<= 128 leaves of >= 64 values)
struct PwTree {
    int32_t s[PW_NODES], n[PW_NODES], child[PW_NODES];   // child: first child's index, -1 = leaf
    float sum[PW_NODES];
    int32_t lvl[14];                                     // level starts (lvl[L] .. lvl[L + 1])
};

__device__ float pw_tree_sum(const uint32_t *a, int m, PwTree &T) {
    const int lane = threadIdx.x & 63;
    auto wsync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    if (lane == 0) {
        T.s[0] = 0;
        T.n[0] = m;
        T.lvl[0] = 0;
        T.lvl[1] = 1;
    }
    wsync();
    int nlev = 1, total = 1;
    for (int L = 0; L < 11; ++L) {   // children of level L's nodes become level L + 1
        const int ls = T.lvl[L], le = T.lvl[L + 1];
        if (ls == le) break;
        int next = le;
        for (int base = ls; base < le; base += 64) {
            const int i = base + lane;
            const bool in = i < le;
            const int nn = in ? T.n[i] : 0;
            const bool split = in && nn > 128;
            const uint64_t bal = __ballot(split);
            const int pos = next + 2 * __popcll(bal & ((1ull << lane) - 1ull));
            if (in) T.child[i] = split ? pos : -1;
            if (split) {
                const int n2 = nn / 2 - (nn / 2) % 8;
                T.s[pos] = T.s[i];
                T.n[pos] = n2;
                T.s[pos + 1] = T.s[i] + n2;
                T.n[pos + 1] = nn - n2;
            }
            next += 2 * __popcll(bal);
        }
        if (lane == 0) T.lvl[L + 2] = next;
        total = next;
        nlev = L + 2;
        wsync();
    }
    // leaves: 8 lanes each (pw_leaf's 8 stride-8 accumulators), 8 leaves per pass over the nodes
    for (int g = 0; g * 8 < total; ++g) {
        const int node = g * 8 + (lane >> 3), j = lane & 7;
        const bool has = node < total && T.child[node] < 0;
        const int ln = has ? T.n[node] : 0;
        const uint32_t *p = a + (has ? T.s[node] : 0);
        const int lim = ln - ln % 8;
        // every load unconditional at a clamped index (p[0] is a key of the chunk): guarded loads
        // compile to exec-masked branches that wait for each load in turn
        float v[16], tl[7];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int i = 8 * q + j;
            v[q] = key2f(p[i < lim ? i : 0]);
        }
#pragma unroll
        for (int q = 0; q < 7; ++q) tl[q] = key2f(p[lim + q < ln ? lim + q : 0]);   // the n % 8 tail
        float r = v[0];
#pragma unroll
        for (int q = 1; q < 16; ++q)
            if (8 * q + j < lim) r = r + v[q];
        r = r + __shfl_xor(r, 1, 64);
        r = r + __shfl_xor(r, 2, 64);
        r = r + __shfl_xor(r, 4, 64);
        if (has && j == 0) {
            float res = ln < 8 ? 0.0f : r;
#pragma unroll
            for (int q = 0; q < 7; ++q)
                if (lim + q < ln) res = res + tl[q];
            T.sum[node] = res;
        }
    }
    wsync();
    // internal nodes bottom-up: sum = left + right (pairwise_sum's return expression)
    for (int L = nlev - 2; L >= 0; --L) {
        for (int i = T.lvl[L] + lane; i < T.lvl[L + 1]; i += 64) {
            const int c = T.child[i];
            if (c >= 0) T.sum[i] = T.sum[c] + T.sum[c + 1];
        }
        wsync();
    }
    return T.sum[0];
}

__global__ void __launch_bounds__(VH_TPB) k_chunk_sums(const uint32_t *__restrict__ keys,
                                                      const VolScalars *sc, int64_t V,
                                                      int64_t max_chunks, float *chunk) {
    __shared__ float s_leaf[VH_TPB / 64][PW_MAX_LEAVES];
    __shared__ PwTree s_tree;   // the volume's partial chunk (one per volume, so one per block)
    const int64_t b = blockIdx.y;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t c = blockIdx.x * (int64_t)(VH_TPB / 64) + w;
    const int64_t n = sc[b].n_mask;
    const int64_t s = c * 8192;
    if (s >= n) return;   // wave-uniform
    const int64_t m = n - s < 8192 ? n - s : 8192;
    const uint32_t *a = keys + b * V + s;
    if (m < 8192) {   // the last chunk of the volume: its own tree
        const float r = pw_tree_sum(a, (int)m, s_tree);
        if (lane == 0) chunk[b * max_chunks + c] = r;
        return;
    }
    // full chunk: 64 leaves of 128, 8 at a time: lane = (leaf, accumulator j) -- pw_leaf's 8
    // stride-8 accumulators run on 8 lanes (loads of a leaf row are 8 consecutive keys), then its
    // fixed combine tree by xor shuffles (a + b == b + a bitwise)
    float v[8][16];   // all 8 groups' loads in flight together (one memory round trip, not 8)
#pragma unroll
    for (int g = 0; g < 8; ++g) {
        const uint32_t *p = a + 128 * (g * 8 + (lane >> 3));
#pragma unroll
        for (int q = 0; q < 16; ++q) v[g][q] = key2f(p[8 * q + (lane & 7)]);
    }
#pragma unroll
    for (int g = 0; g < 8; ++g) {
        const int leaf = g * 8 + (lane >> 3), j = lane & 7;
        float r = v[g][0];
#pragma unroll
        for (int q = 1; q < 16; ++q) r = r + v[g][q];
        r = r + __shfl_xor(r, 1, 64);
        r = r + __shfl_xor(r, 2, 64);
        r = r + __shfl_xor(r, 4, 64);
        if (j == 0) s_leaf[w][leaf] = r;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // perfect binary tree over the 64 leaves: xor shuffles, same pairs and order
    float r = s_leaf[w][lane];
    for (int off = 1; off < 64; off <<= 1) r = r + __shfl_xor(r, off, 64);
    if (lane == 0) chunk[b * max_chunks + c] = r;
}

__global__ void k_mean_p99(const uint32_t *__restrict__ keys, const float *chunk,
                           int64_t max_chunks, int64_t V, int64_t nb, VolScalars *sc) {
    const int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (b >= nb) return;
    const int64_t n = sc[b].n_mask;
    if (n <= 0) {
        sc[b].mean_anchor = __int_as_float(0x7fc00000);
        sc[b].p99 = __int_as_float(0x7fc00000);
        return;
    }
    float S = 0.0f;
    const int64_t nc = (n + 8191) / 8192;
    for (int64_t c = 0; c < nc; ++c) S = S + chunk[b * max_chunks + c];
    sc[b].mean_anchor = (float)((double)S / (double)n);
    const int64_t i99 = (int64_t)((double)n * 0.99);
    sc[b].p99 = key2f(keys[b * V + i99]);
}

// =============================================================================================
// fused classify tile kernel: mean-anchored threshold (:249) -> 3x3 zero-padded median on the
// binary map (scipy medfilt2d, :248-249) -> np.gradient border of the defect map (:250) ->
// linear-binning classes (:256) -> counts (:251,257) (+ optional cohort histogram).
// Tile = TX rows x TY cols x TZ slices; raw map staged in LDS with a 2-voxel in-plane halo,
// defect map with a 1-voxel halo.
// =============================================================================================
#define CL_TX 8
#define CL_TY 16

__device__ __forceinline__ uint8_t lb_class(float nv) {
    // (x<=.16)*1 + (.16<x<=.34)*2 + ... + (x>.88)*6, float32 edges; NaN -> 0
    if (nv <= 0.16f) return 1;
    if (nv <= 0.34f) return 2;
    if (nv <= 0.52f) return 3;
    if (nv <= 0.7f) return 4;
    if (nv <= 0.88f) return 5;
    if (nv > 0.88f) return 6;
    return 0;
}

// Classify / border tile: a block owns CL_TX rows x CL_TY cols x tz slices (tz <= 32, 28 with the
// 3-D slice halo) with a 2-voxel halo in LDS.  Threads map to (slice lane = t & 31, col lane =
// t >> 5): every phase is a loop over rows and col groups with no index division, and a wave
// reads/writes runs of consecutive slices (contiguous bytes).
#define CL_YL (VH_TPB / 32)   // col lanes per block
template <bool CLASSIFY, bool M3D>
__global__ void __launch_bounds__(VH_TPB) k_tile(const float *__restrict__ n4,
                                                const uint8_t *__restrict__ mask,
                                                const uint8_t *__restrict__ in_bin,
                                                const VolScalars *__restrict__ sc, float thresh,
                                                int64_t R, int64_t C, int64_t Z, int64_t V,
                                                int tz, uint8_t *defect, uint8_t *border,
                                                uint8_t *lb, unsigned long long *cnt_out) {
    extern __shared__ uint8_t lds[];
    const int64_t b = blockIdx.y;
    const int64_t ntx = (R + CL_TX - 1) / CL_TX, nty = (C + CL_TY - 1) / CL_TY;
    int64_t bid = blockIdx.x;
    const int64_t tix = bid % ntx; bid /= ntx;
    const int64_t tiy = bid % nty; bid /= nty;
    const int64_t x0 = tix * CL_TX, y0 = tiy * CL_TY, z0 = bid * tz;
    const int tzn = (int)(Z - z0 < tz ? Z - z0 : tz);
    const int EX = CL_TX + 4, EY = CL_TY + 4, DX = CL_TX + 2, DY = CL_TY + 2;
    // M3D (build-defined 3-D morphology): slice halo of 2 (raw) / 1 (defect) as well
    const int EZ = M3D ? tzn + 4 : tzn, DZ = M3D ? tzn + 2 : tzn;
    const int zr = M3D ? 2 : 0, zd = M3D ? 1 : 0;
    const int SZ = 32;                                  // LDS slice pitch
    uint8_t *raw = lds;                                 // [EX][EY][SZ]
    uint8_t *def = lds + EX * EY * SZ;                  // [DX][DY][SZ]
    const int lz = threadIdx.x & 31, ly = threadIdx.x >> 5;
    const float *p4 = CLASSIFY ? n4 + b * V : nullptr;
    const uint8_t *pm = mask + b * V;
    float m = 0.0f, p99 = 0.0f;
    if (CLASSIFY) { m = sc[b].mean_anchor; p99 = sc[b].p99; }
    uint8_t *lbc = def + DX * DY * SZ;                  // [CL_TX][CL_TY][SZ] LB class (CLASSIFY)
    if (CLASSIFY) {
        const int64_t z = z0 - zr + lz;
        const bool zin = lz < EZ && z >= 0 && z < Z;
        const bool zint = lz >= zr && lz < zr + tzn;    // slice inside the output tile
        for (int ey = ly; ey < EY; ey += CL_YL) {
            const int64_t y = y0 - 2 + ey;
            const bool yin = zin && y >= 0 && y < C;
            uint8_t mk[CL_TX + 4];
            float nv[CL_TX + 4];
#pragma unroll
            for (int ex = 0; ex < CL_TX + 4; ++ex) {   // all loads of the column in flight
                const int64_t x = x0 - 2 + ex;
                const bool ok = yin && x >= 0 && x < R;
                const int64_t i = ok ? (x * C + y) * Z + z : 0;
                mk[ex] = ok ? pm[i] : 0;
                nv[ex] = ok ? p4[i] : 0.0f;
            }
            const bool yint = ey >= 2 && ey < 2 + CL_TY && zint;
#pragma unroll
            for (int ex = 0; ex < CL_TX + 4; ++ex) {
                // IEEE f32 division, float32(thresh) (Vent_Analysis.py:247-249)
                const uint8_t v = mk[ex] ? (uint8_t)((nv[ex] / m) < thresh) : (uint8_t)0;
                if (lz < EZ) raw[(ex * EY + ey) * SZ + lz] = v;
                if (yint && ex >= 2 && ex < 2 + CL_TX)   // LB class of an output voxel (:255-256)
                    lbc[((ex - 2) * CL_TY + (ey - 2)) * SZ + (lz - zr)] = mk[ex] ? lb_class(nv[ex] / p99) : 0;
            }
        }
        __syncthreads();
        if (lz < DZ) {
            for (int dx = 0; dx < DX; ++dx)
                for (int dy = ly; dy < DY; dy += CL_YL) {
                    int cnt = 0;
                    if (M3D) {   // 3x3x3 median of a 0/1 volume, zero padded: 1 iff >= 14 of 27
#pragma unroll
                        for (int i = 0; i < 3; ++i)
#pragma unroll
                            for (int j = 0; j < 3; ++j)
#pragma unroll
                                for (int k = 0; k < 3; ++k) cnt += raw[((dx + i) * EY + (dy + j)) * SZ + lz + k];
                    def[(dx * DY + dy) * SZ + lz] = cnt >= 14;
                    } else {     // medfilt2d 3x3 per slice (Vent_Analysis.py:249): >= 5 of 9
#pragma unroll
                        for (int i = 0; i < 3; ++i)
#pragma unroll
                            for (int j = 0; j < 3; ++j) cnt += raw[((dx + i) * EY + (dy + j)) * SZ + lz];
                        def[(dx * DY + dy) * SZ + lz] = cnt >= 5;
                    }
                }
        }
    } else {
        // border of an arbitrary binary volume: stage it as the "defect" map directly
        const uint8_t *pin = in_bin + b * V;
        const int64_t z = z0 - zd + lz;
        const bool zin = lz < DZ && z >= 0 && z < Z;
        for (int dx = 0; dx < DX; ++dx) {
            const int64_t x = x0 - 1 + dx;
            for (int dy = ly; dy < DY; dy += CL_YL) {
                const int64_t y = y0 - 1 + dy;
                uint8_t v = 0;
                if (zin && x >= 0 && x < R && y >= 0 && y < C) v = pin[(x * C + y) * Z + z];
                if (lz < DZ) def[(dx * DY + dy) * SZ + lz] = v;
            }
        }
    }
    __syncthreads();
    unsigned long long n_def = 0, n_lb12 = 0;
    if (lz < tzn) {
        const int64_t z = z0 + lz;
        const int dz = lz + zd;
        for (int ix = 0; ix < CL_TX; ++ix) {
            const int64_t x = x0 + ix;
            if (x >= R) break;
            for (int iy = ly; iy < CL_TY; iy += CL_YL) {
                const int64_t y = y0 + iy;
                if (y >= C) break;
                const int dx = ix + 1, dy = iy + 1;
#define DEF(a, c, e) def[((a) * DY + (c)) * SZ + (e)]
                const uint8_t d = DEF(dx, dy, dz);
                bool gx, gy, gz = false;   // np.gradient != 0: central inside, one-sided at edges
                if (x == 0) gx = DEF(dx + 1, dy, dz) != d;
                else if (x == R - 1) gx = d != DEF(dx - 1, dy, dz);
                else gx = DEF(dx + 1, dy, dz) != DEF(dx - 1, dy, dz);
                if (y == 0) gy = DEF(dx, dy + 1, dz) != d;
                else if (y == C - 1) gy = d != DEF(dx, dy - 1, dz);
                else gy = DEF(dx, dy + 1, dz) != DEF(dx, dy - 1, dz);
                if (M3D && Z > 1) {
                    if (z == 0) gz = DEF(dx, dy, dz + 1) != d;
                    else if (z == Z - 1) gz = d != DEF(dx, dy, dz - 1);
                    else gz = DEF(dx, dy, dz + 1) != DEF(dx, dy, dz - 1);
                }
#undef DEF
                const int64_t i = b * V + (x * C + y) * Z + z;
                border[i] = gx || gy || gz;
                if (CLASSIFY) {
                    defect[i] = d;
                    n_def += d;
                    const uint8_t cls = lbc[(ix * CL_TY + iy) * SZ + lz];
                    lb[i] = cls;
                    n_lb12 += (cls == 1 || cls == 2);
                }
            }
        }
    }
    if (CLASSIFY) {
        // wave reduce, one atomic per wave
        for (int off = 32; off > 0; off >>= 1) {
            n_def += __shfl_down(n_def, off, 64);
            n_lb12 += __shfl_down(n_lb12, off, 64);
        }
        if ((threadIdx.x & 63) == 0) {
            if (n_def) atomicAdd(&cnt_out[b * 2 + 0], n_def);
            if (n_lb12) atomicAdd(&cnt_out[b * 2 + 1], n_lb12);
        }
    }
}

__global__ void k_counts_to_scalars(const unsigned long long *cnt, int64_t nb, VolScalars *sc) {
    int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (b >= nb) return;
    sc[b].n_defect = (int64_t)cnt[b * 2];
    sc[b].n_lb12 = (int64_t)cnt[b * 2 + 1];
}

static void tile_geometry(const vh_batch *b, bool m3d, int &tz, dim3 &grid, size_t &lds) {
    const int tzmax = m3d ? 28 : 32;   // slice tile + halo <= 32 slice lanes
    tz = (int)(b->Z < tzmax ? b->Z : tzmax);
    const int64_t ntx = (b->R + CL_TX - 1) / CL_TX, nty = (b->C + CL_TY - 1) / CL_TY;
    const int64_t ntz = (b->Z + tz - 1) / tz;
    grid = dim3((unsigned)(ntx * nty * ntz), (unsigned)b->nb, 1);
    lds = ((size_t)(CL_TX + 4) * (CL_TY + 4) + (size_t)(CL_TX + 2) * (CL_TY + 2) +
           (size_t)CL_TX * CL_TY) * 32;
}

// =============================================================================================
// Plane-sweep classify / border (the default; k_tile above stays for planes too wide for it).
// A block owns one volume's slab of rows [xa, xb) and a band of columns [ya, yb) with every
// slice -- the whole (y, z) plane when it fits, so there is no y halo -- and walks the slab plane
// by plane with one barrier per plane.  LDS holds rings of the last 4 planes of the raw
// threshold map and of the median-filtered defect map, 4 slices per 32-bit word: the 3x3 (x, y)
// median is a byte-lane sum of 9 words (every byte sum <= 27, so no carries) and a compare by
// adding 128 - k.  Words whose 4 columns hold no mask voxel at this row (outside the columns'
// masked row range, k_mask_stats) are not loaded: their raw and LB bytes are 0.
// Iteration p: loads of plane p + 1 issued; raw(p) -> LDS (and LB of plane p); def(p - 2) from
// raw(p - 3 .. p - 1); defect / border of plane p - 4 from def(p - 5 .. p - 3).  Rings of 4
// slots make every slot written in iteration p distinct from the ones read in it.
// =============================================================================================
#define PS_TPB 256
#define PS_K 4          // words per thread per plane (host picks the band so the plane fits)
#define PS_XS 32        // slab rows

struct PsGeom {
    int R, C, Z, ZW;    // ZW = ceil(Z / 4) words per (x, y) row
    int64_t V, CZ;
    int XS, TY, nxs, nyt;
};

enum { PS_CL2 = 0, PS_CL3 = 1, PS_BORDER = 2 };

// byte lanes >= k (bias = 128 - k, added to every byte lane): 1, else 0
__device__ __forceinline__ uint32_t ps_atleast(uint32_t s, uint32_t bias) {
    return ((s + bias * 0x01010101u) >> 7) & 0x01010101u;
}
// byte lanes != 0: 1, else 0
__device__ __forceinline__ uint32_t ps_nonzero(uint32_t g) {
    return ((((g & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | g) >> 7) & 0x01010101u;
}

// Division-free forms of the classify tests (bit-identical to the IEEE float division): for
// 0 < m < inf and a positive normal float e, RN(v / m) <= e  <=>  v < u * m, or v == u * m when e's
// significand is even (round-half-even picks e), where u = (e + succ(e)) / 2.  u has 25
// significant bits and m 24, so u * m is exact in double; the tie folds into the bound by moving
// it up one double ulp, and as v is a float, "v < bound" equals "v < the bound rounded up to a
// float".  So each test is one float compare; NaN v fails every one, as RN(NaN) <= e does.
// RN(q) < t is RN(q) <= pred(t).
__device__ __forceinline__ float le_bound(float e, float m) {
    const float s = __uint_as_float(__float_as_uint(e) + 1u);
    double u = (((double)e + (double)s) * 0.5) * (double)m;
    if ((__float_as_uint(e) & 1u) == 0u) u = __longlong_as_double(__double_as_longlong(u) + 1);
    float f = (float)u;
    if ((double)f < u) f = __uint_as_float(__float_as_uint(f) + 1u);   // round up (inf stays)
    return f;
}

// per-word flags (precomputed once per block; the word set is the same for every plane)
#define PSF_ZW0 1u      // zw == 0
#define PSF_ZWL 2u      // zw == ZW - 1
#define PSF_Y0 4u       // y == 0
#define PSF_YL 8u       // y == C - 1
#define PSF_ZLAST 16u   // word holds slice Z - 1
#define PSF_BAND 32u    // row inside the band [ya, yb)
#define PSF_NV_SHIFT 8  // bits 8..10: valid slices in the word (1..4)

template <int MODE, bool VEC>
__global__ void __launch_bounds__(PS_TPB) k_plane(const float *__restrict__ n4,
                                                 const uint8_t *__restrict__ mask,
                                                 const uint8_t *__restrict__ in_bin,
                                                 const int32_t *__restrict__ colrange,
                                                 const VolScalars *__restrict__ sc, float thresh,
                                                 PsGeom g, uint8_t *defect, uint8_t *border,
                                                 uint8_t *lb, unsigned long long *cnt_out) {
    constexpr bool CL = MODE != PS_BORDER;
    extern __shared__ uint32_t ps_lds[];
    const int64_t b = blockIdx.y;
    const int xs = (int)(blockIdx.x % (unsigned)g.nxs), yt = (int)(blockIdx.x / (unsigned)g.nxs);
    const int R = g.R, C = g.C, Z = g.Z, ZW = g.ZW;
    const int xa = xs * g.XS, xb = min(xa + g.XS, R);
    const int ya = yt * g.TY, yb = min(ya + g.TY, C);
    const int RW = CL ? (g.TY + 4) * ZW : 0;   // raw slot: rows ya - 2 .. ya + TY + 1
    const int DW = (g.TY + 2) * ZW;            // def slot: rows ya - 1 .. ya + TY
    uint32_t *raw = ps_lds;                    // [4][TY + 4][ZW]
    uint32_t *def = ps_lds + 4 * RW;           // [4][TY + 2][ZW]
    for (int i = threadIdx.x; i < 4 * (RW + DW); i += PS_TPB) ps_lds[i] = 0u;
    const int64_t vb = b * g.V;
    float m = 0.0f, p99 = 0.0f;
    if (CL) { m = sc[b].mean_anchor; p99 = sc[b].p99; }
    // division-free tests when the scalars allow them (block-uniform), else IEEE divisions
    const float tpred = __uint_as_float(__float_as_uint(thresh) - 1u);
    const bool fast = CL && m > 0.0f && m <= FLT_MAX && p99 > 0.0f && p99 <= FLT_MAX &&
                      thresh >= FLT_MIN && thresh <= FLT_MAX && tpred >= FLT_MIN;
    float f_thr = 0.0f, f_lb[5] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    if (fast) {
        f_thr = le_bound(tpred, m);
        const float edges[5] = {0.16f, 0.34f, 0.52f, 0.7f, 0.88f};
        for (int e = 0; e < 5; ++e) f_lb[e] = le_bound(edges[e], p99);
    }

    // word sets: loads (raw rows, or def rows in border mode), def rows, output rows
    const int hl = CL ? 2 : 1;
    const int lylo = max(ya - hl, 0), lyhi = min(yb + hl, C);
    const int dylo = max(ya - 1, 0), dyhi = min(yb + 1, C);
    const int nld = (lyhi - lylo) * ZW, ndf = (dyhi - dylo) * ZW, nout = (yb - ya) * ZW;
    auto flags = [&](int y, int zw) {
        uint32_t f = 0;
        if (zw == 0) f |= PSF_ZW0;
        if (zw == ZW - 1) f |= PSF_ZWL;
        if (y == 0) f |= PSF_Y0;
        if (y == C - 1) f |= PSF_YL;
        if (zw == ((Z - 1) >> 2)) f |= PSF_ZLAST;
        if (y >= ya && y < yb) f |= PSF_BAND;
        f |= (uint32_t)min(4, Z - 4 * zw) << PSF_NV_SHIFT;
        return f;
    };
    int l_goff[PS_K], l_lds[PS_K], l_lo[PS_K], l_hi[PS_K];
    uint32_t l_f[PS_K];
    int d_idx[PS_K];
    uint32_t d_f[PS_K];
    int o_idx[PS_K], o_goff[PS_K];
    uint32_t o_f[PS_K];
#pragma unroll
    for (int k = 0; k < PS_K; ++k) {
        const int w = threadIdx.x + k * PS_TPB;
        l_lo[k] = INT_MAX; l_hi[k] = -1; l_goff[k] = 0; l_lds[k] = 0; l_f[k] = 0;
        if (w < nld) {
            const int y = lylo + w / ZW, zw = w % ZW;
            l_goff[k] = y * Z + 4 * zw;
            l_lds[k] = (y - ya + hl) * ZW + zw;
            l_f[k] = flags(y, zw);
            if (CL) {
                const int nv = min(4, Z - 4 * zw);
                for (int q = 0; q < nv; ++q) {
                    const int32_t *cr = colrange + (b * g.CZ + l_goff[k] + q) * 2;
                    l_lo[k] = min(l_lo[k], cr[0]);
                    l_hi[k] = max(l_hi[k], cr[1]);
                }
            } else {
                l_lo[k] = 0; l_hi[k] = R - 1;
            }
        }
        d_idx[k] = -1; d_f[k] = 0;
        if (CL && w < ndf) {
            const int y = dylo + w / ZW, zw = w % ZW;
            d_idx[k] = (y - ya + 1) * ZW + zw;
            d_f[k] = flags(y, zw);
        }
        o_idx[k] = -1; o_goff[k] = 0; o_f[k] = 0;
        if (w < nout) {
            const int y = ya + w / ZW, zw = w % ZW;
            o_idx[k] = (y - ya + 1) * ZW + zw;
            o_goff[k] = y * Z + 4 * zw;
            o_f[k] = flags(y, zw);
        }
    }

    // plane q's words into registers (zeros for rows outside the volume or the masked range)
    auto load = [&](int q, float4 (&nv)[PS_K], uint32_t (&mk)[PS_K]) {
        const bool qin = q >= 0 && q < R && q <= (CL ? xb + 1 : xb);
        const int64_t base = vb + (int64_t)q * g.CZ;
#pragma unroll
        for (int k = 0; k < PS_K; ++k) {
            nv[k] = make_float4(0.f, 0.f, 0.f, 0.f);
            mk[k] = 0u;
            if (qin && q >= l_lo[k] && q <= l_hi[k]) {
                const int64_t i = base + l_goff[k];
                const uint8_t *src = CL ? mask : in_bin;
                if (VEC) {
                    mk[k] = *reinterpret_cast<const uint32_t *>(src + i);
                    if (CL) nv[k] = *reinterpret_cast<const float4 *>(n4 + i);
                } else {
                    const int nvd = (int)(l_f[k] >> PSF_NV_SHIFT) & 7;
                    float t[4] = {0.f, 0.f, 0.f, 0.f};
                    for (int q2 = 0; q2 < nvd; ++q2) {
                        mk[k] |= (uint32_t)src[i + q2] << (8 * q2);
                        if (CL) t[q2] = n4[i + q2];
                    }
                    nv[k] = make_float4(t[0], t[1], t[2], t[3]);
                }
            }
        }
    };
    auto store_word = [&](uint8_t *dst, int64_t i, uint32_t v, uint32_t f) {
        if (VEC) {
            *reinterpret_cast<uint32_t *>(dst + i) = v;
        } else {
            const int nvd = (int)(f >> PSF_NV_SHIFT) & 7;
            for (int q2 = 0; q2 < nvd; ++q2) dst[i + q2] = (uint8_t)(v >> (8 * q2));
        }
    };

    unsigned long long n_def = 0, n_lb12 = 0;
    auto step = [&](int p, float4 (&nv)[PS_K], uint32_t (&mk)[PS_K], float4 (&nvn)[PS_K],
                    uint32_t (&mkn)[PS_K]) {
        load(p + 1, nvn, mkn);
        if (CL) {
            // raw(p) and the LB classes of plane p (Vent_Analysis.py:247-249, 255-256)
            if (p <= xb + 1) {
                const bool lbp = p >= xa && p < xb;
#pragma unroll
                for (int k = 0; k < PS_K; ++k) {
                    if (threadIdx.x + k * PS_TPB >= nld) continue;
                    const bool lbk = lbp && (l_f[k] & PSF_BAND);   // halo rows: raw only
                    const float v[4] = {nv[k].x, nv[k].y, nv[k].z, nv[k].w};
                    uint32_t r = 0u, c = 0u;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {   // branch-free: deselected bytes give 0
                        const bool on = ((mk[k] >> (8 * q)) & 0xFFu) != 0u;
                        uint32_t below, cls;
                        if (fast) {
                            below = v[q] < f_thr;
                            // LB class = 6 - #(edges with RN(v / p99) <= edge); NaN -> 0
                            const uint32_t nle = (uint32_t)(v[q] < f_lb[0]) + (uint32_t)(v[q] < f_lb[1]) +
                                                 (uint32_t)(v[q] < f_lb[2]) + (uint32_t)(v[q] < f_lb[3]) +
                                                 (uint32_t)(v[q] < f_lb[4]);
                            cls = v[q] == v[q] ? 6u - nle : 0u;
                        } else {
                            // IEEE f32 division, float32(thresh)
                            below = (v[q] / m) < thresh;
                            cls = lb_class(v[q] / p99);
                        }
                        below = on ? below : 0u;
                        cls = (on && lbk) ? cls : 0u;
                        r |= below << (8 * q);
                        c |= cls << (8 * q);
                        n_lb12 += (cls == 1u || cls == 2u);
                    }
                    raw[(p & 3) * RW + l_lds[k]] = r;
                    if (lbk)
                        store_word(lb, vb + (int64_t)p * g.CZ + l_goff[k], c, l_f[k]);
                }
            }
            // def(p - 2): zero-padded 3x3 median per slice (>= 5 of 9) or 3x3x3 (>= 14 of 27)
            const int xd = p - 2;
            if (xd >= xa - 1 && xd <= xb) {
                const uint32_t *r0 = raw + ((p - 3) & 3) * RW, *r1 = raw + ((p - 2) & 3) * RW,
                               *r2 = raw + ((p - 1) & 3) * RW;
#pragma unroll
                for (int k = 0; k < PS_K; ++k) {
                    const int i = d_idx[k];
                    if (i < 0) continue;
                    auto sum9 = [&](int j) {
                        return ((r0[j] + r0[j + ZW]) + r0[j + 2 * ZW]) +
                               ((r1[j] + r1[j + ZW]) + r1[j + 2 * ZW]) +
                               ((r2[j] + r2[j + ZW]) + r2[j + 2 * ZW]);
                    };
                    const uint32_t s0 = sum9(i);
                    uint32_t d;
                    if (MODE == PS_CL3) {
                        const uint32_t sm = (d_f[k] & PSF_ZW0) ? 0u : sum9(i - 1);
                        const uint32_t sp = (d_f[k] & PSF_ZWL) ? 0u : sum9(i + 1);
                        const uint32_t s = s0 + ((s0 << 8) | (sm >> 24)) + ((s0 >> 8) | (sp << 24));
                        d = ps_atleast(s, 128u - 14u);
                    } else {
                        d = ps_atleast(s0, 128u - 5u);
                    }
                    def[(xd & 3) * DW + i] = d;
                }
            }
        } else if (p <= xb) {
            // border of an arbitrary binary volume: the input is the "defect" map
#pragma unroll
            for (int k = 0; k < PS_K; ++k)
                if (threadIdx.x + k * PS_TPB < nld) def[(p & 3) * DW + l_lds[k]] = mk[k];
        }
        // outputs of plane x: np.gradient != 0 (central inside, one-sided at the edges)
        const int x = CL ? p - 4 : p - 2;
        if (x >= xa && x < xb) {
            const uint32_t *dm = def + ((x - 1) & 3) * DW, *d0 = def + (x & 3) * DW,
                           *dp = def + ((x + 1) & 3) * DW;
            const bool xe0 = x == 0, xel = x == R - 1;
#pragma unroll
            for (int k = 0; k < PS_K; ++k) {
                const int i = o_idx[k];
                if (i < 0) continue;
                const uint32_t f = o_f[k];
                const uint32_t D = d0[i];
                const uint32_t ax = (!xe0 && xel) ? D : dp[i], bx = xe0 ? D : dm[i];
                const uint32_t ay = (!(f & PSF_Y0) && (f & PSF_YL)) ? D : d0[i + ZW];
                const uint32_t by = (f & PSF_Y0) ? D : d0[i - ZW];
                uint32_t gr = (ax ^ bx) | (ay ^ by);
                if (MODE == PS_CL3 && Z > 1) {
                    const uint32_t dn = (f & PSF_ZWL) ? 0u : d0[i + 1];
                    const uint32_t dv = (f & PSF_ZW0) ? 0u : d0[i - 1];
                    const uint32_t zp = (D >> 8) | (dn << 24), zm = (D << 8) | (dv >> 24);
                    const uint32_t m0 = (f & PSF_ZW0) ? 0xFFu : 0u;
                    const uint32_t ml = (f & PSF_ZLAST) ? 0xFFu << (8 * ((Z - 1) & 3)) : 0u;
                    gr |= ((zp & ~ml) | (D & ml)) ^ ((zm & ~m0) | (D & m0));
                }
                const int64_t gi = vb + (int64_t)x * g.CZ + o_goff[k];
                store_word(border, gi, ps_nonzero(gr), f);
                if (CL) {
                    store_word(defect, gi, D, f);
                    n_def += (unsigned)__popc(D);
                }
            }
        }
        __syncthreads();
    };

    const int p0 = CL ? xa - 2 : xa - 1, p1 = CL ? xb + 3 : xb + 1;
    float4 nvA[PS_K], nvB[PS_K];
    uint32_t mkA[PS_K], mkB[PS_K];
    load(p0, nvA, mkA);
    __syncthreads();   // LDS cleared
    for (int p = p0; p <= p1; p += 2) {
        step(p, nvA, mkA, nvB, mkB);
        if (p + 1 <= p1) step(p + 1, nvB, mkB, nvA, mkA);
    }
    if (CL) {
        for (int off = 32; off > 0; off >>= 1) {
            n_def += __shfl_down(n_def, off, 64);
            n_lb12 += __shfl_down(n_lb12, off, 64);
        }
        if ((threadIdx.x & 63) == 0) {
            if (n_def) atomicAdd(&cnt_out[b * 2 + 0], n_def);
            if (n_lb12) atomicAdd(&cnt_out[b * 2 + 1], n_lb12);
        }
    }
}

// plane-sweep geometry; false when a band of one row does not fit PS_K words per thread
static bool plane_geometry(const vh_batch *b, int mode, PsGeom &g, dim3 &grid, size_t &lds) {
    if (const char *e = getenv("VH_CLASSIFY_TILE"))
        if (atoi(e)) return false;
    g.R = (int)b->R; g.C = (int)b->C; g.Z = (int)b->Z; g.ZW = (g.Z + 3) / 4;
    g.V = b->V; g.CZ = b->CZ;
    const int cap = PS_K * PS_TPB;
    const int hl = mode == PS_BORDER ? 1 : 2;
    if ((1 + 2 * hl) * g.ZW > cap) return false;
    int nyt = 1;
    while (true) {
        const int ty = (g.C + nyt - 1) / nyt;
        const int rows = nyt == 1 ? g.C : ty + 2 * hl;
        if (rows * g.ZW <= cap) break;
        ++nyt;
    }
    g.nyt = nyt;
    g.TY = (g.C + nyt - 1) / nyt;
    g.XS = PS_XS;
    if (const char *e = getenv("VH_PS_XS")) {
        const int v = atoi(e);
        if (v >= 1) g.XS = v;
    }
    g.nxs = (g.R + g.XS - 1) / g.XS;
    grid = dim3((unsigned)(g.nxs * g.nyt), (unsigned)b->nb, 1);
    lds = (size_t)4 * ((mode == PS_BORDER ? 0 : (g.TY + 4) * g.ZW) + (g.TY + 2) * g.ZW) * 4;
    return lds <= 64 * 1024;
}

template <int MODE>
static void launch_plane(vh_batch *b, const PsGeom &g, dim3 grid, size_t lds, const float *n4,
                         const uint8_t *in_bin, float thresh, uint8_t *border,
                         unsigned long long *cnt) {
    const bool vec = (g.Z & 3) == 0;
    auto fn = vec ? k_plane<MODE, true> : k_plane<MODE, false>;
    fn<<<grid, PS_TPB, lds, b->stream>>>(n4, b->d_mask, in_bin, b->d_colrange, b->d_sc, thresh, g,
                                         b->d_defect, border, b->d_lb, cnt);
}

void vh_launch_border(vh_batch *b, const uint8_t *d_in, uint8_t *d_out) {
    ScopedKTimer tm(b, "border", 2.0 * (double)b->V);
    PsGeom g; dim3 pgrid; size_t plds;
    if (plane_geometry(b, PS_BORDER, g, pgrid, plds)) {
        launch_plane<PS_BORDER>(b, g, pgrid, plds, nullptr, d_in, 0.f, d_out, nullptr);
        VH_CHECK_LAUNCH();
        return;
    }
    int tz; dim3 grid; size_t lds;
    tile_geometry(b, false, tz, grid, lds);
    k_tile<false, false><<<grid, VH_TPB, lds, b->stream>>>(nullptr, b->d_mask, d_in, b->d_sc, 0.f,
                                                         b->R, b->C, b->Z, b->V, tz, nullptr,
                                                         d_out, nullptr, nullptr);
    VH_CHECK_LAUNCH();
}

// =============================================================================================
// k-means VDP (build-defined): 1-D Lloyd, k = 4, on the sorted masked N4
// values; centres start at sorted[floor(n (2j+1) / 2k)]; a value joins the nearest centre (ties
// to the lower); iterate until the partition is stable (<= 300).  One block per volume.
// =============================================================================================
#define KM_K 4
#define KM_TILE 1024
#define KM_LDS_TILES 4096
#define KM_SAMPLES 4096   // LDS sample of the sorted values for the boundary searches
#define KM_TPB 1024

// key i of [lo, hi) as a float, 0 outside: the load is unconditional (index clamped into the range,
// hi > lo), so a group of such loads stays in flight together -- a guarded load compiles to an
// exec-masked branch whose s_waitcnt vmcnt(0) serialises the group
template <typename I>
__device__ __forceinline__ float km_key_in(const uint32_t *k, I i, I lo, I hi) {
    const I c = i < lo ? lo : (i >= hi ? hi - 1 : i);
    const float v = key2f(k[c]);
    return (i >= lo && i < hi) ? v : 0.0f;
}

// wave-cooperative sum of sorted values k[i], i in tile t intersected with [a, e): lane l adds
// elements t*1024 + j*64 + l for j = 0..15 in order, then a fixed shuffle tree (deterministic)
__device__ __forceinline__ double km_tile_sum(const uint32_t *k, int64_t t, int64_t a, int64_t e) {
    const int lane = threadIdx.x & 63;
    double acc = 0.0;
    float v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int64_t i = t * KM_TILE + j * 64 + lane;
        v[j] = km_key_in(k, i, a, e);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) acc += (double)v[j];
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
    return __shfl(acc, 0, 64);
}

// head and tail partial tiles of a cluster together: both tiles' loads are issued before either
// reduction (one memory round trip instead of two); same per-tile arithmetic as km_tile_sum
__device__ __forceinline__ void km_tile_sum2(const uint32_t *k, int64_t t0, int64_t t1, int64_t a,
                                             int64_t e, double &s0, double &s1) {
    const int lane = threadIdx.x & 63;
    float v0[16], v1[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int64_t i0 = t0 * KM_TILE + j * 64 + lane, i1 = t1 * KM_TILE + j * 64 + lane;
        v0[j] = km_key_in(k, i0, a, e);
        v1[j] = km_key_in(k, i1, a, e);
    }
    double acc0 = 0.0, acc1 = 0.0;
#pragma unroll
    for (int j = 0; j < 16; ++j) { acc0 += (double)v0[j]; acc1 += (double)v1[j]; }
    for (int off = 32; off > 0; off >>= 1) {
        acc0 += __shfl_down(acc0, off, 64);
        acc1 += __shfl_down(acc1, off, 64);
    }
    s0 = __shfl(acc0, 0, 64);
    s1 = __shfl(acc1, 0, 64);
}

// first index in [0, n) whose value is strictly closer to chi than to clo (values sorted, so the
// predicate is monotone).  The search first runs over an LDS sample of every stride-th value
// (no memory latency), then 64-ary over the <= stride values left in global memory: one or two
// dependent global rounds per boundary instead of ~4.
__device__ __forceinline__ bool km_closer(double x, double clo, double chi) {
    return fabs(x - chi) < fabs(x - clo);
}

// first sample index js in [0, ns] with the predicate true (ns if none): 64-ary over the LDS sample
__device__ __forceinline__ int64_t km_sample_search(const float *samp, int64_t ns64, double clo, double chi) {
    const int lane = threadIdx.x & 63;
    const int ns = (int)ns64;   // <= KM_SAMPLES: 32-bit index arithmetic (a constant divisor is a mul-hi)
    int slo = 0, shi = ns;      // answer in [slo, shi]
    while (shi - slo > 64) {
        const int span = shi - slo;
        const int p = slo + (span * (lane + 1)) / 65;
        const uint64_t m = __ballot(km_closer((double)samp[p], clo, chi));
        if (m == 0ull) {
            slo = slo + (span * 64) / 65 + 1;
        } else {
            const int f = __ffsll((long long)m) - 1;
            const int pf = slo + (span * (f + 1)) / 65;
            const int pprev = f == 0 ? slo - 1 : slo + (span * f) / 65;
            slo = pprev + 1;
            shi = pf;
        }
    }
    const int p = slo + lane;
    const bool pr = p < shi ? km_closer((double)samp[p], clo, chi) : true;
    return slo + (__ffsll((long long)__ballot(pr)) - 1);
}

__device__ __forceinline__ int64_t km_boundary(const uint32_t *k, int64_t n, double clo, double chi,
                                               const float *samp, int64_t ns, int64_t stride) {
    const int lane = threadIdx.x & 63;
    const int64_t slo = km_sample_search(samp, ns, clo, chi);
    // global: sample js - 1 is false (or none), sample js is true (or none)
    int64_t lo = slo == 0 ? 0 : (slo - 1) * stride + 1;
    int64_t hi = slo >= ns ? n : slo * stride;   // answer in [lo, hi]
    while (hi - lo > 64) {
        const int64_t span = hi - lo;
        const int64_t p = lo + (span * (lane + 1)) / 65;
        const uint64_t m = __ballot(km_closer((double)key2f(k[p]), clo, chi));
        if (m == 0ull) {
            lo = lo + (span * 64) / 65 + 1;
        } else {
            const int f = __ffsll((long long)m) - 1;
            const int64_t pf = lo + (span * (f + 1)) / 65;
            const int64_t pprev = f == 0 ? lo - 1 : lo + (span * f) / 65;
            lo = pprev + 1;
            hi = pf;
        }
    }
    const int64_t p = lo + lane;
    const bool pr = p < hi ? km_closer((double)key2f(k[p]), clo, chi) : true;
    return lo + (__ffsll((long long)__ballot(pr)) - 1);
}

// Tile sums of a volume too large for the LDS prefix (more than KM_LDS_TILES tiles: e.g. one 512^3
// study, 27k tiles), over the whole GPU: one wave per tile (the same km_tile_sum arithmetic), into
// the volume's global tile array; k_kmeans then prefixes it once.  (One workgroup summing every tile
// took 16 ms of config 5's 154 ms.)
__global__ void __launch_bounds__(KM_TPB) k_km_tiles(const uint32_t *__restrict__ keys, int64_t V,
                                                    double *tile_scratch, int64_t max_ktiles,
                                                    const VolScalars *sc) {
    const int64_t b = blockIdx.y;
    const int64_t n = sc[b].n_mask;
    const int64_t nt = (n + KM_TILE - 1) / KM_TILE;
    if (nt <= KM_LDS_TILES) return;   // k_kmeans sums these itself, in LDS
    const int64_t tt = (int64_t)blockIdx.x * (KM_TPB / 64) + (threadIdx.x >> 6);
    if (tt >= nt) return;
    const double ts = km_tile_sum(keys + b * V, tt, 0, n);
    if ((threadIdx.x & 63) == 0) tile_scratch[b * (max_ktiles + 1) + tt] = ts;
}

// The centre update of one Lloyd step (one thread; oracle/vdp_oracle.py kmeans_1d_sorted): every
// non-empty cluster's mean; a cluster left empty takes the value farthest from its own cluster's
// (old) centre among clusters of >= 2 values -- a sorted cluster's farthest values are its two
// ends, ties to the lowest index, never a value at distance 0 -- which leaves its donor's sum
// (scikit-learn's empty-cluster relocation with a fixed tie order); then the centres are sorted.
// Only degenerate data (equal initial centres: two or three distinct values) has empty clusters.
__device__ __forceinline__ double readlane_d(double v, int l) {   // l wave-uniform
    const unsigned long long x = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)x, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(x >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

__device__ __forceinline__ void km_cswap(double &a, double &b, bool do_swap) {
    const double x = a;
    a = do_swap ? b : a;
    b = do_swap ? x : b;
}
// (fully unrolled, register-only: the out-of-line form with indexed local arrays was a call with
// 54 scratch accesses on every Lloyd iteration)
// WAVE: called by a whole wave with wave-uniform arguments (k_kmeans_s): lane j computes mean j, so
// the four IEEE divisions cost one division's latency; else by one thread (k_kmeans).
template <bool WAVE, typename I>
__device__ __forceinline__ void km_update(const uint32_t *k, const I *cut, const double *sum, double *c) {
    double old[KM_K], nc[KM_K], sums[KM_K];
    I wa[KM_K], we[KM_K];
    bool empty[KM_K];
    bool any_empty = false;
#pragma unroll
    for (int j = 0; j < KM_K; ++j) {
        old[j] = nc[j] = c[j];
        wa[j] = cut[j];
        we[j] = cut[j + 1];
        empty[j] = we[j] <= wa[j];
        sums[j] = empty[j] ? 0.0 : sum[j];
        any_empty = any_empty || empty[j];
    }
    if (any_empty) {   // degenerate data only
#pragma unroll
        for (int j = 0; j < KM_K; ++j) {
            if (!empty[j]) continue;
            double best = 0.0, bx = 0.0;
            I bi = -1;
            int bq = -1;
#pragma unroll
            for (int q = 0; q < KM_K; ++q) {
                if (we[q] - wa[q] < 2) continue;
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const I i = e ? we[q] - 1 : wa[q];
                    const double x = (double)key2f(k[i]);
                    const double dd = fabs(x - old[q]);
                    if (dd > best || (dd == best && dd > 0.0 && i < bi)) {
                        best = dd;
                        bi = i;
                        bq = q;
                        bx = x;
                    }
                }
            }
            if (bi >= 0) {
                nc[j] = bx;
#pragma unroll
                for (int q = 0; q < KM_K; ++q)
                    if (q == bq) {
                        sums[q] -= bx;
                        if (bi == wa[q]) ++wa[q]; else --we[q];
                    }
            }
        }
    }
    if (WAVE) {
        const int l = threadIdx.x & 3;
        double sl = sums[0], cl = (double)(we[0] - wa[0]);
#pragma unroll
        for (int j = 1; j < KM_K; ++j)
            if (l == j) { sl = sums[j]; cl = (double)(we[j] - wa[j]); }
        const double ml = sl / cl;
#pragma unroll
        for (int j = 0; j < KM_K; ++j)
            if (!empty[j]) nc[j] = readlane_d(ml, j);
    } else {
#pragma unroll
        for (int j = 0; j < KM_K; ++j)
            if (!empty[j]) nc[j] = sums[j] / (double)(we[j] - wa[j]);
    }
    // insertion sort by adjacent swaps while strictly greater (KM_K = 4, unrolled)
    static_assert(KM_K == 4, "km_update's sort is written for four centres");
    km_cswap(nc[0], nc[1], nc[0] > nc[1]);
    if (nc[1] > nc[2]) {
        km_cswap(nc[1], nc[2], true);
        km_cswap(nc[0], nc[1], nc[0] > nc[1]);
    }
    if (nc[2] > nc[3]) {
        km_cswap(nc[2], nc[3], true);
        if (nc[1] > nc[2]) {
            km_cswap(nc[1], nc[2], true);
            km_cswap(nc[0], nc[1], nc[0] > nc[1]);
        }
    }
#pragma unroll
    for (int j = 0; j < KM_K; ++j) c[j] = nc[j];
}

// One block (16 waves) per volume.  Cluster sums: head partial tile + whole tiles (a difference of
// the exclusive prefix of the tile sums, in LDS or -- large volumes, tile sums from k_km_tiles -- in
// global memory) + tail partial tile (deterministic: fixed orders throughout).
__global__ void __launch_bounds__(KM_TPB) k_kmeans(const uint32_t *__restrict__ keys,
                                                  int64_t V, double *tile_scratch,
                                                  int64_t max_ktiles, VolScalars *sc) {
    __shared__ double s_tiles[KM_LDS_TILES + 1];   // tile sums -> exclusive prefix of them
    __shared__ double s_wtot[KM_TPB / 64];
    __shared__ float s_samp[KM_SAMPLES];
    __shared__ double s_c[KM_K], s_sum[KM_K];
    __shared__ int64_t s_cut[KM_K + 1], s_new[KM_K + 1];
    __shared__ int s_done;
    const int64_t b = blockIdx.x;
    const int64_t n = sc[b].n_mask;
    if (n <= 0) return;
    const uint32_t *k = keys + b * V;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const int64_t nt = (n + KM_TILE - 1) / KM_TILE;
    double *gt = tile_scratch + b * (max_ktiles + 1);   // [nt + 1]: tile sums -> their exclusive prefix
    const bool in_lds = nt <= KM_LDS_TILES;
    if (in_lds)
        for (int64_t tt = w; tt < nt; tt += KM_TPB / 64) {
            const double ts = km_tile_sum(k, tt, 0, n);
            if (lane == 0) s_tiles[tt] = ts;
        }
    const int64_t stride = n <= (int64_t)KM_SAMPLES * 64 ? 64 : (n + KM_SAMPLES - 1) / KM_SAMPLES;
    const int64_t ns = (n - 1) / stride + 1;   // samples at 0, stride, 2 stride, ... < n
    for (int64_t j = t; j < ns; j += KM_TPB) s_samp[j] = key2f(k[j * stride]);
    __syncthreads();
    if (in_lds) {   // exclusive prefix of the tile sums (fixed order: thread chunks, wave scan)
        const int per = (int)((nt + KM_TPB - 1) / KM_TPB);
        const int64_t t0 = (int64_t)t * per, t1 = t0 + per < nt ? t0 + per : nt;
        double tv[KM_LDS_TILES / KM_TPB];
        double mine = 0.0;
        for (int64_t tt = t0; tt < t1; ++tt) { tv[tt - t0] = s_tiles[tt]; mine += tv[tt - t0]; }
        double inc = mine;
        for (int off = 1; off < 64; off <<= 1) {
            const double o = __shfl_up(inc, off, 64);
            if (lane >= off) inc += o;
        }
        double run = __shfl_up(inc, 1, 64);
        if (lane == 0) run = 0.0;
        if (lane == 63) s_wtot[w] = inc;
        __syncthreads();
        for (int ww = 0; ww < w; ++ww) run += s_wtot[ww];
        for (int64_t tt = t0; tt < t1; ++tt) { s_tiles[tt] = run; run += tv[tt - t0]; }
        if (t1 == nt && t0 < t1) s_tiles[nt] = run;
    } else {   // the same fixed-order prefix over k_km_tiles' sums, in place in global memory
        const int64_t per = (nt + KM_TPB - 1) / KM_TPB;
        const int64_t t0 = (int64_t)t * per, t1 = t0 + per < nt ? t0 + per : nt;
        double mine = 0.0;
        for (int64_t tt = t0; tt < t1; ++tt) mine += gt[tt];
        double inc = mine;
        for (int off = 1; off < 64; off <<= 1) {
            const double o = __shfl_up(inc, off, 64);
            if (lane >= off) inc += o;
        }
        double run = __shfl_up(inc, 1, 64);
        if (lane == 0) run = 0.0;
        if (lane == 63) s_wtot[w] = inc;
        __syncthreads();
        for (int ww = 0; ww < w; ++ww) run += s_wtot[ww];
        for (int64_t tt = t0; tt < t1; ++tt) { const double v = gt[tt]; gt[tt] = run; run += v; }
        if (t1 == nt && t0 < t1) gt[nt] = run;
        __threadfence_block();
    }
    if (t < KM_K) s_c[t] = (double)key2f(k[(n * (2 * t + 1)) / (2 * KM_K)]);
    if (t == 0) { s_cut[0] = -1; s_done = 0; }
    __syncthreads();
    int it = 0;
    for (it = 1; it <= 300; ++it) {
        if (w < KM_K - 1) {
            // the boundary against the next LARGER centre value (centres are kept sorted; a centre
            // equal to its predecessor gets no values: ties go to the lowest index).  Wave-uniform.
            double chi = 0.0;
            bool up = false;
            for (int m = w + 1; m < KM_K; ++m)
                if (!up && s_c[m] > s_c[w]) { chi = s_c[m]; up = true; }
            const int64_t c = up ? km_boundary(k, n, s_c[w], chi, s_samp, ns, stride) : n;
            if (lane == 0) s_new[w + 1] = c;
        }
        __syncthreads();
        if (t == 0) {
            s_new[0] = 0;
            s_new[KM_K] = n;
            for (int j = 2; j < KM_K; ++j)
                if (s_new[j] < s_new[j - 1]) s_new[j] = s_new[j - 1];
            bool same = true;
            for (int j = 0; j <= KM_K; ++j) same = same && s_new[j] == s_cut[j];
            s_done = same;
            for (int j = 0; j <= KM_K; ++j) s_cut[j] = s_new[j];
        }
        __syncthreads();
        if (s_done) break;
        if (w < KM_K) {   // wave w updates centre w: head + whole tiles (prefix) + tail
            const int64_t a = s_cut[w], e = s_cut[w + 1];
            if (e > a) {
                const int64_t ta = a / KM_TILE, te = (e - 1) / KM_TILE;
                double head, tail;
                km_tile_sum2(k, ta, te, a, e, head, tail);
                if (lane == 0) {
                    double sum = head;
                    if (te > ta + 1) sum += in_lds ? s_tiles[te] - s_tiles[ta + 1] : gt[te] - gt[ta + 1];
                    if (te != ta) sum += tail;
                    s_sum[w] = sum;
                }
            }
        }
        __syncthreads();
        if (t == 0) km_update<false>(k, s_cut, s_sum, s_c);   // means, empty-cluster relocation, sort
        __syncthreads();
    }
    if (t == 0) {   // VDP_km: the lowest non-empty cluster
        int64_t low = 0;
        for (int j = KM_K - 1; j >= 0; --j)
            if (s_cut[j + 1] > s_cut[j]) low = s_cut[j + 1] - s_cut[j];
        sc[b].n_km0 = low;
        sc[b].km_iters = it;
        for (int j = 0; j < KM_K; ++j) sc[b].km_c[j] = s_c[j];
    }
}

// k-means for volumes of up to KMS_TILES * 64 keys (the 128x128x24 bench studies; larger volumes
// take k_kmeans): the same Lloyd iteration over 64-key tiles.  All 16 waves sum the tiles (16 tiles
// per wave at a time, one exchange reduction for the 16) into an exclusive prefix in LDS and take the
// LDS sample from the same loads (the sample stride is a whole number of tiles).  Then ONE wave runs
// the iterations, with no barrier: per boundary it checks whether the cut still lies in the previous
// iteration's sample interval (two LDS reads; the 64-ary sample search only when it moved), loads
// the 192-key window of sorted keys around that interval (three aligned tiles, holding the interval
// and the tile the cut falls in; the three boundaries' loads in flight together), finds the cut and
// its partial tile sums (below / above the cut inside its tile) in the same registers, and forms the
// four cluster sums from the prefix.  k_kmeans takes two dependent global rounds, four barriers and
// a one-thread update per iteration.
#define KMS_TILES 8192
#define KMS_WAVES (KM_TPB / 64)

// Fixed-order wave sums of N values per lane (N a power of two, 2 <= N <= 64), by halving exchanges:
// step s pairs lane l with l ^ (32 >> s), and the lane with that bit clear keeps the lower half of
// its values (adding its partner's), the other the upper half; then butterflies over the remaining
// lane bits.  Lane l ends with the total of value (l >> (6 - log2 N)); every lane holding a total
// holds the same bits (a + b = b + a).  log2 N + 6 - log2 N = 6 exchanges of N - 1 + 6 - log2 N
// values instead of 6 N.
template <int H, int OFF, int N>
__device__ __forceinline__ void wave_sums_halve(double (&v)[N], int lane) {
    if constexpr (H >= 1) {
        const bool up = (lane & OFF) != 0;
#pragma unroll
        for (int i = 0; i < H; ++i) {
            const double keep = up ? v[H + i] : v[i], send = up ? v[i] : v[H + i];
            v[i] = keep + __shfl_xor(send, OFF, 64);
        }
        wave_sums_halve<H / 2, OFF / 2>(v, lane);
    }
}
template <int N>
__device__ __forceinline__ double wave_sums_x(double (&v)[N]) {
    static_assert(N >= 2 && N <= 64 && (N & (N - 1)) == 0, "N a power of two in [2, 64]");
    const int lane = threadIdx.x & 63;
    wave_sums_halve<N / 2, 32>(v, lane);
#pragma unroll
    for (int off = 32 / N; off >= 1; off >>= 1) v[0] += __shfl_xor(v[0], off, 64);
    return v[0];
}

__device__ __forceinline__ double wave_sum_d(double v) {   // fixed shuffle tree, result in all lanes
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

__global__ void __launch_bounds__(KM_TPB) k_kmeans_s(const uint32_t *__restrict__ keys, int64_t V,
                                                    VolScalars *sc) {
    __shared__ double s_pre[KMS_TILES + 1];   // 64-key tile sums -> their exclusive prefix
    __shared__ double s_wtot[KMS_WAVES];
    __shared__ float s_samp[KM_SAMPLES];
    const int64_t b = blockIdx.x;
    const int64_t n64 = sc[b].n_mask;
    if (n64 <= 0) return;
    if (n64 > (int64_t)KMS_TILES * 64) {   // (the host launches k_kmeans for such volumes)
        if (threadIdx.x == 0) sc[b].km_iters = -1;
        return;
    }
#ifdef KM_PROF
    const uint64_t kp0 = wall_clock64();
#endif
    const uint32_t *k = keys + b * V;
    const int n = (int)n64;   // positions below fit 32 bits (n <= 2^19): half the index instructions
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const int nt = (n + 63) / 64;
    const int tps_log = nt > KM_SAMPLES ? 1 : 0;   // tiles per sample: 1 or 2 (nt <= 2 KM_SAMPLES)
    const int stride = 64 << tps_log;
    const int ns = (n - 1) / stride + 1;   // samples at 0, stride, 2 stride, ... < n
    // tile sums and the sample (key j * stride = the first key of tile j << tps_log)
    for (int t0 = (int)w * 16; t0 < nt; t0 += KMS_WAVES * 16) {
        float f[16];
        double v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) f[q] = km_key_in(k, (t0 + q) * 64 + lane, 0, n);
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            v[q] = (double)f[q];
            const int tq = t0 + q;
            if (lane == 0 && tq < nt && (tq & ((1 << tps_log) - 1)) == 0) s_samp[tq >> tps_log] = f[q];
        }
        const double ts = wave_sums_x<16>(v);
        const int tt = t0 + (lane >> 2);
        if ((lane & 3) == 0 && tt < nt) s_pre[tt] = ts;
    }
    __syncthreads();
    {   // exclusive prefix of the tile sums (fixed order: thread chunks, wave scan)
        const int per = (int)((nt + KM_TPB - 1) / KM_TPB);
        const int t0 = (int)t * per, t1 = t0 + per < nt ? t0 + per : nt;
        double mine = 0.0;   // (each thread rewrites only its own chunk)
        for (int tt = t0; tt < t1; ++tt) mine += s_pre[tt];
        double inc = mine;
        for (int off = 1; off < 64; off <<= 1) {
            const double o = __shfl_up(inc, off, 64);
            if (lane >= off) inc += o;
        }
        double run = __shfl_up(inc, 1, 64);
        if (lane == 0) run = 0.0;
        if (lane == 63) s_wtot[w] = inc;
        __syncthreads();
        for (int ww = 0; ww < w; ++ww) run += s_wtot[ww];
        for (int tt = t0; tt < t1; ++tt) { const double v = s_pre[tt]; s_pre[tt] = run; run += v; }
        if (t1 == nt && t0 < t1) s_pre[nt] = run;
    }
    __syncthreads();
    if (w != 0) return;   // one wave iterates; every value below is wave-uniform
    double c[KM_K];
#pragma unroll
    for (int j = 0; j < KM_K; ++j) c[j] = (double)key2f(k[(int)(((int64_t)n * (2 * j + 1)) / (2 * KM_K))]);
    // the fixed cuts 0 and n: cut 0 has Σ[0, min(64, n)) above it; cut n has Σ[64 floor(n / 64), n)
    // below it
    const int wbn = ((n - 1) / 64) * 64;
    double plo_n;
    {
        const int tn = (n / 64) * 64;
        double lo = 0.0;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const int i = wbn + 64 * q + lane;
            const float x = km_key_in(k, i, (decltype(i))0, (decltype(i))n);
            lo += i >= tn && i < n ? (double)x : 0.0;
        }
        plo_n = wave_sum_d(lo);
    }
    const double phi_0 = s_pre[1] - s_pre[0];
    int cut[KM_K + 1];
    double plo[KM_K + 1], phi[KM_K + 1];
#pragma unroll
    for (int j = 0; j <= KM_K; ++j) { cut[j] = -1; plo[j] = 0.0; phi[j] = 0.0; }
    int jsp[KM_K - 1], wbp[KM_K - 1];
    float wv[KM_K - 1][3];
#pragma unroll
    for (int j = 0; j < KM_K - 1; ++j) {
        jsp[j] = -1;
        wbp[j] = -1;
#pragma unroll
        for (int q = 0; q < 3; ++q) wv[j][q] = 0.0f;
    }
#ifdef KM_PROF
    const uint64_t kp1 = wall_clock64();
    int nsearch = 0;
#endif
    int it = 0;
    for (it = 1; it <= 300; ++it) {
        // sample intervals of the three boundaries (LDS only); a boundary is taken against the next
        // LARGER centre (centres are kept sorted; one equal to its predecessor gets no values)
        bool up[KM_K - 1];
        double clo[KM_K - 1], chi[KM_K - 1];
        int lo[KM_K - 1], hi[KM_K - 1], wb[KM_K - 1];
#pragma unroll
        for (int j = 0; j < KM_K - 1; ++j) {
            up[j] = false;
            chi[j] = 0.0;
#pragma unroll
            for (int m = j + 1; m < KM_K; ++m)
                if (!up[j] && c[m] > c[j]) { chi[j] = c[m]; up[j] = true; }
            clo[j] = c[j];
            lo[j] = hi[j] = n;
            wb[j] = wbn;
            if (up[j]) {
                int js = jsp[j];
                bool still = js >= 0;
                if (still) {   // sample js true (or js = ns) and sample js - 1 false (or js = 0)
                    const bool tr = js < ns ? km_closer((double)s_samp[js], clo[j], chi[j]) : true;
                    const bool fa = js == 0 ? true : !km_closer((double)s_samp[js - 1], clo[j], chi[j]);
                    still = tr && fa;
                }
                if (!still) {
                    js = km_sample_search(s_samp, ns, clo[j], chi[j]);
#ifdef KM_PROF
                    ++nsearch;
#endif
                }
                jsp[j] = js;
                lo[j] = js == 0 ? 0 : (js - 1) * stride + 1;   // the cut is in [lo, hi]
                hi[j] = js >= ns ? n : js * stride;
                wb[j] = (lo[j] / 64) * 64;   // hi - lo < stride <= 128: [wb, wb + 192) holds [lo, hi]
            }                                // and the whole tile of any cut in it
        }
#pragma unroll
        for (int j = 0; j < KM_K - 1; ++j)
            if (wb[j] != wbp[j]) {   // (a boundary whose interval stayed keeps its window)
                wbp[j] = wb[j];
#pragma unroll
                for (int q = 0; q < 3; ++q) wv[j][q] = km_key_in(k, wb[j] + 64 * q + lane, 0, n);
            }
        int nc[KM_K + 1];
        double pv[8];
        nc[0] = 0;
        nc[KM_K] = n;
#pragma unroll
        for (int j = 0; j < KM_K - 1; ++j) {
            int cj = n;
            if (up[j]) {
                uint64_t any = 0ull;
                int first = 192;
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    const int i = wb[j] + 64 * q + lane;
                    const bool pr = i >= lo[j] && i < hi[j] && km_closer((double)wv[j][q], clo[j], chi[j]);
                    const uint64_t m = __ballot(pr);
                    if (!any && m) first = 64 * q + __ffsll((long long)m) - 1;
                    any |= m;
                }
                cj = any ? wb[j] + first : hi[j];
            }
            nc[j + 1] = cj;
            const int tc = (cj / 64) * 64;   // the cut's tile (inside the window)
            double a = 0.0, e = 0.0;
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                const int i = wb[j] + 64 * q + lane;
                const bool in = i >= tc && i < tc + 64 && i < n;
                a += in && i < cj ? (double)wv[j][q] : 0.0;
                e += in && i >= cj ? (double)wv[j][q] : 0.0;
            }
            pv[2 * j] = a;
            pv[2 * j + 1] = e;
        }
        pv[6] = pv[7] = 0.0;
        const double red = wave_sums_x<8>(pv);   // value q's total in lanes 8q .. 8q + 7
        double nlo[KM_K + 1], nhi[KM_K + 1];
        nlo[0] = 0.0;
        nhi[0] = phi_0;
        nlo[KM_K] = plo_n;
        nhi[KM_K] = 0.0;
#pragma unroll
        for (int j = 0; j < KM_K - 1; ++j) {
            nlo[j + 1] = readlane_d(red, 16 * j);
            nhi[j + 1] = readlane_d(red, 16 * j + 8);
        }
#pragma unroll
        for (int j = 2; j < KM_K; ++j)
            if (nc[j] < nc[j - 1]) {   // (as k_kmeans; sorted centres give ordered cuts)
                nc[j] = nc[j - 1];
                nlo[j] = nlo[j - 1];
                nhi[j] = nhi[j - 1];
            }
        bool same = true;
#pragma unroll
        for (int j = 0; j <= KM_K; ++j) same = same && nc[j] == cut[j];
        if (same) break;
        double sum[KM_K];
#pragma unroll
        for (int j = 0; j <= KM_K; ++j) { cut[j] = nc[j]; plo[j] = nlo[j]; phi[j] = nhi[j]; }
#pragma unroll
        for (int j = 0; j < KM_K; ++j) {   // head partial + whole tiles (prefix) + tail partial
            const int a = cut[j], e = cut[j + 1];
            const int ta = a / 64, te = e / 64;
            sum[j] = e <= a ? 0.0
                            : (ta == te ? phi[j] - phi[j + 1] : phi[j] + (s_pre[te] - s_pre[ta + 1]) + plo[j + 1]);
        }
        km_update<true>(k, cut, sum, c);   // means, empty-cluster relocation, sort
    }
    if (lane == 0) {   // VDP_km: the lowest non-empty cluster
        int low = 0;
#pragma unroll
        for (int j = KM_K - 1; j >= 0; --j)
            if (cut[j + 1] > cut[j]) low = cut[j + 1] - cut[j];
        sc[b].n_km0 = low;
        sc[b].km_iters = it;
#pragma unroll
        for (int j = 0; j < KM_K; ++j) sc[b].km_c[j] = c[j];
#ifdef KM_PROF
        const uint64_t kp2 = wall_clock64();
        if (b < 4)
            printf("KMPROF b=%d n=%d it=%d init=%lu loop=%lu searches=%d\n", (int)b, n, it,
                   (unsigned long)(kp1 - kp0), (unsigned long)(kp2 - kp1), nsearch);
#endif
    }
}

// =============================================================================================
// cohort histogram (build-defined, BASELINE config 4): 1024 bins over [0, 1.5) of the
// p99-normalised masked N4 values, bin = int(nv * (1024 / 1.5f)).  Computed from the sorted keys
// (bins are monotone in the value, so each thread's contiguous chunk produces runs of equal bins:
// one LDS atomic per run), per-volume rows, then a fixed-order sum over volumes (no float or
// global atomics: deterministic).
// =============================================================================================
// Rows by search: over the sorted keys the bin g(i) (-1 below 0, 1024 at
// or above 1.5 and for NaN) is non-decreasing when p99 > 0, so a bin's count is the distance
// between the first indices with g >= e and g >= e + 1.  A 1024-key sample in LDS narrows each
// search to one sample interval.  Volumes with p99 <= 0 / inf / NaN take a scan with per-value LDS adds.
__device__ __forceinline__ int cohort_g(uint32_t key, float p99) {
    const float nv = key2f(key) / p99;
    if (nv >= 0.0f && nv < 1.5f) {
        const int bi = (int)(nv * ((float)VH_COHORT_BINS / 1.5f));
        return bi > VH_COHORT_BINS - 1 ? VH_COHORT_BINS - 1 : bi;
    }
    return nv < 0.0f ? -1 : VH_COHORT_BINS;
}

#define CO_TPB 1024
#define CO_SAMPLES 4096   // LDS sample: the global part of an edge's search spans <= n / 4096 + 1 keys
__global__ void __launch_bounds__(CO_TPB) k_cohort_search(const uint32_t *__restrict__ keys,
                                                         const VolScalars *sc, int64_t V,
                                                         uint32_t *rows) {
    __shared__ int s_g[CO_SAMPLES];
    __shared__ int64_t s_first[VH_COHORT_BINS + 1];
    const int64_t b = blockIdx.x;
    const int64_t n = sc[b].n_mask;
    const float p99 = sc[b].p99;
    const uint32_t *k = keys + b * V;
    const int t = threadIdx.x;
    if (n <= 0 || !(p99 > 0.0f) || isinf(p99)) {   // scan path (k_cohort_vol)
        uint32_t *h = reinterpret_cast<uint32_t *>(s_g);
        for (int i = t; i < VH_COHORT_BINS; i += CO_TPB) h[i] = 0u;
        __syncthreads();
        const int64_t per = (n + CO_TPB - 1) / CO_TPB;
        const int64_t cs = t * per < n ? t * per : n, ce = cs + per < n ? cs + per : n;
        for (int64_t i = cs; i < ce; ++i) {
            const float nv = key2f(k[i]) / p99;
            if (nv >= 0.0f && nv < 1.5f) {
                int bi = (int)(nv * ((float)VH_COHORT_BINS / 1.5f));
                atomicAdd(&h[bi > VH_COHORT_BINS - 1 ? VH_COHORT_BINS - 1 : bi], 1u);
            }
        }
        __syncthreads();
        for (int i = t; i < VH_COHORT_BINS; i += CO_TPB) rows[b * VH_COHORT_BINS + i] = h[i];
        return;
    }
    const int S = n < CO_SAMPLES ? (int)n : CO_SAMPLES;
    {   // the sample's loads all in flight (unconditional, index clamped: a guarded load waits)
        uint32_t kv[CO_SAMPLES / CO_TPB];
#pragma unroll
        for (int q = 0; q < CO_SAMPLES / CO_TPB; ++q) {
            const int j = t + q * CO_TPB;
            kv[q] = k[j < S ? ((int64_t)j * n) / S : 0];
        }
#pragma unroll
        for (int q = 0; q < CO_SAMPLES / CO_TPB; ++q) {
            const int j = t + q * CO_TPB;
            if (j < S) s_g[j] = cohort_g(kv[q], p99);
        }
    }
    __syncthreads();
    for (int e = t; e <= VH_COHORT_BINS; e += CO_TPB) {
        // last sample j with g < e (sample positions are increasing, g non-decreasing)
        int lo = -1, hi = S;   // s_g[lo] < e <= s_g[hi] (virtual ends)
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (s_g[mid] < e) lo = mid; else hi = mid;
        }
        // first index i with g(i) >= e lies in (pos(lo), pos(hi)]
        int64_t a = lo < 0 ? -1 : ((int64_t)lo * n) / S, z = hi >= S ? n : ((int64_t)hi * n) / S;
        while (z - a > 1) {
            const int64_t mid = (a + z) >> 1;
            if (cohort_g(k[mid], p99) < e) a = mid; else z = mid;
        }
        s_first[e] = z;
    }
    __syncthreads();
    for (int i = t; i < VH_COHORT_BINS; i += CO_TPB)
        rows[b * VH_COHORT_BINS + i] = (uint32_t)(s_first[i + 1] - s_first[i]);
}

// the cohort: per bin the sum of the volumes' rows (integers: any order gives the same sum).
// Block = 64 bins x 16 volume groups; a thread sums every 16th volume with its loads in flight
// together, then the 16 groups are added in LDS (one thread per bin summing 256 rows in a loop
// waited on its loads: ~0.03 ms of the cohort's 0.09 ms).
#define CS_BINS 64
#define CS_GROUPS 16
__global__ void __launch_bounds__(CS_BINS * CS_GROUPS) k_cohort_sum(const uint32_t *rows, int64_t nb,
                                                                   uint64_t *cohort) {
    __shared__ uint64_t s_part[CS_GROUPS][CS_BINS];
    const int bin = blockIdx.x * CS_BINS + (threadIdx.x % CS_BINS), g = threadIdx.x / CS_BINS;
    uint64_t s = 0;
    int64_t v = g;
    for (; v + 7 * CS_GROUPS < nb; v += 8 * CS_GROUPS) {
        uint32_t r[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) r[q] = rows[(v + q * CS_GROUPS) * VH_COHORT_BINS + bin];
#pragma unroll
        for (int q = 0; q < 8; ++q) s += r[q];
    }
    for (; v < nb; v += CS_GROUPS) s += rows[v * VH_COHORT_BINS + bin];
    s_part[g][threadIdx.x % CS_BINS] = s;
    __syncthreads();
    if (g == 0) {
        uint64_t tot = 0;
        for (int q = 0; q < CS_GROUPS; ++q) tot += s_part[q][threadIdx.x];
        cohort[bin] = tot;
    }
}

// =============================================================================================
// SNR (Vent_Analysis.py:337-357): signal = A[mask>0]; noise = A outside the ix_(rr, cc, ss) box and
// outside the first/last 20 rows.  32-row slabs, one column per lane; signal rows from the
// mask != 0 bitmap, rows that are neither signal nor noise are not loaded.  Per-block double
// partials (fixed order), then a finish kernel.  With N4, k_n4_final computes the same partials
// from the image it already streams (vh_batch::snr_fused) and only the finish runs here.
// =============================================================================================
__global__ void __launch_bounds__(VH_TPB) k_snr(const float *__restrict__ hp,
                                               const uint32_t *__restrict__ colbnz,
                                               const VolScalars *sc, int64_t R, int64_t C,
                                               int64_t Z, int64_t V, int64_t ncb, SnrBox sb) {
    __shared__ uint32_t s_rows[2];
    __shared__ double s_red[4][VH_TPB / 64];
    const int64_t b = blockIdx.y;
    const int64_t CZ = C * Z;
    const int64_t sl = blockIdx.x / ncb;
    const int64_t col = (blockIdx.x % ncb) * VH_TPB + threadIdx.x;
    const int64_t x0 = sl * VH_SLAB;
    const int nr = (int)(R - x0 < VH_SLAB ? R - x0 : VH_SLAB);
    const VolScalars s = sc[b];
    snr_slab_rows(sb, s, b, R, x0, nr, s_rows);
    __syncthreads();
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    if (col < CZ) {
        const int64_t nw = (R + 31) >> 5;
        const uint32_t sig = colbnz[(b * nw + sl) * CZ + col];
        const uint32_t noise = snr_col_noise(sb, s, b, Z, col, s_rows);
        snr_count(acc, noise);
        const uint32_t need = sig | noise;
        const float *a = hp + b * V + x0 * CZ + col;
        for (int i0 = 0; i0 < nr; i0 += 8) {   // 8 rows of loads in flight
            float v[8];
            // unconditional loads at a clamped row, then the selection (a guarded load compiles to
            // a branch that waits for it; nearly every row is signal or noise anyway)
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = a[(int64_t)(i0 + k < nr ? i0 + k : nr - 1) * CZ];
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = (i0 + k < nr && ((need >> (i0 + k)) & 1u)) ? v[k] : 0.0f;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int i = i0 + k;
                if (i >= nr) break;
                snr_add(acc, v[k], (sig >> i) & 1u, (noise >> i) & 1u);
            }
        }
    }
    snr_block_write(acc, s_red, sb.part + (b * sb.nparts + blockIdx.x) * 4);
}

// One wave per volume: lane l sums parts l, l + 64, ... in order, then a fixed shuffle tree (one
// thread per volume walking its parts one load after another took 13 us).
__global__ void k_snr_finish(const double *part, int64_t nparts, int64_t nb, VolScalars *sc) {
    const int64_t b = blockIdx.x * (int64_t)(blockDim.x / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (b >= nb) return;
    double a[4] = {0, 0, 0, 0};
    for (int64_t p = lane; p < nparts; p += 64)
        for (int q = 0; q < 4; ++q) a[q] += part[(b * nparts + p) * 4 + q];
    for (int q = 0; q < 4; ++q)
        for (int off = 32; off > 0; off >>= 1) a[q] += __shfl_xor(a[q], off, 64);
    if (lane != 0) return;
    const double nsig = (double)sc[b].n_mask;
    if (!sc[b].snr_ok || a[3] <= 0.0 || nsig <= 0.0) {
        sc[b].snr = __longlong_as_double(0x7ff8000000000000ll);
        return;
    }
    // (mean(signal) - mean(noise)) / std(noise), ddof 0, double accumulation
    const double ms = a[0] / nsig;
    const double mn = a[1] / a[3];
    double var = a[2] / a[3] - mn * mn;
    if (var < 0.0) var = 0.0;
    sc[b].snr = (ms - mn) / sqrt(var);
}

void vh_launch_snr(vh_batch *b) {
    hipStream_t st = b->stream;
    const SnrBox sb{b->d_rowany, b->d_sliceany, b->d_snrpart, b->slab_blocks};
    if (!b->snr_fused) {
        ScopedKTimer tm(b, "snr", 5.0 * (double)b->V);
        k_snr<<<slab_grid(b), VH_TPB, 0, st>>>(b->d_hp, b->d_colbnz, b->d_sc, b->R, b->C, b->Z,
                                               b->V, b->part_blocks, sb);
        VH_CHECK_LAUNCH();
    }
    k_snr_finish<<<(unsigned)((b->nb + 3) / 4), 256, 0, st>>>(b->d_snrpart, b->slab_blocks, b->nb, b->d_sc);
    VH_CHECK_LAUNCH();
}

// =============================================================================================
// the chain
// =============================================================================================
// k-means of the batch (after the sort) on stream st
static void vh_launch_kmeans(vh_batch *b, hipStream_t st) {
    ScopedKTimer tm(b, "kmeans", 0.0, false, st);
    const int64_t max_ktiles = (b->V + KM_TILE - 1) / KM_TILE;
    // free after the sort: 4V bytes per volume >= 8 (V / 1024 + 1)
    double *scratch = reinterpret_cast<double *>(b->d_keys1);
    if (max_ktiles > KM_LDS_TILES) {
        k_km_tiles<<<dim3((unsigned)((max_ktiles + KM_TPB / 64 - 1) / (KM_TPB / 64)), (unsigned)b->nb),
                     KM_TPB, 0, st>>>(b->d_keys0, b->V, scratch, max_ktiles, b->d_sc);
        VH_CHECK_LAUNCH();
    }
    if (b->V <= (int64_t)KMS_TILES * 64 && !(getenv("VH_KM_OLD") && atoi(getenv("VH_KM_OLD"))))
        k_kmeans_s<<<(unsigned)b->nb, KM_TPB, 0, st>>>(b->d_keys0, b->V, b->d_sc);
    else
        k_kmeans<<<(unsigned)b->nb, KM_TPB, 0, st>>>(b->d_keys0, b->V, scratch, max_ktiles, b->d_sc);
    VH_CHECK_LAUNCH();
}

void vh_launch_vdp_chain(vh_batch *b, const float *d_n4, const vh_run_opts &o) {
    hipStream_t st = b->stream;
    const int64_t CZ = b->CZ;
    // the chain's span on the batch stream (profile runs): its kernels plus the gaps between them
    // (bench.py's non_n4_wall_us_per_step)
    ScopedKTimer chain(b, "vdp_chain", 0.0);
    if (!(o.do_n4 && b->keys_fused)) {   // (after N4, k_n4_final emitted every volume's keys)
        ScopedKTimer tm(b, "gather", 5.0 * (double)b->V);
        k_gather<<<col_grid(b), VH_TPB, 0, st>>>(d_n4, b->d_mask, b->d_colrange, b->d_colstart,
                                                 CZ, b->V, b->d_sc, 0, b->d_keys0);
        VH_CHECK_LAUNCH();
    }
    {
        ScopedKTimer tm(b, "sort", 0.0);
        if (b->nb == 1 && b->V >= ((int64_t)1 << 20)) {   // one large volume: the grid sort
            const int64_t nchunk = (b->V + VSG_CHUNK - 1) / VSG_CHUNK;
            if (b->sortg_cap < nchunk * 256) {
                if (b->d_sortg) HIP_TRY(hipFree(b->d_sortg));
                b->d_sortg = nullptr;
                b->sortg_cap = 0;
                HIP_TRY(hipMalloc(&b->d_sortg, sizeof(uint32_t) * nchunk * 256));
                b->sortg_cap = nchunk * 256;
            }
            uint32_t *cnt = (uint32_t *)b->d_sortg;
            uint32_t *kin = b->d_keys0, *kout = b->d_keys1;
            for (int p = 0; p < 4; ++p) {
                k_sortg_count<<<(unsigned)nchunk, VS_TPB, 0, st>>>(kin, b->d_sc, 0, 8 * p, cnt);
                VH_CHECK_LAUNCH();
                k_sortg_offsets<<<1, VS_TPB, 0, st>>>(cnt, b->d_sc, 0);
                VH_CHECK_LAUNCH();
                k_sortg_scatter<<<(unsigned)nchunk, VS_TPB, 0, st>>>(kin, kout, cnt, b->d_sc, 0, 8 * p);
                VH_CHECK_LAUNCH();
                std::swap(kin, kout);
            }
        } else {
            k_sort_vol<<<(unsigned)b->nb, VS_TPB, 0, st>>>(b->d_keys0, b->d_keys1, b->d_sc, b->V);
            VH_CHECK_LAUNCH();
        }
    }
    {
        ScopedKTimer tm(b, "mean", 0.0);
        const int64_t max_chunks = (b->V + 8191) / 8192;
        float *chunk = reinterpret_cast<float *>(b->d_part);   // part holds >= nb*max_chunks floats
        k_chunk_sums<<<dim3((unsigned)((max_chunks + VH_TPB / 64 - 1) / (VH_TPB / 64)), (unsigned)b->nb),
                       VH_TPB, 0, st>>>(b->d_keys0, b->d_sc, b->V, max_chunks, chunk);
        VH_CHECK_LAUNCH();
        k_mean_p99<<<(unsigned)((b->nb + 63) / 64), 64, 0, st>>>(b->d_keys0, chunk, max_chunks,
                                                                  b->V, b->nb, b->d_sc);
        VH_CHECK_LAUNCH();
    }
    if (o.do_cohort) {
        ScopedKTimer tm(b, "cohort", 0.0);
        uint32_t *rows = b->d_tilecnt;   // free after the sort: nb*256*max_tiles >= nb*1024 u32
        k_cohort_search<<<(unsigned)b->nb, CO_TPB, 0, st>>>(b->d_keys0, b->d_sc, b->V, rows);
        VH_CHECK_LAUNCH();
        k_cohort_sum<<<VH_COHORT_BINS / CS_BINS, CS_BINS * CS_GROUPS, 0, st>>>(rows, b->nb, b->d_cohort);
        VH_CHECK_LAUNCH();
    }
    // k-means next, while the sorted keys the mean and cohort just read are still in L2 / MALL
    // (after the classify sweep's streams it took 148 instead of 140 us; the cohort, moved before
    // the sweep for the same reason, 35 -> 24 us)
    if (o.do_kmeans) vh_launch_kmeans(b, st);
    {
        unsigned long long *cnt = reinterpret_cast<unsigned long long *>(b->d_tilecnt);
        HIP_TRY(hipMemsetAsync(cnt, 0, sizeof(unsigned long long) * 2 * b->nb, st));
        int tz; dim3 grid; size_t lds;
        tile_geometry(b, o.morph3d != 0, tz, grid, lds);
        PsGeom g; dim3 pgrid; size_t plds;
        if (plane_geometry(b, o.morph3d ? PS_CL3 : PS_CL2, g, pgrid, plds)) {
            ScopedKTimer tm(b, "classify", 8.0 * (double)b->V);
            if (o.morph3d)
                launch_plane<PS_CL3>(b, g, pgrid, plds, d_n4, nullptr, o.thresh, b->d_border, cnt);
            else
                launch_plane<PS_CL2>(b, g, pgrid, plds, d_n4, nullptr, o.thresh, b->d_border, cnt);
            VH_CHECK_LAUNCH();
        } else {
            ScopedKTimer tm(b, "classify", 8.0 * (double)b->V);
            if (o.morph3d)
                k_tile<true, true><<<grid, VH_TPB, lds, st>>>(d_n4, b->d_mask, nullptr, b->d_sc,
                                                              o.thresh, b->R, b->C, b->Z, b->V, tz,
                                                              b->d_defect, b->d_border, b->d_lb, cnt);
            else
                k_tile<true, false><<<grid, VH_TPB, lds, st>>>(d_n4, b->d_mask, nullptr, b->d_sc,
                                                               o.thresh, b->R, b->C, b->Z, b->V, tz,
                                                               b->d_defect, b->d_border, b->d_lb, cnt);
            VH_CHECK_LAUNCH();
        }
        k_counts_to_scalars<<<(unsigned)((b->nb + 63) / 64), 64, 0, st>>>(cnt, b->nb, b->d_sc);
        VH_CHECK_LAUNCH();
    }
    if (o.do_snr) vh_launch_snr(b);
}
