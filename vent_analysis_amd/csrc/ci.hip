// ci.hip -- cluster-index map on gfx950 (CI.calculate_CI, CI.py:107-145, and the 95th-percentile
// tail of Vent_Analysis.calculate_CI, Vent_Analysis.py:265-271).
//
// One wave per defect voxel (k_ci_walk): the wave's lanes test consecutive rows of the sphere table
// against the volume's defect bitmap and stop at the first shell boundary b with 2*hits < b
// (C = hits/b < 0.5, CI.py:97), recording the shell.
// Semantics restated in oracle/ci_oracle.c: the bitmap is indexed by the
// Fortran-order linear index L = (i+dx) + (j+dy) s0 + (k+dz) s0 s1 (px2vec, CI.py:65-68), so
// out-of-range rows/cols alias into neighbouring columns/slices and only 0 <= L < N is required;
// table rows whose linear offset repeats an earlier row never count (np.intersect1d uniques).
#include <algorithm>
#include <climits>

#include "vh_internal.h"

#define CI_SENTINEL INT32_MIN

// VH_DEBUG_BOUNDS builds (make DEBUG_BOUNDS=1 -> libventhip_dbg.so): every index the CI kernels
// derive from data (defect list slots, table rows, shells, bitmap words) is checked against its
// buffer's extent before the access; a violation skips the access and records (site, index, extent)
// in g_ci_dbg, which ci_debug_check() reads after the call's stream sync and raises as VH_ERR_HIP.
// Release builds compile the checks away (CI_OK(c, ...) == c is never evaluated as a guard).
#ifdef VH_DEBUG_BOUNDS
static __device__ unsigned long long g_ci_dbg[4];
__device__ __forceinline__ bool ci_ok(bool c, int site, int64_t idx, int64_t ext) {
    if (!c && atomicCAS(&g_ci_dbg[0], 0ull, (unsigned long long)site) == 0ull) {
        atomicExch(&g_ci_dbg[1], (unsigned long long)idx);
        atomicExch(&g_ci_dbg[2], (unsigned long long)ext);
    }
    return c;
}
#define CI_OK(c, site, idx, ext) ci_ok((c), (site), (int64_t)(idx), (int64_t)(ext))
#else
#define CI_OK(c, site, idx, ext) true
#endif

__global__ void k_ci_bitmap(const uint8_t *__restrict__ defect, int64_t s0, int64_t s1,
                            int64_t s2, int64_t V, int64_t words, uint32_t *bits,
                            int32_t *list, unsigned long long *count) {
    const int64_t b = blockIdx.y;
    __shared__ unsigned long long s_cnt, s_base;
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    bool d = false;
    unsigned long long my = 0;
    if (v < V) {
        d = defect[b * V + v] != 0;
        if (d) {
            const int64_t i = v / (s1 * s2), j = (v / s2) % s1, k = v % s2;
            const int64_t L = i + j * s0 + k * s0 * s1;
            if (CI_OK((L >> 5) < words, 1, L, words))
                atomicOr(&bits[b * words + (L >> 5)], 1u << (L & 31));
            my = atomicAdd(&s_cnt, 1ull);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) s_base = s_cnt ? atomicAdd(&count[b], s_cnt) : 0ull;
    __syncthreads();
    if (d && CI_OK((int64_t)(s_base + my) < V, 2, s_base + my, V)) list[b * V + (int64_t)(s_base + my)] = (int32_t)v;
}

// One WAVE per defect voxel: the wave probes CIW_U x 64 consecutive table rows per step (lane l
// tests rows r0 + 64 u + l, u < CIW_U: the CIW_U loads are independent, so one step pays one memory
// latency for 256 rows), the step's hits are CIW_U ballots, and the shell boundaries that fall in
// the step are tested in parallel, 64 at a time (lane i takes the i-th boundary: cumulative hits up
// to row b - 1 are the hits before the step plus popcounts of the ballots below b's); the first
// boundary with 2 hits < b stops the walk.  Every probe of the lane-per-voxel form is made (same rows,
// same order of boundaries; rows past the stop in the last step are probed and ignored).  LDS holds
// the Fortran-order defect bitmap (48 KiB at 128x128x24) and the first CIW_ROWS rows of linear
// offsets and CIW_NBS boundaries (every walk shorter than r ~ 23 at [1.5, 1.5, 10] stays in LDS);
// later rows come from L2.  A block takes voxels blockIdx.x, blockIdx.x + gridDim.x, ... (16 waves
// each) and exits before staging anything when the volume has fewer defect voxels than its first.
#define CIW_TPB 1024
#define CIW_U 4
#define CIW_ROWS 8192
#define CIW_NBS 1024
#define CIW_LDS_MAX (160 * 1024)
__global__ void __launch_bounds__(CIW_TPB) k_ci_walk(const uint32_t *__restrict__ bits,
                                                    const int32_t *__restrict__ list,
                                                    const unsigned long long *count,
                                                    const int32_t *__restrict__ offL, int64_t rows,
                                                    const int32_t *__restrict__ bounds, int64_t nbs,
                                                    int64_t s0, int64_t s1, int64_t s2, int64_t V,
                                                    int64_t words, int stage_bits, int32_t *shell_of,
                                                    uint32_t *hist, int32_t *status) {
    extern __shared__ uint32_t s_lds[];
    const int64_t b = blockIdx.y;
    const int64_t n = (int64_t)count[b];
    constexpr int W = CIW_TPB / 64;
    if (!CI_OK(n <= V, 3, n, V)) return;
    if ((int64_t)blockIdx.x * W >= n) return;   // block-uniform exit, before any staging
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // LDS: offsets [CIW_ROWS], boundaries [CIW_NBS], then the bitmap (stage_bits)
    int32_t *s_off = reinterpret_cast<int32_t *>(s_lds), *s_bnd = s_off + CIW_ROWS;
    const int lrows = (int)(rows < CIW_ROWS ? rows : CIW_ROWS), lnbs = (int)(nbs < CIW_NBS ? nbs : CIW_NBS);
    for (int i = threadIdx.x; i < lrows; i += CIW_TPB) s_off[i] = offL[i];
    for (int i = threadIdx.x; i < lnbs; i += CIW_TPB) s_bnd[i] = bounds[i];
    const uint32_t *bm = bits + b * words;
    if (stage_bits) {
        uint32_t *s_bits = reinterpret_cast<uint32_t *>(s_bnd + CIW_NBS);
        for (int64_t i = threadIdx.x; i < words; i += CIW_TPB) s_bits[i] = bm[i];
        bm = s_bits;
    }
    __syncthreads();
    auto off_at = [&](int64_t r) {
        if (!CI_OK(r >= 0 && r < rows, 4, r, rows)) return (int32_t)CI_SENTINEL;
        return r < lrows ? s_off[r] : offL[r];
    };
    auto bnd_at = [&](int64_t q) {
        if (!CI_OK(q >= 0 && q < nbs, 5, q, nbs)) return (int64_t)INT64_MAX;
        return q < lnbs ? (int64_t)s_bnd[q] : (int64_t)bounds[q];
    };
    const int64_t N = s0 * s1 * s2;
    for (int64_t idx = (int64_t)blockIdx.x * W + w; idx < n; idx += (int64_t)gridDim.x * W) {
        const int32_t v = list[b * V + idx];
        if (!CI_OK(v >= 0 && v < V, 6, v, V)) continue;
        const int64_t i = v / (s1 * s2), j = (v / s2) % s1, k = v % s2;
        const int64_t base = i + j * s0 + k * s0 * s1;   // px2vec (Fortran order, CI.py:65-68)
        int64_t hits = 0, q = 0, row = 0;
        int32_t qstop = -1;
        while (q < nbs && row < rows) {
            uint64_t bal[CIW_U];
            int32_t off[CIW_U];
#pragma unroll
            for (int u = 0; u < CIW_U; ++u) {
                const int64_t r = row + 64 * u + lane;
                off[u] = r < rows ? off_at(r) : CI_SENTINEL;
            }
#pragma unroll
            for (int u = 0; u < CIW_U; ++u) {
                const int64_t L = base + off[u];
                const bool hit = off[u] != CI_SENTINEL && L >= 0 && L < N && CI_OK((L >> 5) < words, 7, L, words) &&
                                 ((bm[L >> 5] >> (L & 31)) & 1u);
                bal[u] = __ballot(hit);
            }
            const int64_t rend = row + 64 * CIW_U;
            // boundaries in (row, rend], 64 per pass, in order
            bool stopped = false;
            for (;;) {
                const int64_t bq = q + lane < nbs ? bnd_at(q + lane) : INT64_MAX;
                const bool inc = bq <= rend;
                bool stop = false;
                if (inc) {
                    int pos = (int)(bq - 1 - row);   // 0 .. 64 CIW_U - 1
                    if (!CI_OK(pos >= 0 && pos < 64 * CIW_U, 8, pos, 64 * CIW_U)) pos = 0;
                    const int u = pos >> 6, pb = pos & 63;
                    int64_t c = hits;
#pragma unroll
                    for (int uu = 0; uu < CIW_U; ++uu)
                        c += uu < u ? __popcll(bal[uu]) : uu == u ? __popcll(bal[uu] & (pb == 63 ? ~0ull : ((2ull << pb) - 1ull))) : 0;
                    stop = 2 * c < bq;
                }
                const uint64_t sb = __ballot(stop);
                if (sb) {
                    qstop = (int32_t)(q + __builtin_ctzll(sb));
                    stopped = true;
                    break;
                }
                const int ninc = __popcll(__ballot(inc));
                q += ninc;
                if (ninc < 64 || q >= nbs) break;
            }
            if (stopped) break;
#pragma unroll
            for (int u = 0; u < CIW_U; ++u) hits += __popcll(bal[u]);
            row = rend;
        }
        if (lane == 0) {
            shell_of[b * V + v] = qstop;
            if (qstop >= 0 && CI_OK(qstop < nbs, 9, qstop, nbs)) atomicAdd(&hist[b * nbs + qstop], 1u);
            else atomicExch(&status[b], 1);
        }
    }
}

// the workspace's zeroing in one launch (four hipMemsetAsync blits before: ~4 us each, r4ab)
__global__ void k_ci_clear(int32_t *status, unsigned long long *count, int64_t nb, uint32_t *bits,
                           int64_t nbits, uint32_t *hist, int64_t nhist) {
    const int64_t i0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x, st = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = i0; i < nbits; i += st) bits[i] = 0u;
    for (int64_t i = i0; i < nhist; i += st) hist[i] = 0u;
    for (int64_t i = i0; i < nb; i += st) {
        status[i] = 0;
        count[i] = 0ull;
    }
}

// The 95th-percentile shell (Vent_Analysis.py:265-271): the first shell q whose cumulative count
// passes i95, one workgroup per volume -- each thread sums a run of consecutive shells, an
// exclusive scan of the run sums finds the run holding the crossing, and that run is walked (one
// thread per volume walked every shell serially: 16 us, r4ab).  Integer sums: order-free.
#define CIF_TPB 256
#define CIF_LDS 16384   // shells staged in LDS (64 KiB)
__global__ void __launch_bounds__(CIF_TPB) k_ci_finish(const uint32_t *hist, const unsigned long long *count,
                                                      const double *radii, int64_t nbs, double minvox,
                                                      int64_t nb, const int32_t *status, VolScalars *sc,
                                                      VolScalars *hsc) {
    __shared__ unsigned long long s_sum[CIF_TPB];
    __shared__ int s_hit;
    const int64_t b = blockIdx.x;
    const int t = threadIdx.x;
    const int64_t D = (int64_t)count[b];
    if (t == 0) {
        const int32_t cs = status[b] ? VH_ERR_MAXRADIUS : (D == 0 ? VH_ERR_EMPTY : VH_OK);
        sc[b].n_ci = D;
        sc[b].ci_status = cs;
        sc[b].ci_scalar = 0.0;
        if (hsc) {   // the host's page-locked copy (vector stores over the link)
            hsc[b].n_ci = D;
            hsc[b].ci_status = cs;
            hsc[b].ci_scalar = 0.0;
        }
        s_hit = -1;
    }
    if (status[b] || D == 0) return;   // block-uniform
    const unsigned long long i95 = (unsigned long long)(int64_t)(0.95 * (double)D);
    const int64_t per = (nbs + CIF_TPB - 1) / CIF_TPB, q0 = t * per, q1 = min(q0 + per, nbs);
    // the histogram staged through LDS by coalesced loads first (one thread's run of dependent-
    // address loads took ~16 us, r4al), when it fits
    extern __shared__ uint32_t s_h[];
    const uint32_t *h = hist + b * nbs;
    if (nbs <= CIF_LDS) {
        for (int64_t q = t; q < nbs; q += CIF_TPB) s_h[q] = h[q];
        __syncthreads();
        h = s_h;
    }
    unsigned long long own = 0;
    for (int64_t q = q0; q < q1; ++q) own += h[q];
    s_sum[t] = own;
    __syncthreads();
    if (t == 0) {   // exclusive scan of the run sums (256 adds) and the run holding the crossing
        unsigned long long run = 0;
        for (int i = 0; i < CIF_TPB; ++i) {
            const unsigned long long v = s_sum[i];
            s_sum[i] = run;
            run += v;
            if (s_hit < 0 && run > i95) s_hit = i;
        }
    }
    __syncthreads();
    if (t == s_hit) {
        unsigned long long cum = s_sum[t];
        for (int64_t q = q0; q < q1; ++q) {
            cum += h[q];
            if (cum > i95) {
                if (!CI_OK(q < nbs, 10, q, nbs)) break;
                sc[b].ci_scalar = radii[q] * minvox;
                if (hsc) hsc[b].ci_scalar = radii[q] * minvox;
                break;
            }
        }
    }
}

__global__ void k_ci_scatter(const int32_t *shell_of, const uint8_t *defect, const double *radii,
                             int64_t nbs, double minvox, int64_t V, double *ci) {
    const int64_t b = blockIdx.y;
    const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (v >= V) return;
    double r = 0.0;
    if (defect[b * V + v]) {
        const int32_t q = shell_of[b * V + v];
        r = q >= 0 && CI_OK(q < nbs, 11, q, nbs) ? radii[q] * minvox : 0.0;
    }
    ci[b * V + v] = r;
}

// host: a compact sphere table uploaded once (vh_ci_table_create): the linear px2vec offsets of
// its rows for one (R, C) -- the stride of L = i + j R + k R C, CI.py:65-68 -- with duplicates
// marked, the shell boundaries and radii, all resident in HBM until vh_ci_table_destroy.
vh_ci_table *vh_ci_table_build(vh_ctx *ctx, int64_t R, int64_t C, const int16_t *offs, const uint8_t *dup,
                               int64_t rows, const int32_t *bounds, const double *radii, int64_t nbs) {
    if (!offs || !dup || !bounds || !radii || rows < 1 || nbs < 1 || R < 1 || C < 1)
        throw VhError{VH_ERR_ARG, "null buffer / empty table"};
    for (int64_t q = 0; q < nbs; ++q)
        if (bounds[q] < 1 || bounds[q] > rows || (q && bounds[q] <= bounds[q - 1]))
            throw VhError{VH_ERR_ARG, "sphere table bounds must be increasing in [1, rows]"};
    std::vector<int32_t> offL(rows);
    for (int64_t r = 0; r < rows; ++r)
        offL[r] = dup[r] ? CI_SENTINEL
                         : (int32_t)(offs[3 * r] + (int64_t)offs[3 * r + 1] * R + (int64_t)offs[3 * r + 2] * R * C);
    HIP_TRY(hipSetDevice(ctx->device));
    vh_ci_table *t = new vh_ci_table;
    t->ctx = ctx;
    t->R = R;
    t->C = C;
    t->rows = rows;
    t->nbs = nbs;
    try {
        HIP_TRY(hipMalloc(&t->d_offL, sizeof(int32_t) * rows));
        HIP_TRY(hipMalloc(&t->d_bounds, sizeof(int32_t) * nbs));
        HIP_TRY(hipMalloc(&t->d_radii, sizeof(double) * nbs));
        HIP_TRY(hipMemcpy(t->d_offL, offL.data(), sizeof(int32_t) * rows, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(t->d_bounds, bounds, sizeof(int32_t) * nbs, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(t->d_radii, radii, sizeof(double) * nbs, hipMemcpyHostToDevice));
    } catch (...) {
        vh_ci_table_free(t);
        throw;
    }
    return t;
}

void vh_ci_table_free(vh_ci_table *t) {
    if (!t) return;
    (void)hipSetDevice(t->ctx->device);
    if (t->d_offL) (void)hipFree(t->d_offL);
    if (t->d_bounds) (void)hipFree(t->d_bounds);
    if (t->d_radii) (void)hipFree(t->d_radii);
    delete t;
}

// results stay on device (d_ci_shell, d_sc); the float64 CI map goes to d_ci (nb*V doubles) when
// given -- device memory, or a device-mapped page-locked host buffer the scatter writes across the
// link -- and the CI scalars also to h_sc (device-mapped host memory) when given.  Enqueued on the
// batch's stream; the caller synchronises.
void vh_ci_run(vh_batch *b, const vh_ci_table *t, double minvox, double *d_ci, VolScalars *h_sc) {
    if (t->R != b->R || t->C != b->C) throw VhError{VH_ERR_ARG, "sphere table built for another (R, C)"};
    hipStream_t st = b->stream;
    const int64_t words = (b->V + 31) / 32, rows = t->rows, nbs = t->nbs;
    // workspace owned by the batch (freed with it): no allocation, and nothing to leak, per call
    if (!b->d_ci_status) {
        HIP_TRY(hipMalloc(&b->d_ci_status, sizeof(int32_t) * b->nb));
        HIP_TRY(hipMalloc(&b->d_ci_count, sizeof(unsigned long long) * b->nb));
    }
    int32_t *d_status = b->d_ci_status;
    unsigned long long *d_count = b->d_ci_count;
    if (!b->d_bitmap) {
        HIP_TRY(hipMalloc(&b->d_bitmap, sizeof(uint32_t) * b->nb * words));
        HIP_TRY(hipMalloc(&b->d_ci_list, sizeof(int32_t) * b->nb * b->V));
        HIP_TRY(hipMalloc(&b->d_ci_shell, sizeof(int32_t) * b->nb * b->V));
    }
    if (nbs > b->ci_nb_cap) {
        if (b->d_ci_hist) HIP_TRY(hipFree(b->d_ci_hist));
        b->d_ci_hist = nullptr;
        b->ci_nb_cap = 0;
        HIP_TRY(hipMalloc(&b->d_ci_hist, sizeof(uint32_t) * b->nb * nbs));
        b->ci_nb_cap = nbs;
    }
    {
        const int64_t big = std::max<int64_t>(b->nb * words, b->nb * nbs);
        k_ci_clear<<<(unsigned)std::min<int64_t>((big + VH_TPB - 1) / VH_TPB, 1024), VH_TPB, 0, st>>>(
            d_status, d_count, b->nb, b->d_bitmap, b->nb * words, b->d_ci_hist, b->nb * nbs);
        VH_CHECK_LAUNCH();
    }
    const dim3 vg((unsigned)((b->V + VH_TPB - 1) / VH_TPB), (unsigned)b->nb);
    k_ci_bitmap<<<vg, VH_TPB, 0, st>>>(b->d_defect, b->R, b->C, b->Z, b->V, words, b->d_bitmap,
                                       b->d_ci_list, d_count);
    VH_CHECK_LAUNCH();
    {
        ScopedKTimer tm(b, "ci_walk", 0.0);
        // one wave per defect voxel, 16 per block; blocks stride over the defect list past 512 per
        // volume (two per CU), and a block past the volume's defect count exits before staging
        const int64_t wg = std::min<int64_t>((b->V + CIW_TPB / 64 - 1) / (CIW_TPB / 64), 512);
        const size_t fixed = sizeof(int32_t) * (CIW_ROWS + CIW_NBS);
        const int stage_bits = fixed + sizeof(uint32_t) * (size_t)words <= CIW_LDS_MAX ? 1 : 0;
        vh_set_max_lds((const void *)k_ci_walk, CIW_LDS_MAX);
        k_ci_walk<<<dim3((unsigned)wg, (unsigned)b->nb), CIW_TPB,
                    fixed + (stage_bits ? sizeof(uint32_t) * (size_t)words : 0), st>>>(
            b->d_bitmap, b->d_ci_list, d_count, t->d_offL, rows, t->d_bounds, nbs, b->R, b->C, b->Z, b->V,
            words, stage_bits, b->d_ci_shell, b->d_ci_hist, d_status);
        VH_CHECK_LAUNCH();
    }
    vh_set_max_lds((const void *)k_ci_finish, (int)(sizeof(uint32_t) * CIF_LDS + 4096));
    k_ci_finish<<<(unsigned)b->nb, CIF_TPB, nbs <= CIF_LDS ? sizeof(uint32_t) * (size_t)nbs : 0, st>>>(
        b->d_ci_hist, d_count, t->d_radii, nbs, minvox, b->nb, d_status, b->d_sc, h_sc);
    VH_CHECK_LAUNCH();
    if (d_ci) {
        k_ci_scatter<<<vg, VH_TPB, 0, st>>>(b->d_ci_shell, b->d_defect, t->d_radii, nbs, minvox, b->V, d_ci);
        VH_CHECK_LAUNCH();
    }
}

// VH_DEBUG_BOUNDS: the first recorded violation of the CI kernels since the last check, raised
// (after the caller's stream sync); a no-op in release builds
void vh_ci_debug_check() {
#ifdef VH_DEBUG_BOUNDS
    unsigned long long h[4] = {0, 0, 0, 0};
    HIP_TRY(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_ci_dbg), sizeof h, 0, hipMemcpyDeviceToHost));
    if (h[0]) {
        const unsigned long long z[4] = {0, 0, 0, 0};
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_ci_dbg), z, sizeof z, 0, hipMemcpyHostToDevice));
        throw VhError{VH_ERR_HIP, "CI bounds check: site " + std::to_string(h[0]) + " index " +
                                      std::to_string((long long)h[1]) + " extent " + std::to_string((long long)h[2])};
    }
#endif
}
