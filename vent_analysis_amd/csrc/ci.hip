// ci.hip -- cluster-index map on gfx950 (CI.calculate_CI, CI.py:107-145, and the 95th-percentile
// tail of Vent_Analysis.calculate_CI, Vent_Analysis.py:265-271).
//
// One lane per defect voxel.  The lanes of a wave walk the sphere table in LOCKSTEP (row index is
// wave-uniform, so the table's row offset is one broadcast load per row for the whole wave), each
// lane testing one bit of the volume's defect bitmap per row.  At every shell boundary b the lane
// stops at the first b with 2*hits < b (C = hits/b < 0.5, CI.py:97) and records the shell.
// Semantics restated in oracle/ci_oracle.c: the bitmap is indexed by the
// Fortran-order linear index L = (i+dx) + (j+dy) s0 + (k+dz) s0 s1 (px2vec, CI.py:65-68), so
// out-of-range rows/cols alias into neighbouring columns/slices and only 0 <= L < N is required;
// table rows whose linear offset repeats an earlier row never count (np.intersect1d uniques).
#include <algorithm>
#include <climits>

#include "vh_internal.h"

#define CI_SENTINEL INT32_MIN

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
            atomicOr(&bits[b * words + (L >> 5)], 1u << (L & 31));
            my = atomicAdd(&s_cnt, 1ull);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) s_base = s_cnt ? atomicAdd(&count[b], s_cnt) : 0ull;
    __syncthreads();
    if (d) list[b * V + (int64_t)(s_base + my)] = (int32_t)v;
}

// One WAVE per defect voxel: the wave walks 64 consecutive table rows per step (lane l probes row
// r0 + l), the step's hits are one ballot, and the shell boundaries that fall in the step are tested
// in parallel (lane i takes the i-th boundary in the step: cumulative hits up to row b - 1 are the
// hits before the step plus a popcount of the ballot's low bits; the first boundary with
// 2 hits < b stops the walk).  Every probe of the lockstep lane-per-voxel form is made (same rows,
// same order of boundaries), but a 128x128x24 study's ~6k defect voxels now fill ~6k waves instead
// of ~93.  The defect bitmap sits in LDS when it fits (48 KiB at 128x128x24).
#define CIW_TPB 1024
#define CIW_LDS_WORDS (40 * 1024)   // bitmaps up to 160 KiB in LDS (V <= 1.3 M voxels)
__global__ void __launch_bounds__(CIW_TPB) k_ci_walk(const uint32_t *__restrict__ bits,
                                                    const int32_t *__restrict__ list,
                                                    const unsigned long long *count,
                                                    const int32_t *__restrict__ offL, int64_t rows,
                                                    const int32_t *__restrict__ bounds, int64_t nbs,
                                                    int64_t s0, int64_t s1, int64_t s2, int64_t V,
                                                    int64_t words, int use_lds, int32_t *shell_of,
                                                    uint32_t *hist, int32_t *status) {
    extern __shared__ uint32_t s_bits[];
    const int64_t b = blockIdx.y;
    const int64_t n = (int64_t)count[b];
    constexpr int W = CIW_TPB / 64;
    if ((int64_t)blockIdx.x * W >= n) return;   // block-uniform exit
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t *bm = bits + b * words;
    if (use_lds) {
        for (int64_t i = threadIdx.x; i < words; i += CIW_TPB) s_bits[i] = bm[i];
        __syncthreads();
        bm = s_bits;
    }
    const int64_t N = s0 * s1 * s2;
    for (int64_t idx = (int64_t)blockIdx.x * W + w; idx < n; idx += (int64_t)gridDim.x * W) {
        const int32_t v = list[b * V + idx];
        const int64_t i = v / (s1 * s2), j = (v / s2) % s1, k = v % s2;
        const int64_t base = i + j * s0 + k * s0 * s1;   // px2vec (Fortran order, CI.py:65-68)
        int64_t hits = 0, q = 0, row = 0;
        int32_t qstop = -1;
        while (q < nbs && row < rows) {
            const int64_t r = row + lane;
            bool hit = false;
            if (r < rows) {
                const int32_t off = offL[r];
                const int64_t L = base + off;
                hit = off != CI_SENTINEL && L >= 0 && L < N && ((bm[L >> 5] >> (L & 31)) & 1u);
            }
            const uint64_t bal = __ballot(hit);
            const int64_t bq = q + lane < nbs ? (int64_t)bounds[q + lane] : INT64_MAX;
            const bool inc = bq <= row + 64;   // boundaries in (row, row + 64]: a prefix of the lanes
            bool stop = false;
            if (inc) {
                const int pos = (int)(bq - 1 - row);   // 0 .. 63
                const uint64_t m = pos == 63 ? ~0ull : ((2ull << pos) - 1ull);
                stop = 2 * (hits + __popcll(bal & m)) < bq;
            }
            const uint64_t sb = __ballot(stop);
            if (sb) {
                qstop = (int32_t)(q + __builtin_ctzll(sb));
                break;
            }
            q += __popcll(__ballot(inc));
            hits += __popcll(bal);
            row += 64;
        }
        if (lane == 0) {
            shell_of[b * V + v] = qstop;
            if (qstop >= 0) atomicAdd(&hist[b * nbs + qstop], 1u);
            else atomicExch(&status[b], 1);
        }
    }
}

__global__ void k_ci_finish(const uint32_t *hist, const unsigned long long *count,
                            const double *radii, int64_t nbs, double minvox, int64_t nb,
                            const int32_t *status, VolScalars *sc) {
    const int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (b >= nb) return;
    const int64_t D = (int64_t)count[b];
    sc[b].n_ci = D;
    sc[b].ci_status = status[b] ? VH_ERR_MAXRADIUS : (D == 0 ? VH_ERR_EMPTY : VH_OK);
    sc[b].ci_scalar = 0.0;
    if (status[b] || D == 0) return;
    const int64_t i95 = (int64_t)(0.95 * (double)D);
    int64_t cum = 0;
    for (int64_t q = 0; q < nbs; ++q) {
        cum += hist[b * nbs + q];
        if (cum > i95) { sc[b].ci_scalar = radii[q] * minvox; return; }
    }
}

__global__ void k_ci_scatter(const int32_t *shell_of, const uint8_t *defect, const double *radii,
                             double minvox, int64_t V, double *ci) {
    const int64_t b = blockIdx.y;
    const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (v >= V) return;
    double r = 0.0;
    if (defect[b * V + v]) {
        const int32_t q = shell_of[b * V + v];
        r = q >= 0 ? radii[q] * minvox : 0.0;
    }
    ci[b * V + v] = r;
}

// host: offs/dup/bounds/radii are host arrays; results stay on device (d_ci_shell, d_sc) and the
// float64 CI map goes to ci_dev (caller-provided device buffer, nb*V doubles).
void vh_ci_run(vh_batch *b, const int16_t *offs, const uint8_t *dup, int64_t rows,
               const int32_t *bounds, const double *radii, int64_t nbs, double minvox,
               double *d_ci) {
    hipStream_t st = b->stream;
    const int64_t words = (b->V + 31) / 32;
    // px2vec strides (CI.py:65-68): s0 = R (rows), s1 = C (cols): L = i + j R + k R C
    std::vector<int32_t> offL(rows);
    for (int64_t r = 0; r < rows; ++r)
        offL[r] = dup[r] ? CI_SENTINEL
                         : (int32_t)(offs[3 * r] + (int64_t)offs[3 * r + 1] * b->R +
                                     (int64_t)offs[3 * r + 2] * b->R * b->C);
    // workspace owned by the batch (freed with it): no allocation, and nothing to leak, per call
    if (rows > b->ci_rows_cap) {
        if (b->d_ci_offL) HIP_TRY(hipFree(b->d_ci_offL));
        b->d_ci_offL = nullptr;
        HIP_TRY(hipMalloc(&b->d_ci_offL, sizeof(int32_t) * rows));
        b->ci_rows_cap = rows;
    }
    if (!b->d_ci_status) {
        HIP_TRY(hipMalloc(&b->d_ci_status, sizeof(int32_t) * b->nb));
        HIP_TRY(hipMalloc(&b->d_ci_count, sizeof(unsigned long long) * b->nb));
    }
    int32_t *d_offL = b->d_ci_offL, *d_status = b->d_ci_status;
    unsigned long long *d_count = b->d_ci_count;
    if (!b->d_bitmap) {
        HIP_TRY(hipMalloc(&b->d_bitmap, sizeof(uint32_t) * b->nb * words));
        HIP_TRY(hipMalloc(&b->d_ci_list, sizeof(int32_t) * b->nb * b->V));
        HIP_TRY(hipMalloc(&b->d_ci_shell, sizeof(int32_t) * b->nb * b->V));
    }
    if (nbs > b->ci_nb_cap) {
        if (b->d_ci_hist) HIP_TRY(hipFree(b->d_ci_hist));
        if (b->d_ci_bounds) HIP_TRY(hipFree(b->d_ci_bounds));
        if (b->d_ci_radii) HIP_TRY(hipFree(b->d_ci_radii));
        b->d_ci_hist = nullptr;
        b->d_ci_bounds = nullptr;
        b->d_ci_radii = nullptr;
        b->ci_nb_cap = 0;
        HIP_TRY(hipMalloc(&b->d_ci_hist, sizeof(uint32_t) * b->nb * nbs));
        HIP_TRY(hipMalloc(&b->d_ci_bounds, sizeof(int32_t) * nbs));
        HIP_TRY(hipMalloc(&b->d_ci_radii, sizeof(double) * nbs));
        b->ci_nb_cap = nbs;
    }
    int32_t *d_bounds = b->d_ci_bounds;
    double *d_radii = b->d_ci_radii;
    HIP_TRY(hipMemcpyAsync(d_offL, offL.data(), sizeof(int32_t) * rows, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(d_bounds, bounds, sizeof(int32_t) * nbs, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(d_radii, radii, sizeof(double) * nbs, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemsetAsync(d_status, 0, sizeof(int32_t) * b->nb, st));
    HIP_TRY(hipMemsetAsync(d_count, 0, sizeof(unsigned long long) * b->nb, st));
    HIP_TRY(hipMemsetAsync(b->d_bitmap, 0, sizeof(uint32_t) * b->nb * words, st));
    HIP_TRY(hipMemsetAsync(b->d_ci_hist, 0, sizeof(uint32_t) * b->nb * nbs, st));
    const dim3 vg((unsigned)((b->V + VH_TPB - 1) / VH_TPB), (unsigned)b->nb);
    k_ci_bitmap<<<vg, VH_TPB, 0, st>>>(b->d_defect, b->R, b->C, b->Z, b->V, words, b->d_bitmap,
                                       b->d_ci_list, d_count);
    VH_CHECK_LAUNCH();
    {
        ScopedKTimer tm(b, "ci_walk", 0.0);
        // one wave per defect voxel: up to V waves per volume, 16 per block, grid-strided beyond
        // 16384 blocks per volume; the block reads the volume's defect count itself
        const int64_t wg = std::min<int64_t>((b->V + CIW_TPB / 64 - 1) / (CIW_TPB / 64), 16384);
        const int use_lds = words <= CIW_LDS_WORDS ? 1 : 0;
        vh_set_max_lds((const void *)k_ci_walk, 160 * 1024);
        k_ci_walk<<<dim3((unsigned)wg, (unsigned)b->nb), CIW_TPB,
                    use_lds ? sizeof(uint32_t) * (size_t)words : 0, st>>>(
            b->d_bitmap, b->d_ci_list, d_count, d_offL, rows, d_bounds, nbs, b->R, b->C, b->Z, b->V,
            words, use_lds, b->d_ci_shell, b->d_ci_hist, d_status);
        VH_CHECK_LAUNCH();
    }
    k_ci_finish<<<(unsigned)((b->nb + 63) / 64), 64, 0, st>>>(b->d_ci_hist, d_count, d_radii, nbs,
                                                              minvox, b->nb, d_status, b->d_sc);
    VH_CHECK_LAUNCH();
    if (d_ci) {
        k_ci_scatter<<<vg, VH_TPB, 0, st>>>(b->d_ci_shell, b->d_defect, d_radii, minvox, b->V, d_ci);
        VH_CHECK_LAUNCH();
    }
    HIP_TRY(hipStreamSynchronize(st));
}
