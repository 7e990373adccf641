// Internal declarations shared by the libventhip translation units (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <atomic>
#include <map>
#include <set>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/vent_hip.h"

#define VH_TPB 256          // threads per block for streaming kernels (4 waves of 64)
#define VH_WAVE 64
#define VH_SORT_TILE 4096   // keys per radix-sort tile (256 threads x 16 keys)
#define VH_SORT_KPT 16
#define VH_MAX_LEVELS 8
#define VH_FFT_P 512
#define VH_MAX_BINS 256

struct VhError {
    int code;
    std::string msg;
};

#define HIP_TRY(expr)                                                                       \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess)                                                               \
            throw VhError{_e == hipErrorOutOfMemory ? VH_ERR_NOMEM : VH_ERR_HIP,            \
                          std::string(#expr) + ": " + hipGetErrorString(_e)};               \
    } while (0)

// VH_SYNC_CHECK=1 (diagnostics): every launch is followed by a device sync, so a kernel fault is
// reported at the launch that caused it (file:line) instead of at a later API call
inline bool vh_sync_check() {
    static const bool on = getenv("VH_SYNC_CHECK") != nullptr;
    return on;
}
#define VH_CHECK_LAUNCH()                                                                   \
    do {                                                                                    \
        HIP_TRY(hipGetLastError());                                                         \
        if (vh_sync_check()) {                                                              \
            const hipError_t _s = hipDeviceSynchronize();                                   \
            if (_s != hipSuccess)                                                           \
                throw VhError{VH_ERR_HIP, std::string("after the launch at ") + __FILE__ + \
                                              ":" + std::to_string(__LINE__) + ": " +       \
                                              hipGetErrorString(_s)};                       \
        }                                                                                   \
    } while (0)

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device): the attribute is
// per device, and batches of several contexts / pipeline slots launch from several host threads.
inline void vh_set_max_lds(const void *fn, int bytes) {
    static std::mutex m;
    static std::set<std::pair<const void *, int>> done;
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    std::lock_guard<std::mutex> g(m);
    if (done.count({fn, dev})) return;
    HIP_TRY(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
    done.insert({fn, dev});
}

// Per-volume device scalars (one record per study).
struct VolScalars {
    int64_t n_mask;          // mask != 0
    int64_t n_mask1;         // mask == 1 (N4 label, LungVolume)
    int64_t first_masked;    // raster index of the first mask==1 voxel (N4 bin-range quirk)
    int64_t n_defect;
    int64_t n_lb12;
    int64_t n_km0;
    float mean_anchor;
    float p99;
    double snr;
    int32_t km_iters;
    int32_t pad0;
    double km_c[4];
    int32_t cmin, cmax;      // SNR column box [cmin, cmax)
    int32_t any_row_empty, any_slice_empty;
    int32_t snr_ok;          // 0 when the reference would raise (no masked column > 0)
    int32_t ci_status;       // VH_OK / VH_ERR_MAXRADIUS
    int32_t row_lo, row_hi;  // first / last row holding any masked voxel
    int64_t n_ci;            // defect voxels for CI
    double ci_scalar;
};

// Per-volume N4 iteration state.
struct N4State {
    float bin_min, bin_max, slope;
    int32_t active;          // 1 while the current level is still iterating
    int32_t iters;           // iterations executed in the current level
    int32_t tlast;           // T buffer (0/1) holding the column tables of the last evaluated field
    uint32_t umax_key, umin_key;  // sortable keys: max over all masked, min over all but first
    float u_first;
    float conv_w;            // S7: ITK's float Welford convergence of the last eval (k_n4_welford)
    double conv;
    int32_t iters_level[VH_MAX_LEVELS];
    float conv_level[VH_MAX_LEVELS];
    uint64_t t_start, t_end;   // k_n4_study: device wall clock (wall_clock64) at the workgroup's start / end
    uint32_t hw_id, xcc_id;    // k_n4_study: where the workgroup ran (HW_REG_HW_ID / HW_REG_XCC_ID)
    int32_t pc_rounds, pc_fallbacks;   // k_n4_study: S7 guess-and-verify rounds / serial fallbacks, all iterations
    int32_t pc_pre;            // k_n4_pcw: the last call decided early (PC_PRE): try again on the next one
    // 1 when conv_w of the last S7 call is a certified bound (an early / stage-0 decision: mu's upper
    // and sig's lower bound, enough for the threshold test only), 0 when it is ITK's float measure.
    // A level's last call is never decided early, so conv_level[] is always the exact measure.
    int32_t conv_bound;
};

// Per-axis, per-level B-spline tables (host-built, identical to oracle/n4_oracle.c).
struct AxisTab {
    int32_t n, ncp;
    std::vector<int32_t> base;
    std::vector<float> w;      // [n][4]
    std::vector<double> sw2;   // [n]
};

struct KTimer {
    std::vector<hipEvent_t> ev;   // pairs (start, stop)
    std::vector<int> slots;       // stamped launches: slots of vh_batch::d_kst
    double bytes_per_launch = 0;
    double total_ms = 0;
    int64_t launches = 0;
};

struct vh_ctx {
    int device = 0;
    std::string last_error;
    void *comm = nullptr;           // ncclComm_t
    int nranks = 1, rank = 0;
    // page-locked, device-mapped CI scalars (k_ci_finish stores them there: no readback copy)
    VolScalars *h_ci_sc = nullptr;
    int64_t h_ci_sc_cap = 0;
    // the host-buffer entry points (vh_n4, vh_vdp, ...) share one cached scratch batch per
    // context; mu serialises them, so a context may be used from several host threads
    vh_batch *scratch = nullptr;
    int profile = 0;                // vh_ctx_profile: time the scratch batch's kernel classes
    std::mutex mu;
    // last_error is written by any failing entry point (several host threads may fail at once on
    // one context, and vh_pipe_run does not hold mu): its own lock, and vh_last_error hands out a
    // per-thread copy
    mutable std::mutex err_mu;
    // vh_recon: its own stream and a cached device buffer (input, line transforms, output, twiddles)
    hipStream_t aux = nullptr;
    // RCCL: every collective of the communicator on this one stream, in program order (batches in
    // flight would otherwise issue them on their own streams, which the GPU may run in a different
    // order than another rank does: a deadlock)
    hipStream_t comm_st = nullptr;
    void *recon_buf = nullptr;
    size_t recon_cap = 0;
};

struct vh_pipe {
    struct Slot {
        vh_batch *b = nullptr;
        float *hp = nullptr, *n4 = nullptr;   // pinned staging [sub][V]
        uint8_t *u8 = nullptr;                // pinned: mask in [sub][V], then the D2H block (scal + [sub][V])
        hipEvent_t done = nullptr;            // recorded after the slot's current chunk's pipeline
        hipEvent_t h2d = nullptr;             // recorded after the slot's current chunk's H2D
        hipEvent_t packed = nullptr;          // recorded after the chunk's output packing (its D2H may start)
        uint8_t *d_pack = nullptr;            // device: the chunk's D2H block: scalars (scal bytes), packed maps
        size_t scal = 0;                      // bytes of the per-study scalars + N4 states block (4 KiB multiple)
        uint8_t *mb = nullptr;                // pinned: mask bits, two chunks' worth (double buffer)
        size_t mb_half = 0;
        VolScalars *sc = nullptr;             // the chunk's per-study scalars / N4 states: views into u8
        N4State *st = nullptr;
        std::vector<vh_vdp_result> res;
    };
    vh_ctx *ctx = nullptr;
    int64_t R = 0, C = 0, Z = 0, sub = 0;
    std::vector<Slot> slot;
    // caller pages pinned in place during a run (released at its end), capped at pin_cap bytes
    // (VH_PIPE_PIN_CAP, default 32 GiB): past the cap a range goes through the pinned staging
    int64_t pin_cap = 0;
    std::atomic<int64_t> pinned{0}, pinned_peak{0}, staged_spans{0};
};

struct vh_batch {
    vh_ctx *ctx = nullptr;
    hipStream_t stream = nullptr;    // every launch and copy of this batch (batches overlap)
    hipStream_t st_n4 = nullptr;     // VH_PRIO: the study kernel alone on a low-priority stream (the
    hipEvent_t ev_n4_pre = nullptr, ev_n4_post = nullptr;   // rest on a high-priority one), joined by events
    hipEvent_t ev_cpre = nullptr, ev_cpost = nullptr;      // the cohort all-reduce on vh_ctx::comm_st
    int32_t *h_flags = nullptr;      // pinned: the sweep driver's per-iteration active counts
    int64_t R = 0, C = 0, Z = 0, V = 0, nb = 0, CZ = 0;
    int64_t max_tiles = 0;
    // inputs / outputs
    float *d_hp = nullptr;
    uint8_t *d_mask = nullptr;
    float *d_n4 = nullptr;
    uint8_t *d_defect = nullptr, *d_border = nullptr, *d_lb = nullptr;
    // mask statistics
    int32_t *d_colrange = nullptr;   // [nb][CZ][2]  first/last masked row of each (col, slice) column
    int32_t *d_colcount = nullptr;   // [nb][CZ]
    uint32_t *d_colbits = nullptr;   // [nb][ceil(R/32)][CZ]  row bitmap of mask == 1 per column
    uint32_t *d_colbnz = nullptr;    // [nb][ceil(R/32)][CZ]  row bitmap of mask != 0 per column
    int64_t *d_colstart = nullptr;   // [nb][CZ]     exclusive prefix of colcount
    uint8_t *d_rowany = nullptr, *d_colany = nullptr, *d_sliceany = nullptr;
    VolScalars *d_sc = nullptr;
    double *d_part = nullptr;        // [nb][part_blocks][4] deterministic partial sums
    int64_t part_blocks = 0;
    double *d_snrpart = nullptr;     // [nb][slab_blocks][4] SNR partial sums (k_snr / k_n4_final)
    int64_t slab_blocks = 0;         // column blocks x 32-row slabs per volume
    bool snr_fused = false;          // k_n4_final computed the SNR partials of this run
    // sort
    uint32_t *d_keys0 = nullptr, *d_keys1 = nullptr;
    uint32_t *d_tilecnt = nullptr;   // [nb][256][max_tiles]
    // cohort
    uint64_t *d_cohort = nullptr;
    // N4 workspace
    float *d_L0 = nullptr, *d_lat = nullptr, *d_E = nullptr;
    unsigned long long *d_numfix = nullptr;   // [nb][lattice][2] 128-bit fixed-point fit sums (S5)
    int32_t *d_rowstart = nullptr;   // [nb][tiles][R] compact offset of each (64-column tile, row)
    uint64_t *d_rowmask = nullptr;   // [nb][tiles][R] mask == 1 lanes of each (tile, row)
    int32_t *d_rrank = nullptr;      // [nb][tiles][R] raster rank of the first masked voxel of (tile, row)
    int32_t *d_iscan = nullptr;      // large volumes: chunk sums of the row-start / raster-rank scans
    int64_t iscan_cap = 0;
    float *d_D = nullptr;            // [nb][VS] B_old - B_new (S7 input): compact order (n4), raster order (n4_study)
    int32_t *d_perm = nullptr;       // [nb][VS] raster rank -> compact index of the mask == 1 voxels (n4)
    // compact N4 state: mask==1 voxels in tile-row order, volume stride VS
    int64_t VS = 0;
    int rsh = 1;                     // compact voxel index = (row << rsh) | column
    bool keys_fused = false;         // k_n4_final wrote the sort keys of binary-mask volumes
    float *d_U = nullptr;            // [nb][VS] U = L0 - B
    int32_t *d_ridx = nullptr;       // [nb][VS] raster index of each compact voxel
    int32_t *d_cp = nullptr;         // [nb + 1] chunk prefix (N4_CH voxels per chunk)
    int32_t *d_cvol = nullptr;       // [chunks] owning volume
    uint64_t *d_hpart = nullptr;     // [chunks][VH_MAX_BINS] per-chunk histograms
    uint64_t *d_hred = nullptr;      // [studies][N4_HSL][2][VH_MAX_BINS] slice sums (k_n4_hred)
    size_t hred_cap = 0;
    double *d_cpart = nullptr;       // [chunks][2] per-chunk convergence sums
    int64_t n4_tiles = 0;
    std::vector<size_t> lvx_off;     // per level: xst / wk3 / wk2 offsets in d_tabs
    double *d_P1 = nullptr, *d_den = nullptr;
    float *d_pcdrift = nullptr;      // [nb][1024] the study kernel's PC guess offsets (PC_DRIFT)
    float *d_T = nullptr;            // [2][nb][CZ][ncx] per-column lattice contraction (new / previous field)
    int64_t t_cap = 0;
    N4State *d_st = nullptr;
    int32_t *d_nactive = nullptr;
    void *d_tabs = nullptr;          // device copy of all per-level axis tables
    int64_t lat_cap = 0, q2_cap = 0;
    std::vector<size_t> tab_off;     // offsets of each (level, axis) table in d_tabs
    vh_n4_params tab_prm{};          // parameters the tables were built for
    bool tabs_valid = false;
    double2 *d_twiddle = nullptr;    // FFT twiddles (host-computed)
    void *d_study_lv = nullptr;      // n4_study.hip: per-level table pointers + iteration caps
    int32_t *d_study_order = nullptr;   // n4_study.hip: workgroup -> study, largest study first
    void *d_pcg = nullptr;           // n4.hip k_n4_pcg: per-block guesses / ends / sums, aggregates
    void *d_study_latg = nullptr;    // n4_study.hip depth 2: the lattice before the last two updates
    size_t study_latg_cap = 0;
    int64_t pcg_cap = 0;             // bytes of d_pcg
    void *d_stg = nullptr;           // n4_study.hip grid form: global sums, records, grid-PC scratch
    int64_t stg_cap = 0;             // bytes of d_stg
    void *d_sortg = nullptr;         // vdp.hip grid sort: per-chunk digit counts / offsets
    int64_t sortg_cap = 0;           // entries of d_sortg
    // CI workspace
    uint32_t *d_bitmap = nullptr;    // [nb][ceil(V/32)] Fortran-order defect bits
    int32_t *d_ci_list = nullptr;    // [nb][V] defect voxel raster indices (compacted)
    int32_t *d_ci_shell = nullptr;   // [nb][V]
    uint32_t *d_ci_hist = nullptr;   // [nb][ci_nb]
    int64_t ci_nb_cap = 0;
    int32_t *d_ci_status = nullptr;  // [nb]
    unsigned long long *d_ci_count = nullptr;   // [nb]
    double *d_ci_map = nullptr;      // [nb][V] float64 CI map (vh_ci)
    int64_t n4_subbatch = 0;         // volumes per N4 sub-batch (0 = whole batch)
    int32_t n4_mode = 0;             // vh_run_opts.n4_mode
    bool n4_used_study = false;      // the last N4 ran the volume-resident kernel
    // timing
    bool profile = false;
    std::map<std::string, KTimer> timers;
    // stamped timers (cooperative launches): [VH_KST_CAP] first-workgroup starts, then
    // [VH_KST_CAP] last-workgroup ends, device wall clock; kst_n slots handed out since the reset
    unsigned long long *d_kst = nullptr;
    int kst_n = 0;
    // last run options
    vh_run_opts opts{};
    bool have_result = false;
};

// a compact sphere table resident in HBM (vh_ci_table_create): linear offsets for one (R, C)
struct vh_ci_table {
    vh_ctx *ctx = nullptr;
    int64_t R = 0, C = 0, rows = 0, nbs = 0;
    int32_t *d_offL = nullptr;       // [rows] px2vec offsets, CI_SENTINEL for duplicate rows
    int32_t *d_bounds = nullptr;     // [nbs] shell prefix lengths
    double *d_radii = nullptr;       // [nbs] r[b - 1]
};

// ---- timing helper ----------------------------------------------------------------------------
// stamped (profiling a cooperative launch): no events; the kernel stamps its own span through
// stamp() (kst_begin / kst_end), because HIP events around hipLaunchCooperativeKernel also time the
// runtime's cooperative handshake (config 5 k_n4_pcg2: 677 us per launch by events against 542 us in
// rocprofv3's trace, whose gaps round the launch are ~13 us each, r6q)
struct ScopedKTimer {
    vh_batch *b;
    KTimer *t;
    hipEvent_t e1 = nullptr;
    unsigned long long *ks = nullptr;
    hipStream_t s = nullptr;   // the stream the timed launches go to (the batch's by default)
    ScopedKTimer(vh_batch *bb, const char *name, double bytes, bool stamped = false,
                 hipStream_t on = nullptr);
    ~ScopedKTimer();
    unsigned long long *stamp() const { return ks; }   // null unless stamped and profiling
};
#define VH_KST_CAP 4096
// a stamped launch's span: thread 0 of every workgroup at its start / end (vector atomics)
__device__ __forceinline__ void kst_begin(unsigned long long *s) {
    if (s && threadIdx.x == 0) atomicMin(s, (unsigned long long)wall_clock64());
}
__device__ __forceinline__ void kst_end(unsigned long long *s) {
    __syncthreads();
    if (s && threadIdx.x == 0) atomicMax(s + VH_KST_CAP, (unsigned long long)wall_clock64());
}

// ---- launchers (defined in vdp.hip / n4.hip / ci.hip) ---------------------------------------
void vh_launch_mask_stats(vh_batch *b);
void vh_launch_vdp_chain(vh_batch *b, const float *d_n4, const vh_run_opts &o);
void vh_launch_snr(vh_batch *b);
void vh_launch_border(vh_batch *b, const uint8_t *d_in, uint8_t *d_out);
void vh_launch_n4(vh_batch *b, const vh_n4_params &prm);
void vh_n4_prepare_tables(vh_batch *b, const vh_n4_params &prm);
vh_ci_table *vh_ci_table_build(vh_ctx *ctx, int64_t R, int64_t C, const int16_t *offs, const uint8_t *dup,
                               int64_t rows, const int32_t *bounds, const double *radii, int64_t nbs);
void vh_ci_table_free(vh_ci_table *t);
void vh_ci_run(vh_batch *b, const vh_ci_table *t, double minvox, double *d_ci, VolScalars *h_sc = nullptr);
void vh_ci_debug_check();   // VH_DEBUG_BOUNDS builds: raise the CI kernels' first bounds violation
void vh_ensure_n4_workspace(vh_batch *b, const vh_n4_params &prm);

// ---- shared host helpers ----------------------------------------------------------------------
void vh_axis_tables(int n, int ncp, float eps, AxisTab &t);
float vh_bspline_eps(int max_spans);

inline dim3 col_grid(const vh_batch *b) {
    return dim3((unsigned)((b->CZ + VH_TPB - 1) / VH_TPB), (unsigned)b->nb, 1);
}
// row-slab column sweeps: blockIdx.x = slab * col_blocks + column block, slabs of 32 rows (one
// bitmap word of d_colbits / d_colbnz), so a column's rows are walked by R / 32 threads
#define VH_SLAB 32
inline dim3 slab_grid(const vh_batch *b) { return dim3((unsigned)b->slab_blocks, (unsigned)b->nb, 1); }

// calculate_SNR's noise box (Vent_Analysis.py:340-351) for the slab sweeps
struct SnrBox {
    const uint8_t *rowany, *sliceany;
    double *part;                    // [nb][nparts][4]: signal sum, noise sum, noise sum of squares, noise count
    int64_t nparts;
};

// ---- device helpers ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t f2key(float f) {
    uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
    uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
    return __uint_as_float(u);
}

// SNR over a 32-row slab: wave 0 sets s_rows[0] = rows inside the noise FOV band (rows 20 ..
// R - 21), s_rows[1] = rows of the box (rows holding mask, row 0 when some row is empty) --
// Vent_Analysis.py:344-351, the quirks as in oracle/vdp_oracle.calculate_snr
__device__ inline void snr_slab_rows(const SnrBox &sb, const VolScalars &s, int64_t b, int64_t R,
                                     int64_t x0, int nr, uint32_t *s_rows) {
    if (threadIdx.x < 64) {
        const int64_t x = x0 + threadIdx.x;
        const bool ok = (int)threadIdx.x < nr;
        const bool fov = ok && x >= 20 && x < R - 20;
        const bool rin = ok && (sb.rowany[b * R + x] || (x == 0 && s.any_row_empty));
        const uint64_t a = __ballot(fov), c = __ballot(rin);
        if (threadIdx.x == 0) { s_rows[0] = (uint32_t)a; s_rows[1] = (uint32_t)c; }
    }
}
// the slab rows of column col that are noise: in the FOV band and outside the box
__device__ inline uint32_t snr_col_noise(const SnrBox &sb, const VolScalars &s, int64_t b,
                                         int64_t Z, int64_t col, const uint32_t *s_rows) {
    const int32_t y = (int32_t)((uint32_t)col / (uint32_t)Z), z = (int32_t)col - y * (int32_t)Z;
    const bool cin = y >= s.cmin && y < s.cmax;
    const bool sin_ = sb.sliceany[b * Z + z] || (z == 0 && s.any_slice_empty);
    return s_rows[0] & ~((cin && sin_) ? s_rows[1] : 0u);
}
// one voxel's contributions (double accumulation, as k_snr always did; a deselected voxel adds
// +0.0, which leaves every sum unchanged).  The noise count is added per slab by snr_count.
__device__ __forceinline__ void snr_add(double (&acc)[4], float v, bool sig, bool noise) {
    const double d = (double)v;
    acc[0] += sig ? d : 0.0;
    const double t = noise ? d : 0.0;
    acc[1] += t;
    acc[2] += t * t;
}
__device__ __forceinline__ void snr_count(double (&acc)[4], uint32_t noise) {
    acc[3] += (double)__popc(noise);
}
// block sums of the 4 partials in a fixed order -> dst[0..3]
__device__ inline void snr_block_write(double (&acc)[4], double (*s_red)[VH_TPB / 64], double *dst) {
    for (int q = 0; q < 4; ++q) {
        double x = acc[q];
        for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
        if ((threadIdx.x & 63) == 0) s_red[q][threadIdx.x >> 6] = x;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        double x = 0.0;
        for (int w = 0; w < VH_TPB / 64; ++w) x += s_red[threadIdx.x][w];
        dst[threadIdx.x] = x;
    }
}

// export.hip (rendering after the hot path)
void vh_overlay_launch(hipStream_t s, const float *d_n4, const uint8_t *d_def, int64_t R, int64_t C,
                       int64_t Z, int64_t nb, uint32_t *d_mm, uint8_t *d_rgb);
void vh_recon_run(hipStream_t st, const double2 *d_in, double2 *d_tmp, double2 *d_out, double2 *d_tw0,
                  double2 *d_tw1, int64_t n0, int64_t n1, int64_t nz);
void vh_montage_run(hipStream_t s, int64_t R, int64_t C, int64_t Z, const void *proton, int p64,
                    const void *hp, int h64, const float *n4, const uint8_t *mborder,
                    const uint8_t *def, const double *ci, const double *parula, int64_t prow,
                    const int64_t crop[6], uint8_t *image);
