// api.hip -- the extern "C" boundary of libventhip.so (include/vent_hip.h).
// Contexts own a HIP stream on one device; batches own the device buffers of nb studies.
// No exception crosses the ABI: every entry point maps failures to a status code and keeps the
// message for vh_last_error().
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <map>
#include <memory>
#include <cstdio>
#include <cstring>
#include <stdexcept>

#ifndef VH_COPY_THREADS
#define VH_COPY_THREADS 8   // host threads per staging copy (each pipe slot copies on its own)
#endif

#include "vh_internal.h"

// ---------------------------------------------------------------------------------------------
// timing
// ---------------------------------------------------------------------------------------------
static void kst_reset(vh_batch *b) {
    HIP_TRY(hipMemsetAsync(b->d_kst, 0xFF, sizeof(unsigned long long) * VH_KST_CAP, b->stream));
    HIP_TRY(hipMemsetAsync(b->d_kst + VH_KST_CAP, 0, sizeof(unsigned long long) * VH_KST_CAP, b->stream));
    b->kst_n = 0;
}

ScopedKTimer::ScopedKTimer(vh_batch *bb, const char *name, double bytes, bool stamped, hipStream_t on)
    : b(bb), t(nullptr), s(on ? on : bb->stream) {
    if (!b->profile) return;
    t = &b->timers[name];
    if (bytes > 0) t->bytes_per_launch = bytes;
    if (stamped) {
        if (!b->d_kst) {
            HIP_TRY(hipMalloc((void **)&b->d_kst, sizeof(unsigned long long) * 2 * VH_KST_CAP));
            kst_reset(b);
        }
        if (b->kst_n < VH_KST_CAP) {
            const int s = b->kst_n++;
            t->slots.push_back(s);
            ks = b->d_kst + s;
            return;
        }   // (every slot taken until the next resolve: events)
    }
    hipEvent_t e0;
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    HIP_TRY(hipEventRecord(e0, s));
    t->ev.push_back(e0);
}
ScopedKTimer::~ScopedKTimer() {
    if (!t || ks) return;
    (void)hipEventRecord(e1, s);
    t->ev.push_back(e1);
}

static void clear_timers(vh_batch *b) {
    for (auto &kv : b->timers)
        for (auto e : kv.second.ev) (void)hipEventDestroy(e);
    b->timers.clear();
    if (b->d_kst && b->kst_n) kst_reset(b);
}

static void resolve_timers(vh_batch *b) {
    std::vector<unsigned long long> ks;
    double ticks_per_ms = 0.0;
    if (b->d_kst && b->kst_n) {   // the stamped launches' spans (wall clock ticks; the rate in kHz)
        HIP_TRY(hipStreamSynchronize(b->stream));
        ks.resize(2 * VH_KST_CAP);
        HIP_TRY(hipMemcpy(ks.data(), b->d_kst, sizeof(unsigned long long) * 2 * VH_KST_CAP,
                          hipMemcpyDeviceToHost));
        int khz = 0;
        HIP_TRY(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, b->ctx->device));
        ticks_per_ms = (double)khz;
    }
    for (auto &kv : b->timers) {
        KTimer &t = kv.second;
        for (size_t i = 0; i + 1 < t.ev.size(); i += 2) {
            float ms = 0.f;
            HIP_TRY(hipEventSynchronize(t.ev[i + 1]));
            HIP_TRY(hipEventElapsedTime(&ms, t.ev[i], t.ev[i + 1]));
            t.total_ms += ms;
            t.launches += 1;
            (void)hipEventDestroy(t.ev[i]);
            (void)hipEventDestroy(t.ev[i + 1]);
        }
        t.ev.clear();
        for (int s : t.slots) {
            const unsigned long long s0 = ks[s], s1 = ks[VH_KST_CAP + s];
            if (s1 >= s0 && ticks_per_ms > 0.0) t.total_ms += (double)(s1 - s0) / ticks_per_ms;
            t.launches += 1;
        }
        t.slots.clear();
    }
    if (!ks.empty()) kst_reset(b);
}

// ---------------------------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------------------------
static int fail(vh_ctx *c, int code, const std::string &msg) {
    if (c) {
        std::lock_guard<std::mutex> g(c->err_mu);
        c->last_error = msg;
    }
    return code;
}

#define API_TRY(ctx, ...)                                                                    \
    try {                                                                                    \
        __VA_ARGS__                                                                          \
    } catch (const VhError &e) {                                                             \
        return fail(ctx, e.code, e.msg);                                                     \
    } catch (const std::bad_alloc &) {                                                       \
        return fail(ctx, VH_ERR_NOMEM, "host allocation failed");                            \
    } catch (const std::exception &e) {                                                      \
        return fail(ctx, VH_ERR_HIP, e.what());                                              \
    } catch (...) {                                                                          \
        return fail(ctx, VH_ERR_HIP, "unknown error");                                       \
    }                                                                                        \
    return VH_OK;

template <typename T>
static void dalloc(T **p, size_t n) {
    HIP_TRY(hipMalloc((void **)p, sizeof(T) * (n ? n : 1)));
}
template <typename T>
static void dfree(T *&p) {
    if (p) (void)hipFree((void *)p);
    p = nullptr;
}

static void check_dims(int64_t R, int64_t C, int64_t Z, int64_t batch) {
    if (R < 2 || C < 2 || Z < 1 || batch < 1)
        throw VhError{VH_ERR_ARG, "dims must be R>=2, C>=2, Z>=1, batch>=1"};
    if (R * C * Z >= (int64_t)1 << 31)
        throw VhError{VH_ERR_ARG, "a volume must have < 2^31 voxels"};
    if (R > 65535 || C * Z > ((int64_t)1 << 31))
        throw VhError{VH_ERR_ARG, "volume dims out of range"};
}

static void batch_free(vh_batch *b) {
    if (!b) return;
    clear_timers(b);
    dfree(b->d_kst);
    dfree(b->d_hp); dfree(b->d_mask); dfree(b->d_n4);
    dfree(b->d_defect); dfree(b->d_border); dfree(b->d_lb);
    dfree(b->d_colrange); dfree(b->d_colcount); dfree(b->d_colstart); dfree(b->d_colbits); dfree(b->d_colbnz); dfree(b->d_snrpart);
    dfree(b->d_rowany); dfree(b->d_colany); dfree(b->d_sliceany);
    dfree(b->d_sc); dfree(b->d_part); dfree(b->d_keys0); dfree(b->d_keys1); dfree(b->d_tilecnt);
    dfree(b->d_cohort);
    dfree(b->d_L0); dfree(b->d_lat); dfree(b->d_E);
    dfree(b->d_numfix); dfree(b->d_rowstart); dfree(b->d_rowmask); dfree(b->d_rrank); dfree(b->d_iscan); dfree(b->d_D); dfree(b->d_perm); dfree(b->d_P1); dfree(b->d_den); dfree(b->d_T); dfree(b->d_pcdrift);
    dfree(b->d_U); dfree(b->d_ridx); dfree(b->d_cp); dfree(b->d_cvol); dfree(b->d_hpart); dfree(b->d_hred); dfree(b->d_cpart); dfree(b->d_st); dfree(b->d_nactive); dfree(b->d_tabs); dfree(b->d_twiddle); dfree(b->d_study_lv); dfree(b->d_study_order); dfree(b->d_pcg); dfree(b->d_stg); dfree(b->d_sortg); dfree(b->d_study_latg);
    dfree(b->d_bitmap); dfree(b->d_ci_list); dfree(b->d_ci_shell); dfree(b->d_ci_hist);
    dfree(b->d_ci_status);
    dfree(b->d_ci_count); dfree(b->d_ci_map);
    if (b->stream) (void)hipStreamDestroy(b->stream);
    if (b->st_n4) (void)hipStreamDestroy(b->st_n4);
    if (b->ev_n4_pre) (void)hipEventDestroy(b->ev_n4_pre);
    if (b->ev_n4_post) (void)hipEventDestroy(b->ev_n4_post);
    if (b->ev_cpre) (void)hipEventDestroy(b->ev_cpre);
    if (b->ev_cpost) (void)hipEventDestroy(b->ev_cpost);
    if (b->h_flags) (void)hipHostFree(b->h_flags);
    delete b;
}

static vh_batch *batch_new(vh_ctx *ctx, int64_t R, int64_t C, int64_t Z, int64_t nb) {
    check_dims(R, C, Z, nb);
    HIP_TRY(hipSetDevice(ctx->device));
    vh_batch *b = new vh_batch;
    b->ctx = ctx;
    // Study-kernel stream (A/B options, off by default).  VH_PRIO=1: the batch's stream at the
    // highest priority and its study kernel on a second stream at the lowest.  VH_ST_RESERVE=k
    // (1-4): the study kernel on a second stream whose CU mask leaves k CUs per XCD to the batch's
    // other kernels (mask bits 33 j + 8 m, j < 8, m < k: one per XCD whether the bits map to XCDs
    // in blocks of 32 or interleaved), so another batch's short kernels never wait for a CU that
    // studies hold.
    const char *pe = getenv("VH_PRIO"), *re = getenv("VH_ST_RESERVE");
    const bool prio = pe && atoi(pe) != 0;
    const int reserve = re ? std::max(0, std::min(4, atoi(re))) : 0;
    int lo = 0, hi = 0;
    if (prio) (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    hipError_t se = prio ? hipStreamCreateWithPriority(&b->stream, hipStreamNonBlocking, hi)
                         : hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking);
    if (se == hipSuccess && reserve > 0) {
        int ncu = 0;
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, ctx->device);
        std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0xffffffffu);
        for (int j = 0; j < 8; ++j)
            for (int m = 0; m < reserve; ++m) {
                const int i = 33 * j + 8 * m;
                if (i < ncu) mask[i / 32] &= ~(1u << (i % 32));
            }
        se = hipExtStreamCreateWithCUMask(&b->st_n4, (uint32_t)mask.size(), mask.data());
    } else if (se == hipSuccess && prio) {
        se = hipStreamCreateWithPriority(&b->st_n4, hipStreamNonBlocking, lo);
    }
    if (se == hipSuccess && b->st_n4)
        se = hipEventCreateWithFlags(&b->ev_n4_pre, hipEventDisableTiming);
    if (se == hipSuccess && b->st_n4)
        se = hipEventCreateWithFlags(&b->ev_n4_post, hipEventDisableTiming);
    if (se != hipSuccess) {
        if (b->ev_n4_pre) (void)hipEventDestroy(b->ev_n4_pre);
        if (b->stream) (void)hipStreamDestroy(b->stream);
        if (b->st_n4) (void)hipStreamDestroy(b->st_n4);
        delete b;
        throw VhError{VH_ERR_HIP, "batch stream creation failed"};
    }
    b->R = R; b->C = C; b->Z = Z; b->nb = nb;
    b->V = R * C * Z;
    b->CZ = C * Z;
    b->max_tiles = (b->V + VH_SORT_TILE - 1) / VH_SORT_TILE;
    const size_t NV = (size_t)nb * b->V;
    try {
        dalloc(&b->d_hp, NV);
        dalloc(&b->d_mask, NV);
        dalloc(&b->d_n4, NV);
        dalloc(&b->d_defect, NV);
        dalloc(&b->d_border, NV);
        dalloc(&b->d_lb, NV);
        dalloc(&b->d_colrange, (size_t)nb * b->CZ * 2);
        dalloc(&b->d_colcount, (size_t)nb * b->CZ);
        dalloc(&b->d_colbits, (size_t)nb * ((R + 31) / 32) * b->CZ);
        dalloc(&b->d_colbnz, (size_t)nb * ((R + 31) / 32) * b->CZ);
        dalloc(&b->d_colstart, (size_t)nb * b->CZ);
        dalloc(&b->d_rowany, (size_t)nb * R);
        dalloc(&b->d_colany, (size_t)nb * C);
        dalloc(&b->d_sliceany, (size_t)nb * Z);
        dalloc(&b->d_sc, (size_t)nb);
        b->part_blocks = (b->CZ + VH_TPB - 1) / VH_TPB;
        b->slab_blocks = b->part_blocks * ((R + VH_SLAB - 1) / VH_SLAB);
        dalloc(&b->d_snrpart, (size_t)nb * b->slab_blocks * 4);
        const int64_t max_chunks = (b->V + 8191) / 8192;
        const int64_t eval_slots = ((b->CZ + 63) / 64) * ((R + 15) / 16);   // n4 eval partial slots
        dalloc(&b->d_part, (size_t)nb * std::max<int64_t>(std::max<int64_t>(b->part_blocks * 4, max_chunks),
                                                         eval_slots * 2));
        dalloc(&b->d_keys0, NV);
        dalloc(&b->d_keys1, NV);
        dalloc(&b->d_tilecnt, (size_t)nb * 256 * b->max_tiles);
        dalloc(&b->d_cohort, (size_t)VH_COHORT_BINS);
        HIP_TRY(hipMemset(b->d_cohort, 0, sizeof(uint64_t) * VH_COHORT_BINS));
    } catch (...) {
        batch_free(b);
        throw;
    }
    return b;
}

static void batch_upload(vh_batch *b, const float *hp, const uint8_t *mask) {
    hipStream_t st = b->stream;
    const size_t NV = (size_t)b->nb * b->V;
    if (hp) HIP_TRY(hipMemcpyAsync(b->d_hp, hp, sizeof(float) * NV, hipMemcpyHostToDevice, st));
    if (mask) HIP_TRY(hipMemcpyAsync(b->d_mask, mask, NV, hipMemcpyHostToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));
}

static void check_n4_params(const vh_batch *b, const vh_n4_params &p) {
    if (p.n_levels < 1 || p.n_levels > VH_MAX_LEVELS || p.spline_order != 3 || p.n_bins < 2 ||
        p.n_bins > VH_MAX_BINS || p.ncp[0] < 4 || p.ncp[1] < 4 || p.ncp[2] < 4 || b->Z < 2 ||
        p.conv_mode < 0 || p.conv_mode > 1)
        throw VhError{VH_ERR_ARG, "unsupported N4 parameters (spline order 3, bins <= 256, ncp >= 4, "
                                  "Z >= 2, conv_mode 0 or 1)"};
    int tot = 0;
    for (int l = 0; l < p.n_levels; ++l) {
        if (p.max_iters[l] < 1) throw VhError{VH_ERR_ARG, "max_iters must be >= 1"};
        tot += p.max_iters[l];
    }
    if (tot > 8 * 1024 - 1) throw VhError{VH_ERR_ARG, "too many N4 iterations"};
}

// n4_src: 0 = run N4 from d_hp, 1 = identity (d_hp), 2 = caller-uploaded d_n4
static void batch_run(vh_batch *b, const vh_run_opts &o, int n4_src) {
    HIP_TRY(hipSetDevice(b->ctx->device));
    b->profile = o.profile != 0;
    b->opts = o;
    b->n4_subbatch = o.n4_subbatch;
    b->n4_mode = o.n4_mode;
    if (o.do_n4) check_n4_params(b, o.n4);
    vh_launch_mask_stats(b);
    const float *n4 = b->d_hp;
    if (o.do_n4) {
        vh_launch_n4(b, o.n4);
        n4 = b->d_n4;
    } else if (n4_src == 2) {
        n4 = b->d_n4;
    }
    vh_launch_vdp_chain(b, n4, o);
    b->have_result = true;
}

// the study kernel's spin-wait watchdog (n4_study.hip st_spin) leaves N4State.active = -2
static void check_n4_watchdog(const N4State *st, int64_t nb) {
    for (int64_t i = 0; i < nb; ++i)
        if (st[i].active == -2) throw VhError{VH_ERR_HIP, "N4 study kernel: a synchronisation wait timed out"};
}

// small device -> host copy ordered on the batch's own stream: a synchronous hipMemcpy goes through
// the null stream, whose hardware queue is shared with one of the pipe slots' streams once there are
// more streams than queues (GPU_MAX_HW_QUEUES), so it waited for that slot's queued work
static void d2h_on_stream(vh_batch *b, void *dst, const void *src, size_t bytes) {
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, b->stream));
    HIP_TRY(hipStreamSynchronize(b->stream));
}

static void fill_results_from(const vh_batch *b, const VolScalars *sc, const N4State *st, vh_vdp_result *res);

static void fill_results(vh_batch *b, vh_vdp_result *res) {
    std::vector<VolScalars> sc(b->nb);
    d2h_on_stream(b, sc.data(), b->d_sc, sizeof(VolScalars) * b->nb);
    std::vector<N4State> st;
    if (b->opts.do_n4) {
        st.resize(b->nb);
        d2h_on_stream(b, st.data(), b->d_st, sizeof(N4State) * b->nb);
    }
    fill_results_from(b, sc.data(), st.data(), res);
}

// per-study results from host copies of the scalars (and N4 states when the batch ran N4)
static void fill_results_from(const vh_batch *b, const VolScalars *sc, const N4State *st, vh_vdp_result *res) {
    if (b->opts.do_n4) check_n4_watchdog(st, b->nb);
    const double *vox = b->opts.vox;
    // np.prod(np.divide(vox, 10)): sequential multiply (Vent_Analysis.py:166, 252)
    const double pv = ((vox[0] / 10.0) * (vox[1] / 10.0)) * (vox[2] / 10.0);
    for (int64_t i = 0; i < b->nb; ++i) {
        vh_vdp_result &r = res[i];
        memset(&r, 0, sizeof r);
        const VolScalars &s = sc[i];
        const double nm = (double)s.n_mask;
        r.n_mask = s.n_mask;
        r.n_defect = s.n_defect;
        r.n_lb12 = s.n_lb12;
        r.n_km0 = s.n_km0;
        r.vdp = (100.0 * (double)s.n_defect) / nm;
        r.vdp_lb = (100.0 * (double)s.n_lb12) / nm;
        r.vdp_km = b->opts.do_kmeans ? (100.0 * (double)s.n_km0) / nm : 0.0;
        r.defect_volume = (double)s.n_defect * pv / 1000.0;
        r.lung_volume = (double)s.n_mask1 * pv / 1000.0;
        for (int j = 0; j < 4; ++j) r.km_centres[j] = s.km_c[j];
        r.snr = b->opts.do_snr ? s.snr : 0.0;
        r.mean_anchor = s.mean_anchor;
        r.p99 = s.p99;
        if (b->opts.do_n4)
            for (int l = 0; l < b->opts.n4.n_levels; ++l) {
                r.n4_iters[l] = st[i].iters_level[l];
                r.n4_conv[l] = st[i].conv_level[l];
            }
    }
}

static void batch_download(vh_batch *b, float *n4, uint8_t *defect, uint8_t *border, uint8_t *lb,
                           vh_vdp_result *res) {
    hipStream_t st = b->stream;
    HIP_TRY(hipStreamSynchronize(st));
    const size_t NV = (size_t)b->nb * b->V;
    if (n4) HIP_TRY(hipMemcpy(n4, b->opts.do_n4 ? b->d_n4 : b->d_hp, sizeof(float) * NV, hipMemcpyDeviceToHost));
    if (defect) HIP_TRY(hipMemcpy(defect, b->d_defect, NV, hipMemcpyDeviceToHost));
    if (border) HIP_TRY(hipMemcpy(border, b->d_border, NV, hipMemcpyDeviceToHost));
    if (lb) HIP_TRY(hipMemcpy(lb, b->d_lb, NV, hipMemcpyDeviceToHost));
    if (res) fill_results(b, res);
}

static void pipe_free(vh_pipe *p) {
    if (!p) return;
    for (auto &q : p->slot) {
        if (q.b) {
            (void)hipStreamSynchronize(q.b->stream);
            batch_free(q.b);
        }
        if (q.hp) (void)hipHostFree(q.hp);
        if (q.d_pack) (void)hipFree(q.d_pack);
        if (q.mb) (void)hipHostFree(q.mb);
        if (q.n4) (void)hipHostFree(q.n4);
        if (q.u8) (void)hipHostFree(q.u8);
        if (q.done) (void)hipEventDestroy(q.done);
        if (q.h2d) (void)hipEventDestroy(q.h2d);
        if (q.packed) (void)hipEventDestroy(q.packed);

    }
    delete p;
}

// The context's cached scratch batch for the host-buffer entry points (caller holds ctx->mu).
static vh_batch *scratch_batch(vh_ctx *ctx, int64_t R, int64_t C, int64_t Z, int64_t nb) {
    vh_batch *&s = ctx->scratch;
    if (s && s->R == R && s->C == C && s->Z == Z && s->nb == nb) return s;
    if (s) {
        (void)hipStreamSynchronize(s->stream);
        batch_free(s);
    }
    s = nullptr;
    s = batch_new(ctx, R, C, Z, nb);
    return s;
}

// ---------------------------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------------------------
extern "C" {

int vh_abi_version(void) { return VH_ABI_VERSION; }

const char *vh_status_string(int s) {
    switch (s) {
        case VH_OK: return "ok";
        case VH_ERR_ARG: return "invalid argument";
        case VH_ERR_HIP: return "HIP runtime error";
        case VH_ERR_NOMEM: return "out of device memory";
        case VH_ERR_MAXRADIUS: return "cluster index: maximum radius reached";
        case VH_ERR_EMPTY: return "empty mask or defect list";
        case VH_ERR_RCCL: return "RCCL error";
        case VH_ERR_NODEV: return "no GPU device";
        case VH_ERR_INDEX: return "index out of range";
        default: return "unknown status";
    }
}

int vh_device_count(int *n) {
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    *n = e == hipSuccess ? c : 0;
    return VH_OK;
}

void vh_n4_default_params(vh_n4_params *p) {
    memset(p, 0, sizeof *p);
    p->n_levels = 4;
    for (int i = 0; i < 4; ++i) p->max_iters[i] = 50;
    p->conv_threshold = 0.001f;
    p->ncp[0] = p->ncp[1] = p->ncp[2] = 4;
    p->spline_order = 3;
    p->n_bins = 200;
    p->wiener_noise = 0.01f;
    p->fwhm = 0.15f;
    p->conv_mode = 0;
}

void vh_default_run_opts(vh_run_opts *o) {
    memset(o, 0, sizeof *o);
    o->do_n4 = 1;
    vh_n4_default_params(&o->n4);
    o->thresh = 0.6f;
    o->do_snr = 1;
    o->do_kmeans = 1;
    o->do_cohort = 0;
    o->profile = 0;
    o->vox[0] = o->vox[1] = o->vox[2] = 1.0;
}

int vh_create(int device, vh_ctx **out) {
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return VH_ERR_NODEV;
    if (device < 0 || device >= n) return VH_ERR_ARG;
    vh_ctx *c = new vh_ctx;
    c->device = device;
    API_TRY(c, {
        HIP_TRY(hipSetDevice(device));
        *out = c;
    })
}

int vh_destroy(vh_ctx *ctx) {
    if (!ctx) return VH_OK;
    (void)hipSetDevice(ctx->device);
    if (ctx->scratch) {
        (void)hipStreamSynchronize(ctx->scratch->stream);
        batch_free(ctx->scratch);
        ctx->scratch = nullptr;
    }
    if (ctx->comm) ncclCommDestroy((ncclComm_t)ctx->comm);
    if (ctx->h_ci_sc) (void)hipHostFree(ctx->h_ci_sc);
    if (ctx->aux) (void)hipStreamDestroy(ctx->aux);
    if (ctx->comm_st) (void)hipStreamDestroy(ctx->comm_st);
    if (ctx->recon_buf) (void)hipFree(ctx->recon_buf);
    delete ctx;
    return VH_OK;
}

const char *vh_last_error(const vh_ctx *ctx) {
    static thread_local std::string copy;   // stable until this thread's next call
    if (!ctx) return "";
    std::lock_guard<std::mutex> g(ctx->err_mu);
    copy = ctx->last_error;
    return copy.c_str();
}

int vh_synchronize(vh_ctx *ctx) {
    API_TRY(ctx, {
        HIP_TRY(hipSetDevice(ctx->device));
        HIP_TRY(hipDeviceSynchronize());
    })
}

int vh_n4(vh_ctx *ctx, const float *hp, const uint8_t *mask, int64_t R, int64_t C, int64_t Z,
          int64_t batch, const vh_n4_params *prm, float *out, int32_t *iters, float *conv) {
    API_TRY(ctx, {
        std::lock_guard<std::mutex> lock(ctx->mu);
        if (!hp || !mask || !out || !prm) throw VhError{VH_ERR_ARG, "null buffer"};
        vh_batch *b = scratch_batch(ctx, R, C, Z, batch);
        check_n4_params(b, *prm);
        batch_upload(b, hp, mask);
        vh_run_opts o;
        vh_default_run_opts(&o);
        o.n4 = *prm;
        o.do_n4 = 1;
        clear_timers(b);
        b->profile = false;
        b->opts = o;
        HIP_TRY(hipSetDevice(ctx->device));
        vh_launch_mask_stats(b);
        vh_launch_n4(b, o.n4);
        HIP_TRY(hipStreamSynchronize(b->stream));
        HIP_TRY(hipMemcpy(out, b->d_n4, sizeof(float) * batch * b->V, hipMemcpyDeviceToHost));
        std::vector<N4State> st(batch);
        HIP_TRY(hipMemcpy(st.data(), b->d_st, sizeof(N4State) * batch, hipMemcpyDeviceToHost));
        check_n4_watchdog(st.data(), batch);
        for (int64_t i = 0; i < batch; ++i)
            for (int l = 0; l < prm->n_levels; ++l) {
                if (iters) iters[i * prm->n_levels + l] = st[i].iters_level[l];
                if (conv) conv[i * prm->n_levels + l] = st[i].conv_level[l];
            }
        std::vector<VolScalars> sc(batch);
        HIP_TRY(hipMemcpy(sc.data(), b->d_sc, sizeof(VolScalars) * batch, hipMemcpyDeviceToHost));
        for (int64_t i = 0; i < batch; ++i)
            if (sc[i].n_mask1 < 2) throw VhError{VH_ERR_EMPTY, "N4 needs at least 2 voxels with mask == 1"};
    })
}

int vh_border(vh_ctx *ctx, const uint8_t *a, int64_t R, int64_t C, int64_t Z, int64_t batch,
              uint8_t *border) {
    API_TRY(ctx, {
        std::lock_guard<std::mutex> lock(ctx->mu);
        if (!a || !border) throw VhError{VH_ERR_ARG, "null buffer"};
        vh_batch *b = scratch_batch(ctx, R, C, Z, batch);
        HIP_TRY(hipSetDevice(ctx->device));
        b->profile = false;
        const size_t NV = (size_t)batch * b->V;
        HIP_TRY(hipMemcpyAsync(b->d_defect, a, NV, hipMemcpyHostToDevice, b->stream));
        vh_launch_border(b, b->d_defect, b->d_border);
        HIP_TRY(hipMemcpyAsync(border, b->d_border, NV, hipMemcpyDeviceToHost, b->stream));
        HIP_TRY(hipStreamSynchronize(b->stream));
    })
}

int vh_snr(vh_ctx *ctx, const float *hp, const uint8_t *mask, int64_t R, int64_t C, int64_t Z,
           int64_t batch, double *snr) {
    API_TRY(ctx, {
        std::lock_guard<std::mutex> lock(ctx->mu);
        if (!hp || !mask || !snr) throw VhError{VH_ERR_ARG, "null buffer"};
        vh_batch *b = scratch_batch(ctx, R, C, Z, batch);
        batch_upload(b, hp, mask);
        HIP_TRY(hipSetDevice(ctx->device));
        b->profile = false;
        vh_launch_mask_stats(b);
        vh_launch_snr(b);
        HIP_TRY(hipStreamSynchronize(b->stream));
        std::vector<VolScalars> sc(batch);
        HIP_TRY(hipMemcpy(sc.data(), b->d_sc, sizeof(VolScalars) * batch, hipMemcpyDeviceToHost));
        for (int64_t i = 0; i < batch; ++i) {
            if (!sc[i].snr_ok) throw VhError{VH_ERR_ARG, "calculate_SNR: no masked column > 0 (numpy min of an empty array)"};
            snr[i] = sc[i].snr;
        }
    })
}

int vh_vdp(vh_ctx *ctx, const float *hp, const float *n4, const uint8_t *mask, int64_t R,
           int64_t C, int64_t Z, int64_t batch, float thresh, const double vox[3],
           uint8_t *defect, uint8_t *defect_border, uint8_t *lb, vh_vdp_result *res) {
    API_TRY(ctx, {
        std::lock_guard<std::mutex> lock(ctx->mu);
        if (!n4 || !mask || !res || !vox) throw VhError{VH_ERR_ARG, "null buffer"};
        vh_batch *b = scratch_batch(ctx, R, C, Z, batch);
        const size_t NV = (size_t)batch * b->V;
        HIP_TRY(hipMemcpyAsync(b->d_n4, n4, sizeof(float) * NV, hipMemcpyHostToDevice, b->stream));
        batch_upload(b, hp, mask);
        vh_run_opts o;
        vh_default_run_opts(&o);
        o.do_n4 = 0;
        o.do_snr = hp != nullptr;
        o.thresh = thresh;
        for (int i = 0; i < 3; ++i) o.vox[i] = vox[i];
        batch_run(b, o, 2);
        batch_download(b, nullptr, defect, defect_border, lb, res);
        std::vector<VolScalars> sc(batch);
        HIP_TRY(hipMemcpy(sc.data(), b->d_sc, sizeof(VolScalars) * batch, hipMemcpyDeviceToHost));
        for (int64_t i = 0; i < batch; ++i) {
            if (sc[i].n_mask <= 0) throw VhError{VH_ERR_EMPTY, "empty mask"};
            if (hp && !sc[i].snr_ok) throw VhError{VH_ERR_ARG, "calculate_SNR: no masked column > 0"};
        }
    })
}

// page-locked host buffers handed out by vh_host_alloc, by base address: a CI map destined for one
// is written there by the scatter kernel directly (device-mapped), with no staging copy
static std::mutex g_host_mu;
static std::map<uintptr_t, std::pair<size_t, void *>> g_host;   // base -> (bytes, device pointer)

static void *host_mapped(const void *p, size_t bytes) {
    std::lock_guard<std::mutex> lock(g_host_mu);
    const uintptr_t a = (uintptr_t)p;
    auto it = g_host.upper_bound(a);
    if (it == g_host.begin()) return nullptr;
    --it;
    if (a + bytes > it->first + it->second.first) return nullptr;
    return (char *)it->second.second + (a - it->first);
}

// CI on host buffers through a device-resident table; shared by vh_ci and vh_ci_tab
static void ci_host(vh_ctx *ctx, const uint8_t *defect, int64_t R, int64_t C, int64_t Z, int64_t batch,
                    const vh_ci_table *t, double minvox, double *ci_array, double *ci_scalar, int32_t *shell) {
    if (!defect || !t) throw VhError{VH_ERR_ARG, "null defect map / table"};
    if (t->ctx != ctx) throw VhError{VH_ERR_ARG, "sphere table of another context"};
    vh_batch *b = scratch_batch(ctx, R, C, Z, batch);
    HIP_TRY(hipSetDevice(ctx->device));
    b->profile = ctx->profile != 0;
    const size_t NV = (size_t)batch * b->V;
    HIP_TRY(hipMemcpyAsync(b->d_defect, defect, NV, hipMemcpyHostToDevice, b->stream));
    // the map straight into the caller's buffer when it is one of vh_host_alloc's (the scatter's
    // stores cross the link; no device map, no copy), else a device map and one D2H
    double *d_map = ci_array ? (double *)host_mapped(ci_array, sizeof(double) * NV) : nullptr;
    if (ci_array && !d_map) {
        if (!b->d_ci_map) HIP_TRY(hipMalloc(&b->d_ci_map, sizeof(double) * NV));
        d_map = b->d_ci_map;
    }
    // the scalars likewise, into the context's device-mapped page-locked array (a small D2H runs as
    // a blit kernel, r4al: 4.7 us plus its gap)
    if (ctx->h_ci_sc_cap < batch) {
        if (ctx->h_ci_sc) HIP_TRY(hipHostFree(ctx->h_ci_sc));
        ctx->h_ci_sc = nullptr;
        ctx->h_ci_sc_cap = 0;
        HIP_TRY(hipHostMalloc((void **)&ctx->h_ci_sc, sizeof(VolScalars) * batch, hipHostMallocDefault));
        ctx->h_ci_sc_cap = batch;
    }
    VolScalars *d_hsc = nullptr;
    HIP_TRY(hipHostGetDevicePointer((void **)&d_hsc, ctx->h_ci_sc, 0));
    vh_ci_run(b, t, minvox, d_map, d_hsc);
    if (ci_array && d_map == b->d_ci_map)
        HIP_TRY(hipMemcpyAsync(ci_array, b->d_ci_map, sizeof(double) * NV, hipMemcpyDeviceToHost, b->stream));
    if (shell) HIP_TRY(hipMemcpyAsync(shell, b->d_ci_shell, sizeof(int32_t) * NV, hipMemcpyDeviceToHost, b->stream));
    HIP_TRY(hipStreamSynchronize(b->stream));
    vh_ci_debug_check();
    const VolScalars *sc = ctx->h_ci_sc;
    for (int64_t i = 0; i < batch; ++i) {
        if (ci_scalar) ci_scalar[i] = sc[i].ci_scalar;
        if (sc[i].ci_status == VH_ERR_MAXRADIUS)
            throw VhError{VH_ERR_MAXRADIUS, "--MAX RADIUS REACHED-- (CI.py:101-103)"};
        if (sc[i].ci_status == VH_ERR_EMPTY)
            throw VhError{VH_ERR_EMPTY, "no defect voxels (Vent_Analysis.py:270 IndexError)"};
    }
}

int vh_ci(vh_ctx *ctx, const uint8_t *defect, int64_t R, int64_t C, int64_t Z, int64_t batch,
          const int16_t *offs, const uint8_t *dup, int64_t rows, const int32_t *bounds,
          const double *radii, int64_t nb, double minvox, double *ci_array, double *ci_scalar,
          int32_t *shell) {
    API_TRY(ctx, {
        std::lock_guard<std::mutex> lock(ctx->mu);
        std::unique_ptr<vh_ci_table, void (*)(vh_ci_table *)> t(
            vh_ci_table_build(ctx, R, C, offs, dup, rows, bounds, radii, nb), vh_ci_table_free);
        ci_host(ctx, defect, R, C, Z, batch, t.get(), minvox, ci_array, ci_scalar, shell);
    })
}

int vh_ci_table_create(vh_ctx *ctx, int64_t R, int64_t C, const int16_t *offs, const uint8_t *dup,
                       int64_t rows, const int32_t *bounds, const double *radii, int64_t nb,
                       vh_ci_table **out) {
    if (out) *out = nullptr;
    API_TRY(ctx, {
        if (!out) throw VhError{VH_ERR_ARG, "null out"};
        std::lock_guard<std::mutex> lock(ctx->mu);
        *out = vh_ci_table_build(ctx, R, C, offs, dup, rows, bounds, radii, nb);
    })
}

// Tables are used only by ci_host on the context's scratch stream, under ctx->mu: taking the lock
// waits for a CI call of another thread, and the scratch stream is drained before the hipFrees, so
// no kernel can read a freed table (the destroy ran with neither).
int vh_ci_table_destroy(vh_ci_table *t) {
    if (!t) return VH_OK;
    vh_ctx *ctx = t->ctx;
    std::lock_guard<std::mutex> lock(ctx->mu);
    (void)hipSetDevice(ctx->device);
    if (ctx->scratch) (void)hipStreamSynchronize(ctx->scratch->stream);
    vh_ci_table_free(t);
    return VH_OK;
}

int vh_ci_tab(vh_ctx *ctx, const uint8_t *defect, int64_t R, int64_t C, int64_t Z, int64_t batch,
              const vh_ci_table *t, double minvox, double *ci_array, double *ci_scalar, int32_t *shell) {
    API_TRY(ctx, {
        std::lock_guard<std::mutex> lock(ctx->mu);
        ci_host(ctx, defect, R, C, Z, batch, t, minvox, ci_array, ci_scalar, shell);
    })
}

int vh_batch_create(vh_ctx *ctx, int64_t R, int64_t C, int64_t Z, int64_t batch, vh_batch **out) {
    *out = nullptr;
    API_TRY(ctx, { *out = batch_new(ctx, R, C, Z, batch); })
}

int vh_batch_destroy(vh_batch *b) {
    if (b) {
        (void)hipSetDevice(b->ctx->device);
        (void)hipStreamSynchronize(b->stream);
        batch_free(b);
    }
    return VH_OK;
}

int vh_batch_upload(vh_batch *b, const float *hp, const uint8_t *mask) {
    API_TRY(b->ctx, {
        HIP_TRY(hipSetDevice(b->ctx->device));
        batch_upload(b, hp, mask);
    })
}

int vh_batch_run(vh_batch *b, const vh_run_opts *opts) {
    API_TRY(b->ctx, {
        if (!opts) throw VhError{VH_ERR_ARG, "null options"};
        batch_run(b, *opts, opts->do_n4 ? 0 : 1);
    })
}

int vh_batch_sync(vh_batch *b) {
    API_TRY(b->ctx, { HIP_TRY(hipStreamSynchronize(b->stream)); })
}

int vh_batch_download(vh_batch *b, float *n4, uint8_t *defect, uint8_t *defect_border, uint8_t *lb,
                      vh_vdp_result *res) {
    API_TRY(b->ctx, {
        if (!b->have_result) throw VhError{VH_ERR_ARG, "vh_batch_run has not been called"};
        batch_download(b, n4, defect, defect_border, lb, res);
    })
}

int vh_batch_cohort_hist(vh_batch *b, uint64_t *hist) {
    API_TRY(b->ctx, {
        HIP_TRY(hipStreamSynchronize(b->stream));
        HIP_TRY(hipMemcpy(hist, b->d_cohort, sizeof(uint64_t) * VH_COHORT_BINS, hipMemcpyDeviceToHost));
    })
}

const char *vh_batch_kernel_names(void) {
    return "mask_stats;gather;sort;mean;classify;cohort;kmeans;snr;border;n4_init;n4_den;n4_hist;"
           "n4_fit;n4_contract;n4_eval;n4_welford;n4_pcw;n4_pcg;n4_final;n4_study;ci_walk;vdp_chain";
}

int vh_batch_reset_timers(vh_batch *b) {
    API_TRY(b->ctx, {
        HIP_TRY(hipStreamSynchronize(b->stream));
        clear_timers(b);
    })
}

int vh_batch_kernel_time(vh_batch *b, const char *name, double *total_ms, int64_t *launches,
                         double *bytes_per_launch) {
    API_TRY(b->ctx, {
        resolve_timers(b);
        auto it = b->timers.find(name);
        if (it == b->timers.end()) {
            *total_ms = 0; *launches = 0;
            if (bytes_per_launch) *bytes_per_launch = 0;
        } else {
            *total_ms = it->second.total_ms;
            *launches = it->second.launches;
            if (bytes_per_launch) *bytes_per_launch = it->second.bytes_per_launch;
        }
    })
}

int vh_ctx_profile(vh_ctx *ctx, int on) {
    API_TRY(ctx, {
        std::lock_guard<std::mutex> lock(ctx->mu);
        ctx->profile = on ? 1 : 0;
        if (ctx->scratch) {
            HIP_TRY(hipStreamSynchronize(ctx->scratch->stream));
            clear_timers(ctx->scratch);
        }
    })
}

int vh_ctx_kernel_time(vh_ctx *ctx, const char *name, double *total_ms, int64_t *launches) {
    API_TRY(ctx, {
        std::lock_guard<std::mutex> lock(ctx->mu);
        if (!name || !total_ms || !launches) throw VhError{VH_ERR_ARG, "null argument"};
        *total_ms = 0;
        *launches = 0;
        if (ctx->scratch) {
            resolve_timers(ctx->scratch);
            auto it = ctx->scratch->timers.find(name);
            if (it != ctx->scratch->timers.end()) {
                *total_ms = it->second.total_ms;
                *launches = it->second.launches;
            }
        }
    })
}

int vh_batch_study_times(vh_batch *b, double *us) {
    API_TRY(b->ctx, {
        if (!us) throw VhError{VH_ERR_ARG, "null buffer"};
        HIP_TRY(hipStreamSynchronize(b->stream));
        for (int64_t i = 0; i < b->nb; ++i) us[i] = 0.0;
        if (!b->have_result || !b->opts.do_n4 || !b->n4_used_study) return VH_OK;
        std::vector<N4State> st(b->nb);
        d2h_on_stream(b, st.data(), b->d_st, sizeof(N4State) * b->nb);
        int rate_khz = 0;
        HIP_TRY(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, b->ctx->device));
        if (rate_khz <= 0) throw VhError{VH_ERR_HIP, "no device wall clock rate"};
        for (int64_t i = 0; i < b->nb; ++i)
            us[i] = (double)(st[i].t_end - st[i].t_start) * 1000.0 / (double)rate_khz;
        if (const char *path = getenv("VH_STUDY_TRACE")) {   // per study: start, end, placement
            if (FILE *f = fopen(path, "a")) {
                for (int64_t i = 0; i < b->nb; ++i)
                    fprintf(f, "%p,%lld,%llu,%llu,%u,%u,%d,%d,%d,%d\n", (void *)b, (long long)i,
                            (unsigned long long)st[i].t_start, (unsigned long long)st[i].t_end,
                            st[i].hw_id, st[i].xcc_id, rate_khz, st[i].pc_rounds,
                            st[i].pc_fallbacks, st[i].iters_level[0] + st[i].iters_level[1] +
                                st[i].iters_level[2] + st[i].iters_level[3]);
                fclose(f);
            }
        }
    })
}

// ---- rendering (export.hip) ------------------------------------------------------------------
int vh_overlay(vh_ctx *ctx, const float *n4, const uint8_t *defect, int64_t R, int64_t C, int64_t Z,
               int64_t batch, uint8_t *rgb) {
    API_TRY(ctx, {
        std::lock_guard<std::mutex> lock(ctx->mu);
        if (!n4 || !defect || !rgb) throw VhError{VH_ERR_ARG, "overlay: null buffer"};
        HIP_TRY(hipSetDevice(ctx->device));
        vh_batch *b = scratch_batch(ctx, R, C, Z, batch);
        const size_t NV = (size_t)batch * R * C * Z;
        HIP_TRY(hipMemcpyAsync(b->d_n4, n4, sizeof(float) * NV, hipMemcpyHostToDevice, b->stream));
        HIP_TRY(hipMemcpyAsync(b->d_defect, defect, NV, hipMemcpyHostToDevice, b->stream));
        // rgb (3 B/voxel) in the sort-key buffer (4 B/voxel), the |x| min/max in the partials
        uint8_t *d_rgb = reinterpret_cast<uint8_t *>(b->d_keys0);
        uint32_t *d_mm = reinterpret_cast<uint32_t *>(b->d_part);
        vh_overlay_launch(b->stream, b->d_n4, b->d_defect, R, C, Z, batch, d_mm, d_rgb);
        HIP_TRY(hipMemcpyAsync(rgb, d_rgb, 3 * NV, hipMemcpyDeviceToHost, b->stream));
        HIP_TRY(hipStreamSynchronize(b->stream));
    })
}

int vh_montage(vh_ctx *ctx, int64_t R, int64_t C, int64_t Z, const void *proton, int proton_is64,
               const void *hp, int hp_is64, const float *n4, const uint8_t *mask_border,
               const uint8_t *defect, const double *ci, const double *parula, int64_t prow,
               const int64_t crop[6], uint8_t *image) {
    API_TRY(ctx, {
        std::lock_guard<std::mutex> lock(ctx->mu);
        if (!proton || !hp || !n4 || !mask_border || !defect || !parula || !crop || !image)
            throw VhError{VH_ERR_ARG, "montage: null buffer"};
        check_dims(R, C, Z, 1);
        HIP_TRY(hipSetDevice(ctx->device));
        vh_batch *b = scratch_batch(ctx, R, C, Z, 1);
        vh_montage_run(b->stream, R, C, Z, proton, proton_is64, hp, hp_is64, n4, mask_border, defect,
                       ci, parula, prow, crop, image);
    })
}

// ---- TWIX recon (recon.hip) -------------------------------------------------------------------
int vh_recon(vh_ctx *ctx, const double *k, int64_t n0, int64_t n1, int64_t nz, double *out) {
    API_TRY(ctx, {
        std::lock_guard<std::mutex> lock(ctx->mu);
        if (!k || !out) throw VhError{VH_ERR_ARG, "recon: null buffer"};
        if (n0 < 1 || n1 < 1 || nz < 1 || n0 > 5120 || n1 > 5120 || n0 * n1 * nz >= ((int64_t)1 << 31))
            throw VhError{VH_ERR_ARG, "recon: dims must be 1 <= n0, n1 <= 5120, n0 n1 nz < 2^31"};
        HIP_TRY(hipSetDevice(ctx->device));
        if (!ctx->aux) HIP_TRY(hipStreamCreateWithFlags(&ctx->aux, hipStreamNonBlocking));
        const size_t NV = (size_t)(n0 * n1 * nz), bytes = sizeof(double2) * (3 * NV + n0 + n1);
        if (bytes > ctx->recon_cap) {
            if (ctx->recon_buf) HIP_TRY(hipFree(ctx->recon_buf));
            ctx->recon_buf = nullptr;
            ctx->recon_cap = 0;
            HIP_TRY(hipMalloc(&ctx->recon_buf, bytes));
            ctx->recon_cap = bytes;
        }
        double2 *d_in = (double2 *)ctx->recon_buf, *d_tmp = d_in + NV, *d_out = d_tmp + NV,
                *d_tw0 = d_out + NV, *d_tw1 = d_tw0 + n0;
        hipStream_t st = ctx->aux;
        HIP_TRY(hipMemcpyAsync(d_in, k, sizeof(double2) * NV, hipMemcpyHostToDevice, st));
        vh_recon_run(st, d_in, d_tmp, d_out, d_tw0, d_tw1, n0, n1, nz);
        HIP_TRY(hipMemcpyAsync(out, d_out, sizeof(double2) * NV, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    })
}

// ---- host-to-host pipeline -----
// pageable <-> pinned staging copies split over host threads: one thread's memcpy (~5-10 GB/s) bounded
// the whole pipeline at about half the device-resident rate; the copy engines and the
// PCIe link are far from busy at that rate
// The three u8 maps of a pipe chunk leave the GPU as one byte per voxel, defect | border << 1 |
// LB class << 2 (0/1, 0/1, 0..6): PCIe carries H2D and D2H together at ~53 GB/s on the box
// (scripts/dev/h2h_probe.py, both directions at once), so the host-to-host rate is link-bound
// near the device rate; this takes 12 -> 10 bytes per voxel.  The slot's host threads unpack.
__global__ void k_pack_maps(const uint8_t *__restrict__ d, const uint8_t *__restrict__ b,
                            const uint8_t *__restrict__ l, uint8_t *__restrict__ out, int64_t n,
                            const uint32_t *__restrict__ sc, int64_t sc_words,
                            const uint32_t *__restrict__ st, int64_t st_words, uint32_t *__restrict__ scal) {
    // the chunk's scalars and N4 states ahead of the maps (the D2H block's head)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < sc_words + st_words;
         i += (int64_t)gridDim.x * blockDim.x)
        scal[i] = i < sc_words ? sc[i] : st[i - sc_words];
    const int64_t n16 = n / 16;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x) {
        const uint4 vd = reinterpret_cast<const uint4 *>(d)[i], vb = reinterpret_cast<const uint4 *>(b)[i],
                    vl = reinterpret_cast<const uint4 *>(l)[i];
        uint4 o;   // bytes pack lane-wise: no carries (defect, border <= 1, class <= 6)
        o.x = vd.x | (vb.x << 1) | (vl.x << 2);
        o.y = vd.y | (vb.y << 1) | (vl.y << 2);
        o.z = vd.z | (vb.z << 1) | (vl.z << 2);
        o.w = vd.w | (vb.w << 1) | (vl.w << 2);
        reinterpret_cast<uint4 *>(out)[i] = o;
    }
    for (int64_t i = n16 * 16 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = (uint8_t)(d[i] | (b[i] << 1) | (l[i] << 2));
}

static void par_memcpy(void *dst, const void *src, size_t bytes);

// studies cnt .. sub - 1 of a ragged pipe chunk := study cnt - 1 (image and mask)
__global__ void k_repeat_last(float *hp, uint8_t *mask, int64_t V, int64_t cnt, int64_t sub) {
    const int64_t n = (sub - cnt) * V;
    const float *sh = hp + (cnt - 1) * V;
    const uint8_t *sm = mask + (cnt - 1) * V;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t v = i % V;
        hp[cnt * V + i] = sh[v];
        mask[cnt * V + i] = sm[v];
    }
}

// The mask crosses PCIe as one bit per voxel (bit i % 8 of byte i / 8); k_unpack_mask restores the
// bytes on the device.  par_pack_mask returns false (nothing usable) if a byte is not 0 / 1.
__global__ void k_unpack_mask(const uint8_t *__restrict__ bits, uint8_t *__restrict__ mask, int64_t n) {
    const int64_t nb = (n + 7) / 8;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t v = bits[i];
        if (i * 8 + 8 <= n) {
            uint64_t w = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) w |= (uint64_t)((v >> k) & 1u) << (8 * k);
            memcpy(mask + i * 8, &w, 8);
        } else {
            for (int64_t k = 0; i * 8 + k < n; ++k) mask[i * 8 + k] = (uint8_t)((v >> k) & 1u);
        }
    }
}

static bool par_pack_mask(const uint8_t *src, uint8_t *dst, size_t n) {
    const size_t chunk = (size_t)8 << 20;   // bytes of mask per task (a multiple of 8)
    const int want = (int)std::max<size_t>(1, std::min<size_t>(VH_COPY_THREADS, (n + chunk - 1) / chunk));
    std::vector<int> bad(want, 0);
    auto run = [&](int t, size_t o, size_t m) {   // [o, o + m), o a multiple of 8
        uint64_t hi = 0;
        size_t i = o;
        for (; i + 8 <= o + m; i += 8) {
            uint64_t w;
            memcpy(&w, src + i, 8);
            hi |= w;
            dst[i / 8] = (uint8_t)((w * 0x0102040810204080ull) >> 56);   // byte k's bit 0 -> bit k
        }
        if (i < o + m) {
            uint8_t v = 0;
            for (size_t k = 0; i + k < o + m; ++k) {
                hi |= src[i + k];
                v |= (uint8_t)((src[i + k] & 1u) << k);
            }
            dst[i / 8] = v;
        }
        bad[t] = (hi & 0xFEFEFEFEFEFEFEFEull) != 0;
    };
    const size_t per = ((n + want - 1) / want + 7) / 8 * 8;
    std::vector<std::thread> th;
    for (int t = 1; t < want; ++t) {
        const size_t o = per * t;
        if (o < n) th.emplace_back(run, t, o, std::min(per, n - o));
    }
    run(0, 0, std::min(per, n));
    for (auto &x : th) x.join();
    for (int t = 0; t < want; ++t)
        if (bad[t]) return false;
    return true;
}

// the caller's maps from the packed bytes (any of d / b / l may be null), on host threads
static void par_unpack_maps(const uint8_t *src, uint8_t *d, uint8_t *b, uint8_t *l, size_t n) {
    const size_t chunk = (size_t)8 << 20;
    const int want = (int)std::min<size_t>(VH_COPY_THREADS, (n + chunk - 1) / chunk);
    auto run = [=](size_t o, size_t m) {
        for (size_t i = o; i < o + m; ++i) {
            const uint8_t v = src[i];
            if (d) d[i] = v & 1u;
            if (b) b[i] = (v >> 1) & 1u;
            if (l) l[i] = v >> 2;
        }
    };
    if (want <= 1) {
        run(0, n);
        return;
    }
    std::vector<std::thread> th;
    const size_t per = (n + want - 1) / want;
    for (int i = 1; i < want; ++i) {
        const size_t o = per * i;
        if (o < n) th.emplace_back(run, o, std::min(per, n - o));
    }
    run(0, std::min(per, n));
    for (auto &t : th) t.join();
}

static void par_memcpy(void *dst, const void *src, size_t bytes) {
    const size_t chunk = (size_t)16 << 20;   // 16 MiB per task
    const int want = (int)std::min<size_t>(VH_COPY_THREADS, (bytes + chunk - 1) / chunk);
    if (want <= 1) {
        memcpy(dst, src, bytes);
        return;
    }
    std::vector<std::thread> th;
    const size_t per = (bytes + want - 1) / want;
    for (int i = 1; i < want; ++i) {
        const size_t o = per * i, n = std::min(per, bytes - o);
        th.emplace_back([=] { memcpy((char *)dst + o, (const char *)src + o, n); });
    }
    memcpy(dst, src, std::min(per, bytes));
    for (auto &t : th) t.join();
}

// One host thread per slot; slot s owns batch b[s] (its own stream) and pinned staging, and takes
// sub-batches s, s + slots, ...  Within a slot the steps are serial (stage in -> H2D -> pipeline ->
// D2H -> stage out); across slots they overlap, so the copy engines, the host memcpys and the
// compute of different sub-batches run at the same time.
int vh_pipe_create(vh_ctx *ctx, int64_t R, int64_t C, int64_t Z, int64_t sub, int slots,
                   vh_pipe **out) {
    *out = nullptr;
    API_TRY(ctx, {
        if (sub < 1 || slots < 1 || slots > 8) throw VhError{VH_ERR_ARG, "pipe: sub >= 1, 1 <= slots <= 8"};
        HIP_TRY(hipSetDevice(ctx->device));
        vh_pipe *p = new vh_pipe;
        p->ctx = ctx;
        p->R = R; p->C = C; p->Z = Z; p->sub = sub;
        // a per-node budget of 32 GiB page-locked, shared by the node's ranks (LOCAL_WORLD_SIZE, as
        // torchrun and bench.py set it): 8 ranks pin at most 4 GiB each
        int64_t local_ranks = 1;
        if (const char *e = getenv("LOCAL_WORLD_SIZE")) local_ranks = std::max<int64_t>(1, atoll(e));
        p->pin_cap = ((int64_t)32 << 30) / local_ranks;
        if (const char *e = getenv("VH_PIPE_PIN_CAP")) p->pin_cap = atoll(e);
        const size_t NV = (size_t)sub * R * C * Z;
        try {
            for (int s = 0; s < slots; ++s) {
                p->slot.emplace_back();
                vh_pipe::Slot &q = p->slot.back();
                q.b = batch_new(ctx, R, C, Z, sub);
                HIP_TRY(hipHostMalloc((void **)&q.hp, sizeof(float) * NV));
                HIP_TRY(hipHostMalloc((void **)&q.n4, sizeof(float) * NV));
                // the chunk's outputs leave the GPU as ONE copy: the per-study scalars and N4 states,
                // then the packed maps.  Small copies (the scalars were two of ~20 / 11 KiB) run as
                // blit kernels (__amd_rocclr_copyBuffer), which wait for a CU like any kernel -- for
                // milliseconds while k_n4_study holds every CU's LDS (r4a trace); one large copy
                // goes to the SDMA engines.
                q.scal = (sizeof(VolScalars) * sub + sizeof(N4State) * sub + 4095) / 4096 * 4096;
                HIP_TRY(hipHostMalloc((void **)&q.u8, 2 * NV + q.scal));   // mask in | scalars + maps out
                HIP_TRY(hipEventCreateWithFlags(&q.done, hipEventDisableTiming));
                HIP_TRY(hipEventCreateWithFlags(&q.h2d, hipEventDisableTiming));
                HIP_TRY(hipEventCreateWithFlags(&q.packed, hipEventDisableTiming));
                HIP_TRY(hipMalloc((void **)&q.d_pack, (size_t)NV + q.scal));
                q.mb_half = ((size_t)NV / 8 + 1 + 63) / 64 * 64;
                HIP_TRY(hipHostMalloc((void **)&q.mb, 2 * q.mb_half));
                q.sc = reinterpret_cast<VolScalars *>(q.u8 + NV);
                q.st = reinterpret_cast<N4State *>(q.u8 + NV + sizeof(VolScalars) * sub);
                q.res.resize(sub);
            }
        } catch (...) {
            pipe_free(p);
            throw;
        }
        *out = p;
    })
}

// Host buffers the copy engines may read / write in place: hipHostRegister pins the caller's pages
// (the page tables only; measured ~0.4-0.5 TB/s on the box, scripts/dev/h2h_probe.py) and the DMA
// then runs at the link rate with no staging memcpy on a host thread.  A buffer that cannot be
// registered (e.g. pages already registered, or VH_PIPE_STAGE=1) goes through the pinned staging.
// First touch of a caller's output pages on several host threads (hipHostRegister would otherwise
// fault in and zero every untouched page on the calling thread: measured 3.8k vs 5.1k vol/s staged)
static void par_touch(void *dst, size_t bytes) {
    const size_t page = 4096, chunk = (size_t)64 << 20;
    const int want = (int)std::min<size_t>(2 * VH_COPY_THREADS, (bytes + chunk - 1) / chunk);
    auto touch = [=](size_t o, size_t n) {
        volatile char *q = (volatile char *)dst + o;
        for (size_t i = 0; i < n; i += page) q[i] = q[i];
    };
    if (want <= 1) {
        touch(0, bytes);
        return;
    }
    std::vector<std::thread> th;
    const size_t per = ((bytes + want - 1) / want + page - 1) / page * page;
    for (int i = 1; i < want; ++i) {
        const size_t o = per * i;
        if (o < bytes) th.emplace_back(touch, o, std::min(per, bytes - o));
    }
    touch(0, std::min(per, bytes));
    for (auto &t : th) t.join();
}

struct HostPin {
    void *p = nullptr;
    size_t n = 0;
    vh_pipe *owner = nullptr;   // the pipe whose pin budget this registration counts against
    HostPin() = default;
    HostPin(const HostPin &) = delete;
    HostPin &operator=(const HostPin &) = delete;
    bool pin(const void *ptr, size_t bytes, bool touch, vh_pipe *pp) {
        if (!ptr || !bytes || getenv("VH_PIPE_STAGE")) return false;
        // the budget first: a run over more than pin_cap bytes of caller memory stages the rest
        // rather than page-locking all of it (counted in staged_spans, vh_pipe_stats)
        const int64_t now = pp->pinned.fetch_add((int64_t)bytes) + (int64_t)bytes;
        if (now > pp->pin_cap) {
            pp->pinned.fetch_sub((int64_t)bytes);
            return false;
        }
        int64_t pk = pp->pinned_peak.load();
        while (now > pk && !pp->pinned_peak.compare_exchange_weak(pk, now)) {
        }
        if (touch) par_touch(const_cast<void *>(ptr), bytes);
        if (hipHostRegister(const_cast<void *>(ptr), bytes, hipHostRegisterDefault) != hipSuccess) {
            (void)hipGetLastError();
            pp->pinned.fetch_sub((int64_t)bytes);
            return false;
        }
        p = const_cast<void *>(ptr);
        n = bytes;
        owner = pp;
        return true;
    }
    ~HostPin() {
        if (p) {
            (void)hipHostUnregister(p);
            owner->pinned.fetch_sub((int64_t)n);
        }
    }
};

struct PipeAbort {   // a pipe slot stopped because another slot failed
    int slot = -1;
};

// One caller range of a pipe chunk.  Only its whole pages are pinned (and DMA'd in place): a page
// it shares with the neighbouring chunk or another buffer must never be registered twice or
// unregistered under another range's copy, so the head and tail fragments (< 1 page each) go
// through the slot's pinned staging at the same offsets.  A range that cannot be pinned is staged.
struct PipeSpan {
    char *p = nullptr;
    size_t n = 0, h = 0, t = 0;
    bool direct = false;
    HostPin pin;
    void plan(const void *ptr, size_t bytes, bool touch, vh_pipe *pp) {
        p = (char *)ptr;
        n = ptr ? bytes : 0;
        if (!n) return;
        const uintptr_t pg = 4096, s0 = (uintptr_t)p, e0 = s0 + n;
        const uintptr_t a = (s0 + pg - 1) / pg * pg, e = e0 / pg * pg;
        if (e <= a || e - a < ((size_t)1 << 20)) return;   // small: staged
        if (!pin.pin((void *)a, e - a, touch, pp)) {
            pp->staged_spans.fetch_add(1);
            return;
        }
        h = a - s0;
        t = e0 - e;
        direct = true;
    }
    void h2d(char *dst, char *stage, hipStream_t st) {
        if (!n) return;
        if (!direct) {
            par_memcpy(stage, p, n);
            HIP_TRY(hipMemcpyAsync(dst, stage, n, hipMemcpyHostToDevice, st));
            return;
        }
        if (h) {
            memcpy(stage, p, h);
            HIP_TRY(hipMemcpyAsync(dst, stage, h, hipMemcpyHostToDevice, st));
        }
        HIP_TRY(hipMemcpyAsync(dst + h, p + h, n - h - t, hipMemcpyHostToDevice, st));
        if (t) {
            memcpy(stage + n - t, p + n - t, t);
            HIP_TRY(hipMemcpyAsync(dst + n - t, stage + n - t, t, hipMemcpyHostToDevice, st));
        }
    }
    void d2h(const char *src, char *stage, hipStream_t st) {
        if (!n) return;
        if (!direct) {
            HIP_TRY(hipMemcpyAsync(stage, src, n, hipMemcpyDeviceToHost, st));
            return;
        }
        if (h) HIP_TRY(hipMemcpyAsync(stage, src, h, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(p + h, src + h, n - h - t, hipMemcpyDeviceToHost, st));
        if (t) HIP_TRY(hipMemcpyAsync(stage + n - t, src + n - t, t, hipMemcpyDeviceToHost, st));
    }
    void d2h_finish(const char *stage) {   // after the stream sync
        if (!n) return;
        if (!direct) {
            par_memcpy(p, stage, n);
            return;
        }
        if (h) memcpy(p, stage, h);
        if (t) memcpy(p + n - t, stage + n - t, t);
    }
};

int vh_pipe_run(vh_pipe *p, const float *hp, const uint8_t *mask, int64_t n, const vh_run_opts *opts,
                float *n4, uint8_t *defect, uint8_t *defect_border, uint8_t *lb, vh_vdp_result *res) {
    API_TRY(p->ctx, {
        if (!opts || !hp || !mask || n < 1) throw VhError{VH_ERR_ARG, "pipe: null input or n < 1"};
        const int64_t V = p->R * p->C * p->Z, sub = p->sub;
        const int64_t nchunk = (n + sub - 1) / sub;
        const int slots = (int)p->slot.size();
        HIP_TRY(hipSetDevice(p->ctx->device));
        std::vector<VhError> err(slots);
        std::vector<int> failed(slots, 0);
        // VH_PIPE_TRACE=1: per chunk, host times (ms from the start) of the input pin + H2D enqueue, the
        // pipeline enqueue, the output pin, the sync, and device times of H2D / compute / D2H ends (stderr)
        struct Mark {
            int64_t k;
            double h[5];
            hipEvent_t e[3];
        };
        const bool trace = getenv("VH_PIPE_TRACE") != nullptr;
        p->pinned_peak = 0;
        p->staged_spans = 0;
        std::vector<std::vector<std::unique_ptr<PipeSpan[]>>> keep(slots);
        std::vector<std::vector<Mark>> marks(slots);
        hipEvent_t ev0 = nullptr;
        const auto c0 = std::chrono::steady_clock::now();
        auto now_ms = [&] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - c0).count(); };
        if (trace) {
            HIP_TRY(hipEventCreate(&ev0));
            HIP_TRY(hipEventRecord(ev0, p->slot[0].b->stream));
        }
        auto mark_ev = [&](Mark &m, int i, hipStream_t st) {
            if (trace && hipEventCreate(&m.e[i]) == hipSuccess) (void)hipEventRecord(m.e[i], st);
        };
        // Chunk k's pipeline waits on the device for chunk k - lag's (lag = the chunks that fill the
        // CUs, VH_PIPE_LAG overrides; 0 = no ordering).  Without it the slots ran in lockstep: all
        // computing together, then all copying out / in together with the GPU idle (~60% of the
        // device rate, VH_PIPE_TRACE); with it the computes are staggered and each chunk's copies
        // overlap the next chunks' compute.  Enqueues happen in chunk order (host-side ticket).
        int cus = 256;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, p->ctx->device);
        int lag = (int)std::max<int64_t>(1, (cus + sub - 1) / sub);
        if (const char *e = getenv("VH_PIPE_LAG")) lag = atoi(e);
        lag = std::min(lag, slots);
        std::mutex tk_mu;
        std::condition_variable tk_cv;
        int64_t tk_next = 0;   // the chunk whose pipeline is enqueued next
        bool tk_abort = false;
        auto ticket_wait = [&](int64_t k) {
            std::unique_lock<std::mutex> lk(tk_mu);
            tk_cv.wait(lk, [&] { return tk_next == k || tk_abort; });
            if (tk_abort && tk_next != k) throw PipeAbort{};
        };
        auto ticket_pass = [&](int64_t k) {
            {
                std::lock_guard<std::mutex> lk(tk_mu);
                if (tk_next == k) tk_next = k + 1;
            }
            tk_cv.notify_all();
        };
        auto ticket_abort = [&] {
            {
                std::lock_guard<std::mutex> lk(tk_mu);
                tk_abort = true;
            }
            tk_cv.notify_all();
        };
        // Per slot, chunk by chunk: prep (host: pin the input pages, pack the mask bits) -> front
        // (enqueue H2D, the pipeline behind its ticket and lag event, the map packing) -> back
        // (first-touch + pin the n4 output pages, enqueue the D2Hs) -> sync -> finish (results,
        // fragments, map unpacking).  The next chunk's prep runs before this chunk's sync and its
        // front right after it, so the host work of finish overlaps the next chunk's H2D and
        // compute (its D2H is enqueued after finish: the staging it writes is free by then).
        struct Chunk {
            int64_t k = -1, v0 = 0, cnt = 0;
            size_t CV = 0;
            PipeSpan *sp = nullptr;
            bool mbits = false;
            uint8_t *mb = nullptr;
            Mark mk{};
        };
        const bool maps = defect || defect_border || lb;
        // A/B switches (VH_PIPE_H2D_ORDER, VH_PIPE_D2H_LATE: 0 / 1) for the copy ordering below
        auto env_flag = [](const char *name, bool dflt) {
            const char *e = getenv(name);
            return e ? atoi(e) != 0 : dflt;
        };
        // H2D order: 0 none, 1 device-side (the H2D waits on the previous chunk's H2D event),
        // 2 host-side (the enqueuing thread waits for that event first)
        const char *ho = getenv("VH_PIPE_H2D_ORDER");
        const int h2d_order = ho ? atoi(ho) : 2;
        // No copy is enqueued before what it depends on has finished (host-side waits): a copy
        // enqueued behind unfinished work waits on the DMA engine's queue and holds back every
        // later copy of that engine -- an H2D stuck behind another chunk's D2H that waits for a
        // kernel which waits for a CU (r4b trace: 30 ms stalls).  The D2H waits for the chunk's
        // packing kernel (not just the pipeline: the packing may itself wait for a free CU).
        const bool d2h_late = env_flag("VH_PIPE_D2H_LATE", true);
        auto work = [&](int s) {
            vh_pipe::Slot &q = p->slot[s];
            vh_batch *b = q.b;
            // mask bytes in (fallback); the D2H block: scalars / states, then the packed maps
            uint8_t *qm = q.u8, *qd = q.u8 + sub * V + q.scal;
            auto prep = [&](Chunk &c, int64_t k) {
                c.k = k;
                c.v0 = k * sub;
                c.cnt = std::min(sub, n - c.v0);
                c.CV = (size_t)c.cnt * V;
                c.mk = Mark{k, {now_ms(), 0, 0, 0, 0}, {nullptr, nullptr, nullptr}};
                // the spans' pins are released only after the whole run (hipHostUnregister waits
                // for the device: released per chunk, it lined every slot up behind the others)
                keep[s].emplace_back(new PipeSpan[3]);
                c.sp = keep[s].back().get();
                c.sp[0].plan(hp + c.v0 * V, sizeof(float) * c.CV, false, p);
                c.mb = q.mb + ((k / slots) & 1) * q.mb_half;   // bits double-buffered across chunks
                c.mbits = !getenv("VH_PIPE_STAGE") && par_pack_mask(mask + c.v0 * V, c.mb, c.CV);
                if (!c.mbits) c.sp[1].plan(mask + c.v0 * V, c.CV, false, p);
            };
            auto front = [&](Chunk &c) {
                const size_t CV = c.CV;
                // enqueues in chunk order; the H2Ds also run in chunk order (each waits for the one
                // before): at the start the first chunks' inputs get the whole link instead of
                // every slot's sharing it
                ticket_wait(c.k);
                try {
                if (h2d_order == 1 && c.k > 0)
                    HIP_TRY(hipStreamWaitEvent(b->stream, p->slot[(c.k - 1) % slots].h2d, 0));
                if (h2d_order == 2 && c.k > 0) HIP_TRY(hipEventSynchronize(p->slot[(c.k - 1) % slots].h2d));
                // the copies first (the event marks their end: the next chunk's H2D waits for it
                // on the host), then the kernels that consume them
                c.sp[0].h2d((char *)b->d_hp, (char *)q.hp, b->stream);
                if (c.mbits) HIP_TRY(hipMemcpyAsync(q.d_pack, c.mb, (CV + 7) / 8, hipMemcpyHostToDevice, b->stream));
                else c.sp[1].h2d((char *)b->d_mask, (char *)qm, b->stream);
                HIP_TRY(hipEventRecord(q.h2d, b->stream));
                if (c.mbits) {
                    k_unpack_mask<<<(unsigned)std::min<int64_t>(4096, ((int64_t)(CV + 7) / 8 + 255) / 256), 256, 0,
                                    b->stream>>>(q.d_pack, b->d_mask, (int64_t)CV);
                    HIP_TRY(hipGetLastError());
                }
                if (c.cnt < sub) {   // ragged tail: repeat the last study (a kernel, not DMA copies)
                    k_repeat_last<<<(unsigned)std::min<int64_t>(4096, (sub - c.cnt) * (V / 4 + 255) / 256 + 1), 256, 0,
                                    b->stream>>>(b->d_hp, b->d_mask, V, c.cnt, sub);
                    HIP_TRY(hipGetLastError());
                }
                mark_ev(c.mk, 0, b->stream);
                c.mk.h[1] = now_ms();
                if (lag > 0 && c.k >= lag)
                    HIP_TRY(hipStreamWaitEvent(b->stream, p->slot[(c.k - lag) % slots].done, 0));
                batch_run(b, *opts, opts->do_n4 ? 0 : 1);
                HIP_TRY(hipEventRecord(q.done, b->stream));
                } catch (...) {
                    ticket_pass(c.k);
                    throw;
                }
                ticket_pass(c.k);
                mark_ev(c.mk, 1, b->stream);
                c.mk.h[2] = now_ms();
                if (maps || res) {   // scalars + the three maps packed into one byte per voxel
                    const int64_t cvm = maps ? (int64_t)CV : 0;
                    const int64_t scw = (int64_t)(sizeof(VolScalars) * sub / 4);
                    const int64_t stw = opts->do_n4 ? (int64_t)(sizeof(N4State) * sub / 4) : 0;
                    k_pack_maps<<<(unsigned)std::min<int64_t>(4096, (cvm / 16 + 255) / 256 + 1), 256, 0,
                                  b->stream>>>(b->d_defect, b->d_border, b->d_lb, q.d_pack + q.scal, cvm,
                                               reinterpret_cast<const uint32_t *>(b->d_sc), scw,
                                               reinterpret_cast<const uint32_t *>(b->d_st), stw,
                                               reinterpret_cast<uint32_t *>(q.d_pack));
                    HIP_TRY(hipGetLastError());
                }
                HIP_TRY(hipEventRecord(q.packed, b->stream));
            };
            auto back_pin = [&](Chunk &c) {   // while the chunk computes: first touch + pin of its output pages
                c.sp[2].plan(n4 ? n4 + c.v0 * V : nullptr, sizeof(float) * c.CV, true, p);
            };
            auto back = [&](Chunk &c) {
                const float *dn4 = opts->do_n4 ? b->d_n4 : b->d_hp;
                c.sp[2].d2h((const char *)dn4, (char *)q.n4, b->stream);
                if (maps || res)   // one D2H: the scalars / states block, then the packed maps
                    HIP_TRY(hipMemcpyAsync(q.u8 + sub * V, q.d_pack, q.scal + (maps ? c.CV : 0),
                                           hipMemcpyDeviceToHost, b->stream));
                mark_ev(c.mk, 2, b->stream);
                c.mk.h[3] = now_ms();
            };
            auto finish = [&](Chunk &c) {
                if (res) {
                    fill_results_from(b, q.sc, q.st, q.res.data());
                    memcpy(res + c.v0, q.res.data(), sizeof(vh_vdp_result) * c.cnt);
                }
                c.sp[2].d2h_finish((const char *)q.n4);
                if (maps)
                    par_unpack_maps(qd, defect ? defect + c.v0 * V : nullptr,
                                    defect_border ? defect_border + c.v0 * V : nullptr,
                                    lb ? lb + c.v0 * V : nullptr, c.CV);
                if (trace) marks[s].push_back(c.mk);
            };
            try {
                HIP_TRY(hipSetDevice(p->ctx->device));
                Chunk cur, nxt;
                if (s < nchunk) {
                    try {
                        prep(cur, s);
                        front(cur);
                        for (;;) {
                            const int64_t kn = cur.k + slots;
                            if (kn < nchunk) prep(nxt, kn);   // host work while the GPU has cur
                            back_pin(cur);
                            // VH_PIPE_D2H_LATE=1 enqueues the D2Hs only once the compute has
                            // finished (A/B: neutral to -2 % on the boxes measured, r3q3; off)
                            if (d2h_late) HIP_TRY(hipEventSynchronize(q.packed));
                            back(cur);
                            HIP_TRY(hipStreamSynchronize(b->stream));
                            cur.mk.h[4] = now_ms();
                            if (kn < nchunk) front(nxt);      // the next chunk's H2D + compute first
                            finish(cur);                      // then this chunk's host side
                            if (kn >= nchunk) break;
                            cur = nxt;
                        }
                    } catch (...) {   // no copy may still touch a pinned range when it is released
                        (void)hipStreamSynchronize(b->stream);
                        throw;
                    }
                }
            } catch (const PipeAbort &) {   // another slot's failure is the one reported
                failed[s] = 2;
            } catch (const VhError &e) {
                err[s] = e;
                failed[s] = 1;
                ticket_abort();
            } catch (const std::exception &e) {
                err[s] = VhError{VH_ERR_HIP, e.what()};
                failed[s] = 1;
                ticket_abort();
            }
        };
        std::vector<std::thread> th;
        for (int s = 1; s < slots; ++s) th.emplace_back(work, s);
        work(0);
        for (auto &t : th) t.join();
        for (int s = 0; s < slots; ++s)   // no copy may still touch a pinned buffer when it is released
            (void)hipStreamSynchronize(p->slot[s].b->stream);
        keep.clear();
        if (trace) {
            fprintf(stderr, "pipe_trace total_ms %.2f\n", now_ms());
            for (int s = 0; s < slots; ++s)
                for (Mark &m : marks[s]) {
                    float d[3] = {-1, -1, -1};
                    for (int i = 0; i < 3; ++i)
                        if (m.e[i]) {
                            (void)hipEventElapsedTime(&d[i], ev0, m.e[i]);
                            (void)hipEventDestroy(m.e[i]);
                        }
                    fprintf(stderr, "pipe_trace slot %d chunk %lld host %.2f %.2f %.2f %.2f %.2f dev %.2f %.2f %.2f\n", s,
                            (long long)m.k, m.h[0], m.h[1], m.h[2], m.h[3], m.h[4], d[0], d[1], d[2]);
                }
            (void)hipEventDestroy(ev0);
        }
        for (int s = 0; s < slots; ++s)
            if (failed[s] == 1) throw err[s];
    })
}

int vh_pipe_stats(vh_pipe *p, int64_t *pinned_peak_bytes, int64_t *staged_spans) {
    if (!p) return VH_ERR_ARG;
    if (pinned_peak_bytes) *pinned_peak_bytes = p->pinned_peak.load();
    if (staged_spans) *staged_spans = p->staged_spans.load();
    return VH_OK;
}

int vh_link_probe(vh_ctx *ctx, int64_t bytes, double out_gbps[3]) {
    API_TRY(ctx, {
        std::lock_guard<std::mutex> lock(ctx->mu);
        if (!out_gbps || bytes <= 0) throw VhError{VH_ERR_ARG, "link probe: bad arguments"};
        HIP_TRY(hipSetDevice(ctx->device));
        void *h_in = nullptr, *h_out = nullptr, *d_in = nullptr, *d_out = nullptr;
        hipStream_t s[2] = {nullptr, nullptr};
        hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
        auto release = [&]() {
            for (auto e : ev) if (e) (void)hipEventDestroy(e);
            for (auto x : s) if (x) (void)hipStreamDestroy(x);
            if (h_in) (void)hipHostFree(h_in);
            if (h_out) (void)hipHostFree(h_out);
            if (d_in) (void)hipFree(d_in);
            if (d_out) (void)hipFree(d_out);
        };
        try {
            HIP_TRY(hipHostMalloc(&h_in, (size_t)bytes, hipHostMallocDefault));
            HIP_TRY(hipHostMalloc(&h_out, (size_t)bytes, hipHostMallocDefault));
            HIP_TRY(hipMalloc(&d_in, (size_t)bytes));
            HIP_TRY(hipMalloc(&d_out, (size_t)bytes));
            std::memset(h_in, 1, (size_t)bytes);
            std::memset(h_out, 2, (size_t)bytes);
            for (auto &x : s) HIP_TRY(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
            for (auto &e : ev) HIP_TRY(hipEventCreate(&e));
            auto h2d = [&]() { HIP_TRY(hipMemcpyAsync(d_in, h_in, (size_t)bytes, hipMemcpyHostToDevice, s[0])); };
            auto d2h = [&]() { HIP_TRY(hipMemcpyAsync(h_out, d_out, (size_t)bytes, hipMemcpyDeviceToHost, s[1])); };
            auto best = [&](int mode) {   // 0 H2D, 1 D2H, 2 both: wall time of the copies, best of 3
                double b = 1e30;
                for (int r = 0; r < 4; ++r) {   // the first pass warms up
                    HIP_TRY(hipDeviceSynchronize());
                    const auto t0 = std::chrono::steady_clock::now();
                    if (mode != 1) h2d();
                    if (mode != 0) d2h();
                    HIP_TRY(hipStreamSynchronize(s[0]));
                    HIP_TRY(hipStreamSynchronize(s[1]));
                    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                    if (r > 0) b = std::min(b, dt);
                }
                return b;
            };
            const double t1 = best(0), t2 = best(1), t3 = best(2);
            out_gbps[0] = (double)bytes / t1 / 1e9;
            out_gbps[1] = (double)bytes / t2 / 1e9;
            out_gbps[2] = 2.0 * (double)bytes / t3 / 1e9;
        } catch (...) {
            release();
            throw;
        }
        release();
    })
}

int vh_host_alloc(vh_ctx *ctx, int64_t bytes, void **out) {
    if (out) *out = nullptr;
    API_TRY(ctx, {
        if (!out || bytes <= 0) throw VhError{VH_ERR_ARG, "host alloc: bad arguments"};
        HIP_TRY(hipSetDevice(ctx->device));
        HIP_TRY(hipHostMalloc(out, (size_t)bytes, hipHostMallocDefault));
        void *dp = nullptr;
        if (hipHostGetDevicePointer(&dp, *out, 0) != hipSuccess || !dp) {
            (void)hipGetLastError();
            dp = nullptr;
        }
        if (dp) {
            std::lock_guard<std::mutex> lock(g_host_mu);
            g_host[(uintptr_t)*out] = {(size_t)bytes, dp};
        }
    })
}

int vh_host_free(void *p) {
    if (p) {
        {
            std::lock_guard<std::mutex> lock(g_host_mu);
            g_host.erase((uintptr_t)p);
        }
        (void)hipHostFree(p);
    }
    return VH_OK;
}

int vh_pipe_destroy(vh_pipe *p) {
    if (p) {
        (void)hipSetDevice(p->ctx->device);
        pipe_free(p);
    }
    return VH_OK;
}

int vh_comm_unique_id(uint8_t id[VH_COMM_ID_BYTES]) {
    static_assert(sizeof(ncclUniqueId) <= VH_COMM_ID_BYTES, "nccl id size");
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return VH_ERR_RCCL;
    memcpy(id, &u, sizeof u);
    return VH_OK;
}

int vh_comm_init(vh_ctx *ctx, int nranks, int rank, const uint8_t id[VH_COMM_ID_BYTES]) {
    API_TRY(ctx, {
        HIP_TRY(hipSetDevice(ctx->device));
        ncclUniqueId u;
        memcpy(&u, id, sizeof u);
        ncclComm_t comm;
        ncclResult_t r = ncclCommInitRank(&comm, nranks, u, rank);
        if (r != ncclSuccess) throw VhError{VH_ERR_RCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(r)};
        ctx->comm = comm;
        ctx->nranks = nranks;
        ctx->rank = rank;
    })
}

int vh_batch_cohort_allreduce(vh_batch *b) {
    API_TRY(b->ctx, {
        vh_ctx *c = b->ctx;
        if (!c->comm) throw VhError{VH_ERR_ARG, "vh_comm_init has not been called"};
        HIP_TRY(hipSetDevice(c->device));
        if (!c->comm_st) HIP_TRY(hipStreamCreateWithFlags(&c->comm_st, hipStreamNonBlocking));
        if (!b->ev_cpre) HIP_TRY(hipEventCreateWithFlags(&b->ev_cpre, hipEventDisableTiming));
        if (!b->ev_cpost) HIP_TRY(hipEventCreateWithFlags(&b->ev_cpost, hipEventDisableTiming));
        // after this batch's work, on the communicator's stream (program order across batches),
        // and the batch's later work after it
        HIP_TRY(hipEventRecord(b->ev_cpre, b->stream));
        HIP_TRY(hipStreamWaitEvent(c->comm_st, b->ev_cpre, 0));
        ncclResult_t r = ncclAllReduce(b->d_cohort, b->d_cohort, VH_COHORT_BINS, ncclUint64, ncclSum,
                                       (ncclComm_t)c->comm, c->comm_st);
        if (r != ncclSuccess) throw VhError{VH_ERR_RCCL, std::string("ncclAllReduce: ") + ncclGetErrorString(r)};
        HIP_TRY(hipEventRecord(b->ev_cpost, c->comm_st));
        HIP_TRY(hipStreamWaitEvent(b->stream, b->ev_cpost, 0));
    })
}

int vh_comm_info(vh_ctx *ctx, int *nranks, int *rank) {
    API_TRY(ctx, {
        if (!nranks || !rank) throw VhError{VH_ERR_ARG, "null out"};
        if (!ctx->comm) throw VhError{VH_ERR_ARG, "vh_comm_init has not been called"};
        int n = 0, r = -1;
        ncclResult_t e = ncclCommCount((ncclComm_t)ctx->comm, &n);
        if (e != ncclSuccess) throw VhError{VH_ERR_RCCL, std::string("ncclCommCount: ") + ncclGetErrorString(e)};
        e = ncclCommUserRank((ncclComm_t)ctx->comm, &r);
        if (e != ncclSuccess) throw VhError{VH_ERR_RCCL, std::string("ncclCommUserRank: ") + ncclGetErrorString(e)};
        *nranks = n;
        *rank = r;
    })
}

int vh_comm_destroy(vh_ctx *ctx) {
    if (ctx && ctx->comm) {
        ncclCommDestroy((ncclComm_t)ctx->comm);
        ctx->comm = nullptr;
    }
    return VH_OK;
}

}  // extern "C"
