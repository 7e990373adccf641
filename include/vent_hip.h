/* vent_hip.h -- C-ABI of libventhip.so, the MI355X (gfx950) implementation of the Vent_Analysis
 * voxel hot path (N4 -> mean-anchored / linear-binning / k-means VDP -> defect morphology -> CI).
 *
 * Plain C types only (no torch, no HIP types).  Every function returns an int status (VH_OK = 0)
 * and never throws across the boundary; vh_last_error() gives the message of the last failure on
 * a context.  Host buffers are caller-allocated and C-contiguous in numpy's (rows, cols, slices)
 * order (slice axis fastest, as Vent_Analysis.openSingleDICOM produces, Vent_Analysis.py:179);
 * device buffers are owned by the library.  A context is bound to one GPU; each batch owns its HIP
 * stream.  The host-buffer entry points (vh_n4 ... vh_ci) share a per-context scratch batch behind a
 * per-context mutex, so a context may be used from several host threads; batches are independent.
 *
 * Reference interface each entry point replaces (file:line in thomenr/Vent_Analysis):
 *   vh_n4        Vent_Analysis.N4_bias_correction            Vent_Analysis.py:316-334
 *   vh_snr       Vent_Analysis.calculate_SNR                 Vent_Analysis.py:337-357
 *   vh_border    Vent_Analysis.calculateBorder               Vent_Analysis.py:225-231
 *   vh_vdp       Vent_Analysis.calculate_VDP (post-N4 part)  Vent_Analysis.py:239-263
 *   vh_ci        CI.calculate_CI + Vent_Analysis.calculate_CI CI.py:107-145, Vent_Analysis.py:265-271
 *   vh_ci_table_* / vh_ci_tab  the same with the sphere table resident in HBM (CI.getSpherePix's
 *                cached table, CI.py:33-63, uploaded once)
 *   vh_overlay   Vent_Analysis.exportDICOM (pixel data)       Vent_Analysis.py:381-428
 *   vh_montage   Vent_Analysis.screenShot (montage array)     Vent_Analysis.py:458-520
 *   vh_recon     Vent_Analysis.process_RAW (k-space -> image) Vent_Analysis.py:537-540
 *   vh_batch_*   the same pipeline over a device-resident batch of studies (build-defined)
 *   vh_pipe_*    the batch pipeline fed from host memory with overlapped transfers (build-defined)
 *   vh_comm_*    cohort histogram all-reduce over RCCL (build-defined, BASELINE config 4)
 */
#ifndef VENT_HIP_H
#define VENT_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VH_ABI_VERSION 8

/* status codes */
#define VH_OK 0
#define VH_ERR_ARG 1          /* bad argument (maps to ValueError/TypeError in the shim) */
#define VH_ERR_HIP 2          /* HIP runtime failure */
#define VH_ERR_NOMEM 3        /* device allocation failed */
#define VH_ERR_MAXRADIUS 4    /* CI: sphere reached the table's last radius (CI.py:101-103, ValueError) */
#define VH_ERR_EMPTY 5        /* empty mask / defect list (Vent_Analysis.py:270 IndexError) */
#define VH_ERR_RCCL 6         /* RCCL failure */
#define VH_ERR_NODEV 7        /* no GPU visible */
#define VH_ERR_INDEX 8        /* index out of range (maps to IndexError): screenShot's parula lookup */

typedef struct vh_ctx vh_ctx;
typedef struct vh_batch vh_batch;
typedef struct vh_ci_table vh_ci_table;

/* N4 parameters; vh_n4_default_params() fills the SimpleITK 2.3.1 defaults the reference runs with
 * (Vent_Analysis.py:330: no setter is called).  ncp is given per numpy axis (rows, cols, slices). */
typedef struct {
    int32_t n_levels;        /* 4  = len(MaximumNumberOfIterations) */
    int32_t max_iters[8];    /* 50, 50, 50, 50 */
    float conv_threshold;    /* 0.001 */
    int32_t ncp[3];          /* 4, 4, 4 control points per axis at level 0 */
    int32_t spline_order;    /* 3 (only 3 supported) */
    int32_t n_bins;          /* 200 histogram bins (<= 256) */
    float wiener_noise;      /* 0.01 */
    float fwhm;              /* 0.15 bias-field FWHM */
    int32_t conv_mode;       /* 0 (default): ITK's convergence measure -- the float (RealType) Welford
                                recurrence over the masked voxels in raster order, whose rounding
                                drift sets SimpleITK's iteration counts; a serial recurrence.
                                1: the exact coefficient of variation it approximates (double,
                                order-free; faster, but stops at different iterations than
                                SimpleITK -- see DESIGN.md §6) */
} vh_n4_params;

/* Per-volume scalars of calculate_VDP / calculate_CI (metadata keys of Vent_Analysis.py:78-103). */
typedef struct {
    double vdp;              /* metadata['VDP']        100*sum(defect)/sum(mask)            :251 */
    double vdp_lb;           /* metadata['VDP_lb']     100*count(LB in {1,2})/sum(mask)     :257 */
    double vdp_km;           /* metadata['VDP_km']     build-defined 1-D k-means (k=4)       :259-261 */
    double defect_volume;    /* metadata['DefectVolume'] litres                              :252 */
    double lung_volume;      /* metadata['LungVolume']   litres                              :166 */
    double km_centres[4];
    double snr;              /* metadata['SNR'] (double accumulation; the shim casts to HPvent's
                                float dtype like numpy)                                      :241 */
    float mean_anchor;       /* np.mean(sorted masked N4) (float32, numpy reduction order)  :246 */
    float p99;               /* sorted[int(0.99 n)]                                          :255 */
    int64_t n_mask;          /* voxels with mask > 0 */
    int64_t n_defect;
    int64_t n_lb12;
    int64_t n_km0;
    int32_t n4_iters[8];     /* N4 iterations executed per level (0 when N4 skipped) */
    float n4_conv[8];        /* last convergence measure per level */
} vh_vdp_result;

/* Options for vh_batch_run. */
typedef struct {
    int32_t do_n4;           /* 1: N4 on HPvent (calculate_VDP);  0: N4 := identity (HPvent) */
    vh_n4_params n4;
    float thresh;            /* mean-anchored threshold (calculate_VDP thresh=0.6) */
    int32_t do_snr;
    int32_t do_kmeans;
    int32_t do_cohort;       /* accumulate the cohort histogram (1024 u64 bins, [0,1.5) of p99-normalised masked N4) */
    int32_t profile;         /* 1: time kernel classes with HIP events (vh_batch_kernel_time) */
    double vox[3];           /* voxel size (mm) for the volume scalars */
    int32_t n4_subbatch;     /* volumes per N4 sub-batch (0 = whole batch); smaller sub-batches
                                keep an iteration's working set in the 256 MiB Infinity Cache */
    int32_t morph3d;         /* build-defined 3-D morphology (BASELINE config 5): 3x3x3 majority
                                (>= 14 of 27, zero padded) and np.gradient != 0 along all three
                                axes, instead of the reference's per-slice medfilt2d / 2-D border */
    int32_t n4_mode;         /* N4 driver: 0 auto, 1 per-iteration sweeps over the batch (any size),
                                2 volume-resident (one workgroup per study, the whole iteration
                                loop in one launch; studies whose N4 state fits in LDS),
                                3 grid form (each study over G cooperating workgroups, one
                                launch per study; auto picks it for a batch of one study) */
} vh_run_opts;

#define VH_COHORT_BINS 1024

/* ---- library / context ---------------------------------------------------------------------- */
int vh_abi_version(void);
const char *vh_status_string(int status);
int vh_device_count(int *n);
void vh_n4_default_params(vh_n4_params *p);
void vh_default_run_opts(vh_run_opts *o);
int vh_create(int device, vh_ctx **out);
int vh_destroy(vh_ctx *ctx);
const char *vh_last_error(const vh_ctx *ctx);
int vh_synchronize(vh_ctx *ctx);

/* ---- host-buffer entry points (one call = upload, compute, download) --------------------------
 * hp: float32, mask: uint8 0/1, shapes [batch][R][C][Z]. */
int vh_n4(vh_ctx *ctx, const float *hp, const uint8_t *mask, int64_t R, int64_t C, int64_t Z,
          int64_t batch, const vh_n4_params *prm, float *out, int32_t *iters /* [batch][n_levels] */,
          float *conv /* [batch][n_levels], nullable */);
int vh_border(vh_ctx *ctx, const uint8_t *a, int64_t R, int64_t C, int64_t Z, int64_t batch,
              uint8_t *border);
int vh_snr(vh_ctx *ctx, const float *hp, const uint8_t *mask, int64_t R, int64_t C, int64_t Z,
           int64_t batch, double *snr);
/* calculate_VDP after N4.  hp may be NULL (no SNR).  Outputs: defect / defect_border / lb uint8
 * volumes (any may be NULL), res[batch]. */
int vh_vdp(vh_ctx *ctx, const float *hp, const float *n4, const uint8_t *mask, int64_t R,
           int64_t C, int64_t Z, int64_t batch, float thresh, const double vox[3],
           uint8_t *defect, uint8_t *defect_border, uint8_t *lb, vh_vdp_result *res);
/* Cluster index map.  The sphere table comes from the host (reference-identical rows; see
 * vent_analysis_amd/sphere.py): offs int16 [rows][3] (dx,dy,dz), dup uint8 [rows], bounds int32
 * [nb] prefix lengths, radii float64 [nb] (= r[b-1]).  Outputs: ci_array float64 volume,
 * ci_scalar[batch] (95th-percentile CV, Vent_Analysis.py:268-270), shell int32 volume (nullable). */
int vh_ci(vh_ctx *ctx, const uint8_t *defect, int64_t R, int64_t C, int64_t Z, int64_t batch,
          const int16_t *offs, const uint8_t *dup, int64_t rows, const int32_t *bounds,
          const double *radii, int64_t nb, double minvox, double *ci_array, double *ci_scalar,
          int32_t *shell);
/* The sphere table uploaded once for volumes of R rows and C columns (the px2vec stride of
 * CI.py:65-68): the same arrays as vh_ci; it stays in HBM until vh_ci_table_destroy.  vh_ci_tab is
 * vh_ci with such a table (ci_array and shell nullable): no per-call table work or upload. */
int vh_ci_table_create(vh_ctx *ctx, int64_t R, int64_t C, const int16_t *offs, const uint8_t *dup,
                       int64_t rows, const int32_t *bounds, const double *radii, int64_t nb,
                       vh_ci_table **out);
int vh_ci_table_destroy(vh_ci_table *t);
int vh_ci_tab(vh_ctx *ctx, const uint8_t *defect, int64_t R, int64_t C, int64_t Z, int64_t batch,
              const vh_ci_table *t, double minvox, double *ci_array, double *ci_scalar, int32_t *shell);

/* ---- device-resident batch pipeline ---------------------------------------------------------- */
int vh_batch_create(vh_ctx *ctx, int64_t R, int64_t C, int64_t Z, int64_t batch, vh_batch **out);
int vh_batch_destroy(vh_batch *b);
int vh_batch_upload(vh_batch *b, const float *hp, const uint8_t *mask);
int vh_batch_run(vh_batch *b, const vh_run_opts *opts);      /* enqueue; returns before the GPU ends */
int vh_batch_sync(vh_batch *b);
int vh_batch_download(vh_batch *b, float *n4, uint8_t *defect, uint8_t *defect_border, uint8_t *lb,
                      vh_vdp_result *res /* [batch] */);
int vh_batch_cohort_hist(vh_batch *b, uint64_t *hist /* [VH_COHORT_BINS] */);
/* Kernel-class timing from HIP events on the context stream (opts.profile = 1).  name is one of
 * the classes listed by vh_batch_kernel_names (';'-separated). */
const char *vh_batch_kernel_names(void);
/* Discard accumulated kernel timings (timings accumulate over vh_batch_run calls). */
int vh_batch_reset_timers(vh_batch *b);
int vh_batch_kernel_time(vh_batch *b, const char *name, double *total_ms, int64_t *launches,
                         double *bytes_per_launch);

/* Kernel-class timing of the host-buffer entry points (vh_ci, vh_vdp, ...): on = 1 makes them time
 * their kernel classes with HIP events on the context's scratch batch (timings accumulate; setting
 * the switch discards them); vh_ctx_kernel_time reads them like vh_batch_kernel_time. */
int vh_ctx_profile(vh_ctx *ctx, int on);
int vh_ctx_kernel_time(vh_ctx *ctx, const char *name, double *total_ms, int64_t *launches);

/* Per-study wall time (microseconds, device wall clock) of the last vh_batch_run's volume-resident
 * N4 kernel (one workgroup per study: the slowest study bounds the launch); zeros when that run did
 * not use it.  us[batch]. */
int vh_batch_study_times(vh_batch *b, double *us);

/* ---- rendering after the hot path ---------------------------------- */
/* exportDICOM's pixel data (Vent_Analysis.py:387-393): BW = uint8(normalize(|N4HPvent|) * 255) in
 * float32, RGB = (BW*(defect==0) + 255*(defect==1), BW*(defect==0), BW*(defect==0)).  n4 float32
 * and defect uint8 volumes [batch][R][C][Z]; rgb uint8 [batch][Z][R][C][3] -- the frame order of
 * np.transpose(RGB, (2,0,1,3)) (:393) and, frame by frame, the PACS branch's RGB[:,:,i,:] (:411). */
int vh_overlay(vh_ctx *ctx, const float *n4, const uint8_t *defect, int64_t R, int64_t C, int64_t Z,
               int64_t batch, uint8_t *rgb);
/* screenShot's montage array (Vent_Analysis.py:467-495) before the text overlay: the 7 x ns grid
 * (blank, blank, proton, HPvent, N4 + mask border, N4 + defects, N4 + parula CI) over the crop
 * crop = {r0, nr, c0, nc, s0, ns} (cropToData(mask, border=5), :430-456), as uint8(IMAGE * 255)
 * [7 nr][ns nc][3].  proton / hp are float32 (is64 = 0) or float64 (is64 = 1); ci float64 or NULL
 * (the reference's blank CI panel); parula float64 [prow][3].  A CI colour index outside the table
 * returns VH_ERR_INDEX (IndexError), a NaN CI VH_ERR_ARG (ValueError). */
int vh_montage(vh_ctx *ctx, int64_t R, int64_t C, int64_t Z, const void *proton, int proton_is64,
               const void *hp, int hp_is64, const float *n4, const uint8_t *mask_border,
               const uint8_t *defect, const double *ci, const double *parula, int64_t prow,
               const int64_t crop[6], uint8_t *image);

/* ---- TWIX raw reconstruction --------------------------------------- */
/* process_RAW's image from raw k-space (Vent_Analysis.py:537-540): for every slice k,
 * fftshift(fft2(fftshift(K[:, :, k]))) in complex128, then np.transpose(., (1, 0, 2))[:, ::-1, :].
 * k: complex128 as interleaved (re, im) doubles, C order [n0][n1][nz]; out: complex128 [n1][n0][nz].
 * (The twix file parse, mapvbvd at :532-536, stays on the host.)  1 <= n0, n1 <= 5120. */
int vh_recon(vh_ctx *ctx, const double *k, int64_t n0, int64_t n1, int64_t nz, double *out);

/* ---- host-to-host pipeline ------------------------------------------------------------------ */
/* Streams n host-resident studies through `slots` device batches of `sub` volumes each (one HIP
 * stream and one host thread per slot, pinned staging per slot): while one slot computes, the
 * others upload their next sub-batch or download their last results.  Outputs are host arrays of
 * n volumes (any may be NULL); res[n].  A ragged last sub-batch is padded with copies of its last
 * study (results discarded).  Build-defined: SURVEY section 8(e) partitioning on one GPU. */
typedef struct vh_pipe vh_pipe;
int vh_pipe_create(vh_ctx *ctx, int64_t R, int64_t C, int64_t Z, int64_t sub, int slots,
                   vh_pipe **out);
int vh_pipe_run(vh_pipe *p, const float *hp, const uint8_t *mask, int64_t n, const vh_run_opts *opts,
                float *n4, uint8_t *defect, uint8_t *defect_border, uint8_t *lb,
                vh_vdp_result *res);
int vh_pipe_destroy(vh_pipe *p);
/* The last vh_pipe_run's peak of caller memory pinned in place (bytes) and the caller ranges that
 * went through the pinned staging instead (not registrable, or past the VH_PIPE_PIN_CAP budget,
 * default 32 GiB per node divided by LOCAL_WORLD_SIZE: a long cohort run never page-locks more than
 * that at once). */
int vh_pipe_stats(vh_pipe *p, int64_t *pinned_peak_bytes, int64_t *staged_spans);
/* This GPU's PCIe link with pinned host memory (bench.py's host-to-host bound): bytes copied H2D
 * alone, D2H alone and both at once on two streams, best of 3; out_gbps = {h2d, d2h, both}. */
int vh_link_probe(vh_ctx *ctx, int64_t bytes, double out_gbps[3]);
/* Page-locked host memory on the context's device (hipHostMalloc) for result arrays the caller
 * reuses: a D2H into it runs at the link rate with no runtime staging.  vh_host_free takes any
 * pointer vh_host_alloc returned (also after vh_destroy). */
int vh_host_alloc(vh_ctx *ctx, int64_t bytes, void **out);
int vh_host_free(void *p);

/* ---- multi-GPU (RCCL over xGMI) -------------------------------------------------------------- */
#define VH_COMM_ID_BYTES 128
int vh_comm_unique_id(uint8_t id[VH_COMM_ID_BYTES]);
int vh_comm_init(vh_ctx *ctx, int nranks, int rank, const uint8_t id[VH_COMM_ID_BYTES]);
/* Sum the batch's device cohort histogram over all ranks of the context's communicator. */
int vh_batch_cohort_allreduce(vh_batch *b);
/* The communicator as RCCL sees it: its rank count (ncclCommCount) and this context's rank
 * (ncclCommUserRank).  bench.py's N > 1 line reports both (ABI 8). */
int vh_comm_info(vh_ctx *ctx, int *nranks, int *rank);
int vh_comm_destroy(vh_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif /* VENT_HIP_H */
