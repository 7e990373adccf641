// export.hip -- the rendering steps that follow the hot path, on device.
//
//  * exportDICOM (Vent_Analysis.py:381-397): BW = uint8(normalize(|N4HPvent|) * 255) in float32,
//    RGB = (BW*(defect==0) + 255*(defect==1), BW*(defect==0), BW*(defect==0)).  Written
//    slice-major [Z][R][C][3]: the frame order of np.transpose(RGB, (2,0,1,3)) (:393) and, frame
//    by frame, the RGB[:,:,i,:] images of the PACS branch (:410-411).
//  * screenShot (Vent_Analysis.py:458-500): the 7-row montage (blank, blank, proton, HPvent,
//    N4 + mask border, N4 + defects, N4 + parula CI) over the mask's bounding box, each panel
//    normalised over the crop, stored as uint8(IMAGE * 255) with IMAGE in float64.
//
// Both are per-voxel maps: HBM-bound streaming (overlay: 4 B N4 + 1 B defect in, 3 B out per
// voxel) with the volume min/max as an order-free integer reduction (float bits of |x| are
// monotone), so every output byte is bit-identical to numpy's.
#include "vh_internal.h"

#define OV_COLS 64     // columns per overlay block (one wave's worth of output words per slice)
#define OV_ZC 64       // slices per overlay block
#define OV_WORDS (OV_COLS * 3 / 4)

// numpy's float -> uint8 cast on x86-64 goes through int32 (NaN / out of range -> INT_MIN) and
// keeps the low byte: 300 -> 44, -1 -> 255, 1e10 -> 0 (checked against numpy 2.2).
__device__ __forceinline__ uint8_t np_u8(double v) {
    if (!(v > -2147483649.0 && v < 2147483648.0)) return 0;
    return (uint8_t)(uint32_t)(int32_t)v;
}

// sortable keys of doubles (monotone in the value for non-NaN inputs)
__device__ __forceinline__ uint64_t d2key(double d) {
    uint64_t u = (uint64_t)__double_as_longlong(d);
    return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double key2d(uint64_t k) {
    uint64_t u = (k & 0x8000000000000000ull) ? (k & 0x7fffffffffffffffull) : ~k;
    return __longlong_as_double((long long)u);
}

// ---- exportDICOM overlay ----------------------------------------------------------------------
__global__ void k_absmm_init(uint32_t *mm, int64_t nb) {
    int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v < nb) {
        mm[2 * v] = 0xffffffffu;
        mm[2 * v + 1] = 0u;
    }
}

// Per-volume min / max of |x| as float bits.  |NaN| sorts above +inf, so hi > 0x7f800000 flags a
// NaN (numpy's min and max then both return NaN).
__global__ __launch_bounds__(VH_TPB) void k_absminmax(const float *__restrict__ x, int64_t V,
                                                      uint32_t *__restrict__ mm) {
    const float *p = x + (int64_t)blockIdx.y * V;
    uint32_t lo = 0xffffffffu, hi = 0u;
    const int64_t stride = (int64_t)gridDim.x * VH_TPB;
    const int64_t t0 = (int64_t)blockIdx.x * VH_TPB + threadIdx.x;
    if ((V & 3) == 0) {
        const float4 *p4 = reinterpret_cast<const float4 *>(p);
        const int64_t n4 = V >> 2;
        for (int64_t i = t0; i < n4; i += stride) {
            const float4 v = p4[i];
            const uint32_t a = __float_as_uint(v.x) & 0x7fffffffu, b = __float_as_uint(v.y) & 0x7fffffffu;
            const uint32_t c = __float_as_uint(v.z) & 0x7fffffffu, d = __float_as_uint(v.w) & 0x7fffffffu;
            lo = min(lo, min(min(a, b), min(c, d)));
            hi = max(hi, max(max(a, b), max(c, d)));
        }
    } else {
        for (int64_t i = t0; i < V; i += stride) {
            const uint32_t a = __float_as_uint(p[i]) & 0x7fffffffu;
            lo = min(lo, a);
            hi = max(hi, a);
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        lo = min(lo, (uint32_t)__shfl_xor((int)lo, o));
        hi = max(hi, (uint32_t)__shfl_xor((int)hi, o));
    }
    __shared__ uint32_t s[2][VH_TPB / VH_WAVE];
    const int w = threadIdx.x / VH_WAVE;
    if ((threadIdx.x & (VH_WAVE - 1)) == 0) {
        s[0][w] = lo;
        s[1][w] = hi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < VH_TPB / VH_WAVE; ++k) {
            lo = min(lo, s[0][k]);
            hi = max(hi, s[1][k]);
        }
        atomicMin(&mm[2 * blockIdx.y], lo);
        atomicMax(&mm[2 * blockIdx.y + 1], hi);
    }
}

// One block = one row r, 64 columns, up to 64 slices of one volume.  Reads the block's
// contiguous [c][z] run of N4 / defect, composes the RGB triples into LDS in [z][c][3] order and
// writes each slice's 192-byte row segment out as dwords.
__global__ __launch_bounds__(VH_TPB) void k_overlay(const float *__restrict__ n4,
                                                    const uint8_t *__restrict__ def,
                                                    const uint32_t *__restrict__ mm, int64_t R,
                                                    int64_t C, int64_t Z, int ncc,
                                                    uint8_t *__restrict__ rgb) {
    __shared__ uint32_t sbuf[OV_ZC * OV_WORDS];
    uint8_t *sb = reinterpret_cast<uint8_t *>(sbuf);
    const int cchunk = blockIdx.x % ncc, zchunk = blockIdx.x / ncc;
    const int64_t r = blockIdx.y, vol = blockIdx.z;
    const int64_t c0 = (int64_t)cchunk * OV_COLS, z0 = (int64_t)zchunk * OV_ZC;
    const int nc = (int)min((int64_t)OV_COLS, C - c0), nz = (int)min((int64_t)OV_ZC, Z - z0);
    const uint32_t lo = mm[2 * vol], hi = mm[2 * vol + 1];
    const bool nan = hi > 0x7f800000u;
    const float mn = __uint_as_float(lo), mx = __uint_as_float(hi);
    const float rng = mx - mn;   // np.max(x) - np.min(x), float32
    const int64_t base = ((vol * R + r) * C + c0) * Z + z0;
    const int n = nc * nz;
    for (int j = threadIdx.x; j < n; j += VH_TPB) {
        const int c = j / nz, z = j - c * nz;
        const int64_t idx = base + (int64_t)c * Z + z;
        const float x = fabsf(n4[idx]);
        const uint8_t d = def[idx];
        uint8_t bw = 0;
        if (!nan) {
            const float v = (rng != 0.f) ? (x - mn) / rng : x;   // normalize (:233-237)
            bw = np_u8((double)(v * 255.f));                      // * (2**8 - 1), astype uint8
        }
        const uint8_t g = d == 0 ? bw : (uint8_t)0;
        const int o = (z * nc + c) * 3;
        sb[o] = (uint8_t)(g + (d == 1 ? 255 : 0));
        sb[o + 1] = g;
        sb[o + 2] = g;
    }
    __syncthreads();
    const int64_t plane = R * C * 3;
    const int64_t out0 = ((vol * Z + z0) * R + r) * C * 3 + c0 * 3;
    if ((C & 3) == 0 && nc == OV_COLS) {   // dword stores: each slice segment is 48 aligned words
        for (int w = threadIdx.x; w < nz * OV_WORDS; w += VH_TPB) {
            const int z = w / OV_WORDS, k = w - z * OV_WORDS;
            reinterpret_cast<uint32_t *>(rgb + out0 + z * plane)[k] = sbuf[w];
        }
    } else {
        const int seg = nc * 3;
        for (int bidx = threadIdx.x; bidx < nz * seg; bidx += VH_TPB) {
            const int z = bidx / seg, k = bidx - z * seg;
            rgb[out0 + z * plane + k] = sb[bidx];
        }
    }
}

void vh_overlay_launch(hipStream_t s, const float *d_n4, const uint8_t *d_def, int64_t R,
                       int64_t C, int64_t Z, int64_t nb, uint32_t *d_mm, uint8_t *d_rgb) {
    const int64_t V = R * C * Z;
    if (nb > 65535 || R > 65535) throw VhError{VH_ERR_ARG, "overlay: batch or rows out of range"};
    k_absmm_init<<<(unsigned)((nb + VH_TPB - 1) / VH_TPB), VH_TPB, 0, s>>>(d_mm, nb);
    VH_CHECK_LAUNCH();
    const int64_t per = std::max<int64_t>(1, std::min<int64_t>(1024, (V + VH_TPB * 16 - 1) / (VH_TPB * 16)));
    k_absminmax<<<dim3((unsigned)per, (unsigned)nb), VH_TPB, 0, s>>>(d_n4, V, d_mm);
    VH_CHECK_LAUNCH();
    const int ncc = (int)((C + OV_COLS - 1) / OV_COLS);
    const int nzc = (int)((Z + OV_ZC - 1) / OV_ZC);
    k_overlay<<<dim3((unsigned)(ncc * nzc), (unsigned)R, (unsigned)nb), VH_TPB, 0, s>>>(
        d_n4, d_def, d_mm, R, C, Z, ncc, d_rgb);
    VH_CHECK_LAUNCH();
}

// ---- screenShot montage -----------------------------------------------------------------------
struct MontageArgs {
    const void *proton;   // float32 or float64 volume
    const void *hp;
    const float *n4;
    const uint8_t *mborder;
    const uint8_t *def;
    const double *ci;     // nullable: blank CI panel (the reference's except: CI = blank, :478-479)
    const double *parula; // [prow][3]
    int64_t prow;
    int p64, h64;         // 1: float64 volume, 0: float32
    int64_t R, C, Z;
    int64_t r0, nr, c0, nc, s0, ns;
};

__device__ __forceinline__ double load_as_double(const void *p, int is64, int64_t i) {
    return is64 ? static_cast<const double *>(p)[i] : (double)static_cast<const float *>(p)[i];
}

// min / max over the crop of proton, HPvent and N4 (keys[2a] = min, keys[2a+1] = max)
__global__ __launch_bounds__(VH_TPB) void k_crop_minmax(MontageArgs a, uint64_t *keys) {
    const int64_t n = a.nr * a.nc * a.ns;
    uint64_t lo[3] = {~0ull, ~0ull, ~0ull}, hi[3] = {0ull, 0ull, 0ull};
    for (int64_t t = (int64_t)blockIdx.x * VH_TPB + threadIdx.x; t < n;
         t += (int64_t)gridDim.x * VH_TPB) {
        const int64_t s = t % a.ns, j = (t / a.ns) % a.nc, i = t / (a.ns * a.nc);
        const int64_t idx = ((a.r0 + i) * a.C + a.c0 + j) * a.Z + a.s0 + s;
        const uint64_t k0 = d2key(load_as_double(a.proton, a.p64, idx));
        const uint64_t k1 = d2key(load_as_double(a.hp, a.h64, idx));
        const uint64_t k2 = d2key((double)a.n4[idx]);
        lo[0] = min(lo[0], k0); hi[0] = max(hi[0], k0);
        lo[1] = min(lo[1], k1); hi[1] = max(hi[1], k1);
        lo[2] = min(lo[2], k2); hi[2] = max(hi[2], k2);
    }
    for (int q = 0; q < 3; ++q) {
        for (int o = 32; o > 0; o >>= 1) {
            lo[q] = min(lo[q], (uint64_t)__shfl_xor((unsigned long long)lo[q], o));
            hi[q] = max(hi[q], (uint64_t)__shfl_xor((unsigned long long)hi[q], o));
        }
        if ((threadIdx.x & (VH_WAVE - 1)) == 0) {
            atomicMin((unsigned long long *)&keys[2 * q], (unsigned long long)lo[q]);
            atomicMax((unsigned long long *)&keys[2 * q + 1], (unsigned long long)hi[q]);
        }
    }
}

// the screenShot normalize (:460-464) in the array's own float type, widened to float64
__device__ __forceinline__ double norm_val(const void *p, int is64, int64_t idx, double mn,
                                           double mx) {
    if (is64) {
        const double x = static_cast<const double *>(p)[idx];
        const double rng = mx - mn;
        return rng == 0.0 ? x : (x - mn) / rng;
    }
    const float x = static_cast<const float *>(p)[idx];
    const float fmn = (float)mn, rng = (float)mx - (float)mn;
    return (double)(rng == 0.f ? x : (x - fmn) / rng);
}

// One thread per montage pixel.  Grid row g of the 7 x ns montage holds panel g, column s holds
// crop slice s (skimage.util.montage, grid_shape=(7, ns), padding 0: images fill row-major).
__global__ __launch_bounds__(VH_TPB) void k_montage(MontageArgs a, const uint64_t *keys,
                                                    uint8_t *__restrict__ img,
                                                    int32_t *__restrict__ err) {
    const int64_t W = a.ns * a.nc, H = 7 * a.nr;
    const int64_t t = (int64_t)blockIdx.x * VH_TPB + threadIdx.x;
    if (t >= W * H) return;
    const int64_t y = t / W, x = t - y * W;
    const int g = (int)(y / a.nr);
    const int64_t i = y - g * a.nr, s = x / a.nc, j = x - s * a.nc;
    const int64_t idx = ((a.r0 + i) * a.C + a.c0 + j) * a.Z + a.s0 + s;
    double rv = 0.0, gv = 0.0, bv = 0.0;
    if (g == 2 || g == 3) {
        const int q = g - 2;
        rv = gv = bv = norm_val(q == 0 ? a.proton : a.hp, q == 0 ? a.p64 : a.h64, idx,
                                key2d(keys[2 * q]), key2d(keys[2 * q + 1]));
    } else if (g >= 4) {
        const double n = norm_val(a.n4, 0, idx, key2d(keys[4]), key2d(keys[5]));
        if (g == 4) {          // N4*(~border) + {0,1,1}*border
            const bool bd = a.mborder[idx] != 0;
            rv = bd ? 0.0 : n;
            gv = bv = bd ? 1.0 : n;
        } else if (g == 5) {   // N4*(~defArr) + {defArr, 0, 0}
            const bool df = a.def[idx] != 0;
            rv = df ? 1.0 : n;
            gv = bv = df ? 0.0 : n;
        } else {               // N4*(CI==0) + parula[int(CI*64/40)]*(CI>0)
            const double ci = a.ci ? a.ci[idx] : 0.0;
            const double tt = ci * 64.0 / 40.0;
            if (tt != tt) {
                atomicOr(err, 2);   // int(NaN): ValueError
            } else if (!(tt < 9.2e18 && tt > -9.2e18) || (int64_t)tt >= a.prow ||
                       (int64_t)tt < -a.prow) {
                atomicOr(err, 1);   // parula index out of range: IndexError
            } else if (ci > 0.0) {
                const double *p = a.parula + 3 * (int64_t)tt;
                rv = p[0]; gv = p[1]; bv = p[2];
            } else if (ci == 0.0) {
                rv = gv = bv = n;
            }
        }
    }
    uint8_t *o = img + t * 3;
    o[0] = np_u8(rv * 255.0);
    o[1] = np_u8(gv * 255.0);
    o[2] = np_u8(bv * 255.0);
}

static void *dcopy(const void *h, size_t bytes, hipStream_t s) {
    void *d = nullptr;
    HIP_TRY(hipMalloc(&d, bytes ? bytes : 1));
    if (h && bytes) HIP_TRY(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s));
    return d;
}

void vh_montage_run(hipStream_t s, int64_t R, int64_t C, int64_t Z, const void *proton, int p64,
                    const void *hp, int h64, const float *n4, const uint8_t *mborder,
                    const uint8_t *def, const double *ci, const double *parula, int64_t prow,
                    const int64_t crop[6], uint8_t *image) {
    MontageArgs a{};
    a.R = R; a.C = C; a.Z = Z;
    a.r0 = crop[0]; a.nr = crop[1]; a.c0 = crop[2]; a.nc = crop[3]; a.s0 = crop[4]; a.ns = crop[5];
    if (a.nr <= 0 || a.nc <= 0 || a.ns <= 0 || a.r0 < 0 || a.c0 < 0 || a.s0 < 0 ||
        a.r0 + a.nr > R || a.c0 + a.nc > C || a.s0 + a.ns > Z)
        throw VhError{VH_ERR_ARG, "montage: crop outside the volume"};
    if (prow <= 0) throw VhError{VH_ERR_ARG, "montage: empty colour table"};
    a.p64 = p64; a.h64 = h64; a.prow = prow;
    const size_t V = (size_t)(R * C * Z);
    std::vector<void *> owned;
    auto up = [&](const void *h, size_t bytes) {
        void *d = dcopy(h, bytes, s);
        owned.push_back(d);
        return d;
    };
    int32_t herr = 0;
    uint64_t hkeys[6] = {~0ull, 0ull, ~0ull, 0ull, ~0ull, 0ull};
    const int64_t npix = 7 * a.nr * a.ns * a.nc;
    try {
        a.proton = up(proton, V * (p64 ? 8 : 4));
        a.hp = up(hp, V * (h64 ? 8 : 4));
        a.n4 = (const float *)up(n4, V * 4);
        a.mborder = (const uint8_t *)up(mborder, V);
        a.def = (const uint8_t *)up(def, V);
        a.ci = ci ? (const double *)up(ci, V * 8) : nullptr;
        a.parula = (const double *)up(parula, (size_t)prow * 3 * 8);
        uint64_t *d_keys = (uint64_t *)up(hkeys, sizeof(hkeys));
        int32_t *d_err = (int32_t *)up(&herr, sizeof(herr));
        uint8_t *d_img = (uint8_t *)up(nullptr, (size_t)npix * 3);
        const int64_t ncrop = a.nr * a.nc * a.ns;
        const int64_t mblocks = std::max<int64_t>(1, std::min<int64_t>(1024, (ncrop + VH_TPB - 1) / VH_TPB));
        k_crop_minmax<<<(unsigned)mblocks, VH_TPB, 0, s>>>(a, d_keys);
        VH_CHECK_LAUNCH();
        k_montage<<<(unsigned)((npix + VH_TPB - 1) / VH_TPB), VH_TPB, 0, s>>>(a, d_keys, d_img, d_err);
        VH_CHECK_LAUNCH();
        HIP_TRY(hipMemcpyAsync(image, d_img, (size_t)npix * 3, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(&herr, d_err, sizeof(herr), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    } catch (...) {
        (void)hipStreamSynchronize(s);
        for (void *p : owned) (void)hipFree(p);
        throw;
    }
    for (void *p : owned) (void)hipFree(p);
    if (herr & 2) throw VhError{VH_ERR_ARG, "cannot convert float NaN to integer (CI colour index)"};
    if (herr & 1) throw VhError{VH_ERR_INDEX, "CI colour index out of range of the colour table "
                                              "(int(CI*64/40), Vent_Analysis.py:482-484)"};
}
