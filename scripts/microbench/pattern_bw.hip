// Microbenchmark: achievable HBM bandwidth of the N4 eval access pattern on gfx950.
// 256 volumes of 128x128x24 f32; "masked" voxels = an ellipsoid pair (~21%).
//  A: flat contiguous stream   (read 2 arrays, write 2 arrays, every voxel)
//  B: column sweep, lane = column, rows walked in chunks of 8 (all voxels)
//  C: column sweep with mask bits (only masked voxels), like k_n4_eval
//  D: tiled layout [tile][row][256 cols] column sweep with mask bits
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cmath>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
constexpr int R = 128, C = 128, Z = 24, CZ = C * Z, V = R * CZ;

__global__ void flat(const float4* a, const float4* b, float4* c, float4* d, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float4 x = a[i], y = b[i];
    c[i] = make_float4(x.x - y.x, x.y - y.y, x.z - y.z, x.w - y.w);
    d[i] = make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);
  }
}

template <bool MASKED>
__global__ void sweep(const float* a, float* bb, float* u, const unsigned* bits, int nvol) {
  const int vol = blockIdx.y;
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= CZ) return;
  const float* A = a + (long)vol * V + col; float* B = bb + (long)vol * V + col; float* U = u + (long)vol * V + col;
  const unsigned* cb = bits + (long)vol * 4 * CZ + col;
  for (int x0 = 0; x0 < R; x0 += 8) {
    unsigned m = MASKED ? (cb[(x0 >> 5) * CZ] >> (x0 & 31)) & 0xff : 0xff;
    float la[8], ba[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { la[k] = (m >> k) & 1 ? A[(long)(x0 + k) * CZ] : 0.f; ba[k] = (m >> k) & 1 ? B[(long)(x0 + k) * CZ] : 0.f; }
#pragma unroll
    for (int k = 0; k < 8; ++k) if ((m >> k) & 1) { B[(long)(x0 + k) * CZ] = la[k] - ba[k]; U[(long)(x0 + k) * CZ] = la[k] + ba[k]; }
  }
}

// tiled layout: volume -> [tile][row][256]
__global__ void sweep_tiled(const float* a, float* bb, float* u, const unsigned* bits, int nvol) {
  const int vol = blockIdx.y, tile = blockIdx.x, t = threadIdx.x;
  const int col = tile * 256 + t;
  if (col >= CZ) return;
  const long base = (long)vol * V + (long)tile * R * 256 + t;
  const unsigned* cb = bits + (long)vol * 4 * CZ + col;
  for (int x0 = 0; x0 < R; x0 += 8) {
    unsigned m = (cb[(x0 >> 5) * CZ] >> (x0 & 31)) & 0xff;
    float la[8], ba[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { la[k] = (m >> k) & 1 ? a[base + (long)(x0 + k) * 256] : 0.f; ba[k] = (m >> k) & 1 ? bb[base + (long)(x0 + k) * 256] : 0.f; }
#pragma unroll
    for (int k = 0; k < 8; ++k) if ((m >> k) & 1) { bb[base + (long)(x0 + k) * 256] = la[k] - ba[k]; u[base + (long)(x0 + k) * 256] = la[k] + ba[k]; }
  }
}

// E: dense layout, one wave per (64-column tile, SEG-row segment): one round trip per wave
template <int SEG>
__global__ void seg_dense(const float* a, float* bb, float* u, const unsigned* bits, int nvol) {
  const int vol = blockIdx.z, seg = blockIdx.y;
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= CZ) return;
  const int x0 = seg * SEG;
  const float* A = a + (long)vol * V + col; float* B = bb + (long)vol * V + col; float* U = u + (long)vol * V + col;
  const unsigned m = (bits[(long)vol * 4 * CZ + (x0 >> 5) * CZ + col] >> (x0 & 31)) & ((1u << SEG) - 1u);
  if (!m) return;
  float la[SEG], ba[SEG];
#pragma unroll
  for (int k = 0; k < SEG; ++k) { la[k] = (m >> k) & 1 ? A[(long)(x0 + k) * CZ] : 0.f; ba[k] = (m >> k) & 1 ? B[(long)(x0 + k) * CZ] : 0.f; }
#pragma unroll
  for (int k = 0; k < SEG; ++k) if ((m >> k) & 1) { B[(long)(x0 + k) * CZ] = la[k] - ba[k]; U[(long)(x0 + k) * CZ] = la[k] + ba[k]; }
}

// F: compact tile-row layout: per (64-col tile, row) the masked lanes contiguous; offsets table
template <int SEG>
__global__ void seg_compact(const float* a, float* bb, float* u, const unsigned* bits, const int* rs, int nvol, long cap) {
  const int vol = blockIdx.z, seg = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int tile = blockIdx.x * 4 + wave;
  const int col = tile * 64 + lane;
  const bool valid = col < CZ;
  const int x0 = seg * SEG;
  const unsigned m = valid ? (bits[(long)vol * 4 * CZ + (x0 >> 5) * CZ + col] >> (x0 & 31)) & ((1u << SEG) - 1u) : 0u;
  const float* A = a + (long)vol * cap; float* B = bb + (long)vol * cap; float* U = u + (long)vol * cap;
  const int* r = rs + (long)tile * R;
  int off[SEG];
#pragma unroll
  for (int k = 0; k < SEG; ++k) {
    const unsigned long long bal = __ballot((m >> k) & 1u);
    off[k] = r[x0 + k] + __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
  }
  float la[SEG], ba[SEG];
#pragma unroll
  for (int k = 0; k < SEG; ++k) { la[k] = (m >> k) & 1 ? A[off[k]] : 0.f; ba[k] = (m >> k) & 1 ? B[off[k]] : 0.f; }
#pragma unroll
  for (int k = 0; k < SEG; ++k) if ((m >> k) & 1) { B[off[k]] = la[k] - ba[k]; U[off[k]] = la[k] + ba[k]; }
}

int main() {
  const int nvol = 256;
  const long N = (long)nvol * V;
  float *a, *b, *c, *d; unsigned* bits;
  CHK(hipMalloc(&a, N * 4)); CHK(hipMalloc(&b, N * 4)); CHK(hipMalloc(&c, N * 4)); CHK(hipMalloc(&d, N * 4));
  CHK(hipMalloc(&bits, (long)nvol * 4 * CZ * 4));
  CHK(hipMemset(a, 0, N * 4)); CHK(hipMemset(b, 0, N * 4));
  std::vector<unsigned> hb(4 * CZ, 0); long nm = 0;
  for (int x = 0; x < R; ++x) for (int y = 0; y < C; ++y) for (int z = 0; z < Z; ++z) {
    bool m = false;
    for (double cc : {0.32, 0.68}) {
      double dx = (x - R / 2.0) / (0.35 * R), dy = (y - cc * C) / (0.17 * C), dz = (z - Z / 2.0) / (0.42 * Z);
      if (dx * dx + dy * dy + dz * dz <= 1) m = true;
    }
    if (m) { hb[(x >> 5) * CZ + y * Z + z] |= 1u << (x & 31); ++nm; }
  }
  for (int v = 0; v < nvol; ++v) CHK(hipMemcpy(bits + (long)v * 4 * CZ, hb.data(), 4 * CZ * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto launch, double bytes) {
    for (int i = 0; i < 3; ++i) launch();
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    const int it = 20;
    for (int i = 0; i < it; ++i) launch();
    CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
    float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-34s %8.1f us  %7.1f GB/s (bytes %.1f MB)\n", name, ms * 1e3 / it, bytes / (ms * 1e-3 / it) / 1e9, bytes / 1e6);
    return 0;
  };
  printf("masked fraction %.3f\n", (double)nm / V);
  timeit("A flat contiguous 4 arrays", [&] { flat<<<4096, 256>>>((float4*)a, (float4*)b, (float4*)c, (float4*)d, N / 4); }, 16.0 * N);
  timeit("B column sweep dense", [&] { sweep<false><<<dim3(CZ / 256, nvol), 256>>>(a, b, c, bits, nvol); }, 16.0 * N);
  timeit("C column sweep masked", [&] { sweep<true><<<dim3(CZ / 256, nvol), 256>>>(a, b, c, bits, nvol); }, 16.0 * nm * nvol);
  timeit("E dense segments of 16", [&] { seg_dense<16><<<dim3(CZ / 256, R / 16, nvol), 256>>>(a, b, c, bits, nvol); }, 16.0 * nm * nvol);
  timeit("E dense segments of 8", [&] { seg_dense<8><<<dim3(CZ / 256, R / 8, nvol), 256>>>(a, b, c, bits, nvol); }, 16.0 * nm * nvol);
  {
    // compact offsets: per tile (64 cols) per row, prefix over rows of popcounts
    std::vector<int> rs(CZ / 64 * R);
    long acc = 0;
    for (int t = 0; t < CZ / 64; ++t) for (int x = 0; x < R; ++x) {
      rs[t * R + x] = (int)acc;
      for (int l = 0; l < 64; ++l) { int col = t * 64 + l; acc += (hb[(x >> 5) * CZ + col] >> (x & 31)) & 1u; }
    }
    int* drs; CHK(hipMalloc(&drs, rs.size() * 4)); CHK(hipMemcpy(drs, rs.data(), rs.size() * 4, hipMemcpyHostToDevice));
    long cap = acc;
    timeit("F compact segments of 16", [&] { seg_compact<16><<<dim3(CZ / 256, R / 16, nvol), 256>>>(a, b, c, bits, drs, nvol, cap); }, 16.0 * nm * nvol);
    timeit("F compact segments of 32", [&] { seg_compact<32><<<dim3(CZ / 256, R / 32, nvol), 256>>>(a, b, c, bits, drs, nvol, cap); }, 16.0 * nm * nvol);
  }
  timeit("D tiled column sweep masked", [&] { sweep_tiled<<<dim3(CZ / 256, nvol), 256>>>(a, b, c, bits, nvol); }, 16.0 * nm * nvol);
  return 0;
}
