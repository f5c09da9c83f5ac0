// Random 8-B gathers on MI355X: how fast does a wave64 gather p[col] for uniformly random
// columns, as a function of the gathered vector's size (L2 4 MiB/XCD, Infinity Cache 256 MiB,
// HBM beyond)?  This decides whether column-segment blocking of the irregular SpMV (all waves
// gathering from one MALL-sized segment of p at a time) pays (profiles/r3_gather_probe.md).
//   hipcc --offload-arch=gfx950 -O3 bench/gather_probe.hip -o build/gather_probe && ./build/gather_probe
// Two kernels:
//   hash   columns from a counter hash in registers: the gather alone
//   sell   SELL-64-shaped: per entry a 4-B column and an 8-B value streamed (coalesced), then the
//          gather -- the irregular SpMV's inner loop (12 B of stream + one gather per entry)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      printf("%s: %s\n", #x, hipGetErrorString(e));                        \
      return 1;                                                            \
    }                                                                      \
  } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

template <int UNR>
__global__ __launch_bounds__(256) void k_hash(const double* __restrict__ p, uint32_t n, int iters, double* out) {
  double acc = 0;
  const uint32_t gid = blockIdx.x * 256 + threadIdx.x;
  for (int k = 0; k < iters; k += UNR) {
    double v[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const uint32_t c = (uint32_t)(((uint64_t)hash32(gid * 0x9E3779B9U + (uint32_t)(k + u)) * n) >> 32);
      v[u] = p[c];
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) acc += v[u];
  }
  if (acc == 12345.678) *out = acc;
}

// segment sweep: every thread walks G segments of S doubles in order and gathers `per` random
// doubles from each (UNR in flight): the tile kernel's access pattern without its stream / LDS
template <int UNR>
__global__ __launch_bounds__(256) void k_seg(const double* __restrict__ p, uint32_t S, int G, int per, double* out) {
  double acc = 0;
  const uint32_t gid = blockIdx.x * 256 + threadIdx.x;
  for (int g = 0; g < G; ++g) {
    const double* pg = p + (size_t)g * S;
    for (int k = 0; k < per; k += UNR) {
      double v[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const uint32_t c = (uint32_t)(((uint64_t)hash32(gid * 0x9E3779B9U + (uint32_t)(g * per + k + u)) * S) >> 32);
        v[u] = pg[c];
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) acc += v[u];
    }
  }
  if (acc == 12345.678) *out = acc;
}

// bisection between k_seg (L2 hits) and k_tile (misses): F bit 0 = tile bounds from memory (tptr),
// bit 1 = LDS accumulators (ds_add_f64), bit 2 = the tile is `per64 + 1` entries (a remainder pass),
// bit 3 = pacing barrier per segment (the workgroups of group blockIdx % 8; counters 256 B apart,
// gentle polling), bit 4 = packed (row, column) and value streamed from memory (NT loads) instead
// of hashed in registers
template <int F, int U = 4>
__global__ __launch_bounds__(256) void k_tt(const double* __restrict__ p, const int64_t* __restrict__ tptr,
                                            const uint32_t* __restrict__ idx, const double* __restrict__ vals,
                                            uint32_t S, int G, int per64, double* __restrict__ y,
                                            unsigned* __restrict__ arr, int D = 0) {
  __shared__ double acc[4][1024];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  double* a = acc[wv];
  double racc = 0.0;
  if (F & 2)
    for (int r = lane; r < 1024; r += 64) a[r] = 0.0;
  const int64_t len = (int64_t)per64 + ((F & 4) ? 1 : 0);
  for (int g = 0; g < G; ++g) {
    int64_t lo, hi;
    if (F & 1) {
      lo = tptr[wave * G + g];
      hi = tptr[wave * G + g + 1];
    } else {
      lo = (wave * G + g) * len;
      hi = lo + len;
    }
    const double* pg = p + (size_t)g * S;
    int64_t k = lo + lane;
    for (; k + (U - 1) * 64 < hi; k += U * 64) {
      double x[U], v[U];
      uint32_t h[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (F & 16) {
          h[u] = __builtin_nontemporal_load(&idx[k + u * 64]);
          v[u] = __builtin_nontemporal_load(&vals[k + u * 64]);
        } else {
          h[u] = hash32((uint32_t)(k + u * 64) * 0x9E3779B9U);
          v[u] = 0.5;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        x[u] = pg[(F & 16) ? (h[u] & 0x3FFFFFu) : (uint32_t)(((uint64_t)h[u] * S) >> 32)];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (F & 2) atomicAdd(&a[(F & 16) ? (h[u] >> 22) : (h[u] & 1023)], v[u] * x[u]);
        else racc = fma(v[u], x[u], racc);
      }
    }
    for (; k < hi; k += 64) {
      const uint32_t h = (F & 16) ? idx[k] : hash32((uint32_t)k * 0x9E3779B9U);
      const double v = (F & 16) ? vals[k] : 0.5;
      const double x = pg[(F & 16) ? (h & 0x3FFFFFu) : (uint32_t)(((uint64_t)h * S) >> 32)];
      if (F & 2) atomicAdd(&a[(F & 16) ? (h >> 22) : (h & 1023)], v * x);
      else racc = fma(v, x, racc);
    }
    if (F & 8) {
      __syncthreads();
      if (threadIdx.x == 0) {
        const int grp = blockIdx.x & 7;
        const unsigned nwg = (gridDim.x - grp + 7) / 8;
        unsigned* c = arr + grp * 64;  // one 256-B block per group
        __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned target = g + 1 > D ? (unsigned)(g + 1 - D) * nwg : 0u;
        int spin = 0;
        for (; spin < 20000; ++spin) {
          if (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
          __builtin_amdgcn_s_sleep(8);
        }
        if (spin == 20000) __hip_atomic_fetch_add(arr + 8 * 64, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
    }
  }
  if (F & 2)
    for (int r = lane; r < 1024; r += 64) racc += a[r];
  y[wave * 64 + lane] = racc;
}

// slices of 64 rows x w slots, column-major; grid-stride over slices
template <int UNR>
__global__ __launch_bounds__(256) void k_sell(const int32_t* __restrict__ cols, const double* __restrict__ vals,
                                              const double* __restrict__ p, int64_t nslices, int w,
                                              double* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  for (int64_t s = wave; s < nslices; s += nwaves) {
    const int64_t base = s * 64 * w + lane;
    double acc = 0;
    for (int j = 0; j < w; j += UNR) {
      int32_t c[UNR];
      double a[UNR], g[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        c[u] = __builtin_nontemporal_load(&cols[base + (int64_t)(j + u) * 64]);
        a[u] = __builtin_nontemporal_load(&vals[base + (int64_t)(j + u) * 64]);
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) g[u] = p[c[u]];
#pragma unroll
      for (int u = 0; u < UNR; ++u) acc = fma(a[u], g[u], acc);
    }
    y[s * 64 + lane] = acc;
  }
}

// L2-blocked COO tiles: wave w owns B consecutive rows (accumulators in LDS) and walks the column
// segments g = 0..G-1 of size S in order, so every wave of the chip gathers from the same
// S-double segment of p at about the same time (L2-resident); tile (block, g) is a flat list of
// packed (row in block << 22 | column in segment) + value, spread over the 64 lanes.
// V: 0 = as described; 1 = register accumulation instead of the LDS atomics (wrong sums: a cost
// probe); 2 = packed indices from a hash instead of the stream; 3 = no gather (p[...] -> 1.0);
// 4 = 2 and 1 (hash indices, register accumulation)
// pacing: ngrp > 0 = after every segment the workgroup adds to its group's arrival counter (group =
// blockIdx % ngrp, i.e. the XCD under round-robin dispatch) and waits (bounded spin, pacing only)
// until every workgroup of the group has finished that segment
template <int B, int UNR, int V>
__global__ __launch_bounds__(256) void k_tile(const uint32_t* __restrict__ idx, const double* __restrict__ vals,
                                              const int64_t* __restrict__ tptr, const double* __restrict__ p,
                                              int64_t nblocks, int G, int S, double* __restrict__ y,
                                              unsigned* __restrict__ arr, int ngrp) {
  __shared__ double acc[4][B];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  double* a = acc[wv];
  double racc = 0.0;
  for (int64_t b = wave; b < nblocks; b += nwaves) {
    for (int r = lane; r < B; r += 64) a[r] = 0.0;
    for (int g = 0; g < G; ++g) {
      const int64_t lo = tptr[b * G + g], hi = tptr[b * G + g + 1];
      const double* pg = p + (int64_t)g * S;
      int64_t k = lo + lane;
      for (; k + (UNR - 1) * 64 < hi; k += UNR * 64) {
        uint32_t q[UNR];
        double v[UNR], x[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          if constexpr (V == 2 || V == 4) {
            const uint32_t h = hash32((uint32_t)(k + u * 64) * 0x9E3779B9U);
            q[u] = ((h & (B - 1)) << 22) | ((h >> 10) & (uint32_t)(S - 1));
            v[u] = 0.5;
          } else {
            q[u] = __builtin_nontemporal_load(&idx[k + u * 64]);
            v[u] = __builtin_nontemporal_load(&vals[k + u * 64]);
          }
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) x[u] = V == 3 ? 1.0 : pg[q[u] & 0x3FFFFFu];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          if constexpr (V == 1 || V == 4) racc = fma(v[u], x[u], racc);
          else atomicAdd(&a[q[u] >> 22], v[u] * x[u]);
        }
      }
      for (; k < hi; k += 64) {
        const uint32_t q = idx[k];
        atomicAdd(&a[q >> 22], vals[k] * pg[q & 0x3FFFFFu]);
      }
    }
    for (int r = lane; r < B; r += 64) y[b * B + r] = a[r] + racc;
  }
}

__global__ void k_fill_tiles(uint32_t* idx, int64_t m, int B, int S, uint32_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t h1 = hash32((uint32_t)i * 0x9E3779B9U ^ seed), h2 = hash32(h1 ^ 0x5bd1e995U);
    idx[i] = ((uint32_t)(((uint64_t)h1 * B) >> 32) << 22) | (uint32_t)(((uint64_t)h2 * S) >> 32);
  }
}

__global__ void k_fill_cols(int32_t* cols, int64_t m, uint32_t n, uint32_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
    cols[i] = (int32_t)(((uint64_t)hash32((uint32_t)i * 0x9E3779B9U ^ seed ^ (uint32_t)(i >> 32)) * n) >> 32);
}
__global__ void k_fill_d(double* a, int64_t m, double v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
    a[i] = v + (double)(i & 7);
}

int main(int argc, char** argv) {
  // ./gather_probe            all sections
  // ./gather_probe tile S B V P  one tile configuration (for counter runs); P = pacing groups
  const bool only_tile = argc >= 6 && std::string(argv[1]) == "tile";
  const int arg_P = only_tile ? std::atoi(argv[5]) : 0;
  const int arg_S = only_tile ? std::atoi(argv[2]) : 0, arg_B = only_tile ? std::atoi(argv[3]) : 0,
            arg_V = only_tile ? std::atoi(argv[4]) : -1;
  int ncu = 256;
  {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    ncu = prop.multiProcessorCount;
  }
  const int64_t max_table = 1600ll << 20;  // 1.6 GB (>= the tile section's 1e8 columns)
  double *p = nullptr, *out = nullptr, *y = nullptr, *vals = nullptr;
  int32_t* cols = nullptr;
  CK(hipMalloc(&p, max_table));
  CK(hipMalloc(&out, 8));
  hipLaunchKernelGGL(k_fill_d, dim3(4096), dim3(256), 0, 0, p, max_table / 8, 1.0);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int64_t sizes_all[] = {4, 16, 32, 64, 128, 192, 256, 384, 512, 800, 1600};
  const bool skip_rand = only_tile || (argc >= 2 && std::string(argv[1]) != "all");
  std::vector<int64_t> sizes_mb(sizes_all, sizes_all + (skip_rand ? 0 : 11));
  // --- hash kernel: gathers only ---
  const int iters = 512;
  const int grid = ncu * 8;
  printf("# kernel=hash grid=%d x 256 threads, %d gathers per thread\n", grid, iters);
  printf("table_MB  ms  Ggathers_per_s  GB_per_s_at_64B\n");
  for (int64_t mb : sizes_mb) {
    const uint32_t n = (uint32_t)((mb << 20) / 8);
    hipLaunchKernelGGL(k_hash<8>, dim3(grid), dim3(256), 0, 0, p, n, iters, out);
    CK(hipEventRecord(e0));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_hash<8>, dim3(grid), dim3(256), 0, 0, p, n, iters, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 5;
    const double g = (double)grid * 256 * iters / (ms * 1e-3) / 1e9;
    printf("%6lld  %8.3f  %8.2f  %8.1f\n", (long long)mb, ms, g, g * 64);
  }
  // --- SELL-shaped kernel: 12 B of stream + one gather per entry ---
  const int w = 128;                        // slots per slice
  const int64_t nslices = skip_rand ? 64 : 65536;  // 4.19 M rows x 128 = 537 M entries (2.1 GB cols + 4.3 GB vals)
  const int64_t m = nslices * 64 * w;
  CK(hipMalloc(&cols, m * 4));
  CK(hipMalloc(&vals, m * 8));
  CK(hipMalloc(&y, nslices * 64 * 8));
  hipLaunchKernelGGL(k_fill_d, dim3(4096), dim3(256), 0, 0, vals, m, 0.5);
  printf("# kernel=sell %lld slices x 64 rows x %d slots = %lld entries\n", (long long)nslices, w, (long long)m);
  printf("table_MB  grid_bpc  ms  Gentries_per_s  stream_TB_per_s\n");
  for (int64_t mb : sizes_mb) {
    const uint32_t n = (uint32_t)((mb << 20) / 8);
    hipLaunchKernelGGL(k_fill_cols, dim3(4096), dim3(256), 0, 0, cols, m, n, 12345u);
    for (int bpc : {4, 8}) {
      const int g = ncu * bpc;
      hipLaunchKernelGGL(k_sell<8>, dim3(g), dim3(256), 0, 0, cols, vals, p, nslices, w, y);
      CK(hipEventRecord(e0));
      for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k_sell<8>, dim3(g), dim3(256), 0, 0, cols, vals, p, nslices, w, y);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= 3;
      const double ge = (double)m / (ms * 1e-3) / 1e9;
      printf("%6lld  %d  %8.3f  %8.2f  %6.2f\n", (long long)mb, bpc, ms, ge, ge * 12 / 1e3);
    }
  }
  // --- segment sweep (gathers only) ---
  if (argc >= 2 && (std::string(argv[1]) == "seg" || std::string(argv[1]) == "seg1")) {
    const bool one = std::string(argv[1]) == "seg1";
    printf("# kernel=seg: every thread sweeps segments of S doubles, `per` random gathers each\n");
    printf("S  G  per  UNR  wg_per_cu  ms  Ggathers_per_s\n");
    for (int S : {32768, 262144, 524288}) {
      if (one && S != 262144) continue;
      const int G = (int)(100000000ll / S);
      for (int bpc : {4, 8}) {
        for (int unr : {4, 8}) {
          if (one && (bpc != 4 || unr != 4)) continue;
          const int gr = ncu * bpc;
          const int per = (int)(2800000000ll / ((int64_t)gr * 256 * G)) / 8 * 8;
          auto launch = [&]() {
            if (unr == 4) hipLaunchKernelGGL(k_seg<4>, dim3(gr), dim3(256), 0, 0, p, (uint32_t)S, G, per, out);
            else hipLaunchKernelGGL(k_seg<8>, dim3(gr), dim3(256), 0, 0, p, (uint32_t)S, G, per, out);
          };
          launch();
          CK(hipEventRecord(e0));
          launch();
          CK(hipEventRecord(e1));
          CK(hipEventSynchronize(e1));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          printf("%d  %d  %d  %d  %d  %8.3f  %8.2f\n", S, G, per, unr, bpc, ms,
                 (double)gr * 256 * G * per / (ms * 1e-3) / 1e9);
        }
      }
    }
    return 0;
  }
  if (argc >= 2 && std::string(argv[1]) == "tt") {
    printf("# kernel=tt: 4096 waves, segments of S doubles over 1e8 columns, ~1792 * S / 262144 entries per wave and segment\n");
    printf("F  S  D  ms  Ggathers_per_s  arrivals  timeouts\n");
    const int gr = ncu * 4;
    const int64_t nw = (int64_t)gr * 4;
    int64_t* tp = nullptr;
    double* yy = nullptr;
    CK(hipMalloc(&yy, nw * 64 * 8));
    unsigned* arr = nullptr;
    CK(hipMalloc(&arr, 16 * 64 * sizeof(unsigned)));
    uint32_t* sidx = nullptr;
    double* svals = nullptr;
    const int64_t m_all = nw * 381 * (int64_t)(1792 + 1) + (1 << 20);
    CK(hipMalloc(&sidx, m_all * 4));
    CK(hipMalloc(&svals, m_all * 8));
    hipLaunchKernelGGL(k_fill_d, dim3(4096), dim3(256), 0, 0, svals, m_all, 0.25);
    struct Cfg { int F; uint32_t S; int D; };
    std::vector<Cfg> cfgs = {{0, 262144, 0}, {26, 262144, 0}, {26, 262144, 1}, {26, 262144, 2}, {26, 131072, 0},
                             {26, 131072, 1}, {26, 131072, 2}, {26, 131072, 3}, {26, 65536, 2}, {26, 65536, 4},
                             {30, 131072, 2}, {18, 131072, 0}};
    uint32_t filled_S = 0;
    for (const Cfg& c : cfgs) {
      const int F = c.F, D = c.D;
      const uint32_t S = c.S;
      const int G = (int)(100000000ll / S);
      const int per64 = (int)(1792ll * S / 262144);
      if (filled_S != S) {
        hipLaunchKernelGGL(k_fill_tiles, dim3(4096), dim3(256), 0, 0, sidx, m_all, 1024, (int)S, 4242u);
        filled_S = S;
      }
      const int64_t len = per64 + ((F & 4) ? 1 : 0);
      std::vector<int64_t> h(nw * G + 1);
      for (int64_t t = 0; t <= nw * G; ++t) h[t] = t * len;
      CK(hipMalloc(&tp, h.size() * 8));
      CK(hipMemcpy(tp, h.data(), h.size() * 8, hipMemcpyHostToDevice));
      auto launch = [&]() {
        (void)hipMemsetAsync(arr, 0, 16 * 64 * sizeof(unsigned), 0);
#define TT(f) case f: hipLaunchKernelGGL((k_tt<f, 4>), dim3(gr), dim3(256), 0, 0, p, tp, sidx, svals, S, G, per64, yy, arr, D); break
        switch (F) { TT(0); TT(18); TT(26); TT(30); }
#undef TT
      };
      launch();
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      unsigned hc[16 * 64];
      CK(hipMemcpy(hc, arr, sizeof(hc), hipMemcpyDeviceToHost));
      printf("F%d  %u  %d  %8.3f  %8.2f  %u  %u\n", F, S, D, ms, (double)nw * G * len / (ms * 1e-3) / 1e9, hc[0],
             hc[8 * 64]);
      CK(hipFree(tp));
    }
    return 0;
  }
  // --- L2-blocked COO tiles over an 800 MB vector (1e8 columns) ---
  {
    const int64_t ncols = 100000000;
    const double L = 668.0;  // entries per row
    printf("# kernel=tile  rows per wave B, segment S doubles, 1e8 columns, %.0f entries per row\n", L);
    printf("V  pacing_groups  B  S  G  rows  entries  ms  Gentries_per_s\n");
    const int64_t rows = 4 << 20;
    CK(hipFree(cols));
    CK(hipFree(vals));
    CK(hipFree(y));
    const int64_t mmax = (int64_t)(rows * L) + (1 << 20);
    uint32_t* idx = nullptr;
    CK(hipMalloc(&idx, mmax * 4));
    CK(hipMalloc(&vals, mmax * 8));
    CK(hipMalloc(&y, rows * 8));
    hipLaunchKernelGGL(k_fill_d, dim3(4096), dim3(256), 0, 0, vals, mmax, 0.5);
    std::vector<int> Ss = {65536, 131072, 262144, 524288}, Bs = {1024}, Vs = {0, 2}, Vps = {0, 1, 8};
    if (only_tile) Ss = {arg_S}, Bs = {arg_B}, Vs = {arg_V}, Vps = {arg_P};
    unsigned* arr = nullptr;
    CK(hipMalloc(&arr, 64 * sizeof(unsigned)));
    for (int S : Ss) {
      for (int B : Bs)
      for (int V : Vs)
      for (int Vp : Vps) {
        const int G = (int)((ncols + S - 1) / S);
        const int64_t nb = rows / B;
        int64_t per = (int64_t)(B * L * (double)S / (double)ncols);  // entries per tile
        if (nb * G * per > mmax) per = mmax / (nb * G);
        std::vector<int64_t> tp(nb * G + 1);
        for (int64_t t = 0; t <= nb * G; ++t) tp[t] = t * per;
        const int64_t m = nb * G * per;
        int64_t* dtp = nullptr;
        CK(hipMalloc(&dtp, tp.size() * 8));
        CK(hipMemcpy(dtp, tp.data(), tp.size() * 8, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_fill_tiles, dim3(4096), dim3(256), 0, 0, idx, m, B, S, 777u);
        const int ngrp = Vp >= 0 ? Vp : 0;
        auto launch = [&]() {
          (void)hipMemsetAsync(arr, 0, 64 * sizeof(unsigned), 0);
          if (V == 0) hipLaunchKernelGGL((k_tile<1024, 4, 0>), dim3(ncu * 4), dim3(256), 0, 0, idx, vals, dtp, p, nb, G, S, y, arr, ngrp);
          if (V == 1) hipLaunchKernelGGL((k_tile<1024, 4, 1>), dim3(ncu * 4), dim3(256), 0, 0, idx, vals, dtp, p, nb, G, S, y, arr, ngrp);
          if (V == 2) hipLaunchKernelGGL((k_tile<1024, 4, 2>), dim3(ncu * 4), dim3(256), 0, 0, idx, vals, dtp, p, nb, G, S, y, arr, ngrp);
          if (V == 3) hipLaunchKernelGGL((k_tile<1024, 4, 3>), dim3(ncu * 4), dim3(256), 0, 0, idx, vals, dtp, p, nb, G, S, y, arr, ngrp);
          if (V == 4) hipLaunchKernelGGL((k_tile<1024, 4, 4>), dim3(ncu * 4), dim3(256), 0, 0, idx, vals, dtp, p, nb, G, S, y, arr, ngrp);
        };
        launch();
        CK(hipEventRecord(e0));
        for (int r = 0; r < 3; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= 3;
        printf("V%d  grp%d  %d  %d  %d  %lld  %lld  %8.3f  %8.2f\n", V, ngrp, B, S, G, (long long)rows, (long long)m, ms,
               (double)m / (ms * 1e-3) / 1e9);
        CK(hipFree(dtp));
      }
    }
  }
  CK(hipDeviceSynchronize());
  printf("done\n");
  return 0;
}
