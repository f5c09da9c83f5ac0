// Does walking every other pass backwards let the next pass read what the last one wrote from the
// 256 MiB MALL?  The three-term pass's memory pattern (read p_{k-1}, p_{k-2} three lines ahead,
// write p_k; vectors rotate) over a sequence of passes, each wave walking one 64-row slice column
// down its run of lines; "fwd" walks every pass top-down, "alt" walks odd passes bottom-up, so the
// lines a pass wrote last are the ones the next pass reads first.  Prints ms per pass and TB/s of
// the modelled traffic (2 reads + 1 write per row), plain and non-temporal stores.
//   hipcc --offload-arch=gfx950 -O3 bench/mall_reverse.hip -o build/mall_reverse && ./build/mall_reverse
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <bool REV, bool NT>
__global__ __launch_bounds__(256) void k_dir(const double* __restrict__ pa, const double* __restrict__ pb,
                                             double* __restrict__ pc, int64_t lines, int64_t line_len, int64_t runs) {
  constexpr int D = 3;
  const int lane = threadIdx.x & 63;
  const int64_t cols = line_len / 64;
  const int64_t gw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (int64_t)gridDim.x * 4;
  const int64_t chunk = (lines + runs - 1) / runs;
  for (int64_t job = gw; job < cols * runs; job += nw) {
    const int64_t col = job % cols, l0 = (job / cols) * chunk;
    const int64_t l1 = l0 + chunk < lines ? l0 + chunk : lines;
    if (l1 - l0 <= D) continue;
    const int64_t first = REV ? l1 - 1 : l0;
    const int64_t st = REV ? -line_len : line_len;
    const double* a = pa + first * line_len + col * 64 + lane;
    const double* b = pb + first * line_len + col * 64 + lane;
    double* o = pc + first * line_len + col * 64 + lane;
    double qa[D], qb[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      qa[d] = a[d * st];
      qb[d] = b[d * st];
    }
    const int64_t n = l1 - l0 - D;
    for (int64_t m = 0; m + D <= n; m += D) {
#pragma unroll
      for (int u = 0; u < D; ++u) {
        const double na = a[(m + u + D) * st], nb = b[(m + u + D) * st];
        const double v = qa[u] + 0.5 * qb[u];
        if constexpr (NT) __builtin_nontemporal_store(v, &o[(m + u) * st]);
        else o[(m + u) * st] = v;
        qa[u] = na;
        qb[u] = nb;
      }
    }
  }
}

int main() {
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int64_t N : {4096, 8192, 16384}) {
    const int64_t n = N * N;
    double* v[3];
    for (int i = 0; i < 3; ++i) {
      CK(hipMalloc(&v[i], n * 8));
      CK(hipMemset(v[i], 0, n * 8));
    }
    const int bpc = N <= 4096 ? 4 : 8;
    const int grid = ncu * bpc;
    const int64_t cols = N / 64, nw = (int64_t)grid * 4, runs = nw > cols ? nw / cols : 1;
    for (int nt = 0; nt < 2; ++nt) {
      for (int alt = 0; alt < 2; ++alt) {
        auto pass = [&](int k) {
          const double* a = v[(k + 2) % 3];
          const double* b = v[(k + 1) % 3];
          double* c = v[k % 3];
          const bool rev = alt && (k & 1);
          if (nt) {
            if (rev) hipLaunchKernelGGL((k_dir<true, true>), dim3(grid), dim3(256), 0, 0, a, b, c, N, N, runs);
            else hipLaunchKernelGGL((k_dir<false, true>), dim3(grid), dim3(256), 0, 0, a, b, c, N, N, runs);
          } else {
            if (rev) hipLaunchKernelGGL((k_dir<true, false>), dim3(grid), dim3(256), 0, 0, a, b, c, N, N, runs);
            else hipLaunchKernelGGL((k_dir<false, false>), dim3(grid), dim3(256), 0, 0, a, b, c, N, N, runs);
          }
        };
        for (int k = 0; k < 4; ++k) pass(k);
        const int reps = N <= 4096 ? 200 : 20;
        CK(hipEventRecord(e0));
        for (int k = 0; k < reps; ++k) pass(k);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("N %5lld  %s stores  %s  %.4f ms/pass  %.2f TB/s\n", (long long)N, nt ? "nt   " : "plain",
               alt ? "alt" : "fwd", ms, 3.0 * n * 8 / (ms * 1e-3) / 1e12);
        fflush(stdout);
      }
    }
    for (int i = 0; i < 3; ++i) CK(hipFree(v[i]));
  }
  return 0;
}
