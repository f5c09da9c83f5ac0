// The even three-term pass's memory pattern without its arithmetic: every wave walks one column of
// a (lines x line_len) grid down its run of lines, per line step reading two vectors (p_{k-1},
// p_{k-2}) D lines ahead and writing one (p_k, non-temporal) -- W doubles per lane per stream
// (W = 1: one 64-row slice per wave, 8-B lanes, as the lean pass; W = 2: two slices, 16-B lanes).
// Prints TB/s of the modelled traffic (2 reads + 1 write per row).
//   hipcc --offload-arch=gfx950 -O3 bench/carry_pattern.hip -o build/carry_pattern && ./build/carry_pattern
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int W> struct Vec;
template <> struct Vec<1> { typedef double T; };
typedef double d2v __attribute__((ext_vector_type(2)));
template <> struct Vec<2> { typedef d2v T; };

__device__ __forceinline__ double add(double a, double b) { return a + 0.5 * b; }
__device__ __forceinline__ d2v add(d2v a, d2v b) { return a + 0.5 * b; }

// D-line chains rotated by renaming under a D-step unroll
// NT: non-temporal stores; OUTC: write a third buffer instead of overwriting pb (in place, as the pass)
template <int W, int D, bool NT = true, bool OUTC = false, bool NOST = false>
__global__ __launch_bounds__(256) void k_walk(const double* __restrict__ pa, double* __restrict__ pb, int64_t lines,
                                              int64_t line_len, int64_t runs, double* __restrict__ pc) {
  typedef typename Vec<W>::T T;
  const int lane = threadIdx.x & 63;
  const int64_t cols = line_len / (64 * W);
  const int64_t gw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (int64_t)gridDim.x * 4;
  const int64_t chunk = (lines + runs - 1) / runs;
  for (int64_t job = gw; job < cols * runs; job += nw) {
    const int64_t col = job % cols, l0 = (job / cols) * chunk;
    const int64_t l1 = l0 + chunk < lines ? l0 + chunk : lines;
    if (l1 - l0 <= D) continue;
    const T* a = reinterpret_cast<const T*>(pa + l0 * line_len + col * 64 * W) + lane;
    const T* b = reinterpret_cast<const T*>(pb + l0 * line_len + col * 64 * W) + lane;
    T* o = reinterpret_cast<T*>((OUTC ? pc : pb) + l0 * line_len + col * 64 * W) + lane;
    T acc = T{};
    const int64_t ls = line_len / W;  // one line, in T
    T qa[D], qb[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      qa[d] = a[d * ls];
      qb[d] = b[d * ls];
    }
    int64_t m = 0;
    const int64_t n = l1 - l0 - D;
    for (; m + D <= n; m += D) {
#pragma unroll
      for (int u = 0; u < D; ++u) {
        const T na = a[(m + u + D) * ls], nb = b[(m + u + D) * ls];
        if constexpr (NOST) acc = add(acc, add(qa[u], qb[u]));
        else if constexpr (NT) __builtin_nontemporal_store(add(qa[u], qb[u]), &o[(m + u) * ls]);
        else o[(m + u) * ls] = add(qa[u], qb[u]);
        qa[u] = na;
        qb[u] = nb;
      }
    }
    if constexpr (NOST) {
      if (lines < 0) o[0] = acc;  // keeps the loads
    }
  }
}

int main() {
  const int64_t line_len = 16384, lines = 16384, n = line_len * lines;
  double *a, *b, *c;
  CK(hipMalloc(&a, n * 8));
  CK(hipMalloc(&b, n * 8 + 4096));
  CK(hipMalloc(&c, n * 8 + 4096));
  CK(hipMemset(a, 0, n * 8));
  CK(hipMemset(b, 0, n * 8));
  CK(hipMemset(c, 0, n * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  auto run = [&](const char* name, auto kern, int bpc, int64_t cols, double streams = 3.0) {
    const int grid = ncu * bpc;
    const int64_t nw = (int64_t)grid * 4, runs = nw > cols ? nw / cols : 1;
    for (int it = 0; it < 2; ++it) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, a, b, lines, line_len, runs, c);
    hipEventRecord(e0);
    const int reps = 10;
    for (int it = 0; it < reps; ++it) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, a, b, lines, line_len, runs, c);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    printf("%-34s blocks/CU %2d  %.3f ms  %.2f TB/s\n", name, bpc, ms, streams * n * 8 / (ms * 1e-3) / 1e12);
    fflush(stdout);
  };
  for (int bpc : {8, 16}) {
    run("W=1 D=3 in place, nt", k_walk<1, 3>, bpc, line_len / 64);
    run("W=1 D=3 in place, plain stores", k_walk<1, 3, false>, bpc, line_len / 64);
    run("W=1 D=3 third buffer, nt", k_walk<1, 3, true, true>, bpc, line_len / 64);
    run("W=1 D=3 third buffer, plain", k_walk<1, 3, false, true>, bpc, line_len / 64);
    run("W=1 D=3 reads only (2R)", k_walk<1, 3, true, false, true>, bpc, line_len / 64, 2.0);
    run("W=2 D=3 in place, nt", k_walk<2, 3>, bpc, line_len / 128);
    run("W=2 D=3 third buffer, nt", k_walk<2, 3, true, true>, bpc, line_len / 128);
  }
  return 0;
}
