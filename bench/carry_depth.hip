// Is the 4096^2 even pass latency-bound (bytes in flight per SIMD) or bound by its pattern?  The even
// three-term pass's memory pattern alone (every wave walks one 64-row slice column down its run of
// lines; per line step two vectors read D lines ahead, one written in place, bench/carry_pattern.hip)
// at the lean kernel's occupancy and geometry: 4096 x 4096, runs = waves / columns, waves per SIMD set
// by padding each block's LDS.  Two ways to keep lines in flight:
//   reg  D lines per vector in VGPRs (the lean kernel's chains)
//   glds an R-line ring per wave in LDS filled by LDS-DMA (global_load_lds_dwordx4: lanes 0-31 fetch
//        the line of a, lanes 32-63 the line of b, 1 KiB per step), counted vmcnt, ds_read_b64 per lane
// Prints TB/s of the modelled traffic (2 reads + 1 write per row).
//   hipcc --offload-arch=gfx950 -O3 bench/carry_depth.hip -o build/carry_depth && ./build/carry_depth
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

typedef __attribute__((address_space(3))) char lds_char;
typedef __attribute__((address_space(1))) char g_char;

template <int D>
__global__ __launch_bounds__(256) void k_reg(const double* __restrict__ pa, double* __restrict__ pb, int64_t lines,
                                             int64_t line_len, int64_t runs) {
  extern __shared__ char pad[];
  if (lines < 0) pad[threadIdx.x] = 0;  // the padding limits blocks per CU
  const int lane = threadIdx.x & 63;
  const int64_t cols = line_len / 64;
  const int64_t gw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (int64_t)gridDim.x * 4;
  const int64_t chunk = (lines + runs - 1) / runs;
  for (int64_t job = gw; job < cols * runs; job += nw) {
    const int64_t col = job % cols, l0 = (job / cols) * chunk;
    const int64_t l1 = l0 + chunk < lines ? l0 + chunk : lines;
    if (l1 - l0 <= D) continue;
    const double* a = pa + l0 * line_len + col * 64 + lane;
    double* b = pb + l0 * line_len + col * 64 + lane;
    double qa[D], qb[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      qa[d] = a[d * line_len];
      qb[d] = b[d * line_len];
    }
    int64_t m = 0;
    const int64_t n = l1 - l0 - D;
    for (; m + D <= n; m += D) {
#pragma unroll
      for (int u = 0; u < D; ++u) {
        const double na = a[(m + u + D) * line_len], nb = b[(m + u + D) * line_len];
        __builtin_nontemporal_store(qa[u] + 0.5 * qb[u], &b[(m + u) * line_len]);
        qa[u] = na;
        qb[u] = nb;
      }
    }
  }
}

// the reg pattern plus pieces of the real lean step (PIECES bits): 1 = an edge load per line (lanes 0 / 63,
// a compact 2-per-slice array, D lines ahead) and two edge-array stores (lanes 0 / 63, plain); 2 = the
// step's arithmetic shape: two dependent 5-FMA stencils with DPP lane shifts and four dot-product FMAs
template <int D, int PIECES>
__global__ __launch_bounds__(256) void k_step(const double* __restrict__ pa, double* __restrict__ pb, int64_t lines,
                                              int64_t line_len, int64_t runs, const double* __restrict__ ea,
                                              double* __restrict__ eb, double* __restrict__ out) {
  extern __shared__ char pad[];
  if (lines < 0) pad[threadIdx.x] = 0;
  const int lane = threadIdx.x & 63;
  const int64_t cols = line_len / 64;
  const int64_t gw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (int64_t)gridDim.x * 4;
  const int64_t chunk = (lines + runs - 1) / runs;
  const bool edge = lane == 0 || lane == 63;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0, carry = 0.0;
  for (int64_t job = gw; job < cols * runs; job += nw) {
    const int64_t col = job % cols, l0 = (job / cols) * chunk;
    const int64_t l1 = l0 + chunk < lines ? l0 + chunk : lines;
    if (l1 - l0 <= D) continue;
    const double* a = pa + l0 * line_len + col * 64 + lane;
    double* b = pb + l0 * line_len + col * 64 + lane;
    const int64_t es = 2 * cols;  // one line of the edge arrays
    const double* ex = ea + l0 * es + 2 * col + (lane == 63);
    double* ey = eb + l0 * es + 2 * col + (lane == 63);
    // the neighbouring slices' edge rows (inside the array: the first / last column reads its own row)
    const int nbo = lane == 0 ? (col == 0 ? 0 : -1) : (col == cols - 1 ? 0 : 1);
    double qa[D], qb[D], qe[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      qa[d] = a[d * line_len];
      qb[d] = b[d * line_len];
      if constexpr (PIECES & 16) qe[d] = edge ? a[d * line_len + nbo] : 0.0;
      else if constexpr (PIECES & 1) qe[d] = edge ? ex[d * es] : 0.0;
    }
    int64_t m = 0;
    const int64_t n = l1 - l0 - D;
    for (; m + D <= n; m += D) {
#pragma unroll
      for (int u = 0; u < D; ++u) {
        const double na = a[(m + u + D) * line_len], nb = b[(m + u + D) * line_len];
        double ne = 0.0;
        if constexpr (PIECES & 16) ne = edge ? a[(m + u + D) * line_len + nbo] : 0.0;
        else if constexpr (PIECES & 1) ne = edge ? ex[(m + u + D) * es] : 0.0;
        double v = qa[u] + 0.5 * qb[u];
        if constexpr (PIECES & 2) {
          const double up = __shfl_down(qa[u], 1), dn = __shfl_up(qa[u], 1);
          double t = fma(0.25, dn, 0.0);
          t = fma(0.25, up, t);
          t = fma(-1.0, qa[u], t);
          t = fma(0.25, carry, t);
          t = fma(0.25, qb[u], t);
          const double pk = fma(0.5, qa[u], fma(-0.1, t, qb[u]));
          const double up2 = __shfl_down(pk, 1), dn2 = __shfl_up(pk, 1);
          double w = fma(0.25, dn2, 0.0);
          w = fma(0.25, up2, w);
          w = fma(-1.0, pk, w);
          w = fma(0.25, v, w);
          w = fma(0.25, carry, w);
          s0 = fma(pk, w, s0);
          s1 = fma(t, w, s1);
          s2 = fma(w, w, s2);
          s3 = fma(t, t, s3);
          carry = pk;
          v = pk;
        }
        if constexpr (PIECES & 1) {
          v += qe[u];
          if constexpr ((PIECES & 4) == 0) {  // the lean kernel's layout: r / Ap of the slice's two edge rows
            if (edge) {                       // in two compact arrays, 2 doubles per slice (16 B partial sectors)
              ey[(m + u) * es] = v;
              if constexpr ((PIECES & 32) == 0) ey[(m + u) * es + es / 2] = v;  // 32: only one of them
            }
          } else if constexpr ((PIECES & 8) == 0) {  // merged: [r_lo, ap_lo, r_hi, ap_hi] = one 32-B sector per
            if (edge) {                               // slice and line, written whole by one store instruction
              typedef double d2 __attribute__((ext_vector_type(2)));
              *(d2*)(eb + (l0 + m + u) * 2 * es + 4 * col + 2 * (lane == 63)) = d2{v, v};
            }
          }
          qe[u] = ne;
        }
        __builtin_nontemporal_store(v, &b[(m + u) * line_len]);
        qa[u] = na;
        qb[u] = nb;
      }
    }
  }
  if (s0 + s1 + s2 + s3 == 12345.0) out[0] = 1.0;
}

// R-line ring per wave: slot s = 1 KiB ([a line | b line]); wave-private, no barriers
template <int R>
__global__ __launch_bounds__(256) void k_glds(const double* __restrict__ pa, double* __restrict__ pb, int64_t lines,
                                              int64_t line_len, int64_t runs) {
  extern __shared__ char smem[];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  lds_char* ring = (lds_char*)smem + wv * R * 1024;
  const int64_t cols = line_len / 64;
  const int64_t gw = (int64_t)blockIdx.x * 4 + wv, nw = (int64_t)gridDim.x * 4;
  const int64_t chunk = (lines + runs - 1) / runs;
  for (int64_t job = gw; job < cols * runs; job += nw) {
    const int64_t col = job % cols, l0 = (job / cols) * chunk;
    const int64_t l1 = l0 + chunk < lines ? l0 + chunk : lines;
    if (l1 - l0 <= R) continue;
    // lane l < 32 fetches 16 B of a's line, lane l >= 32 16 B of b's
    const double* src0 = (lane < 32 ? pa : (const double*)pb) + l0 * line_len + col * 64 + 2 * (lane & 31);
    double* b = pb + l0 * line_len + col * 64 + lane;
    auto fetch = [&](int64_t j, int slot) {
      __builtin_amdgcn_global_load_lds((const g_char*)(const void*)(src0 + j * line_len), ring + slot * 1024, 16, 0, 0);
    };
#pragma unroll
    for (int d = 0; d < R; ++d) fetch(d, d);
    const int64_t n = l1 - l0 - R;
    int64_t m = 0;
    for (; m + R <= n; m += R) {
#pragma unroll
      for (int u = 0; u < R; ++u) {
        // slot u's fetch is older than the R - 1 fetches and R - 1 stores issued since (steady state;
        // in the first round only the R - 1 prologue fetches are certain): all but those complete
        if (m == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(R - 1) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (R - 1)) : "memory");
        const double va = *(const double*)(ring + u * 1024 + 8 * lane);
        const double vb = *(const double*)(ring + u * 1024 + 512 + 8 * lane);
        __builtin_nontemporal_store(va + 0.5 * vb, &b[(m + u) * line_len]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot u read before it is refilled
        fetch(m + u + R, u);
      }
    }
  }
}

int main(int argc, char** argv) {
  // argv[1]: grid edge (default 4096); argv[2] == "steps": only the lean-step piece variants
  const int64_t line_len = argc > 1 ? std::atoi(argv[1]) : 4096, lines = line_len, n = line_len * lines;
  const bool steps_only = argc > 2 && argv[2][0] == 's';
  double *a, *b;
  CK(hipMalloc(&a, n * 8));
  CK(hipMalloc(&b, n * 8 + 4096));
  CK(hipMemset(a, 0, n * 8));
  CK(hipMemset(b, 0, n * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  auto run = [&](const char* name, auto kern, int wps, size_t lds_need) -> int {
    // blocks per CU = waves per SIMD (4 waves per block): pad each block's LDS to 160 KiB / wps
    const size_t lds = std::max<size_t>(lds_need, (size_t)(163840 / wps) & ~(size_t)1023);
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const int grid = ncu * wps;
    const int64_t nw = (int64_t)grid * 4, cols = line_len / 64, runs = nw > cols ? nw / cols : 1;
    for (int it = 0; it < 3; ++it) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, 0, a, b, lines, line_len, runs);
    CK(hipGetLastError());
    hipEventRecord(e0);
    const int reps = 50;
    for (int it = 0; it < reps; ++it) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, 0, a, b, lines, line_len, runs);
    hipEventRecord(e1);
    CK(hipEventSynchronize(e1));
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    printf("{\"variant\": \"%s\", \"waves_per_simd\": %d, \"lds\": %zu, \"us\": %.2f, \"tbps\": %.3f}\n", name, wps, lds,
           1e3 * ms, 3.0 * n * 8 / (ms * 1e-3) / 1e12);
    fflush(stdout);
    return 0;
  };
  for (int wps : {4, 5, 8}) {
    if (steps_only) break;
    if (run("reg D=3", k_reg<3>, wps, 0)) return 1;
    if (run("reg D=4", k_reg<4>, wps, 0)) return 1;
    if (run("reg D=6", k_reg<6>, wps, 0)) return 1;
  }
  double *ea, *eb;
  const int64_t ne = 2 * (line_len / 64) * lines;
  CK(hipMalloc(&ea, ne * 8));
  CK(hipMalloc(&eb, 2 * ne * 8 + 4096));
  CK(hipMemset(ea, 0, ne * 8));
  auto runs_ = [&](const char* name, auto kern, int wps) -> int {
    const size_t lds = (size_t)(163840 / wps) & ~(size_t)1023;
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const int grid = ncu * wps;
    const int64_t nw = (int64_t)grid * 4, cols = line_len / 64, runs = nw > cols ? nw / cols : 1;
    for (int it = 0; it < 3; ++it)
      hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, 0, a, b, lines, line_len, runs, ea, eb, eb + 2 * ne);
    CK(hipGetLastError());
    hipEventRecord(e0);
    const int reps = 50;
    for (int it = 0; it < reps; ++it)
      hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, 0, a, b, lines, line_len, runs, ea, eb, eb + 2 * ne);
    hipEventRecord(e1);
    CK(hipEventSynchronize(e1));
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    printf("{\"variant\": \"%s\", \"waves_per_simd\": %d, \"us\": %.2f, \"tbps\": %.3f}\n", name, wps, 1e3 * ms,
           3.0 * n * 8 / (ms * 1e-3) / 1e12);
    fflush(stdout);
    return 0;
  };
  for (int wps : {5, 8}) {
    if (runs_("step D=3 pieces 0", k_step<3, 0>, wps)) return 1;
    if (runs_("step D=3 edges", k_step<3, 1>, wps)) return 1;
    if (runs_("step D=3 arithmetic", k_step<3, 2>, wps)) return 1;
    if (runs_("step D=3 edges+arithmetic", k_step<3, 3>, wps)) return 1;
    if (runs_("step D=6 edges+arithmetic", k_step<6, 3>, wps)) return 1;
    if (runs_("step D=3 edge loads, no stores", k_step<3, 13>, wps)) return 1;
    if (runs_("step D=3 edges+arith, one store", k_step<3, 32 | 2 | 1>, wps)) return 1;
    if (runs_("step D=3 neighbour-row loads, no stores", k_step<3, 16 | 8 | 4 | 1>, wps)) return 1;
    if (runs_("step D=3 neighbour-row loads+arith, no stores", k_step<3, 16 | 8 | 4 | 2 | 1>, wps)) return 1;
    if (runs_("step D=4 neighbour-row loads+arith, no stores", k_step<4, 16 | 8 | 4 | 2 | 1>, wps)) return 1;
    if (runs_("step D=3 edges, merged 32-B sectors", k_step<3, 5>, wps)) return 1;
    if (runs_("step D=3 edges+arith, merged", k_step<3, 7>, wps)) return 1;
    if (runs_("step D=6 edges+arith, merged", k_step<6, 7>, wps)) return 1;
  }
  for (int wps : {4, 5}) {
    if (steps_only) break;
    if (run("glds R=4", k_glds<4>, wps, 4 * 4 * 1024)) return 1;
    if (run("glds R=6", k_glds<6>, wps, 4 * 6 * 1024)) return 1;
    if (run("glds R=8", k_glds<8>, wps, 4 * 8 * 1024)) return 1;
  }
  return 0;
}
