// Is the ~10 % run-to-run bimodality of the CG benches (e.g. 3-D 497-505 vs 545-551 it/s in
// separate processes on one box, profiles/) a property of the process or of the allocation?
// One process: several allocation sets of 3 x 2 GiB, an "update" stream kernel (2 reads + 1
// write of 16-B lanes) timed on each; sets are kept alive (new physical memory each time), then
// half are freed and re-allocated.
//   hipcc --offload-arch=gfx950 -O3 bench/mode_probe.hip -o build/mode_probe && ./build/mode_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ __launch_bounds__(256) void k_update(double2* __restrict__ c, const double2* __restrict__ a,
                                                const double2* __restrict__ b, size_t n2) {
  const size_t stride = (size_t)gridDim.x * 256;
  for (size_t k = (size_t)blockIdx.x * 256 + threadIdx.x; k < n2; k += stride) {
    const double2 x = a[k], y = b[k];
    c[k] = make_double2(x.x + 0.5 * y.x, x.y + 0.5 * y.y);
  }
}

int main() {
  const size_t n = (size_t)1 << 28;  // doubles per array (2 GiB)
  const size_t n2 = n / 2;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct Set { double *a, *b, *c; };
  std::vector<Set> sets;
  auto alloc = [&](Set& s) -> int {
    CK(hipMalloc(&s.a, n * 8));
    CK(hipMalloc(&s.b, n * 8));
    CK(hipMalloc(&s.c, n * 8));
    CK(hipMemset(s.a, 0, n * 8));
    CK(hipMemset(s.b, 0, n * 8));
    CK(hipMemset(s.c, 0, n * 8));
    return 0;
  };
  auto measure = [&](const Set& s, const char* tag, int i) -> int {
    const int grid = cus * 8;
    float best = 1e30f;
    for (int rep = 0; rep < 6; ++rep) {
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(k_update, dim3(grid), dim3(256), 0, 0, (double2*)s.c, (const double2*)s.a,
                         (const double2*)s.b, n2);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    printf("{\"phase\": \"%s\", \"set\": %d, \"a\": \"%p\", \"TB_s\": %.3f}\n", tag, i, (void*)s.a,
           n * 24.0 / (best * 1e-3) / 1e12);
    fflush(stdout);
    return 0;
  };
  for (int i = 0; i < 6; ++i) {
    sets.push_back({});
    if (alloc(sets.back())) return 1;
    if (measure(sets.back(), "fresh", i)) return 1;
  }
  for (int i = 0; i < 6; ++i)
    if (measure(sets[i], "again", i)) return 1;
  for (int i = 0; i < 6; i += 2) {
    CK(hipFree(sets[i].a));
    CK(hipFree(sets[i].b));
    CK(hipFree(sets[i].c));
  }
  for (int i = 0; i < 6; i += 2) {
    if (alloc(sets[i])) return 1;
    if (measure(sets[i], "realloc", i)) return 1;
  }
  return 0;
}
