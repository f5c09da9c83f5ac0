// Is the ~10 % run-to-run bimodality of the CG benches (e.g. 3-D 497-505 vs 545-551 it/s in
// separate processes on one box) a property of the process or of the allocation?
// One process: several allocation sets of 3 x 2 GiB; on each, a read-only stream per array and an
// "update" stream kernel (2 reads + 1 write of 16-B lanes) are timed.  Sets are kept alive (new
// physical memory each time), then half are freed and re-allocated.  Mode "arena": the three
// arrays of a set are carved from one 6 GiB allocation; mode "spacer": a spacer allocation of
// (set index + 1) x 6 MiB precedes each array.
//   hipcc --offload-arch=gfx950 -O3 bench/mode_probe.hip -o build/mode_probe && ./build/mode_probe [sep|arena|spacer]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
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

__global__ __launch_bounds__(256) void k_read(const double2* __restrict__ a, size_t n2, double* out) {
  const size_t stride = (size_t)gridDim.x * 256;
  double acc = 0.0;
  for (size_t k = (size_t)blockIdx.x * 256 + threadIdx.x; k < n2; k += stride) acc += a[k].x + a[k].y;
  if (acc == 12345.678) *out = acc;
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "sep";
  const size_t n = (size_t)1 << 28;  // doubles per array (2 GiB)
  const size_t n2 = n / 2;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  double* out = nullptr;
  CK(hipMalloc(&out, 8));
  struct Set { double *a, *b, *c; std::vector<void*> extra; };
  std::vector<Set> sets;
  auto alloc = [&](Set& s, int idx) -> int {
    if (!strcmp(mode, "arena")) {
      double* base = nullptr;
      CK(hipMalloc(&base, 3 * n * 8));
      s.a = base;
      s.b = base + n;
      s.c = base + 2 * n;
      s.extra.push_back(base);
    } else {
      double** dst[3] = {&s.a, &s.b, &s.c};
      for (int i = 0; i < 3; ++i) {
        if (!strcmp(mode, "spacer")) {
          void* sp = nullptr;
          CK(hipMalloc(&sp, (size_t)(idx + 1) * (6u << 20)));
          s.extra.push_back(sp);
        }
        CK(hipMalloc(dst[i], n * 8));
        s.extra.push_back(*dst[i]);
      }
    }
    CK(hipMemset(s.a, 0, n * 8));
    CK(hipMemset(s.b, 0, n * 8));
    CK(hipMemset(s.c, 0, n * 8));
    return 0;
  };
  auto best_ms = [&](auto launch) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      (void)hipEventRecord(e0);
      launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      best = ms < best ? ms : best;
    }
    return best;
  };
  auto measure = [&](const Set& s, const char* tag, int i) -> int {
    const int grid = cus * 8;
    double rd[3];
    const double* arr[3] = {s.a, s.b, s.c};
    for (int q = 0; q < 3; ++q) {
      const float ms = best_ms([&] {
        hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, (const double2*)arr[q], n2, out);
      });
      rd[q] = n * 8.0 / (ms * 1e-3) / 1e12;
    }
    const float ms = best_ms([&] {
      hipLaunchKernelGGL(k_update, dim3(grid), dim3(256), 0, 0, (double2*)s.c, (const double2*)s.a,
                         (const double2*)s.b, n2);
    });
    printf("{\"mode\": \"%s\", \"phase\": \"%s\", \"set\": %d, \"read_TB_s\": [%.3f, %.3f, %.3f], \"update_TB_s\": %.3f}\n",
           mode, tag, i, rd[0], rd[1], rd[2], n * 24.0 / (ms * 1e-3) / 1e12);
    fflush(stdout);
    return 0;
  };
  if (!strcmp(mode, "skew")) {
    // one allocation per array with 8 MiB of slack; b and c start at byte offsets sb, sc into
    // theirs: does the update stream's speed depend on the relative offsets (same pages)?
    const size_t slack = (size_t)8 << 20;
    char *a, *b, *c;
    CK(hipMalloc(&a, n * 8 + slack));
    CK(hipMalloc(&b, n * 8 + slack));
    CK(hipMalloc(&c, n * 8 + slack));
    CK(hipMemset(a, 0, n * 8 + slack));
    CK(hipMemset(b, 0, n * 8 + slack));
    CK(hipMemset(c, 0, n * 8 + slack));
    const size_t sk[] = {0, 4096, 32768, 262144, 1 << 20, 3 << 20, (3 << 20) + 65536};
    for (int rep = 0; rep < 2; ++rep)
      for (size_t sb : sk) {
        printf("{\"sb\": %zu, \"update_TB_s\": [", sb);
        for (size_t sc : sk) {
          const float ms = best_ms([&] {
            hipLaunchKernelGGL(k_update, dim3(cus * 8), dim3(256), 0, 0, (double2*)(c + sc), (const double2*)a,
                               (const double2*)(b + sb), n2);
          });
          printf("%s%.3f", sc ? ", " : "", n * 24.0 / (ms * 1e-3) / 1e12);
        }
        printf("]}\n");
        fflush(stdout);
      }
    return 0;
  }
  for (int i = 0; i < 6; ++i) {
    sets.push_back({});
    if (alloc(sets.back(), i)) return 1;
    if (measure(sets.back(), "fresh", i)) return 1;
  }
  for (int i = 0; i < 6; i += 2) {
    for (void* p : sets[i].extra) CK(hipFree(p));
    sets[i].extra.clear();
  }
  for (int i = 0; i < 6; i += 2) {
    if (alloc(sets[i], i)) return 1;
    if (measure(sets[i], "realloc", i)) return 1;
  }
  return 0;
}
