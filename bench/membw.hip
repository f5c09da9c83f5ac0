// HBM bandwidth ceilings on this MI355X for the access mixes the CG kernels use:
// read-only reduction, copy, "update" (2 reads + 1 write, like the residual
// update), each with 16-B lanes, several grid sizes and unroll depths.
//   hipcc --offload-arch=gfx950 -O3 bench/membw.hip -o build/membw && ./build/membw
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int UNR>
__global__ __launch_bounds__(256) void k_read(const double2* __restrict__ a, size_t n2, double* out) {
  double acc = 0;
  const size_t stride = (size_t)gridDim.x * 256;
  size_t k = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; k + (UNR - 1) * stride < n2; k += UNR * stride) {
    double2 v[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) v[u] = a[k + u * stride];
#pragma unroll
    for (int u = 0; u < UNR; ++u) acc += v[u].x + v[u].y;
  }
  if (acc == 12345.678) *out = acc;
}

template <int UNR>
__global__ __launch_bounds__(256) void k_copy(const double2* __restrict__ a, double2* __restrict__ b, size_t n2) {
  const size_t stride = (size_t)gridDim.x * 256;
  size_t k = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; k + (UNR - 1) * stride < n2; k += UNR * stride) {
    double2 v[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) v[u] = a[k + u * stride];
#pragma unroll
    for (int u = 0; u < UNR; ++u) b[k + u * stride] = v[u];
  }
}

template <int UNR>
__global__ __launch_bounds__(256) void k_update(double2* __restrict__ r, const double2* __restrict__ a, size_t n2,
                                                double* out) {
  double acc = 0;
  const size_t stride = (size_t)gridDim.x * 256;
  size_t k = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; k + (UNR - 1) * stride < n2; k += UNR * stride) {
    double2 v[UNR], w[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) { v[u] = r[k + u * stride]; w[u] = a[k + u * stride]; }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      v[u].x -= 0.5 * w[u].x; v[u].y -= 0.5 * w[u].y;
      r[k + u * stride] = v[u];
      acc += v[u].x * v[u].x + v[u].y * v[u].y;
    }
  }
  if (acc == 12345.678) *out = acc;
}

int main() {
  const size_t n = (size_t)1 << 28;  // doubles per array (2 GiB) = the 16384^2 vector size
  double *a, *b, *out;
  CK(hipMalloc(&a, n * 8));
  CK(hipMalloc(&b, n * 8));
  CK(hipMalloc(&out, 8));
  CK(hipMemset(a, 0, n * 8));
  CK(hipMemset(b, 0, n * 8));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const size_t n2 = n / 2;
  auto timeit = [&](auto launch, double bytes, const char* name, int grid, int unr) {
    launch();
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(e0);
      launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      best = ms < best ? ms : best;
    }
    printf("{\"kernel\": \"%s\", \"grid\": %d, \"unroll\": %d, \"ms\": %.4f, \"TB_s\": %.3f}\n", name, grid, unr,
           best, bytes / (best * 1e-3) / 1e12);
  };
  for (int bpc : {4, 8, 16, 32}) {
    const int grid = cus * bpc;
#define RUN(U)                                                                                                  \
  timeit([&] { hipLaunchKernelGGL(k_read<U>, dim3(grid), dim3(256), 0, 0, (const double2*)a, n2, out); }, n * 8.0, \
         "read", grid, U);                                                                                      \
  timeit([&] { hipLaunchKernelGGL(k_copy<U>, dim3(grid), dim3(256), 0, 0, (const double2*)a, (double2*)b, n2); },  \
         n * 16.0, "copy", grid, U);                                                                            \
  timeit([&] { hipLaunchKernelGGL(k_update<U>, dim3(grid), dim3(256), 0, 0, (double2*)b, (const double2*)a, n2, out); }, \
         n * 24.0, "update", grid, U);
    RUN(1) RUN(2) RUN(4)
  }
  return 0;
}
