// On-device matrix/RHS generation for each rank's owned rows (SURVEY.md §2.7
// N1-N4): count -> scan -> fill, so a 200 GB/GPU matrix never passes through
// host memory (the reference builds its 3x3 matrix on the host and copies it,
// CUDACG.cu:93-134).  Also CSR -> SELL-64 conversion.
#include <hip/hip_runtime.h>

#include "mcg/check.hpp"
#include "mcg/kernels.hpp"

namespace mcg {
namespace kern {

namespace {

constexpr int kGenBlock = 256;
constexpr int kScanItems = 16;                       // items per thread
constexpr int kScanChunk = kGenBlock * kScanItems;   // 4096 items per block

__global__ __launch_bounds__(kGenBlock) void k_rowlen(ProblemSpec s, int64_t row_begin, int64_t n,
                                                      int64_t* __restrict__ rowptr) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    rowptr[i + 1] = row_length(s, row_begin + i);
  if (blockIdx.x == 0 && threadIdx.x == 0) rowptr[0] = 0;
}

// block-wide inclusive scan of one value per thread (256 threads), returns the
// inclusive prefix for this thread and writes the block total to *total.
__device__ int64_t block_scan_inclusive(int64_t v, int64_t* sh, int64_t* total) {
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int off = 1; off < kGenBlock; off <<= 1) {
    const int64_t add = t >= off ? sh[t - off] : 0;
    __syncthreads();
    sh[t] += add;
    __syncthreads();
  }
  const int64_t r = sh[t];
  if (total) *total = sh[kGenBlock - 1];
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(kGenBlock) void k_scan_blocksums(const int64_t* __restrict__ a,
                                                              int64_t n, int64_t* __restrict__ sums) {
  __shared__ int64_t sh[kGenBlock];
  const int64_t base = (int64_t)blockIdx.x * kScanChunk + (int64_t)threadIdx.x * kScanItems;
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k)
    if (base + k < n) s += a[base + k];
  int64_t tot;
  block_scan_inclusive(s, sh, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// single block: exclusive scan of nb block sums in place
__global__ __launch_bounds__(kGenBlock) void k_scan_sums(int64_t* __restrict__ sums, int64_t nb) {
  __shared__ int64_t sh[kGenBlock];
  const int64_t per = (nb + kGenBlock - 1) / kGenBlock;
  const int64_t b0 = threadIdx.x * per;
  int64_t s = 0;
  for (int64_t k = 0; k < per; ++k)
    if (b0 + k < nb) s += sums[b0 + k];
  const int64_t incl = block_scan_inclusive(s, sh, nullptr);
  int64_t run = incl - s;
  for (int64_t k = 0; k < per; ++k)
    if (b0 + k < nb) {
      const int64_t v = sums[b0 + k];
      sums[b0 + k] = run;
      run += v;
    }
}

__global__ __launch_bounds__(kGenBlock) void k_scan_apply(int64_t* __restrict__ a, int64_t n,
                                                          const int64_t* __restrict__ sums) {
  __shared__ int64_t sh[kGenBlock];
  const int64_t base = (int64_t)blockIdx.x * kScanChunk + (int64_t)threadIdx.x * kScanItems;
  int64_t v[kScanItems];
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    v[k] = (base + k < n) ? a[base + k] : 0;
    s += v[k];
  }
  const int64_t incl = block_scan_inclusive(s, sh, nullptr);
  int64_t run = sums[blockIdx.x] + incl - s;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    run += v[k];
    if (base + k < n) a[base + k] = run;
  }
}

template <typename IdxT>
__global__ __launch_bounds__(kGenBlock) void k_fill(ProblemSpec s, int64_t row_begin, int64_t n,
                                                    int64_t col_lo, int64_t pad,
                                                    const int64_t* __restrict__ rp64,
                                                    IdxT* __restrict__ rp_out,
                                                    int32_t* __restrict__ cols,
                                                    double* __restrict__ vals) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    int64_t k = rp64[i];
    const int64_t len = rp64[i + 1] - k;
    if (rp_out) {
      rp_out[i] = (IdxT)k;
      if (i == n - 1) rp_out[n] = (IdxT)rp64[n];
    }
    for_each_entry(s, row_begin + i, [&](int64_t c, double v) {
      cols[k] = (int32_t)(c - col_lo + pad);
      vals[k] = v;
      ++k;
    }, len);
  }
}

__global__ __launch_bounds__(kGenBlock) void k_rhs(ProblemSpec s, int64_t row_begin, int64_t n,
                                                   double* __restrict__ b) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    b[i] = rhs_value(s, row_begin + i);
}

// one thread per 64-row slice: slice_ptr[s+1] = 64 * max row length
__global__ __launch_bounds__(kGenBlock) void k_sell_widths(const int64_t* __restrict__ rp, int64_t n,
                                                           int64_t* __restrict__ sp) {
  const int64_t ns = (n + 63) / 64;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t sl = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; sl < ns; sl += stride) {
    int64_t w = 0;
    const int64_t r1 = (sl + 1) * 64 < n ? (sl + 1) * 64 : n;
    for (int64_t r = sl * 64; r < r1; ++r) {
      const int64_t len = rp[r + 1] - rp[r];
      w = len > w ? len : w;
    }
    sp[sl + 1] = 64 * w;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) sp[0] = 0;
}

template <typename IdxT>
__global__ __launch_bounds__(kGenBlock) void k_csr_to_sell(const IdxT* __restrict__ rp,
                                                           const int32_t* __restrict__ cols,
                                                           const double* __restrict__ vals, int64_t n,
                                                           int64_t own_off, const int64_t* __restrict__ sp,
                                                           int32_t* __restrict__ scols,
                                                           double* __restrict__ svals,
                                                           int16_t* __restrict__ dcols) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n_pad = (n + 63) / 64 * 64;  // lanes past the last row of the last slice get padding too
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_pad; i += stride) {
    const int64_t sl = i >> 6, l = i & 63;
    const int64_t base = sp[sl], w = (sp[sl + 1] - base) >> 6;
    const bool row = i < n;
    const int64_t rs = row ? (int64_t)rp[i] : 0, len = row ? (int64_t)rp[i + 1] - rs : 0;
    const int64_t own_col = own_off + (row ? i : n - 1);  // a valid ext column for padding gathers
    for (int64_t j = 0; j < w; ++j) {
      const int64_t dst = base + 64 * j + l;
      const int32_t c = j < len ? cols[rs + j] : (int32_t)own_col;  // padding: valid column, value 0
      if (dcols) dcols[dst] = (int16_t)(c - (own_off + i));
      else scols[dst] = c;
      svals[dst] = j < len ? vals[rs + j] : 0.0;
    }
  }
}

// direct SELL-64 fill: one thread per padded row, entries generated in the same order as
// k_fill (so the SELL matrix equals the CSR -> SELL conversion entry for entry)
__global__ __launch_bounds__(kGenBlock) void k_fill_sell(ProblemSpec s, int64_t row_begin, int64_t n, int64_t col_lo,
                                                         int64_t pad, int64_t own_off,
                                                         const int64_t* __restrict__ rp64,
                                                         const int64_t* __restrict__ sp,
                                                         int32_t* __restrict__ scols, int16_t* __restrict__ dcols,
                                                         double* __restrict__ svals) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n_pad = (n + 63) / 64 * 64;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_pad; i += stride) {
    const int64_t sl = i >> 6, l = i & 63;
    const int64_t base = sp[sl], w = (sp[sl + 1] - base) >> 6;
    const bool row = i < n;
    const int64_t len = row ? rp64[i + 1] - rp64[i] : 0;
    const int64_t own_col = own_off + (row ? i : n - 1);  // a valid ext column for padding gathers
    int64_t j = 0;
    if (row)
      for_each_entry(s, row_begin + i, [&](int64_t c, double v) {
        const int64_t dst = base + 64 * j + l;
        const int64_t ec = c - col_lo + pad;
        if (dcols) dcols[dst] = (int16_t)(ec - (own_off + i));
        else scols[dst] = (int32_t)ec;
        svals[dst] = v;
        ++j;
      }, len);
    for (; j < w; ++j) {
      const int64_t dst = base + 64 * j + l;
      if (dcols) dcols[dst] = (int16_t)(own_col - (own_off + i));
      else scols[dst] = (int32_t)own_col;
      svals[dst] = 0.0;
    }
  }
}

// SELL-64/aligned (wide random SPD): candidate t reaches the matrix from some row of the slice
// [g0, g0 + 64) (global rows, g0 + 63 clamped to n - 1) iff d_t <= g1 (lower) / d_t <= n - 1 - g0 (upper)
__device__ __forceinline__ void aligned_counts(const ProblemSpec& s, int64_t g0, int64_t g1, int64_t& nlo,
                                               int64_t& nhi) {
  const int64_t n = s.rows, W = s.band;
  nlo = 0;
  nhi = 0;
  for (int64_t t = 0; t < W; ++t) {  // d_t increases with t
    const int64_t d = randspd_offset(s, t);
    if (d <= g1) nlo = t + 1;
    if (d <= n - 1 - g0) nhi = t + 1;
  }
}

__global__ __launch_bounds__(kGenBlock) void k_aligned_widths(ProblemSpec s, int64_t row_begin, int64_t n,
                                                              int64_t* __restrict__ sp) {
  const int64_t ns = (n + 63) / 64;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t sl = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; sl < ns; sl += stride) {
    const int64_t g0 = row_begin + sl * 64, g1 = row_begin + ((sl + 1) * 64 < n ? (sl + 1) * 64 : n) - 1;
    int64_t nlo, nhi;
    aligned_counts(s, g0, g1, nlo, nhi);
    sp[sl + 1] = 64 * (nlo + 1 + nhi);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) sp[0] = 0;
}

// one thread per padded row; slots in ascending column order (lower candidates descending, the
// diagonal, upper ascending): the same entries in the same order as k_fill_sell, plus zeros
__global__ __launch_bounds__(kGenBlock) void k_fill_aligned(ProblemSpec s, int64_t row_begin, int64_t n,
                                                            const int64_t* __restrict__ rp64,
                                                            const int64_t* __restrict__ sp,
                                                            int32_t* __restrict__ soffs, double* __restrict__ svals) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n_pad = (n + 63) / 64 * 64, N = s.rows;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_pad; i += stride) {
    const int64_t sl = i >> 6, l = i & 63;
    const int64_t base = sp[sl], w = (sp[sl + 1] - base) >> 6;
    const int64_t g0 = row_begin + sl * 64, g1 = row_begin + ((sl + 1) * 64 < n ? (sl + 1) * 64 : n) - 1;
    int64_t nlo, nhi;
    aligned_counts(s, g0, g1, nlo, nhi);
    const bool row = i < n;
    const int64_t g = row_begin + i;
    for (int64_t j = 0; j < w; ++j) {
      int64_t o;
      double v = 0.0;
      if (j < nlo) {  // lower candidate t = nlo - 1 - j
        o = -randspd_offset(s, nlo - 1 - j);
        const int64_t c = g + o;
        if (row && c >= 0 && randspd_present(s, c, g)) v = -randspd_weight(s, c, g);
      } else if (j == nlo) {
        o = 0;
        if (row) v = (double)(rp64[i + 1] - rp64[i]);  // diagonal = row length (problem.hpp)
      } else {  // upper candidate t = j - nlo - 1
        o = randspd_offset(s, j - nlo - 1);
        const int64_t c = g + o;
        if (row && c < N && randspd_present(s, g, c)) v = -randspd_weight(s, g, c);
      }
      if (l == 0) soffs[(base >> 6) + j] = (int32_t)o;
      svals[base + 64 * j + l] = v;
    }
  }
}

__global__ __launch_bounds__(kGenBlock) void k_max_i64(const int64_t* __restrict__ a, int64_t n,
                                                       unsigned long long* __restrict__ out) {
  int64_t m = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) m = a[i] > m ? a[i] : m;
  for (int off = 32; off > 0; off >>= 1) {
    const int64_t o = __shfl_down(m, off, 64);
    m = o > m ? o : m;
  }
  if ((threadIdx.x & 63) == 0) atomicMax(out, (unsigned long long)m);
}

int gen_grid(int64_t n) {
  int64_t g = (n + kGenBlock - 1) / kGenBlock;
  const int64_t cap = (int64_t)num_cus() * 16;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

int num_cus() {
  static int cached = -1;
  if (cached < 0) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
      cached = prop.multiProcessorCount;
    else
      cached = 256;
  }
  return cached;
}

int grid_for(int64_t work_items, int block, int blocks_per_cu) {
  int64_t g = (work_items + block - 1) / block;
  const int64_t cap = (int64_t)num_cus() * blocks_per_cu;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

void gen_rowlen(const ProblemSpec& s, int64_t row_begin, int64_t n, int64_t* rowptr, hipStream_t st) {
  hipLaunchKernelGGL(k_rowlen, dim3(gen_grid(n)), dim3(kGenBlock), 0, st, s, row_begin, n, rowptr);
  MCG_HIP(hipGetLastError(), "kernel launch failed(gen_rowlen)");
}

int64_t scan_tmp_elems(int64_t n) { return (n + kScanChunk - 1) / kScanChunk + 1; }

void scan_inclusive_i64(int64_t* a, int64_t n, int64_t* tmp, hipStream_t st) {
  if (n <= 0) return;
  const int64_t nb = (n + kScanChunk - 1) / kScanChunk;
  MCG_CHECK(nb < (int64_t)1 << 31, "scan too large");
  hipLaunchKernelGGL(k_scan_blocksums, dim3((unsigned)nb), dim3(kGenBlock), 0, st, a, n, tmp);
  hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(kGenBlock), 0, st, tmp, nb);
  hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)nb), dim3(kGenBlock), 0, st, a, n, tmp);
  MCG_HIP(hipGetLastError(), "kernel launch failed(scan)");
}

template <typename IdxT>
void gen_fill(const ProblemSpec& s, int64_t row_begin, int64_t n, int64_t col_lo, int64_t pad,
              const int64_t* rowptr64, IdxT* rowptr_out, int32_t* cols, double* vals, hipStream_t st) {
  hipLaunchKernelGGL(k_fill<IdxT>, dim3(gen_grid(n)), dim3(kGenBlock), 0, st, s, row_begin, n, col_lo,
                     pad, rowptr64, rowptr_out, cols, vals);
  MCG_HIP(hipGetLastError(), "kernel launch failed(gen_fill)");
}
template void gen_fill<int32_t>(const ProblemSpec&, int64_t, int64_t, int64_t, int64_t, const int64_t*,
                                int32_t*, int32_t*, double*, hipStream_t);
template void gen_fill<int64_t>(const ProblemSpec&, int64_t, int64_t, int64_t, int64_t, const int64_t*,
                                int64_t*, int32_t*, double*, hipStream_t);

void gen_rhs(const ProblemSpec& s, int64_t row_begin, int64_t n, double* b, hipStream_t st) {
  hipLaunchKernelGGL(k_rhs, dim3(gen_grid(n)), dim3(kGenBlock), 0, st, s, row_begin, n, b);
  MCG_HIP(hipGetLastError(), "kernel launch failed(gen_rhs)");
}

int64_t max_i64(const int64_t* a, int64_t n, hipStream_t st) {
  unsigned long long* d = nullptr;
  MCG_HIP(hipMallocAsync(reinterpret_cast<void**>(&d), sizeof(unsigned long long), st), "device malloc failed(max)");
  MCG_HIP(hipMemsetAsync(d, 0, sizeof(unsigned long long), st), "device memset failed");
  if (n > 0) hipLaunchKernelGGL(k_max_i64, dim3(gen_grid(n)), dim3(kGenBlock), 0, st, a, n, d);
  unsigned long long h = 0;
  MCG_HIP(hipMemcpyAsync(&h, d, sizeof(h), hipMemcpyDeviceToHost, st), "memcpy from device to host failed");
  MCG_HIP(hipStreamSynchronize(st), "device synchronize failed");
  (void)hipFreeAsync(d, st);
  return (int64_t)h;
}

void gen_fill_sell(const ProblemSpec& s, int64_t row_begin, int64_t n, int64_t col_lo, int64_t pad, int64_t own_off,
                   const int64_t* rowptr64, const int64_t* slice_ptr, int32_t* scols, int16_t* dcols, double* svals,
                   hipStream_t st) {
  if (n <= 0) return;
  MCG_CHECK((scols == nullptr) != (dcols == nullptr), "gen_fill_sell: exactly one column array");
  hipLaunchKernelGGL(k_fill_sell, dim3(gen_grid(n)), dim3(kGenBlock), 0, st, s, row_begin, n, col_lo, pad, own_off,
                     rowptr64, slice_ptr, scols, dcols, svals);
  MCG_HIP(hipGetLastError(), "kernel launch failed(gen_fill_sell)");
}

void randspd_aligned_widths(const ProblemSpec& s, int64_t row_begin, int64_t n, int64_t* slice_ptr,
                            hipStream_t st) {
  MCG_CHECK(s.kind == ProblemKind::RandomSPD, "aligned SELL: random-SPD family only");
  const int64_t ns = (n + 63) / 64;
  if (ns == 0) return;
  hipLaunchKernelGGL(k_aligned_widths, dim3(gen_grid(ns)), dim3(kGenBlock), 0, st, s, row_begin, n, slice_ptr);
  MCG_HIP(hipGetLastError(), "kernel launch failed(aligned_widths)");
}

void randspd_fill_aligned(const ProblemSpec& s, int64_t row_begin, int64_t n, const int64_t* rowptr64,
                          const int64_t* slice_ptr, int32_t* soffs, double* svals, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_fill_aligned, dim3(gen_grid(n)), dim3(kGenBlock), 0, st, s, row_begin, n, rowptr64, slice_ptr,
                     soffs, svals);
  MCG_HIP(hipGetLastError(), "kernel launch failed(fill_aligned)");
}

void sell_slice_widths(const int64_t* rowptr64, int64_t n, int64_t* slice_ptr, hipStream_t st) {
  const int64_t ns = (n + 63) / 64;
  hipLaunchKernelGGL(k_sell_widths, dim3(gen_grid(ns)), dim3(kGenBlock), 0, st, rowptr64, n, slice_ptr);
  MCG_HIP(hipGetLastError(), "kernel launch failed(sell_widths)");
}

template <typename IdxT>
void csr_to_sell(const IdxT* rowptr, const int32_t* cols, const double* vals, int64_t n, int64_t own_off,
                 const int64_t* slice_ptr, int32_t* scols, double* svals, hipStream_t st, int16_t* dcols) {
  hipLaunchKernelGGL(k_csr_to_sell<IdxT>, dim3(gen_grid(n)), dim3(kGenBlock), 0, st, rowptr, cols, vals,
                     n, own_off, slice_ptr, scols, svals, dcols);
  MCG_HIP(hipGetLastError(), "kernel launch failed(csr_to_sell)");
}
template void csr_to_sell<int32_t>(const int32_t*, const int32_t*, const double*, int64_t, int64_t,
                                   const int64_t*, int32_t*, double*, hipStream_t, int16_t*);
template void csr_to_sell<int64_t>(const int64_t*, const int32_t*, const double*, int64_t, int64_t,
                                   const int64_t*, int32_t*, double*, hipStream_t, int16_t*);

}  // namespace kern
}  // namespace mcg
