// SELL-64/c8: a dictionary-coded SELL-64 format.  Every stored entry is ONE byte,
// an index into a per-rank table of distinct (column offset from the row's own
// ext column, value) pairs, held in LDS by the SpMV kernels.  Applies when the
// matrix has few distinct values and few distinct column offsets — the case for
// constant-coefficient stencil discretisations such as the 5-/7-pt Poisson
// operators (3 values x 5/7 offsets = 15/21 codes).  Matrices that do not fit
// (e.g. the random-SPD family) keep SELL-64/d16 (2-B offset + 8-B value) or SELL-64.
// Offsets are any int32 (the 7-pt operator's +-N^2 planes do not fit d16).
//
// This is value/index compression of a stored matrix (CSR-VI / CSR-DU style):
// every nonzero is still stored, read and multiplied; it only shrinks the matrix
// stream from 10 B to 1 B per entry, which is what bounds a memory-bound CG pass.
// The dictionary is the product {values} x {offsets}: code = vi * n_offsets + di.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "mcg/check.hpp"
#include "mcg/kernels.hpp"

namespace mcg {
namespace kern {
namespace {

constexpr int kBlock = 256;
constexpr int kHashSlots = 1024;                      // hash-set slots (power of two)
constexpr int kMaxValues = 256;                       // beyond this the format cannot apply
constexpr unsigned long long kEmpty = 0xFFF80000DEADBEEFull;  // a NaN payload no generator produces

__device__ __forceinline__ unsigned hash64(unsigned long long k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  return (unsigned)k & (kHashSlots - 1);
}

struct DictScratch {
  unsigned long long keys[2][kHashSlots];  // [0] value bit patterns, [1] column offsets
  unsigned count[2];
  unsigned overflow;  // bit0: too many distinct keys, bit2: sentinel value seen
};

// insert `key` into hash set t (open addressing, linear probing); read before the
// atomic, so a matrix with a handful of distinct entries costs plain L2 hits
__device__ __forceinline__ bool set_insert(DictScratch* __restrict__ d, int t, unsigned long long key) {
  unsigned h = hash64(key);
  for (int probe = 0; probe < kHashSlots; ++probe) {
    unsigned long long cur = d->keys[t][h];
    if (cur == key) return true;
    if (cur == kEmpty) {
      cur = atomicCAS(&d->keys[t][h], kEmpty, key);
      if (cur == kEmpty) {
        if (atomicAdd(&d->count[t], 1u) >= (unsigned)kMaxValues) atomicOr(&d->overflow, 1u);
        return true;
      }
      if (cur == key) return true;
    }
    h = (h + 1) & (kHashSlots - 1);
  }
  atomicOr(&d->overflow, 1u);
  return false;
}

// collect the distinct value bit patterns and column offsets (from the row's own ext column)
template <typename IdxT>
__global__ __launch_bounds__(kBlock) void k_dict_collect(const IdxT* __restrict__ rp, const int32_t* __restrict__ cols,
                                                         const double* __restrict__ vals, int64_t n, int64_t own_off,
                                                         DictScratch* __restrict__ d) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    if (d->overflow) return;
    for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
      const unsigned long long off = (unsigned long long)((int64_t)cols[k] - (own_off + i));
      const unsigned long long key = (unsigned long long)__double_as_longlong(vals[k]);
      if (key == kEmpty) {
        atomicOr(&d->overflow, 4u);
        return;
      }
      if (!set_insert(d, 0, key) || !set_insert(d, 1, off)) return;
    }
  }
}

__global__ void k_dict_init(DictScratch* d) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < kHashSlots; i += gridDim.x * blockDim.x)
    d->keys[0][i] = d->keys[1][i] = kEmpty;
  if (blockIdx.x == 0 && threadIdx.x == 0) d->count[0] = d->count[1] = d->overflow = 0;
}

// one thread per row of the padded slice set: write the codes of row i, entry j
// at base + 64 j + lane (column-major, like the other SELL arrays)
template <typename IdxT>
__global__ __launch_bounds__(kBlock) void k_csr_to_sell_c8(const IdxT* __restrict__ rp, const int32_t* __restrict__ cols,
                                                           const double* __restrict__ vals, int64_t n, int64_t own_off,
                                                           const int64_t* __restrict__ sp,
                                                           const double2* __restrict__ dict, int nv, int nd,
                                                           uint8_t* __restrict__ codes) {
  __shared__ unsigned long long s_v[kMaxValues];
  __shared__ int32_t s_d[kMaxValues];
  for (int k = threadIdx.x; k < nv; k += kBlock) s_v[k] = (unsigned long long)__double_as_longlong(dict[k * nd].x);
  for (int k = threadIdx.x; k < nd; k += kBlock) s_d[k] = (int32_t)__double_as_longlong(dict[k].y);
  __syncthreads();
  int pad_v = 0, pad_d = 0;  // padding = (offset 0, value +0.0); both are in the dictionary by construction
  for (int k = 0; k < nv; ++k)
    if (s_v[k] == 0ull) pad_v = k;
  for (int k = 0; k < nd; ++k)
    if (s_d[k] == 0) pad_d = k;
  const uint8_t pad_code = (uint8_t)(pad_v * nd + pad_d);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n_pad = (n + 63) / 64 * 64;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_pad; i += stride) {
    const int64_t sl = i >> 6, l = i & 63;
    const int64_t base = sp[sl], w = (sp[sl + 1] - base) >> 6;
    const bool row = i < n;
    const int64_t rs = row ? (int64_t)rp[i] : 0, len = row ? (int64_t)rp[i + 1] - rs : 0;
    for (int64_t j = 0; j < w; ++j) {
      uint8_t code = pad_code;
      if (j < len) {
        const unsigned long long key = (unsigned long long)__double_as_longlong(vals[rs + j]);
        const int32_t off = (int32_t)((int64_t)cols[rs + j] - (own_off + i));
        int vi = 0, di = 0;
        for (int k = 0; k < nv; ++k)
          if (s_v[k] == key) vi = k;
        for (int k = 0; k < nd; ++k)
          if (s_d[k] == off) di = k;
        code = (uint8_t)(vi * nd + di);
      }
      codes[base + 64 * j + l] = code;
    }
  }
}

int dict_grid(int64_t n) {
  int64_t g = (n + kBlock - 1) / kBlock;
  const int64_t cap = (int64_t)num_cus() * 16;
  return (int)std::max<int64_t>(1, std::min(g, cap));
}

}  // namespace

template <typename IdxT>
bool sell_dict_build(const IdxT* rowptr, const int32_t* cols, const double* vals, int64_t n, int64_t own_off,
                     std::vector<double2>& dict, int& nv, int& nd, hipStream_t st) {
  DictScratch* d = nullptr;
  MCG_HIP(hipMallocAsync(reinterpret_cast<void**>(&d), sizeof(DictScratch), st), "device malloc failed(dict)");
  hipLaunchKernelGGL(k_dict_init, dim3(8), dim3(kBlock), 0, st, d);
  if (n > 0)
    hipLaunchKernelGGL(k_dict_collect<IdxT>, dim3(dict_grid(n)), dim3(kBlock), 0, st, rowptr, cols, vals, n, own_off,
                       d);
  MCG_HIP(hipGetLastError(), "kernel launch failed(dict)");
  std::vector<unsigned char> raw(sizeof(DictScratch));
  MCG_HIP(hipMemcpyAsync(raw.data(), d, raw.size(), hipMemcpyDeviceToHost, st), "memcpy from device to host failed");
  MCG_HIP(hipStreamSynchronize(st), "device synchronize failed(dict)");
  (void)hipFreeAsync(d, st);
  DictScratch h;
  std::memcpy(&h, raw.data(), sizeof(h));
  if (h.overflow) return false;
  std::vector<unsigned long long> v;
  for (unsigned long long k : h.keys[0])
    if (k != kEmpty) v.push_back(k);
  if (std::find(v.begin(), v.end(), 0ull) == v.end()) v.push_back(0ull);  // padding value +0.0
  std::sort(v.begin(), v.end());
  std::vector<int64_t> o;
  for (unsigned long long k : h.keys[1])
    if (k != kEmpty) o.push_back((int64_t)k);
  if (std::find(o.begin(), o.end(), 0) == o.end()) o.push_back(0);  // padding offset (own column)
  std::sort(o.begin(), o.end());
  if (v.size() * o.size() > 256) return false;
  nv = (int)v.size();
  nd = (int)o.size();
  dict.resize(v.size() * o.size());
  for (int a = 0; a < nv; ++a)
    for (int b = 0; b < nd; ++b) {
      double val;
      std::memcpy(&val, &v[a], 8);
      long long off = o[b];
      double offbits;
      std::memcpy(&offbits, &off, 8);
      dict[a * nd + b] = make_double2(val, offbits);  // .y holds the int64 offset's bits
    }
  return true;
}
template bool sell_dict_build<int32_t>(const int32_t*, const int32_t*, const double*, int64_t, int64_t,
                                       std::vector<double2>&, int&, int&, hipStream_t);
template bool sell_dict_build<int64_t>(const int64_t*, const int32_t*, const double*, int64_t, int64_t,
                                       std::vector<double2>&, int&, int&, hipStream_t);

template <typename IdxT>
void csr_to_sell_c8(const IdxT* rowptr, const int32_t* cols, const double* vals, int64_t n, int64_t own_off,
                    const int64_t* slice_ptr, const double2* dict, int nv, int nd, uint8_t* codes, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_csr_to_sell_c8<IdxT>, dim3(dict_grid(n)), dim3(kBlock), 0, st, rowptr, cols, vals, n, own_off,
                     slice_ptr, dict, nv, nd, codes);
  MCG_HIP(hipGetLastError(), "kernel launch failed(csr_to_sell_c8)");
}
template void csr_to_sell_c8<int32_t>(const int32_t*, const int32_t*, const double*, int64_t, int64_t,
                                      const int64_t*, const double2*, int, int, uint8_t*, hipStream_t);
template void csr_to_sell_c8<int64_t>(const int64_t*, const int32_t*, const double*, int64_t, int64_t,
                                      const int64_t*, const double2*, int, int, uint8_t*, hipStream_t);

}  // namespace kern
}  // namespace mcg
