// SELL-64/c8: a dictionary-coded SELL-64 format.  Every stored entry is ONE byte,
// an index into a per-rank table of distinct (column offset from the row's own
// ext column, value) pairs, held in LDS by the SpMV kernels.  Applies when the
// matrix has few distinct values and few distinct column offsets — the case for
// constant-coefficient stencil discretisations such as the 5-/7-pt Poisson
// operators (3 values x 5/7 offsets = 15/21 codes).  Matrices that do not fit
// (e.g. the random-SPD family) keep SELL-64/d16 (2-B offset + 8-B value) or SELL-64.
// Offsets are any int32 (the 7-pt operator's +-N^2 planes do not fit d16).
//
// Built from the generated SELL-64(/d16) arrays, which it then replaces.
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

// column of SELL entry `dst` of padded row i (ext index)
__device__ __forceinline__ int64_t sell_col(const SellDev& S, int64_t dst, int64_t i) {
  return S.dcols ? S.own_off + i + S.dcols[dst] : (int64_t)S.cols[dst];
}

// collect the distinct value bit patterns and column offsets (from the row's own ext
// column) over every stored SELL entry, padding included (value 0, offset 0)
__global__ __launch_bounds__(kBlock) void k_dict_collect(SellDev S, DictScratch* __restrict__ d) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n_pad = (S.n_rows + 63) / 64 * 64;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_pad; i += stride) {
    if (d->overflow) return;
    const int64_t sl = i >> 6, l = i & 63;
    const int64_t base = S.slice_ptr[sl], w = (S.slice_ptr[sl + 1] - base) >> 6;
    const int64_t own = S.own_off + (i < S.n_rows ? i : S.n_rows - 1);
    for (int64_t j = 0; j < w; ++j) {
      const int64_t dst = base + 64 * j + l;
      const unsigned long long off = (unsigned long long)(sell_col(S, dst, i) - own);
      const unsigned long long key = (unsigned long long)__double_as_longlong(S.vals[dst]);
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

// one thread per padded row: code of SELL entry (i, j) at the same slot (base + 64 j + lane)
__global__ __launch_bounds__(kBlock) void k_sell_to_c8(SellDev S, const double2* __restrict__ dict, int nv, int nd,
                                                       uint8_t* __restrict__ codes) {
  __shared__ unsigned long long s_v[kMaxValues];
  __shared__ int64_t s_d[kMaxValues];
  for (int k = threadIdx.x; k < nv; k += kBlock) s_v[k] = (unsigned long long)__double_as_longlong(dict[k * nd].x);
  for (int k = threadIdx.x; k < nd; k += kBlock) s_d[k] = (int64_t)__double_as_longlong(dict[k].y);
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n_pad = (S.n_rows + 63) / 64 * 64;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_pad; i += stride) {
    const int64_t sl = i >> 6, l = i & 63;
    const int64_t base = S.slice_ptr[sl], w = (S.slice_ptr[sl + 1] - base) >> 6;
    const int64_t own = S.own_off + (i < S.n_rows ? i : S.n_rows - 1);
    for (int64_t j = 0; j < w; ++j) {
      const int64_t dst = base + 64 * j + l;
      const unsigned long long key = (unsigned long long)__double_as_longlong(S.vals[dst]);
      const int64_t off = sell_col(S, dst, i) - own;
      int vi = 0, di = 0;
      for (int k = 0; k < nv; ++k)
        if (s_v[k] == key) vi = k;
      for (int k = 0; k < nd; ++k)
        if (s_d[k] == off) di = k;
      codes[dst] = (uint8_t)(vi * nd + di);
    }
  }
}


int dict_grid(int64_t n) {
  int64_t g = (n + kBlock - 1) / kBlock;
  const int64_t cap = (int64_t)num_cus() * 16;
  return (int)std::max<int64_t>(1, std::min(g, cap));
}

}  // namespace


bool sell_dict_build(const SellDev& S, std::vector<double2>& dict, int& nv, int& nd, hipStream_t st) {
  DictScratch* d = nullptr;
  MCG_HIP(hipMallocAsync(reinterpret_cast<void**>(&d), sizeof(DictScratch), st), "device malloc failed(dict)");
  hipLaunchKernelGGL(k_dict_init, dim3(8), dim3(kBlock), 0, st, d);
  if (S.n_rows > 0) hipLaunchKernelGGL(k_dict_collect, dim3(dict_grid(S.n_rows)), dim3(kBlock), 0, st, S, d);
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
      double val, offbits;
      std::memcpy(&val, &v[a], 8);
      const long long off = o[b];
      std::memcpy(&offbits, &off, 8);
      dict[a * nd + b] = make_double2(val, offbits);  // .y holds the int64 offset's bits
    }
  return true;
}

void sell_to_c8(const SellDev& S, const double2* dict, int nv, int nd, uint8_t* codes, hipStream_t st) {
  if (S.n_rows <= 0) return;
  hipLaunchKernelGGL(k_sell_to_c8, dim3(dict_grid(S.n_rows)), dim3(kBlock), 0, st, S, dict, nv, nd, codes);
  MCG_HIP(hipGetLastError(), "kernel launch failed(sell_to_c8)");
}

}  // namespace kern
}  // namespace mcg
