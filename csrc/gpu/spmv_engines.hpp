// Device-side SpMV "engines" shared by the fused CG kernel and the plain SpMV op.
//
// Each engine walks the rows of a launch (TileRanges: up to two local row ranges)
// and calls  epi(row, sum)  with  sum = sum_j A[row,j] * gather(col_j).  The
// gather functor is where the fused CG kernel recomputes p_k = r + beta p_{k-1}
// for neighbouring rows.  All engines issue their loads in batches (clamped
// indices + selects instead of per-element branches) so that a wave keeps many
// independent loads in flight — a dependent load chain per nonzero is what
// bounded the first version of the kernel (one L2 round trip per nnz).
//
//   csr_lds     256-row tiles; the tile's rowptr and its contiguous nnz range are
//               staged through LDS with 16-B loads (4 double2 + 2 int4 per lane,
//               all issued before the first LDS write), then each thread walks
//               its row out of LDS in batches of U entries.
//   csr_direct  thread per row, no LDS: U clamped loads of cols/vals per batch,
//               then U gathers (L1 absorbs the stride-U*8 B access pattern).
//   csr_vector  G lanes per row (CSR-vector), all G/passes of a 256-row tile
//               batched, group reduction with xor-shuffles, LDS transpose so the
//               epilogue is thread-per-row and fully coalesced.
//   csr_adaptive per-tile choice (the tile is the row-length bin): thread per row
//               when every row of the tile has <= G entries, else csr_vector's body.
//   sell        one wave per 64-row SELL slice, entries column-major (every load
//               is one coalesced 512-B / 256-B wave access), U per batch.
#pragma once

#include <hip/hip_runtime.h>

#include "mcg/kernels.hpp"

namespace mcg {
namespace kern {
namespace eng {

constexpr int kBS = 256;  // threads per block = rows per CSR tile
constexpr int kWaves = kBS / 64;
// LDS stager capacity per chunk: 1023 double2 + 511 int4 fit one 4+2 load batch per lane
constexpr int kCap = 2044;
constexpr int kV2 = 4;  // double2 per lane per chunk  (kCap/2 + 1 <= 4*256)
constexpr int kC4 = 2;  // int4 per lane per chunk     (kCap/4 + 1 <= 2*256)

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  return v;
}

// fixed-order block reduction -> *out (thread 0)
template <int BS>
__device__ __forceinline__ void block_partial(double v, double* sh, double* out) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < BS / 64; ++w) s += sh[w];
    *out = s;
  }
}

__device__ __forceinline__ void tile_rows(const TileRanges& tr, int64_t t, int64_t& r0, int64_t& r1) {
  if (t < tr.nt0) {
    r0 = tr.b0 + t * kTileRows;
    r1 = r0 + kTileRows < tr.e0 ? r0 + kTileRows : tr.e0;
  } else {
    t -= tr.nt0;
    r0 = tr.b1 + t * kTileRows;
    r1 = r0 + kTileRows < tr.e1 ? r0 + kTileRows : tr.e1;
  }
}

__device__ __forceinline__ int64_t imin(int64_t a, int64_t b) { return a < b ? a : b; }
__device__ __forceinline__ int64_t imax(int64_t a, int64_t b) { return a > b ? a : b; }

// Work distribution over tiles.  Plain: unit u takes tiles u, u+U, u+2U, ...
// XCD-aware (tr.xcd = X > 1, grid divisible by X): blocks b and b+X are observed
// to land on the same XCD, so the blocks with b % X == x sweep a contiguous 1/X
// of the tiles together; the stencil neighbours of a tile (i +- N rows) are then
// read by blocks on the same XCD at about the same time and hit that XCD's L2.
// Speed only: every tile is visited exactly once for any placement.
struct TileCursor {
  int64_t t, end, step;
};
__device__ __forceinline__ TileCursor tile_cursor(const TileRanges& tr, int64_t sub, int64_t nsub) {
  const int64_t blk = blockIdx.x, nblk = gridDim.x;
  TileCursor c;
  if (tr.strip > 0) {  // contiguous run of (permuted) units per wave, see TileRanges::strip
    const int64_t nw = nblk * nsub, gw = blk * nsub + sub;
    const int64_t chunk = (tr.ntiles + nw - 1) / nw;
    c.t = gw * chunk;
    c.end = imin(tr.ntiles, c.t + chunk);
    c.step = 1;
  } else if (tr.xcd > 1 && nblk % tr.xcd == 0) {
    const int64_t X = tr.xcd, x = blk % X, lb = blk / X, nb = nblk / X;
    const int64_t per = (tr.ntiles + X - 1) / X;
    const int64_t start = x * per;
    c.end = imin(tr.ntiles, start + per);
    c.t = start + lb * nsub + sub;
    c.step = nb * nsub;
  } else {
    c.t = blk * nsub + sub;
    c.end = tr.ntiles;
    c.step = nblk * nsub;
  }
  return c;
}

// unit (slice / row tile) visited at cursor position t
__device__ __forceinline__ int64_t tile_unit(const TileRanges& tr, int64_t t) {
  if (tr.strip > 0) {
    const int64_t L = tr.nt0 / tr.strip;
    return tr.b0 + (t % L) * tr.strip + t / L;
  }
  return t < tr.nt0 ? tr.b0 + t : tr.b1 + (t - tr.nt0);
}

// matrix streams are read once per SpMV: non-temporal loads keep them from
// evicting the gathered vectors out of L2 / the Infinity Cache
template <bool NT, typename T>
__device__ __forceinline__ T ld(const T* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

// ---------------------------------------------------------------------------
template <typename IdxT, int U, class Gather, class Epi>
__device__ __forceinline__ void csr_lds(const CsrDev<IdxT>& A, const TileRanges& tr, Gather&& gather, Epi&& epi) {
  __shared__ __attribute__((aligned(16))) double2 s_v2[kV2 * kBS];
  __shared__ __attribute__((aligned(16))) int4 s_c4[kC4 * kBS];
  __shared__ int64_t s_rp[kBS + 1];
  const double* s_v = reinterpret_cast<const double*>(s_v2);
  const int32_t* s_c = reinterpret_cast<const int32_t*>(s_c4);
  const int t = threadIdx.x;
  for (TileCursor cur = tile_cursor(tr, 0, 1); cur.t < cur.end; cur.t += cur.step) {
    int64_t r0, r1;
    tile_rows(tr, cur.t, r0, r1);
    const int nr = (int)(r1 - r0);
    if (t < nr) s_rp[t] = (int64_t)A.rowptr[r0 + t];
    if (t == 0) s_rp[nr] = (int64_t)A.rowptr[r0 + nr];
    __syncthreads();
    const int64_t rs = s_rp[0], re = s_rp[nr];
    int64_t my_b = 0, my_e = 0;
    if (t < nr) {
      my_b = s_rp[t];
      my_e = s_rp[t + 1];
    }
    double sum = 0.0;
    for (int64_t cs = rs; cs < re; cs += kCap) {
      const int64_t ce = imin(re, cs + kCap);
      const int64_t vb = cs & ~(int64_t)1, cb = cs & ~(int64_t)3;
      const int nv2 = (int)((ce - vb + 1) >> 1), nc4 = (int)((ce - cb + 3) >> 2);
      const double2* gv = reinterpret_cast<const double2*>(A.vals + vb);
      const int4* gc = reinterpret_cast<const int4*>(A.cols + cb);
      double2 vr[kV2];
      int4 cr[kC4];
#pragma unroll
      for (int u = 0; u < kV2; ++u) vr[u] = gv[imin(t + u * kBS, nv2 - 1)];
#pragma unroll
      for (int u = 0; u < kC4; ++u) cr[u] = gc[imin(t + u * kBS, nc4 - 1)];
#pragma unroll
      for (int u = 0; u < kV2; ++u)
        if (t + u * kBS < nv2) s_v2[t + u * kBS] = vr[u];
#pragma unroll
      for (int u = 0; u < kC4; ++u)
        if (t + u * kBS < nc4) s_c4[t + u * kBS] = cr[u];
      __syncthreads();
      const int64_t jb = imax(my_b, cs), je = imin(my_e, ce);
      for (int64_t j0 = jb; j0 < je; j0 += U) {
        int32_t c[U];
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t j = imin(j0 + u, je - 1);
          c[u] = s_c[j - cb];
          v[u] = s_v[j - vb];
        }
        double g[U];
#pragma unroll
        for (int u = 0; u < U; ++u) g[u] = gather(c[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) sum = (j0 + u < je) ? fma(v[u], g[u], sum) : sum;
      }
      __syncthreads();
    }
    if (t < nr) epi(r0 + t, sum);
  }
}

// ---------------------------------------------------------------------------
template <typename IdxT, int U, bool NT, class Gather, class Epi>
__device__ __forceinline__ void csr_direct(const CsrDev<IdxT>& A, const TileRanges& tr, Gather&& gather, Epi&& epi) {
  const int t = threadIdx.x;
  for (TileCursor cur = tile_cursor(tr, 0, 1); cur.t < cur.end; cur.t += cur.step) {
    int64_t r0, r1;
    tile_rows(tr, cur.t, r0, r1);
    if (r0 + t >= r1) continue;
    const int64_t i = r0 + t;
    const int64_t rs = (int64_t)ld<NT>(A.rowptr + i), re = (int64_t)ld<NT>(A.rowptr + i + 1);
    double sum = 0.0;
    for (int64_t j0 = rs; j0 < re; j0 += U) {
      int32_t c[U];
      double v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t j = imin(j0 + u, re - 1);
        c[u] = ld<NT>(A.cols + j);
        v[u] = ld<NT>(A.vals + j);
      }
      double g[U];
#pragma unroll
      for (int u = 0; u < U; ++u) g[u] = gather(c[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) sum = (j0 + u < re) ? fma(v[u], g[u], sum) : sum;
    }
    epi(i, sum);
  }
}

// ---------------------------------------------------------------------------
template <typename IdxT, int G, class Gather, class Epi>
__device__ __forceinline__ void csr_vector(const CsrDev<IdxT>& A, const TileRanges& tr, Gather&& gather, Epi&& epi) {
  static_assert(G == 4 || G == 8 || G == 16, "lanes per row");
  constexpr int RPP = kBS / G;  // rows per pass; G passes cover a 256-row tile
  __shared__ double s_sum[kBS];
  const int t = threadIdx.x, sub = t & (G - 1), grp = t / G;
  for (TileCursor cur = tile_cursor(tr, 0, 1); cur.t < cur.end; cur.t += cur.step) {
    int64_t r0, r1;
    tile_rows(tr, cur.t, r0, r1);
    const int nr = (int)(r1 - r0);
    int64_t rs[G], re[G];
#pragma unroll
    for (int p = 0; p < G; ++p) {
      const int lr = p * RPP + grp;
      const int64_t ii = r0 + (lr < nr ? lr : nr - 1);
      rs[p] = (int64_t)A.rowptr[ii];
      re[p] = lr < nr ? (int64_t)A.rowptr[ii + 1] : rs[p];
    }
    int32_t c[G];
    double v[G];
#pragma unroll
    for (int p = 0; p < G; ++p) {
      const int64_t j = rs[p] + sub;
      const int64_t jj = re[p] > rs[p] ? imin(j, re[p] - 1) : 0;
      c[p] = A.cols[jj];
      v[p] = A.vals[jj];
    }
    double s[G];
#pragma unroll
    for (int p = 0; p < G; ++p) {
      const double g = gather(c[p]);
      s[p] = (rs[p] + sub < re[p]) ? v[p] * g : 0.0;
    }
    // rows longer than G: rare remainder
#pragma unroll
    for (int p = 0; p < G; ++p)
      for (int64_t j = rs[p] + sub + G; j < re[p]; j += G) s[p] = fma(A.vals[j], gather(A.cols[j]), s[p]);
#pragma unroll
    for (int p = 0; p < G; ++p) {
      double x = s[p];
#pragma unroll
      for (int off = G / 2; off > 0; off >>= 1) x += __shfl_xor(x, off, G);
      if (sub == 0) s_sum[p * RPP + grp] = x;
    }
    __syncthreads();
    if (t < nr) epi(r0 + t, s_sum[t]);
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Row-length-adaptive CSR (the tile is the bin): each 256-row tile reads its row pointers, and one
// block vote (__syncthreads_or) sends it down the thread-per-row path when every row has <= G
// entries, or the G-lanes-per-row path (csr_vector's tile body) when any row is longer.  A few long
// rows then cost their own tiles a vector pass instead of pushing every row of the matrix onto it
// (the old per-matrix choice by max_row_len), and short-row tiles keep csr_direct's batched loads.
template <typename IdxT, int U, int G, class Gather, class Epi>
__device__ __forceinline__ void csr_adaptive(const CsrDev<IdxT>& A, const TileRanges& tr, Gather&& gather,
                                             Epi&& epi) {
  static_assert(G == 4 || G == 8 || G == 16, "lanes per row");
  constexpr int RPP = kBS / G;
  __shared__ double s_sum[kBS];
  const int t = threadIdx.x, sub = t & (G - 1), grp = t / G;
  for (TileCursor cur = tile_cursor(tr, 0, 1); cur.t < cur.end; cur.t += cur.step) {
    int64_t r0, r1;
    tile_rows(tr, cur.t, r0, r1);
    const int nr = (int)(r1 - r0);
    int64_t rs = 0, re = 0;
    if (t < nr) {
      rs = (int64_t)A.rowptr[r0 + t];
      re = (int64_t)A.rowptr[r0 + t + 1];
    }
    if (!__syncthreads_or(re - rs > G)) {  // short-row tile: thread per row (csr_direct)
      double sum = 0.0;
      for (int64_t j0 = rs; j0 < re; j0 += U) {
        int32_t c[U];
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t j = imin(j0 + u, re - 1);
          c[u] = A.cols[j];
          v[u] = A.vals[j];
        }
        double g[U];
#pragma unroll
        for (int u = 0; u < U; ++u) g[u] = gather(c[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) sum = (j0 + u < re) ? fma(v[u], g[u], sum) : sum;
      }
      if (t < nr) epi(r0 + t, sum);
      continue;
    }
    // long-row tile: G lanes per row, G passes of RPP rows (csr_vector's body)
    int64_t qs[G], qe[G];
#pragma unroll
    for (int p = 0; p < G; ++p) {
      const int lr = p * RPP + grp;
      const int64_t ii = r0 + (lr < nr ? lr : nr - 1);
      qs[p] = (int64_t)A.rowptr[ii];
      qe[p] = lr < nr ? (int64_t)A.rowptr[ii + 1] : qs[p];
    }
    double sp[G];
#pragma unroll
    for (int p = 0; p < G; ++p) {
      const int64_t j = qs[p] + sub;
      const int64_t jj = qe[p] > qs[p] ? imin(j, qe[p] - 1) : 0;
      const double g = gather(A.cols[jj]);
      sp[p] = (j < qe[p]) ? A.vals[jj] * g : 0.0;
    }
#pragma unroll
    for (int p = 0; p < G; ++p)
      for (int64_t j = qs[p] + sub + G; j < qe[p]; j += G) sp[p] = fma(A.vals[j], gather(A.cols[j]), sp[p]);
#pragma unroll
    for (int p = 0; p < G; ++p) {
      double x = sp[p];
#pragma unroll
      for (int off = G / 2; off > 0; off >>= 1) x += __shfl_xor(x, off, G);
      if (sub == 0) s_sum[p * RPP + grp] = x;
    }
    __syncthreads();
    if (t < nr) epi(r0 + t, s_sum[t]);
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// SELL-64: one wave computes the 64 row sums of slice `sl` (lane = row in slice).
// CM (column mode): 0 int32 ext columns, 1 int16 offsets from the row's own ext
// column (SellDev::dcols), 3 one offset per slot shared by the slice's 64 rows
// (SellDev::soffs, SELL-64/aligned), 2 one-byte dictionary codes (SellDev::codes) looked up
// in `dict` (an LDS copy of the {value, offset} table) — every lane of a stencil
// slice reads the same code at entry j, so the LDS read is a broadcast.
template <int U, bool NT, int CM, class Gather>
__device__ __forceinline__ double sell_slice(const SellDev& A, int64_t sl, const double2* dict, Gather&& gather) {
  const int lane = threadIdx.x & 63;
  const int64_t base = A.slice_ptr[sl];
  const int w = (int)((A.slice_ptr[sl + 1] - base) >> 6);
  const int32_t* __restrict__ cp = A.cols + base + lane;
  const int16_t* __restrict__ dp = A.dcols + base + lane;
  const uint8_t* __restrict__ kp = A.codes + base + lane;
  const int32_t rowcol = (int32_t)(A.own_off + sl * 64 + lane);
  const double* __restrict__ vp = A.vals + base + lane;
  double sum = 0.0;
  for (int j0 = 0; j0 < w; j0 += U) {
    int32_t c[U];
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = (j0 + u < w ? j0 + u : w - 1) * 64;
      if constexpr (CM == 2) {
        const double2 q = dict[ld<NT>(kp + j)];
        c[u] = rowcol + (int32_t)__double_as_longlong(q.y);
        v[u] = q.x;
      } else if constexpr (CM == 3) {
        // slot offset: one wave-uniform value per slot (the slice's list), clamped column
        const int64_t cc = (int64_t)rowcol + A.soffs[(base >> 6) + (j >> 6)];
        c[u] = (int32_t)(cc < 0 ? 0 : (cc >= A.ext_len ? A.ext_len - 1 : cc));
        v[u] = ld<NT>(vp + j);
      } else {
        if constexpr (CM == 1) c[u] = rowcol + (int32_t)ld<NT>(dp + j);
        else c[u] = ld<NT>(cp + j);
        v[u] = ld<NT>(vp + j);
      }
    }
    double g[U];
#pragma unroll
    for (int u = 0; u < U; ++u) g[u] = gather(c[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) sum = (j0 + u < w) ? fma(v[u], g[u], sum) : sum;
  }
  return sum;
}

// SELL-64: `sr` in slice units; one wave per slice.
template <int U, bool NT, int CM, class Gather, class Epi>
__device__ __forceinline__ void sell(const SellDev& A, const TileRanges& sr, Gather&& gather, Epi&& epi) {
  const int lane = threadIdx.x & 63;
  __shared__ double2 s_dict[CM == 2 ? 256 : 1];
  if constexpr (CM == 2) {
    for (int k = threadIdx.x; k < A.ndict; k += kBS) s_dict[k] = A.dict[k];
    __syncthreads();
  }
  const int64_t w_in_blk = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  for (TileCursor cur = tile_cursor(sr, w_in_blk, kWaves); cur.t < cur.end; cur.t += cur.step) {
    const int64_t sl = tile_unit(sr, cur.t);
    const double sum = sell_slice<U, NT, CM>(A, sl, s_dict, gather);
    const int64_t i = sl * 64 + lane;
    if (i < A.n_rows) epi(A.perm ? (int64_t)A.perm[i] : i, sum);
  }
}

// SELL-64/aligned, slots [j_begin, j_end) of the slice at `base` only, added to `sum`
template <int U, bool NT, class Gather>
__device__ __forceinline__ double aligned_run(const SellDev& A, int64_t base, int j_begin, int j_end, int32_t rowcol,
                                              double sum, Gather&& gather) {
  const int lane = threadIdx.x & 63;
  const double* __restrict__ vp = A.vals + base + lane;
  const int32_t* __restrict__ op = A.soffs + (base >> 6);
  for (int j0 = j_begin; j0 < j_end; j0 += U) {
    int32_t c[U];
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = j0 + u < j_end ? j0 + u : j_end - 1;
      const int64_t cc = (int64_t)rowcol + op[j];
      c[u] = (int32_t)(cc < 0 ? 0 : (cc >= A.ext_len ? A.ext_len - 1 : cc));
      v[u] = ld<NT>(vp + (int64_t)j * 64);
    }
    double g[U];
#pragma unroll
    for (int u = 0; u < U; ++u) g[u] = gather(c[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) sum = (j0 + u < j_end) ? fma(v[u], g[u], sum) : sum;
  }
  return sum;
}

// SELL-64/aligned split by column ownership (the all-gather overlap): slots sort by offset, so the
// slots whose 64 columns all lie in the rank's own block are one run [a, b) per slice
// (SellDev::local_slots).  REMOTE = false sums that run (before the all-gather lands); REMOTE =
// true the rest, [0, a) then [b, w).
template <int U, bool NT, bool REMOTE, class Gather, class Epi>
__device__ __forceinline__ void sell_aligned_part(const SellDev& A, const TileRanges& sr, Gather&& gather, Epi&& epi) {
  const int lane = threadIdx.x & 63;
  const int64_t w_in_blk = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int2* __restrict__ ls = reinterpret_cast<const int2*>(A.local_slots);
  for (TileCursor cur = tile_cursor(sr, w_in_blk, kWaves); cur.t < cur.end; cur.t += cur.step) {
    const int64_t sl = tile_unit(sr, cur.t);
    const int64_t base = A.slice_ptr[sl];
    const int w = (int)((A.slice_ptr[sl + 1] - base) >> 6);
    const int2 ab = ls[sl];
    const int32_t rowcol = (int32_t)(A.own_off + sl * 64 + lane);
    double sum = 0.0;
    if constexpr (REMOTE) {
      sum = aligned_run<U, NT>(A, base, 0, ab.x, rowcol, sum, gather);
      sum = aligned_run<U, NT>(A, base, ab.y, w, rowcol, sum, gather);
    } else {
      sum = aligned_run<U, NT>(A, base, ab.x, ab.y, rowcol, sum, gather);
    }
    const int64_t i = sl * 64 + lane;
    if (i < A.n_rows) epi(i, sum);
  }
}

}  // namespace eng
}  // namespace kern
}  // namespace mcg
