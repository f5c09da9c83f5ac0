// CG hot-path kernels for gfx950 (CDNA4): wave64, 256 CUs / 8 XCDs, HBM3E.
//
// One CG iteration k of the reference (CUDACG.cu:269-352: SpMV, dot, 2 AXPY,
// nrm2, SCAL+AXPY = 7 library launches, 2 blocking D2H reads) becomes
//
//   cg_spmv_fused  (K_A)  p_k  = r_k + beta_{k-1} p_{k-1}          [on the fly]
//                         Ap   = A p_k                              [CSR/SELL]
//                         x   += alpha_{k-1} p_{k-1}                [deferred x update]
//                         partial(p_k . Ap)
//   cg_reduce(A)          rho <- rr_new ; pAp <- sum partials   (+ RCCL all-reduce)
//   cg_update_r    (K_B)  r   -= alpha_k Ap ; partial(r . r)
//   cg_reduce(B)          rr_new <- sum partials ; iter++      (+ RCCL all-reduce)
//
// i.e. two streaming passes (136 B/row for a 5-pt CSR row instead of the
// reference's ~192 B/row) and two 1-block reductions; all
// scalars stay on the device.  The p_k values a row needs from its neighbours
// are recomputed from r and p_{k-1} (bit-identical to what the owner stores),
// so the separate AYPX pass disappears; p is double-buffered by iteration parity.
//
// Reductions are fixed-order (block partials -> one block), so results are
// bitwise reproducible run to run at fixed grid size and rank count.
#include <hip/hip_runtime.h>

#include <cmath>

#include "mcg/check.hpp"
#include "mcg/kernels.hpp"
#include "spmv_engines.hpp"

namespace mcg {

TileRanges make_tiles(int64_t b0, int64_t e0, int64_t b1, int64_t e1, int64_t tile) {
  TileRanges t;
  t.b0 = b0; t.e0 = e0 > b0 ? e0 : b0;
  t.b1 = b1; t.e1 = e1 > b1 ? e1 : b1;
  t.nt0 = (t.e0 - t.b0 + tile - 1) / tile;
  t.ntiles = t.nt0 + (t.e1 - t.b1 + tile - 1) / tile;
  return t;
}

namespace kern {
namespace {

using eng::kBS;
using eng::kWaves;
using eng::block_partial;
using eng::tile_rows;
using eng::wave_sum;
constexpr int kReduceBS = 1024;

__device__ __forceinline__ TileRanges make_tiles_dev(int64_t n_units) {
  TileRanges t;
  t.b0 = 0;
  t.e0 = n_units;
  t.nt0 = n_units;
  t.ntiles = n_units;
  return t;
}

struct Scalars {
  double alpha, beta;
  bool conv;
};

// alpha_{k-1}, beta_{k-1} and the convergence decision, recomputed by every
// thread from the device-resident state (identical inputs -> identical values)
__device__ __forceinline__ Scalars load_scalars(const CgState* __restrict__ st, double tol, int first,
                                                int final_mode) {
  const double rr = st->rr_new, rho = st->rho, pAp = st->pAp;
  Scalars s;
  s.conv = final_mode || (!first && sqrt(rr) < tol);
  s.alpha = first ? 0.0 : rho / pAp;
  s.beta = first ? 0.0 : rr / rho;
  return s;
}

// ---------------------------------------------------------------------------
// K_A: fused SpMV (CSR).  ENG: 0 = LDS-staged tiles, 1 = direct, 2 = CSR-vector.
// P = batch size U (ENG 0/1) or lanes per row G (ENG 2).
template <int ENG, typename IdxT, int P>
__global__ __launch_bounds__(kBS) void k_cg_spmv_fused(CsrDev<IdxT> A, const double* __restrict__ r,
                                                       const double* __restrict__ pold,
                                                       double* __restrict__ pnew, double* __restrict__ x,
                                                       double* __restrict__ Ap, int64_t own, TileRanges tr,
                                                       double* __restrict__ partials,
                                                       const CgState* __restrict__ st, double tol, int first,
                                                       int final_mode) {
  __shared__ double s_red[kWaves];
  if (st->done) return;
  const Scalars sc = load_scalars(st, tol, first, final_mode);
  const double alpha = sc.alpha, beta = sc.beta;
  if (sc.conv) {
    // the loop exits (CUDACG.cu:333): only the deferred x += alpha_{k-1} p_{k-1}
    for (int64_t tile = blockIdx.x; tile < tr.ntiles; tile += gridDim.x) {
      int64_t r0, r1;
      tile_rows(tr, tile, r0, r1);
      const int64_t i = r0 + threadIdx.x;
      if (i < r1) x[i] = fma(alpha, pold[own + i], x[i]);
    }
    return;
  }
  double acc = 0.0;
  auto gather = [&](int32_t c) { return fma(beta, pold[c], r[c]); };
  auto epi = [&](int64_t i, double sum) {
    const double po = pold[own + i];
    const double pi = fma(beta, po, r[own + i]);
    pnew[own + i] = pi;
    Ap[i] = sum;
    x[i] = fma(alpha, po, x[i]);
    acc = fma(pi, sum, acc);
  };
  if constexpr (ENG == 0) eng::csr_lds<IdxT, P>(A, tr, gather, epi);
  else if constexpr (ENG == 1) eng::csr_direct<IdxT, P, false>(A, tr, gather, epi);
  else if constexpr (ENG == 3) eng::csr_direct<IdxT, P, true>(A, tr, gather, epi);
  else if constexpr (ENG == 4) eng::csr_adaptive<IdxT, P, 16>(A, tr, gather, epi);
  else eng::csr_vector<IdxT, P>(A, tr, gather, epi);
  block_partial<kBS>(acc, s_red, partials + blockIdx.x);
}

// K_A: fused SpMV (SELL-64: one wave per 64-row slice, column-major entries).
// CM: column mode of eng::sell (0 int32, 1 d16, 2 c8).
template <int U, int CM>
__global__ __launch_bounds__(kBS) void k_cg_spmv_fused_sell(SellDev A, const double* __restrict__ r,
                                                            const double* __restrict__ pold,
                                                            double* __restrict__ pnew, double* __restrict__ x,
                                                            double* __restrict__ Ap, int64_t own, TileRanges sr,
                                                            double* __restrict__ partials,
                                                            const CgState* __restrict__ st, double tol,
                                                            int first, int final_mode) {
  __shared__ double s_red[kWaves];
  if (st->done) return;
  const Scalars sc = load_scalars(st, tol, first, final_mode);
  const double alpha = sc.alpha, beta = sc.beta;
  if (sc.conv) {
    const int lane = threadIdx.x & 63;
    const int64_t wid = blockIdx.x * kWaves + (threadIdx.x >> 6), nw = (int64_t)gridDim.x * kWaves;
    for (int64_t t = wid; t < sr.ntiles; t += nw) {
      const int64_t sl = t < sr.nt0 ? sr.b0 + t : sr.b1 + (t - sr.nt0);
      const int64_t i = sl * 64 + lane;
      if (i < A.n_rows) x[i] = fma(alpha, pold[own + i], x[i]);
    }
    return;
  }
  double acc = 0.0;
  auto gather = [&](int32_t c) { return fma(beta, pold[c], r[c]); };
  auto epi = [&](int64_t i, double sum) {
    const double po = pold[own + i];
    const double pi = fma(beta, po, r[own + i]);
    pnew[own + i] = pi;
    Ap[i] = sum;
    x[i] = fma(alpha, po, x[i]);
    acc = fma(pi, sum, acc);
  };
  eng::sell<U, false, CM>(A, sr, gather, epi);
  block_partial<kBS>(acc, s_red, partials + blockIdx.x);
}

// K_B: r -= alpha Ap ; partial(r . r)      (16 B per lane per load, UNR double2 in flight)
template <int UNR>
__global__ __launch_bounds__(kBS) void k_cg_update_r(double* __restrict__ r, const double* __restrict__ Ap,
                                                     int64_t n, double* __restrict__ partials,
                                                     const CgState* __restrict__ st) {
  __shared__ double s_red[kWaves];
  if (st->done) return;
  const double alpha = st->rho / st->pAp;
  const double na = -alpha;  // CUDACG.cu:320-321 : axpy with tmp2 = -alpha
  double acc = 0.0;
  const int64_t n2 = n >> 1;
  double2* __restrict__ r2 = reinterpret_cast<double2*>(r);
  const double2* __restrict__ a2 = reinterpret_cast<const double2*>(Ap);
  const int64_t stride = (int64_t)gridDim.x * kBS;
  int64_t k = (int64_t)blockIdx.x * kBS + threadIdx.x;
  for (; k + (UNR - 1) * stride < n2; k += UNR * stride) {
    double2 v[UNR], a[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      v[u] = r2[k + u * stride];
      a[u] = a2[k + u * stride];
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      v[u].x = fma(na, a[u].x, v[u].x);
      v[u].y = fma(na, a[u].y, v[u].y);
      r2[k + u * stride] = v[u];
      acc = fma(v[u].x, v[u].x, acc);
      acc = fma(v[u].y, v[u].y, acc);
    }
  }
  for (; k < n2; k += stride) {
    double2 v = r2[k];
    const double2 a = a2[k];
    v.x = fma(na, a.x, v.x);
    v.y = fma(na, a.y, v.y);
    r2[k] = v;
    acc = fma(v.x, v.x, acc);
    acc = fma(v.y, v.y, acc);
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    const double v = fma(na, Ap[n - 1], r[n - 1]);
    r[n - 1] = v;
    acc = fma(v, v, acc);
  }
  block_partial<kBS>(acc, s_red, partials + blockIdx.x);
}

__global__ __launch_bounds__(kBS) void k_dot_partials(const double* __restrict__ a, const double* __restrict__ b,
                                                      int64_t n, double* __restrict__ partials) {
  __shared__ double s_red[kWaves];
  double acc = 0.0;
  const int64_t n2 = n >> 1;
  const double2* __restrict__ a2 = reinterpret_cast<const double2*>(a);
  const double2* __restrict__ b2 = reinterpret_cast<const double2*>(b);
  const int64_t stride = (int64_t)gridDim.x * kBS;
  for (int64_t k = (int64_t)blockIdx.x * kBS + threadIdx.x; k < n2; k += stride) {
    const double2 u = a2[k], v = b2[k];
    acc = fma(u.x, v.x, acc);
    acc = fma(u.y, v.y, acc);
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) acc = fma(a[n - 1], b[n - 1], acc);
  block_partial<kBS>(acc, s_red, partials + blockIdx.x);
}

__device__ __forceinline__ double reduce_partials_1block(const double* __restrict__ p, int np, double* sh) {
  // 8 independent loads in flight per thread (a latency-bound single block); the order of the
  // additions depends only on np, so the sum is bitwise reproducible
  double s = 0.0;
  int i = threadIdx.x;
  for (; i + 7 * kReduceBS < np; i += 8 * kReduceBS) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[i + u * kReduceBS];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; i < np; i += kReduceBS) s += p[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  double tot = 0.0;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int w = 0; w < kReduceBS / 64; ++w) tot += sh[w];
  }
  return tot;  // valid in thread 0
}

__global__ __launch_bounds__(kReduceBS) void k_cg_reduce(const double* __restrict__ partials, int np,
                                                         CgState* __restrict__ st, int mode, int first,
                                                         double tol) {
  __shared__ double sh[kReduceBS / 64];
  const double tot = reduce_partials_1block(partials, np, sh);
  if (threadIdx.x != 0) return;
  switch (mode) {
    case kReduceInit:
      st->rr_new = tot;
      st->rr0 = tot;
      st->rho = 0.0;
      st->pAp = 0.0;
      st->rr_final = 0.0;
      st->iter = 0;
      st->done = 0;
      st->conv_iter = 0;
      st->converged = 0;
      st->breakdown = 0;
      break;
    case kReduceA: {
      if (st->done) { st->pAp = 0.0; break; }  // keep no-op all-reduces finite
      const double rr = st->rr_new;
      if (!first && sqrt(rr) < tol) {  // CUDACG.cu:333 — break after x/r update
        st->done = 1;
        st->converged = 1;
        st->conv_iter = st->iter;
        st->rr_final = rr;
        st->pAp = 0.0;
        break;
      }
      if (!isfinite(rr)) {
        st->done = 3;
        st->breakdown = 1;
        st->conv_iter = st->iter;
        st->rr_final = rr;
        st->pAp = 0.0;
        break;
      }
      st->rho = rr;
      st->pAp = tot;
      break;
    }
    case kReduceB:
      if (st->done) { st->rr_new = 0.0; break; }
      st->rr_new = tot;
      st->iter += 1;
      break;
    case kReduceFinal:
      if (st->done) break;
      st->done = 2;
      st->converged = sqrt(st->rr_new) < tol ? 1 : 0;
      st->conv_iter = st->iter;
      st->rr_final = st->rr_new;
      break;
    default: break;
  }
}

__global__ __launch_bounds__(kReduceBS) void k_sum_partials(const double* __restrict__ partials, int np,
                                                            double* __restrict__ out) {
  __shared__ double sh[kReduceBS / 64];
  const double tot = reduce_partials_1block(partials, np, sh);
  if (threadIdx.x == 0) *out = tot;
}

// ---------------------------------------------------------------------------
// unfused building blocks
template <int ENG, typename IdxT>
__global__ __launch_bounds__(kBS) void k_spmv_csr(CsrDev<IdxT> A, const double* __restrict__ xv,
                                                  double* __restrict__ y, TileRanges tr) {
  auto gather = [&](int32_t c) { return xv[c]; };
  auto epi = [&](int64_t i, double sum) { y[i] = sum; };
  if constexpr (ENG == 0) eng::csr_lds<IdxT, 8>(A, tr, gather, epi);
  else eng::csr_direct<IdxT, 8, false>(A, tr, gather, epi);
}

template <int CM>
__global__ __launch_bounds__(kBS) void k_spmv_sell(SellDev A, const double* __restrict__ xv,
                                                   double* __restrict__ y) {
  const TileRanges sr = make_tiles_dev((A.n_rows + 63) / 64);
  eng::sell<8, false, CM>(A, sr, [&](int32_t c) { return xv[c]; }, [&](int64_t i, double sum) { y[i] = sum; });
}

__global__ __launch_bounds__(kBS) void k_axpy(double alpha, const double* __restrict__ xv,
                                              double* __restrict__ y, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * kBS;
  for (int64_t i = (int64_t)blockIdx.x * kBS + threadIdx.x; i < n; i += stride) y[i] = fma(alpha, xv[i], y[i]);
}

__global__ __launch_bounds__(kBS) void k_xpby(const double* __restrict__ xv, double beta,
                                              double* __restrict__ y, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * kBS;
  for (int64_t i = (int64_t)blockIdx.x * kBS + threadIdx.x; i < n; i += stride) y[i] = fma(beta, y[i], xv[i]);
}

}  // namespace

// ---------------------------------------------------------------------------
// launchers
namespace {
template <typename IdxT, int ENG, int P>
void launch_fused(const CsrDev<IdxT>& A, const double* r, const double* po, double* pn, double* x, double* Ap,
                  int64_t own, const TileRanges& tr, double* partials, int grid, const CgState* st, double tol,
                  int first, int final_mode, hipStream_t stream) {
  hipLaunchKernelGGL((k_cg_spmv_fused<ENG, IdxT, P>), dim3(grid), dim3(kBS), 0, stream, A, r, po, pn, x, Ap, own,
                     tr, partials, st, tol, first, final_mode);
}
}  // namespace

int spmv_param_for(int variant, int64_t max_row_len) {
  if (variant == 2) return max_row_len <= 4 ? 4 : (max_row_len <= 8 ? 8 : 16);
  return max_row_len <= 4 ? 4 : (max_row_len <= 6 ? 6 : 8);
}

template <typename IdxT>
void cg_spmv_fused(const CsrDev<IdxT>& A, const double* r_ext, const double* pold_ext, double* pnew_ext,
                   double* x, double* Ap, int64_t own_off, const TileRanges& tr, double* partials, int grid,
                   const CgState* st, double tol, int first, int final_mode, int variant, int param,
                   hipStream_t stream) {
  if (tr.ntiles == 0) return;
#define MCG_FUSED(E, P) \
  launch_fused<IdxT, E, P>(A, r_ext, pold_ext, pnew_ext, x, Ap, own_off, tr, partials, grid, st, tol, first, final_mode, stream)
  if (variant == 0) {
    if (param <= 4) MCG_FUSED(0, 4); else if (param <= 6) MCG_FUSED(0, 6); else MCG_FUSED(0, 8);
  } else if (variant == 1) {
    if (param <= 4) MCG_FUSED(1, 4); else if (param <= 6) MCG_FUSED(1, 6); else MCG_FUSED(1, 8);
  } else if (variant == 3) {
    if (param <= 4) MCG_FUSED(3, 4); else if (param <= 6) MCG_FUSED(3, 6); else MCG_FUSED(3, 8);
  } else if (variant == 4) {
    if (param <= 4) MCG_FUSED(4, 4); else if (param <= 6) MCG_FUSED(4, 6); else MCG_FUSED(4, 8);
  } else {
    if (param <= 4) MCG_FUSED(2, 4); else if (param <= 8) MCG_FUSED(2, 8); else MCG_FUSED(2, 16);
  }
#undef MCG_FUSED
  MCG_HIP(hipGetLastError(), "compute mv failed(Ap)");
}
template void cg_spmv_fused<int32_t>(const CsrDev<int32_t>&, const double*, const double*, double*, double*,
                                     double*, int64_t, const TileRanges&, double*, int, const CgState*, double,
                                     int, int, int, int, hipStream_t);
template void cg_spmv_fused<int64_t>(const CsrDev<int64_t>&, const double*, const double*, double*, double*,
                                     double*, int64_t, const TileRanges&, double*, int, const CgState*, double,
                                     int, int, int, int, hipStream_t);

void cg_spmv_fused_sell(const SellDev& A, const double* r_ext, const double* pold_ext, double* pnew_ext,
                        double* x, double* Ap, int64_t own_off, const TileRanges& slices, double* partials,
                        int grid, const CgState* st, double tol, int first, int final_mode, int param,
                        int flags, hipStream_t stream) {
  if (slices.ntiles == 0) return;
#define MCG_SELL(U)                                                                                     \
  do {                                                                                                  \
    if (flags & 8)                                                                                      \
      hipLaunchKernelGGL((k_cg_spmv_fused_sell<U, 2>), dim3(grid), dim3(kBS), 0, stream, A, r_ext,          \
                         pold_ext, pnew_ext, x, Ap, own_off, slices, partials, st, tol, first, final_mode); \
    else if (flags & 4)                                                                                 \
      hipLaunchKernelGGL((k_cg_spmv_fused_sell<U, 1>), dim3(grid), dim3(kBS), 0, stream, A, r_ext,          \
                         pold_ext, pnew_ext, x, Ap, own_off, slices, partials, st, tol, first, final_mode); \
    else                                                                                                \
      hipLaunchKernelGGL((k_cg_spmv_fused_sell<U, 0>), dim3(grid), dim3(kBS), 0, stream, A, r_ext,          \
                         pold_ext, pnew_ext, x, Ap, own_off, slices, partials, st, tol, first, final_mode); \
  } while (0)
  if (param <= 4) MCG_SELL(4);
  else if (param == 5) MCG_SELL(5);
  else if (param <= 6) MCG_SELL(6);
  else if (param == 7) MCG_SELL(7);
  else MCG_SELL(8);
#undef MCG_SELL
  MCG_HIP(hipGetLastError(), "compute mv failed(Ap)");
}

void cg_update_r(double* r_own, const double* Ap, int64_t n, double* partials, int grid, const CgState* st,
                 int unroll, hipStream_t stream) {
  if (unroll >= 4)
    hipLaunchKernelGGL(k_cg_update_r<4>, dim3(grid), dim3(kBS), 0, stream, r_own, Ap, n, partials, st);
  else if (unroll == 2)
    hipLaunchKernelGGL(k_cg_update_r<2>, dim3(grid), dim3(kBS), 0, stream, r_own, Ap, n, partials, st);
  else
    hipLaunchKernelGGL(k_cg_update_r<1>, dim3(grid), dim3(kBS), 0, stream, r_own, Ap, n, partials, st);
  MCG_HIP(hipGetLastError(), "compute axpy failed(r)");
}

void cg_reduce(const double* partials, int np, CgState* st, int mode, int first, double tol,
               hipStream_t stream) {
  hipLaunchKernelGGL(k_cg_reduce, dim3(1), dim3(kReduceBS), 0, stream, partials, np, st, mode, first, tol);
  MCG_HIP(hipGetLastError(), "compute dot failed(tmp)");
}

void dot_partials(const double* a, const double* b, int64_t n, double* partials, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(k_dot_partials, dim3(grid), dim3(kBS), 0, stream, a, b, n, partials);
  MCG_HIP(hipGetLastError(), "compute norm2 failed(r)");
}

void sum_partials(const double* partials, int np, double* out, hipStream_t stream) {
  hipLaunchKernelGGL(k_sum_partials, dim3(1), dim3(kReduceBS), 0, stream, partials, np, out);
  MCG_HIP(hipGetLastError(), "compute dot failed");
}

template <typename IdxT>
void spmv_csr(const CsrDev<IdxT>& A, const double* x, double* y, hipStream_t stream, int variant) {
  const TileRanges tr = make_tiles(0, A.n_rows);
  if (tr.ntiles == 0) return;
  const int grid = grid_for(tr.ntiles * kTileRows, kBS, 8);
  if (variant == 1)
    hipLaunchKernelGGL((k_spmv_csr<1, IdxT>), dim3(grid), dim3(kBS), 0, stream, A, x, y, tr);
  else
    hipLaunchKernelGGL((k_spmv_csr<0, IdxT>), dim3(grid), dim3(kBS), 0, stream, A, x, y, tr);
  MCG_HIP(hipGetLastError(), "compute mv failed(Ap)");
}
template void spmv_csr<int32_t>(const CsrDev<int32_t>&, const double*, double*, hipStream_t, int);
template void spmv_csr<int64_t>(const CsrDev<int64_t>&, const double*, double*, hipStream_t, int);

void spmv_sell(const SellDev& A, const double* x, double* y, hipStream_t stream) {
  const int64_t ns = (A.n_rows + 63) / 64;
  if (ns == 0) return;
  const int grid = grid_for(ns * 64, kBS, 8);
  if (A.soffs)
    hipLaunchKernelGGL(k_spmv_sell<3>, dim3(grid), dim3(kBS), 0, stream, A, x, y);
  else if (A.codes)
    hipLaunchKernelGGL(k_spmv_sell<2>, dim3(grid), dim3(kBS), 0, stream, A, x, y);
  else if (A.dcols)
    hipLaunchKernelGGL(k_spmv_sell<1>, dim3(grid), dim3(kBS), 0, stream, A, x, y);
  else
    hipLaunchKernelGGL(k_spmv_sell<0>, dim3(grid), dim3(kBS), 0, stream, A, x, y);
  MCG_HIP(hipGetLastError(), "compute mv failed(Ap)");
}

void axpy(double alpha, const double* x, double* y, int64_t n, hipStream_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_axpy, dim3(grid_for(n, kBS, 8)), dim3(kBS), 0, stream, alpha, x, y, n);
  MCG_HIP(hipGetLastError(), "compute axpy failed");
}

void xpby(const double* x, double beta, double* y, int64_t n, hipStream_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_xpby, dim3(grid_for(n, kBS, 8)), dim3(kBS), 0, stream, x, beta, y, n);
  MCG_HIP(hipGetLastError(), "compute axpy failed(p)");
}

}  // namespace kern
}  // namespace mcg
