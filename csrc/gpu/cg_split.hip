// Materialized-p single-reduction CG: the irregular-sparsity path (BASELINE.json config 5).
//
// The fused pass (cg_fused1.hip) never stores p_k: every gather recomputes it from
// {r_{k-1}, Ap_{k-1}} and p_{k-1} of the column (24 B per nonzero gathered, two ghost vectors
// exchanged).  That is the right trade for stencils, whose gathers hit the cache, but for long,
// unstructured rows the gathers ARE the traffic: at ~1000 nonzeros per row spread over the whole
// vector, 24 B per gather is 3x the 8 B of a gather of a stored p.  Here an iteration is
//
//   U_k  (elementwise, owned rows)  x += a p_{k-1};  r_k = r_{k-1} - a Ap_{k-1};
//                                   p_k = r_k + b p_{k-1}            (a, b from the last sums)
//   halo / all-gather of p_k (the only ghost vector)
//   S_k  (SpMV, the engines of spmv_engines.hpp)  Ap_k = A p_k gathering p only, partials of
//        {p_k.Ap_k, r_k.Ap_k, Ap_k.Ap_k, r_k.r_k}, reduced in the kernel (kernels.hpp RedCtl)
//   one 32-B all-reduce
//
// with exactly the scalars of the fused pass (f1_scalars: a_k = rr_k / pAp_k, b_k from the
// expanded ||r_k - a_k Ap_k||^2), so the two passes are the same recurrence; x is updated every
// iteration (no pairing), r and Ap exist only for owned rows, p once (ext layout).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "mcg/check.hpp"
#include "mcg/kernels.hpp"
#include "spmv_engines.hpp"

namespace mcg {
namespace kern {
namespace {

#include "f1_common.hpp"

template <bool FINAL>
__global__ __launch_bounds__(kBS) void k_split_update(double* __restrict__ x, double* __restrict__ r,
                                                      const double* __restrict__ Ap, double* __restrict__ p,
                                                      int64_t n, CgState* st, double tol, int first, int check,
                                                      double* __restrict__ partials, int pstride) {
  const F1Scalars sc = f1_scalars(st, tol, first, check);
  if (st->done || sc.conv) return;  // x_{k-1} is the answer (x is never behind: no paired updates)
  const double a = sc.alpha, b = sc.beta, na = -a;
  double s_rr = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * kBS + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBS) {
    const double pold = p[i];
    st_stream(&x[i], fma(a, pold, x[i]));
    const double rk = fma(na, Ap[i], r[i]);
    st_stream(&r[i], rk);
    if constexpr (FINAL) s_rr = fma(rk, rk, s_rr);
    else p[i] = fma(b, pold, rk);  // re-read by this iteration's SpMV: a cached store
  }
  if constexpr (FINAL) block_partial4(0.0, 0.0, 0.0, s_rr, partials, pstride);
}

// FMT: 0 CSR thread-per-row (U), 5 CSR-vector (G = U lanes per row), 1 SELL-64, 3 SELL-64/d16,
// 4 SELL-64/c8, 6 SELL-64/aligned
template <int FMT, typename IdxT, int U>
__global__ __launch_bounds__(kBS) void k_split_spmv(CsrDev<IdxT> A, SellDev S, const double* __restrict__ p,
                                                    const double* __restrict__ r, double* __restrict__ Ap,
                                                    int64_t own, TileRanges tr, double* __restrict__ partials,
                                                    int pstride, CgState* st, double tol, int first, int check,
                                                    RedCtl rc) {
  const F1Scalars sc = f1_scalars(st, tol, first, check);
  if (st->done || sc.conv) {
    f1_finish(0.0, 0.0, 0.0, 0.0, partials, pstride, rc, st, tol);
    return;
  }
  double s_pap = 0.0, s_rap = 0.0, s_apap = 0.0, s_rr = 0.0;
  auto gather = [&](int32_t c) { return p[c]; };
  auto epi = [&](int64_t i, double sum) {
    const double pk = p[own + i], rk = r[i];
    st_stream(&Ap[i], sum);
    s_pap = fma(pk, sum, s_pap);
    s_rap = fma(rk, sum, s_rap);
    s_apap = fma(sum, sum, s_apap);
    s_rr = fma(rk, rk, s_rr);
  };
  if constexpr (FMT == 0) eng::csr_adaptive<IdxT, U, 16>(A, tr, gather, epi);
  else if constexpr (FMT == 5) eng::csr_vector<IdxT, U>(A, tr, gather, epi);
  else if constexpr (FMT == 1) eng::sell<U, false, 0>(S, tr, gather, epi);
  else if constexpr (FMT == 3) eng::sell<U, false, 1>(S, tr, gather, epi);
  else if constexpr (FMT == 6) eng::sell<U, false, 3>(S, tr, gather, epi);
  else eng::sell<U, false, 2>(S, tr, gather, epi);
  f1_finish(s_pap, s_rap, s_apap, s_rr, partials, pstride, rc, st, tol);
}

// SELL-64/aligned in two halves around the all-gather of p_k (kernels.hpp cg_split_spmv `part`):
// LOCAL (part 1) sums the own-block slots and stores the partial row sums in Ap; the remote half
// (part 2) adds the other slots to them and runs the epilogue of k_split_spmv
template <int U, bool REMOTE>
__global__ __launch_bounds__(kBS) void k_split_spmv_aligned_part(SellDev S, const double* __restrict__ p,
                                                                 const double* __restrict__ r, double* __restrict__ Ap,
                                                                 int64_t own, TileRanges tr,
                                                                 double* __restrict__ partials, int pstride,
                                                                 CgState* st, double tol, int first, int check,
                                                                 RedCtl rc) {
  const F1Scalars sc = f1_scalars(st, tol, first, check);
  if (st->done || sc.conv) {
    if constexpr (REMOTE) f1_finish(0.0, 0.0, 0.0, 0.0, partials, pstride, rc, st, tol);
    return;
  }
  auto gather = [&](int32_t c) { return p[c]; };
  if constexpr (!REMOTE) {
    eng::sell_aligned_part<U, false, false>(S, tr, gather, [&](int64_t i, double sum) { Ap[i] = sum; });
  } else {
    double s_pap = 0.0, s_rap = 0.0, s_apap = 0.0, s_rr = 0.0;
    eng::sell_aligned_part<U, false, true>(S, tr, gather, [&](int64_t i, double rem) {
      const double sum = Ap[i] + rem;
      const double pk = p[own + i], rk = r[i];
      st_stream(&Ap[i], sum);
      s_pap = fma(pk, sum, s_pap);
      s_rap = fma(rk, sum, s_rap);
      s_apap = fma(sum, sum, s_apap);
      s_rr = fma(rk, rk, s_rr);
    });
    f1_finish(s_pap, s_rap, s_apap, s_rr, partials, pstride, rc, st, tol);
  }
}

// one thread per slice: binary searches over the slice's ascending slot offsets
__global__ __launch_bounds__(kBS) void k_aligned_local_slots(SellDev S, int32_t* __restrict__ out) {
  const int64_t ns = (S.n_rows + 63) / 64;
  for (int64_t sl = (int64_t)blockIdx.x * kBS + threadIdx.x; sl < ns; sl += (int64_t)gridDim.x * kBS) {
    const int64_t base = S.slice_ptr[sl];
    const int w = (int)((S.slice_ptr[sl + 1] - base) >> 6);
    const int32_t* o = S.soffs + (base >> 6);
    // lane columns own_off + 64 sl + [0, 64) + o inside [own_off, own_off + n_rows):
    // o >= -64 sl  and  o < n_rows - 63 - 64 sl
    const int64_t lo = -64 * sl, hi = S.n_rows - 63 - 64 * sl;
    auto first_ge = [&](int64_t t) {
      int a = 0, b = w;
      while (a < b) {
        const int m = (a + b) >> 1;
        if ((int64_t)o[m] < t) a = m + 1;
        else b = m;
      }
      return a;
    };
    const int a = first_ge(lo);
    int b = first_ge(hi);
    b = b < a ? a : b;
    out[2 * sl] = a;
    out[2 * sl + 1] = b;
  }
}

}  // namespace

void aligned_local_slots(const SellDev& S, int32_t* out, hipStream_t st) {
  const int64_t ns = (S.n_rows + 63) / 64;
  if (ns == 0) return;
  MCG_CHECK(S.soffs && S.slice_ptr, "aligned_local_slots: not an aligned SELL matrix");
  const int grid = (int)std::min<int64_t>((ns + kBS - 1) / kBS, 4096);
  hipLaunchKernelGGL(k_aligned_local_slots, dim3(grid), dim3(kBS), 0, st, S, out);
  MCG_HIP(hipGetLastError(), "kernel launch failed(aligned_local_slots)");
}

void cg_split_update(double* x, double* r, const double* Ap, double* p_own, int64_t n, CgState* st, double tol,
                     int first, int check, int final_mode, double* partials, int pstride, int grid,
                     hipStream_t stream) {
  if (grid <= 0) return;
  if (final_mode)
    hipLaunchKernelGGL(k_split_update<true>, dim3(grid), dim3(kBS), 0, stream, x, r, Ap, p_own, n, st, tol, first,
                       check, partials, pstride);
  else
    hipLaunchKernelGGL(k_split_update<false>, dim3(grid), dim3(kBS), 0, stream, x, r, Ap, p_own, n, st, tol, first,
                       check, partials, pstride);
  MCG_HIP(hipGetLastError(), "compute axpy failed(r)");
}

template <typename IdxT>
void cg_split_spmv(int fmt, int param, const CsrDev<IdxT>& A, const SellDev& S, const double* p_ext, const double* r,
                   double* Ap, int64_t own_off, const TileRanges& tr, double* partials, int pstride, int grid,
                   CgState* st, double tol, int first, int check, hipStream_t stream, const RedCtl& rc, int part) {
  if (tr.ntiles == 0 || grid == 0) return;
  MCG_CHECK(rc.ngroups == 0 || (rc.base % kRedGroup == 0 && rc.cnt && rc.lvl2), "in-kernel reduction: bad control block");
  if (part != 0) {
    MCG_CHECK(fmt == 6 && S.local_slots && S.soffs, "split SpMV halves: SELL-64/aligned with local slot runs only");
#define MCG_P(U, R)                                                                                                   \
  hipLaunchKernelGGL((k_split_spmv_aligned_part<U, R>), dim3(grid), dim3(kBS), 0, stream, S, p_ext, r, Ap, own_off, \
                     tr, partials, pstride, st, tol, first, check, rc)
    if (part == 1) {
      if (param <= 4) MCG_P(4, false);
      else if (param <= 6) MCG_P(6, false);
      else MCG_P(8, false);
    } else {
      if (param <= 4) MCG_P(4, true);
      else if (param <= 6) MCG_P(6, true);
      else MCG_P(8, true);
    }
#undef MCG_P
    MCG_HIP(hipGetLastError(), "compute mv failed(Ap)");
    return;
  }
#define MCG_S(F, U)                                                                                             \
  hipLaunchKernelGGL((k_split_spmv<F, IdxT, U>), dim3(grid), dim3(kBS), 0, stream, A, S, p_ext, r, Ap, own_off, tr, \
                     partials, pstride, st, tol, first, check, rc)
#define MCG_SU(F)                         \
  do {                                    \
    if (param <= 4) MCG_S(F, 4);          \
    else if (param <= 6) MCG_S(F, 6);     \
    else MCG_S(F, 8);                     \
  } while (0)
  if (fmt == 5) {
    if (param <= 4) MCG_S(5, 4);
    else if (param <= 8) MCG_S(5, 8);
    else MCG_S(5, 16);
  } else if (fmt == 0) MCG_SU(0);
  else if (fmt == 1) MCG_SU(1);
  else if (fmt == 3) MCG_SU(3);
  else if (fmt == 6) MCG_SU(6);
  else MCG_SU(4);
#undef MCG_SU
#undef MCG_S
  MCG_HIP(hipGetLastError(), "compute mv failed(Ap)");
}
template void cg_split_spmv<int32_t>(int, int, const CsrDev<int32_t>&, const SellDev&, const double*, const double*,
                                     double*, int64_t, const TileRanges&, double*, int, int, CgState*, double, int, int,
                                     hipStream_t, const RedCtl&, int);
template void cg_split_spmv<int64_t>(int, int, const CsrDev<int64_t>&, const SellDev&, const double*, const double*,
                                     double*, int64_t, const TileRanges&, double*, int, int, CgState*, double, int, int,
                                     hipStream_t, const RedCtl&, int);

}  // namespace kern
}  // namespace mcg
