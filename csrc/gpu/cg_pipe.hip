// Pipelined CG (Ghysels & Vanroose 2014), the opt-in latency-tolerant recurrence (recurrence = 2).
//
// The reference blocks on two reductions per iteration (CUDACG.cu:304, 328); the single-reduction
// form (cg_fused1.hip) has one, but it still sits between two passes: pass k+1 needs alpha_k.  Here
// the one reduction of an iteration overlaps the SpMV that does not depend on it:
//
//   AR_i  (side stream)  gamma_i = r_i.r_i, delta_i = w_i.r_i          (32-B all-reduce)
//   S_i   (compute)      q_i = A w_i                                    (overlaps AR_i)
//   U_i   (compute)      beta_i = gamma_i / gamma_{i-1};  alpha_i = gamma_i / (delta_i - beta_i gamma_i / alpha_{i-1})
//                        z_i = q_i + beta_i z_{i-1};  s_i = w_i + beta_i s_{i-1};  p_i = r_i + beta_i p_{i-1}
//                        x_{i+1} = x_i + alpha_i p_i;  r_{i+1} = r_i - alpha_i s_i;  w_{i+1} = w_i - alpha_i z_i
//                        partials of gamma_{i+1}, delta_{i+1}  (in-kernel reduction, like the fused pass)
//
// with w = A r, s = A p, z = A s kept by recurrences (exact CG in exact arithmetic).  The extra
// recurrences drift in floating point, so every `rr_period` iterations r, w, s, z are recomputed
// from x and p (residual replacement: 4 SpMVs).  Stopping follows the reference: ||r_k|| < tol with
// the absolute tol, tested on gamma_k = ||r_k||^2, x_k is the answer, k = SpMVs of the recurrence.
//
// Costs per row and iteration: U reads q, z, s, p, x, r, w and writes all but q (104 B) and S
// reads w and writes q (+ the matrix): 3x the bytes of the fused single-reduction pass, so it only
// pays where the all-reduce latency exceeds the SpMV (small per-rank work at many ranks).
#include <hip/hip_runtime.h>

#include <cmath>

#include "mcg/check.hpp"
#include "mcg/kernels.hpp"
#include "spmv_engines.hpp"

namespace mcg {
namespace kern {
namespace {

#include "f1_common.hpp"

struct PipeScalars {
  double alpha, beta;
  bool conv, bad;
};

__device__ __forceinline__ PipeScalars pipe_scalars(const CgState* st, double tol, int first, int check) {
  PipeScalars s;
  const double g = st->red[0], d = st->red[1];
  s.conv = check && sqrt(g) < tol;
  s.bad = check && !isfinite(g);
  if (first) {
    s.beta = 0.0;
    s.alpha = g / d;
  } else {
    s.beta = g / st->rho;
    s.alpha = g / (d - s.beta * g / st->a_prev);
  }
  return s;
}

// bookkeeping of the last arriver: latch on gamma_i, or rotate (rho = gamma_i, a_prev = alpha_i)
// and store the new local sums {gamma_{i+1}, delta_{i+1}} for the all-reduce
__device__ __forceinline__ void pipe_bookkeep(CgState* st, const double* tot, int check, int first, double tol) {
  auto zero = [&] {
    for (int q = 0; q < 4; ++q) st->red[q] = 0.0;
  };
  if (st->done) {
    zero();
    return;
  }
  const PipeScalars s = pipe_scalars(st, tol, first, check);
  if (s.conv || s.bad) {
    st->done = s.conv ? 1 : 3;
    st->converged = s.conv ? 1 : 0;
    st->breakdown = s.bad ? 1 : 0;
    st->conv_iter = st->iter;
    st->rr_final = st->red[0];
    zero();
    return;
  }
  st->rho = st->red[0];
  st->a_prev = s.alpha;
  st->red[0] = tot[0];
  st->red[1] = tot[1];
  st->red[2] = 0.0;
  st->red[3] = tot[0];  // result(): ||r|| of an unlatched state
  st->rr_new = tot[0];
  st->iter += 1;
}

// the in-kernel two-level reduction of f1_common.hpp with the pipelined bookkeeping
__device__ __noinline__ void pipe_reduce_tail(double* out, int pstride, RedCtl rc, CgState* st, double tol) {
  last_arriver_reduce<2>(
      out, pstride, rc, [] { return 0; }, [&](const double* t, int) { pipe_bookkeep(st, t, rc.check, rc.first, tol); });
}

__global__ __launch_bounds__(kBS) void k_pipe_update(PipeVectors v, int64_t n, double* __restrict__ partials,
                                                     int pstride, CgState* st, double tol, RedCtl rc) {
  const PipeScalars sc = pipe_scalars(st, tol, rc.first, rc.check);
  double s_g = 0.0, s_d = 0.0;
  if (!st->done && !sc.conv && !sc.bad) {
    const double a = sc.alpha, b = sc.beta, na = -a;
    for (int64_t i = (int64_t)blockIdx.x * kBS + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBS) {
      const double zi = fma(b, v.z[i], v.q[i]);
      const double si = fma(b, v.s[i], v.w[i]);
      const double pi = fma(b, v.p[i], v.r[i]);
      const double ri = fma(na, si, v.r[i]);
      const double wi = fma(na, zi, v.w[i]);
      v.z[i] = zi;
      v.s[i] = si;
      v.p[i] = pi;
      st_stream(&v.x[i], fma(a, pi, v.x[i]));
      v.r[i] = ri;
      v.w[i] = wi;
      s_g = fma(ri, ri, s_g);
      s_d = fma(wi, ri, s_d);
    }
  }
  block_partial4(s_g, s_d, 0.0, 0.0, partials, pstride, true);
  pipe_reduce_tail(partials, pstride, rc, st, tol);
}

// {r.r, w.r} block partials of the owned rows (init / residual replacement), then k_pipe_sum
__global__ __launch_bounds__(kBS) void k_pipe_dots(const double* __restrict__ r, const double* __restrict__ w, int64_t n,
                                                   double* __restrict__ partials, int pstride) {
  double s_g = 0.0, s_d = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * kBS + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBS) {
    s_g = fma(r[i], r[i], s_g);
    s_d = fma(w[i], r[i], s_d);
  }
  block_partial4(s_g, s_d, 0.0, 0.0, partials, pstride);
}

// mode 0 (init): red = {gamma_0, delta_0} local, rr0, iter = 0; mode 1 (residual replacement):
// red = the recomputed local sums (the all-reduce that follows makes them global)
__global__ __launch_bounds__(64) void k_pipe_sum(const double* __restrict__ partials, int pstride, int np, CgState* st,
                                                 int mode) {
  double t[2] = {0.0, 0.0};
  for (int j = threadIdx.x; j < np; j += 64) {
    t[0] += partials[j];
    t[1] += partials[pstride + j];
  }
  t[0] = eng::wave_sum(t[0]);
  t[1] = eng::wave_sum(t[1]);
  if (threadIdx.x == 0) {
    if (st->done) return;
    st->red[0] = t[0];
    st->red[1] = t[1];
    st->red[2] = 0.0;
    st->red[3] = t[0];
    st->rr_new = t[0];
    if (mode == 0) {
      st->rr0 = t[0];
      st->iter = 0;
      st->rho = 0.0;
      st->a_prev = 0.0;
    }
  }
}

// finalize(): gamma_m after the last update (all-reduced): converged flag, latch
__global__ void k_pipe_final(CgState* st, double tol) {
  if (st->done) return;
  const double g = st->red[0];
  st->done = 2;
  st->converged = sqrt(g) < tol ? 1 : 0;
  st->breakdown = isfinite(g) ? 0 : 1;
  st->conv_iter = st->iter;
  st->rr_final = g;
}

__global__ __launch_bounds__(kBS) void k_sub(const double* __restrict__ b, const double* __restrict__ y,
                                             double* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * kBS + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBS) out[i] = b[i] - y[i];
}

}  // namespace

void cg_pipe_update(const PipeVectors& v, int64_t n, double* partials, int pstride, int grid, CgState* st, double tol,
                    hipStream_t stream, const RedCtl& rc) {
  MCG_CHECK(rc.ngroups > 0 && rc.base == 0 && rc.cnt && rc.lvl2, "pipelined CG: in-kernel reduction not set up");
  hipLaunchKernelGGL(k_pipe_update, dim3(grid), dim3(kBS), 0, stream, v, n, partials, pstride, st, tol, rc);
  MCG_HIP(hipGetLastError(), "compute axpy failed(r)");
}

void cg_pipe_dots(const double* r, const double* w, int64_t n, double* partials, int pstride, int grid, CgState* st,
                  int mode, hipStream_t stream) {
  hipLaunchKernelGGL(k_pipe_dots, dim3(grid), dim3(kBS), 0, stream, r, w, n, partials, pstride);
  hipLaunchKernelGGL(k_pipe_sum, dim3(1), dim3(64), 0, stream, partials, pstride, grid, st, mode);
  MCG_HIP(hipGetLastError(), "compute norm2 failed(r)");
}

void cg_pipe_final(CgState* st, double tol, hipStream_t stream) {
  hipLaunchKernelGGL(k_pipe_final, dim3(1), dim3(1), 0, stream, st, tol);
  MCG_HIP(hipGetLastError(), "compute norm2 failed(rho)");
}

void sub_vec(const double* b, const double* y, double* out, int64_t n, hipStream_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_sub, dim3(grid_for(n, kBS, 8)), dim3(kBS), 0, stream, b, y, out, n);
  MCG_HIP(hipGetLastError(), "compute axpy failed(r)");
}

}  // namespace kern
}  // namespace mcg
