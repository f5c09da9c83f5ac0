// Device helpers shared by the single-reduction passes (cg_fused1.hip: fused pass; cg_split.hip:
// the materialized-p split pass): the per-pass scalars, block partials, the in-kernel two-level
// reduction and the CgState bookkeeping.  Included inside namespace mcg::kern::(anonymous).
#pragma once

using eng::kBS;
using eng::kWaves;

struct F1Scalars {
  double alpha, beta;
  bool conv;
};

__device__ __forceinline__ F1Scalars f1_scalars(const CgState* st, double tol, int first, int check) {
  F1Scalars s;
  const double pAp = st->red[0], rAp = st->red[1], ApAp = st->red[2], rr = st->red[3];
  s.conv = check && sqrt(rr) < tol;  // ||r_{k-1}|| < tol : the reference's break (CUDACG.cu:333)
  if (first) {
    s.alpha = 0.0;
    s.beta = 0.0;
  } else {
    s.alpha = rr / pAp;
    double est = fma(s.alpha * s.alpha, ApAp, fma(-2.0 * s.alpha, rAp, rr));  // ||r_{k-1} - a Ap_{k-1}||^2
    est = est > 0.0 ? est : 0.0;
    s.beta = est / rr;
  }
  return s;
}

// agent-scope (write-through, L1-bypassing) 8-B accesses for the in-kernel reduction's hand-offs
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;
__device__ __forceinline__ void st_wt(double* p, double v) {
  __hip_atomic_store((gu64*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_wt(const double* p) {
  return __longlong_as_double((long long)__hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// four fixed-order block partials -> partials[q * pstride + blockIdx.x] (write-through when an
// in-kernel reduction reads them)
template <int NW = kWaves>  // waves per block (the tiles' 16-wave workgroups: 16)
__device__ __forceinline__ void block_partial4(double a0, double a1, double a2, double a3, double* __restrict__ out,
                                               int pstride, bool wt = false) {
  __shared__ double sh[4][NW];
  a0 = eng::wave_sum(a0);
  a1 = eng::wave_sum(a1);
  a2 = eng::wave_sum(a2);
  a3 = eng::wave_sum(a3);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sh[0][w] = a0;
    sh[1][w] = a1;
    sh[2][w] = a2;
    sh[3][w] = a3;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < NW; ++k) s += sh[threadIdx.x][k];
    if (wt) st_wt(&out[threadIdx.x * pstride + blockIdx.x], s);
    else out[threadIdx.x * pstride + blockIdx.x] = s;
  }
}

// The CgState fields the bookkeeping reads.  Nothing writes them inside a pass before its grid's
// last arriver does, so the in-kernel reduction loads them early, in every group winner, under the
// round trips that follow (profiles/r6/waves: ~1 us of dependent misses a pass when loaded last).
struct BookSnap {
  double red[4];
  int iter, done, clamps;
};
__device__ __forceinline__ BookSnap book_snap(const CgState* st) {
  BookSnap s;
#pragma unroll
  for (int q = 0; q < 4; ++q) s.red[q] = st->red[q];
  s.iter = st->iter;
  s.done = st->done;
  s.clamps = st->clamps;
  return s;
}
// the snapshot is the same in every lane: held in SGPRs across the reduction's round trips
__device__ __forceinline__ double rfl_d(double x) {
  return __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(x)),
                          __builtin_amdgcn_readfirstlane(__double2loint(x)));
}
__device__ __forceinline__ BookSnap rfl(const BookSnap& s) {
  BookSnap u;
#pragma unroll
  for (int q = 0; q < 4; ++q) u.red[q] = rfl_d(s.red[q]);
  u.iter = __builtin_amdgcn_readfirstlane(s.iter);
  u.done = __builtin_amdgcn_readfirstlane(s.done);
  u.clamps = __builtin_amdgcn_readfirstlane(s.clamps);
  return u;
}
__device__ __forceinline__ int rfl(int x) { return x; }

// CgState update from a fused pass's sums tot[4] (local; the all-reduce that follows makes them
// global): the convergence / breakdown latch on the previous pass's GLOBAL r.r, a_prev, the new
// sums, the iteration count.  cg_reduce_f1 mode 0 and the in-kernel reduction share this code;
// s = book_snap(st) taken any time after the pass's start.
__device__ __forceinline__ void f1_bookkeep(CgState* st, const BookSnap& s, const double* tot, int check, int first,
                                            double tol) {
  auto zero = [&] {
    for (int q = 0; q < 4; ++q) st->red[q] = 0.0;
  };
  if (s.done) { zero(); return; }
  const double rr_prev = s.red[3];
  if (check && sqrt(rr_prev) < tol) {
    st->done = 1;
    st->converged = 1;
    st->conv_iter = s.iter - 1;
    st->rr_final = rr_prev;
    zero();
    return;
  }
  if (check && !isfinite(rr_prev)) {
    st->done = 3;
    st->breakdown = 1;
    st->conv_iter = s.iter - 1;
    st->rr_final = rr_prev;
    zero();
    return;
  }
  // alpha of the pass whose (global) sums are being replaced — the pass after next pairs it
  // into its x update; same division as f1_scalars so the bits agree
  st->a_prev = first ? 0.0 : s.red[3] / s.red[0];
  st->b_prev = 0.0;
  if (!first) {  // the clamp in f1_scalars, re-evaluated on the same global sums: count when it fired
    const double a = s.red[3] / s.red[0];
    const double est = fma(a * a, s.red[2], fma(-2.0 * a, s.red[1], s.red[3]));
    if (!(est > 0.0)) st->clamps = s.clamps + 1;
    st->b_prev = (est > 0.0 ? est : 0.0) / s.red[3];  // f1_scalars' beta, same operations: same bits
  }
  for (int q = 0; q < 4; ++q) st->red[q] = tot[q];
  st->rr_new = tot[3];
  st->iter = s.iter + 1;
}
__device__ __forceinline__ void f1_bookkeep(CgState* st, const double* tot, int check, int first, double tol) {
  f1_bookkeep(st, book_snap(st), tot, check, first, tol);
}

// In-kernel two-level last-arriver reduction (kernels.hpp RedCtl) of NV block sums, then
// book(totals) in lane 0 of the grid's last arriver.  Runs in wave 0 after block_partial4(wt =
// true): lanes 0..NV-1 of that wave stored the block's partials write-through.  Every hand-off is
//   write-through (sc0 sc1) stores -> s_waitcnt vmcnt(0) -> one relaxed agent-scope atomic add,
// and the last arriver (told by the value its add returned) reads with write-through (sc1) loads
// only (MI355X_MICROARCH.md, visibility: valid forms, first table row): the stores have reached
// the device-coherent level before the add is issued, and the loads cannot be served from a stale
// L1/L2 line.  The ordering is pinned for the compiler as well: the waits are asm volatile with a
// memory clobber (no store or load crosses them), and the winner's path starts with one more
// compiler barrier, so no load of the hand-off can be hoisted above the atomic it depends on.  An
// agent release fence on every block's add (buffer_wbl2, ~1.7 us a block) would order nothing the
// write-through path has not ordered already.
#if defined(MCG_CARRY_DIAG)
// diagnostic build: the grid's last arriver's wall clock at each step of the reduction tail (profiles/r6/waves)
__device__ unsigned long long g_red_diag[8];
#define MCG_RED_T(i) (t_red[i] = wall_clock64())
#else
#define MCG_RED_T(i) ((void)0)
#endif
template <int NV, typename Pre, typename Book>
__device__ __forceinline__ void last_arriver_reduce(const double* out, int pstride, const RedCtl& rc, Pre&& pre,
                                                    Book&& book) {
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
#if defined(MCG_CARRY_DIAG)
  unsigned long long t_red[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
  MCG_RED_T(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  MCG_RED_T(1);
  const int g = (rc.base + (int)blockIdx.x) / kRedGroup;
  const int g0 = g * kRedGroup - rc.base;  // the group's first slot, relative to `out`
  const int gsize = min(kRedGroup, (int)gridDim.x - g0);
  unsigned old = 0;
  if (lane == 0) old = __hip_atomic_fetch_add((gu32*)&rc.cnt[g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  old = __shfl(old, 0, 64);
  MCG_RED_T(2);
  if (old != (unsigned)(gsize - 1)) return;
  asm volatile("" ::: "memory");
  if (lane == 0) __hip_atomic_store((gu32*)&rc.cnt[g], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  auto snap = pre();  // issued ahead of the group's loads: its latency hides under theirs
  double v[NV];
#pragma unroll
  for (int q = 0; q < NV; ++q) v[q] = lane < gsize ? ld_wt(&out[q * pstride + g0 + lane]) : 0.0;
  snap = rfl(snap);  // arrives with the group's loads; into SGPRs before the sums' VGPR peak
#pragma unroll
  for (int q = 0; q < NV; ++q) v[q] = eng::wave_sum(v[q]);
  MCG_RED_T(3);
  if (lane == 0) {
#pragma unroll
    for (int q = 0; q < NV; ++q) st_wt(&rc.lvl2[q * rc.l2s + g], v[q]);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  MCG_RED_T(4);
  if (lane == 0) old = __hip_atomic_fetch_add((gu32*)&rc.cnt[rc.top], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  old = __shfl(old, 0, 64);
  MCG_RED_T(5);
  if (old != (unsigned)(rc.ngroups - 1)) return;
  asm volatile("" ::: "memory");
  if (lane == 0) __hip_atomic_store((gu32*)&rc.cnt[rc.top], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  double t[NV];
#pragma unroll
  for (int q = 0; q < NV; ++q) t[q] = 0.0;
  for (int j = lane; j < rc.ngroups; j += 64) {
#pragma unroll
    for (int q = 0; q < NV; ++q) t[q] += ld_wt(&rc.lvl2[q * rc.l2s + j]);
  }
#pragma unroll
  for (int q = 0; q < NV; ++q) t[q] = eng::wave_sum(t[q]);
  MCG_RED_T(6);
  if (lane == 0) book(t, snap);
#if defined(MCG_CARRY_DIAG)
  MCG_RED_T(7);
  if (lane == 0)
    for (int i = 0; i < 8; ++i) g_red_diag[i] = t_red[i];
#endif
}

__device__ __noinline__ void f1_reduce_tail(double* out, int pstride, RedCtl rc, CgState* st, double tol) {
  last_arriver_reduce<4>(
      out, pstride, rc, [&] { return book_snap(st); },
      [&](const double* t, const BookSnap& s) { f1_bookkeep(st, s, t, rc.check, rc.first, tol); });
}

// end of a fused pass: block partials, then (rc on) the in-kernel reduction
template <int NW = kWaves>
__device__ __forceinline__ void f1_finish(double a0, double a1, double a2, double a3, double* __restrict__ out,
                                          int pstride, const RedCtl& rc, CgState* st, double tol) {
  block_partial4<NW>(a0, a1, a2, a3, out, pstride, rc.ngroups > 0);
  if (rc.ngroups > 0) f1_reduce_tail(out, pstride, rc, st, tol);
}

// non-temporal stores for the vectors the pass writes: they are re-read only by the next pass,
// after ~GBs of other traffic, so caching them is useless (A/B on 16384^2: +1.5-2 %,
// profiles/ab_nt_stores.log; -DMCG_NT_STORES=0 restores plain stores)
#ifndef MCG_NT_STORES
#define MCG_NT_STORES 1
#endif
template <typename T>
__device__ __forceinline__ void st_stream(T* p, T v) {
  if constexpr (MCG_NT_STORES) __builtin_nontemporal_store(v, p);
  else *p = v;
}
__device__ __forceinline__ void st_stream(double2* p, double2 v) {
  typedef double d2v __attribute__((ext_vector_type(2)));
  if constexpr (MCG_NT_STORES) {
    d2v w = {v.x, v.y};
    __builtin_nontemporal_store(w, reinterpret_cast<d2v*>(p));
  } else {
    *p = v;
  }
}

