// 3-D (7-pt) Ap-recomputing plane carry (the 2-D line carry's scheme, cg_carry_ar.hip, one plane deep;
// the kernel's own comment below), its lean plane runs and the host dispatcher cg_carry_ar3.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <type_traits>
#include <vector>

#include "mcg/check.hpp"
#include "mcg/kernels.hpp"
#include "spmv_engines.hpp"

namespace mcg {
namespace kern {
namespace {

#include "f1_common.hpp"
#include "carry_common.hpp"

// ---------------------------------------------------------------------------
// 3-D (7-pt) Ap-recomputing plane carry: the carried "line" is a plane (LO = N^2 rows), the
// matrix SELL-64/dia4 with the seven canonical offsets (-N^2, -N, -1, 0, +1, +N, +N^2).  A block
// of KW waves walks KW consecutive grid lines (y) of one x slice down the rank's planes (the 3-D
// store-form pass's block exchange, k_cg_f1_carry M2 == 2): the +-N neighbours of a wave's rows are
// the previous / next wave's rows, exchanged through LDS once per step (p_{k-1} of plane m + 1 for
// the recomputation of Ap_{k-1}, p_k of plane m for Ap_k).  The block's first / last wave take the
// grid line outside the block from memory -- its r, p and Ap_{k-1}, gathered two planes ahead --
// so Ap is stored (ext layout, v.ap_new) only where a neighbour needs it: the block's outer lines,
// the slices' edge rows (lanes 0 / 63, the x neighbours of other blocks' rows) and, at P > 1
// (gfull), the rank's first / last plane (the halo carries {r, Ap, p} of the ghost planes).
// Per row and iteration: r, p read + written once (32 B), x every second pass (12 B), Ap of 2 of
// KW lines written and read (4 B at KW = 8), 3.5 B of codes: ~52 B instead of the store form's 67.

// the KW-wave block's four fixed-order partials (block_partial4 for KW waves) + the in-kernel reduction
template <int KW>
__device__ __forceinline__ void ar3_finish(double a0, double a1, double a2, double a3, double* __restrict__ out,
                                           int pstride, const RedCtl& rc, CgState* st, double tol) {
  __shared__ double sh[4][KW];
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
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < KW; ++k) t += sh[threadIdx.x][k];
    if (rc.ngroups > 0) st_wt(&out[threadIdx.x * pstride + blockIdx.x], t);
    else out[threadIdx.x * pstride + blockIdx.x] = t;
  }
  if (rc.ngroups > 0) f1_reduce_tail(out, pstride, rc, st, tol);
}

// BIG (lean kernels): past 2^29 doubles a run's planes (N^2 rows each) do not fit 32-bit byte offsets
// from kernel-wide bases, so the lean loop re-bases its ext / x pointers every unrolled step group
// VC: SELL-64/diav 3-D (variable coefficients, S.cvd / cve / cvs / cvt) instead of dia4 codes; the
// lean loop carries the streamed values per lane, so these kernels run 2 waves per SIMD (256 VGPRs)
template <int QD, bool PAIR, int KW, bool P3, bool LEAN = false, bool BIG = false, bool VC = false, bool T3 = false>
__global__ __launch_bounds__(64 * KW, VC ? 2 : 4) void k_cg_carry_ar3(SellDev S, F1Vectors v, int64_t own,
                                                                          TileRanges tr, int32_t LN, int gfull,
                                                                          double* __restrict__ partials, int pstride,
                                                                          CgState* st, double tol, int first,
                                                                          int check, RedCtl rc) {
  static_assert(KW >= 2 && QD >= 2, "3-D carry: >= 2 waves per block, operands >= 2 planes ahead");
  static_assert(!(VC && BIG), "3-D diav: 32-bit byte offsets (ranks below 2^29 rows)");
  static_assert(!T3 || (P3 && LEAN), "3-D three p buffers: the lean kernels");
  constexpr int U = 7;
  using Co = ArCodes<VC ? 6 : 4, U>;
  __shared__ double s_val[16];
  __shared__ double s_x[2][2][KW][64];  // [step parity][p_{k-1}(m+1), p_k(m)][wave][lane]
  const F1Scalars sc = f1_scalars(st, tol, first, check);
  if (st->done || sc.conv) {
    ar3_finish<KW>(0.0, 0.0, 0.0, 0.0, partials, pstride, rc, st, tol);
    return;
  }
  if constexpr (!VC) {
    if (threadIdx.x < 16) s_val[threadIdx.x] = S.dvals[threadIdx.x];
  }
  __syncthreads();
  const double a = sc.alpha, b = sc.beta, na = -a, ap = st->a_prev;
  // three-term form (P3, as in k_cg_carry_ar): r_{k-1} = p_{k-1} - b_prev p_{k-2} on the run's own
  // planes; r stored (as that recovered value) only where another wave reads it: the block's outer
  // lines, the slices' edge rows and the run's first / last plane (the halo's source at P > 1);
  // pass 0 runs the two-term kernel (see k_cg_carry_ar).  T3 (lean kernels, three p buffers:
  // F1Vectors::p_m2): p_{k-2} is never overwritten during the pass, so every one of those readers
  // recovers r from p_{k-1} / p_{k-2} itself and no r is stored at all (512^3: 1103 vs 1010 it/s,
  // profiles/r5/p3buf3d)
  constexpr bool rfull = !P3;
  const double nbp = P3 ? -st->b_prev : 0.0;
  const double* __restrict__ ro = v.r_old;
  const double* __restrict__ po = v.p_old;
  double* __restrict__ rn = v.r_new;
  double* __restrict__ pn = v.p_new;
  double* __restrict__ x = v.x;
  const double* __restrict__ apo = v.ap_old;  // Ap_{k-1}: outer lines, edge rows, ghost planes
  double* __restrict__ apw = v.ap_new;
  // P3: the slices' edge rows' Ap and r in compact per-slice arrays (2 doubles per slice each, as
  // k_cg_carry_ar), not scattered through the ext-layout vectors; pass 0 (two-term kernel) fills them
  const double* __restrict__ eao = v.ape_old;
  double* __restrict__ ean = v.ape_new;
  const double* __restrict__ reo = v.re_old;
  double* __restrict__ ren = v.re_new;
  const int64_t nsl = tr.nt0;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t SS = tr.strip;            // slices per plane
  const int32_t LO = (int32_t)(SS * 64);  // one plane
  const int64_t nl = tr.nt0 / SS;         // the rank's planes
  const int64_t G = LN / 64;              // slices per grid line
  const int64_t jpr = (LN / KW) * G;      // jobs (y group, x slice) per run of planes
  const int64_t nb = gridDim.x, blk = blockIdx.x;
  const int64_t lb = (nb % 8 == 0) ? (blk % 8) * (nb / 8) + blk / 8 : blk;  // XCD-aware (k_cg_f1_carry)
  const int64_t runs = tr.runs3 > 0 ? tr.runs3 : (nb > jpr ? nb / jpr : 1);
  const int64_t chunk = (nl + runs - 1) / runs;
  const int32_t ext32 = (int32_t)v.ext_len;
  constexpr bool ntl = false;  // plain loads (non-temporal measured slower: 281 vs 302 it/s 2-D)
  const bool odn = wv == 0, oup = wv == KW - 1;  // outer waves: the line below / above the block
  const int32_t fo = odn ? -LN : LN;
  double s_pap = 0.0, s_rap = 0.0, s_apap = 0.0, s_rr = 0.0;
  struct Raw {
    double r, p;
  };
  struct Edge {
    double r, a, p;
  };
  struct XP {
    double pkm2, xo;
  };
  struct Far {  // the outside line's row (outer waves): r, p, Ap of iteration k-1
    double r, p, a;
  };
  auto stencil = [&](const Co& c, double mid, double edge, double dnl, double upl, double dnn, double upn) {
    const double sh_up = lane_up(mid);
    const double sh_dn = lane_dn(mid);
    const double upv = lane == 63 ? edge : sh_up;
    const double dnv = lane == 0 ? edge : sh_dn;
    const double g[7] = {dnl, dnn, dnv, mid, upv, upn, upl};
    double sum = 0.0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (VC) sum = fma(c.k[u], g[u], sum);
      else sum = fma(s_val[(c.pk[0] >> (4 * u)) & 15u], g[u], sum);
    }
    return sum;
  };
  auto pk_of = [&](double r, double a_, double p) { return fma(b, p, fma(na, a_, r)); };
  // neighbour waves' values through LDS (outer waves: `far` for the side outside the block)
  auto nbr = [&](int par, int which, double far, double& dn, double& up) {
    const double* sx = &s_x[par][which][0][lane];
    const double vd = sx[(odn ? wv : wv - 1) * 64], vu = sx[(oup ? wv : wv + 1) * 64];
    dn = odn ? far : vd;
    up = oup ? far : vu;
  };
  for (int64_t job = lb; job < jpr * runs; job += nb) {
    const int64_t run = job / jpr, q = job % jpr;
    const int64_t col = ((q / G) * KW + wv) * G + q % G;  // slice of grid line y = yg KW + wv, x slice q % G
    const int64_t l0 = run * chunk;
    const int64_t l1 = l0 + chunk < nl ? l0 + chunk : nl;
    if (l0 >= l1) continue;  // block-uniform
    const int64_t sl0 = l0 * SS + col;
    const int32_t e0 = (int32_t)(own + sl0 * 64);
    const int32_t i0 = (int32_t)(sl0 * 64);
    const int32_t n_run = (int32_t)(l1 - l0);
    if constexpr (P3) {
      // Lean run (the 2-D kernel's, per wave, with the +-N rows through LDS as in the step below):
      // the seven values in scalar registers, no codes streamed, global base + 32-bit byte offset
      // accesses; bitwise what the generic step computes.  Block-uniform: the waves exchange rows
      // every step, so the block takes it only when every wave's run qualifies (one barrier,
      // which is also the barrier after the previous job's last LDS reads).  A wave on the grid's
      // first / last y line has no far row (its -N / +N slot is absent): it reads its own row,
      // which the absent slot's 0 multiplies as it would the clamped one.
      // Streams: operands RD = 3 planes ahead (the stencil of plane m + 1 needs plane m + 2), edge /
      // far rows and x ED = 2 ahead (their values are short-lived; 128 VGPRs); the 6-step unroll
      // renames both chain lengths
      constexpr int LD = 3, ED = 2, UNR = 6;
      uint32_t WA = 0, WB = 0, WC = 0;
      if constexpr (LEAN && !VC) {  // every run checked at setup (carry_lean_failures)
        (void)lean_eligible<true>(S.dpat, l0, l1, nl, SS, col, v.ext_len, WA, WB, WC, BIG ? 1 : 0);
        __syncthreads();  // the previous job's last step has read its LDS slots
      }
      if constexpr (LEAN && VC) {
        // Variable coefficients (SELL-64/diav 3-D): the loop below with the seven values of a plane
        // per lane instead of in scalar registers.  Streamed from HBM: the row's own d, e, s, t (32 B;
        // the arrays have one plane in front).  Re-read from cache: south s[i - N] (the neighbouring
        // wave's line of the same plane, loaded there this step) and lane 0's west e[i - 1].  Carried:
        // west = e one lane down (DPP), down = the previous plane's t.  A value of 0 (absent entry:
        // grid edges) multiplies the same clamped, finite operand as the generic step; every run of
        // >= 3 planes qualifies (setup).  Coefficients 2 planes ahead.
        struct VSet {
          double v[7];
        };
        struct CRaw {
          double d, e, s, t, ss, ee;
        };
        __syncthreads();  // the previous job's last step has read its LDS slots
        const int64_t yl = (q / G) * KW + wv;  // the wave's grid line
        const bool fnone = (odn && yl == 0) || (oup && yl == LN - 1);
        const bool z0 = q % G == 0, z63 = q % G == G - 1;  // slices at a grid line's start / end
        const bool hi = lane == 63, edge_lane = lane == 0 || lane == 63;
        const bool outer = odn || oup;
        const uint32_t l8 = (uint32_t)lane << 3;
        const uint32_t LOB = (uint32_t)LO << 3;
        const uint32_t SB = (uint32_t)(2 * SS) << 3;
        const uint32_t NB = (uint32_t)LN << 3;  // one grid line of rows
        const uint32_t ob0 = (uint32_t)e0 << 3, xb0 = (uint32_t)i0 << 3;
        const uint32_t kb0 = ((uint32_t)i0 << 3) + LOB;
        const uint32_t cb0 = (uint32_t)(2 * (l0 * SS + col) - 1) << 3;
        const uint32_t oc = hi ? (z63 ? 16u : 24u) : (z0 ? 8u : 0u);
        const uint32_t op = hi ? (z63 ? 512u : 520u) : (z0 ? 8u : 0u);
        const uint32_t fob = fnone ? 0u : (uint32_t)fo << 3;
        const int32_t jlo = -(e0 / LO), jhi = (ext32 - 64 - e0) / LO;
        const int32_t rlo = -(int32_t)l0, rhi = (int32_t)(nl - 1 - l0);
        auto jc = [&](int32_t j) { return j < jlo ? jlo : (j > jhi ? jhi : j); };
        auto rc_ = [&](int32_t j) { return j < rlo ? rlo : (j > rhi ? rhi : j); };
        auto line_ofs = [&](int32_t j) { return ob0 + (uint32_t)j * LOB; };
        PullBases pl;  // in-kernel halo (the 2-D lean loops')
        pl.at(v, 0);
        // T3: p_{k-2} read-only in its own buffer; r_{k-1} recovered everywhere (the dia4 loop below)
        const double* __restrict__ pm2 = T3 ? v.p_m2 : (const double*)pn;
        auto rv = [&](double r, double p) { return T3 ? fma(nbp, r, p) : r; };
        auto raw_ld = [&](int32_t j, int32_t k) {
          Raw r;
          const uint32_t o = line_ofs(k) + l8;
          r.r = T3 ? g_ld(pm2, o) : g_ld((j >= 0 && j < n_run) ? (const double*)pn : ro, o);
          r.p = pl.ld_p(pl.side(l0 + k, nl), po, o);
          return r;
        };
        auto ap_gh = [&](int32_t j) { return pl.ld_ap(pl.side(l0 + j, nl), apo, line_ofs(j) + l8); };
        auto edge_ld = [&](int32_t j) {
          Edge r;
          const uint32_t c = cb0 + (uint32_t)rc_(j) * SB + oc;
          r.r = T3 ? g_ld(pm2, line_ofs(jc(j)) - 8u + op) : g_ld(reo, c);
          r.a = g_ld(eao, c);
          r.p = g_ld(po, line_ofs(jc(j)) - 8u + op);
          return r;
        };
        auto edge_un = [&](int32_t j) {
          Edge r;
          const uint32_t c = cb0 + (uint32_t)j * SB + oc;
          r.r = T3 ? g_ld(pm2, line_ofs(j) - 8u + op) : g_ld(reo, c);
          r.a = g_ld(eao, c);
          r.p = g_ld(po, line_ofs(j) - 8u + op);
          return r;
        };
        auto rghost = [&](int32_t j, const Raw& qq) { return fma(nbp, g_ld(T3 ? pm2 : (const double*)pn, line_ofs(j) + l8), qq.p); };
        auto is_ghost = [&](int32_t j) { return gfull && (l0 + j == -1 || l0 + j == nl) && j >= jlo && j <= jhi; };
        auto far_ld = [&](int32_t k) {
          Far f{0.0, 0.0, 0.0};
          if (outer) {
            const uint32_t o = line_ofs(k) + l8 + fob;
            f.r = g_ld(T3 ? pm2 : ro, o);
            f.p = g_ld(po, o);
            f.a = g_ld(apo, o);
          }
          return f;
        };
        auto x_at = [&](int32_t j) {
          if constexpr (PAIR) return g_ld(x, xb0 + (uint32_t)(j < n_run - 1 ? j : n_run - 1) * LOB + l8);
          else return 0.0;
        };
        // plane j's values (j >= rlo - 1: the front plane, whose t alone is read; its south / west
        // loads take plane rlo's addresses instead, which stay inside the arrays)
        auto coef_ld = [&](int32_t j, int32_t jo) {
          CRaw c;
          const uint32_t o = kb0 + (uint32_t)j * LOB + l8, oo = kb0 + (uint32_t)jo * LOB;
          c.d = g_ld(S.cvd, o);
          c.e = g_ld(S.cve, o);
          c.s = g_ld(S.cvs, o);
          c.t = g_ld(S.cvt, o);
          c.ss = g_ld(S.cvs, oo + l8 - NB);
          c.ee = g_ld(S.cve, oo - 8u);
          return c;
        };
        auto coef_at = [&](int32_t j) {
          const int32_t k = j < rlo - 1 ? rlo - 1 : (j > rhi ? rhi : j);
          return coef_ld(k, k < rlo ? rlo : k);
        };
        auto coef_un = [&](int32_t j) { return coef_ld(j, j); };
        auto mkv = [&](const CRaw& c, double t_dn) {
          VSet V;
          V.v[0] = t_dn;
          V.v[1] = c.ss;
          V.v[2] = lane_dn_or(c.e, c.ee);
          V.v[3] = c.d;
          V.v[4] = c.e;
          V.v[5] = c.s;
          V.v[6] = c.t;
          return V;
        };
        auto stencil_v = [&](const VSet& V, double mid, double edge, double dnl, double upl, double dnn, double upn) {
          const double upv = lane_up_or(mid, edge);
          const double dnv = lane_dn_or(mid, edge);
          double sum = fma(V.v[0], dnl, 0.0);
          sum = fma(V.v[1], dnn, sum);
          sum = fma(V.v[2], dnv, sum);
          sum = fma(V.v[3], mid, sum);
          sum = fma(V.v[4], upv, sum);
          sum = fma(V.v[5], upn, sum);
          return fma(V.v[6], upl, sum);
        };
        auto epk = [&](const Edge& e) { return pk_of(rv(e.r, e.p), e.a, e.p); };
        const Raw rm2 = raw_ld(-2, jc(-2)), rm1 = raw_ld(-1, jc(-1)), r0 = raw_ld(0, 0);
        Raw qv[LD - 1];
#pragma unroll
        for (int d = 0; d < LD - 1; ++d) qv[d] = raw_ld(1 + d, jc(1 + d));
        const Edge edm1 = edge_ld(-1), ed0 = edge_ld(0);
        Edge ev[ED - 1];
#pragma unroll
        for (int d = 0; d < ED - 1; ++d) ev[d] = edge_ld(1 + d);
        const Far fm1 = far_ld(jc(-1)), f0 = far_ld(0);
        Far fv[ED - 1];
#pragma unroll
        for (int d = 0; d < ED - 1; ++d) fv[d] = far_ld(jc(1 + d));
        double xs[ED - 1];
#pragma unroll
        for (int d = 0; d < ED - 1; ++d) xs[d] = x_at(d);
        const CRaw cm2 = coef_at(-2), cm1 = coef_at(-1), c0 = coef_at(0);
        CRaw cq = coef_at(1);  // plane m + 1
        s_x[1][0][wv][lane] = rm1.p;
        s_x[1][1][wv][lane] = r0.p;
        __syncthreads();
        double pr_pk = 0.0;
        if (l0 >= 1) {
          double dn, up;
          nbr(1, 0, fm1.p, dn, up);
          const double t = stencil_v(mkv(cm1, cm2.t), rm1.p, edm1.p, rm2.p, r0.p, dn, up);
          pr_pk = fma(b, rm1.p, fma(na, t, rv(rm1.r, rm1.p)));
        } else if (is_ghost(-1)) {
          pr_pk = pk_of(rghost(-1, rm1), ap_gh(-1), rm1.p);
          if (pl.p[0] != nullptr) g_st(const_cast<double*>(po), line_ofs(-1) + l8, rm1.p);
        }
        VSet Vs = mkv(c0, cm1.t);  // plane m
        double o_pold = r0.p, o_pm2 = r0.r, o_rk, o_pk;
        {
          double dn, up;
          nbr(1, 1, f0.p, dn, up);
          const double t = stencil_v(Vs, r0.p, ed0.p, rm1.p, qv[0].p, dn, up);
          o_rk = fma(na, t, fma(nbp, r0.r, r0.p));
          o_pk = fma(b, r0.p, o_rk);
        }
        double o_epk = epk(ed0);
        double o_fpk = pk_of(rv(f0.r, f0.p), f0.a, f0.p);
        // next: 1 plane m + 1 owned, 2 a ghost plane, 0 none
        auto lstep = [&](auto clc, int32_t m, int next) __attribute__((always_inline)) {
          constexpr bool CL = decltype(clc)::value;
          const int par = m & 1;
          const uint32_t ob = line_ofs(m);
          const double rr = fma(-b, o_pold, o_pk);
          if constexpr (!T3) {
            if (m == 0 || m == n_run - 1) g_st_nt(rn, ob + l8, rr);
            else if (outer) g_st(rn, ob + l8, rr);
          }
          const Raw qn = raw_ld(m + LD, CL ? jc(m + LD) : m + LD);
          const Edge en2 = CL ? edge_ld(m + ED) : edge_un(m + ED);
          const Far fn = far_ld(CL ? jc(m + ED) : m + ED);
          const double xn = x_at(m + ED - 1);
          const CRaw cn = CL ? coef_at(m + 2) : coef_un(m + 2);
          s_x[par][0][wv][lane] = qv[0].p;
          s_x[par][1][wv][lane] = o_pk;
          __syncthreads();
          const VSet Vt = mkv(cq, Vs.v[6]);  // plane m + 1 (down: plane m's up values)
          double rk1 = 0.0, pk1 = 0.0;
          if (next == 1) {
            double dn, up;
            nbr(par, 0, fv[0].p, dn, up);
            const double t = stencil_v(Vt, qv[0].p, ev[0].p, o_pold, qv[1].p, dn, up);
            rk1 = fma(na, t, (T3 || m + 1 < n_run) ? fma(nbp, qv[0].r, qv[0].p) : qv[0].r);
            pk1 = fma(b, qv[0].p, rk1);
          } else if (CL && next == 2) {
            rk1 = fma(na, ap_gh(m + 1), rghost(m + 1, qv[0]));
            pk1 = fma(b, qv[0].p, rk1);
            if (pl.p[1] != nullptr) g_st(const_cast<double*>(po), line_ofs(m + 1) + l8, qv[0].p);
          }
          double kdn, kup;
          nbr(par, 1, o_fpk, kdn, kup);
          const double sum = stencil_v(Vs, o_pk, o_epk, pr_pk, pk1, kdn, kup);
          if constexpr (PAIR) g_st_nt(x, xb0 + (uint32_t)m * LOB + l8, fma(a, o_pold, fma(ap, o_pm2, xs[0])));
          const bool bnd = CL && gfull && (l0 + m == 0 || l0 + m == nl - 1);  // the halo's source planes
          if constexpr (CL) pl.st_pub(bnd, pn, ob + l8, o_pk, true);
          else g_st_nt(pn, ob + l8, o_pk);
          if (bnd) pl.st_pub(true, apw, ob + l8, sum, false);
          else if (outer) g_st(apw, ob + l8, sum);
          if (edge_lane) {
            const uint32_t sb = cb0 + (uint32_t)m * SB + (hi ? 16u : 8u);
            g_st(ean, sb, sum);
            if constexpr (!T3) g_st(ren, sb, rr);
          }
          s_pap = fma(o_pk, sum, s_pap);
          s_rap = fma(o_rk, sum, s_rap);
          s_apap = fma(sum, sum, s_apap);
          s_rr = fma(o_rk, o_rk, s_rr);
          pr_pk = o_pk;
          o_pk = pk1;
          o_rk = rk1;
          o_pold = qv[0].p;
          o_pm2 = qv[0].r;
          o_epk = epk(ev[0]);
          o_fpk = pk_of(rv(fv[0].r, fv[0].p), fv[0].a, fv[0].p);
          Vs = Vt;
          cq = cn;
#pragma unroll
          for (int d = 0; d + 1 < LD - 1; ++d) qv[d] = qv[d + 1];
#pragma unroll
          for (int d = 0; d + 1 < ED - 1; ++d) {
            ev[d] = ev[d + 1];
            fv[d] = fv[d + 1];
            xs[d] = xs[d + 1];
          }
          qv[LD - 2] = qn;
          ev[ED - 2] = en2;
          fv[ED - 2] = fn;
          xs[ED - 2] = xn;
        };
        const std::true_type clamped;
        const std::false_type unclamped;
        const int32_t m_lo = l0 == 0 ? 1 : 0;
        const int32_t m_hi = min(n_run - 1, (int32_t)(nl - 1 - LD - l0));
        int32_t m = 0;
        if (m_lo == 1) lstep(clamped, 0, 1);
        m = m_lo;
        for (; m + UNR - 1 <= m_hi; m += UNR) {
#pragma unroll
          for (int u = 0; u < UNR; ++u) lstep(unclamped, m + u, 1);
        }
        for (; m <= m_hi; ++m) lstep(unclamped, m, 1);
        for (; m < n_run; ++m) {
          const bool lastl = l0 + m == nl - 1;
          lstep(clamped, m, !lastl ? 1 : (is_ghost(m + 1) ? 2 : 0));
        }
        pl.release(l0, l1, nl);
        continue;
      }
      if constexpr (LEAN && !VC) {
        struct VSet {
          double v[7];
        };
        auto vals = [&](uint32_t P) {
          VSet V;
#pragma unroll
          for (int u = 0; u < 7; ++u) V.v[u] = uni_d(s_val[(P >> (4 * u)) & 15u]);
          return V;
        };
        const bool z0 = (WB >> 28) & 1u, z63 = (WB >> 29) & 1u;
        const int64_t yl = (q / G) * KW + wv;  // the wave's grid line
        const bool fnone = (odn && yl == 0) || (oup && yl == LN - 1);
        {
          const VSet VB = vals(WB);
          const bool hi = lane == 63, edge_lane = lane == 0 || lane == 63;
          const bool zlo = lane == 0 && z0, zhi = hi && z63;  // lanes whose -1 / +1 entry is absent
          const bool outer = odn || oup;
          const uint32_t l8 = (uint32_t)lane << 3;
          const uint32_t LOB = (uint32_t)LO << 3;                         // one plane of the vectors
          const uint32_t SB = (uint32_t)(2 * SS) << 3;                    // one plane of the edge arrays
          // BIG: pointers based at the run's plane -3 (ext) / 0 (x) once (the setup keeps every run's
          // planes -3 .. end + 4 within 4 GiB: carry3_runs max_chunk; a base moved along the run spilled
          // 60 VGPRs and ran at half the rate); the 32-bit offsets are then planes from there.  !BIG:
          // kernel-wide bases
          int32_t mb = 0;
          const double *po_ = po, *ro_ = ro, *apo_ = apo;
          double *pn_ = pn, *rn_ = rn, *x_ = x, *apw_ = apw;
          // T3 (three p buffers): p_{k-2} read-only in its own buffer, so r_{k-1} is recovered from
          // p_{k-1} / p_{k-2} on every plane, outer line and edge row -- no r stored anywhere
          const double* pm2_ = T3 ? v.p_m2 : (const double*)pn;
          auto rebase = [&](int32_t m) {
            if constexpr (BIG) {
              mb = m;
              const int64_t eb = (int64_t)e0 + (int64_t)(m - 3) * LO, xb = (int64_t)i0 + (int64_t)m * LO;
              if constexpr (T3) pm2_ = v.p_m2 + eb;
              po_ = po + eb;
              ro_ = ro + eb;
              apo_ = apo + eb;
              pn_ = pn + eb;
              rn_ = rn + eb;
              apw_ = apw + eb;
              x_ = x + xb;
            }
          };
          rebase(0);
          const uint32_t ob0 = BIG ? 3u * ((uint32_t)LO << 3) : (uint32_t)e0 << 3;  // plane 0 (ext layout)
          const uint32_t xb0 = BIG ? 0u : (uint32_t)i0 << 3;                         // plane 0 of x
          const uint32_t cb0 = (uint32_t)(2 * (l0 * SS + col) - 1) << 3;  // edge arrays: 2 s - 1 of plane 0
          const uint32_t oc = hi ? (z63 ? 16u : 24u) : (z0 ? 8u : 0u);
          const uint32_t op = hi ? (z63 ? 512u : 520u) : (z0 ? 8u : 0u);
          const uint32_t fob = fnone ? 0u : (uint32_t)fo << 3;  // the far row, bytes from the wave's own
          // planes of the ext vectors (ghosts included; the generic ebase) and of the rank (oline)
          const int32_t jlo = -(e0 / LO), jhi = (ext32 - 64 - e0) / LO;
          const int32_t rlo = -(int32_t)l0, rhi = (int32_t)(nl - 1 - l0);
          auto jc = [&](int32_t j) { return j < jlo ? jlo : (j > jhi ? jhi : j); };
          auto rc_ = [&](int32_t j) { return j < rlo ? rlo : (j > rhi ? rhi : j); };
          auto line_ofs = [&](int32_t j) { return ob0 + (uint32_t)(j - mb) * LOB; };
          PullBases pl;  // in-kernel halo (the 2-D lean loops'; BIG: based like po_, at plane -3)
          pl.at(v, BIG ? (int64_t)e0 - 3 * (int64_t)LO : 0);
          auto raw_ld = [&](int32_t j, int32_t k) {  // plane j's source, plane k's address
            Raw r;
            const uint32_t o = line_ofs(k) + l8;
            r.r = T3 ? g_ld(pm2_, o) : g_ld((j >= 0 && j < n_run) ? (const double*)pn_ : ro_, o);
            r.p = pl.ld_p(pl.side(l0 + k, nl), po_, o);
            return r;
          };
          auto ap_gh = [&](int32_t j) { return pl.ld_ap(pl.side(l0 + j, nl), apo_, line_ofs(j) + l8); };
          auto edge_ld = [&](int32_t j) {  // plane j (clamped: compact index to the rank, row to ext)
            Edge r;
            const uint32_t c = cb0 + (uint32_t)rc_(j) * SB + oc;
            r.r = T3 ? g_ld(pm2_, line_ofs(jc(j)) - 8u + op) : g_ld(reo, c);  // T3: the row's p_{k-2}
            r.a = g_ld(eao, c);
            r.p = g_ld(po_, line_ofs(jc(j)) - 8u + op);
            return r;
          };
          auto edge_un = [&](int32_t j) {
            Edge r;
            const uint32_t c = cb0 + (uint32_t)j * SB + oc;
            r.r = T3 ? g_ld(pm2_, line_ofs(j) - 8u + op) : g_ld(reo, c);
            r.a = g_ld(eao, c);
            r.p = g_ld(po_, line_ofs(j) - 8u + op);
            return r;
          };
          auto rghost = [&](int32_t j, const Raw& q) { return fma(nbp, g_ld(T3 ? pm2_ : (const double*)pn_, line_ofs(j) + l8), q.p); };
          auto is_ghost = [&](int32_t j) { return gfull && (l0 + j == -1 || l0 + j == nl) && j >= jlo && j <= jhi; };
          auto far_ld = [&](int32_t k) {
            Far f{0.0, 0.0, 0.0};
            if (outer) {
              const uint32_t o = line_ofs(k) + l8 + fob;
              f.r = g_ld(T3 ? pm2_ : ro_, o);
              f.p = g_ld(po_, o);
              f.a = g_ld(apo_, o);
            }
            return f;
          };
          auto x_at = [&](int32_t j) {
            if constexpr (PAIR) return g_ld(x_, xb0 + (uint32_t)((j < n_run - 1 ? j : n_run - 1) - mb) * LOB + l8);
            else return 0.0;
          };
          auto ez = [&](double e) { return e; };
          auto stencil_u = [&](const VSet& V, double mid, double edge, double dnl, double upl, double dnn, double upn) {
            const double upv = lane_up_or(mid, edge);
            const double dnv = lane_dn_or(mid, edge);
            const double cm = zlo ? 0.0 : V.v[2], cp = zhi ? 0.0 : V.v[4];  // loop-invariant
            double sum = fma(V.v[0], dnl, 0.0);
            sum = fma(V.v[1], dnn, sum);
            sum = fma(cm, dnv, sum);
            sum = fma(V.v[3], mid, sum);
            sum = fma(cp, upv, sum);
            sum = fma(V.v[5], upn, sum);
            return fma(V.v[6], upl, sum);
          };
          // T3: the loaded r is p_{k-2}; recovered at the use, not at the (early) load
          auto rv = [&](double r, double p) { return T3 ? fma(nbp, r, p) : r; };
          auto epk = [&](const Edge& e) { return pk_of(rv(e.r, e.p), e.a, e.p); };
          // prologue (the generic one's): planes -2 .. LD - 1
          const Raw rm2 = raw_ld(-2, jc(-2)), rm1 = raw_ld(-1, jc(-1)), r0 = raw_ld(0, 0);
          Raw qv[LD - 1];  // planes m + 1 .. m + LD - 1
#pragma unroll
          for (int d = 0; d < LD - 1; ++d) qv[d] = raw_ld(1 + d, jc(1 + d));
          const Edge edm1 = edge_ld(-1), ed0 = edge_ld(0);
          Edge ev[ED - 1];  // planes m + 1 .. m + ED - 1
#pragma unroll
          for (int d = 0; d < ED - 1; ++d) ev[d] = edge_ld(1 + d);
          const Far fm1 = far_ld(jc(-1)), f0 = far_ld(0);
          Far fv[ED - 1];
#pragma unroll
          for (int d = 0; d < ED - 1; ++d) fv[d] = far_ld(jc(1 + d));
          double xs[ED - 1];  // planes m .. m + ED - 2
#pragma unroll
          for (int d = 0; d < ED - 1; ++d) xs[d] = x_at(d);
          s_x[1][0][wv][lane] = rm1.p;
          s_x[1][1][wv][lane] = r0.p;
          __syncthreads();
          double pr_pk = 0.0;
          if (l0 >= 1) {
            double dn, up;
            nbr(1, 0, fm1.p, dn, up);
            const VSet Vm = l0 == 1 ? vals(WA) : VB;
            const double t = stencil_u(Vm, rm1.p, ez(edm1.p), rm2.p, r0.p, dn, up);
            pr_pk = fma(b, rm1.p, fma(na, t, rv(rm1.r, rm1.p)));
          } else if (is_ghost(-1)) {
            pr_pk = pk_of(rghost(-1, rm1), ap_gh(-1), rm1.p);
            if (pl.p[0] != nullptr) g_st(const_cast<double*>(po_), line_ofs(-1) + l8, rm1.p);
          }
          double o_pold = r0.p, o_pm2 = r0.r, o_rk, o_pk;
          {
            double dn, up;
            nbr(1, 1, f0.p, dn, up);
            const VSet V0 = l0 == 0 ? vals(WA) : VB;
            const double t = stencil_u(V0, r0.p, ez(ed0.p), rm1.p, qv[0].p, dn, up);
            o_rk = fma(na, t, fma(nbp, r0.r, r0.p));
            o_pk = fma(b, r0.p, o_rk);
          }
          double o_epk = epk(ed0);
          double o_fpk = pk_of(rv(f0.r, f0.p), f0.a, f0.p);
          // next: 1 plane m + 1 owned (values Vt), 2 a ghost plane, 0 none
          auto lstep = [&](auto clc, int32_t m, const VSet& Vs, const VSet& Vt, int next) __attribute__((always_inline)) {
            constexpr bool CL = decltype(clc)::value;
            const int par = m & 1;
            const uint32_t ob = line_ofs(m);
            const double rr = fma(-b, o_pold, o_pk);
            if constexpr (!T3) {
              if (m == 0 || m == n_run - 1) g_st_nt(rn_, ob + l8, rr);
              else if (outer) g_st(rn_, ob + l8, rr);
            }
            const int32_t kn = CL ? jc(m + LD) : m + LD;
            const Raw qn = raw_ld(m + LD, kn);
            const Edge en2 = CL ? edge_ld(m + ED) : edge_un(m + ED);
            const Far fn = far_ld(CL ? jc(m + ED) : m + ED);
            const double xn = x_at(m + ED - 1);
            s_x[par][0][wv][lane] = qv[0].p;
            s_x[par][1][wv][lane] = o_pk;
            __syncthreads();
            double rk1 = 0.0, pk1 = 0.0;
            if (next == 1) {
              double dn, up;
              nbr(par, 0, fv[0].p, dn, up);
              const double t = stencil_u(Vt, qv[0].p, ez(ev[0].p), o_pold, qv[1].p, dn, up);
              rk1 = fma(na, t, (T3 || m + 1 < n_run) ? fma(nbp, qv[0].r, qv[0].p) : qv[0].r);
              pk1 = fma(b, qv[0].p, rk1);
            } else if (CL && next == 2) {
              rk1 = fma(na, ap_gh(m + 1), rghost(m + 1, qv[0]));
              pk1 = fma(b, qv[0].p, rk1);
              if (pl.p[1] != nullptr) g_st(const_cast<double*>(po_), line_ofs(m + 1) + l8, qv[0].p);
            }
            double kdn, kup;
            nbr(par, 1, o_fpk, kdn, kup);
            const double sum = stencil_u(Vs, o_pk, o_epk, pr_pk, pk1, kdn, kup);
            if constexpr (PAIR) g_st_nt(x_, xb0 + (uint32_t)(m - mb) * LOB + l8, fma(a, o_pold, fma(ap, o_pm2, xs[0])));
            const bool bnd = CL && gfull && (l0 + m == 0 || l0 + m == nl - 1);  // the halo's source planes
            if constexpr (CL) pl.st_pub(bnd, pn_, ob + l8, o_pk, true);
            else g_st_nt(pn_, ob + l8, o_pk);
            if (bnd) pl.st_pub(true, apw_, ob + l8, sum, false);
            else if (outer) g_st(apw_, ob + l8, sum);
            if (edge_lane) {
              const uint32_t sb = cb0 + (uint32_t)m * SB + (hi ? 16u : 8u);  // 2 s, 2 s + 1
              g_st(ean, sb, sum);
              if constexpr (!T3) g_st(ren, sb, rr);
            }
            s_pap = fma(o_pk, sum, s_pap);
            s_rap = fma(o_rk, sum, s_rap);
            s_apap = fma(sum, sum, s_apap);
            s_rr = fma(o_rk, o_rk, s_rr);
            pr_pk = o_pk;
            o_pk = pk1;
            o_rk = rk1;
            o_pold = qv[0].p;
            o_pm2 = qv[0].r;
            o_epk = epk(ev[0]);
            o_fpk = pk_of(rv(fv[0].r, fv[0].p), fv[0].a, fv[0].p);
#pragma unroll
            for (int d = 0; d + 1 < LD - 1; ++d) qv[d] = qv[d + 1];
#pragma unroll
            for (int d = 0; d + 1 < ED - 1; ++d) {
              ev[d] = ev[d + 1];
              fv[d] = fv[d + 1];
              xs[d] = xs[d + 1];
            }
            qv[LD - 2] = qn;
            ev[ED - 2] = en2;
            fv[ED - 2] = fn;
            xs[ED - 2] = xn;
          };
          const std::true_type clamped;
          const std::false_type unclamped;
          const int32_t m_lo = l0 == 0 ? 1 : 0;
          const int32_t m_hi = min(n_run - 1, (int32_t)(nl - 1 - LD - l0));
          int32_t m = 0;
          if (m_lo == 1) lstep(clamped, 0, vals(WA), VB, 1);
          m = m_lo;
          for (; m + UNR - 1 <= m_hi; m += UNR) {
#pragma unroll
            for (int u = 0; u < UNR; ++u) lstep(unclamped, m + u, VB, VB, 1);
          }
          for (; m <= m_hi; ++m) lstep(unclamped, m, VB, VB, 1);
          if (m < n_run) {
            const VSet VL = vals(WC);
            for (; m < n_run; ++m) {
              const bool lastl = l0 + m == nl - 1;
              const bool nextc = l0 + m + 1 == nl - 1;
              lstep(clamped, m, lastl ? VL : VB, nextc ? VL : VB, !lastl ? 1 : (is_ghost(m + 1) ? 2 : 0));
            }
          }
          pl.release(l0, l1, nl);
        }
        continue;
      }
    }
    if constexpr (!LEAN) {
    const int32_t jmax = (ext32 - 64 - e0) / LO;
    const int32_t jmin = -(e0 / LO);
    auto ebase = [&](int32_t j) { return e0 + (j < jmin ? jmin : (j > jmax ? jmax : j)) * LO; };
    auto owned = [&](int32_t j) { return l0 + j >= 0 && l0 + j < nl; };
    auto oline = [&](int32_t j) {
      const int64_t L = l0 + j;
      return L < 0 ? (int64_t)0 : (L >= nl ? nl - 1 : L);
    };
    auto clampr = [&](int32_t e) { return e < 0 ? 0 : (e >= ext32 ? ext32 - 1 : e); };
    auto inrun = [&](int32_t j) { return !rfull && j >= 0 && j < n_run; };
    auto load_raw = [&](int32_t j, Raw& r) {
      const int32_t e = ebase(j) + lane;
      r.r = ld_once((inrun(j) ? (const double*)pn : ro) + e, ntl);
      r.p = ld_once(po + e, ntl);
    };
    auto rof = [&](int32_t j, const Raw& q) { return inrun(j) ? fma(nbp, q.r, q.p) : q.r; };
    auto load_edge = [&](int32_t j, Edge& r) {
      const int32_t e = ebase(j);
      if (lane == 0 || lane == 63) {
        const int32_t row = clampr(lane == 0 ? e - 1 : e + 64);
        r.p = po[row];
        if constexpr (P3) {
          const int64_t sj = oline(j) * SS + col;
          const int64_t c = lane == 0 ? (sj >= 1 ? 2 * (sj - 1) + 1 : 0) : (sj + 1 < nsl ? 2 * (sj + 1) : 2 * nsl - 1);
          r.r = reo[c];
          r.a = eao[c];
        } else {
          r.r = ro[row];
          r.a = apo[row];
        }
      }
    };
    auto load_far = [&](int32_t j, Far& f) {
      if (odn || oup) {
        const int32_t row = clampr(ebase(j) + lane + fo);
        f.r = ro[row];
        f.p = po[row];
        f.a = apo[row];
      }
    };
    auto load_xp = [&](int32_t j, XP& r) {
      if constexpr (PAIR) {
        const int32_t mm = j < n_run - 1 ? j : n_run - 1;
        if constexpr (!P3) r.pkm2 = ld_once(pn + e0 + mm * LO + lane, ntl);  // P3: already read (o_pm2)
        r.xo = ld_once(x + i0 + mm * LO + lane, ntl);
      }
    };
    auto load_codes = [&](int32_t j, Co& c) {
      if constexpr (VC) {  // diav: the row's own values, south / west / down from the partners
        const int64_t f = (oline(j) * SS + col) * 64 + lane + LO;
        c.k[0] = S.cvt[f - LO];
        c.k[1] = S.cvs[f - LN];
        c.k[2] = S.cve[f - 1];
        c.k[3] = S.cvd[f];
        c.k[4] = S.cve[f];
        c.k[5] = S.cvs[f];
        c.k[6] = S.cvt[f];
      } else {
        ar_load_dia<U>(S.dia4 + (oline(j) * SS + col) * (32 * U), lane, c);
      }
    };
    auto ghost = [&](int32_t j) { return gfull && (l0 + j == -1 || l0 + j == nl) && j >= jmin && j <= jmax; };
    // ghost plane's r_{k-1}: P3 recovers it from the halo's p's (k_cg_carry_ar's rghost)
    auto rghost = [&](int32_t j, const Raw& q) { return P3 && !first ? fma(nbp, pn[ebase(j) + lane], q.p) : q.r; };
    auto edge_pk = [&](const Edge& e) { return pk_of(e.r, e.a, e.p); };

    __syncthreads();  // the previous job's last step has read its LDS slots
    // prologue: planes -2 .. QD, edges / codes of -1 .. 1, the outside rows of -1 .. 1
    Raw rm2, rm1, r0, rq[QD];
    load_raw(-2, rm2);
    load_raw(-1, rm1);
    load_raw(0, r0);
#pragma unroll
    for (int d = 0; d < QD; ++d) load_raw(1 + d, rq[d]);
    Edge edm1{0.0, 0.0, 0.0}, ed0{0.0, 0.0, 0.0}, ed1{0.0, 0.0, 0.0};
    load_edge(-1, edm1);
    load_edge(0, ed0);
    load_edge(1, ed1);
    Co cm1, c0, c1;
    load_codes(-1, cm1);
    load_codes(0, c0);
    load_codes(1, c1);
    Far fm1{0.0, 0.0, 0.0}, f0{0.0, 0.0, 0.0}, fa{0.0, 0.0, 0.0};
    load_far(-1, fm1);
    load_far(0, f0);
    load_far(1, fa);
    XP x0{0.0, 0.0};
    load_xp(0, x0);
    // p_{k-1} of planes -1 and 0 for the +-N neighbours of the prologue's recomputations
    s_x[1][0][wv][lane] = rm1.p;
    s_x[1][1][wv][lane] = r0.p;
    __syncthreads();
    double pr_pk = 0.0;
    if (owned(-1)) {
      double dn, up;
      nbr(1, 0, fm1.p, dn, up);
      const double t = stencil(cm1, rm1.p, edm1.p, rm2.p, r0.p, dn, up);
      pr_pk = fma(b, rm1.p, fma(na, t, rof(-1, rm1)));
    } else if (ghost(-1)) {
      pr_pk = pk_of(rghost(-1, rm1), apo[ebase(-1) + lane], rm1.p);
    }
    double o_pold = r0.p, o_pm2 = r0.r, o_rk, o_pk;
    {
      double dn, up;
      nbr(1, 1, f0.p, dn, up);
      const double t = stencil(c0, r0.p, ed0.p, rm1.p, rq[0].p, dn, up);
      o_rk = fma(na, t, rof(0, r0));
      o_pk = fma(b, r0.p, o_rk);
    }
    double o_epk = edge_pk(ed0);
    double o_fpk = pk_of(f0.r, f0.a, f0.p);  // p_k of the outside row, plane 0
    for (int32_t m = 0; m < n_run; ++m) {
      const int par = m & 1;
      if constexpr (P3) {  // r_k of plane m where another wave or rank reads it (stored early: short live range)
        const int32_t eb = e0 + m * LO;
        if (m == 0 || m == n_run - 1) st_stream(&(rn + eb)[lane], fma(-b, o_pold, o_pk));
        else if (odn || oup) rn[eb + lane] = fma(-b, o_pold, o_pk);  // edge rows: compact (below)
      }
      // 1. loads for later steps: codes / edges of plane m + 2, the outside row of m + 2, x / p_{k-2}
      //    of m + 1, operands of m + 1 + QD
      Co c2;
      load_codes(m + 2, c2);
      // P3: the edge and outside rows of plane m + 2 are loaded at the end of the step instead
      // (one set live instead of two: the three-term kernel is at the 128-VGPR limit)
      Edge ed2{0.0, 0.0, 0.0};
      Far fb{0.0, 0.0, 0.0};
      if constexpr (!P3) {
        load_edge(m + 2, ed2);
        load_far(m + 2, fb);
      }
      XP x1{0.0, 0.0};
      if constexpr (!P3) load_xp(m + 1, x1);  // P3: at the end of the step (below)
      Raw rnq;
      load_raw(m + 1 + QD, rnq);
      // 2. exchange: p_{k-1} of plane m + 1 and p_k of plane m with the neighbouring waves
      s_x[par][0][wv][lane] = rq[0].p;
      s_x[par][1][wv][lane] = o_pk;
      __syncthreads();
      // 3. r_k, p_k of plane m + 1: Ap_{k-1} recomputed (owned) or exchanged (ghost plane)
      double rk1 = 0.0, pk1 = 0.0;
      if (owned(m + 1)) {
        double dn, up;
        nbr(par, 0, fa.p, dn, up);
        const double t = stencil(c1, rq[0].p, ed1.p, o_pold, rq[1].p, dn, up);
        rk1 = fma(na, t, rof(m + 1, rq[0]));
        pk1 = fma(b, rq[0].p, rk1);
      } else if (ghost(m + 1)) {
        const double t = apo[ebase(m + 1) + lane];
        rk1 = fma(na, t, rghost(m + 1, rq[0]));
        pk1 = fma(b, rq[0].p, rk1);
      }
      // 4. Ap_k of plane m, stores, partials
      double kdn, kup;
      nbr(par, 1, o_fpk, kdn, kup);
      const double sum = stencil(c0, o_pk, o_epk, pr_pk, pk1, kdn, kup);
      const int32_t eb = e0 + m * LO;
      if constexpr (!P3) st_stream(&(rn + eb)[lane], o_rk);  // P3: stored at the step's start
      if constexpr (PAIR) st_stream(&(x + i0 + m * LO)[lane], fma(a, o_pold, fma(ap, P3 ? o_pm2 : x0.pkm2, x0.xo)));
      st_stream(&(pn + eb)[lane], o_pk);
      const bool edge_lane = lane == 0 || lane == 63;
      if (odn || oup || (!P3 && edge_lane) || (gfull && (l0 + m == 0 || l0 + m == nl - 1))) apw[eb + lane] = sum;
      if (edge_lane && (P3 || ean != nullptr)) {  // compact edge rows (P3, and pass 0 of a P3 run)
        const int64_t c = 2 * ((l0 + m) * SS + col) + (lane == 63 ? 1 : 0);
        ean[c] = sum;
        ren[c] = P3 ? fma(-b, o_pold, o_pk) : o_rk;
      }
      s_pap = fma(o_pk, sum, s_pap);
      s_rap = fma(o_rk, sum, s_rap);
      s_apap = fma(sum, sum, s_apap);
      s_rr = fma(o_rk, o_rk, s_rr);
      // 5. rotate
      pr_pk = o_pk;
      o_pk = pk1;
      o_rk = rk1;
      o_pold = rq[0].p;
      o_pm2 = rq[0].r;
      o_epk = edge_pk(ed1);
      o_fpk = pk_of(fa.r, fa.a, fa.p);
      if constexpr (P3) {
        load_edge(m + 2, ed1);
        load_far(m + 2, fa);
        load_xp(m + 1, x0);
      } else {
        fa = fb;
        ed1 = ed2;
      }
#pragma unroll
      for (int d = 0; d + 1 < QD; ++d) rq[d] = rq[d + 1];
      rq[QD - 1] = rnq;
      if constexpr (!P3) x0 = x1;
      c0 = c1;
      c1 = c2;
    }
    }  // !LEAN
  }
  ar3_finish<KW>(s_pap, s_rap, s_apap, s_rr, partials, pstride, rc, st, tol);
}

}  // namespace

void cg_carry_ar3(int depth, int kw, const SellDev& S, const F1Vectors& v, int64_t own_off, const TileRanges& tr,
                  int32_t ln, bool gfull, double* partials, int pstride, int grid, CgState* st, double tol,
                  int first, int check, int k, int final_mode, hipStream_t stream, const RedCtl& rc, bool p3,
                  bool lean) {
  if (tr.ntiles == 0 || grid == 0) return;
  MCG_CHECK(tr.strip > 0 && tr.nt0 == tr.ntiles && tr.nt0 % tr.strip == 0 && tr.b0 == 0 && ln % 64 == 0 &&
                (int64_t)ln * ln == (int64_t)tr.strip * 64 && kw == (S.cvt != nullptr ? 8 : 16) && ln % kw == 0,
            "3-D Ap-recomputing carry: one launch over the rank's whole planes, N a multiple of 64, blocks of 16 waves (diav: 8)");
  const bool vc = S.cvt != nullptr;  // SELL-64/diav 3-D
  MCG_CHECK(vc || (S.dia4 != nullptr && S.dvals != nullptr), "3-D Ap-recomputing carry: dia4 codes missing");
  MCG_CHECK(!vc || (S.cvd && S.cve && S.cvs && v.ext_len < ((int64_t)1 << 29) &&
                    (tr.nt0 * 64 + tr.strip * 64) < ((int64_t)1 << 29)),
            "3-D diav carry: 8 waves per block, ranks below 2^29 rows");
  MCG_CHECK(v.ap_old != nullptr && v.ap_new != nullptr && v.r_old && v.p_old && v.r_new && v.p_new,
            "3-D Ap-recomputing carry: vectors missing");
  MCG_CHECK(rc.ngroups == 0 || (!final_mode && rc.base % kRedGroup == 0 && rc.cnt && rc.lvl2),
            "in-kernel reduction: bad control block");
  if (final_mode) {
    if (vc)
      hipLaunchKernelGGL((k_ar_final<6, 7>), dim3(grid), dim3(kBS), 0, stream, S, v, own_off, tr.nt0 * 64,
                         (int32_t)(tr.strip * 64), ln, partials, pstride, st, tol, first, check, k, p3);
    else
      hipLaunchKernelGGL((k_ar_final<4, 7>), dim3(grid), dim3(kBS), 0, stream, S, v, own_off, tr.nt0 * 64,
                         (int32_t)(tr.strip * 64), ln, partials, pstride, st, tol, first, check, k, p3);
    MCG_HIP(hipGetLastError(), "compute axpy failed(r)");
    return;
  }
  const bool pair = (k & 1) != 0;
  const int qd = depth >= 3 ? 3 : 2;
  const int g = gfull ? 1 : 0;
  MCG_CHECK(v.p_m2 == nullptr || (lean && p3), "3-D three p buffers: lean kernels");
  if (vc) {
#define MCG_A3V(PAIR, KW, P3, LEAN, ...)                                                                       \
  hipLaunchKernelGGL((k_cg_carry_ar3<2, PAIR, KW, P3, LEAN, false, true, ##__VA_ARGS__>), dim3(grid), dim3(64 * KW), 0, \
                     stream, S, v, own_off, tr, ln, g, partials, pstride, st, tol, first, check, rc)
#define MCG_A3VK(PAIR, P3, LEAN, ...) MCG_A3V(PAIR, 8, P3, LEAN, ##__VA_ARGS__)
#define MCG_A3VP(PAIR)                                          \
  do {                                                          \
    if (p3 && !first && lean && v.p_m2) MCG_A3VK(PAIR, true, true, true); \
    else if (p3 && !first && lean) MCG_A3VK(PAIR, true, true);  \
    else if (p3 && !first) MCG_A3VK(PAIR, true, false);         \
    else MCG_A3VK(PAIR, false, false);                          \
  } while (0)
    if (pair) MCG_A3VP(true);
    else MCG_A3VP(false);
#undef MCG_A3VP
#undef MCG_A3VK
#undef MCG_A3V
    MCG_HIP(hipGetLastError(), "compute mv failed(Ap)");
    return;
  }
  const bool big = v.ext_len >= ((int64_t)1 << 29);  // lean kernels: per-run bases
  const bool t3 = v.p_m2 != nullptr;                  // three p buffers (kernel comment)
  MCG_CHECK(!t3 || (lean && S.dpat != nullptr), "3-D three p buffers: lean dia4 kernels");
#define MCG_A3(QD, PAIR, KW, P3, ...)                                                                         \
  hipLaunchKernelGGL((k_cg_carry_ar3<QD, PAIR, KW, P3, ##__VA_ARGS__>), dim3(grid), dim3(64 * KW), 0, stream, S, v, \
                     own_off, tr, ln, g, partials, pstride, st, tol, first, check, rc)
#define MCG_A3P(QD, PAIR, KW)                                         \
  do {                                                                \
    if (p3 && !first && lean && S.dpat != nullptr && big && t3) MCG_A3(QD, PAIR, KW, true, true, true, false, true); \
    else if (p3 && !first && lean && S.dpat != nullptr && big) MCG_A3(QD, PAIR, KW, true, true, true); \
    else if (p3 && !first && lean && S.dpat != nullptr && t3) MCG_A3(QD, PAIR, KW, true, true, false, false, true); \
    else if (p3 && !first && lean && S.dpat != nullptr) MCG_A3(QD, PAIR, KW, true, true); \
    else if (p3 && !first) MCG_A3(QD, PAIR, KW, true);                \
    else MCG_A3(QD, PAIR, KW, false);                                 \
  } while (0)
#define MCG_A3K(QD, PAIR) MCG_A3P(QD, PAIR, 16)
  if (qd == 2) { if (pair) MCG_A3K(2, true); else MCG_A3K(2, false); }
  else { if (pair) MCG_A3K(3, true); else MCG_A3K(3, false); }
#undef MCG_A3K
#undef MCG_A3P
#undef MCG_A3
  MCG_HIP(hipGetLastError(), "compute mv failed(Ap)");
}

}  // namespace kern
}  // namespace mcg
