// Line-carry single-reduction pass that does not store Ap ("Ap recomputed").
//
// The line-carry pass (cg_fused1.hip, k_cg_f1_carry) stores {r_k, Ap_k} as 16-B pairs because
// pass k+1 forms r_{k+1} = r_k - a_k Ap_k for every row it touches (its own and, through p_{k+1}
// of the neighbours, the stencil's), and a_k is only known after pass k's global reduction.
// Per row and iteration that is 16 B read + 16 B written for {r, Ap} next to 8 + 8 B for p.
//
// Here Ap_{k-1} is not stored: pass k recomputes it as A p_{k-1} from the p_{k-1} it reads
// anyway.  The recomputation has the producing pass's exact fma order over the same entries and
// the same p_{k-1} values (which are the values the owners stored), so r_k, p_k, Ap_k and the
// dot products are bit for bit those of the storing pass.  A wave walking down a column of
// slices needs p_k of line m+1 for Ap_k(m); p_k(m+1) needs Ap_{k-1}(m+1), i.e. p_{k-1} of lines
// m .. m+2: the carried window is one line deeper, and each row's r and p are read once and
// written once (32 B/row instead of 48 B; the matrix codes once, carried from the recomputation
// into the row sums one step later).
//
// Two places cannot recompute:
//  * the rows just across a slice edge (the +-1 neighbours of lanes 0 / 63), which belong to
//    the neighbouring column's wave: their Ap_{k-1} comes from a compact per-slice array of the
//    two edge rows' Ap (ape: 2 doubles per 64-row slice, 1/4 B per row written);
//  * the ghost lines of a multi-rank run, whose matrix rows another rank owns: each rank stores
//    the full Ap of its first and last line (apx, ext layout) and the halo carries {r, Ap, p}
//    of those lines as before.
// 2-D stencils with only 0, +-1, +-one-line offsets (the specialised carry: SELL-64/c8 or /c4
// dictionary codes).  Final mode (finalize(): r_m, x_m, ||r_m||^2) is a plain row-parallel
// kernel with the same recomputation (k_ar_final, carry_common.hpp).  The 3-D plane carry is
// cg_carry_ar3.hip, the formats and setup checks carry_formats.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
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

// LEAN > 0: lean-only kernel (every run checked at setup) for at least LEAN waves per SIMD
// BIG (lean kernels): the rank's vectors exceed 2^29 doubles, so each run re-bases its global pointers
// (64-bit, scalar registers) at its own first lines and keeps 32-bit byte offsets inside the run
// EP (lean dia4 kernels): packed edges -- the three values a slice-edge lane needs per line (its
// neighbour row's r_{k-1}, Ap_{k-1}, p_{k-1}) arrive in ONE load per line, lanes 0 / 15 / 7 fetching
// lane 0's and lanes 63 / 48 / 56 lane 63's, and move to lanes 0 / 63 by row_mirror /
// row_half_mirror DPP (one move serves both ends).  A line in flight then holds 2 instead of 6
// VGPRs of edges, which buys a wave per SIMD (LEAN 5) or a line of prefetch depth
// T3 (lean dia4 / diav kernels, F1Vectors::p_m2): three p buffers -- p_k goes to a buffer this pass does not
// read, so p_{k-2} stays intact all pass.  r is recovered from p_{k-1}, p_{k-2} on every line (no
// stored r at run ends), and the neighbouring slices' edge rows are recomputed from their p_{k-1},
// p_{k-2} (the owner's stencil in the owner's fma order: the same bits it stored) instead of read from
// compact edge arrays: no edge-array loads or stores at all (bench/carry_depth.hip: the pattern with
// the edge stores 77 us at 4096^2, with neighbour-row loads instead 58; profiles/r5/depth).  The diav
// loop (CM 5) recovers r the same way but still stores and reads its edge rows' Ap (per-row values)
#if defined(MCG_CARRY_DIAG)
// diagnostic build (profiles/r6/waves): per wave of one launch -- entry, end of its jobs, end of the
// reduction (wall clock, 100 MHz) and where it ran (XCC_ID << 32 | HW_ID)
constexpr int kCarryDiagMax = 8192;
__device__ unsigned long long g_carry_diag[4 * kCarryDiagMax];
#endif

// COMBO (the T3 lean kernels of a split rank's lean launch): the lean stretches of every run
// (TileRanges::sub_ranges), and with gen_blocks > 0 the first gen_blocks workgroups run the generic step over
// the listed ranges -- one launch, no side stream
template <int CM, int U, int QD, bool PAIR, bool P3, int UN = 1, int LEAN = 0, bool BIG = false, bool EP = false,
          bool T3 = false, bool COMBO = false>
__global__ __launch_bounds__(kBS, (LEAN > 0 ? LEAN : 4)) void k_cg_carry_ar(SellDev S, F1Vectors v, int64_t own, TileRanges tr,
                                                     double* __restrict__ partials, int pstride, CgState* st,
                                                     double tol, int first, int check, RedCtl rc) {
  __shared__ double2 s_dict[CM >= 4 ? 1 : 256];
  __shared__ double s_val[16];  // dia4 values
#if defined(MCG_CARRY_DIAG)
  const unsigned long long t_in = wall_clock64();
#endif
  const F1Scalars sc = f1_scalars(st, tol, first, check);
  if (st->done || sc.conv) {
    f1_finish(0.0, 0.0, 0.0, 0.0, partials, pstride, rc, st, tol);
    return;
  }
  if constexpr (CM == 4) {
    if (threadIdx.x < 16) s_val[threadIdx.x] = S.dvals[threadIdx.x];
  } else if constexpr (CM != 5) {
    for (int q = threadIdx.x; q < S.ndict; q += kBS) s_dict[q] = S.dict[q];
  }
  __syncthreads();
  const double a = sc.alpha, b = sc.beta, na = -a, ap = st->a_prev;
  // three-term form (P3): r_{k-1} = p_{k-1} - b_prev p_{k-2} from the two p's the pass reads anyway
  // (p_{k-2} is the buffer p_k overwrites), so r is stored only where another wave or rank reads
  // it: the slices' edge rows and every row of a run's first / last line (which include the
  // rank's first / last line, the halo's source).  Pass 0 (r_{-1} = b in the full vector) runs the
  // two-term kernel: with beta = 0 its r_0 equals the recovered value bit for bit
  constexpr bool rfull = !P3;
  const double nbp = P3 ? -st->b_prev : 0.0;
  const double* __restrict__ ro = v.r_old;
  const double* __restrict__ po = v.p_old;
  double* __restrict__ rn = v.r_new;
  double* __restrict__ pn = v.p_new;
  double* __restrict__ x = v.x;
  const double* __restrict__ apx_o = v.ap_old;  // multi-rank: ghost lines' Ap_{k-1}
  double* __restrict__ apx_n = v.ap_new;        // multi-rank: first / last line's Ap_k for the neighbours
  double* __restrict__ en = v.ape_new;
  const double* __restrict__ reo = v.re_old;  // P3: edge rows' r_{k-1}
  double* __restrict__ ren = v.re_new;        // edge rows' r_k (P3; and pass 0 of a P3 run, two-term kernel)
  const int lane = threadIdx.x & 63;
  const int64_t SS = tr.strip;            // slices per line
  const int32_t LO = (int32_t)(SS * 64);  // one line
  const int64_t nl = tr.nt0 / SS;         // the rank's lines (the launch covers them all)
  const int64_t nsl = tr.nt0;             // the rank's slices
  // COMBO: workgroups [0, gen_blocks) take the listed generic ranges (gen_blocks a multiple of 8, so the
  // lean workgroups keep their XCDs), the others the lean launch's jobs
  const int64_t gb = COMBO ? (int64_t)tr.gen_blocks : 0;
  const bool gblk = COMBO && (int64_t)blockIdx.x < gb;
  const int64_t nb = gblk ? gb : gridDim.x - gb, blk = gblk ? blockIdx.x : blockIdx.x - gb;
  const int64_t lb = (nb % 8 == 0) ? (blk % 8) * (nb / 8) + blk / 8 : blk;  // XCD-aware (k_cg_f1_carry)
  const int64_t nw = nb * kWaves;
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  int64_t gw = lb * kWaves + wv;
#if defined(MCG_COLMAP_SPREAD)
  // diagnostic build (profiles/r6/colmap): a block's waves take columns SS / kWaves apart, so every slice
  // edge lies between two blocks (the default: a block's waves take kWaves adjacent columns)
  if (SS % kWaves == 0 && gw < (nw / SS) * SS) {
    const int64_t w = gw % SS, q = w / kWaves, u = w % kWaves;
    gw = gw - w + u * (SS / kWaves) + q;
  }
#endif
  int64_t runs, chunk;
  const int64_t njobs = carry_jobs(nw, SS, nl, runs, chunk);
  const int32_t ext32 = (int32_t)v.ext_len;
  constexpr bool ntl = false;  // plain loads (non-temporal measured slower: 281 vs 302 it/s 2-D)
  const double* __restrict__ eo = v.ape_old;
  const uint32_t* __restrict__ meta = S.smeta;
  // a zero the compiler cannot see through: wave-uniform metadata loads stay vector loads (vmcnt,
  // in order with the prefetches) instead of scalar loads, whose out-of-order lgkmcnt wait would
  // also wait for every LDS dictionary read of the step
  int vz;
  asm volatile("v_mov_b32 %0, 0" : "=v"(vz));
  double s_pap = 0.0, s_rap = 0.0, s_apap = 0.0, s_rr = 0.0;

  // r = r_{k-1}, or (P3, a line of this run) p_{k-2}: see rof()
  struct Raw {
    double r, p;
  };
  // the row just before (lane 0) / after (lane 63) the slice on a line: r, Ap (the neighbouring
  // slice's edge row, ape), p -- loaded by those two lanes only; other lanes' values are unused
  struct Edge {
    double r, a, p;
    uint32_t c;  // T3, generic step: the neighbouring edge row's dia4 codes
  };
  struct XP {
    double pkm2, xo;
  };
  // row sum over a slice's entries: p of the row, of row +-1 (neighbouring lanes; lanes 0 / 63
  // take `edge`), of the next / previous line.  Same select chain and fma order as the storing pass.
  auto stencil = [&](const ArCodes<CM, U>& c, double mid, double edge, double dnl, double upl) {
    const double sh_up = lane_up(mid);
    const double sh_dn = lane_dn(mid);
    const double upv = lane == 63 ? edge : sh_up;
    const double dnv = lane == 0 ? edge : sh_dn;
    double sum = 0.0;
    if constexpr (CM == 5) {  // the row's own coefficients, canonical column order
      const double g[5] = {dnl, dnv, mid, upv, upl};
#pragma unroll
      for (int u = 0; u < 5; ++u) sum = fma(c.k[u], g[u], sum);
      return sum;
    }
    else if constexpr (CM == 4) {  // slot u = the u-th canonical offset: ascending columns, no selects
      const double g[5] = {dnl, dnv, mid, upv, upl};
#pragma unroll
      for (int u = 0; u < 5; ++u) sum = fma(s_val[(c.pk[0] >> (4 * u)) & 15u], g[u], sum);
      return sum;
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        double val;
        const int32_t off = ar_entry<CM, U>(s_dict, c, u, val);
        double t = off == LO ? upl : dnl;
        asm volatile("" : "+v"(t));
        t = off == -1 ? dnv : t;
        asm volatile("" : "+v"(t));
        t = off == 1 ? upv : t;
        asm volatile("" : "+v"(t));
        const double g = off == 0 ? mid : t;
        sum = (u < c.w) ? fma(val, g, sum) : sum;
      }
      return sum;
    }
  };
  // T3 generic launch of a split rank (TileRanges::gen_pieces / gen_list): the listed generic runs of the lean
  // launch's decomposition, each in K pieces on K waves
  // a split rank on three p buffers (TileRanges::sub_ranges): the lean launch takes every lean stretch of its
  // runs (next_lean_range), the generic launch the listed ranges left between them (col, first, end line)
  // (compile-time false outside the split kernels: the lean-only kernels keep their register allocation)
  const bool listed = gblk || (LEAN == 0 && T3 && tr.lean_split == 2 && tr.sub_ranges != 0 && tr.gen_list != nullptr);
  const bool subr = COMBO && T3 && tr.lean_split == 1 && tr.sub_ranges != 0 && !gblk;
  for (int64_t job = gw; job < (listed ? (int64_t)tr.ngen : njobs); job += nw) {
    int64_t col, L0, L1;
    if (listed) {
      col = tr.gen_list[3 * job];
      L0 = tr.gen_list[3 * job + 1];
      L1 = tr.gen_list[3 * job + 2];
    } else {
      carry_run(job, SS, nl, chunk, col, L0, L1);
    }
    uint32_t sWA = 0u, sWB = 0u, sWC = 0u;
    for (int64_t from = L0, more = 1; more;) {
    int64_t l0 = L0, l1 = L1;
    if (subr) {
      if (!next_lean_range<true>(S.dpat, from, L1, nl, SS, col, v.ext_len, l0, l1, sWA, sWB, sWC)) break;
      from = l1;
    } else {
      more = 0;
    }
    if (l0 >= l1) continue;
    const int64_t sl0 = l0 * SS + col;
    const int32_t e0 = (int32_t)(own + sl0 * 64);
    const int32_t i0 = (int32_t)(sl0 * 64);
    const int32_t n_run = (int32_t)(l1 - l0);
    if constexpr (CM == 4 && P3) {
      // Lean run.  A run whose lines l0 - 1 .. l1 carry uniform value patterns in this slice column
      // (SellDev::dpat: every row the same value index per slot; one pattern B for the inner lines,
      // the grid's first / last line may have their own, A / C) runs the loop below instead of
      // step(): the values in scalar registers, no codes streamed or decoded, every access a
      // kernel-wide global base plus a 32-bit byte offset, the slice-edge select folded into the
      // lane shift.  It computes what step() computes, in the same fma order (bitwise equal): same
      // loads (p_{k-2} for lines of the run, the stored r_{k-1} beyond it, lines clamped to the
      // rank's), same stores (r in full on the run's first / last line, compact edge rows), same
      // partials.  A slice at the start / end of a grid line (lane 0 / 63 without its -1 / +1
      // entry: dpat bits 28 / 29) gives that lane the absent entry's value, +0.0, as its -1 / +1
      // coefficient: per-lane coefficients for those two slots (the same fma).  Every
      // stream is a chain of LD registers (operands LD lines ahead, edges LD, x LD - 1) that the
      // LD-step unroll rotates by renaming: no move of a register whose load is in flight.  Ghost
      // lines (P > 1) as in step(): their Ap_{k-1} exchanged (apx), r recovered from the halo's
      // p's; the rank's first / last line stores its Ap_k for the neighbours.
      // LEAN > 0 kernels only: the setup checked every run of the launch (carry_lean_failures), and
      // the kernel has no generic step at all (one kernel with both measured slower for each)
      constexpr int LD = QD + 1;
      uint32_t WA, WB, WC;
      // lean_split: both launches decide a run the same way (size mode 1 in both: it only differs from
      // mode 0 past 2^29 rows, where the lean launch runs the BIG kernels)
      // (T3 on a split rank: also the neighbouring columns' patterns, whose edge rows the lean run recomputes;
      // with sub-ranges the lean stretch is eligible by construction and a listed range is generic)
      const bool elig = subr ? true
                             : (listed ? false
                                       : lean_eligible<true>(S.dpat, L0, L1, nl, SS, col, v.ext_len, WA, WB, WC,
                                                             (BIG || tr.lean_split != 0) ? 1 : 0, COMBO && tr.lean_split != 0));
      if (subr) {
        WA = sWA;
        WB = sWB;
        WC = sWC;
      }
      if (tr.lean_split == 1 && !elig && !gblk) continue;  // the generic launch takes this run
      if (tr.lean_split == 2 && elig) continue;            // the lean launch took it
      if (LEAN > 0 && !gblk) {
        struct VSet {
          double v[5];
        };
        auto vals = [&](uint32_t P) {
          VSet V;
#pragma unroll
          for (int u = 0; u < 5; ++u) V.v[u] = uni_d(s_val[(P >> (4 * u)) & 15u]);
          return V;
        };
        const bool z0 = (WB >> 28) & 1u, z63 = (WB >> 29) & 1u;
        {
          const VSet VB = vals(WB);
          const bool hi = lane == 63, edge_lane = lane == 0 || lane == 63;
          const bool zlo = lane == 0 && z0, zhi = hi && z63;  // lanes whose -1 / +1 entry is absent
          const uint32_t l8 = (uint32_t)lane << 3;
          const uint32_t LOB = (uint32_t)LO << 3;                         // one line of the vectors
          const uint32_t SB = (uint32_t)(2 * SS) << 3;                    // one line of the edge arrays
          // BIG: byte offsets from per-run bases (ext index e0 - 3 lines, x index i0)
          const int64_t rb = BIG ? (int64_t)e0 - 3 * (int64_t)LO : 0;
          const int64_t xr = BIG ? (int64_t)i0 : 0;
          const double* __restrict__ po_ = po + rb;
          const double* __restrict__ ro_ = ro + rb;
          double* __restrict__ pn_ = pn + rb;
          double* __restrict__ rn_ = rn + rb;
          double* __restrict__ x_ = x + xr;
          const double* __restrict__ pm2_ = (T3 ? v.p_m2 : (const double*)pn) + rb;  // T3: p_{k-2}, read-only
          const double* __restrict__ apo_ = apx_o + rb;
          double* __restrict__ apn_ = apx_n + rb;
          PullBases pl;  // in-kernel halo: the ghost lines from the neighbours' rows
          pl.at(v, rb);
          const uint32_t ob0 = BIG ? 3u * ((uint32_t)LO << 3) : (uint32_t)e0 << 3;  // line 0 (ext layout)
          const uint32_t xb0 = BIG ? 0u : (uint32_t)i0 << 3;                         // line 0 of x
          const uint32_t cb0 = (uint32_t)(2 * (l0 * SS + col) - 1) << 3;  // edge arrays: 2 s - 1 of line 0
          // lane 0: entry 2 s - 1 and row e - 1, lane 63: 2 s + 2 and row e + 64; a lane without
          // its edge entry reads its own slice's (in range at the rank's first / last slice)
          const uint32_t oc = hi ? (z63 ? 16u : 24u) : (z0 ? 8u : 0u);
          const uint32_t op = hi ? (z63 ? 512u : 520u) : (z0 ? 8u : 0u);
          // lines of the ext vectors (ghosts included; step()'s ebase) and of the rank (oline)
          const int32_t jlo = -(e0 / LO), jhi = (ext32 - 64 - e0) / LO;
          const int32_t rlo = -(int32_t)l0, rhi = (int32_t)(nl - 1 - l0);
          auto jc = [&](int32_t j) { return j < jlo ? jlo : (j > jhi ? jhi : j); };
          auto rc_ = [&](int32_t j) { return j < rlo ? rlo : (j > rhi ? rhi : j); };
          auto line_ofs = [&](int32_t j) { return ob0 + (uint32_t)j * LOB; };
          auto raw_at = [&](int32_t j) {
            Raw q;
            const int32_t jj = jc(j);
            const uint32_t o = line_ofs(jj) + l8;
            q.r = T3 ? g_ld(pm2_, o) : g_ld((j >= 0 && j < n_run) ? (const double*)pn_ : ro_, o);
            q.p = pl.ld_p(pl.side(l0 + jj, nl), po_, o);
            return q;
          };
          // a ghost line's Ap_{k-1}: the neighbour's stored first / last line
          auto ap_gh = [&](int32_t j) { return pl.ld_ap(pl.side(l0 + j, nl), apo_, line_ofs(j) + l8); };
          // EP: lane roles (kernel comment) -- r: lanes 0 / 63, Ap: 15 / 48, p: 7 / 56; the other lanes
          // repeat lane 0's r load (the same address: no extra traffic).  Per lane a 64-bit base (reo,
          // eo or po_) and the byte offset of line 0 plus a per-line stride (SB, or LOB for p)
          const int erole = !EP ? 0 : (lane == 15 || lane == 48) ? 1 : (lane == 7 || lane == 56) ? 2 : 0;
          const bool eright = lane >= 32;
          const bool erz = eright ? z63 : z0;
          const uint32_t eoc = eright ? (erz ? 16u : 24u) : (erz ? 8u : 0u);
          const uint32_t eop = eright ? (erz ? 512u : 520u) : (erz ? 8u : 0u);
          const bool erole_ok = erole != 0 || lane == 0 || lane == 63;
          const char* ebase = (const char*)(erole == 1 ? eo : erole == 2 ? po_ : reo);
          const uint32_t eoff0 = erole == 2 ? ob0 - 8u + eop : cb0 + (erole_ok ? eoc : oc);
          const uint32_t estr = erole == 2 ? LOB : SB;
          auto edge_pk_ld = [&](int32_t jr, int32_t jp) {  // jr: line of the edge arrays, jp: line of po
            const uint32_t o = eoff0 + (uint32_t)(erole == 2 ? jp : jr) * estr;
            return *(const g_double*)((const g_char*)(const g_double*)ebase + o);
          };
          // T3 edges: the neighbouring slice's edge row (nb: row -1 / 64) and the row beyond it (nb2: -2 /
          // 65) of line j -- per lane a byte offset from the line start and a base.  EP: lanes 0 / 63 p_{k-2}
          // (nb), 15 / 48 p_{k-1} (nb2), 7 / 56 p_{k-1} (nb) (the other lanes repeat lane 0's / 63's
          // load); otherwise every lane loads the three for its own -1 / +1 side.  A slice that starts /
          // ends a grid line reads its own row (the value meets a zero coefficient).
          const bool er3 = EP ? eright : hi;
          const bool erz3 = er3 ? z63 : z0;
          const int32_t eo_nb = er3 ? 504 + (erz3 ? 0 : 8) : (erz3 ? 0 : -8);
          const int32_t eo_nb2 = er3 ? 504 + (erz3 ? 0 : 16) : (erz3 ? 0 : -16);
          const int32_t eo_ep = erole == 1 ? eo_nb2 : eo_nb;
          const char* ebase3 = (const char*)(erole == 0 ? pm2_ : po_);
          auto t3_at = [&](int32_t j, int32_t off, const double* base, bool pulled_p) {
            const int32_t jj = jc(j);
            const uint32_t o = (uint32_t)((int32_t)line_ofs(jj) + off);
            return pulled_p ? pl.ld_p(pl.side(l0 + jj, nl), base, o) : g_ld(base, o);
          };
          auto edge3 = [&](int32_t j, bool un) {
            Edge q;
            if constexpr (EP) {
              const int32_t jj = un ? j : jc(j);
              const uint32_t o = (uint32_t)((int32_t)line_ofs(jj) + eo_ep);
              const int sd = un ? -1 : pl.side(l0 + jj, nl);
              if (sd >= 0 && erole != 0) q.r = pl.ld_p(sd, po_, o);  // a pulled ghost line's p_{k-1}
              else q.r = *(const g_double*)((const g_char*)(const g_double*)ebase3 + o);
              q.a = q.p = 0.0;
            } else {
              q.r = t3_at(un ? j : j, eo_nb - (hi ? 504 : 0) + (int32_t)l8, pm2_, false);
              q.a = t3_at(j, eo_nb2 - (hi ? 504 : 0) + (int32_t)l8, po_, true);
              q.p = t3_at(j, eo_nb - (hi ? 504 : 0) + (int32_t)l8, po_, true);
            }
            return q;
          };
          auto edge_at = [&](int32_t j) {
            Edge q;
            if constexpr (T3) return edge3(j, false);
            if constexpr (EP) {
              q.r = edge_pk_ld(rc_(j), jc(j));
              q.a = q.p = 0.0;
            } else {
              const uint32_t c = cb0 + (uint32_t)rc_(j) * SB + oc;
              q.r = g_ld(reo, c);
              q.a = g_ld(eo, c);
              q.p = g_ld(po_, line_ofs(jc(j)) - 8u + op);
            }
            return q;
          };
          // a ghost line's r_{k-1} (step()'s rghost): from the halo's p_{k-2} in p_new's ghost rows
          auto rghost = [&](int32_t j, const Raw& q) { return fma(nbp, g_ld(T3 ? pm2_ : (const double*)pn_, line_ofs(j) + l8), q.p); };
          auto is_ghost = [&](int32_t j) { return apx_o != nullptr && (l0 + j == -1 || l0 + j == nl) && j >= jlo && j <= jhi; };
          auto raw_un = [&](int32_t j) {  // a line of the run or below it, inside the rank
            Raw q;
            const uint32_t o = line_ofs(j) + l8;
            q.r = g_ld(T3 ? pm2_ : (j < n_run ? (const double*)pn_ : ro_), o);
            q.p = g_ld(po_, o);
            return q;
          };
          auto edge_un = [&](int32_t j) {
            Edge q;
            if constexpr (T3) return edge3(j, true);
            if constexpr (EP) {
              q.r = edge_pk_ld(j, j);
              q.a = q.p = 0.0;
            } else {
              const uint32_t c = cb0 + (uint32_t)j * SB + oc;
              q.r = g_ld(reo, c);
              q.a = g_ld(eo, c);
              q.p = g_ld(po_, line_ofs(j) - 8u + op);
            }
            return q;
          };
          auto x_at = [&](int32_t j) {
            if constexpr (PAIR) return g_ld(x_, xb0 + (uint32_t)(j < n_run - 1 ? j : n_run - 1) * LOB + l8);
            else return 0.0;
          };
          auto ez = [&](double e) { return e; };
          // an edge's p_{k-1} / p_k in lanes 0 and 63 (EP: gathered from the role lanes by DPP)
          auto e_p = [&](const Edge& q) {
            if constexpr (EP) {
              const double v = q.r;
              const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x141, 0xf, 0xf, false);  // row_half_mirror
              const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x141, 0xf, 0xf, false);
              return __hiloint2double(hi, lo);
            } else {
              return q.p;
            }
          };
          auto stencil_u = [&](const VSet& V, double mid, double edge, double dnl, double upl) {
            const double upv = lane_up_or(mid, edge);
            const double dnv = lane_dn_or(mid, edge);
            const double cm = zlo ? 0.0 : V.v[1], cp = zhi ? 0.0 : V.v[3];  // loop-invariant
            double sum = fma(V.v[0], dnl, 0.0);
            sum = fma(cm, dnv, sum);
            sum = fma(V.v[2], mid, sum);
            sum = fma(cp, upv, sum);
            return fma(V.v[4], upl, sum);
          };
          // a first / last line of the other parity's runs (TileRanges::alt_chunk): r stored there too
          const int32_t ach = tr.alt_chunk;
          auto alt_edge = [&](int32_t m) {
            if (ach <= 0) return false;
            const int32_t l = (int32_t)l0 + m, md = l % ach;
            return md == 0 || md == ach - 1 || l == (int32_t)nl - 1;
          };
          auto epk = [&](const Edge& q) {
            if constexpr (EP) {
              const double v = q.r;
              const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x140, 0xf, 0xf, false);  // row_mirror
              const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x140, 0xf, 0xf, false);
              return fma(b, e_p(q), fma(na, __hiloint2double(hi, lo), v));
            } else {
              return fma(b, q.p, fma(na, q.a, q.r));
            }
          };
          // T3: the neighbouring edge row's p_k, recomputed as its owner computed it (the owner's stencil
          // over its p_{k-1}: lines j - 1 / j + 1 (prev / next), its inner neighbour nb2, itself, and the
          // row across the slice edge -- this lane's own p_{k-1}, `own`; coefficients V of line j)
          auto epk3 = [&](double prev, const Edge& q, double next, double own, const VSet& V) {
            const double p1 = e_p(q);
            double p1b, p2;
            if constexpr (EP) {
              const double v = q.r;
              const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x140, 0xf, 0xf, false);  // row_mirror
              const int hi2 = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x140, 0xf, 0xf, false);
              p1b = __hiloint2double(hi2, lo);
              p2 = v;
            } else {
              p1b = q.a;
              p2 = q.r;
            }
            const double dnv = hi ? own : p1b, upv = hi ? p1b : own;
            double t = fma(V.v[0], prev, 0.0);
            t = fma(V.v[1], dnv, t);
            t = fma(V.v[2], p1, t);
            t = fma(V.v[3], upv, t);
            t = fma(V.v[4], next, t);
            return fma(b, p1, fma(na, t, fma(nbp, p2, p1)));
          };
          // prologue (step()'s): lines -2 .. LD - 1
          const Raw rm2 = raw_at(-2), rm1 = raw_at(-1), r0 = raw_at(0);
          Raw q[LD - 1];  // lines m + 1 .. m + LD - 1
#pragma unroll
          for (int d = 0; d < LD - 1; ++d) q[d] = raw_at(1 + d);
          const Edge edm1 = edge_at(-1), ed0 = edge_at(0);
          Edge e[LD - 1];  // lines m + 1 .. m + LD - 1
#pragma unroll
          for (int d = 0; d < LD - 1; ++d) e[d] = edge_at(1 + d);
          // x chain: lines m .. m + XD - 1 (EP: one line shorter, 2 VGPRs for the 5-wave kernels)
          constexpr int XD = EP ? LD - 2 : LD - 1;
          double xs[XD];
#pragma unroll
          for (int d = 0; d < XD; ++d) xs[d] = x_at(d);
          double pr_pk = 0.0;  // p_k of line -1: owned, a ghost, or none
          if (l0 >= 1) {
            const VSet Vm = l0 == 1 ? vals(WA) : VB;
            pr_pk = fma(b, rm1.p, fma(na, stencil_u(Vm, rm1.p, ez(e_p(edm1)), rm2.p, r0.p), T3 ? fma(nbp, rm1.r, rm1.p) : rm1.r));
          } else if (is_ghost(-1)) {
            pr_pk = fma(b, rm1.p, fma(na, ap_gh(-1), rghost(-1, rm1)));
            // pulled: this p_{k-1} is the next pass's p_{k-2} of the ghost line (rghost)
            if (pl.p[0] != nullptr) g_st(const_cast<double*>(po_), line_ofs(-1) + l8, rm1.p);
          }
          double o_pold = r0.p, o_pm2 = r0.r, o_rk, o_pk;
          {
            const VSet V0 = l0 == 0 ? vals(WA) : VB;
            o_rk = fma(na, stencil_u(V0, r0.p, ez(e_p(ed0)), rm1.p, q[0].p), fma(nbp, r0.r, r0.p));
            o_pk = fma(b, r0.p, o_rk);
          }
          double o_epk, ep_prev = 0.0;  // T3: p_{k-1} of the neighbouring edge row, line m (carried)
          if constexpr (T3) {
            const VSet V0 = l0 == 0 ? vals(WA) : VB;
            o_epk = epk3(e_p(edm1), ed0, e_p(e[0]), r0.p, V0);
            ep_prev = e_p(ed0);
          } else {
            o_epk = epk(ed0);
          }
          // step m: Ap_{k-1} of line m + 1 (next: 1 owned, values Vt; 2 a ghost line; 0 none) and
          // Ap_k of line m (values Vs)
          auto lstep = [&](auto clc, int32_t m, const VSet& Vs, const VSet& Vt, int next) __attribute__((always_inline)) {
            // CL: loads that may reach past the rank's last line (clamped); the main loop's never do
            constexpr bool CL = decltype(clc)::value;
            const Raw qn = CL ? raw_at(m + LD) : raw_un(m + LD);
            const Edge en2 = CL ? edge_at(m + LD) : edge_un(m + LD);
            const double xn = x_at(m + XD);
            double rk1 = 0.0, pk1 = 0.0;
            if (next == 1) {
              const double t = stencil_u(Vt, q[0].p, ez(e_p(e[0])), o_pold, q[1].p);
              rk1 = fma(na, t, (T3 || m + 1 < n_run) ? fma(nbp, q[0].r, q[0].p) : q[0].r);
              pk1 = fma(b, q[0].p, rk1);
            } else if (CL && next == 2) {
              rk1 = fma(na, ap_gh(m + 1), rghost(m + 1, q[0]));
              pk1 = fma(b, q[0].p, rk1);
              if (pl.p[1] != nullptr) g_st(const_cast<double*>(po_), line_ofs(m + 1) + l8, q[0].p);
            }
            const double sum = stencil_u(Vs, o_pk, o_epk, pr_pk, pk1);
            const uint32_t ob = line_ofs(m);
            const double rr = fma(-b, o_pold, o_pk);
            if constexpr (!T3) {  // T3: nobody reads a stored r or edge row
              if (m == 0 || m == n_run - 1 || alt_edge(m)) g_st_nt(rn_, ob + l8, rr);
              if (edge_lane) {
                const uint32_t sb = cb0 + (uint32_t)m * SB + (hi ? 16u : 8u);  // 2 s, 2 s + 1
                g_st(ren, sb, rr);
                g_st(en, sb, sum);
              }
            }
            if constexpr (PAIR) g_st_nt(x_, xb0 + (uint32_t)m * LOB + l8, fma(a, o_pold, fma(ap, o_pm2, xs[0])));
            const bool bnd = l0 + m == 0 || l0 + m == nl - 1;  // the halo's source lines
            if constexpr (CL) pl.st_pub(bnd, pn_, ob + l8, o_pk, true);
            else g_st_nt(pn_, ob + l8, o_pk);
            if (CL && apx_n != nullptr && bnd) pl.st_pub(true, apn_, ob + l8, sum, false);
            s_pap = fma(o_pk, sum, s_pap);
            s_rap = fma(o_rk, sum, s_rap);
            s_apap = fma(sum, sum, s_apap);
            s_rr = fma(o_rk, o_rk, s_rr);
            pr_pk = o_pk;
            o_pk = pk1;
            o_rk = rk1;
            o_pold = q[0].p;
            o_pm2 = q[0].r;
            if constexpr (T3) {
              if (next == 1) {
                const double ep0 = e_p(e[0]);
                o_epk = epk3(ep_prev, e[0], e_p(e[1]), q[0].p, Vt);
                ep_prev = ep0;
              }
            } else {
              o_epk = epk(e[0]);
            }
#pragma unroll
            for (int d = 0; d + 1 < LD - 1; ++d) {
              q[d] = q[d + 1];
              e[d] = e[d + 1];
            }
#pragma unroll
            for (int d = 0; d + 1 < XD; ++d) xs[d] = xs[d + 1];
            q[LD - 2] = qn;
            e[LD - 2] = en2;
            xs[XD - 1] = xn;
          };
          // main loop: steps whose lines m, m + 1 are inner lines and whose loads (line m + LD) stay
          // inside the rank, [m_lo, m_hi]; then the clamped tail
          const std::true_type clamped;
          const std::false_type unclamped;
          const int32_t m_lo = l0 == 0 ? 1 : 0;
          const int32_t m_hi = min(n_run - 1, (int32_t)(nl - 1 - LD - l0));
          int32_t m = 0;
          if (m_lo == 1) lstep(clamped, 0, vals(WA), VB, 1);
          m = m_lo;
          for (; m + LD - 1 <= m_hi; m += LD) {
#pragma unroll
            for (int u = 0; u < LD; ++u) lstep(unclamped, m + u, VB, VB, 1);
          }
          for (; m <= m_hi; ++m) lstep(unclamped, m, VB, VB, 1);
          if (m < n_run) {  // near the rank's last line: clamped loads, its values C
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
    if constexpr (CM == 5 && P3 && LEAN > 0) {
      // Lean run with variable coefficients (SELL-64/diav): the CM == 4 lean loop above with the
      // five values of a line streamed instead of held in scalar registers.  Per line the row's own
      // d, e, s and the east value of the row before the slice (lane 0's west coefficient) are
      // loaded LD lines ahead with the operands; the west column is e shifted one lane (DPP), the
      // north column the previous line's s (carried).  Every run of >= 3 lines qualifies (the setup
      // checks the launch's runs); same sums in the same fma order as step() with CM == 5.
      constexpr int LD = QD + 1;
      struct VSet {
        double v[5];
      };
      struct CRaw {
        double d, e, s, ee;
      };
      const bool z0 = col == 0, z63 = col == SS - 1;  // slices at a grid line's start / end
      const bool hi = lane == 63, edge_lane = lane == 0 || lane == 63;
      const uint32_t l8 = (uint32_t)lane << 3;
      const uint32_t LOB = (uint32_t)LO << 3;
      const uint32_t SB = (uint32_t)(2 * SS) << 3;
      const int64_t rb = BIG ? (int64_t)e0 - 3 * (int64_t)LO : 0;  // BIG: per-run bases (see the CM == 4 loop)
      const int64_t xr = BIG ? (int64_t)i0 : 0;
      const double* __restrict__ po_ = po + rb;
      const double* __restrict__ ro_ = ro + rb;
      double* __restrict__ pn_ = pn + rb;
      double* __restrict__ rn_ = rn + rb;
      double* __restrict__ x_ = x + xr;
      const double* __restrict__ apo_ = apx_o + rb;
      double* __restrict__ apn_ = apx_n + rb;
      PullBases pl;  // in-kernel halo (the dia4 lean loop's)
      pl.at(v, rb);
      // T3 (three p buffers, not BIG): p_{k-2} read-only in its own buffer, r_{k-1} recovered from p_{k-1} /
      // p_{k-2} on every line and edge row (no r stored); the edge rows' Ap still stored (compact arrays)
      const double* __restrict__ pm2_ = T3 ? v.p_m2 + rb : (const double*)pn_;
      auto rv = [&](double r, double p) { return T3 ? fma(nbp, r, p) : r; };
      const int64_t kr = BIG ? (int64_t)i0 - 2 * (int64_t)LO : 0;  // lines -2 .. of the run: offsets >= 0
      const double* __restrict__ cvd_ = S.cvd + kr;
      const double* __restrict__ cve_ = S.cve + kr;
      const double* __restrict__ cvs_ = S.cvs + kr;
      const uint32_t ob0 = BIG ? 3u * LOB : (uint32_t)e0 << 3;
      const uint32_t xb0 = BIG ? 0u : (uint32_t)i0 << 3;
      // the coefficient arrays have one line in front: line j of the run at kb0 + j LOB
      const uint32_t kb0 = BIG ? 3u * LOB : ((uint32_t)i0 << 3) + LOB;
      const uint32_t cb0 = (uint32_t)(2 * (l0 * SS + col) - 1) << 3;
      const uint32_t oc = hi ? (z63 ? 16u : 24u) : (z0 ? 8u : 0u);
      const uint32_t op = hi ? (z63 ? 512u : 520u) : (z0 ? 8u : 0u);
      const int32_t jlo = -(e0 / LO), jhi = (ext32 - 64 - e0) / LO;
      const int32_t rlo = -(int32_t)l0, rhi = (int32_t)(nl - 1 - l0);
      auto jc = [&](int32_t j) { return j < jlo ? jlo : (j > jhi ? jhi : j); };
      auto rc_ = [&](int32_t j) { return j < rlo ? rlo : (j > rhi ? rhi : j); };
      auto kc = [&](int32_t j) { return j < rlo - 1 ? rlo - 1 : (j > rhi ? rhi : j); };
      auto line_ofs = [&](int32_t j) { return ob0 + (uint32_t)j * LOB; };
      auto raw_at = [&](int32_t j) {
        Raw q;
        const int32_t jj = jc(j);
        const uint32_t o = line_ofs(jj) + l8;
        q.r = T3 ? g_ld(pm2_, o) : g_ld((j >= 0 && j < n_run) ? (const double*)pn_ : ro_, o);
        q.p = pl.ld_p(pl.side(l0 + jj, nl), po_, o);
        return q;
      };
      auto ap_gh = [&](int32_t j) { return pl.ld_ap(pl.side(l0 + j, nl), apo_, line_ofs(j) + l8); };
      auto edge_at = [&](int32_t j) {
        Edge q;
        const uint32_t c = cb0 + (uint32_t)rc_(j) * SB + oc;
        q.r = T3 ? g_ld(pm2_, line_ofs(jc(j)) - 8u + op) : g_ld(reo, c);
        q.a = g_ld(eo, c);
        q.p = g_ld(po_, line_ofs(jc(j)) - 8u + op);
        return q;
      };
      auto coef_ofs = [&](int32_t j) { return kb0 + (uint32_t)j * LOB; };
      // o >= one line inside the loop; the prologue's front line may start at offset 0 (its ee is
      // never used there)
      auto coef_ld = [&](uint32_t o) {
        CRaw c;
        c.d = g_ld(cvd_, o + l8);
        c.e = g_ld(cve_, o + l8);
        c.s = g_ld(cvs_, o + l8);
        c.ee = g_ld(cve_, o >= 8u ? o - 8u : o);
        return c;
      };
      auto rghost = [&](int32_t j, const Raw& q) { return fma(nbp, g_ld(T3 ? pm2_ : (const double*)pn_, line_ofs(j) + l8), q.p); };
      auto is_ghost = [&](int32_t j) { return apx_o != nullptr && (l0 + j == -1 || l0 + j == nl) && j >= jlo && j <= jhi; };
      auto raw_un = [&](int32_t j) {
        Raw q;
        const uint32_t o = line_ofs(j) + l8;
        q.r = T3 ? g_ld(pm2_, o) : g_ld(j < n_run ? (const double*)pn_ : ro_, o);
        q.p = g_ld(po_, o);
        return q;
      };
      auto edge_un = [&](int32_t j) {
        Edge q;
        const uint32_t c = cb0 + (uint32_t)j * SB + oc;
        q.r = T3 ? g_ld(pm2_, line_ofs(j) - 8u + op) : g_ld(reo, c);
        q.a = g_ld(eo, c);
        q.p = g_ld(po_, line_ofs(j) - 8u + op);
        return q;
      };
      auto x_at = [&](int32_t j) {
        if constexpr (PAIR) return g_ld(x_, xb0 + (uint32_t)(j < n_run - 1 ? j : n_run - 1) * LOB + l8);
        else return 0.0;
      };
      auto mkv = [&](const CRaw& c, double s_up) {
        VSet V;
        V.v[0] = s_up;
        V.v[1] = lane_dn_or(c.e, c.ee);
        V.v[2] = c.d;
        V.v[3] = c.e;
        V.v[4] = c.s;
        return V;
      };
      auto stencil_v = [&](const VSet& V, double mid, double edge, double dnl, double upl) {
        const double upv = lane_up_or(mid, edge);
        const double dnv = lane_dn_or(mid, edge);
        double sum = fma(V.v[0], dnl, 0.0);
        sum = fma(V.v[1], dnv, sum);
        sum = fma(V.v[2], mid, sum);
        sum = fma(V.v[3], upv, sum);
        return fma(V.v[4], upl, sum);
      };
      auto epk = [&](const Edge& q) { return fma(b, q.p, fma(na, q.a, rv(q.r, q.p))); };
      const Raw rm2 = raw_at(-2), rm1 = raw_at(-1), r0 = raw_at(0);
      Raw q[LD - 1];
#pragma unroll
      for (int d = 0; d < LD - 1; ++d) q[d] = raw_at(1 + d);
      const Edge edm1 = edge_at(-1), ed0 = edge_at(0);
      Edge e[LD - 1];
#pragma unroll
      for (int d = 0; d < LD - 1; ++d) e[d] = edge_at(1 + d);
      double xs[LD - 1];
#pragma unroll
      for (int d = 0; d < LD - 1; ++d) xs[d] = x_at(d);
      const CRaw cm2 = coef_ld(coef_ofs(kc(-2))), cm1 = coef_ld(coef_ofs(kc(-1))), c0 = coef_ld(coef_ofs(0));
      CRaw cq[LD - 1];  // coefficients of lines m + 1 .. m + LD - 1
#pragma unroll
      for (int d = 0; d < LD - 1; ++d) cq[d] = coef_ld(coef_ofs(kc(1 + d)));
      double pr_pk = 0.0;
      if (l0 >= 1) {
        pr_pk = fma(b, rm1.p, fma(na, stencil_v(mkv(cm1, cm2.s), rm1.p, edm1.p, rm2.p, r0.p), rv(rm1.r, rm1.p)));
      } else if (is_ghost(-1)) {
        pr_pk = fma(b, rm1.p, fma(na, ap_gh(-1), rghost(-1, rm1)));
        if (pl.p[0] != nullptr) g_st(const_cast<double*>(po_), line_ofs(-1) + l8, rm1.p);
      }
      VSet Vs = mkv(c0, cm1.s);  // line m
      double o_pold = r0.p, o_pm2 = r0.r, o_rk, o_pk;
      o_rk = fma(na, stencil_v(Vs, r0.p, ed0.p, rm1.p, q[0].p), fma(nbp, r0.r, r0.p));
      o_pk = fma(b, r0.p, o_rk);
      double o_epk = epk(ed0);
      auto lstep = [&](auto clc, int32_t m, int next) __attribute__((always_inline)) {
        constexpr bool CL = decltype(clc)::value;
        const Raw qn = CL ? raw_at(m + LD) : raw_un(m + LD);
        const Edge en2 = CL ? edge_at(m + LD) : edge_un(m + LD);
        const double xn = x_at(m + LD - 1);
        const CRaw cn = coef_ld(coef_ofs(CL ? kc(m + LD) : m + LD));
        const VSet Vt = mkv(cq[0], Vs.v[4]);  // line m + 1
        double rk1 = 0.0, pk1 = 0.0;
        if (next == 1) {
          const double t = stencil_v(Vt, q[0].p, e[0].p, o_pold, q[1].p);
          rk1 = fma(na, t, (T3 || m + 1 < n_run) ? fma(nbp, q[0].r, q[0].p) : q[0].r);
          pk1 = fma(b, q[0].p, rk1);
        } else if (CL && next == 2) {
          rk1 = fma(na, ap_gh(m + 1), rghost(m + 1, q[0]));
          pk1 = fma(b, q[0].p, rk1);
          if (pl.p[1] != nullptr) g_st(const_cast<double*>(po_), line_ofs(m + 1) + l8, q[0].p);
        }
        const double sum = stencil_v(Vs, o_pk, o_epk, pr_pk, pk1);
        const uint32_t ob = line_ofs(m);
        const double rr = fma(-b, o_pold, o_pk);
        if constexpr (!T3) {
          if (m == 0 || m == n_run - 1) g_st_nt(rn_, ob + l8, rr);
        }
        if (edge_lane) {
          const uint32_t sb = cb0 + (uint32_t)m * SB + (hi ? 16u : 8u);
          if constexpr (!T3) g_st(ren, sb, rr);
          g_st(en, sb, sum);
        }
        if constexpr (PAIR) g_st_nt(x_, xb0 + (uint32_t)m * LOB + l8, fma(a, o_pold, fma(ap, o_pm2, xs[0])));
        const bool bnd = l0 + m == 0 || l0 + m == nl - 1;
        if constexpr (CL) pl.st_pub(bnd, pn_, ob + l8, o_pk, true);
        else g_st_nt(pn_, ob + l8, o_pk);
        if (CL && apx_n != nullptr && bnd) pl.st_pub(true, apn_, ob + l8, sum, false);
        s_pap = fma(o_pk, sum, s_pap);
        s_rap = fma(o_rk, sum, s_rap);
        s_apap = fma(sum, sum, s_apap);
        s_rr = fma(o_rk, o_rk, s_rr);
        pr_pk = o_pk;
        o_pk = pk1;
        o_rk = rk1;
        o_pold = q[0].p;
        o_pm2 = q[0].r;
        o_epk = epk(e[0]);
        Vs = Vt;
#pragma unroll
        for (int d = 0; d + 1 < LD - 1; ++d) {
          q[d] = q[d + 1];
          e[d] = e[d + 1];
          xs[d] = xs[d + 1];
          cq[d] = cq[d + 1];
        }
        q[LD - 2] = qn;
        e[LD - 2] = en2;
        xs[LD - 2] = xn;
        cq[LD - 2] = cn;
      };
      const std::true_type clamped;
      const std::false_type unclamped;
      const int32_t m_lo = l0 == 0 ? 1 : 0;  // the rank's first line stores its Ap_k (clamped step)
      const int32_t m_hi = min(n_run - 1, (int32_t)(nl - 1 - LD - l0));
      int32_t m = 0;
      if (m_lo == 1) lstep(clamped, 0, 1);
      m = m_lo;
      for (; m + LD - 1 <= m_hi; m += LD) {
#pragma unroll
        for (int u = 0; u < LD; ++u) lstep(unclamped, m + u, 1);
      }
      for (; m <= m_hi; ++m) lstep(unclamped, m, 1);
      for (; m < n_run; ++m) {
        const bool lastl = l0 + m == nl - 1;
        lstep(clamped, m, !lastl ? 1 : (is_ghost(m + 1) ? 2 : 0));
      }
      pl.release(l0, l1, nl);
      continue;
    }
    if (LEAN == 0 || gblk) {
    // lines j (relative to l0) inside the ext vectors: [jmin, jmax]; loads clamp to them (values
    // of lines that do not exist are never multiplied: the matrix has no entry for them)
    const int32_t jmax = (ext32 - 64 - e0) / LO;
    const int32_t jmin = -(e0 / LO);
    auto ebase = [&](int32_t j) { return e0 + (j < jmin ? jmin : (j > jmax ? jmax : j)) * LO; };
    auto owned = [&](int32_t j) { return l0 + j >= 0 && l0 + j < nl; };
    auto oline = [&](int32_t j) {  // clamped to the rank's lines
      const int64_t L = l0 + j;
      return L < 0 ? (int64_t)0 : (L >= nl ? nl - 1 : L);
    };
    // P3: lines of this run take p_{k-2} (their r is recovered at use), others the stored r; the
    // pointer is chosen before the load (wave-uniform), the recovery selected after it arrives
    auto inrun = [&](int32_t j) { return !rfull && j >= 0 && j < n_run; };
    // in-kernel halo (lean_split ranks: the generic runs that hold a rank-end line): a ghost line's
    // p_{k-1} and Ap_{k-1} from the neighbour's rows, the rank's first / last line published
    // write-through, as in the lean loops (PullBases)
    PullBases pl;
    pl.at(v, 0);
    auto gside = [&](int32_t j) { return pl.side(l0 + (j < jmin ? jmin : (j > jmax ? jmax : j)), nl); };
    // T3 (three p buffers, a split rank's generic runs): p_{k-2} read-only in its own buffer on every line,
    // r_{k-1} recovered everywhere (no stored r); the neighbouring slices' edge rows recomputed from their
    // codes and p's (load_edge / edge_pk3) -- no compact edge arrays, as in the lean T3 loop
    const double* __restrict__ pm2 = T3 ? v.p_m2 : (const double*)pn;
    auto load_raw = [&](int32_t j, Raw& q) {
      const int32_t e = ebase(j) + lane;
      q.r = ld_once((T3 ? pm2 : (inrun(j) ? (const double*)pn : ro)) + e, ntl);
      const int sd = gside(j);
      q.p = sd != 0 ? ld_sys(pl.p[sd - 1] + e, 0u) : ld_once(po + e, ntl);
    };
    // a pulled ghost line's p_{k-1} kept in this rank's ghost rows: the next pass's p_{k-2} there (rghost)
    auto keep_ghost_p = [&](int32_t j, const Raw& q) {
      if (gside(j) != 0) const_cast<double*>(po)[ebase(j) + lane] = q.p;
    };
    auto ghost_ap = [&](int32_t j) {
      const int sd = gside(j);
      return sd != 0 ? ld_sys(pl.ap[sd - 1] + (ebase(j) + lane), 0u) : apx_o[ebase(j) + lane];
    };
    auto rof = [&](int32_t j, const Raw& q) { return (T3 || inrun(j)) ? fma(nbp, q.r, q.p) : q.r; };
    auto load_edge = [&](int32_t j, Edge& q) {
      const int32_t e = ebase(j);
      const int64_t s = oline(j) * SS + col;
      if constexpr (T3) {
        // the neighbouring edge row (row -1 / 64 of the slice: lane 63 of slice s - 1 / lane 0 of s + 1) and
        // the row beyond it (-2 / 65): their p_{k-1} (a pulled ghost line's from the neighbour's rows), the
        // edge row's p_{k-2} and its codes; edge_pk3 recomputes its p_k in its owner's fma order
        if (lane == 0 || lane == 63) {
          const bool hi = lane == 63;
          const int32_t row = hi ? (e + 64 < ext32 ? e + 64 : ext32 - 1) : (e >= 1 ? e - 1 : 0);
          const int32_t row2 = hi ? (row + 1 < ext32 ? row + 1 : ext32 - 1) : (row >= 1 ? row - 1 : 0);
          const int sd = gside(j);
          q.p = sd != 0 ? ld_sys(pl.p[sd - 1] + row, 0u) : po[row];
          q.a = sd != 0 ? ld_sys(pl.p[sd - 1] + row2, 0u) : po[row2];
          q.r = pm2[row];
          const int64_t sn = hi ? (s + 1 < nsl ? s + 1 : nsl - 1) : (s >= 1 ? s - 1 : 0);
          ArCodes<4, 5> ce;
          ar_load_dia<5>(S.dia4 + sn * 160, hi ? 0 : 63, ce);
          q.c = ce.pk[0];
        }
        return;
      }
      if constexpr (P3 && MCG_EDGE_BRANCHLESS) {
        // every lane loads (lanes 1-62 at lane 0's addresses, the same cache lines): selects instead
        // of exec-mask branches around the two edge lanes
        const bool hi = lane == 63;
        const int32_t row = hi ? (e + 64 < ext32 ? e + 64 : ext32 - 1) : (e >= 1 ? e - 1 : 0);
        const int64_t c = hi ? (s + 1 < nsl ? 2 * (s + 1) : 2 * nsl - 1) : (s >= 1 ? 2 * (s - 1) + 1 : 0);
        q.r = reo[c];
        q.p = po[row];
        q.a = eo[c];
        return;
      }
      if (lane == 0) {
        const int32_t row = e >= 1 ? e - 1 : 0;
        const int64_t c = s >= 1 ? 2 * (s - 1) + 1 : 0;
        q.r = P3 ? reo[c] : ro[row];
        q.p = po[row];
        q.a = eo[c];
      } else if (lane == 63) {
        const int32_t row = e + 64 < ext32 ? e + 64 : ext32 - 1;
        const int64_t c = s + 1 < nsl ? 2 * (s + 1) : 2 * nsl - 1;
        q.r = P3 ? reo[c] : ro[row];
        q.p = po[row];
        q.a = eo[c];
      }
    };
    auto load_xp = [&](int32_t j, XP& q) {
      if constexpr (PAIR) {
        const int32_t mm = j < n_run - 1 ? j : n_run - 1;
        if constexpr (!P3) q.pkm2 = ld_once(pn + e0 + mm * LO + lane, ntl);  // P3: already read (o_pm2)
        q.xo = ld_once(x + i0 + mm * LO + lane, ntl);
      }
    };
    // dia4: the "metadata" is the slice index (fixed 160 B per slice, nothing to load)
    auto load_meta = [&](int32_t j) {
      if constexpr (CM >= 4) return (uint32_t)(oline(j) * SS + col);
      else return meta[oline(j) * SS + col + vz];
    };
    auto load_codes = [&](uint32_t mt, ArCodes<CM, U>& c) {
      if constexpr (CM == 5) {  // diav: own d, e, s; north = s one line up, west = e of the row before
        const int64_t f = (int64_t)mt * 64 + LO;
        c.k[0] = S.cvs[f - LO + lane];
        c.k[2] = S.cvd[f + lane];
        c.k[3] = S.cve[f + lane];
        c.k[4] = S.cvs[f + lane];
        c.k[1] = lane_dn_or(c.k[3], S.cve[f - 1]);
      } else if constexpr (CM == 4) ar_load_dia<U>(S.dia4 + (int64_t)mt * 160, lane, c);
      else ar_load_codes<CM, U>(S, (int64_t)(mt & 0x0fffffffu) << 6, (int)(mt >> 28), lane, c);
    };
    auto edge_p = [&](const Edge& q) { return q.p; };
    auto edge_pk = [&](const Edge& q) { return fma(b, q.p, fma(na, q.a, q.r)); };  // p_k of the edge row
    // T3: the edge row's p_k from its p_{k-1} on lines j - 1 / j + 1 (prev / next), the row beyond it (q.a),
    // itself, this lane's own p_{k-1} (own) and its codes -- the owner's stencil (canonical slot order)
    auto edge_pk3 = [&](double prev, const Edge& q, double next, double own) {
      const bool hi = lane == 63;
      const double g[5] = {prev, hi ? own : q.a, q.p, hi ? q.a : own, next};
      double t = 0.0;
#pragma unroll
      for (int u = 0; u < 5; ++u) t = fma(s_val[(q.c >> (4 * u)) & 15u], g[u], t);
      return fma(b, q.p, fma(na, t, fma(nbp, q.r, q.p)));
    };
    // ghost line: Ap_{k-1} exchanged by the halo (multi-rank only)
    auto ghost = [&](int32_t j) { return apx_o != nullptr && (l0 + j == -1 || l0 + j == nl) && j >= jmin && j <= jmax; };
    // r_{k-1} of a ghost line (P > 1).  P3: recovered like an own line -- no wave writes the ghost
    // rows, and the halo delivered p_{k-2} into p_new's ghost rows two iterations ago -- so the halo
    // carries {Ap, p} and not r (one extra load, at a run's outer step only)
    auto rghost = [&](int32_t j, const Raw& q) {
      if constexpr (T3) return fma(nbp, q.r, q.p);  // q.r: p_{k-2} of the ghost rows (load_raw)
      return P3 && !first ? fma(nbp, pn[ebase(j) + lane], q.p) : q.r;
    };

    // prologue: p_k of lines -1 and 0, r_k of line 0; operands of lines 1 .. QD, codes of 0, 1
    Raw rm2, rm1, r0, rq[QD];
    load_raw(-2, rm2);
    load_raw(-1, rm1);
    load_raw(0, r0);
#pragma unroll
    for (int d = 0; d < QD; ++d) load_raw(1 + d, rq[d]);
    Edge edm1, ed0, ed1;
    load_edge(-1, edm1);
    load_edge(0, ed0);
    load_edge(1, ed1);
    ArCodes<CM, U> cm1, c0, c1;
    load_codes(load_meta(-1), cm1);
    load_codes(load_meta(0), c0);
    load_codes(load_meta(1), c1);
    uint32_t mt2 = load_meta(2);  // codes metadata one step ahead of the codes loads
    XP x0{0.0, 0.0};
    load_xp(0, x0);
    // even three-term pass (E3): edge rows two lines ahead, so the operand, codes and edge streams
    // are chains of 3 registers that the 3-step unroll renames -- no register whose load is in
    // flight is moved at the end of a step (a move waits for its load, which drained every step's
    // prefetches before the next step)
    constexpr bool E3 = P3 && !PAIR && UN == 3 && QD == 2;
    Edge ed2p;
    if constexpr (E3) load_edge(2, ed2p);
    double pr_pk = 0.0;
    if (owned(-1)) {
      const double t = stencil(cm1, rm1.p, edge_p(edm1), rm2.p, r0.p);
      pr_pk = fma(b, rm1.p, fma(na, t, rof(-1, rm1)));
    } else if (ghost(-1)) {
      const double t = ghost_ap(-1);
      pr_pk = fma(b, rm1.p, fma(na, t, rghost(-1, rm1)));
      keep_ghost_p(-1, rm1);
    }
    double o_pold = r0.p, o_pm2 = r0.r, o_rk, o_pk;
    {
      const double t = stencil(c0, r0.p, edge_p(ed0), rm1.p, rq[0].p);
      o_rk = fma(na, t, rof(0, r0));
      o_pk = fma(b, r0.p, o_rk);
    }
    double o_epk, ep_m = 0.0;  // T3: p_{k-1} of the neighbouring edge row, line m (carried)
    if constexpr (T3) {
      o_epk = edge_pk3(edm1.p, ed0, ed1.p, r0.p);
      ep_m = ed0.p;
    } else {
      o_epk = edge_pk(ed0);
    }
    // one line step; the rotation at its end is register renaming once the driver below unrolls
    // the steps by the rotation period (a rolled loop pays ~30 64-bit moves per step)
    auto step = [&](int32_t m) {
      // 1. loads for later steps, in the order they are waited for: metadata of line m + 3, codes
      //    of line m + 2 (metadata from the previous step), edges of line m + 2, x / p_{k-2} of
      //    line m + 1, operands of line m + 1 + QD.  All vector loads: the in-order vmcnt lets
      //    every wait leave the younger prefetches in flight
      const uint32_t mt3 = load_meta(m + 3);
      ArCodes<CM, U> c2;
      load_codes(mt2, c2);
      Edge ed2;  // edges of line m + 2 (E3: m + 3)
      load_edge(m + (E3 ? 3 : 2), ed2);
      XP x1{0.0, 0.0};
      load_xp(m + 1, x1);
      Raw rnq;
      load_raw(m + 1 + QD, rnq);
      // 2. r_k, p_k of line m + 1: Ap_{k-1} recomputed (owned) or exchanged (ghost line)
      double rk1 = 0.0, pk1 = 0.0;
      if (owned(m + 1)) {
        const double t = stencil(c1, rq[0].p, edge_p(ed1), o_pold, rq[1].p);
        rk1 = fma(na, t, rof(m + 1, rq[0]));
        pk1 = fma(b, rq[0].p, rk1);
      } else if (ghost(m + 1)) {
        const double t = ghost_ap(m + 1);
        rk1 = fma(na, t, rghost(m + 1, rq[0]));
        pk1 = fma(b, rq[0].p, rk1);
        keep_ghost_p(m + 1, rq[0]);
      }
      // 3. Ap_k of line m, stores, partials
      const double sum = stencil(c0, o_pk, o_epk, pr_pk, pk1);
      const int32_t eb = e0 + m * LO;
      const int64_t s = (l0 + m) * SS + col;
      if constexpr (T3) {
        // nobody reads a stored r or edge row
      } else if constexpr (P3) {
        // r_k only where another wave (edge rows: compact, next to their Ap; the run's outer
        // lines) or rank reads it, and as the value the next pass recovers from the stored p's,
        // fma(-b, p_{k-1}, p_k): every reader of a row's r_k -- owner, neighbouring wave,
        // neighbouring rank -- uses the same bits
        const double rr = fma(-b, o_pold, o_pk);
        if (m == 0 || m == n_run - 1) st_stream(&(rn + eb)[lane], rr);
        if (lane == 0 || lane == 63) ren[2 * s + (lane == 63 ? 1 : 0)] = rr;
      } else {
        st_stream(&(rn + eb)[lane], o_rk);
        if (ren != nullptr && (lane == 0 || lane == 63)) ren[2 * s + (lane == 63 ? 1 : 0)] = o_rk;
      }
      if constexpr (PAIR) st_stream(&(x + i0 + m * LO)[lane], fma(a, o_pold, fma(ap, P3 ? o_pm2 : x0.pkm2, x0.xo)));
      const bool bnd = l0 + m == 0 || l0 + m == nl - 1;  // the halo's source lines
      if (pl.pub && bnd) st_sys(pn + eb, (uint32_t)lane << 3, o_pk);
      else st_stream(&(pn + eb)[lane], o_pk);
      if constexpr (!T3)
        if (lane == 0 || lane == 63) en[2 * s + (lane == 63 ? 1 : 0)] = sum;
      if (apx_n != nullptr && bnd) {
        if (pl.pub) st_sys(apx_n + eb, (uint32_t)lane << 3, sum);
        else apx_n[eb + lane] = sum;
      }
      s_pap = fma(o_pk, sum, s_pap);
      s_rap = fma(o_rk, sum, s_rap);
      s_apap = fma(sum, sum, s_apap);
      s_rr = fma(o_rk, o_rk, s_rr);
      // 4. rotate
      pr_pk = o_pk;
      o_pk = pk1;
      o_rk = rk1;
      if constexpr (T3) {
        if constexpr (E3) o_epk = edge_pk3(ep_m, ed1, ed2p.p, rq[0].p);
        else o_epk = edge_pk3(ep_m, ed1, ed2.p, rq[0].p);
        ep_m = ed1.p;
      } else {
        o_epk = edge_pk(ed1);
      }
      o_pold = rq[0].p;
      o_pm2 = rq[0].r;
      if constexpr (E3) {
        ed1 = ed2p;
        ed2p = ed2;
      } else {
        ed1 = ed2;
      }
#pragma unroll
      for (int d = 0; d + 1 < QD; ++d) rq[d] = rq[d + 1];
      rq[QD - 1] = rnq;
      x0 = x1;
      c0 = c1;
      c1 = c2;
      mt2 = mt3;
    };
    // P3 even passes: unrolled by 3, the period of the codes / p_k chains (the odd pass, with x, then
    // spills; it runs at the HBM rate rolled)
    constexpr int kUn = (P3 && !PAIR) ? UN : 1;
    int32_t m = 0;
    if constexpr (kUn > 1) {
      for (; m + kUn <= n_run; m += kUn) {
#pragma unroll
        for (int u = 0; u < kUn; ++u) step(m + u);
      }
    }
    for (; m < n_run; ++m) step(m);
    pl.release(l0, l1, nl);
    }  // !LEAN
    }  // sub-ranges
  }
#if defined(MCG_CARRY_DIAG)
  const unsigned long long t_work = wall_clock64();
#endif
  f1_finish(s_pap, s_rap, s_apap, s_rr, partials, pstride, rc, st, tol);
#if defined(MCG_CARRY_DIAG)
  const int64_t dw = blk * kWaves + (threadIdx.x >> 6);
  if (lane == 0 && dw < kCarryDiagMax) {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4), xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);
    g_carry_diag[4 * dw] = t_in;
    g_carry_diag[4 * dw + 1] = t_work;
    g_carry_diag[4 * dw + 2] = wall_clock64();
    g_carry_diag[4 * dw + 3] = ((unsigned long long)xcc << 32) | hw;
  }
#endif
}


}  // namespace

void cg_carry_ar(int cm, int param, int depth, const SellDev& S, const F1Vectors& v, int64_t own_off,
                 const TileRanges& tr, double* partials, int pstride, int grid, CgState* st, double tol, int first,
                 int check, int k, int final_mode, hipStream_t stream, const RedCtl& rc, bool p3, int unroll,
                 bool lean) {
  if (tr.ntiles == 0 || grid == 0) return;
  MCG_CHECK(tr.strip > 0 && tr.nt0 == tr.ntiles && tr.nt0 % tr.strip == 0 && tr.b0 == 0,
            "Ap-recomputing carry: one launch over the rank's whole grid lines");
  MCG_CHECK((cm == 2 || cm == 4 || cm == 5) && param >= 4 && param <= 5 && (cm == 5 || S.dict != nullptr),
            "Ap-recomputing carry: SELL-64/c8, /c4, /dia4 or /diav rows of at most 5 entries");
  MCG_CHECK(cm != 4 || (S.dia4 != nullptr && S.dvals != nullptr), "Ap-recomputing carry: dia4 codes missing");
  MCG_CHECK(cm != 5 || (S.cvd != nullptr && S.cve != nullptr && S.cvs != nullptr),
            "Ap-recomputing carry: diav coefficients missing");
  MCG_CHECK(final_mode || cm >= 4 || S.smeta != nullptr, "Ap-recomputing carry: slice metadata missing");
  MCG_CHECK(v.ape_old != nullptr && v.ape_new != nullptr && v.r_old && v.p_old && v.r_new && v.p_new,
            "Ap-recomputing carry: vectors missing");
  MCG_CHECK((v.ap_old == nullptr) == (v.ap_new == nullptr), "Ap-recomputing carry: boundary Ap buffers");
  MCG_CHECK(rc.ngroups == 0 || (!final_mode && rc.base % kRedGroup == 0 && rc.cnt && rc.lvl2),
            "in-kernel reduction: bad control block");
  MCG_CHECK(!p3 || cm >= 4, "three-term carry: SELL-64/dia4 or /diav only");
  const bool p3k = p3 && !first;  // pass 0: the two-term kernel (r_{-1} = b stored in full)
  if (final_mode) {
    const int64_t n = tr.nt0 * 64;
#define MCG_AF(CM, U)                                                                                        \
  hipLaunchKernelGGL((k_ar_final<CM, U>), dim3(grid), dim3(kBS), 0, stream, S, v, own_off, n, \
                     (int32_t)(tr.strip * 64), 0, partials, pstride, st, tol, first, check, k, p3)
    if (cm == 4) MCG_AF(4, 5);
    else if (cm == 5) MCG_AF(5, 5);
    else { if (param == 4) MCG_AF(2, 4); else MCG_AF(2, 5); }
#undef MCG_AF
    MCG_HIP(hipGetLastError(), "compute axpy failed(r)");
    return;
  }
  const bool pair = (k & 1) != 0;
  const bool big = v.ext_len >= ((int64_t)1 << 29);  // lean kernels: per-run 64-bit bases
#if defined(MCG_CARRY_DIAG)
  // diagnostic build: after the launches numbered MCG_CARRY_DIAG_AT and the next one (eager runs), the
  // per-wave records into MCG_CARRY_DIAG_FILE.<launch>
  struct DiagDump {
    hipStream_t s;
    int grid;
    ~DiagDump() {
      static int launch = 0;
      static const int at = std::getenv("MCG_CARRY_DIAG_AT") ? std::atoi(std::getenv("MCG_CARRY_DIAG_AT")) : -1;
      const char* fn = std::getenv("MCG_CARRY_DIAG_FILE");
      const int me = launch++;
      if (fn == nullptr || at < 0 || (me != at && me != at + 1)) return;
      std::vector<unsigned long long> d(4 * kCarryDiagMax);
      if (hipStreamSynchronize(s) != hipSuccess) return;
      if (hipMemcpyFromSymbol(d.data(), HIP_SYMBOL(g_carry_diag), d.size() * sizeof(unsigned long long)) != hipSuccess) return;
      const std::string path = std::string(fn) + "." + std::to_string(me);
      unsigned long long rd[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      (void)hipMemcpyFromSymbol(rd, HIP_SYMBOL(g_red_diag), sizeof(rd));
      if (FILE* fr = std::fopen((path + ".red").c_str(), "w")) {  // the reduction tail's steps (f1_common.hpp)
        for (int i = 0; i < 8; ++i) std::fprintf(fr, "%llu\n", rd[i]);
        std::fclose(fr);
      }
      if (FILE* fo = std::fopen(path.c_str(), "w")) {
        const int nw = std::min(grid * kWaves, kCarryDiagMax);
        for (int w = 0; w < nw; ++w)
          std::fprintf(fo, "%d %d %llu %llu %llu %u %u\n", w / kWaves, w % kWaves, d[4 * w], d[4 * w + 1], d[4 * w + 2],
                       (unsigned)(d[4 * w + 3] & 0xffffffffu), (unsigned)(d[4 * w + 3] >> 32));
        std::fclose(fo);
      }
    }
  } diag_dump{stream, grid};
#endif
  MCG_CHECK(v.ext_len < ((int64_t)1 << 31), "Ap-recomputing carry: a rank's vectors must stay below 2^31 rows");
  if (cm == 4 && p3k && lean && S.dpat != nullptr) {  // lean-only kernels (4 waves per SIMD)
    const bool t3 = v.p_m2 != nullptr;  // three p buffers (kernel comment)
#define MCG_LW(QD, PAIR)                                                                                       \
  do {                                                                                                         \
    if (big && t3)                                                                                             \
      hipLaunchKernelGGL((k_cg_carry_ar<4, 5, QD, PAIR, true, 1, 4, true, false, true>), dim3(grid), dim3(kBS), 0, stream, \
                         S, v, own_off, tr, partials, pstride, st, tol, first, check, rc);                     \
    else if (big)                                                                                              \
      hipLaunchKernelGGL((k_cg_carry_ar<4, 5, QD, PAIR, true, 1, 4, true>), dim3(grid), dim3(kBS), 0, stream, S, v, \
                         own_off, tr, partials, pstride, st, tol, first, check, rc);                           \
    else if (t3)                                                                                               \
      hipLaunchKernelGGL((k_cg_carry_ar<4, 5, QD, PAIR, true, 1, 4, false, false, true>), dim3(grid), dim3(kBS), 0, stream, \
                         S, v, own_off, tr, partials, pstride, st, tol, first, check, rc);                     \
    else                                                                                                       \
      hipLaunchKernelGGL((k_cg_carry_ar<4, 5, QD, PAIR, true, 1, 4>), dim3(grid), dim3(kBS), 0, stream, S, v, own_off, \
                         tr, partials, pstride, st, tol, first, check, rc);                                    \
  } while (0)
#define MCG_LWE(QD, PAIR, W)                                                                                   \
  do {                                                                                                         \
    if (t3)                                                                                                    \
      hipLaunchKernelGGL((k_cg_carry_ar<4, 5, QD, PAIR, true, 1, W, false, true, true>), dim3(grid), dim3(kBS), 0, stream, \
                         S, v, own_off, tr, partials, pstride, st, tol, first, check, rc);                     \
    else                                                                                                       \
      hipLaunchKernelGGL((k_cg_carry_ar<4, 5, QD, PAIR, true, 1, W, false, true>), dim3(grid), dim3(kBS), 0, stream, S, \
                         v, own_off, tr, partials, pstride, st, tol, first, check, rc);                        \
  } while (0)
    // packed edges (depth 13: QD 3 at 5 waves per SIMD, 15: QD 3 at 6 (even passes whose runs keep >= 64
    // lines; with three p buffers 80 VGPRs: r4's two-buffer kernel spilled there), 14: QD 4 at 4 (odd), the
    // setup's auto_mix_; measured and dropped: QD 5 at 4 for the odd passes, the same rate; r5: QD 4 for
    // the even ones at 5 / 6 (16384^2 644.6 / 620.1 vs 646.0, profiles/r5/mix/qd4); r5 also dropped depth
    // 2, 4 (3 waves per SIMD) and 6 (2): profiles/r3/lean, r4/mix)
    if (depth == 13 && !big) { if (pair) MCG_LWE(3, true, 5); else MCG_LWE(3, false, 5); }
    else if (depth == 15 && !big && !pair) MCG_LWE(3, false, 6);  // even passes at 6 waves per SIMD
    else if (depth == 14 && !big && t3 && tr.sub_ranges != 0) {
      // a split rank's lean launch (COMBO): the lean stretches, and (gen_blocks > 0) the generic ranges'
      // workgroups ahead of the lean ones in the same launch
      MCG_CHECK(tr.gen_blocks % 8 == 0 && grid > tr.gen_blocks && (tr.gen_blocks == 0 || tr.gen_list != nullptr),
                "lean split: the combined launch's generic workgroups");
      if (pair)
        hipLaunchKernelGGL((k_cg_carry_ar<4, 5, 4, true, true, 1, 4, false, true, true, true>), dim3(grid), dim3(kBS), 0,
                           stream, S, v, own_off, tr, partials, pstride, st, tol, first, check, rc);
      else
        hipLaunchKernelGGL((k_cg_carry_ar<4, 5, 4, false, true, 1, 4, false, true, true, true>), dim3(grid), dim3(kBS), 0,
                           stream, S, v, own_off, tr, partials, pstride, st, tol, first, check, rc);
    }
    else if (depth == 14 && !big) { if (pair) MCG_LWE(4, true, 4); else MCG_LWE(4, false, 4); }
    else { if (pair) MCG_LW(3, true); else MCG_LW(3, false); }
#undef MCG_LWE
#undef MCG_LW
    MCG_HIP(hipGetLastError(), "compute mv failed(Ap)");
    return;
  }
  if (cm == 5 && p3k && lean) {  // diav lean-only kernels: the streamed coefficients need more VGPRs
#define MCG_LV(QD, PAIR)                                                                                        \
  do {                                                                                                          \
    if (v.p_m2 != nullptr)                                                                                      \
      hipLaunchKernelGGL((k_cg_carry_ar<5, 5, QD, PAIR, true, 1, kLeanV, false, false, true>), dim3(grid), dim3(kBS), 0, \
                         stream, S, v, own_off, tr, partials, pstride, st, tol, first, check, rc);              \
    else if (big)                                                                                               \
      hipLaunchKernelGGL((k_cg_carry_ar<5, 5, QD, PAIR, true, 1, kLeanV, true>), dim3(grid), dim3(kBS), 0, stream, S, \
                         v, own_off, tr, partials, pstride, st, tol, first, check, rc);                         \
    else                                                                                                        \
      hipLaunchKernelGGL((k_cg_carry_ar<5, 5, QD, PAIR, true, 1, kLeanV>), dim3(grid), dim3(kBS), 0, stream, S, v, \
                         own_off, tr, partials, pstride, st, tol, first, check, rc);                            \
  } while (0)
    MCG_CHECK(v.p_m2 == nullptr || !big, "diav carry, three p buffers: ranks below 2^29 rows");
    if (depth >= 3) { if (pair) MCG_LV(3, true); else MCG_LV(3, false); }
    else { if (pair) MCG_LV(2, true); else MCG_LV(2, false); }
#undef MCG_LV
    MCG_HIP(hipGetLastError(), "compute mv failed(Ap)");
    return;
  }
  const int qd = depth <= 2 ? 2 : 3;  // operand prefetch depth in lines (solver: 2 or 3)
#define MCG_A(CM, U, QD, PAIR, P3, ...)                                                                 \
  hipLaunchKernelGGL((k_cg_carry_ar<CM, U, QD, PAIR, P3, ##__VA_ARGS__>), dim3(grid), dim3(kBS), 0, stream, S, v, \
                     own_off, tr, partials, pstride, st, tol, first, check, rc)
#define MCG_AP(CM, U, QD)                                        \
  do {                                                           \
    if constexpr (CM >= 4) {                                     \
      if (p3k) {                                                 \
        if (pair) MCG_A(CM, U, QD, true, true);                  \
        else if (unroll > 1) MCG_A(CM, U, QD, false, true, 3);   \
        else MCG_A(CM, U, QD, false, true);                      \
        break;                                                   \
      }                                                          \
    }                                                            \
    if (pair) MCG_A(CM, U, QD, true, false);                     \
    else MCG_A(CM, U, QD, false, false);                         \
  } while (0)
#define MCG_AQ(CM, U)                         \
  do {                                        \
    if (qd == 2) MCG_AP(CM, U, 2);            \
    else MCG_AP(CM, U, 3);                    \
  } while (0)
  if (cm == 4 && p3k && v.p_m2 != nullptr) {
    // three p buffers on a split rank's generic runs (T3: no stored r or edge rows)
    // (the even passes rolled at depth 3: the 3-step unroll at depth 2 spills 13 VGPRs with the recomputed edges;
    // also every run of a one-launch pass -- the setup's placement probe)
    if (pair) MCG_A(4, 5, 3, true, true, 1, 0, false, false, true);
    else MCG_A(4, 5, 3, false, true, 1, 0, false, false, true);
  } else if (cm == 4) MCG_AQ(4, 5);
  else if (cm == 5) MCG_AQ(5, 5);
  else { if (param == 4) MCG_AQ(2, 4); else MCG_AQ(2, 5); }
#undef MCG_AQ
#undef MCG_AP
#undef MCG_A
  MCG_HIP(hipGetLastError(), "compute mv failed(Ap)");
}

}  // namespace kern
}  // namespace mcg
