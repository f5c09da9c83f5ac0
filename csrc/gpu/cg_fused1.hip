// Single-reduction fused CG iteration (one streaming pass + one reduction + one
// 32-byte all-reduce per iteration).  See kernels.hpp "cg_fused1" for the math.
//
// Compared with the two-pass form in cg_kernels.hip (K_A SpMV pass + K_B residual
// pass, two reductions, two all-reduces), the residual update r_k = r_{k-1} -
// a Ap_{k-1} moves into the next SpMV pass, where the neighbours' p_k values are
// recomputed from (r_{k-1}, Ap_{k-1}, p_{k-1}) exactly as their owners compute them.
// HBM traffic per 5-pt SELL row drops from ~132 B to ~124 B, the per-iteration
// kernel count from 4 to 2, and — what matters for multi-GPU strong scaling —
// the latency-bound all-reduces from two to one.  r, Ap and p are
// double-buffered by iteration parity because neighbours gather the old values
// while the owner writes the new ones.
#include <hip/hip_runtime.h>

#include <cmath>
#include <mutex>
#include <type_traits>

#include "mcg/check.hpp"
#include "mcg/kernels.hpp"
#include "spmv_engines.hpp"

namespace mcg {
namespace kern {
namespace {

#include "f1_common.hpp"
constexpr int kReduceBS = 1024;

template <int FMT, typename IdxT, int U, bool RA>
__global__ __launch_bounds__(kBS) void k_cg_f1(CsrDev<IdxT> A, SellDev S, F1Vectors v, int64_t own, TileRanges tr,
                                               double* __restrict__ partials, int pstride,
                                               CgState* st, double tol, int first, int check,
                                               int final_mode, int k, RedCtl rc) {
  const int done = st->done;
  const F1Scalars sc = f1_scalars(st, tol, first, check);
  if ((done || sc.conv) && !final_mode) {  // x_{k-1} is the answer; the reduce latches
    f1_finish(0.0, 0.0, 0.0, 0.0, partials, pstride, rc, st, tol);
    return;
  }
  const double a = sc.alpha, b = sc.beta, na = -a, ap = st->a_prev;
  const double* __restrict__ ro = v.r_old;
  const double* __restrict__ apo = v.ap_old;
  const double* __restrict__ po = v.p_old;
  double* __restrict__ rn = v.r_new;
  double* __restrict__ apn = v.ap_new;
  double* __restrict__ pn = v.p_new;
  double* __restrict__ x = v.x;
  const double2* __restrict__ rao = v.ra_old;
  double2* __restrict__ ran = v.ra_new;
  // r_k = r_{k-1} - a Ap_{k-1} at ext index e (one 16-B load in the interleaved layout)
  auto r_next = [&](int64_t e) -> double {
    if constexpr (RA) {
      const double2 q = rao[e];
      return fma(na, q.y, q.x);
    } else {
      return fma(na, apo[e], ro[e]);
    }
  };
  double s_pap = 0.0, s_rap = 0.0, s_apap = 0.0, s_rr = 0.0;
  if (final_mode) {
    // every owned row of the launch, no SpMV
    auto for_rows = [&](auto&& f) {
      const int64_t n = FMT == 0 ? A.n_rows : S.n_rows;
      const int64_t unit = FMT == 0 ? kTileRows : 64;
      const int64_t sub = FMT == 0 ? 0 : (threadIdx.x >> 6), nsub = FMT == 0 ? 1 : kWaves;
      const int64_t lane = FMT == 0 ? threadIdx.x : (threadIdx.x & 63);
      for (eng::TileCursor cur = eng::tile_cursor(tr, sub, nsub); cur.t < cur.end; cur.t += cur.step) {
        const int64_t t = cur.t;
        const int64_t u0 = FMT == 0 ? (t < tr.nt0 ? tr.b0 + t * kTileRows : tr.b1 + (t - tr.nt0) * kTileRows)
                                    : eng::tile_unit(tr, t);
        const int64_t i = (FMT == 0 ? u0 : u0 * unit) + lane;
        const int64_t lim = FMT == 0 ? (t < tr.nt0 ? tr.e0 : tr.e1) : n;
        if (i < lim && i < n) f(i);
      }
    };
    if (done || sc.conv) {
      // converged: the answer is x_m; if m is even its a_{m-1} p_{m-1} term is still pending
      // (odd passes apply x updates in pairs) -> one-term catch-up from the parity-1 p buffer
      const int64_t m = done ? (done == 1 ? st->conv_iter : -1) : k - 1;
      if (m >= 2 && (m & 1) == 0) for_rows([&](int64_t i) { x[i] = fma(ap, v.p_fix[own + i], x[i]); });
      return;
    }
    // last iteration's r and x updates only: r_m, x_m (paired when m is odd), partial ||r_m||^2
    const bool pair = (k & 1) && k >= 3;
    for_rows([&](int64_t i) {
      const double rk = r_next(own + i);
      if constexpr (RA) ran[own + i] = make_double2(rk, 0.0);
      else rn[own + i] = rk;
      x[i] = pair ? fma(a, po[own + i], fma(ap, pn[own + i], x[i])) : fma(a, po[own + i], x[i]);
      s_rr = fma(rk, rk, s_rr);
    });
    block_partial4(0.0, 0.0, 0.0, s_rr, partials, pstride);
    return;
  }
  const bool pair = (k & 1) != 0;  // odd pass: x += a_{k-2} p_{k-2} + a_{k-1} p_{k-1}; even: x untouched
  auto gather = [&](int32_t c) { return fma(b, po[c], r_next(c)); };
  auto epi = [&](int64_t i, double sum) {
    const int64_t e = own + i;
    const double rk = r_next(e);
    const double pold = po[e];
    const double pk = fma(b, pold, rk);
    if constexpr (RA) {
      st_stream(&ran[e], make_double2(rk, sum));
    } else {
      rn[e] = rk;
      apn[e] = sum;
    }
    if (pair) st_stream(&x[i], fma(a, pold, fma(ap, pn[e], x[i])));  // pn[e] = p_{k-2} until overwritten below
    st_stream(&pn[e], pk);
    s_pap = fma(pk, sum, s_pap);
    s_rap = fma(rk, sum, s_rap);
    s_apap = fma(sum, sum, s_apap);
    s_rr = fma(rk, rk, s_rr);
  };
  if constexpr (FMT == 0) eng::csr_adaptive<IdxT, U, 16>(A, tr, gather, epi);  // = csr_direct on short-row tiles
  else if constexpr (FMT == 1) eng::sell<U, false, 0>(S, tr, gather, epi);
  else if constexpr (FMT == 3) eng::sell<U, false, 1>(S, tr, gather, epi);
  else eng::sell<U, false, 2>(S, tr, gather, epi);
  f1_finish(s_pap, s_rap, s_apap, s_rr, partials, pstride, rc, st, tol);
}

// ---------------------------------------------------------------------------
// Software-pipelined single-reduction pass for short-row SELL-64/d16 and /c8 matrices with
// the interleaved {r, Ap} layout (the stencil path: every slice fits ONE batch, w <= U).
//
// The generic engine walks a slice as load codes -> gather -> sum -> epilogue loads -> stores:
// three dependent memory round trips per slice, ~7 us per slice per wave under load, so the
// pass was latency bound (~9 cycles/row/CU against ~3 of L1 bandwidth).  Here a wave issues,
// at the top of slice s: its own-row operands ({r, Ap}, p_{k-1}, and for paired x updates
// p_{k-2} and x), the NEXT slice's slice pointers and codes, then the gathers of slice s.  The
// arithmetic (sum order, every fma) is exactly the generic kernel's, so results are bitwise
// identical (tests/test_gpu_solver.py).
template <int CM, int U>
__global__ __launch_bounds__(kBS) void k_cg_f1_pipe(SellDev S, F1Vectors v, int64_t own, TileRanges tr,
                                                    double* __restrict__ partials, int pstride,
                                                    CgState* st, double tol, int first,
                                                    int check, int k, RedCtl rc) {
  __shared__ double2 s_dict[CM == 2 ? 256 : 1];
  const F1Scalars sc = f1_scalars(st, tol, first, check);
  if (st->done || sc.conv) {
    f1_finish(0.0, 0.0, 0.0, 0.0, partials, pstride, rc, st, tol);
    return;
  }
  if constexpr (CM == 2) {
    for (int q = threadIdx.x; q < S.ndict; q += kBS) s_dict[q] = S.dict[q];
    __syncthreads();
  }
  const double a = sc.alpha, b = sc.beta, na = -a, ap = st->a_prev;
  const bool pair = (k & 1) != 0;
  const double* __restrict__ po = v.p_old;
  double* __restrict__ pn = v.p_new;
  double* __restrict__ x = v.x;
  const double2* __restrict__ rao = v.ra_old;
  double2* __restrict__ ran = v.ra_new;
  const int lane = threadIdx.x & 63;
  const int64_t wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t n = S.n_rows;
  double s_pap = 0.0, s_rap = 0.0, s_apap = 0.0, s_rr = 0.0;
  using CodeT = typename std::conditional<CM == 2, uint8_t, int16_t>::type;
  const CodeT* __restrict__ codes = CM == 2 ? reinterpret_cast<const CodeT*>(S.codes)
                                            : reinterpret_cast<const CodeT*>(S.dcols);
  const double* __restrict__ svals = S.vals;
  auto slice_of = [&](int64_t t) { return eng::tile_unit(tr, t); };
  eng::TileCursor cur = eng::tile_cursor(tr, wave, kWaves);
  if (cur.t < cur.end) {
    int64_t sl = slice_of(cur.t);
    int64_t base = S.slice_ptr[sl];
    int w = (int)((S.slice_ptr[sl + 1] - base) >> 6);
    CodeT K[U];
    double V[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t j = base + lane + 64 * (u < w ? u : w - 1);
      K[u] = codes[j];
      if constexpr (CM != 2) V[u] = svals[j];
    }
    for (;;) {
      const int64_t i = sl * 64 + lane;
      const bool live = i < n;
      const int64_t e = own + (live ? i : n - 1);
      // own-row operands: independent of the gathers, issued first
      const double2 qo = rao[e];
      const double pold = po[e];
      const double pkm2 = pair ? pn[e] : 0.0;
      const double xo = (pair && live) ? x[i] : 0.0;
      // next slice: pointers + codes (one round trip ahead)
      const int64_t tn = cur.t + cur.step;
      const bool has_next = tn < cur.end;
      int64_t sl_n = sl, base_n = base;
      int w_n = w;
      CodeT Kn[U];
      double Vn[U];
      if (has_next) {
        sl_n = slice_of(tn);
        base_n = S.slice_ptr[sl_n];
        w_n = (int)((S.slice_ptr[sl_n + 1] - base_n) >> 6);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t j = base_n + lane + 64 * (u < w_n ? u : w_n - 1);
          Kn[u] = codes[j];
          if constexpr (CM != 2) Vn[u] = svals[j];
        }
      }
      // this slice: decode, gather p_k = r_k + b p_{k-1} of every column, row sums
      const int32_t rowcol = (int32_t)(own + i);
      int32_t c[U];
      double val[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if constexpr (CM == 2) {
          const double2 q = s_dict[K[u]];
          c[u] = rowcol + (int32_t)__double_as_longlong(q.y);
          val[u] = q.x;
        } else {
          c[u] = rowcol + (int32_t)K[u];
          val[u] = V[u];
        }
      }
      double g[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const double2 q = rao[c[u]];
        g[u] = fma(b, po[c[u]], fma(na, q.y, q.x));
      }
      double sum = 0.0;
#pragma unroll
      for (int u = 0; u < U; ++u) sum = (u < w) ? fma(val[u], g[u], sum) : sum;
      if (live) {
        const double rk = fma(na, qo.y, qo.x);
        const double pk = fma(b, pold, rk);
        st_stream(&ran[e], make_double2(rk, sum));
        if (pair) st_stream(&x[i], fma(a, pold, fma(ap, pkm2, xo)));
        st_stream(&pn[e], pk);
        s_pap = fma(pk, sum, s_pap);
        s_rap = fma(rk, sum, s_rap);
        s_apap = fma(sum, sum, s_apap);
        s_rr = fma(rk, rk, s_rr);
      }
      if (!has_next) break;
      cur.t = tn;
      sl = sl_n;
      base = base_n;
      w = w_n;
      for (int u = 0; u < U; ++u) {  // register renames after full unrolling of the body
        K[u] = Kn[u];
        if constexpr (CM != 2) V[u] = Vn[u];
      }
    }
  }
  f1_finish(s_pap, s_rap, s_apap, s_rr, partials, pstride, rc, st, tol);
}

// loads of data one wave reads once (line-carry operands): optionally non-temporal
__device__ __forceinline__ double ld_once(const double* p, bool nt) { return nt ? __builtin_nontemporal_load(p) : *p; }
__device__ __forceinline__ double2 ld_once(const double2* p, bool nt) {
  typedef double d2v __attribute__((ext_vector_type(2)));
  if (nt) {
    const d2v w = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(p));
    return make_double2(w.x, w.y);
  }
  return *p;
}

// ---------------------------------------------------------------------------
// Line-carry single-reduction pass: SELL-64/d16 or /c8 with the interleaved {r, Ap} layout,
// every slice width <= U, the launch's slices whole grid lines of S slices (structured-grid
// stencils: S = line (2-D) or plane (3-D) length / 64).
//
// In the generic pass every row's vector operands are read three times: as the +L neighbour
// of the row one line up (L = 64 S rows), as the row itself, and as the -L neighbour of the
// row one line down.  Those reads are L rows apart, issued by waves anywhere on the chip, and
// about half of them miss the XCD's L2 (profiles/r1_poisson16384_1gpu_final.md: 16 GB of
// L2->fabric reads per pass against 7.8 GB of model traffic).  Here a wave walks DOWN one
// column of slices (s, s + S, s + 2S, ...): the slice it reads as the +L neighbour at line l
// is its own slice at line l + 1 and the -L neighbour at line l + 2, so p_k of the previous,
// current and next line stay in registers and each row's operands come from memory once.
// The +-1 neighbours are the neighbouring lanes' p_k (a shuffle; lanes 0 / 63 load the row
// across the slice edge with the line's operands).  So in the steady state every operand is
// in registers and the only loads are the prefetches (operands PD lines ahead, codes two):
// gathering +-1 from memory read each vector line twice from the fabric (the line, loaded PD
// steps earlier, had left the XCD's L2) and exposed a memory latency per step.  Offsets that
// are not carried (a run's first / last line, +-N in 3-D) take a slow path that gathers from
// memory.
// Every value is the generic pass's fma sequence; only the blocking of the dot-product
// partials differs (fixed per launch geometry: still bitwise reproducible run to run).
//
// M2 (3-D stencils, plane carry: the carried "line" is a plane, L = N^2): the +-N neighbours
// (offset LO2 = N rows: slices N/64 apart in the same plane, worked at the same step by the
// neighbouring columns' waves on the same XCD) are gathered from the L2 one line ahead, issued
// before the prefetches, and carried into the step as p_k.
// M2 == 1: every wave gathers both.  M2 == 2 (block exchange, LO2 a multiple of 64): the kWaves
// waves of a block walk the columns of kWaves consecutive grid lines of one plane (same x slice),
// so the +-N neighbour of wave w's rows is wave w +- 1's rows: each wave puts the next plane's p_k
// (computed a step ahead from its prefetched operands) in LDS, one barrier per step, and only
// the block's first / last wave gathers its outer +-N rows from memory.  The gathers missed the
// L2 about a third of the time (the neighbouring columns' waves drift apart); this is the
// same p_k values, bit for bit, with 1/kWaves of the gathers.
// (M2: at least 4 waves per SIMD requested -- the +-N rows push the odd pass just past 128 VGPRs)
template <int CM, int U, int PD, bool PAIR, bool GEN, int M2>
__global__ __launch_bounds__(kBS, M2 ? 4 : 1) void k_cg_f1_carry(SellDev S, F1Vectors v, int64_t own, TileRanges tr,
                                                     double* __restrict__ partials, int pstride,
                                                     CgState* st, double tol, int first,
                                                     int check, int32_t LO2, RedCtl rc) {
  __shared__ double2 s_dict[CM >= 2 ? 256 : 1];
  __shared__ double s_far[M2 == 2 ? 2 * kWaves * 64 : 1];  // [step parity][wave][lane]: p_k of the next plane
  const F1Scalars sc = f1_scalars(st, tol, first, check);
  if (st->done || sc.conv) {
    f1_finish(0.0, 0.0, 0.0, 0.0, partials, pstride, rc, st, tol);
    return;
  }
  if constexpr (CM >= 2) {
    for (int q = threadIdx.x; q < S.ndict; q += kBS) s_dict[q] = S.dict[q];
    __syncthreads();
  }
  const double a = sc.alpha, b = sc.beta, na = -a, ap = st->a_prev;
  const double* __restrict__ po = v.p_old;
  double* __restrict__ pn = v.p_new;
  double* __restrict__ x = v.x;
  const double2* __restrict__ rao = v.ra_old;
  double2* __restrict__ ran = v.ra_new;
  const double* __restrict__ svals = S.vals;
  const int lane = threadIdx.x & 63;
  const int64_t SS = tr.strip;              // slices per line
  const int32_t LO = (int32_t)(SS * 64);    // the carried column offset: one line
  const int64_t nl = tr.nt0 / SS;           // lines in the launch
  // XCD-aware wave numbering (speed only): blocks b and b + 8 are observed to share an XCD, so
  // consecutive logical waves -- neighbouring columns of the same lines -- run on one XCD
  const int64_t nb = gridDim.x, blk = blockIdx.x;
  const int64_t lb = (nb % 8 == 0) ? (blk % 8) * (nb / 8) + blk / 8 : blk;
  const int64_t nw = nb * kWaves;
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t gw = lb * kWaves + wv;
  const int64_t runs = nw > SS ? nw / SS : 1;  // line chunks per column
  const int64_t chunk = (nl + runs - 1) / runs;
  // jobs: (column, run of lines).  M2 == 2: one job per block, its waves the columns of kWaves
  // consecutive grid lines of the plane (G slices per grid line)
  const int64_t G = M2 == 2 ? LO2 / 64 : 1;
  const int64_t njobs = M2 == 2 ? SS / kWaves * runs : SS * runs;
  const bool fu_g = M2 != 2 || wv == kWaves - 1, fd_g = M2 != 2 || wv == 0;  // +-LO2 rows from memory
  double s_pap = 0.0, s_rap = 0.0, s_apap = 0.0, s_rr = 0.0;
  // operands of a line (prefetched PD lines ahead): {r_{k-1}, Ap_{k-1}} and p_{k-1}
  struct Raw {
    double2 q;
    double pold;
  };
  // the rows just before / after a slice (the +-1 neighbours of lanes 0 / 63, in the adjacent
  // slice column): wave-uniform addresses through a constant-address-space view -> scalar loads
  // (SGPRs, the lgkm counter: no vector registers, no queueing behind the vector prefetches)
  struct Edge {
    double2 qd, qu;
    double pd, pu;
  };
  // paired x updates (odd passes): p_{k-2} (read before this pass overwrites it) and x
  struct XP {
    double pkm2, xo;
  };
  // a slice's codes: c8 bytes packed four per register (the dictionary is re-read from LDS
  // when the row sums are formed); d16 offsets + values
  struct Codes {
    uint32_t pk[CM >= 2 ? (U + 3) / 4 : 1];
    int16_t d[CM >= 2 ? 1 : U];
    double v[CM >= 2 ? 1 : U];
    int w;
  };
  typedef __attribute__((address_space(4))) const double KD;
  KD* __restrict__ k_ra = (KD*)rao;
  KD* __restrict__ k_po = (KD*)po;
  // p_k = r_k + b p_{k-1} from the old values (the generic pass's gather, bit for bit)
  auto pk_of = [&](double2 q, double pold) { return fma(b, pold, fma(na, q.y, q.x)); };
  // entry u of a slice: {value, column offset from the row's own column}
  auto entry = [&](const Codes& c, int u, double& val) -> int32_t {
    if constexpr (CM >= 2) {
      const double2 q = s_dict[(c.pk[u >> 2] >> (8 * (u & 3))) & 255u];
      val = q.x;
      return (int32_t)__double_as_longlong(q.y);
    } else {
      val = c.v[u];
      return (int32_t)c.d[u];
    }
  };
  // Addressing: every per-line access is a wave-uniform base (SGPRs) + the lane, so the loads
  // are saddr + voffset forms and the per-step scalar work is a few adds.  Loads are never
  // conditional: line indices are clamped to lines that exist (values past the run are unused).
  const int32_t ext32 = (int32_t)v.ext_len;
  constexpr bool ntl = false;  // plain loads (non-temporal measured slower: 281 vs 302 it/s 2-D)
  for (int64_t job = M2 == 2 ? lb : gw; job < njobs; job += M2 == 2 ? nb : nw) {
    int64_t col, l0;
    if constexpr (M2 == 2) {
      const int64_t q = job % (SS / kWaves);
      col = ((q / G) * kWaves + wv) * G + q % G;
      l0 = (job / (SS / kWaves)) * chunk;
    } else {
      col = job % SS;
      l0 = (job / SS) * chunk;
    }
    const int64_t l1 = l0 + chunk < nl ? l0 + chunk : nl;
    if (l0 >= l1) continue;
    const int64_t sl0 = tr.b0 + l0 * SS + col;
    const int32_t e0 = (int32_t)(own + sl0 * 64);  // ext index of lane 0's row at line l0
    const int32_t i0 = (int32_t)(sl0 * 64);        // owned index of the same row
    const int32_t n_run = (int32_t)(l1 - l0);
    // lines (relative to l0) whose operands exist: [-1 if the line before exists, la]
    const int32_t la = (e0 + n_run * LO + 63 < ext32) ? n_run : n_run - 1;
    const bool prev_exists = e0 - LO >= 0;
    auto ebase = [&](int32_t m) { return e0 + m * LO; };             // ext index, line l0 + m
    auto sbase = [&](int32_t m) { return sl0 + (int64_t)m * SS; };   // slice, line l0 + m
    auto load_raw = [&](int32_t m, Raw& r) {
      const int32_t eb = ebase(m < la ? m : la);
      r.q = ld_once(rao + eb + lane, ntl);
      r.pold = ld_once(po + eb + lane, ntl);
    };
    auto load_edge = [&](int32_t m, Edge& r) {  // m <= n_run - 1 (owned lines)
      const int32_t eb = ebase(m);
      const int32_t dn = eb >= 1 ? eb - 1 : 0, up = eb + 64 < ext32 ? eb + 64 : ext32 - 1;
      r.qd = make_double2(k_ra[2 * dn], k_ra[2 * dn + 1]);
      r.pd = k_po[dn];
      r.qu = make_double2(k_ra[2 * up], k_ra[2 * up + 1]);
      r.pu = k_po[up];
    };
    auto edge_ok = [&](int32_t m) {  // lanes 0 / 63: the row across the slice edge exists
      const int32_t eb = ebase(m);
      return lane == 0 ? eb >= 1 : eb + 64 < ext32;
    };
    auto load_xp = [&](int32_t m, XP& r) {  // owned lines only
      if constexpr (PAIR) {
        const int32_t mm = m < n_run - 1 ? m : n_run - 1;
        r.pkm2 = ld_once(pn + ebase(mm) + lane, ntl);
        r.xo = ld_once(x + i0 + mm * LO + lane, ntl);
      }
    };
    auto load_codes = [&](int32_t m, Codes& c) {  // owned lines only
      const int64_t sl = sbase(m < n_run - 1 ? m : n_run - 1);
      const int64_t base = S.slice_ptr[sl];
      c.w = (int)((S.slice_ptr[sl + 1] - base) >> 6);
      if constexpr (CM == 2) {
        const uint8_t* __restrict__ cp = S.codes + base;
#pragma unroll
        for (int q = 0; q < (U + 3) / 4; ++q) c.pk[q] = 0u;
#pragma unroll
        for (int u = 0; u < U; ++u) c.pk[u >> 2] |= (uint32_t)cp[64 * u + lane] << (8 * (u & 3));
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t j = base + lane + 64 * (u < c.w ? u : c.w - 1);
          c.d[u] = S.dcols[j];
          c.v[u] = svals[j];
        }
      }
    };
    // M2: p_k of the rows +-LO2 away (clamped indices; values of rows that do not exist are
    // never used: the matrix has no entry for them)
    struct Far {
      double2 qu, qd;
      double pu, pd;
    };
    auto load_far = [&](int32_t m, Far& f, bool up, bool dn) {  // up / dn wave-uniform
      if constexpr (M2) {
        const int32_t e = ebase(m < n_run - 1 ? m : n_run - 1) + lane;
        const int32_t cu = e + LO2 < ext32 ? e + LO2 : ext32 - 1, cd = e - LO2 >= 0 ? e - LO2 : 0;
        if (up) {
          f.qu = rao[cu];
          f.pu = po[cu];
        }
        if (dn) {
          f.qd = rao[cd];
          f.pd = po[cd];
        }
      }
    };
    // prologue: the line before the run (if it exists), operands of lines 0 .. PD, codes of
    // lines 0, 1, edges + x / p_{k-2} of line 0
    Raw r0, rq[PD];
    load_raw(0, r0);
    bool pv = prev_exists;
    double pr_pk = 0.0;
    {
      const int32_t eb = prev_exists ? e0 - LO : e0;
      pr_pk = pk_of((rao + eb)[lane], (po + eb)[lane]);
    }
    Edge ed0;
    load_edge(0, ed0);
    XP x0{0.0, 0.0};
    load_xp(0, x0);
#pragma unroll
    for (int d = 0; d < PD; ++d) load_raw(1 + d, rq[d]);
    Codes c0, c1;
    load_codes(0, c0);
    load_codes(1, c1);
    double o_rk = fma(na, r0.q.y, r0.q.x);
    double o_pk = fma(b, r0.pold, o_rk);
    double o_pold = r0.pold;
    double o_epk = lane == 0 ? pk_of(ed0.qd, ed0.pd) : pk_of(ed0.qu, ed0.pu);  // lanes 0 / 63
    bool o_eok = edge_ok(0);
    double o_fu = 0.0, o_fd = 0.0;  // M2: p_k of rows +LO2 / -LO2
    if constexpr (M2) {
      Far f0;
      load_far(0, f0, true, true);
      o_fu = pk_of(f0.qu, f0.pu);
      o_fd = pk_of(f0.qd, f0.pd);
    }
    for (int32_t m = 0; m < n_run; ++m) {
      const bool nv = m + 1 <= la;
      // 1. loads, in the order they are waited for: (M2) the next line's +-LO2 rows, its edges
      //    (scalar) and x / p_{k-2}, then the codes of line m + 2 and the operands of line
      //    m + 1 + PD
      Far f1{make_double2(0.0, 0.0), make_double2(0.0, 0.0), 0.0, 0.0};
      load_far(m + 1, f1, fu_g, fd_g);
      Edge ed1;
      load_edge(m + 1 < n_run ? m + 1 : m, ed1);
      XP x1{0.0, 0.0};
      load_xp(m + 1, x1);
      Codes c2;
      load_codes(m + 2, c2);
      Raw rn;
      load_raw(m + 1 + PD, rn);
      // 2. this line's row sums from registers: own row, next / previous line (carried), row
      //    +- 1 (the neighbouring lanes; lanes 0 / 63 the edge rows).  GEN: an entry that is
      //    none of these (other offsets such as +-N in 3-D) sends the wave down a slow path
      //    that redoes the sums with memory gathers; !GEN: the dictionary has no such offset.
      const double n_pk = pk_of(rq[0].q, rq[0].pold);
      if constexpr (M2 == 2) s_far[(((m + 1) & 1) * kWaves + wv) * 64 + lane] = n_pk;
      const double sh_up = __shfl_down(o_pk, 1, 64);
      const double sh_dn = __shfl_up(o_pk, 1, 64);
      const double up_pk = lane == 63 ? o_epk : sh_up;  // row + 1
      const double dn_pk = lane == 0 ? o_epk : sh_dn;   // row - 1
      const bool up_ok = lane < 63 || o_eok, dn_ok = lane > 0 || o_eok;
      // branch-free (selects): per-lane if / else chains become exec-mask branches
      auto reg_value = [&](int32_t off, double& g) -> bool {
        const bool k0 = off == 0, k1 = (off == 1) & up_ok, k2 = (off == -1) & dn_ok;
        const bool k3 = nv & (off == LO), k4 = pv & (off == -LO);
        const bool k5 = M2 && off == LO2, k6 = M2 && off == -LO2;
        // each select pinned in a register (an opaque asm operand): left alone, the optimiser
        // turns the chain into a stack table of the candidates + a computed-address load
        double t = k3 ? n_pk : pr_pk;
        asm volatile("" : "+v"(t));
        if constexpr (M2) {
          t = k5 ? o_fu : t;
          asm volatile("" : "+v"(t));
          t = k6 ? o_fd : t;
          asm volatile("" : "+v"(t));
        }
        t = k2 ? dn_pk : t;
        asm volatile("" : "+v"(t));
        t = k1 ? up_pk : t;
        asm volatile("" : "+v"(t));
        g = k0 ? o_pk : t;
        return k0 | k1 | k2 | k3 | k4 | k5 | k6;
      };
      double sum = 0.0;
      bool all_reg = true;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        double val, g = 0.0;
        const int32_t off = entry(c0, u, val);
        all_reg = (u >= c0.w || reg_value(off, g)) && all_reg;
        sum = (u < c0.w) ? fma(val, g, sum) : sum;
      }
      const int32_t eb = ebase(m);
      if constexpr (GEN) {
        if (__builtin_expect(!__all(all_reg), 0)) {
          const int32_t rowcol = eb + lane;
          sum = 0.0;
#pragma unroll
          for (int u = 0; u < U; ++u) {
            double val, g = 0.0;
            const int32_t off = entry(c0, u, val);
            if (u < c0.w && !reg_value(off, g)) g = pk_of(rao[rowcol + off], po[rowcol + off]);
            sum = (u < c0.w) ? fma(val, g, sum) : sum;
          }
        }
      }
      st_stream(&(ran + eb)[lane], make_double2(o_rk, sum));
      if constexpr (PAIR) st_stream(&(x + i0 + m * LO)[lane], fma(a, o_pold, fma(ap, x0.pkm2, x0.xo)));
      st_stream(&(pn + eb)[lane], o_pk);
      s_pap = fma(o_pk, sum, s_pap);
      s_rap = fma(o_rk, sum, s_rap);
      s_apap = fma(sum, sum, s_apap);
      s_rr = fma(o_rk, o_rk, s_rr);
      // 3. rotate the carried lines and the prefetch pipeline
      pr_pk = o_pk;
      pv = true;
      o_rk = fma(na, rq[0].q.y, rq[0].q.x);
      o_pk = n_pk;
      o_pold = rq[0].pold;
      o_epk = lane == 0 ? pk_of(ed1.qd, ed1.pd) : pk_of(ed1.qu, ed1.pu);
      o_eok = edge_ok(m + 1);
      if constexpr (M2 == 2) {
        // the neighbouring waves' next-plane p_k (written this step; the other parity's slots
        // were last read before this step's barrier by every wave)
        __syncthreads();
        const double* sf = s_far + ((m + 1) & 1) * kWaves * 64 + lane;
        o_fu = fu_g ? pk_of(f1.qu, f1.pu) : sf[(wv < kWaves - 1 ? wv + 1 : wv) * 64];
        o_fd = fd_g ? pk_of(f1.qd, f1.pd) : sf[(wv > 0 ? wv - 1 : wv) * 64];
      } else if constexpr (M2) {
        o_fu = pk_of(f1.qu, f1.pu);
        o_fd = pk_of(f1.qd, f1.pd);
      }
#pragma unroll
      for (int d = 0; d + 1 < PD; ++d) rq[d] = rq[d + 1];
      rq[PD - 1] = rn;
      x0 = x1;
      c0 = c1;
      c1 = c2;
    }
  }
  f1_finish(s_pap, s_rap, s_apap, s_rr, partials, pstride, rc, st, tol);
}

__global__ __launch_bounds__(kReduceBS) void k_cg_reduce_f1(const double* __restrict__ partials, int pstride, int np,
                                                            CgState* __restrict__ st, int mode, int check, int first,
                                                            double tol) {
  __shared__ double sh[4][kReduceBS / 64];
  // 4 x 4 independent loads in flight per thread (a latency-bound single block); fixed order
  double s[4] = {0.0, 0.0, 0.0, 0.0};
  int i = threadIdx.x;
  for (; i + 3 * kReduceBS < np; i += 4 * kReduceBS) {
    double v[4][4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int u = 0; u < 4; ++u) v[q][u] = partials[q * pstride + i + u * kReduceBS];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int u = 0; u < 4; ++u) s[q] += v[q][u];
  }
  for (; i < np; i += kReduceBS) {
#pragma unroll
    for (int q = 0; q < 4; ++q) s[q] += partials[q * pstride + i];
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const double w = eng::wave_sum(s[q]);
    if ((threadIdx.x & 63) == 0) sh[q][threadIdx.x >> 6] = w;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  double tot[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    tot[q] = 0.0;
    for (int w = 0; w < kReduceBS / 64; ++w) tot[q] += sh[q][w];
  }
  if (mode == 2) {  // latch after the final pass's all-reduce
    if (st->done) return;
    st->done = 2;
    st->rr_final = st->red[3];
    st->converged = sqrt(st->red[3]) < tol ? 1 : 0;
    st->conv_iter = st->iter;
    return;
  }
  if (mode == 1) {
    // the final pass: the latch tests exactly as mode 0, then only rr is kept
    if (st->done || (check && (sqrt(st->red[3]) < tol || !isfinite(st->red[3])))) {
      f1_bookkeep(st, tot, check, first, tol);
      return;
    }
    st->red[0] = st->red[1] = st->red[2] = 0.0;
    st->red[3] = tot[3];
    return;
  }
  f1_bookkeep(st, tot, check, first, tol);
}

// ---------------------------------------------------------------------------
// Windowed single-reduction pass for long banded rows (random-SPD family).
//
// The plain pass recomputes p_k = r_k + b p_{k-1} at EVERY gather (one 16-B {r, Ap}
// load + one 8-B p load per nonzero, scattered over a +-band window — for ~1000
// nonzeros per row that L2->L1 gather traffic, not HBM, bounds the kernel).  Here a
// 1024-thread block owns a chunk of 16 consecutive slices (1024 rows), computes
// p_k ONCE for every ext column the chunk touches into an LDS window
// [win_lo, win_hi), and the 16 waves gather from LDS.  Applies when every chunk's
// window fits the LDS budget (band <= ~4-9K at 1-2 blocks per CU).
constexpr int kWinWaves = kWinRows / 64;
constexpr int kWinBS = kWinRows;

template <int CM, int U, bool RA>
__global__ __launch_bounds__(kWinBS) void k_cg_f1_win(SellDev S, F1Vectors v, int64_t own, TileRanges tr,
                                                      const int32_t* __restrict__ win,
                                                      double* __restrict__ partials, int pstride,
                                                      CgState* st, double tol, int first,
                                                      int check, int k, RedCtl rc) {
  extern __shared__ double s_win[];
  __shared__ double s_part[4][kWinWaves];
  const F1Scalars sc = f1_scalars(st, tol, first, check);
  const bool skip = st->done || sc.conv;
  const double a = sc.alpha, b = sc.beta, na = -a, ap = st->a_prev;
  const bool pair = (k & 1) != 0;  // paired x updates (see k_cg_f1)
  const double* __restrict__ ro = v.r_old;
  const double* __restrict__ apo = v.ap_old;
  const double* __restrict__ po = v.p_old;
  double* __restrict__ rn = v.r_new;
  double* __restrict__ apn = v.ap_new;
  double* __restrict__ pn = v.p_new;
  double* __restrict__ x = v.x;
  const double2* __restrict__ rao = v.ra_old;
  double2* __restrict__ ran = v.ra_new;
  auto r_next = [&](int64_t e) -> double {
    if constexpr (RA) {
      const double2 q = rao[e];
      return fma(na, q.y, q.x);
    } else {
      return fma(na, apo[e], ro[e]);
    }
  };
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  double s_pap = 0.0, s_rap = 0.0, s_apap = 0.0, s_rr = 0.0;
  // chunks of kWinWaves slices touched by the (up to two) slice ranges of this launch
  const int64_t c0 = tr.b0 / kWinWaves, n0 = tr.e0 > tr.b0 ? (tr.e0 + kWinWaves - 1) / kWinWaves - c0 : 0;
  const int64_t c1 = tr.b1 / kWinWaves, n1 = tr.e1 > tr.b1 ? (tr.e1 + kWinWaves - 1) / kWinWaves - c1 : 0;
  for (int64_t q = skip ? n0 + n1 : blockIdx.x; q < n0 + n1; q += gridDim.x) {
    const bool r0 = q < n0;
    const int64_t chunk = r0 ? c0 + q : c1 + (q - n0);
    const int64_t lo = win[2 * chunk], hi = win[2 * chunk + 1];
    for (int64_t e = lo + threadIdx.x; e < hi; e += kWinBS) s_win[e - lo] = fma(b, po[e], r_next(e));
    __syncthreads();
    const int64_t sl = chunk * kWinWaves + wave;
    if (sl >= (r0 ? tr.b0 : tr.b1) && sl < (r0 ? tr.e0 : tr.e1)) {
      const double* __restrict__ wl = s_win - lo;
      const double sum = eng::sell_slice<U, false, CM>(S, sl, nullptr, [&](int32_t c) { return wl[c]; });
      const int64_t i = sl * 64 + lane;
      if (i < S.n_rows) {
        const int64_t e = own + i;
        const double rk = r_next(e);
        const double pold = po[e];
        const double pk = wl[e];  // = fma(b, pold, rk), staged above
        if constexpr (RA) {
          ran[e] = make_double2(rk, sum);
        } else {
          rn[e] = rk;
          apn[e] = sum;
        }
        if (pair) x[i] = fma(a, pold, fma(ap, pn[e], x[i]));
        pn[e] = pk;
        s_pap = fma(pk, sum, s_pap);
        s_rap = fma(rk, sum, s_rap);
        s_apap = fma(sum, sum, s_apap);
        s_rr = fma(rk, rk, s_rr);
      }
    }
    __syncthreads();
  }
  s_pap = eng::wave_sum(s_pap);
  s_rap = eng::wave_sum(s_rap);
  s_apap = eng::wave_sum(s_apap);
  s_rr = eng::wave_sum(s_rr);
  if (lane == 0) {
    s_part[0][wave] = s_pap;
    s_part[1][wave] = s_rap;
    s_part[2][wave] = s_apap;
    s_part[3][wave] = s_rr;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < kWinWaves; ++k) t += s_part[threadIdx.x][k];
    if (rc.ngroups > 0) st_wt(&partials[threadIdx.x * pstride + blockIdx.x], t);
    else partials[threadIdx.x * pstride + blockIdx.x] = t;
  }
  if (rc.ngroups > 0) f1_reduce_tail(partials, pstride, rc, st, tol);
}

// per-chunk [lo, hi) ext-column window: one block per chunk, one thread per padded row
__global__ __launch_bounds__(kWinRows) void k_chunk_windows(SellDev S, int32_t* __restrict__ win) {
  __shared__ int s_lo, s_hi;
  if (threadIdx.x == 0) {
    s_lo = 0x7fffffff;
    s_hi = -1;
  }
  __syncthreads();
  const int64_t n = S.n_rows;
  const int64_t i = (int64_t)blockIdx.x * kWinRows + threadIdx.x;
  const int64_t n_pad = (n + 63) / 64 * 64;
  if (i < n_pad) {
    const int64_t sl = i >> 6, l = i & 63;
    const int64_t base = S.slice_ptr[sl], w = (S.slice_ptr[sl + 1] - base) >> 6;
    // the row's own column is always gathered (the epilogue; tail lanes stand in for row n - 1)
    int lo = (int)(S.own_off + (i < n ? i : n - 1)), hi = lo;
    for (int64_t j = 0; j < w; ++j) {
      const int64_t dst = base + 64 * j + l;
      const int c = S.dcols ? (int)(S.own_off + i + S.dcols[dst]) : S.cols[dst];
      lo = min(lo, c);
      hi = max(hi, c);
    }
    atomicMin(&s_lo, lo);
    atomicMax(&s_hi, hi);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    win[2 * blockIdx.x] = s_lo;
    win[2 * blockIdx.x + 1] = s_hi + 1;
  }
}

__global__ void k_pack_pairs(const double* __restrict__ a, double2* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = make_double2(a[i], 0.0);
}

}  // namespace

int64_t win_chunks(const TileRanges& tr) {
  const int64_t n0 = tr.e0 > tr.b0 ? (tr.e0 + kWinWaves - 1) / kWinWaves - tr.b0 / kWinWaves : 0;
  const int64_t n1 = tr.e1 > tr.b1 ? (tr.e1 + kWinWaves - 1) / kWinWaves - tr.b1 / kWinWaves : 0;
  return n0 + n1;
}

void chunk_windows(const SellDev& S, int32_t* win, hipStream_t stream) {
  const int64_t nch = (S.n_rows + kWinRows - 1) / kWinRows;
  if (nch == 0) return;
  MCG_CHECK(nch < ((int64_t)1 << 31), "too many window chunks");
  hipLaunchKernelGGL(k_chunk_windows, dim3((unsigned)nch), dim3(kWinRows), 0, stream, S, win);
  MCG_HIP(hipGetLastError(), "kernel launch failed(chunk_windows)");
}

// raise the dynamic-LDS limit of every windowed instantiation (setup time, not per launch).  The
// attribute is per function and process-wide: solvers of several ranks in one process (LocalComm
// threads) prepare different widths, so the limit only ever grows (a rank must never lower it
// under another rank's launch).
void cg_fused1_win_prepare(int win_doubles) {
  const int lds = win_doubles * (int)sizeof(double);
  MCG_CHECK((size_t)lds <= kWinMaxLds, "window exceeds the LDS budget");
  static std::mutex mu;
  static int prepared = 0;
  std::lock_guard<std::mutex> lk(mu);
  if (lds <= prepared) return;
  prepared = lds;
  const void* fns[] = {
      reinterpret_cast<const void*>(&k_cg_f1_win<0, 4, false>), reinterpret_cast<const void*>(&k_cg_f1_win<0, 6, false>),
      reinterpret_cast<const void*>(&k_cg_f1_win<0, 8, false>), reinterpret_cast<const void*>(&k_cg_f1_win<0, 4, true>),
      reinterpret_cast<const void*>(&k_cg_f1_win<0, 6, true>),  reinterpret_cast<const void*>(&k_cg_f1_win<0, 8, true>),
      reinterpret_cast<const void*>(&k_cg_f1_win<1, 4, false>), reinterpret_cast<const void*>(&k_cg_f1_win<1, 6, false>),
      reinterpret_cast<const void*>(&k_cg_f1_win<1, 8, false>), reinterpret_cast<const void*>(&k_cg_f1_win<1, 4, true>),
      reinterpret_cast<const void*>(&k_cg_f1_win<1, 6, true>),  reinterpret_cast<const void*>(&k_cg_f1_win<1, 8, true>)};
  for (const void* f : fns)
    MCG_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds), "kernel attribute failed(LDS)");
}

void cg_fused1_win(int cm, int param, const SellDev& S, const F1Vectors& v, int64_t own_off, const TileRanges& tr,
                   const int32_t* win, int win_doubles, double* partials, int pstride, int grid, CgState* st,
                   double tol, int first, int check, int k, hipStream_t stream, const RedCtl& rc) {
  if (tr.ntiles == 0 || grid == 0) return;
  const size_t lds = (size_t)win_doubles * sizeof(double);
  MCG_CHECK(lds <= kWinMaxLds, "window exceeds the LDS budget");
  MCG_CHECK(cm == 0 || cm == 1, "windowed pass supports SELL-64 and SELL-64/d16");
  MCG_CHECK(rc.ngroups == 0 || (rc.base % kRedGroup == 0 && rc.cnt && rc.lvl2), "in-kernel reduction: bad control block");
#define MCG_W(CM, U, RA)                                                                                      \
  hipLaunchKernelGGL((k_cg_f1_win<CM, U, RA>), dim3(grid), dim3(kWinBS), lds, stream, S, v, own_off, tr, win, \
                     partials, pstride, st, tol, first, check, k, rc)
#define MCG_WU(CM, RA) \
  do { if (param <= 4) MCG_W(CM, 4, RA); else if (param <= 6) MCG_W(CM, 6, RA); else MCG_W(CM, 8, RA); } while (0)
  const bool ra = v.ra_old != nullptr;
  if (cm == 0) { if (ra) MCG_WU(0, true); else MCG_WU(0, false); }
  else { if (ra) MCG_WU(1, true); else MCG_WU(1, false); }
#undef MCG_WU
#undef MCG_W
  MCG_HIP(hipGetLastError(), "compute mv failed(Ap)");
}

bool carry_block_exchange_ok(int param, int32_t lo2, int64_t strip) {
  return lo2 > 0 && lo2 % 64 == 0 && (param == 7 || param == 8) && strip % (kWaves * (lo2 / 64)) == 0;
}

void cg_fused1_carry(int cm, int param, int depth, bool general, int32_t lo2, bool block_exchange, const SellDev& S,
                     const F1Vectors& v, int64_t own_off, const TileRanges& tr, double* partials, int pstride,
                     int grid, CgState* st, double tol, int first, int check, int k, hipStream_t stream,
                     const RedCtl& rc) {
  if (tr.ntiles == 0 || grid == 0) return;
  MCG_CHECK(tr.strip > 0 && tr.nt0 == tr.ntiles && tr.nt0 % tr.strip == 0, "line-carry pass needs whole grid lines");
  MCG_CHECK(v.ra_old != nullptr && cm >= 1 && cm <= 2 && param >= 4 && param <= 8,
            "line-carry pass needs SELL-64 d16/c8 with interleaved pairs");
  MCG_CHECK(depth == 1 || depth == 3, "line-carry prefetch depth must be 1 (3-D) or 3 (2-D)");
  MCG_CHECK(rc.ngroups == 0 || (rc.base % kRedGroup == 0 && rc.cnt && rc.lvl2), "in-kernel reduction: bad control block");
  MCG_CHECK(general || cm >= 2, "the specialised line-carry pass needs the c8 dictionary");
  MCG_CHECK(lo2 == 0 || (cm == 2 && !general && lo2 > 1), "the +-LO2 carry needs the specialised c8 pass");
  MCG_CHECK(!block_exchange || carry_block_exchange_ok(param, lo2, tr.strip),
            "plane-carry block exchange needs +-LO2 whole slices, kWaves | grid lines per plane, 7-8 entries per row");
  const bool pair = (k & 1) != 0;
#define MCG_C(CM, U, PD, PAIR, GEN, M2)                                                                         \
  hipLaunchKernelGGL((k_cg_f1_carry<CM, U, PD, PAIR, GEN, M2>), dim3(grid), dim3(kBS), 0, stream, S, v, own_off, \
                     tr, partials, pstride, st, tol, first, check, lo2, rc)
#define MCG_CP(CM, U, PD, GEN, M2)                     \
  do {                                                 \
    if (pair) MCG_C(CM, U, PD, true, GEN, M2);         \
    else MCG_C(CM, U, PD, false, GEN, M2);             \
  } while (0)
#define MCG_CD(CM, U, GEN, M2)                         \
  do {                                                 \
    if (depth == 1) MCG_CP(CM, U, 1, GEN, M2);         \
    else MCG_CP(CM, U, 3, GEN, M2);                    \
  } while (0)
#define MCG_CU(CM, GEN, M2)                       \
  do {                                            \
    if (param == 4) MCG_CD(CM, 4, GEN, M2);       \
    else if (param == 5) MCG_CD(CM, 5, GEN, M2);  \
    else if (param == 6) MCG_CD(CM, 6, GEN, M2);  \
    else if (param == 7) MCG_CD(CM, 7, GEN, M2);  \
    else MCG_CD(CM, 8, GEN, M2);                  \
  } while (0)
  if (cm == 2) {
    if (general) MCG_CU(2, true, 0);
    else if (lo2 > 0 && block_exchange) {
      if (param == 7) MCG_CD(2, 7, false, 2);
      else MCG_CD(2, 8, false, 2);
    } else if (lo2 > 0) MCG_CU(2, false, 1);
    else MCG_CU(2, false, 0);
  } else {
    MCG_CU(1, true, 0);
  }
#undef MCG_CU
#undef MCG_CD
#undef MCG_CP
#undef MCG_C
  MCG_HIP(hipGetLastError(), "compute mv failed(Ap)");
}

void pack_pairs(const double* a, double2* out, int64_t n, hipStream_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_pack_pairs, dim3(grid_for(n, 256, 4)), dim3(256), 0, stream, a, out, n);
  MCG_HIP(hipGetLastError(), "vector copy failed(r)");
}

template <typename IdxT>
void cg_fused1(int fmt, int param, const CsrDev<IdxT>& A, const SellDev& S, const F1Vectors& v, int64_t own_off,
               const TileRanges& tr, double* partials, int pstride, int grid, CgState* st, double tol,
               int first, int check, int final_mode, int k, hipStream_t stream, bool pipe, const RedCtl& rc) {
  if (tr.ntiles == 0 || grid == 0) return;
  MCG_CHECK(rc.ngroups == 0 || (!final_mode && rc.base % kRedGroup == 0 && rc.cnt && rc.lvl2),
            "in-kernel reduction: bad control block");
#define MCG_F1(F, U, RA)                                                                                   \
  hipLaunchKernelGGL((k_cg_f1<F, IdxT, U, RA>), dim3(grid), dim3(kBS), 0, stream, A, S, v, own_off, tr, \
                     partials, pstride, st, tol, first, check, final_mode, k, rc)
// SELL engines take U = 4..8 (U = the slice width avoids clamped duplicate gathers)
#define MCG_F1U(F, RA)                                  \
  do {                                                  \
    if (param <= 4) MCG_F1(F, 4, RA);                   \
    else if (param == 5 && F >= 3) MCG_F1(F, 5, RA);    \
    else if (param <= 6) MCG_F1(F, 6, RA);              \
    else if (param == 7 && F >= 3) MCG_F1(F, 7, RA);    \
    else MCG_F1(F, 8, RA);                              \
  } while (0)
  const bool ra = v.ra_old != nullptr;
  MCG_CHECK(!ra || fmt == 1 || fmt == 3 || fmt == 4, "interleaved r/Ap layout needs a SELL format");
  if (pipe && !final_mode && ra && (fmt == 3 || fmt == 4) && param >= 4 && param <= 8) {
#define MCG_PIPE(CM, U)                                                                                        \
  hipLaunchKernelGGL((k_cg_f1_pipe<CM, U>), dim3(grid), dim3(kBS), 0, stream, S, v, own_off, tr, partials, pstride, \
                     st, tol, first, check, k, rc)
#define MCG_PIPEU(CM)                          \
  do {                                         \
    if (param == 4) MCG_PIPE(CM, 4);           \
    else if (param == 5) MCG_PIPE(CM, 5);      \
    else if (param == 6) MCG_PIPE(CM, 6);      \
    else if (param == 7) MCG_PIPE(CM, 7);      \
    else MCG_PIPE(CM, 8);                      \
  } while (0)
    if (fmt == 4) MCG_PIPEU(2);
    else MCG_PIPEU(1);
#undef MCG_PIPEU
#undef MCG_PIPE
    MCG_HIP(hipGetLastError(), "compute mv failed(Ap)");
    return;
  }
  if (fmt == 0) MCG_F1U(0, false);
  else if (fmt == 1) { if (ra) MCG_F1U(1, true); else MCG_F1U(1, false); }
  else if (fmt == 3) { if (ra) MCG_F1U(3, true); else MCG_F1U(3, false); }
  else { if (ra) MCG_F1U(4, true); else MCG_F1U(4, false); }
#undef MCG_F1U
#undef MCG_F1
  MCG_HIP(hipGetLastError(), "compute mv failed(Ap)");
}
template void cg_fused1<int32_t>(int, int, const CsrDev<int32_t>&, const SellDev&, const F1Vectors&, int64_t,
                                 const TileRanges&, double*, int, int, CgState*, double, int, int, int, int,
                                 hipStream_t, bool, const RedCtl&);
template void cg_fused1<int64_t>(int, int, const CsrDev<int64_t>&, const SellDev&, const F1Vectors&, int64_t,
                                 const TileRanges&, double*, int, int, CgState*, double, int, int, int, int,
                                 hipStream_t, bool, const RedCtl&);

void cg_reduce_f1(const double* partials, int pstride, int np, CgState* st, int mode, int check, int first,
                  double tol, hipStream_t stream) {
  hipLaunchKernelGGL(k_cg_reduce_f1, dim3(1), dim3(kReduceBS), 0, stream, partials, pstride, np, st, mode, check,
                     first, tol);
  MCG_HIP(hipGetLastError(), "compute dot failed(tmp)");
}

}  // namespace kern
}  // namespace mcg
