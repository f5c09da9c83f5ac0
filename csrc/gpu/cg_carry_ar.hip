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
// kernel with the same recomputation.
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

#ifndef MCG_EDGE_BRANCHLESS
#define MCG_EDGE_BRANCHLESS 1
#endif

// waves per SIMD the diav lean-only kernels are built for (their coefficient chains need the VGPRs)
constexpr int kLeanV = 3;

__device__ __forceinline__ double ld_once(const double* p, bool nt) { return nt ? __builtin_nontemporal_load(p) : *p; }

// a slice's codes for one lane: c4 nibbles / c8 bytes packed into 32-bit registers (entry u at
// bit CB * u); w = the slice's width
template <int CM, int U>
struct ArCodes {
  static constexpr int CB = CM >= 3 ? 4 : 8;
  uint32_t pk[(U * CB + 31) / 32];
  int w;
};

// SELL-64/diav (variable coefficients): the row's five coefficients in column order (north, west,
// diagonal, east, south), loaded per line instead of decoded
template <int U>
struct ArCodes<5, U> {
  double k[5];
  int w = 5;
};
// 3-D (CM 6): down, south, west, diagonal, east, north, up
template <int U>
struct ArCodes<6, U> {
  double k[7];
  int w = 7;
};

// codes of slice row `lane` from its first slot `base` (slots, multiple of 64) and width w
template <int CM, int U>
__device__ __forceinline__ void ar_load_codes(const SellDev& S, int64_t base, int w, int lane, ArCodes<CM, U>& c) {
  constexpr int CB = ArCodes<CM, U>::CB;
  c.w = w;
#pragma unroll
  for (int q = 0; q < (U * CB + 31) / 32; ++q) c.pk[q] = 0u;
  static_assert(CM == 2, "per-entry codes: SELL-64/c8");
  const uint8_t* __restrict__ cp = S.codes + base;
#pragma unroll
  for (int u = 0; u < U; ++u) c.pk[(u * CB) >> 5] |= (uint32_t)cp[64 * u + lane] << ((u * CB) & 31);
}

// SELL-64/dia4: the U value indices of slice row `lane` (slot u at bit 4 u); sp = the slice's 32 U bytes
template <int U>
__device__ __forceinline__ void ar_load_dia(const uint8_t* __restrict__ sp, int lane, ArCodes<4, U>& c) {
  static_assert(U == 5 || U == 7, "dia4: the five (2-D) or seven (3-D) canonical offsets");
  c.w = U;
  const int sh = (lane & 1) * 4;
  uint32_t pk = 0u;
#pragma unroll
  for (int u = 0; u < U; ++u) pk |= (((uint32_t)sp[32 * u + (lane >> 1)] >> sh) & 15u) << (4 * u);
  c.pk[0] = pk;
}

template <int CM, int U>
__device__ __forceinline__ int32_t ar_entry(const double2* dict, const ArCodes<CM, U>& c, int u, double& val) {
  constexpr int CB = ArCodes<CM, U>::CB;
  const double2 q = dict[(c.pk[(u * CB) >> 5] >> ((u * CB) & 31)) & ((1u << CB) - 1u)];
  val = q.x;
  return (int32_t)__double_as_longlong(q.y);
}

// whole-wave lane shifts through DPP (no LDS, so no lgkmcnt wait): value of lane + 1 / lane - 1
__device__ __forceinline__ double lane_up(double v) {  // wave_shl:1
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x130, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x130, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double lane_dn(double v) {  // wave_shr:1
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x138, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x138, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}

// lane + 1 / lane - 1 with lane 63 / lane 0 (no source lane) keeping `edge`: the DPP move's old
// value is the select (a stencil's row just across the slice edge), so no compare or cndmask
__device__ __forceinline__ double lane_up_or(double v, double edge) {  // wave_shl:1
  const int lo = __builtin_amdgcn_update_dpp(__double2loint(edge), __double2loint(v), 0x130, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(__double2hiint(edge), __double2hiint(v), 0x130, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double lane_dn_or(double v, double edge) {  // wave_shr:1
  const int lo = __builtin_amdgcn_update_dpp(__double2loint(edge), __double2loint(v), 0x138, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(__double2hiint(edge), __double2hiint(v), 0x138, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}

// a wave-uniform value in scalar registers (the compiler cannot prove a loaded value uniform)
__device__ __forceinline__ uint64_t uni_u64(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ double uni_d(double v) {
  return __longlong_as_double((long long)uni_u64((uint64_t)__double_as_longlong(v)));
}
// global-memory accesses at a kernel-wide base plus a 32-bit byte offset (global_load / store's
// saddr + voffset form: the base stays in scalar registers, one 32-bit add per address)
typedef __attribute__((address_space(1))) double g_double;
typedef __attribute__((address_space(1))) char g_char;
__device__ __forceinline__ double g_ld(const double* base, uint32_t bo) {
  return *(const g_double*)((const g_char*)(const g_double*)base + bo);
}
__device__ __forceinline__ void g_st(double* base, uint32_t bo, double v) { *(g_double*)((g_char*)(g_double*)base + bo) = v; }
__device__ __forceinline__ void g_st_nt(double* base, uint32_t bo, double v) {
  if constexpr (MCG_NT_STORES) __builtin_nontemporal_store(v, (g_double*)((g_char*)(g_double*)base + bo));
  else *(g_double*)((g_char*)(g_double*)base + bo) = v;
}
// In-kernel halo (F1Vectors::pull_*): a neighbour's rows are loaded at system scope (sc0 sc1: past
// this device's L2, so a line another device or process rewrote since is never served stale), and the
// rank's own first / last line is stored the same way (written through to memory, where the
// neighbour's next pass reads it once the all-reduce between the two passes has completed)
typedef __attribute__((address_space(1))) unsigned long long g_u64;
__device__ __forceinline__ double ld_sys(const double* base, uint32_t bo) {
  g_u64* p = (g_u64*)((g_char*)(g_double*)const_cast<double*>(base) + bo);
  return __longlong_as_double((long long)__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
}
__device__ __forceinline__ void st_sys(double* base, uint32_t bo, double v) {
  g_u64* p = (g_u64*)((g_char*)(g_double*)base + bo);
  __hip_atomic_store(p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// a pulled ghost line's loads: side 0 = a local line, 1 / 2 = the lo / hi neighbour's rows
struct PullBases {
  const double *p[2], *ap[2];
  int pub;
  __device__ __forceinline__ void at(const F1Vectors& v, int64_t rb) {
    for (int s = 0; s < 2; ++s) {
      p[s] = v.pull_p[s] ? v.pull_p[s] + rb : nullptr;
      ap[s] = v.pull_ap[s] ? v.pull_ap[s] + rb : nullptr;
    }
    pub = v.pull_pub;
  }
  // line l (rank-relative, wave-uniform) of a rank of nl lines
  __device__ __forceinline__ int side(int64_t l, int64_t nl) const {
    return (p[0] != nullptr && l == -1) ? 1 : ((p[1] != nullptr && l == nl) ? 2 : 0);
  }
  __device__ __forceinline__ double ld_p(int s, const double* local, uint32_t o) const {
    return s == 0 ? g_ld(local, o) : ld_sys(p[s - 1], o);
  }
  __device__ __forceinline__ double ld_ap(int s, const double* local, uint32_t o) const {
    return s == 0 ? g_ld(local, o) : ld_sys(ap[s - 1], o);
  }
  // the first / last line's p_k or Ap_k (CL steps only)
  __device__ __forceinline__ void st_pub(bool boundary, double* base, uint32_t o, double v, bool nt) const {
    if (pub && boundary) st_sys(base, o, v);
    else if (nt) g_st_nt(base, o, v);
    else g_st(base, o, v);
  }
};

// Lean-run eligibility of one slice column's run [l0, l1) of a rank's nl lines (ss slices per
// line): lines l0 - 1 .. l1 carry uniform patterns (one, B, for the inner lines; the rank's first
// / last line their own, A / C, with B's slice-edge bits), and a column at a grid line's start /
// end has the absent edge entry.  UNI: the caller is a wave (one run; values made wave-uniform).
template <bool UNI>
__device__ __forceinline__ bool lean_eligible(const uint64_t* __restrict__ dpat, int64_t l0, int64_t l1, int64_t nl,
                                              int64_t ss, int64_t col, int64_t ext_len, uint32_t& WA, uint32_t& WB,
                                              uint32_t& WC, int big = 0) {
  auto ld = [&](int64_t i) { return UNI ? uni_u64(dpat[i]) : dpat[i]; };
  WA = WB = WC = 0u;
  // 32-bit byte offsets: from kernel-wide bases (ext_len < 2^29), or past that (BIG kernels) from
  // per-run bases (big = 1: lines / planes -3 .. the run's end + 4 inside 4 GiB) or bases moved
  // along the run (big = 2, the 3-D loop)
  if (dpat == nullptr || l1 - l0 < 3 || nl < 4) return false;
  if (ext_len >= ((int64_t)1 << 29) &&
      (big == 0 || ext_len >= ((int64_t)1 << 31) || (big == 1 && (l1 - l0 + 8) * ss * 512 >= ((int64_t)1 << 32))))
    return false;
  const int64_t ia = l0 - 1 > 1 ? l0 - 1 : 1, ib = l1 < nl - 2 ? l1 : nl - 2;  // inner lines of l0 - 1 .. l1
  const uint64_t wb = ld(ia * ss + col);
  WB = (uint32_t)wb;
  bool go = (WB >> 31) != 0u && (int64_t)(wb >> 32) >= ib - ia + 1;
  if (l0 <= 1) {
    WA = (uint32_t)ld(col);
    go = go && (WA >> 31) != 0u && ((WA ^ WB) & (3u << 28)) == 0u;
  }
  if (l1 >= nl - 1) {
    WC = (uint32_t)ld((nl - 1) * ss + col);
    go = go && (WC >> 31) != 0u && ((WC ^ WB) & (3u << 28)) == 0u;
  }
  return go && (col != 0 || ((WB >> 28) & 1u)) && (col != ss - 1 || ((WB >> 29) & 1u));
}

// The 2-D carry's job decomposition: job -> (slice column, run of lines [l0, l1)) for a launch of nw
// waves over nl lines of ss slices.  Returns the number of jobs.
__host__ __device__ __forceinline__ int64_t carry_jobs(int64_t nw, int64_t ss, int64_t nl, int64_t& runs,
                                                       int64_t& chunk) {
  runs = nw > ss ? nw / ss : 1;
  chunk = (nl + runs - 1) / runs;
  return ss * runs;
}
__host__ __device__ __forceinline__ void carry_run(int64_t job, int64_t ss, int64_t nl, int64_t chunk, int64_t& col,
                                                   int64_t& l0, int64_t& l1) {
  col = job % ss;
  l0 = (job / ss) * chunk;
  l1 = l0 + chunk < nl ? l0 + chunk : nl;
}

__global__ __launch_bounds__(256) void k_pull_probe(const double* __restrict__ base, int64_t n, double* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = ld_sys(base + i, 0u);
}

// per-slice metadata for the carry's codes loads: first slot / 64 (28 bits) | width << 28
__global__ void k_slice_meta(const int64_t* __restrict__ slice_ptr, int64_t ns, uint32_t* __restrict__ meta) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < ns; s += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = slice_ptr[s];
    meta[s] = (uint32_t)(b >> 6) | ((uint32_t)((slice_ptr[s + 1] - b) >> 6) << 28);
  }
}

// LEAN > 0: lean-only kernel (every run checked at setup) for at least LEAN waves per SIMD
// BIG (lean kernels): the rank's vectors exceed 2^29 doubles, so each run re-bases its global pointers
// (64-bit, scalar registers) at its own first lines and keeps 32-bit byte offsets inside the run
// EP (lean dia4 kernels): packed edges -- the three values a slice-edge lane needs per line (its
// neighbour row's r_{k-1}, Ap_{k-1}, p_{k-1}) arrive in ONE load per line, lanes 0 / 15 / 7 fetching
// lane 0's and lanes 63 / 48 / 56 lane 63's, and move to lanes 0 / 63 by row_mirror /
// row_half_mirror DPP (one move serves both ends).  A line in flight then holds 2 instead of 6
// VGPRs of edges, which buys a wave per SIMD (LEAN 5) or a line of prefetch depth
template <int CM, int U, int QD, bool PAIR, bool P3, int UN = 1, int LEAN = 0, bool BIG = false, bool EP = false>
__global__ __launch_bounds__(kBS, (LEAN > 0 ? LEAN : 4)) void k_cg_carry_ar(SellDev S, F1Vectors v, int64_t own, TileRanges tr,
                                                     double* __restrict__ partials, int pstride, CgState* st,
                                                     double tol, int first, int check, RedCtl rc) {
  __shared__ double2 s_dict[CM >= 4 ? 1 : 256];
  __shared__ double s_val[16];  // dia4 values
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
  const int64_t nb = gridDim.x, blk = blockIdx.x;
  const int64_t lb = (nb % 8 == 0) ? (blk % 8) * (nb / 8) + blk / 8 : blk;  // XCD-aware (k_cg_f1_carry)
  const int64_t nw = nb * kWaves;
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t gw = lb * kWaves + wv;
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
  for (int64_t job = gw; job < njobs; job += nw) {
    int64_t col, l0, l1;
    carry_run(job, SS, nl, chunk, col, l0, l1);
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
      const bool elig = lean_eligible<true>(S.dpat, l0, l1, nl, SS, col, v.ext_len, WA, WB, WC,
                                            (BIG || tr.lean_split != 0) ? 1 : 0);
      if (tr.lean_split == 1 && !elig) continue;  // the generic launch takes this run
      if (tr.lean_split == 2 && elig) continue;   // the lean launch took it
      if constexpr (LEAN > 0) {
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
            q.r = g_ld((j >= 0 && j < n_run) ? (const double*)pn_ : ro_, o);
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
          auto edge_at = [&](int32_t j) {
            Edge q;
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
          auto rghost = [&](int32_t j, const Raw& q) { return fma(nbp, g_ld(pn_, line_ofs(j) + l8), q.p); };
          auto is_ghost = [&](int32_t j) { return apx_o != nullptr && (l0 + j == -1 || l0 + j == nl) && j >= jlo && j <= jhi; };
          auto raw_un = [&](int32_t j) {  // a line of the run or below it, inside the rank
            Raw q;
            const uint32_t o = line_ofs(j) + l8;
            q.r = g_ld(j < n_run ? (const double*)pn_ : ro_, o);
            q.p = g_ld(po_, o);
            return q;
          };
          auto edge_un = [&](int32_t j) {
            Edge q;
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
            pr_pk = fma(b, rm1.p, fma(na, stencil_u(Vm, rm1.p, ez(e_p(edm1)), rm2.p, r0.p), rm1.r));
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
          double o_epk = epk(ed0);
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
              rk1 = fma(na, t, m + 1 < n_run ? fma(nbp, q[0].r, q[0].p) : q[0].r);
              pk1 = fma(b, q[0].p, rk1);
            } else if (CL && next == 2) {
              rk1 = fma(na, ap_gh(m + 1), rghost(m + 1, q[0]));
              pk1 = fma(b, q[0].p, rk1);
              if (pl.p[1] != nullptr) g_st(const_cast<double*>(po_), line_ofs(m + 1) + l8, q[0].p);
            }
            const double sum = stencil_u(Vs, o_pk, o_epk, pr_pk, pk1);
            const uint32_t ob = line_ofs(m);
            const double rr = fma(-b, o_pold, o_pk);
            if (m == 0 || m == n_run - 1 || alt_edge(m)) g_st_nt(rn_, ob + l8, rr);
            if (edge_lane) {
              const uint32_t sb = cb0 + (uint32_t)m * SB + (hi ? 16u : 8u);  // 2 s, 2 s + 1
              g_st(ren, sb, rr);
              g_st(en, sb, sum);
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
            o_epk = epk(e[0]);
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
        q.r = g_ld((j >= 0 && j < n_run) ? (const double*)pn_ : ro_, o);
        q.p = pl.ld_p(pl.side(l0 + jj, nl), po_, o);
        return q;
      };
      auto ap_gh = [&](int32_t j) { return pl.ld_ap(pl.side(l0 + j, nl), apo_, line_ofs(j) + l8); };
      auto edge_at = [&](int32_t j) {
        Edge q;
        const uint32_t c = cb0 + (uint32_t)rc_(j) * SB + oc;
        q.r = g_ld(reo, c);
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
      auto rghost = [&](int32_t j, const Raw& q) { return fma(nbp, g_ld(pn_, line_ofs(j) + l8), q.p); };
      auto is_ghost = [&](int32_t j) { return apx_o != nullptr && (l0 + j == -1 || l0 + j == nl) && j >= jlo && j <= jhi; };
      auto raw_un = [&](int32_t j) {
        Raw q;
        const uint32_t o = line_ofs(j) + l8;
        q.r = g_ld(j < n_run ? (const double*)pn_ : ro_, o);
        q.p = g_ld(po_, o);
        return q;
      };
      auto edge_un = [&](int32_t j) {
        Edge q;
        const uint32_t c = cb0 + (uint32_t)j * SB + oc;
        q.r = g_ld(reo, c);
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
      auto epk = [&](const Edge& q) { return fma(b, q.p, fma(na, q.a, q.r)); };
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
        pr_pk = fma(b, rm1.p, fma(na, stencil_v(mkv(cm1, cm2.s), rm1.p, edm1.p, rm2.p, r0.p), rm1.r));
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
          rk1 = fma(na, t, m + 1 < n_run ? fma(nbp, q[0].r, q[0].p) : q[0].r);
          pk1 = fma(b, q[0].p, rk1);
        } else if (CL && next == 2) {
          rk1 = fma(na, ap_gh(m + 1), rghost(m + 1, q[0]));
          pk1 = fma(b, q[0].p, rk1);
          if (pl.p[1] != nullptr) g_st(const_cast<double*>(po_), line_ofs(m + 1) + l8, q[0].p);
        }
        const double sum = stencil_v(Vs, o_pk, o_epk, pr_pk, pk1);
        const uint32_t ob = line_ofs(m);
        const double rr = fma(-b, o_pold, o_pk);
        if (m == 0 || m == n_run - 1) g_st_nt(rn_, ob + l8, rr);
        if (edge_lane) {
          const uint32_t sb = cb0 + (uint32_t)m * SB + (hi ? 16u : 8u);
          g_st(ren, sb, rr);
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
      continue;
    }
    if constexpr (LEAN == 0) {
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
    auto load_raw = [&](int32_t j, Raw& q) {
      const int32_t e = ebase(j) + lane;
      q.r = ld_once((inrun(j) ? (const double*)pn : ro) + e, ntl);
      q.p = ld_once(po + e, ntl);
    };
    auto rof = [&](int32_t j, const Raw& q) { return inrun(j) ? fma(nbp, q.r, q.p) : q.r; };
    auto load_edge = [&](int32_t j, Edge& q) {
      const int32_t e = ebase(j);
      const int64_t s = oline(j) * SS + col;
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
    // ghost line: Ap_{k-1} exchanged by the halo (multi-rank only)
    auto ghost = [&](int32_t j) { return apx_o != nullptr && (l0 + j == -1 || l0 + j == nl) && j >= jmin && j <= jmax; };
    // r_{k-1} of a ghost line (P > 1).  P3: recovered like an own line -- no wave writes the ghost
    // rows, and the halo delivered p_{k-2} into p_new's ghost rows two iterations ago -- so the halo
    // carries {Ap, p} and not r (one extra load, at a run's outer step only)
    auto rghost = [&](int32_t j, const Raw& q) { return P3 && !first ? fma(nbp, pn[ebase(j) + lane], q.p) : q.r; };

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
      const double t = apx_o[ebase(-1) + lane];
      pr_pk = fma(b, rm1.p, fma(na, t, rghost(-1, rm1)));
    }
    double o_pold = r0.p, o_pm2 = r0.r, o_rk, o_pk;
    {
      const double t = stencil(c0, r0.p, edge_p(ed0), rm1.p, rq[0].p);
      o_rk = fma(na, t, rof(0, r0));
      o_pk = fma(b, r0.p, o_rk);
    }
    double o_epk = edge_pk(ed0);
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
        const double t = apx_o[ebase(m + 1) + lane];
        rk1 = fma(na, t, rghost(m + 1, rq[0]));
        pk1 = fma(b, rq[0].p, rk1);
      }
      // 3. Ap_k of line m, stores, partials
      const double sum = stencil(c0, o_pk, o_epk, pr_pk, pk1);
      const int32_t eb = e0 + m * LO;
      const int64_t s = (l0 + m) * SS + col;
      if constexpr (P3) {
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
      st_stream(&(pn + eb)[lane], o_pk);
      if (lane == 0 || lane == 63) en[2 * s + (lane == 63 ? 1 : 0)] = sum;
      if (apx_n != nullptr && (l0 + m == 0 || l0 + m == nl - 1)) apx_n[eb + lane] = sum;
      s_pap = fma(o_pk, sum, s_pap);
      s_rap = fma(o_rk, sum, s_rap);
      s_apap = fma(sum, sum, s_apap);
      s_rr = fma(o_rk, o_rk, s_rr);
      // 4. rotate
      pr_pk = o_pk;
      o_pk = pk1;
      o_rk = rk1;
      o_pold = rq[0].p;
      o_pm2 = rq[0].r;
      o_epk = edge_pk(ed1);
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
    }  // !LEAN
  }
  f1_finish(s_pap, s_rap, s_apap, s_rr, partials, pstride, rc, st, tol);
}

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
template <int QD, bool PAIR, int KW, bool P3, bool LEAN = false, bool BIG = false, bool VC = false>
__global__ __launch_bounds__(64 * KW, VC ? 2 : 4) void k_cg_carry_ar3(SellDev S, F1Vectors v, int64_t own,
                                                                          TileRanges tr, int32_t LN, int gfull,
                                                                          double* __restrict__ partials, int pstride,
                                                                          CgState* st, double tol, int first,
                                                                          int check, RedCtl rc) {
  static_assert(KW >= 2 && QD >= 2, "3-D carry: >= 2 waves per block, operands >= 2 planes ahead");
  static_assert(!(VC && BIG), "3-D diav: 32-bit byte offsets (ranks below 2^29 rows)");
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
  // pass 0 runs the two-term kernel (see k_cg_carry_ar)
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
        auto raw_ld = [&](int32_t j, int32_t k) {
          Raw r;
          const uint32_t o = line_ofs(k) + l8;
          r.r = g_ld((j >= 0 && j < n_run) ? (const double*)pn : ro, o);
          r.p = pl.ld_p(pl.side(l0 + k, nl), po, o);
          return r;
        };
        auto ap_gh = [&](int32_t j) { return pl.ld_ap(pl.side(l0 + j, nl), apo, line_ofs(j) + l8); };
        auto edge_ld = [&](int32_t j) {
          Edge r;
          const uint32_t c = cb0 + (uint32_t)rc_(j) * SB + oc;
          r.r = g_ld(reo, c);
          r.a = g_ld(eao, c);
          r.p = g_ld(po, line_ofs(jc(j)) - 8u + op);
          return r;
        };
        auto edge_un = [&](int32_t j) {
          Edge r;
          const uint32_t c = cb0 + (uint32_t)j * SB + oc;
          r.r = g_ld(reo, c);
          r.a = g_ld(eao, c);
          r.p = g_ld(po, line_ofs(j) - 8u + op);
          return r;
        };
        auto rghost = [&](int32_t j, const Raw& qq) { return fma(nbp, g_ld(pn, line_ofs(j) + l8), qq.p); };
        auto is_ghost = [&](int32_t j) { return gfull && (l0 + j == -1 || l0 + j == nl) && j >= jlo && j <= jhi; };
        auto far_ld = [&](int32_t k) {
          Far f{0.0, 0.0, 0.0};
          if (outer) {
            const uint32_t o = line_ofs(k) + l8 + fob;
            f.r = g_ld(ro, o);
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
        auto epk = [&](const Edge& e) { return pk_of(e.r, e.a, e.p); };
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
          pr_pk = fma(b, rm1.p, fma(na, t, rm1.r));
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
        double o_fpk = pk_of(f0.r, f0.a, f0.p);
        // next: 1 plane m + 1 owned, 2 a ghost plane, 0 none
        auto lstep = [&](auto clc, int32_t m, int next) __attribute__((always_inline)) {
          constexpr bool CL = decltype(clc)::value;
          const int par = m & 1;
          const uint32_t ob = line_ofs(m);
          const double rr = fma(-b, o_pold, o_pk);
          if (m == 0 || m == n_run - 1) g_st_nt(rn, ob + l8, rr);
          else if (outer) g_st(rn, ob + l8, rr);
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
            rk1 = fma(na, t, m + 1 < n_run ? fma(nbp, qv[0].r, qv[0].p) : qv[0].r);
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
            g_st(ren, sb, rr);
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
          o_fpk = pk_of(fv[0].r, fv[0].a, fv[0].p);
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
          auto rebase = [&](int32_t m) {
            if constexpr (BIG) {
              mb = m;
              const int64_t eb = (int64_t)e0 + (int64_t)(m - 3) * LO, xb = (int64_t)i0 + (int64_t)m * LO;
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
            r.r = g_ld((j >= 0 && j < n_run) ? (const double*)pn_ : ro_, o);
            r.p = pl.ld_p(pl.side(l0 + k, nl), po_, o);
            return r;
          };
          auto ap_gh = [&](int32_t j) { return pl.ld_ap(pl.side(l0 + j, nl), apo_, line_ofs(j) + l8); };
          auto edge_ld = [&](int32_t j) {  // plane j (clamped: compact index to the rank, row to ext)
            Edge r;
            const uint32_t c = cb0 + (uint32_t)rc_(j) * SB + oc;
            r.r = g_ld(reo, c);
            r.a = g_ld(eao, c);
            r.p = g_ld(po_, line_ofs(jc(j)) - 8u + op);
            return r;
          };
          auto edge_un = [&](int32_t j) {
            Edge r;
            const uint32_t c = cb0 + (uint32_t)j * SB + oc;
            r.r = g_ld(reo, c);
            r.a = g_ld(eao, c);
            r.p = g_ld(po_, line_ofs(j) - 8u + op);
            return r;
          };
          auto rghost = [&](int32_t j, const Raw& q) { return fma(nbp, g_ld(pn_, line_ofs(j) + l8), q.p); };
          auto is_ghost = [&](int32_t j) { return gfull && (l0 + j == -1 || l0 + j == nl) && j >= jlo && j <= jhi; };
          auto far_ld = [&](int32_t k) {
            Far f{0.0, 0.0, 0.0};
            if (outer) {
              const uint32_t o = line_ofs(k) + l8 + fob;
              f.r = g_ld(ro_, o);
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
          auto epk = [&](const Edge& e) { return pk_of(e.r, e.a, e.p); };
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
            pr_pk = fma(b, rm1.p, fma(na, t, rm1.r));
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
          double o_fpk = pk_of(f0.r, f0.a, f0.p);
          // next: 1 plane m + 1 owned (values Vt), 2 a ghost plane, 0 none
          auto lstep = [&](auto clc, int32_t m, const VSet& Vs, const VSet& Vt, int next) __attribute__((always_inline)) {
            constexpr bool CL = decltype(clc)::value;
            const int par = m & 1;
            const uint32_t ob = line_ofs(m);
            const double rr = fma(-b, o_pold, o_pk);
            if (m == 0 || m == n_run - 1) g_st_nt(rn_, ob + l8, rr);
            else if (outer) g_st(rn_, ob + l8, rr);
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
              rk1 = fma(na, t, m + 1 < n_run ? fma(nbp, qv[0].r, qv[0].p) : qv[0].r);
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
              g_st(ren, sb, rr);
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
            o_fpk = pk_of(fv[0].r, fv[0].a, fv[0].p);
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

// finalize(): r_m = r_{m-1} - a A p_{m-1} (recomputed, same fma order), x_m, partial ||r_m||^2;
// or, when the run latched, the one-term x catch-up of an even m (k_cg_f1's final mode)
template <int CM, int U>
__global__ __launch_bounds__(kBS) void k_ar_final(SellDev S, F1Vectors v, int64_t own, int64_t n, int32_t lo, int32_t ln,
                                                  double* __restrict__ partials, int pstride, CgState* st,
                                                  double tol, int first, int check, int k, bool p3) {
  const int done = st->done;
  const F1Scalars sc = f1_scalars(st, tol, first, check);
  const double a = sc.alpha, na = -a, ap = st->a_prev;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  if (done || sc.conv) {
    const int64_t m = done ? (done == 1 ? st->conv_iter : -1) : k - 1;
    if (m >= 2 && (m & 1) == 0)
      for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        v.x[i] = fma(ap, v.p_fix[own + i], v.x[i]);
    return;
  }
  const bool pair = (k & 1) && k >= 3;
  double s_rr = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t e = own + i;
    ArCodes<CM, U> c;
    double t = 0.0;
    if constexpr (CM == 5) {  // diav: west / north from the partners' east / south (symmetric)
      const int64_t f = i + lo;
      const double kk[5] = {S.cvs[f - lo], S.cve[f - 1], S.cvd[f], S.cve[f], S.cvs[f]};
      const int64_t o5[5] = {-(int64_t)lo, -1, 0, 1, (int64_t)lo};
#pragma unroll
      for (int u = 0; u < 5; ++u) {
        int64_t q = e + o5[u];
        q = q < 0 ? 0 : (q >= v.ext_len ? v.ext_len - 1 : q);
        t = fma(kk[u], v.p_old[q], t);
      }
      (void)c;
    } else if constexpr (CM == 6) {  // 3-D diav (lo = plane, ln = N): south / down from the partners too
      const int64_t f = i + lo;
      const double kk[7] = {S.cvt[f - lo], S.cvs[f - ln], S.cve[f - 1], S.cvd[f], S.cve[f], S.cvs[f], S.cvt[f]};
      const int64_t o7[7] = {-(int64_t)lo, -(int64_t)ln, -1, 0, 1, (int64_t)ln, (int64_t)lo};
#pragma unroll
      for (int u = 0; u < 7; ++u) {
        int64_t q = e + o7[u];
        q = q < 0 ? 0 : (q >= v.ext_len ? v.ext_len - 1 : q);
        t = fma(kk[u], v.p_old[q], t);
      }
      (void)c;
    } else if constexpr (CM == 4) {  // absent entries: value 0 times a clamped (finite) operand
      ar_load_dia<U>(S.dia4 + (i >> 6) * (32 * U), (int)(i & 63), c);
      const int64_t o5[5] = {-(int64_t)lo, -1, 0, 1, (int64_t)lo};
      const int64_t o7[7] = {-(int64_t)lo, -(int64_t)ln, -1, 0, 1, (int64_t)ln, (int64_t)lo};
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t off = U == 5 ? o5[u] : o7[u];
        int64_t q = e + off;
        q = q < 0 ? 0 : (q >= v.ext_len ? v.ext_len - 1 : q);
        t = fma(S.dvals[(c.pk[0] >> (4 * u)) & 15u], v.p_old[q], t);
      }
    } else {
      const int64_t base = S.slice_ptr[i >> 6];
      ar_load_codes<CM, U>(S, base, (int)((S.slice_ptr[(i >> 6) + 1] - base) >> 6), (int)(i & 63), c);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        double val;
        const int32_t off = ar_entry<CM, U>(S.dict, c, u, val);
        if (u < c.w) t = fma(val, v.p_old[e + off], t);
      }
    }
    // three-term carry: r_{m-1} = p_{m-1} - b_prev p_{m-2} (p_new still holds p_{m-2})
    const double ro = (p3 && !first) ? fma(-st->b_prev, v.p_new[e], v.p_old[e]) : v.r_old[e];
    const double rk = fma(na, t, ro);
    v.r_new[e] = rk;
    v.x[i] = pair ? fma(a, v.p_old[e], fma(ap, v.p_new[e], v.x[i])) : fma(a, v.p_old[e], v.x[i]);
    s_rr = fma(rk, rk, s_rr);
  }
  block_partial4(0.0, 0.0, 0.0, s_rr, partials, pstride);
}

// SELL-64/c8 -> /dia4: one thread per row pair (lanes 2i, 2i+1 of a slice share the bytes).
// Entries with value +-0 (SELL padding) are skipped; any other entry must sit at a canonical
// offset, in strictly increasing offset order along the row's slots (else `bad`).
struct DiaOffs {
  int64_t o[7];
  int n;
};
__global__ __launch_bounds__(256) void k_sell_to_dia4(SellDev S, int nd, DiaOffs co, int zero_vi,
                                                      uint8_t* __restrict__ dia, unsigned* __restrict__ bad) {
  const int64_t npairs = (S.n_rows + 63) / 64 * 32;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < npairs; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t sl = t >> 5;
    const int l0 = (int)(t & 31) * 2;
    const int64_t base = S.slice_ptr[sl], w = (S.slice_ptr[sl + 1] - base) >> 6;
    uint32_t vi[2][7];
    for (int h = 0; h < 2; ++h) {
      for (int u = 0; u < 7; ++u) vi[h][u] = (uint32_t)zero_vi;
      int prev = -1;
      for (int64_t j = 0; j < w; ++j) {
        const int code = S.codes[base + 64 * j + l0 + h];
        const double2 q = S.dict[code];
        if ((__double_as_longlong(q.x) & 0x7fffffffffffffffll) == 0) continue;
        const int64_t off = (int64_t)__double_as_longlong(q.y);
        int cls = -1;
        for (int u = 0; u < co.n; ++u)
          if (off == co.o[u]) cls = u;
        if (cls <= prev) {
          atomicOr(bad, 1u);
          return;
        }
        prev = cls;
        vi[h][cls] = (uint32_t)(code / nd);
      }
    }
    for (int u = 0; u < co.n; ++u) dia[(sl * co.n + u) * 32 + (l0 >> 1)] = (uint8_t)(vi[0][u] | (vi[1][u] << 4));
  }
}

// dvals[a] = value a of the c8 dictionary (dict[a * nd].x), zero-padded to 16
__global__ void k_dia_vals(const double2* __restrict__ dict, int nv, int nd, double* __restrict__ dvals) {
  const int a = threadIdx.x;
  if (a < 16) dvals[a] = a < nv ? dict[a * nd].x : 0.0;
}

// SELL-64 -> /diav, one thread per local row.  CHECK = 0: the row's entries in slot order must sit at
// offsets -line, -1, 0, +1, +line, strictly increasing (else `bad`); d, e, s stored (absent: +0.0), a
// first-line row's north value into the front line of cvs.  CHECK = 1 (after the fill): the west /
// north values must equal the partners' east / south (the kernels take them from there).
// CM: 0 int32 ext columns, 1 d16 offsets, 2 c8 codes
// plane > 0 (3-D): seven classes (-plane, -line, -1, 0, +1, +line, +plane), arrays shifted by one
// plane, the front plane of cvt holding the plane-0 down values; check: down = cvt[i - plane] too.
template <int CM, bool CHECK>
__global__ __launch_bounds__(256) void k_sell_to_diav(SellDev S, int64_t line, int64_t plane, double* __restrict__ cvd,
                                                      double* __restrict__ cve, double* __restrict__ cvs,
                                                      double* __restrict__ cvt, unsigned* __restrict__ bad) {
  const int64_t n = S.n_rows;
  const int64_t fr = plane > 0 ? plane : line;  // rows in front of each array
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t sl = i >> 6, lane = i & 63;
    const int64_t base = S.slice_ptr[sl], w = (S.slice_ptr[sl + 1] - base) >> 6;
    const int64_t rowcol = S.own_off + i;
    double v7[7] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    int prev = -1;
    for (int64_t j = 0; j < w; ++j) {
      const int64_t k = base + 64 * j + lane;
      int64_t off;
      double val;
      if constexpr (CM == 2) {
        const double2 q = S.dict[S.codes[k]];
        val = q.x;
        off = (int64_t)__double_as_longlong(q.y);
      } else {
        val = S.vals[k];
        off = (CM == 1 ? rowcol + (int64_t)S.dcols[k] : (int64_t)S.cols[k]) - rowcol;
      }
      if (val == 0.0) continue;  // SELL padding (and explicit zeros: they add nothing)
      const int cls = off == -line ? 1 : (off == -1 ? 2 : (off == 0 ? 3 : (off == 1 ? 4 : (off == line ? 5 :
                      (plane > 0 && off == -plane ? 0 : (plane > 0 && off == plane ? 6 : -1))))));
      if (cls <= prev) {
        atomicOr(bad, 1u);
        return;
      }
      prev = cls;
      v7[cls] = val;
    }
    if constexpr (!CHECK) {
      cvd[fr + i] = v7[3];
      cve[fr + i] = v7[4];
      cvs[fr + i] = v7[5];
      if (plane > 0) {
        cvt[fr + i] = v7[6];
        if (i < plane) cvt[i] = v7[0];
      } else if (i < line) {
        cvs[i] = v7[1];
      }
    } else {
      // a row at a grid line's start has no west entry, and the row before it (a line's end) no east
      // one; 3-D: a line's row at y = 0 has no south entry, and its partner (y = N - 1 of the plane
      // before, or the front's zeros) no north one
      bool ok = v7[2] == cve[fr + i - 1];
      if (plane > 0) ok = ok && v7[1] == cvs[fr + i - line] && (i < plane || v7[0] == cvt[i]);
      else ok = ok && (i < line || v7[1] == cvs[i]);
      if (!ok) atomicOr(bad, 2u);
    }
  }
}

// SellDev::dpat, pass 1: a slice's pattern word -- bit 31 and the slot indices (4 bits per slot,
// bits 0..27) when each slot holds one value index for all 64 rows, else 0.  One exception is
// allowed per slice edge: lane 0's entry in the -1 slot (sm) and lane 63's in the +1 slot (sp)
// may be absent (the zero value index zv) while the other 63 lanes hold the slot's index -- a
// slice that starts / ends a grid line -- flagged in bit 28 / 29
__global__ __launch_bounds__(256) void k_dia_pattern(const uint8_t* __restrict__ dia, int64_t ns, int nslot, int sm,
                                                     int sp, int zv, uint64_t* __restrict__ dpat) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < ns; s += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* sp_ = dia + s * 32 * nslot;
    uint32_t w = 1u << 31;
    for (int u = 0; u < nslot && w != 0u; ++u) {
      const uint8_t* b = sp_ + 32 * u;
      const uint32_t maj = (uint32_t)(b[0] >> 4);  // lane 1
      bool same = true;
      for (int i = 1; i < 31; ++i) same = same && b[i] == (uint8_t)(maj | (maj << 4));
      const uint32_t l0 = b[0] & 15u, l63 = (uint32_t)(b[31] >> 4), l62 = b[31] & 15u;
      same = same && l62 == maj;
      if (l0 != maj) {
        if (u == sm && l0 == (uint32_t)zv) w |= 1u << 28;
        else same = false;
      }
      if (l63 != maj) {
        if (u == sp && l63 == (uint32_t)zv) w |= 1u << 29;
        else same = false;
      }
      w = same ? (w | (maj << (4 * u))) : 0u;
    }
    dpat[s] = w;
  }
}

// pass 2: one thread per slice column walks its lines upwards and counts, per slice, the lines
// from it down the column that carry the same uniform pattern; also counts the uniform slices
__global__ __launch_bounds__(256) void k_dia_runs(uint64_t* __restrict__ dpat, int64_t ss, int64_t nl,
                                                  unsigned long long* __restrict__ nuni) {
  const int64_t col = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= ss) return;
  uint64_t len = 0;
  uint32_t prev = 0;
  unsigned long long cnt = 0;
  for (int64_t l = nl - 1; l >= 0; --l) {
    const int64_t s = l * ss + col;
    const uint32_t w = (uint32_t)dpat[s];
    len = (w >> 31) ? (w == prev ? len + 1 : 1) : 0;
    cnt += (w >> 31);
    prev = w;
    dpat[s] = (len << 32) | w;
  }
  atomicAdd(nuni, cnt);
}

// carry_lean_failures: one thread per (job, wave) of the launch's job decomposition (k_cg_carry_ar:
// kw = 0, one wave per job; k_cg_carry_ar3: kw waves per job, their slice columns)
__global__ __launch_bounds__(256) void k_lean_check(const uint64_t* __restrict__ dpat, int64_t ss, int64_t nl,
                                                    int64_t ext_len, int64_t grid, int kw, int64_t ln,
                                                    int runs3,
                                                    unsigned long long* __restrict__ fails) {
  const int64_t waves = kw > 0 ? kw : 1;
  int64_t jobs, runs, chunk;
  if (kw == 0) {
    jobs = carry_jobs(grid * kWaves, ss, nl, runs, chunk);
  } else {
    const int64_t jpr = (ln / kw) * (ln / 64);
    runs = runs3 > 0 ? runs3 : (grid > jpr ? grid / jpr : 1);
    jobs = jpr * runs;
    chunk = (nl + runs - 1) / runs;
  }
  unsigned long long f = 0;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < jobs * waves; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t job = t / waves, wv = t % waves;
    int64_t col, l0, l1;
    if (kw == 0) {
      carry_run(job, ss, nl, chunk, col, l0, l1);
    } else {
      const int64_t jpr = (ln / kw) * (ln / 64), G = ln / 64, q = job % jpr;
      col = ((q / G) * kw + wv) * G + q % G;
      l0 = (job / jpr) * chunk;
      l1 = l0 + chunk < nl ? l0 + chunk : nl;
    }
    if (l0 >= l1) continue;
    uint32_t a, b, c;
    // past 2^29 the BIG kernels re-base: per run (2-D), along the run (3-D)
    if (!lean_eligible<false>(dpat, l0, l1, nl, ss, col, ext_len, a, b, c, 1)) ++f;
  }
  if (f) atomicAdd(fails, f);
}

}  // namespace

int32_t carry3_runs(int64_t nb, int64_t jpr, int64_t nl, int64_t max_chunk) {
  if (nb <= 0 || jpr <= 0 || nl <= 0) return 1;
  int32_t best = 1;
  int64_t best_cost = INT64_MAX;
  for (int64_t r = 1; r <= 64 && (r == 1 || nl / r >= 4); ++r) {
    if (max_chunk > 0 && (nl + r - 1) / r > max_chunk) continue;  // BIG: a run within 4 GiB of its base
    const int64_t rounds = (jpr * r + nb - 1) / nb, cost = rounds * ((nl + r - 1) / r + 3);
    if (cost < best_cost) {
      best_cost = cost;
      best = (int32_t)r;
    }
  }
  return best;
}

void pull_probe(const double* base, int64_t n, double* out, hipStream_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_pull_probe, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 1024)), dim3(256), 0, stream, base, n,
                     out);
  MCG_HIP(hipGetLastError(), "kernel launch failed(pull probe)");
}

void carry_jobs_host(int64_t nw, int64_t ss, int64_t nl, int64_t& runs, int64_t& chunk) {
  (void)carry_jobs(nw, ss, nl, runs, chunk);
}

int64_t carry_lean_failures(const uint64_t* dpat, int64_t ss, int64_t nl, int64_t ext_len, int grid, int kw,
                            int32_t ln, hipStream_t stream, int runs3) {
  MCG_CHECK(dpat != nullptr && ss > 0 && nl > 0 && grid > 0 && (kw == 0 || (ln % 64 == 0 && ln % kw == 0)),
            "lean check: bad launch geometry");
  unsigned long long* f = nullptr;
  MCG_HIP(hipMallocAsync(reinterpret_cast<void**>(&f), sizeof(unsigned long long), stream), "device malloc failed(lean)");
  MCG_HIP(hipMemsetAsync(f, 0, sizeof(unsigned long long), stream), "device memset failed");
  hipLaunchKernelGGL(k_lean_check, dim3(64), dim3(256), 0, stream, dpat, ss, nl, ext_len, (int64_t)grid, kw,
                     (int64_t)ln, runs3, f);
  MCG_HIP(hipGetLastError(), "kernel launch failed(lean check)");
  unsigned long long h = 0;
  MCG_HIP(hipMemcpyAsync(&h, f, sizeof(h), hipMemcpyDeviceToHost, stream), "memcpy from device to host failed");
  MCG_HIP(hipStreamSynchronize(stream), "device synchronize failed(lean check)");
  (void)hipFreeAsync(f, stream);
  return (int64_t)h;
}

int64_t dia_patterns(const uint8_t* dia4, const double* dvals, int64_t ns, int64_t ss, int nslot, uint64_t* dpat,
                     hipStream_t stream) {
  MCG_CHECK(dia4 != nullptr && dvals != nullptr && dpat != nullptr && ss > 0 && ns % ss == 0 &&
                (nslot == 5 || nslot == 7),
            "dia4 patterns: whole lines of slices");
  if (ns <= 0) return 0;
  // the value index of +0.0 (absent entries; sell_to_dia4 guarantees one)
  double hv[16];
  MCG_HIP(hipMemcpyAsync(hv, dvals, sizeof(hv), hipMemcpyDeviceToHost, stream), "memcpy from device to host failed(A)");
  MCG_HIP(hipStreamSynchronize(stream), "device synchronize failed(A)");
  int zv = -1;
  for (int a = 0; a < 16 && zv < 0; ++a)
    if (hv[a] == 0.0 && !std::signbit(hv[a])) zv = a;
  MCG_CHECK(zv >= 0, "dia4 patterns: no zero value");
  const int sm = nslot == 5 ? 1 : 2, sp = nslot == 5 ? 3 : 4;  // slots of the -1 / +1 offsets
  unsigned long long* cnt = nullptr;
  MCG_HIP(hipMallocAsync(reinterpret_cast<void**>(&cnt), sizeof(unsigned long long), stream), "device malloc failed(dia4)");
  MCG_HIP(hipMemsetAsync(cnt, 0, sizeof(unsigned long long), stream), "device memset failed");
  hipLaunchKernelGGL(k_dia_pattern, dim3(grid_for(ns, 256, 4)), dim3(256), 0, stream, dia4, ns, nslot, sm, sp, zv,
                     dpat);
  hipLaunchKernelGGL(k_dia_runs, dim3((unsigned)((ss + 255) / 256)), dim3(256), 0, stream, dpat, ss, ns / ss, cnt);
  MCG_HIP(hipGetLastError(), "kernel launch failed(dia4 patterns)");
  unsigned long long h = 0;
  MCG_HIP(hipMemcpyAsync(&h, cnt, sizeof(h), hipMemcpyDeviceToHost, stream), "memcpy from device to host failed");
  MCG_HIP(hipStreamSynchronize(stream), "device synchronize failed(dia4 patterns)");
  (void)hipFreeAsync(cnt, stream);
  return (int64_t)h;
}

bool sell_to_diav(const SellDev& S, int64_t line, double* cv, hipStream_t stream, int64_t plane) {
  const int64_t n = S.n_rows;
  const int64_t fr = plane > 0 ? plane : line;
  MCG_CHECK(cv != nullptr && line >= 64 && line % 64 == 0 && n % fr == 0 && (plane == 0 || plane == line * line),
            "diav: whole 64-row grid lines (3-D: whole planes)");
  if (line > INT32_MAX / 2) return false;
  const int na = plane > 0 ? 4 : 3;
  MCG_HIP(hipMemsetAsync(cv, 0, (size_t)na * (n + fr) * sizeof(double), stream), "device memset failed(diav)");
  unsigned* bad = nullptr;
  MCG_HIP(hipMallocAsync(reinterpret_cast<void**>(&bad), sizeof(unsigned), stream), "device malloc failed(diav)");
  MCG_HIP(hipMemsetAsync(bad, 0, sizeof(unsigned), stream), "device memset failed");
  double *cd = cv, *ce = cv + (n + fr), *cs = cv + 2 * (n + fr), *ct = plane > 0 ? cv + 3 * (n + fr) : nullptr;
  const unsigned g = (unsigned)std::min<int64_t>(std::max<int64_t>((n + 255) / 256, 1), 8192);
#define MCG_DV(CM)                                                                                             \
  do {                                                                                                         \
    hipLaunchKernelGGL((k_sell_to_diav<CM, false>), dim3(g), dim3(256), 0, stream, S, line, plane, cd, ce, cs, ct, \
                       bad);                                                                                   \
    hipLaunchKernelGGL((k_sell_to_diav<CM, true>), dim3(g), dim3(256), 0, stream, S, line, plane, cd, ce, cs, ct, \
                       bad);                                                                                   \
  } while (0)
  if (n > 0) {
    if (S.codes != nullptr) MCG_DV(2);
    else if (S.dcols != nullptr) MCG_DV(1);
    else MCG_DV(0);
  }
#undef MCG_DV
  MCG_HIP(hipGetLastError(), "kernel launch failed(diav)");
  unsigned h = 0;
  MCG_HIP(hipMemcpyAsync(&h, bad, sizeof(unsigned), hipMemcpyDeviceToHost, stream), "memcpy from device to host failed");
  MCG_HIP(hipStreamSynchronize(stream), "device synchronize failed(diav)");
  (void)hipFreeAsync(bad, stream);
  return h == 0;
}

void slice_meta(const int64_t* slice_ptr, int64_t n_slices, uint32_t* meta, hipStream_t stream) {
  if (n_slices <= 0) return;
  hipLaunchKernelGGL(k_slice_meta, dim3(grid_for(n_slices, 256, 4)), dim3(256), 0, stream, slice_ptr, n_slices, meta);
  MCG_HIP(hipGetLastError(), "kernel launch failed(slice_meta)");
}

bool sell_to_dia4(const SellDev& S, int nd, int64_t line, int64_t ln, uint8_t* dia4, double* dvals,
                  hipStream_t stream) {
  MCG_CHECK(S.codes != nullptr && S.dict != nullptr && nd > 0 && S.ndict % nd == 0, "dia4: c8 dictionary missing");
  const int nv = S.ndict / nd;
  if (nv > 16 || line <= 1 || line > INT32_MAX || ln < 0 || (ln > 0 && (ln <= 1 || ln >= line))) return false;
  DiaOffs co{};
  if (ln == 0) {
    const int64_t o[5] = {-line, -1, 0, 1, line};
    co.n = 5;
    for (int u = 0; u < 5; ++u) co.o[u] = o[u];
  } else {
    const int64_t o[7] = {-line, -ln, -1, 0, 1, ln, line};
    co.n = 7;
    for (int u = 0; u < 7; ++u) co.o[u] = o[u];
  }
  // the padding value +0.0 is always in the (sorted) value list
  std::vector<double2> dict(S.ndict);
  MCG_HIP(hipMemcpyAsync(dict.data(), S.dict, dict.size() * sizeof(double2), hipMemcpyDeviceToHost, stream),
          "memcpy from device to host failed(A)");
  MCG_HIP(hipStreamSynchronize(stream), "device synchronize failed(A)");
  int zero_vi = -1;
  for (int a = 0; a < nv; ++a)
    if (dict[(size_t)a * nd].x == 0.0 && !std::signbit(dict[(size_t)a * nd].x)) zero_vi = a;
  if (zero_vi < 0) return false;
  unsigned* bad = nullptr;
  MCG_HIP(hipMallocAsync(reinterpret_cast<void**>(&bad), sizeof(unsigned), stream), "device malloc failed(dia4)");
  MCG_HIP(hipMemsetAsync(bad, 0, sizeof(unsigned), stream), "device memset failed");
  const int64_t npairs = (S.n_rows + 63) / 64 * 32;
  if (npairs > 0)
    hipLaunchKernelGGL(k_sell_to_dia4, dim3((unsigned)std::min<int64_t>((npairs + 255) / 256, 65536)), dim3(256), 0,
                       stream, S, nd, co, zero_vi, dia4, bad);
  hipLaunchKernelGGL(k_dia_vals, dim3(1), dim3(64), 0, stream, S.dict, nv, nd, dvals);
  MCG_HIP(hipGetLastError(), "kernel launch failed(dia4)");
  unsigned h = 0;
  MCG_HIP(hipMemcpyAsync(&h, bad, sizeof(unsigned), hipMemcpyDeviceToHost, stream), "memcpy from device to host failed");
  MCG_HIP(hipStreamSynchronize(stream), "device synchronize failed(dia4)");
  (void)hipFreeAsync(bad, stream);
  return h == 0;
}

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
  MCG_CHECK(v.ext_len < ((int64_t)1 << 31), "Ap-recomputing carry: a rank's vectors must stay below 2^31 rows");
  if (cm == 4 && p3k && lean && S.dpat != nullptr) {  // lean-only kernels (4 waves per SIMD)
#define MCG_LW(QD, PAIR)                                                                                       \
  do {                                                                                                         \
    if (big)                                                                                                   \
      hipLaunchKernelGGL((k_cg_carry_ar<4, 5, QD, PAIR, true, 1, 4, true>), dim3(grid), dim3(kBS), 0, stream, S, v, \
                         own_off, tr, partials, pstride, st, tol, first, check, rc);                           \
    else                                                                                                       \
      hipLaunchKernelGGL((k_cg_carry_ar<4, 5, QD, PAIR, true, 1, 4>), dim3(grid), dim3(kBS), 0, stream, S, v, own_off, \
                         tr, partials, pstride, st, tol, first, check, rc);                                    \
  } while (0)
#define MCG_LWE(QD, PAIR, W)                                                                                   \
  hipLaunchKernelGGL((k_cg_carry_ar<4, 5, QD, PAIR, true, 1, W, false, true>), dim3(grid), dim3(kBS), 0, stream, S, v, \
                     own_off, tr, partials, pstride, st, tol, first, check, rc)
    // packed edges (depth 13: QD 3 at 5 waves per SIMD, 14: QD 4 at 4, the setup's auto_mix_ for the
    // 4-blocks-per-CU grids; measured and dropped: QD 5 at 4 for the odd passes, the same rate, and QD
    // 3 at 6 for the even ones, which spills in the loop: 4096^2 7200 vs 9470 it/s, profiles/r4/mix2;
    // r5 also dropped depth 2, 4 (3 waves per SIMD) and 6 (2): profiles/r3/lean, r4/mix)
    if (depth == 13 && !big) { if (pair) MCG_LWE(3, true, 5); else MCG_LWE(3, false, 5); }
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
    if (big)                                                                                                    \
      hipLaunchKernelGGL((k_cg_carry_ar<5, 5, QD, PAIR, true, 1, kLeanV, true>), dim3(grid), dim3(kBS), 0, stream, S, \
                         v, own_off, tr, partials, pstride, st, tol, first, check, rc);                         \
    else                                                                                                        \
      hipLaunchKernelGGL((k_cg_carry_ar<5, 5, QD, PAIR, true, 1, kLeanV>), dim3(grid), dim3(kBS), 0, stream, S, v, \
                         own_off, tr, partials, pstride, st, tol, first, check, rc);                            \
  } while (0)
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
  if (cm == 4) MCG_AQ(4, 5);
  else if (cm == 5) MCG_AQ(5, 5);
  else { if (param == 4) MCG_AQ(2, 4); else MCG_AQ(2, 5); }
#undef MCG_AQ
#undef MCG_AP
#undef MCG_A
  MCG_HIP(hipGetLastError(), "compute mv failed(Ap)");
}

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
  if (vc) {
#define MCG_A3V(PAIR, KW, P3, LEAN)                                                                            \
  hipLaunchKernelGGL((k_cg_carry_ar3<2, PAIR, KW, P3, LEAN, false, true>), dim3(grid), dim3(64 * KW), 0, stream, \
                     S, v, own_off, tr, ln, g, partials, pstride, st, tol, first, check, rc)
#define MCG_A3VK(PAIR, P3, LEAN) MCG_A3V(PAIR, 8, P3, LEAN)
#define MCG_A3VP(PAIR)                                          \
  do {                                                          \
    if (p3 && !first && lean) MCG_A3VK(PAIR, true, true);       \
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
#define MCG_A3(QD, PAIR, KW, P3, ...)                                                                         \
  hipLaunchKernelGGL((k_cg_carry_ar3<QD, PAIR, KW, P3, ##__VA_ARGS__>), dim3(grid), dim3(64 * KW), 0, stream, S, v, \
                     own_off, tr, ln, g, partials, pstride, st, tol, first, check, rc)
#define MCG_A3P(QD, PAIR, KW)                                         \
  do {                                                                \
    if (p3 && !first && lean && S.dpat != nullptr && big) MCG_A3(QD, PAIR, KW, true, true, true); \
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
