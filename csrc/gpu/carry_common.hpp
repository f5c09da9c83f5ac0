// Device helpers of the Ap-recomputing carries (cg_carry_ar.hip: 2-D line carry, cg_carry_ar3.hip:
// 3-D plane carry, carry_formats.hip: their matrix formats and setup checks): slice codes, lane
// moves, 32-bit-offset global accesses, the in-kernel halo's system-scope loads / stores, lean-run
// eligibility, the job -> run mapping, and the row-parallel final-mode kernel both carries share.
// Included inside namespace mcg::kern::{anonymous} after f1_common.hpp.
#pragma once

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
// MCG_PULL_FENCE: how a publishing wave ends its run.  1 (default): it waits for its stores
// (s_waitcnt vmcnt(0)) -- they are write-through, so acknowledged means in the memory the
// neighbours read; 2: a full system-scope release fence (buffer_wbl2 sc0 sc1 + the wait), which also
// writes back every dirty line of the XCD's L2 -- measured 29-30 % slower on the P = 8 shares
// (16384^2: 3432-3437 vs 4634-4869 it/s, 512^3: 5040-5124 vs 7169-7241, profiles/r6/fence/); 0: nothing
#ifndef MCG_PULL_FENCE
#define MCG_PULL_FENCE 1
#endif
// The in-kernel halo's memory-model argument.  Rank B's pass k stores its first / last line (p_k,
// Ap_k) with relaxed system-scope stores (st_sys: sc0 sc1, written through past B's L2 to its HBM),
// and the wave that stored them ends its run waiting for them (release(): the stores are complete --
// acknowledged by the memory that serves remote readers -- before anything the wave does later, its
// end included; a system-scope release fence would add only the write-back of the L2's OTHER dirty
// lines, which no neighbour reads, and costs 29 % of the pass).  B's kernel end precedes B's all-reduce of pass k in stream order; rank
// A's pass k + 1 follows A's all-reduce of pass k, which cannot complete before B contributed
// (RCCL: the data dependence of the sum; the IPC all-reduce: B's flag, stored after its own release).
// So A's pass k + 1, whose system-scope loads (ld_sys: past A's caches, over xGMI) read B's lines of
// pass k (p_{k-1} / Ap_{k-1} of pass k + 1), sees them; B's pass k + 1 rewrites the other p / apx
// buffers, never the ones A reads in pass k + 1, and rewrites these only in pass k + 2, after A's pass
// k + 1 has contributed to the next all-reduce.  The transport probe re-checks the whole chain on the
// job's fabric at setup (the pulled iterations must reproduce the exchanged ones bit for bit).
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
  // the end of a run [l0, l1) that published the rank's first / last line (the argument above); one
  // per publishing wave
  __device__ __forceinline__ void release(int64_t l0, int64_t l1, int64_t nl) const {
    if constexpr (MCG_PULL_FENCE == 1) {
      if (pub && (l0 == 0 || l1 == nl)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if constexpr (MCG_PULL_FENCE == 2) {
      if (pub && (l0 == 0 || l1 == nl)) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    }
  }
};

// Lean-run eligibility of one slice column's run [l0, l1) of a rank's nl lines (ss slices per
// line): lines l0 - 1 .. l1 carry uniform patterns (one, B, for the inner lines; the rank's first
// / last line their own, A / C, with B's slice-edge bits), and a column at a grid line's start /
// end has the absent edge entry.  UNI: the caller is a wave (one run; values made wave-uniform).
// nbr (three p buffers on a split rank, T3): the neighbouring columns' slices on those lines carry the
// same value pattern too -- a three-buffer lean run recomputes their edge rows with its own line's values
template <bool UNI>
__device__ __forceinline__ bool lean_eligible(const uint64_t* __restrict__ dpat, int64_t l0, int64_t l1, int64_t nl,
                                              int64_t ss, int64_t col, int64_t ext_len, uint32_t& WA, uint32_t& WB,
                                              uint32_t& WC, int big = 0, bool nbr = false) {
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
  go = go && (col != 0 || ((WB >> 28) & 1u)) && (col != ss - 1 || ((WB >> 29) & 1u));
  if (nbr && go) {
    const uint32_t m = ~(3u << 28);  // uniform flag and values; the slice-edge bits are the column's own
    for (int d = -1; d <= 1; d += 2) {
      const int64_t c = col + d;
      if (c < 0 || c >= ss) continue;
      const uint64_t wn = ld(ia * ss + c);
      go = go && ((((uint32_t)wn ^ WB) & m) == 0u) && (int64_t)(wn >> 32) >= ib - ia + 1;
      if (l0 <= 1) go = go && ((((uint32_t)ld(c) ^ WA) & m) == 0u);
      if (l1 >= nl - 1) go = go && ((((uint32_t)ld((nl - 1) * ss + c) ^ WC) & m) == 0u);
    }
  }
  return go;
}

// A split rank on three p buffers (TileRanges::sub_ranges): the next lean sub-range [a, b) of the run [L0, L1)
// at or after line `from` -- the stretch from `from` over which lines a - 1 .. b carry one pattern in this
// column and its neighbours (lean_eligible with nbr, WA / WB / WC set), at least 3 lines; false when none is
// left.  A T3 run needs nothing stored by its neighbours, so the lean launch takes every such stretch and
// the generic launch only the lines around the odd slices (split_generic_ranges lists them: the same walk).
template <bool UNI>
__device__ __forceinline__ bool next_lean_range(const uint64_t* __restrict__ dpat, int64_t from, int64_t L1, int64_t nl,
                                                int64_t ss, int64_t col, int64_t ext_len, int64_t& a, int64_t& b,
                                                uint32_t& WA, uint32_t& WB, uint32_t& WC) {
  auto ld = [&](int64_t i) { return UNI ? uni_u64(dpat[i]) : dpat[i]; };
  const uint32_t vm = ~(3u << 28);  // uniform flag and values (the slice-edge bits are each column's own)
  for (int64_t x = from; x + 3 <= L1;) {
    // lines ia .. ia + len - 1 identical in each of the three columns (k_dia_runs' counts)
    const int64_t ia = x - 1 > 1 ? x - 1 : 1;
    int64_t len = INT64_MAX;
    uint32_t w0 = 0u;
    int bad = 0;  // 1: a non-uniform slice on line ia, 2: the columns' patterns differ there
    for (int d = -1; d <= 1 && bad == 0; ++d) {
      const int64_t c = col + d;
      if (c < 0 || c >= ss) continue;
      const uint64_t wn = ld(ia * ss + c);
      if (((uint32_t)wn >> 31) == 0u) bad = 1;
      else if (w0 != 0u && (((uint32_t)wn ^ w0) & vm) != 0u) bad = 2;
      w0 = (uint32_t)wn;
      len = (int64_t)(wn >> 32) < len ? (int64_t)(wn >> 32) : len;
    }
    if (bad == 1) {  // the next candidate starts past that line
      x = ia + 2;
      continue;
    }
    if (bad == 2) {  // they differ all along the shortest stretch
      x = ia + len + 1;
      continue;
    }
    const int64_t y = ia + len - 1 >= nl - 2 ? L1 : (ia + len - 1 < L1 ? ia + len - 1 : L1);
    if (y - x >= 3 && lean_eligible<UNI>(dpat, x, y, nl, ss, col, ext_len, WA, WB, WC, 1, true)) {
      a = x;
      b = y;
      return true;
    }
    // the rank's last line (pattern C) may be what fails: the stretch short of it
    const int64_t y2 = y < nl - 2 ? y : nl - 2;
    if (y2 - x >= 3 && y2 != y && lean_eligible<UNI>(dpat, x, y2, nl, ss, col, ext_len, WA, WB, WC, 1, true)) {
      a = x;
      b = y2;
      return true;
    }
    ++x;  // (the rank's first line, pattern A, for x <= 1)
  }
  return false;
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
    if (m >= 2 && (m & 1) == 0) {
      const double* pf = v.p_fix3[0] != nullptr ? v.p_fix3[(m - 1) % 3] : v.p_fix;  // p_{m-1}
      for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        v.x[i] = fma(ap, pf[own + i], v.x[i]);
    }
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
