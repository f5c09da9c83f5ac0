// The carries' matrix formats and setup checks: SELL-64/c8 -> /dia4 (byte codes of the canonical
// stencil offsets + a <= 16-value table) and -> /diav (streamed per-row coefficients), the per-slice
// metadata, the uniform-slice patterns of the lean runs (dia_patterns) and their setup check
// (carry_lean_failures), the 3-D run split (carry3_runs) and the in-kernel halo's read-back probe.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <type_traits>
#include <array>
#include <vector>

#include "mcg/check.hpp"
#include "mcg/kernels.hpp"
#include "spmv_engines.hpp"

namespace mcg {
namespace kern {
namespace {

#include "f1_common.hpp"
#include "carry_common.hpp"

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
                                                    int runs3, bool nbr,
                                                    unsigned long long* __restrict__ fails, uint8_t* __restrict__ flags) {
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
    const bool ok = lean_eligible<false>(dpat, l0, l1, nl, ss, col, ext_len, a, b, c, 1, nbr);
    if (!ok) ++f;
    if (flags != nullptr && kw == 0) flags[job] = ok ? 0 : 1;
  }
  if (f) atomicAdd(fails, f);
}

// split_generic_ranges: one thread per job of the lean launch; the lines its lean stretches leave
// (next_lean_range, the walk the lean kernel makes) as ranges of at most maxlen lines
__global__ __launch_bounds__(256) void k_split_ranges(const uint64_t* __restrict__ dpat, int64_t ss, int64_t nl,
                                                      int64_t ext_len, int64_t grid, int maxlen, int cap,
                                                      unsigned* __restrict__ cnt, int32_t* __restrict__ out) {
  int64_t runs, chunk;
  const int64_t jobs = carry_jobs(grid * kWaves, ss, nl, runs, chunk);
  for (int64_t job = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; job < jobs; job += (int64_t)gridDim.x * blockDim.x) {
    int64_t col, L0, L1;
    carry_run(job, ss, nl, chunk, col, L0, L1);
    auto emit = [&](int64_t a, int64_t b) {
      for (int64_t x = a; x < b; x += maxlen) {
        const unsigned i = atomicAdd(cnt, 1u);
        if ((int)i < cap) {
          out[3 * i] = (int32_t)col;
          out[3 * i + 1] = (int32_t)x;
          out[3 * i + 2] = (int32_t)(x + maxlen < b ? x + maxlen : b);
        }
      }
    };
    int64_t from = L0, a = 0, b = 0;
    uint32_t wa, wb, wc;
    while (from < L1 && next_lean_range<false>(dpat, from, L1, nl, ss, col, ext_len, a, b, wa, wb, wc)) {
      emit(from, a);
      from = b;
    }
    emit(from, L1);
  }
}

// dia_lines_uniform: slices whose masked pattern word differs from their line's first slice
__global__ __launch_bounds__(256) void k_lines_uniform(const uint64_t* __restrict__ dpat, int64_t ss, int64_t nl,
                                                       unsigned long long* __restrict__ bad) {
  const uint32_t mask = ~(3u << 28);
  unsigned long long b = 0;
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < ss * nl; s += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t w = (uint32_t)dpat[s], w0 = (uint32_t)dpat[(s / ss) * ss];
    b += ((w >> 31) == 0u || (w & mask) != (w0 & mask)) ? 1u : 0u;
  }
  if (b) atomicAdd(bad, b);
}

}  // namespace

bool dia_lines_uniform(const uint64_t* dpat, int64_t ss, int64_t nl, hipStream_t stream) {
  if (dpat == nullptr || ss <= 0 || nl <= 0) return false;
  unsigned long long* f = nullptr;
  MCG_HIP(hipMallocAsync(reinterpret_cast<void**>(&f), sizeof(unsigned long long), stream), "device malloc failed(lines)");
  MCG_HIP(hipMemsetAsync(f, 0, sizeof(unsigned long long), stream), "device memset failed");
  hipLaunchKernelGGL(k_lines_uniform, dim3(grid_for(ss * nl, 256, 4)), dim3(256), 0, stream, dpat, ss, nl, f);
  MCG_HIP(hipGetLastError(), "kernel launch failed(lines uniform)");
  unsigned long long h = 1;
  MCG_HIP(hipMemcpyAsync(&h, f, sizeof(h), hipMemcpyDeviceToHost, stream), "memcpy from device to host failed");
  MCG_HIP(hipStreamSynchronize(stream), "device synchronize failed(lines uniform)");
  (void)hipFreeAsync(f, stream);
  return h == 0;
}

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

bool split_generic_ranges(const uint64_t* dpat, int64_t ss, int64_t nl, int64_t ext_len, int grid, int maxlen,
                          std::vector<int32_t>& ranges, hipStream_t stream) {
  MCG_CHECK(dpat != nullptr && ss > 0 && nl > 0 && grid > 0 && maxlen > 0, "split ranges: bad geometry");
  int64_t runs = 0, chunk = 0;
  const int64_t jobs = carry_jobs((int64_t)grid * kWaves, ss, nl, runs, chunk);
  // never overflows: lean stretches are >= 3 lines, so a run of L lines leaves at most L / 4 + 1 gaps, and
  // cutting them at maxlen lines adds at most L / maxlen pieces
  const int64_t cap64 = nl * ss / 4 + nl * ss / maxlen + jobs + 1024;
  MCG_CHECK(cap64 < ((int64_t)1 << 29), "split ranges: too many slices");
  const int cap = (int)cap64;
  unsigned* cnt = nullptr;
  int32_t* out = nullptr;
  MCG_HIP(hipMallocAsync(reinterpret_cast<void**>(&cnt), sizeof(unsigned), stream), "device malloc failed(ranges)");
  MCG_HIP(hipMallocAsync(reinterpret_cast<void**>(&out), (size_t)cap * 3 * sizeof(int32_t), stream), "device malloc failed(ranges)");
  MCG_HIP(hipMemsetAsync(cnt, 0, sizeof(unsigned), stream), "device memset failed");
  hipLaunchKernelGGL(k_split_ranges, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>((jobs + 255) / 256, 1024))),
                     dim3(256), 0, stream, dpat, ss, nl, ext_len, (int64_t)grid, maxlen, cap, cnt, out);
  MCG_HIP(hipGetLastError(), "kernel launch failed(split ranges)");
  unsigned h = 0;
  MCG_HIP(hipMemcpyAsync(&h, cnt, sizeof(h), hipMemcpyDeviceToHost, stream), "memcpy from device to host failed");
  MCG_HIP(hipStreamSynchronize(stream), "device synchronize failed(split ranges)");
  const bool ok = (int64_t)h <= cap;
  ranges.assign((size_t)(ok ? h : 0) * 3, 0);
  if (ok && h > 0) {
    MCG_HIP(hipMemcpy(ranges.data(), out, ranges.size() * sizeof(int32_t), hipMemcpyDeviceToHost),
            "memcpy from device to host failed(ranges)");
    // a fixed order (the atomic append's is not): by first line, then column -- the generic launch's waves
    // and so its partial slots take the ranges in this order
    std::vector<std::array<int32_t, 3>> t(h);
    for (size_t i = 0; i < h; ++i) t[i] = {ranges[3 * i + 1], ranges[3 * i], ranges[3 * i + 2]};
    std::sort(t.begin(), t.end());
    for (size_t i = 0; i < h; ++i) {
      ranges[3 * i] = t[i][1];
      ranges[3 * i + 1] = t[i][0];
      ranges[3 * i + 2] = t[i][2];
    }
  }
  (void)hipFreeAsync(cnt, stream);
  (void)hipFreeAsync(out, stream);
  return ok;
}

int64_t carry_lean_failures(const uint64_t* dpat, int64_t ss, int64_t nl, int64_t ext_len, int grid, int kw,
                            int32_t ln, hipStream_t stream, int runs3, bool nbr, std::vector<int32_t>* failed) {
  MCG_CHECK(dpat != nullptr && ss > 0 && nl > 0 && grid > 0 && (kw == 0 || (ln % 64 == 0 && ln % kw == 0)),
            "lean check: bad launch geometry");
  unsigned long long* f = nullptr;
  MCG_HIP(hipMallocAsync(reinterpret_cast<void**>(&f), sizeof(unsigned long long), stream), "device malloc failed(lean)");
  MCG_HIP(hipMemsetAsync(f, 0, sizeof(unsigned long long), stream), "device memset failed");
  int64_t njobs = 0, runs = 0, chunk = 0;
  uint8_t* fl = nullptr;
  if (failed != nullptr) {
    MCG_CHECK(kw == 0, "lean check: the failing-job list is for the 2-D carry");
    njobs = carry_jobs((int64_t)grid * kWaves, ss, nl, runs, chunk);
    MCG_HIP(hipMallocAsync(reinterpret_cast<void**>(&fl), (size_t)std::max<int64_t>(njobs, 1), stream),
            "device malloc failed(lean)");
  }
  hipLaunchKernelGGL(k_lean_check, dim3(64), dim3(256), 0, stream, dpat, ss, nl, ext_len, (int64_t)grid, kw,
                     (int64_t)ln, runs3, nbr, f, fl);
  MCG_HIP(hipGetLastError(), "kernel launch failed(lean check)");
  unsigned long long h = 0;
  MCG_HIP(hipMemcpyAsync(&h, f, sizeof(h), hipMemcpyDeviceToHost, stream), "memcpy from device to host failed");
  std::vector<uint8_t> hf((size_t)njobs);
  if (fl != nullptr && njobs > 0)
    MCG_HIP(hipMemcpyAsync(hf.data(), fl, (size_t)njobs, hipMemcpyDeviceToHost, stream), "memcpy from device to host failed");
  MCG_HIP(hipStreamSynchronize(stream), "device synchronize failed(lean check)");
  (void)hipFreeAsync(f, stream);
  if (fl != nullptr) (void)hipFreeAsync(fl, stream);
  if (failed != nullptr) {
    failed->clear();
    for (int64_t j = 0; j < njobs; ++j)
      if (hf[(size_t)j]) failed->push_back((int32_t)j);
  }
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

}  // namespace kern
}  // namespace mcg
