// L2-segment COO tiles: the SpMV of genuinely irregular matrices (BASELINE.json config 5 with the
// scrambled random-SPD family, or a user CSR whose columns are scattered).
//
// Why: a gather of p[col] for a random column misses the XCD's 4 MiB L2, and those misses are
// served at ~55 G requests/s whether p sits in the 256 MiB Infinity Cache or in HBM (the
// reference's cuSPARSE CSR SpMV, CUDACG.cu:288, has the same access pattern).  Gathers that hit
// the L2 run 4-5x faster (bench/gather_probe.hip, profiles/r3_gather_probe.md).  So the columns
// are cut into segments of S = 2^seg_shift doubles (default 2^18 = 2 MiB, half an XCD's L2;
// PassForm::tile_seg_log2), every wave owns kTileB = 1024 rows (their running sums live in LDS), and
// ALL waves sweep the segments in the same order: while the chip works on segment g, the XCDs' L2s
// hold p[g S, (g + 1) S) and the gathers hit.
//
// Storage (12 B per nonzero, like CSR): tile (b, g) = the nonzeros of row block b whose column is in
// segment g, a flat list of (row in block << 22 | column in segment) and the value;
// tptr[b * G + g] .. tptr[b * G + g + 1].  A wave spreads its tile over its 64 lanes and adds every
// product into the row's LDS slot (ds_add_f64); the wave owns those slots, so no other wave's adds
// interleave with its own, batch after batch in program order.  Inside ONE batch two lanes can hold
// entries of the same row; the order in which one ds_add_f64 applies same-address lanes is a
// hardware behaviour, not an architectural guarantee.  It is observed fixed on MI355X (repeated
// solves, graph and eager, bit for bit: tests/test_gpu_irregular.py, a tile built to collide), so
// the results are run-to-run bitwise on this hardware, not by construction.
//
// Pacing: waves left alone drift apart by a few segments within a sweep (a dependent load or a
// ragged tile end is enough), the L2 then holds none of the segments in flight and the hit rate
// falls from ~96 % to ~20 % (TCC counters, profiles/r3_gather_probe.md).  After each segment a
// workgroup therefore adds to its group's arrival counter (group = blockIdx % 8, i.e. the XCD
// under round-robin dispatch) and waits until all but 1/8 of the group's workgroups have finished
// that segment (stragglers do not stall the rest).  The wait is bounded (kPaceSpins polls): it
// paces, it never decides correctness, so a workgroup that is not co-resident only costs time.
// (r4 also measured, and r5 deleted: 960-row blocks for 5 workgroups per CU, 12 entries per lane in
// flight, fp32 storage of exact values, a prefetch of the next segment, counter polling and waiting
// for every workgroup -- each slower on config 5, profiles/r4/c5tb, c5v32, c5.)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mcg/check.hpp"
#include "mcg/kernels.hpp"
#include "spmv_engines.hpp"

namespace mcg {
namespace kern {
namespace {

#include "f1_common.hpp"

constexpr int kPaceSpins = 4000;      // ~1 ms of polling at most per segment step
constexpr int kPaceSleep = 8;         // s_sleep units (64 clocks) between two polls of a waiting workgroup
constexpr uint32_t kColMask = (1u << 22) - 1;

// `live` (thread 0's, per workgroup): cleared after the first wait that times out -- the group is not
// co-resident (another kernel holds CUs, or several ranks share the GPU), so this workgroup stops
// waiting for the rest of the launch instead of paying the cap at every segment.
//
// Step flags: the arrival whose add completes step s (the counter's return value says so: the counter
// passes every integer once) raises the group's step flag to s + 1 in 8 replicas on lines of their
// own; the waiters poll one replica each, which the XCD's L2 serves until the flag changes (polling
// the arrival counter itself, whose line every arrival writes, queued the arrivals behind the polls:
// 14.3 vs 17.5 it/s, profiles/r4/c5).
template <bool PRIO = true>
__device__ __forceinline__ void pace_step(const TilesDev& T, int step, int* live, int* behind) {
  __syncthreads();
  if (threadIdx.x == 0 && T.pace != nullptr && *live) {
    const int grp = blockIdx.x & 7;
    const unsigned nwg = (gridDim.x - grp + 7) >> 3;
    const unsigned slack = nwg >> 3;  // all but 1/8 of the group
    unsigned* c = T.pace + grp * 64;  // one 256-B block per group
    const unsigned old = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned* f = T.pace + kTilePaceCnt + grp * 8 * 64;
    const unsigned done = old + 1 + slack;
    if (done % nwg == 0)
      for (int r = 0; r < 8; ++r) __hip_atomic_fetch_max(f + r * 64, done / nwg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned* fr = f + ((blockIdx.x >> 3) & 7) * 64;
    const unsigned need = (unsigned)step + 1;  // the group has finished this segment
    int spin = 0;
    for (; spin < kPaceSpins; ++spin) {
      if (__hip_atomic_load(fr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= need) break;
      for (int z = 0; z < kPaceSleep; ++z) __builtin_amdgcn_s_sleep(1);
    }
    if (spin == kPaceSpins) *live = 0;
    *behind = spin == 0;  // arrived after the group had moved on: a straggler
  }
  __syncthreads();
  // A straggler's waves issue first during the next segment.  The wave arbiter favours older waves,
  // so on every CU the last-dispatched of its four workgroups fell behind at every step and the
  // others waited for it: 31 % of each workgroup's time at the pacing steps, bimodal within each CU
  // (profiles/r5/c5/README.md).  Feedback priority: 20.4-20.5 vs 19.5-19.6 it/s (with 10 entries per
  // lane); a static priority by dispatch order 19.6, three levels by arrival order 20.4-20.5.  Only
  // with 10 entries per lane: the 201 GB share's 8-per-lane tiles ran 9.17-9.24 with it, 9.51-9.53
  // without (profiles/r5/c5/prio/ab.md).
  if (PRIO && *behind) __builtin_amdgcn_s_setprio(3);
  else if (PRIO) __builtin_amdgcn_s_setprio(0);
}

// ABL bit 16 (diagnostic): per-workgroup wall-clock ticks spent waiting at the pacing steps and in total
constexpr int kTileDiagMax = 4096;
__device__ unsigned long long g_tile_diag[3 * kTileDiagMax];

// one batch of a tile: entries e = k + u * 64 < hi (non-temporal: streamed once)
template <int ABL, int TU>
__device__ __forceinline__ void tile_batch_load(const TilesDev& T, int64_t k, int64_t hi, uint32_t* q, double* v) {
#pragma unroll
  for (int u = 0; u < TU; ++u) {
    const int64_t e = k + u * 64;
    if constexpr ((ABL & 8) != 0) {
      q[u] = (uint32_t)e & 1023u;
      v[u] = 1.0;
      continue;
    }
    q[u] = e < hi ? __builtin_nontemporal_load(&T.idx[e]) : 0u;
    v[u] = e < hi ? __builtin_nontemporal_load(&T.vals[e]) : 0.0;
  }
}

// MODE 0: the split pass's SpMV (Ap_k = A p_k + the 4 partials + in-kernel reduction, as
// k_split_spmv); MODE 1: plain y = A x (true residual, ops).
// PART (MODE 0, all-gather overlap): 0 = every segment; 1 = only the segments [g_lo, g_hi) inside
// this rank's own block of p (they are final before the all-gather of p_k lands), the partial row
// sums stored in Ap, no partials; 2 = the other segments, added to those sums, then the epilogue
// (as k_split_spmv_aligned_part's halves)
// kTileB rows per block: 32 KiB of row sums, 4 workgroups per CU
// ABL (diagnostic ablations, MCG_TILES_ABLATE, results wrong), bits: 1 = no LDS adds (the products summed in
// a register), 2 = no gathers (the values themselves added), 4 = no pacing, 8 = no tile loads, 32 = every
// segment's gathers from segment 0 (always L2-hot), 64 = no straggler priority
// TU: entries per lane in flight, 8 or 10 (TilesDev::tu; software-pipelined: the next batch's indices and
// values load while this batch gathers).  The order of the adds is the same for either (ascending entry
// index), so the results are too.
// W: waves per workgroup -- 4 (four workgroups per CU, the default) or 16 (one per CU: the pacing
// step's barrier then holds waves of one age, so no CU has a youngest workgroup to fall behind;
// PassForm::tile_waves, an experiment: profiles/r6/c5)
template <int MODE, int PART = 0, int ABL = 0, int TU = 10, int W = 4>
__global__ __launch_bounds__(W * 64) __attribute__((amdgpu_waves_per_eu(4))) void k_tiles(TilesDev T, const double* __restrict__ p, const double* __restrict__ r,
                                               double* __restrict__ Ap, int64_t own, double* __restrict__ partials,
                                               int pstride, CgState* st, double tol, int first, int check, RedCtl rc) {
  constexpr int TB = kTileB;
  __shared__ double acc[W][TB];
  __shared__ int s_behind;
  int live = 0;  // thread 0's (the only one that paces)
  if constexpr (MODE == 0) {
    const F1Scalars sc = f1_scalars(st, tol, first, check);
    if (st->done || sc.conv) {  // uniform over the grid: every workgroup leaves, no pacing
      if constexpr (PART != 1) f1_finish<W>(0.0, 0.0, 0.0, 0.0, partials, pstride, rc, st, tol);
      return;
    }
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t nwaves = (int64_t)gridDim.x * W;
  const int64_t wave = (int64_t)blockIdx.x * W + wv;
  const int64_t rounds = (T.nblocks + nwaves - 1) / nwaves;
  const int G = T.G;
  // the segments this launch sweeps, in order: seg(0 .. ns - 1)
  const int glo = PART == 0 ? 0 : T.g_lo, ghi = PART == 0 ? 0 : T.g_hi;
  const int ns = PART == 0 ? G : (PART == 1 ? ghi - glo : G - (ghi - glo));
  auto seg = [&](int i) { return PART == 0 ? i : (PART == 1 ? glo + i : (i < glo ? i : i - glo + ghi)); };
  double* a = acc[wv];
  double s_pap = 0.0, s_rap = 0.0, s_apap = 0.0, s_rr = 0.0;
  int step = 0;
  if (threadIdx.x == 0) {
    live = 1;
    s_behind = 0;
  }
  unsigned long long t_wait = 0;
  const unsigned long long t_start = (ABL & 16) ? wall_clock64() : 0ull;
  for (int64_t rd = 0; rd < rounds; ++rd) {
    const int64_t b = wave + rd * nwaves;
    const bool active = b < T.nblocks;
    for (int rr = lane; rr < TB; rr += 64) a[rr] = 0.0;
    // tile g of block b = [tptr[b G + g], tptr[b G + g + 1])
    int64_t lo = 0, hi = 0;
    uint32_t q[TU];
    double v[TU];
    if (active && ns > 0) {
      const int g0 = seg(0);
      lo = T.tptr[b * G + g0];
      hi = T.tptr[b * G + g0 + 1];
      tile_batch_load<ABL, TU>(T, lo + lane, hi, q, v);
    }
    for (int i = 0; i < ns; ++i, ++step) {
      const int g = seg(i);
      int64_t lo_next = hi, hi_next = hi;
      if (active) {
        const double* __restrict__ pg = p + ((ABL & 32) ? 0 : ((int64_t)g << T.seg_shift));
        for (int64_t k = lo + lane; k < hi; k += TU * 64) {
          uint32_t qn[TU];
          double vn[TU], x[TU];
          tile_batch_load<ABL, TU>(T, k + TU * 64, hi, qn, vn);  // next batch in flight during this one's gathers
#pragma unroll
          for (int u = 0; u < TU; ++u) x[u] = (ABL & 2) ? 1.0 : (k + u * 64 < hi ? pg[q[u] & kColMask] : 0.0);
          if constexpr ((ABL & 1) != 0) {
#pragma unroll
            for (int u = 0; u < TU; ++u) s_rr = fma(v[u], x[u], s_rr);
          } else {
#pragma unroll
            for (int u = 0; u < TU; ++u)
              if (k + u * 64 < hi) atomicAdd(&a[q[u] >> 22], v[u] * x[u]);
          }
#pragma unroll
          for (int u = 0; u < TU; ++u) {
            q[u] = qn[u];
            v[u] = vn[u];
          }
        }
        // the next tile's first batch loads while the workgroup waits at the pacing step
        if (i + 1 < ns) {
          const int gn = seg(i + 1);
          lo_next = T.tptr[b * G + gn];
          hi_next = T.tptr[b * G + gn + 1];
          tile_batch_load<ABL, TU>(T, lo_next + lane, hi_next, q, v);
        }
      }
      if constexpr ((ABL & 16) != 0) {
        const unsigned long long w0 = wall_clock64();
        pace_step<TU == 10 && (ABL & 64) == 0>(T, step, &live, &s_behind);
        t_wait += wall_clock64() - w0;
      } else if constexpr ((ABL & 4) == 0) {
        pace_step<TU == 10 && (ABL & 64) == 0>(T, step, &live, &s_behind);
      }
      lo = lo_next;
      hi = hi_next;
    }
    if (active) {
      const int64_t r0 = b * TB;
      for (int rr = lane; rr < TB; rr += 64) {
        const int64_t i = r0 + rr;
        if (i >= T.n_rows) break;
        if constexpr (MODE == 0 && PART == 1) {
          Ap[i] = a[rr];  // the own-segment part of the row sum; part 2 adds the rest
        } else if constexpr (MODE == 0) {
          const double sum = PART == 2 ? Ap[i] + a[rr] : a[rr];
          const double pk = p[own + i], rk = r[i];
          st_stream(&Ap[i], sum);
          s_pap = fma(pk, sum, s_pap);
          s_rap = fma(rk, sum, s_rap);
          s_apap = fma(sum, sum, s_apap);
          s_rr = fma(rk, rk, s_rr);
        } else {
          Ap[i] = a[rr];
        }
      }
    }
    __syncthreads();
  }
  if constexpr (MODE == 1 && (ABL & 1) != 0) {
    if (s_rr == 1.2345e-300) Ap[0] = s_rr;  // keeps the gathers of the no-LDS-add ablation live
  }
  if constexpr ((ABL & 16) != 0) {
    if (threadIdx.x == 0 && blockIdx.x < kTileDiagMax) {
      g_tile_diag[2 * blockIdx.x] = t_wait;
      g_tile_diag[2 * blockIdx.x + 1] = wall_clock64() - t_start;
      // where the workgroup ran: HW_ID (cu / sh / se) and XCC_ID
      const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4), xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);
      g_tile_diag[2 * kTileDiagMax + blockIdx.x] = ((unsigned long long)xcc << 32) | hw;
    }
  }
  if constexpr (MODE == 0 && PART != 1) f1_finish<W>(s_pap, s_rap, s_apap, s_rr, partials, pstride, rc, st, tol);
}

// ---- setup: count / fill one row block per 64-thread workgroup (LDS counters per segment) ----
struct GenSrc {  // a generated family (problem.hpp), global rows row_begin + i, ext columns
  ProblemSpec s;
  int64_t row_begin, col_lo, pad;
  const int64_t* rp64;  // inclusive-scanned row lengths (the random-SPD diagonal = the row length)
  template <class F>
  __device__ void row(int64_t i, F&& f) const {
    for_each_entry(s, row_begin + i, [&](int64_t c, double v) { f(c - col_lo + pad, v); }, rp64[i + 1] - rp64[i]);
  }
};
struct CsrSrc {  // a user matrix's rows on the device (local CSR, ext columns)
  const int64_t* rp;
  const int32_t* cols;
  const double* vals;
  template <class F>
  __device__ void row(int64_t i, F&& f) const {
    for (int64_t k = rp[i]; k < rp[i + 1]; ++k) f((int64_t)cols[k], vals[k]);
  }
};

// FILL = false: tptr[b * G + g + 1] = entries of tile (b, g); FILL = true: write the tiles (tptr =
// exclusive offsets).  Lanes take rows rr = lane, lane + 64, ... of the block in lockstep; the order
// of one LDS atomic's same-address lanes (observed fixed, as above) orders a batch's appends.
template <bool FILL, class Src>
__global__ __launch_bounds__(64) void k_tiles_build(Src src, int64_t n, int tb, int G, int seg_shift, int64_t* __restrict__ tptr,
                                                    uint32_t* __restrict__ idx, double* __restrict__ vals) {
  extern __shared__ int cnt[];
  const int64_t b = blockIdx.x;
  const int lane = threadIdx.x;
  for (int g = lane; g < G; g += 64) cnt[g] = 0;
  __syncthreads();
  const uint32_t mask = (1u << seg_shift) - 1u;
  for (int rr = lane; rr < tb; rr += 64) {
    const int64_t i = b * tb + rr;
    if (i >= n) break;
    src.row(i, [&](int64_t ec, double v) {
      const int g = (int)(ec >> seg_shift);
      const int pos = atomicAdd(&cnt[g], 1);
      if constexpr (FILL) {
        const int64_t dst = tptr[b * G + g] + pos;
        idx[dst] = ((uint32_t)rr << 22) | ((uint32_t)ec & mask);
        vals[dst] = v;
      }
    });
  }
  __syncthreads();
  if constexpr (!FILL)
    for (int g = lane; g < G; g += 64) tptr[b * G + g + 1] = cnt[g];
}

}  // namespace

TilesGeometry tiles_geometry(int64_t n_rows, int64_t ext_len, int seg_shift) {
  const int tb = kTileB;
  TilesGeometry t;
  t.tb = tb;
  t.seg_shift = seg_shift;
  t.nblocks = (n_rows + tb - 1) / tb;
  t.G = (int)std::max<int64_t>(1, (ext_len + ((int64_t)1 << seg_shift) - 1) >> seg_shift);
  return t;
}

int tiles_grid(int ncu, int ww) {
  MCG_CHECK(ww == 4 || ww == 8 || ww == 16, "tiles: 4, 8 or 16 waves per workgroup");
  int per_cu = 0;
  const void* f = ww == 16 ? reinterpret_cast<const void*>(&k_tiles<0, 0, 0, 10, 16>)
                  : ww == 8 ? reinterpret_cast<const void*>(&k_tiles<0, 0, 0, 10, 8>)
                            : reinterpret_cast<const void*>(&k_tiles<0, 0, 0, 10>);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, ww * 64, 0) != hipSuccess || per_cu < 1) per_cu = 1;
  (void)hipGetLastError();
  // every workgroup resident on the solver's CUs (pacing waits on them): 16 waves per CU either way
  return std::min(per_cu, 16 / ww) * std::max(1, ncu);
}

namespace {
template <class Src>
void tiles_build_impl(const Src& src, int64_t n, const TilesGeometry& geo, const TilesOut& o, bool fill, hipStream_t st) {
  MCG_CHECK(geo.G <= kTileMaxSegments, "tiles: too many column segments for the LDS counters");
  MCG_CHECK(geo.seg_shift <= 22, "tiles: segments are at most 2^22 columns");
  MCG_CHECK(!fill || o.vals != nullptr, "tiles: fill needs the value array");
  if (geo.nblocks == 0) return;
  const size_t lds = (size_t)geo.G * sizeof(int);
  const dim3 grid((unsigned)geo.nblocks);
  if (!fill)
    hipLaunchKernelGGL((k_tiles_build<false, Src>), grid, dim3(64), lds, st, src, n, geo.tb, geo.G, geo.seg_shift,
                       o.tptr, o.idx, nullptr);
  else
    hipLaunchKernelGGL((k_tiles_build<true, Src>), grid, dim3(64), lds, st, src, n, geo.tb, geo.G, geo.seg_shift,
                       o.tptr, o.idx, o.vals);
  MCG_HIP(hipGetLastError(), "kernel launch failed(tiles_build)");
}
}  // namespace

void tiles_build_gen(const ProblemSpec& s, int64_t row_begin, int64_t n, int64_t col_lo, int64_t pad,
                     const int64_t* rp64, const TilesGeometry& geo, const TilesOut& out, bool fill, hipStream_t st) {
  tiles_build_impl(GenSrc{s, row_begin, col_lo, pad, rp64}, n, geo, out, fill, st);
}

void tiles_build_csr(const int64_t* rp, const int32_t* cols, const double* cvals, int64_t n, const TilesGeometry& geo,
                     const TilesOut& out, bool fill, hipStream_t st) {
  tiles_build_impl(CsrSrc{rp, cols, cvals}, n, geo, out, fill, st);
}

void cg_split_spmv_tiles(const TilesDev& T, const double* p_ext, const double* r, double* Ap, int64_t own_off,
                         double* partials, int pstride, int grid, CgState* st, double tol, int first, int check,
                         hipStream_t stream, const RedCtl& rc, int part) {
  if (grid <= 0) return;
  MCG_CHECK(rc.ngroups == 0 || (rc.base % kRedGroup == 0 && rc.cnt && rc.lvl2), "in-kernel reduction: bad control block");
  MCG_CHECK(part == 0 || (T.g_lo >= 0 && T.g_lo <= T.g_hi && T.g_hi <= T.G), "tiles: bad own-segment range");
  MCG_CHECK(part != 1 || rc.ngroups == 0, "tiles: the own-segment half writes no partials");
  MCG_CHECK(T.tb == kTileB && (T.tu == 8 || T.tu == 10), "tiles: 1024 rows per block, 8 or 10 entries per lane");
  MCG_CHECK(T.ww == 4 || T.ww == 8 || T.ww == 16, "tiles: 4, 8 or 16 waves per workgroup");
  if (T.pace) MCG_HIP(hipMemsetAsync(T.pace, 0, kTilePaceWords * sizeof(unsigned), stream), "device memset failed");
#define MCG_TL(PART, ABL, TU)                                                                                          \
  do {                                                                                                                 \
    if (T.ww == 16 && ABL == 0)                                                                                        \
      hipLaunchKernelGGL((k_tiles<0, PART, ABL, TU, 16>), dim3(grid), dim3(1024), 0, stream, T, p_ext, r, Ap, own_off,  \
                         partials, pstride, st, tol, first, check, rc);                                               \
    else if (T.ww == 8 && ABL == 0)                                                                                    \
      hipLaunchKernelGGL((k_tiles<0, PART, ABL, TU, 8>), dim3(grid), dim3(512), 0, stream, T, p_ext, r, Ap, own_off,    \
                         partials, pstride, st, tol, first, check, rc);                                               \
    else                                                                                                               \
      hipLaunchKernelGGL((k_tiles<0, PART, ABL, TU>), dim3(grid), dim3(256), 0, stream, T, p_ext, r, Ap, own_off,      \
                         partials, pstride, st, tol, first, check, rc);                                               \
  } while (0)
  static const int ablate = [] {
    const char* e = std::getenv("MCG_TILES_ABLATE");
    return e ? std::atoi(e) : 0;
  }();
  // the ablations (diagnostic, results wrong) run the 10-per-lane kernels only
#define MCG_TLA(PART)                          \
  do {                                         \
    if (ablate == 3) MCG_TL(PART, 3, 10);      \
    else if (ablate == 4) MCG_TL(PART, 4, 10); \
    else if (ablate == 7) MCG_TL(PART, 7, 10); \
    else if (ablate == 15) MCG_TL(PART, 15, 10); \
    else if (ablate == 64) MCG_TL(PART, 64, 10); \
    else if (T.tu == 10) MCG_TL(PART, 0, 10);  \
    else MCG_TL(PART, 0, 8);                   \
  } while (0)
  if (part == 1) MCG_TLA(1);
  else if (part == 2) MCG_TLA(2);
  else MCG_TLA(0);
#undef MCG_TLA
#undef MCG_TL
  MCG_HIP(hipGetLastError(), "compute mv failed(Ap)");
}

void spmv_tiles(const TilesDev& T, const double* x_ext, double* y, int grid, hipStream_t stream) {
  if (grid <= 0 || T.nblocks == 0) return;
  MCG_CHECK(T.tb == kTileB && (T.tu == 8 || T.tu == 10), "tiles: 1024 rows per block, 8 or 10 entries per lane");
  if (T.pace) MCG_HIP(hipMemsetAsync(T.pace, 0, kTilePaceWords * sizeof(unsigned), stream), "device memset failed");
  static const int ablate = [] {
    const char* e = std::getenv("MCG_TILES_ABLATE");
    return e ? std::atoi(e) : 0;
  }();
#define MCG_T1(ABL, TU)                                                                                                \
  do {                                                                                                                 \
    if (T.ww == 16 && ABL == 0)                                                                                        \
      hipLaunchKernelGGL((k_tiles<1, 0, ABL, TU, 16>), dim3(grid), dim3(1024), 0, stream, T, x_ext, nullptr, y, 0,      \
                         nullptr, 0, nullptr, 0.0, 0, 0, RedCtl());                                                   \
    else if (T.ww == 8 && ABL == 0)                                                                                    \
      hipLaunchKernelGGL((k_tiles<1, 0, ABL, TU, 8>), dim3(grid), dim3(512), 0, stream, T, x_ext, nullptr, y, 0,        \
                         nullptr, 0, nullptr, 0.0, 0, 0, RedCtl());                                                   \
    else                                                                                                               \
      hipLaunchKernelGGL((k_tiles<1, 0, ABL, TU>), dim3(grid), dim3(256), 0, stream, T, x_ext, nullptr, y, 0, nullptr, \
                         0, nullptr, 0.0, 0, 0, RedCtl());                                                            \
  } while (0)
  if (ablate == 1) MCG_T1(1, 10);
  else if (ablate == 2) MCG_T1(2, 10);
  else if (ablate == 3) MCG_T1(3, 10);
  else if (ablate == 4) MCG_T1(4, 10);
  else if (ablate == 7) MCG_T1(7, 10);
  else if (ablate == 15) MCG_T1(15, 10);
  else if (ablate == 16) MCG_T1(16, 10);
  else if (ablate == 32) MCG_T1(32, 10);
  else if (T.tu == 10) MCG_T1(0, 10);
  else MCG_T1(0, 8);
#undef MCG_T1
  if (ablate & 16) {  // diagnostic: the pacing waits' share of each workgroup's time
    std::vector<unsigned long long> d(3 * kTileDiagMax);
    MCG_HIP(hipStreamSynchronize(stream), "tiles diag sync failed");
    MCG_HIP(hipMemcpyFromSymbol(d.data(), HIP_SYMBOL(g_tile_diag), d.size() * sizeof(unsigned long long)), "tiles diag copy failed");
    const int nb = std::min(grid, kTileDiagMax);
    double w = 0, t = 0, tmax = 0, tmin = 1e300;
    for (int i = 0; i < nb; ++i) {
      w += (double)d[2 * i];
      t += (double)d[2 * i + 1];
      tmax = std::max(tmax, (double)d[2 * i + 1]);
      tmin = std::min(tmin, (double)d[2 * i + 1]);
    }
    std::fprintf(stderr, "{\"tiles_diag\": {\"workgroups\": %d, \"wait_frac\": %.4f, \"mean_ticks\": %.0f, \"min_ticks\": %.0f, \"max_ticks\": %.0f}}\n",
                 nb, t > 0 ? w / t : 0.0, t / nb, tmin, tmax);
    if (const char* fn = std::getenv("MCG_TILES_DIAG_FILE")) {  // one line per workgroup: block wait total hw_id xcc
      if (FILE* fo = std::fopen(fn, "w")) {
        for (int i = 0; i < nb; ++i) {
          const unsigned long long h = d[2 * kTileDiagMax + i];
          std::fprintf(fo, "%d %llu %llu %u %u\n", i, d[2 * i], d[2 * i + 1], (unsigned)(h & 0xffffffffu), (unsigned)(h >> 32));
        }
        std::fclose(fo);
      }
    }
  }
  MCG_HIP(hipGetLastError(), "compute mv failed(y)");
}

}  // namespace kern
}  // namespace mcg
