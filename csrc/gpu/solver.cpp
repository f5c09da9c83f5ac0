#include "mcg/solver.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <thread>

#include "mcg/check.hpp"
#include "mcg/trace.hpp"

namespace mcg {

namespace {
constexpr int kCsrBlocksPerCuCap = 6;  // LDS-limited residency of the CSR tile kernel (26.7 KB/block)

// SELL-64/aligned slots per nonzero expected for a wide random SPD matrix: a slice keeps the
// ~W candidates that reach the matrix from it; a row holds 1 + (W/2)(q_row + q_mean) of them,
// q = min(1, density * f) with f uniform on [0.25, 1.75] (problem.hpp randspd_density)
double randspd_aligned_fill(const ProblemSpec& s) {
  double qm = 0.0;
  for (int k = 0; k < 1000; ++k) qm += std::min(1.0, s.density * (0.25 + 1.5 * (k + 0.5) / 1000.0));
  qm /= 1000.0;
  return (double)(s.band + 1) / (1.0 + (double)s.band * qm);
}

// stored SELL-64 slots of rows taken in the order `order` (slice = 64 consecutive slots)
int64_t sell_slots(const HostCsr& A, const std::vector<int32_t>* order) {
  const int64_t n = A.n_rows;
  int64_t total = 0;
  for (int64_t s0 = 0; s0 < n; s0 += 64) {
    int64_t w = 0;
    for (int64_t i = s0; i < std::min(n, s0 + 64); ++i) {
      const int64_t r = order ? (*order)[i] : i;
      w = std::max<int64_t>(w, A.rowptr[r + 1] - A.rowptr[r]);
    }
    total += 64 * w;
  }
  return total;
}

// SELL-C-sigma: rows sorted by length (descending, stable) inside windows of `sigma` rows that
// never cross a cut (the interior / boundary slice ranges must keep their rows), so each 64-row
// slice holds rows of similar length.  Rewrites A in slot order; perm[slot] = local row.
bool sigma_sort(HostCsr& A, int64_t sigma, std::vector<int64_t> cuts, bool force, std::vector<int32_t>& perm) {
  const int64_t n = A.n_rows;
  std::vector<int32_t> order(n);
  for (int64_t i = 0; i < n; ++i) order[i] = (int32_t)i;
  cuts.push_back(0);
  cuts.push_back(n);
  std::sort(cuts.begin(), cuts.end());
  for (size_t c = 0; c + 1 < cuts.size(); ++c)
    for (int64_t a = cuts[c]; a < cuts[c + 1]; a += sigma) {
      const int64_t b = std::min(cuts[c + 1], a + sigma);
      std::stable_sort(order.begin() + a, order.begin() + b, [&](int32_t x, int32_t y) {
        return A.rowptr[x + 1] - A.rowptr[x] > A.rowptr[y + 1] - A.rowptr[y];
      });
    }
  const int64_t before = sell_slots(A, nullptr), after = sell_slots(A, &order);
  if (!force && (double)after > 0.9 * (double)before) return false;
  HostCsr P;
  P.n_rows = n;
  P.rowptr.assign(n + 1, 0);
  for (int64_t i = 0; i < n; ++i) P.rowptr[i + 1] = P.rowptr[i] + (A.rowptr[order[i] + 1] - A.rowptr[order[i]]);
  P.cols.resize(A.cols.size());
  P.vals.resize(A.vals.size());
  for (int64_t i = 0; i < n; ++i) {
    const int64_t r = order[i];
    std::copy(A.cols.begin() + A.rowptr[r], A.cols.begin() + A.rowptr[r + 1], P.cols.begin() + P.rowptr[i]);
    std::copy(A.vals.begin() + A.rowptr[r], A.vals.begin() + A.rowptr[r + 1], P.vals.begin() + P.rowptr[i]);
  }
  A = std::move(P);
  perm = std::move(order);
  return true;
}
}  // namespace

GpuCgSolver::GpuCgSolver(const ProblemSpec& spec, const CgOptions& opt, int rank, int world, Communicator* comm)
    : spec_(spec), opt_(opt), rank_(rank), world_(world), comm_(comm) {
  MCG_CHECK(world >= 1 && rank >= 0 && rank < world, "invalid rank/world");
  MCG_CHECK(world == 1 || comm != nullptr, "multi-rank solver needs a communicator");
  RowPartition part = partition_rows(spec_, world_, opt_.halo_mode);
  L_ = make_layout(spec_, part, rank_);
  // column indices are int32 in every format (CSR cols, SELL cols / ext offsets, kernel gathers)
  MCG_CHECK(L_.ext_len < ((int64_t)1 << 31) - 64,
            "a rank's rows + ghosts exceed int32 column indices (2^31): use more ranks");
  if (opt_.format == 2 || opt_.format == 3) {  // SELL-64 with 16-bit column offsets, if the bandwidth fits int16
    d16_ = bandwidth(spec_) <= 32767;
    c8_ = opt_.format == 3;  // dictionary codes: decided in setup() from the actual entries (fallback d16)
    opt_.format = 1;
  }
  // auto: the single-reduction form (one pass, one all-reduce per iteration) when P > 1 or on
  // SELL, where its interleaved {r, Ap} gathers make it the faster pass (profiles/sweep_ra_*)
  if (opt_.recurrence < 0) opt_.recurrence = (world_ > 1 || opt_.format == 1) ? 1 : 0;
  {
    const bool ra_ok = opt_.recurrence == 1 && opt_.format == 1;
    if (opt_.interleave < 0) opt_.interleave = ra_ok ? 1 : 0;
    MCG_CHECK(!opt_.interleave || ra_ok, "interleaved r/Ap layout needs the single-reduction recurrence on SELL");
  }
  use_comm_ = comm_ != nullptr && (world_ > 1 || opt_.force_comm);
  use_halo_ = use_comm_ && L_.has_halo();
  // one communicator for halo and all-reduce: every collective in one stream order on s0_
  if (use_comm_ && comm_->serialized()) opt_.overlap = false;
  if (use_comm_ && !comm_->graph_capturable()) opt_.use_graph = false;
  MCG_CHECK(opt_.graph_iters >= 2 && opt_.graph_iters % 2 == 0, "graph_iters must be even and >= 2");
  if (opt_.inject_nan_at >= 0) opt_.use_graph = false;  // the hook runs between eager iterations
  MCG_CHECK(opt_.recurrence >= -1 && opt_.recurrence <= 2, "recurrence must be -1 (auto), 0, 1 or 2 (pipelined)");
  // pipelined CG: a residual replacement every pipe_rr iterations is an eager step (no capture)
  if (opt_.recurrence == 2 && opt_.pipe_rr != 0) opt_.use_graph = false;
  // halo prefetch crosses iteration (and graph-launch) boundaries: eager runs only (and not for
  // the split pass, whose ghosts come from its own update kernel; decided in setup())
  prefetch_halo_ = use_halo_ && opt_.overlap && !opt_.use_graph && !L_.allgather;
  ncu_ = kern::num_cus();
  s0_ = Stream(true, 0);
  s1_ = Stream(true, -1);  // comm stream at higher priority: halo kernels start first
  ev_r_ = Event(true);
  ev_h_ = Event(true);
  ev_t0_ = Event(true, true);
  ev_t1_ = Event(true, true);
  ev_poll_[0] = Event(true);
  ev_poll_[1] = Event(true);
  ev_sync_[0] = Event(true);
  ev_sync_[1] = Event(true);
  host_st_ = PinnedBuffer<CgState>(2);
}

GpuCgSolver::~GpuCgSolver() {
  drop_graphs_();
  if (s0_.get()) (void)hipStreamSynchronize(s0_);
  if (s1_.get()) (void)hipStreamSynchronize(s1_);
}

template <typename IdxT>
void GpuCgSolver::build_csr_(DeviceBuffer<int64_t>& rp64, const HostCsr* user) {
  const int64_t n = L_.n_local();
  if (user) {  // user matrix: upload this rank's rows (columns already in ext coordinates)
    const size_t nnz = user->cols.size();
    if (nnz) {
      MCG_HIP(hipMemcpy(cols_.get(), user->cols.data(), nnz * sizeof(int32_t), hipMemcpyHostToDevice),
              "memcpy from host to device failed(A)");
      MCG_HIP(hipMemcpy(vals_.get(), user->vals.data(), nnz * sizeof(double), hipMemcpyHostToDevice),
              "memcpy from host to device failed(A)");
    }
    if constexpr (sizeof(IdxT) == 4) {
      std::vector<int32_t> rp(user->rowptr.begin(), user->rowptr.end());
      rp32_.allocate(n + 1, "A");
      MCG_HIP(hipMemcpy(rp32_.get(), rp.data(), rp.size() * sizeof(int32_t), hipMemcpyHostToDevice),
              "memcpy from host to device failed(A)");
    }
    return;
  }
  if constexpr (sizeof(IdxT) == 4) {
    rp32_.allocate(n + 1, "A");
    kern::gen_fill<int32_t>(spec_, L_.row_begin, n, L_.col_lo, L_.pad, rp64.get(), rp32_.get(), cols_.get(),
                            vals_.get(), s0_);
  } else {
    kern::gen_fill<int64_t>(spec_, L_.row_begin, n, L_.col_lo, L_.pad, rp64.get(), nullptr, cols_.get(),
                            vals_.get(), s0_);
  }
}

void GpuCgSolver::setup() {
  trace::Range tr_("mcg.setup");
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  const int64_t n = L_.n_local();
  fingerprint_ = problem_fingerprint(spec_);
  info_.n_global = L_.n_global;
  info_.n_local = n;
  info_.ext_len = L_.ext_len;
  info_.halo_in = L_.halo_rows_in();
  info_.halo_out = L_.halo_rows_out();
  info_.interior_rows = L_.interior_end - L_.interior_begin;
  info_.format = d16_ ? 2 : opt_.format;
  info_.recurrence = opt_.recurrence;
  info_.pipe_rr = opt_.recurrence == 2 ? opt_.pipe_rr : 0;
  MCG_CHECK(opt_.recurrence == 2 || opt_.pipe_rr == 0, "pipe_rr needs the pipelined recurrence (2)");
  info_.interleave = opt_.interleave == 1;

  // ---- A: count -> scan -> fill (owned rows, ext-local columns) ----
  // generated families on the device; a user matrix (kind Csr) from its host rows
  DeviceBuffer<int64_t> rp64(n + 1, "A");
  HostCsr user;
  const bool is_user = spec_.kind == ProblemKind::Csr;
  // ---- irregular sparsity: L2-segment COO tiles (the split pass's SpMV) ----
  // auto: the scrambled random SPD, or a user matrix that is not a grid stencil on the all-gather
  // layout (its columns are scattered over the whole vector); the same decision on every rank
  // (the spec and the layout kind are global)
  tiles_ = opt_.recurrence >= 1 && (opt_.pmat != 0 || opt_.recurrence == 2) && opt_.tiles != 0 &&
           (opt_.tiles == 1 || scrambled(spec_) || (is_user && L_.allgather && stencil_line(spec_) == 0));
  if (is_user) {
    user = build_local_csr(spec_, L_);
    if (opt_.format == 1 && !tiles_ && opt_.sell_sigma != 0 && n > 64 && (opt_.sell_sigma > 0 || stencil_line(spec_) == 0)) {
      // SELL-C-sigma (int32 columns): the windows never mix interior and boundary slices (auto: not
      // for a detected grid stencil, whose rows stay in grid order for the line / plane carry)
      const int64_t sig = opt_.sell_sigma > 1 ? (opt_.sell_sigma + 63) / 64 * 64 : 4096;
      std::vector<int64_t> cuts;
      if (use_halo_ && opt_.overlap && !L_.allgather) {
        cuts.push_back(std::min<int64_t>(n, (L_.interior_begin + 63) / 64 * 64));
        cuts.push_back(std::max<int64_t>(0, L_.interior_end / 64 * 64));
      }
      std::vector<int32_t> perm;
      if (sigma_sort(user, sig, cuts, opt_.sell_sigma > 0, perm)) {
        perm_.allocate(n, "A");
        MCG_HIP(hipMemcpy(perm_.get(), perm.data(), n * sizeof(int32_t), hipMemcpyHostToDevice),
                "memcpy from host to device failed(A)");
        info_.sigma = (int)sig;
        d16_ = false;  // offsets are relative to the slot's row: plain int32 columns with a permutation
        c8_ = false;
        info_.format = 1;
      }
    }
    MCG_HIP(hipMemcpy(rp64.get(), user.rowptr.data(), (n + 1) * sizeof(int64_t), hipMemcpyHostToDevice),
            "memcpy from host to device failed(A)");
    info_.max_row_len = 0;
    for (int64_t i = 0; i < n; ++i)
      info_.max_row_len = std::max<int64_t>(info_.max_row_len, user.rowptr[i + 1] - user.rowptr[i]);
  } else {
    kern::gen_rowlen(spec_, L_.row_begin, n, rp64.get(), s0_);
    info_.max_row_len = kern::max_i64(rp64.get() + 1, n, s0_);  // row lengths, before the scan
    DeviceBuffer<int64_t> tmp(kern::scan_tmp_elems(n), "A");
    kern::scan_inclusive_i64(rp64.get() + 1, n, tmp.get(), s0_);
    MCG_HIP(hipStreamSynchronize(s0_), "device synchronize failed(A)");
  }
  int64_t nnz = 0;
  MCG_HIP(hipMemcpy(&nnz, rp64.get() + n, sizeof(int64_t), hipMemcpyDeviceToHost),
          "memcpy from device to host failed(A)");
  // engine choice: short rows -> thread-per-row engines, long rows -> CSR-vector
  // CSR engine: thread per row when every row is short; else row-length-adaptive per 256-row tile
  // (eng::csr_adaptive: thread per row or 16 lanes per row, by one block vote per tile)
  info_.spmv_variant = opt_.spmv_variant >= 0 ? opt_.spmv_variant : (info_.max_row_len > 16 ? 4 : 1);
  info_.spmv_param = kern::spmv_param_for(info_.spmv_variant, info_.max_row_len);
  // SELL: one batch = the slice width when it is 4..8 (no clamped duplicate gathers)
  if (opt_.format == 1) info_.spmv_param = (int)std::max<int64_t>(4, std::min<int64_t>(8, info_.max_row_len));
  info_.nnz_local = nnz;
  info_.idx64 = nnz >= ((int64_t)1 << 31) - 64 || opt_.force_idx64;

  size_t matrix_bytes = 0;
  if (tiles_) {
    tgeo_ = kern::tiles_geometry(n, L_.ext_len, std::max(10, std::min(22, opt_.tile_seg_log2)));
    MCG_CHECK(tgeo_.G <= kern::kTileMaxSegments, "tiles: too many column segments (raise tile_seg_log2)");
    tptr_.allocate(tgeo_.nblocks * tgeo_.G + 1, "A");
    MCG_HIP(hipMemsetAsync(tptr_.get(), 0, tptr_.bytes(), s0_), "device memset failed(A)");
    tidx_.allocate(std::max<int64_t>(nnz, 1), "A", 64);
    tvals_.allocate(std::max<int64_t>(nnz, 1), "A", 64);
    tpace_.allocate(kern::kTilePaceWords, "A");
    DeviceBuffer<int32_t> tc;
    DeviceBuffer<double> tv;
    if (is_user && nnz) {  // this rank's rows on the device (temporary CSR, ext columns)
      tc.allocate(nnz, "A");
      tv.allocate(nnz, "A");
      MCG_HIP(hipMemcpy(tc.get(), user.cols.data(), nnz * sizeof(int32_t), hipMemcpyHostToDevice),
              "memcpy from host to device failed(A)");
      MCG_HIP(hipMemcpy(tv.get(), user.vals.data(), nnz * sizeof(double), hipMemcpyHostToDevice),
              "memcpy from host to device failed(A)");
    }
    const int64_t ntp = tgeo_.nblocks * tgeo_.G;
    for (int fill = 0; fill < 2; ++fill) {
      if (is_user) kern::tiles_build_csr(rp64.get(), tc.get(), tv.get(), n, tgeo_, tptr_.get(), tidx_.get(), tvals_.get(), fill, s0_);
      else kern::tiles_build_gen(spec_, L_.row_begin, n, L_.col_lo, L_.pad, rp64.get(), tgeo_, tptr_.get(), tidx_.get(),
                                 tvals_.get(), fill, s0_);
      if (!fill && ntp > 0) {  // tile sizes -> offsets
        DeviceBuffer<int64_t> tmp(kern::scan_tmp_elems(ntp), "A");
        kern::scan_inclusive_i64(tptr_.get() + 1, ntp, tmp.get(), s0_);
        MCG_HIP(hipStreamSynchronize(s0_), "device synchronize failed(A)");
      }
    }
    MCG_HIP(hipStreamSynchronize(s0_), "device synchronize failed(A)");
    int64_t tot = 0;
    MCG_HIP(hipMemcpy(&tot, tptr_.get() + ntp, sizeof(int64_t), hipMemcpyDeviceToHost),
            "memcpy from device to host failed(A)");
    MCG_CHECK(tot == nnz, "tiles: the fill does not match the row lengths");
    d16_ = false;
    c8_ = false;
    info_.format = 5;
    info_.sell_fill = 1.0;
    matrix_bytes = (size_t)nnz * 12 + tptr_.bytes();
  } else if (opt_.format == 1) {
    // ---- SELL-64, generated directly (no CSR intermediate: peak memory = the SELL arrays) ----
    const int64_t ns = (n + 63) / 64;
    slice_ptr_.allocate(ns + 1, "A");
    // SELL-64/aligned: the same decision on every rank (from the spec, not from this rank's rows),
    // since it implies the split pass and with it the ghost vectors exchanged
    aligned_ = spec_.kind == ProblemKind::RandomSPD && spec_.spread > 0 && !spec_.scramble && opt_.recurrence == 1 &&
               opt_.pmat != 0 && opt_.sell_aligned != 0 &&
               (opt_.sell_aligned == 1 || randspd_aligned_fill(spec_) <= 1.6);
    if (aligned_) kern::randspd_aligned_widths(spec_, L_.row_begin, n, slice_ptr_.get(), s0_);
    else kern::sell_slice_widths(rp64.get(), n, slice_ptr_.get(), s0_);
    {
      DeviceBuffer<int64_t> tmp(kern::scan_tmp_elems(ns), "A");
      kern::scan_inclusive_i64(slice_ptr_.get() + 1, ns, tmp.get(), s0_);
      MCG_HIP(hipStreamSynchronize(s0_), "device synchronize failed(A)");
    }
    int64_t total = 0;
    MCG_HIP(hipMemcpy(&total, slice_ptr_.get() + ns, sizeof(int64_t), hipMemcpyDeviceToHost),
            "memcpy from device to host failed(A)");
    if (aligned_) {
      d16_ = false;
      c8_ = false;
      info_.format = 4;
      soffs_.allocate(std::max<int64_t>(total / 64, 1), "A");
    } else if (d16_) dcols_.allocate(total, "A", 16);
    else cols_.allocate(total, "A", 8);
    vals_.allocate(total, "A", 8);
    if (aligned_) {
      kern::randspd_fill_aligned(spec_, L_.row_begin, n, rp64.get(), slice_ptr_.get(), soffs_.get(), vals_.get(),
                                 s0_);
      MCG_HIP(hipStreamSynchronize(s0_), "device synchronize failed(A)");
    } else if (is_user) {  // host rows -> device CSR (temporary) -> SELL-64(/d16)
      DeviceBuffer<int32_t> tc(std::max<int64_t>(nnz, 1), "A");
      DeviceBuffer<double> tv(std::max<int64_t>(nnz, 1), "A");
      if (nnz) {
        MCG_HIP(hipMemcpy(tc.get(), user.cols.data(), nnz * sizeof(int32_t), hipMemcpyHostToDevice),
                "memcpy from host to device failed(A)");
        MCG_HIP(hipMemcpy(tv.get(), user.vals.data(), nnz * sizeof(double), hipMemcpyHostToDevice),
                "memcpy from host to device failed(A)");
      }
      if (n > 0)
        kern::csr_to_sell<int64_t>(rp64.get(), tc.get(), tv.get(), n, L_.own_off, slice_ptr_.get(),
                                   d16_ ? nullptr : cols_.get(), vals_.get(), s0_, d16_ ? dcols_.get() : nullptr);
      MCG_HIP(hipStreamSynchronize(s0_), "device synchronize failed(A)");
    } else {
      kern::gen_fill_sell(spec_, L_.row_begin, n, L_.col_lo, L_.pad, L_.own_off, rp64.get(), slice_ptr_.get(),
                          cols_.get(), dcols_.get(), vals_.get(), s0_);
    }
    matrix_bytes = aligned_ ? total * 8 + (total / 64) * 4 + (ns + 1) * 8 : total * (d16_ ? 10 : 12) + (ns + 1) * 8;
    if (c8_) {  // SELL-64/c8 when the (value, offset) dictionary fits one byte
      std::vector<double2> dict;
      int nv = 0, nd = 0;
      c8_ = kern::sell_dict_build(sell_view(), dict, nv, nd, s0_);
      if (c8_) {
        ndict_ = (int)dict.size();
        dict_offsets_.clear();
        for (int q = 0; q < nd; ++q) {  // dict[vi * nd + di].y = bits of offset di
          long long off;
          std::memcpy(&off, &dict[q].y, sizeof(off));
          dict_offsets_.push_back((int64_t)off);
        }
        dict_.allocate(dict.size(), "A");
        MCG_HIP(hipMemcpy(dict_.get(), dict.data(), dict.size() * sizeof(double2), hipMemcpyHostToDevice),
                "memcpy from host to device failed(A)");
        codes_.allocate(total, "A", 512);  // the line-carry pass reads all U <= 8 entry slots of a slice
        kern::sell_to_c8(sell_view(), dict_.get(), nv, nd, codes_.get(), s0_);
        MCG_HIP(hipStreamSynchronize(s0_), "device synchronize failed(A)");
        cols_.release();
        dcols_.release();
        vals_.release();
        info_.format = 3;
        matrix_bytes = total + (ns + 1) * 8;
      }
    }
    info_.sell_fill = nnz > 0 ? (double)total / (double)nnz : 1.0;
    if (!c8_ && !perm_.get() && !aligned_ && opt_.recurrence == 1 && opt_.window != 0 &&
        n > 0) {
      // windowed pass: per-chunk column windows of the generated matrix
      const int64_t nch = (n + kern::kWinRows - 1) / kern::kWinRows;
      win_.allocate(2 * nch, "A");
      kern::chunk_windows(sell_view(), win_.get(), s0_);
      std::vector<int32_t> w(2 * nch);
      MCG_HIP(hipMemcpyAsync(w.data(), win_.get(), w.size() * sizeof(int32_t), hipMemcpyDeviceToHost, s0_),
              "memcpy from device to host failed(A)");
      MCG_HIP(hipStreamSynchronize(s0_), "device synchronize failed(A)");
      int64_t width = 0;
      for (int64_t c = 0; c < nch; ++c) width = std::max<int64_t>(width, (int64_t)w[2 * c + 1] - w[2 * c]);
      const bool fits = width * (int64_t)sizeof(double) <= (int64_t)kern::kWinMaxLds;
      const bool dense_rows = nnz >= 32 * n;
      MCG_CHECK(opt_.window != 1 || fits, "windowed pass: a chunk's column window exceeds the LDS budget");
      if (fits && (opt_.window == 1 || dense_rows)) {
        win_doubles_ = (int)width;
        kern::cg_fused1_win_prepare(win_doubles_);
      } else {
        win_.release();
      }
    }
    MCG_HIP(hipStreamSynchronize(s0_), "device synchronize failed(A)");
  } else {
    cols_.allocate(nnz, "A", 8);
    vals_.allocate(nnz, "A", 8);
    if (info_.idx64) build_csr_<int64_t>(rp64, is_user ? &user : nullptr);
    else build_csr_<int32_t>(rp64, is_user ? &user : nullptr);
    matrix_bytes = nnz * 12 + (n + 1) * (info_.idx64 ? 8 : 4);
    if (info_.idx64) rp64_ = std::move(rp64);
  }

  // ---- iteration form for long / unstructured rows: the materialized-p split pass ----
  pmat_ = opt_.recurrence == 1 && opt_.pmat != 0 &&
          (opt_.pmat == 1 || aligned_ || tiles_ || (win_doubles_ == 0 && !c8_ && (L_.allgather || nnz >= 32 * n)));
  // the pass form decides which ghost vectors are exchanged ({r, Ap} + p, or p alone): every rank
  // must take the same one, whatever its own rows look like
  if (use_comm_ && world_ > 1) pmat_ = all_ranks_agree_(pmat_);
  MCG_CHECK(!aligned_ || pmat_, "aligned SELL needs the split pass");
  MCG_CHECK(!tiles_ || pmat_ || opt_.recurrence == 2, "tiles need the split pass on every rank");
  info_.tiles = tiles_;
  info_.tile_segments = tiles_ ? tgeo_.G : 0;
  if (pmat_) {
    opt_.interleave = 0;
    info_.interleave = false;
    prefetch_halo_ = false;
  }
  info_.pmat = pmat_;
  info_.allgather = L_.allgather;
  halo_ahead_ = opt_.halo_ahead != 0 && use_halo_ && opt_.overlap && !pmat_ && !L_.allgather && opt_.recurrence == 1;
  if (halo_ahead_) prefetch_halo_ = false;
  info_.halo_ahead = halo_ahead_;
  split_ = use_halo_ && opt_.overlap && !halo_ahead_;
  if (opt_.recurrence == 2) split_ = prefetch_halo_ = false;  // pipelined: the all-reduce is what overlaps
  // all-gather overlap: the own-block slots of each aligned slice are summed while p_k's all-gather
  // is in flight (aligned_ is decided from the spec and the layout is the same kind on every rank,
  // so every rank takes the same launches)
  ag_overlap_ = aligned_ && pmat_ && use_halo_ && L_.allgather && opt_.overlap && opt_.ag_overlap != 0 && n > 0;
  if (ag_overlap_) {
    const int64_t ns = (n + 63) / 64;
    lslots_.allocate(2 * ns, "A");
    kern::aligned_local_slots(sell_view(), lslots_.get(), s0_);
    std::vector<int32_t> ab(2 * ns);
    std::vector<int64_t> sp(ns + 1);
    MCG_HIP(hipMemcpyAsync(ab.data(), lslots_.get(), ab.size() * sizeof(int32_t), hipMemcpyDeviceToHost, s0_),
            "memcpy from device to host failed(A)");
    MCG_HIP(hipMemcpyAsync(sp.data(), slice_ptr_.get(), sp.size() * sizeof(int64_t), hipMemcpyDeviceToHost, s0_),
            "memcpy from device to host failed(A)");
    MCG_HIP(hipStreamSynchronize(s0_), "device synchronize failed(A)");
    int64_t loc = 0;
    for (int64_t s = 0; s < ns; ++s) loc += ab[2 * s + 1] - ab[2 * s];
    info_.ag_local_frac = sp[ns] > 0 ? (double)(64 * loc) / (double)sp[ns] : 0.0;
  }
  info_.ag_overlap = ag_overlap_;

  // ---- vectors ----
  b_.allocate(n, "b", 8);
  if (is_user) {  // the user's b (or the spec's rhs kind), built on the host
    const std::vector<double> hb = build_rhs(spec_, L_.row_begin, L_.row_end);
    if (n) MCG_HIP(hipMemcpy(b_.get(), hb.data(), n * sizeof(double), hipMemcpyHostToDevice),
                   "memcpy from host to device failed(b)");
  } else {
    kern::gen_rhs(spec_, L_.row_begin, n, b_.get(), s0_);
  }

  // ---- launch geometry ----
  const int bpc = opt_.blocks_per_cu > 0 ? opt_.blocks_per_cu : (opt_.format == 1 ? 48 : 8);
  info_.window = win_doubles_;
  pipe_ = opt_.pipeline != 0 && opt_.format == 1 && (d16_ || c8_) && opt_.interleave == 1 &&
          info_.max_row_len <= 8 && info_.spmv_param >= info_.max_row_len;
  MCG_CHECK(opt_.pipeline != 1 || pipe_, "pipelined pass needs SELL d16/c8, interleave and rows <= param <= 8");
  info_.pipeline = pipe_;
  auto grid_a = [&](const TileRanges& t) {
    if (t.ntiles == 0) return 0;
    if (win_doubles_ > 0) {  // 1024-thread chunk blocks: 2 per CU while the window fits half the LDS
      const int per_cu = win_doubles_ * 8 <= 75 * 1024 ? 2 : 1;
      return (int)std::max<int64_t>(1, std::min<int64_t>(kern::win_chunks(t), (int64_t)ncu_ * per_cu));
    }
    if (opt_.format == 1) return kern::grid_for(t.ntiles * 64, 256, bpc);
    if (info_.spmv_variant == 0)  // LDS-limited residency
      return kern::grid_for(t.ntiles * kTileRows, 256, std::min(bpc, kCsrBlocksPerCuCap));
    return kern::grid_for(t.ntiles * kTileRows, 256, bpc);
  };
  auto ranges = [&](int64_t b0, int64_t e0, int64_t b1, int64_t e1) {
    if (opt_.format == 1) {  // slice units; rows [b,e) -> whole slices
      return make_tiles(b0 / 64, (e0 + 63) / 64, b1 / 64, (e1 + 63) / 64, 1);
    }
    return make_tiles(b0, e0, b1, e1);
  };
  tr_all_ = ranges(0, n, 0, 0);
  g_all_ = grid_a(tr_all_);
  if (split_) {
    int64_t ib = L_.interior_begin, ie = L_.interior_end;
    if (opt_.format == 1) {  // interior launch takes only whole slices inside the interior
      const int64_t sb = (ib + 63) / 64, se = ie / 64;
      if (se > sb) {
        tr_int_ = make_tiles(sb, se, 0, 0, 1);
        tr_bnd_ = make_tiles(0, sb, se, (n + 63) / 64, 1);
      } else {
        tr_int_ = make_tiles(0, 0, 0, 0, 1);
        tr_bnd_ = make_tiles(0, (n + 63) / 64, 0, 0, 1);
      }
    } else {
      tr_int_ = make_tiles(ib, ie);
      tr_bnd_ = make_tiles(0, ib, ie, n);
    }
    g_int_ = grid_a(tr_int_);
    g_bnd_ = grid_a(tr_bnd_);
  }
  if (tiles_) {  // one launch over every row block: the resident workgroups (the pacing waits on each)
    g_all_ = n > 0 ? kern::tiles_grid() : 0;
    if (opt_.blocks_per_cu > 0) g_all_ = std::min(g_all_, ncu_ * opt_.blocks_per_cu);  // fewer waves: more rounds
    g_int_ = 0;
    g_bnd_ = g_all_;
  }
  if (opt_.format == 1 && stencil_plane(spec_) > 0 && win_doubles_ == 0 &&
      opt_.blocks_per_cu <= 0 && partition_granule(spec_) % 64 == 0) {
    // 3-D stencil, generic pass: XCD-aware sweep with one plane of slices per step.  Each XCD
    // walks a contiguous 1/8 of the slices with grid / 8 blocks x 4 waves = P slices (one plane)
    // per grid-stride step, so a row's +-N^2 (previous / next plane) neighbours are the same
    // wave's previous / next slice and hit the L2 (512^3: 400 vs 312 it/s,
    // profiles/sweep_xcd_3d.log).  Speed only: every slice is still visited once.
    const int64_t P = partition_granule(spec_) / 64;
    const int64_t cus = ncu_;
    int64_t g = std::min<int64_t>(std::max<int64_t>(2 * P, cus * 4), cus * 64) / 8 * 8;
    auto apply = [&](TileRanges& t, int& grid) {
      if (t.ntiles == 0 || g < 8) return;
      t.xcd = 8;
      grid = (int)g;
    };
    apply(tr_all_, g_all_);
    if (split_) apply(tr_int_, g_int_);
    info_.xcd_map = true;
  }
  {
    // line-carry pass: whole 64-row slices per grid line (2-D) / plane (3-D), the stencil path's
    // format and layout; applies to a launch whose slices are one range of whole lines
    const int64_t gl = partition_granule(spec_);
    const bool ok = opt_.recurrence == 1 && opt_.format == 1 && (d16_ || c8_) && opt_.interleave == 1 &&
                    win_doubles_ == 0 && info_.max_row_len <= 8 &&
                    info_.spmv_param >= info_.max_row_len && info_.spmv_param >= 4 && gl > 1 && gl % 64 == 0 &&
                    n % gl == 0 && L_.row_begin % gl == 0 && !perm_.get();
    MCG_CHECK(opt_.carry != 1 || ok,
              "line-carry pass needs SELL d16/c8, interleaved pairs, rows <= param <= 8 and whole 64-row grid lines");
    if (ok && opt_.carry != 0) {
      const int64_t S = gl / 64;
      // auto grid: 8 blocks per CU (two rounds of resident blocks, so CUs that finish early take more
      // jobs) when the launch has >= 4096 lines, else 4 (shorter runs would re-read their prologue
      // lines too often): 16384^2 509-516 vs 500-508 it/s, 4096^2 7224 vs 7028, a P = 8 rank's 2048
      // lines 3919 at 4 vs 3850 at 8 (profiles/r2s6_carry_grid.md)
      auto apply = [&](TileRanges& t, int& grid) {
        if (t.ntiles == 0 || t.nt0 != t.ntiles || t.b0 % S != 0 || t.nt0 % S != 0 || t.nt0 / S < 2) return false;
        t.strip = (int32_t)S;
        grid = ncu_ * (t.nt0 / S >= 4096 ? 8 : 4);
        return true;
      };
      // the specialised pass (no slow path) when every stored offset is carried: 0, +-1, +-one line
      // 3-D: the carried line is a plane (N^2 rows) and +-N is a second carried offset
      carry_lo2_ = stencil_plane(spec_) > 0 ? (int32_t)stencil_line(spec_) : 0;
      carry_general_ = !c8_;
      for (int64_t off : dict_offsets_)
        if (off != 0 && off != 1 && off != -1 && off != 64 * S && off != -64 * S &&
            (carry_lo2_ == 0 || (off != carry_lo2_ && off != -carry_lo2_)))
          carry_general_ = true;
      if (carry_general_) carry_lo2_ = 0;
      // auto: only the specialised pass (2-D stencils); with the slow path (3-D's +-N gathers) it
      // measured slower than the generic pass (288 vs 311 it/s at 512^3, profiles/sweep_carry.log)
      if (opt_.carry == 1 || !carry_general_) carry_all_ = apply(tr_all_, g_all_);
      if (split_ && (opt_.carry == 1 || !carry_general_)) carry_int_ = apply(tr_int_, g_int_);
    }
    info_.carry = carry_all_ || carry_int_;
    // Ap recomputed instead of stored: the specialised 2-D pass over every owned line in one launch
    // (with a split launch the boundary rows' generic pass would need the stored Ap); 3-D: the plane
    // carry with +-N through LDS, on SELL-64/dia4 only
    const bool ar_any = opt_.ap_recompute != 0 && carry_all_ && !carry_general_ && c8_ && !split_ &&
                        tr_all_.b0 == 0 && tr_all_.strip > 0;
    const int kw = opt_.carry3_kw;
    const bool ar2 = ar_any && carry_lo2_ == 0 && info_.spmv_param <= 5;
    const bool ar3 = ar_any && carry_lo2_ > 0 && carry_lo2_ % 64 == 0 && info_.spmv_param <= 7 &&
                     opt_.carry_dia != 0 && (kw == 4 || kw == 8 || kw == 16) && carry_lo2_ % kw == 0 &&
                     (int64_t)carry_lo2_ * carry_lo2_ == gl;
    MCG_CHECK(opt_.carry_dia != 1 || ar2 || ar3,
              "carry_dia needs the Ap-recomputing line / plane carry (ap_recompute)");
    if ((ar2 || ar3) && opt_.carry_dia != 0 && n > 0) {  // SELL-64/dia4 from the c8 codes (replaces c4 + metadata)
      const int64_t ns = (n + 63) / 64;
      const int nslot = ar3 ? 7 : 5;
      dia4_.allocate(ns * 32 * nslot, "A", 256);
      dvals_.allocate(16, "A");
      const bool ok = kern::sell_to_dia4(sell_view(), (int)dict_offsets_.size(), (int64_t)tr_all_.strip * 64,
                                         ar3 ? (int64_t)carry_lo2_ : 0, dia4_.get(), dvals_.get(), s0_);
      MCG_CHECK(ok || opt_.carry_dia != 1, "carry_dia: the matrix is not a canonical 2-D 5-point / 3-D 7-point pattern");
      if (!ok) {
        dia4_.release();
        dvals_.release();
      }
    }
    ar3_ = ar3 && dia4_.get() != nullptr;
    ar_ = ar2 || ar3_;
    // every rank takes the same pass form: it decides the vectors the halo carries ({r, Ap} pairs or
    // r / Ap / p) and their widths (one all-reduce of a flag at setup, like pmat)
    if (use_comm_ && world_ > 1 && !all_ranks_agree_(ar_) && ar_) {
      ar_ = ar3_ = false;
      dia4_.release();
      dvals_.release();
    }
    MCG_CHECK(opt_.ap_recompute != 1 || ar_,
              "ap_recompute needs the specialised line-carry pass over all lines (2-D: c8, <= 5 entries per row; "
              "3-D: dia4, N a multiple of 64 and of carry3_kw)");
    // 4 waves per SIMD (one round of resident blocks)
    if (ar3_) g_all_ = std::max(1, ncu_ * 16 / kw);
    info_.ar3_kw = ar3_ ? kw : 0;
    info_.carry_xchg = info_.carry && carry_lo2_ > 0 &&
                       kern::carry_block_exchange_ok(info_.spmv_param, carry_lo2_, gl / 64);
  }
  if (ar_) {  // r and p in the plain ext layout (no {r, Ap} pairs); the pipelined generic pass reads pairs
    opt_.interleave = 0;
    pipe_ = false;
    info_.pipeline = false;
  }
  info_.ap_recompute = ar_;
  info_.interleave = opt_.interleave == 1;
  info_.dia4 = dia4_.get() != nullptr;
  // three-term form: the 2-D dia4 carry (the halo still carries r of the ghost lines: every rank
  // stores r on its first / last line in either form, so ranks need not agree on it)
  // auto: on for the 2-D line carry and the 3-D plane carry (whose three-term kernel spills a few
  // registers at 16-wave blocks and is still 15 % faster: profiles/r2s6_p3_16384.md)
  p3_ = ar_ && info_.dia4 && opt_.p3 != 0;
  // every rank takes the same form: it decides how many vectors the halo carries ({Ap, p} or {r, Ap, p})
  if (use_comm_ && world_ > 1 && !all_ranks_agree_(p3_)) p3_ = false;
  MCG_CHECK(opt_.p3 != 1 || p3_, "p3 needs the Ap-recomputing line / plane carry on SELL-64/dia4");
  info_.p3 = p3_;
  if (ar_ && !info_.dia4 && n > 0) {
    const int64_t ns = (n + 63) / 64;
    int64_t slots = 0;
    MCG_HIP(hipMemcpy(&slots, slice_ptr_.get() + ns, sizeof(int64_t), hipMemcpyDeviceToHost),
            "memcpy from device to host failed(A)");
    MCG_CHECK((slots >> 6) < ((int64_t)1 << 28) && info_.max_row_len < 16, "slice metadata overflows 28 bits");
    smeta_.allocate(ns, "A");
    kern::slice_meta(slice_ptr_.get(), ns, smeta_.get(), s0_);
  }
  allocate_vectors_();
  g_b_ = kern::grid_for((n + 1) / 2, 256, 4);  // residual update / dot kernels: 1024 blocks (best measured)
  info_.grid_a = g_all_;
  info_.grid_b = g_b_;
  const bool split = split_;
  fused_red_ = (opt_.recurrence == 1 && opt_.fused_reduce != 0) || opt_.recurrence == 2;
  auto groups = [](int g) { return (g + kern::kRedGroup - 1) / kern::kRedGroup; };
  // the boundary launch's partials start on a reduction-group boundary: round the interior grid up
  // (the extra blocks find no work in the grid-stride loops and contribute zero partials)
  if (split && fused_red_ && g_int_ > 0) g_int_ = groups(g_int_) * kern::kRedGroup;
  bnd_base_ = split ? g_int_ : 0;
  const int np = std::max({g_all_, split ? g_int_ + g_bnd_ : 0, g_b_, 1});
  pstride_ = np + 64;
  partials_.allocate((size_t)pstride_ * (opt_.recurrence >= 1 ? 4 : 1), "partials");
  st_.allocate(1, "state");
  MCG_HIP(hipMemsetAsync(partials_.get(), 0, partials_.bytes(), s0_), "device memset failed");
  MCG_HIP(hipMemsetAsync(st_.get(), 0, sizeof(CgState), s0_), "device memset failed");
  if (fused_red_) {
    red_groups_all_ = groups(g_all_);
    red_groups_split_ = split ? groups(g_int_) + groups(g_bnd_) : 0;
    red_groups_b_ = groups(g_b_);  // the pipelined update's grid
    red_l2s_ = std::max({red_groups_all_, red_groups_split_, red_groups_b_, 1});
    red_cnt_.allocate(red_l2s_ + 1, "partials");
    red_l2_.allocate((size_t)4 * red_l2s_, "partials");
    MCG_HIP(hipMemsetAsync(red_cnt_.get(), 0, red_cnt_.bytes(), s0_), "device memset failed");
    MCG_HIP(hipMemsetAsync(red_l2_.get(), 0, red_l2_.bytes(), s0_), "device memset failed");
  }
  info_.fused_reduce = fused_red_;
  MCG_HIP(hipStreamSynchronize(s0_), "device synchronize failed");

  info_.device_bytes = matrix_bytes + (size_t)(3 * n + 3 * L_.ext_len) * 8 + (rp64_.bytes());
  const double vec_a = 8.0 * (1 + 1 + 1 + 2 + 1);  // r, pold gathers (ideal), pnew, x rw, Ap
  const double vec_b = 24.0;                        // r rw, Ap
  info_.bytes_per_iter_model = (double)matrix_bytes + (vec_a + vec_b) * n;
  // single-reduction pass: gathers r, Ap, p (ideal 24), writes r, p, Ap 24; x rw 16 + p_{k-2} 8
  // every second pass (paired x updates) = 12 per pass
  if (opt_.recurrence == 1) info_.bytes_per_iter_model = (double)matrix_bytes + 60.0 * n;
  // pipelined: S reads w (ideal gathers) and writes q (16 B), U reads 7 and writes 6 vectors (104 B)
  if (opt_.recurrence == 2) info_.bytes_per_iter_model = (double)matrix_bytes + 120.0 * n;
  if (opt_.recurrence == 1) info_.device_bytes += (size_t)(3 * L_.ext_len - n) * 8;
  if (pmat_) {  // U: x rw, r rw, Ap r, p rw = 56 B; S: r, Ap 16 B + one pass over p (ideal gathers) 8 B
    info_.bytes_per_iter_model = (double)matrix_bytes + 80.0 * n;
    info_.device_bytes = matrix_bytes + (size_t)(4 * n + L_.ext_len) * 8 + rp64_.bytes();
  }
  if (ar3_) {  // r rw, p rw 32; x 12; Ap of 2 of kw lines written + read, edge rows 0.5; dia4 codes 3.5
    // three-term form: p_{k-1}, p_{k-2} read + p_k written 24, x 8, r + Ap of the outer lines / edges
    info_.bytes_per_iter_model = (double)dia4_.bytes() + ((p3_ ? 32.5 : 44.5) + (p3_ ? 24.0 : 16.0) / info_.ar3_kw) * n;
    info_.device_bytes = matrix_bytes + rp64_.bytes() + b_.bytes() + dia4_.bytes();
    for (DeviceBuffer<double>* v : vectors_()) info_.device_bytes += v->bytes();
  } else if (ar_) {  // r rw, p rw 32 B; x rw 16 + p_{k-2} 8 every second pass = 12; edge Ap 0.25; + the codes it streams
    const double streamed = info_.dia4 ? (double)dia4_.bytes() : (double)matrix_bytes;
    // three-term form: p_{k-1}, p_{k-2} read, p_k written 24 B; x rw every second pass 8; edge r + Ap 0.5
    info_.bytes_per_iter_model = streamed + (p3_ ? 32.5 : 44.25) * n;
    info_.device_bytes = matrix_bytes + rp64_.bytes() + b_.bytes() + dia4_.bytes() + smeta_.bytes();
    for (DeviceBuffer<double>* v : vectors_()) info_.device_bytes += v->bytes();
  }
  // vectors allocated with room for the placement probe's start offsets hold that headroom too
  for (DeviceBuffer<double>* v : vectors_()) info_.device_bytes += v->lead_capacity() * sizeof(double);
  probe_placement_();
  if (opt_.recurrence == 2) pick_pipe_order_();
  setup_done_ = true;
  setup_seconds_ = std::chrono::duration<double>(clk::now() - t0).count();
}

// Pipelined CG: which branch of the fork after U_{k-1} -- S_k or the all-reduce -- is enqueued first.
// A graph runs a node's first-created child on the parent's queue and the others on helper queues,
// and a dependency across queues costs 5-11 us here (rocprofv3 kernel trace, profiles/
// r3_pipelined_cg.md), so the longer branch stays on the launch queue.  Both are timed once (3
// launches after a warm-up; the all-reduce is collective, so every rank times it at this point of
// setup).  The order changes scheduling only, never the arithmetic: ranks may decide differently.
void GpuCgSolver::pick_pipe_order_() {
  pipe_ar_first_ = false;
  if (!(use_comm_ && opt_.overlap && !comm_->serialized())) return;
  Event a(true, true), b(true, true);
  auto time_us = [&](auto&& f) {
    f();
    MCG_HIP(hipEventRecord(a, s0_), "event record failed");
    for (int i = 0; i < 3; ++i) f();
    MCG_HIP(hipEventRecord(b, s0_), "event record failed");
    MCG_HIP(hipEventSynchronize(b), "event synchronize failed");
    float ms = 0.f;
    MCG_HIP(hipEventElapsedTime(&ms, a, b), "event elapsed time failed");
    return 1e3 * ms / 3.0;
  };
  const double t_s = time_us([&] { spmv_plain_(w_.get(), q_.get(), s0_); });
  const double t_ar = time_us([&] { comm_->allreduce_sum(st_.get()->red, 4, s0_); });
  pipe_ar_first_ = t_ar > t_s;
  info_.pipe_ar_first = pipe_ar_first_;
  info_.pipe_spmv_us = t_s;
  info_.pipe_allreduce_us = t_ar;
}

// true iff `mine` is true on every rank (one all-reduce of a flag at setup; not in the loop)
bool GpuCgSolver::all_ranks_agree_(bool mine) {
  if (!comm_->moves_data()) return mine;
  DeviceBuffer<double> f(1, "state");
  const double v = mine ? 1.0 : 0.0;
  MCG_HIP(hipMemcpyAsync(f.get(), &v, sizeof(double), hipMemcpyHostToDevice, s0_), "memcpy from host to device failed");
  comm_->allreduce_sum(f.get(), 1, s0_);
  double all = 0.0;
  MCG_HIP(hipMemcpyAsync(&all, f.get(), sizeof(double), hipMemcpyDeviceToHost, s0_), "memcpy from device to host failed");
  MCG_HIP(hipStreamSynchronize(s0_), "device synchronize failed");
  return all == (double)world_;
}

std::vector<DeviceBuffer<double>*> GpuCgSolver::vectors_() {
  return {&x_, &r_, &r1_, &Ap_, &Ap1_, &ra_[0], &ra_[1], &p_[0], &p_[1], &ape_[0], &ape_[1], &apx_[0], &apx_[1],
          &w_, &z_, &q_};
}

void GpuCgSolver::allocate_vectors_() {
  const int64_t n = L_.n_local();
  if (opt_.recurrence == 2) {  // pipelined: r, w, p, s gathered by SpMVs (ext); x, z, q owned
    x_.allocate(n, "x", 8);
    r_.allocate(L_.ext_len, "r", 8);
    w_.allocate(L_.ext_len, "r", 8);
    p_[0].allocate(L_.ext_len, "p", 8);
    Ap_.allocate(L_.ext_len, "Ap", 8);  // s = A p
    z_.allocate(n, "Ap", 8);
    q_.allocate(n, "Ap", 8);
    if (opt_.pipe_rr < 0) xe_.allocate(L_.ext_len, "x", 8);  // x in the ext layout for r = b - A x
    return;
  }
  if (pmat_) {  // split pass: r, Ap, x owned only; p once in the ext layout (the only gathered vector)
    x_.allocate(n, "x", 8);
    r_.allocate(n, "r", 8);
    Ap_.allocate(n, "Ap", 8);
    p_[0].allocate(L_.ext_len, "p", 8);
    return;
  }
  // with the placement probe, every vector gets room for leads up to kLeadCap (probe_placement_)
  const size_t cap = opt_.placement_tries > 1 && opt_.placement_leads > 1 && opt_.recurrence == 1 ? kLeadCap : 0;
  x_.allocate(n, "x", 8, 0, cap);
  if (ar_) {  // r, p by parity (ext layout); Ap only for slice edges (+ first / last / ghost lines at P > 1)
    r_.allocate(L_.ext_len, "r", 8, 0, cap);
    r1_.allocate(L_.ext_len, "r", 8, 0, cap);
    const int64_t ns = (n + 63) / 64;
    if (!ar3_ || p3_) {  // 3-D two-term: the slices' edge rows go through the ext-layout Ap like the outer lines
      // three-term form: the edge rows' r behind their Ap (F1Vectors::re_old / re_new)
      const int64_t per = p3_ ? 4 : 2;
      ape_[0].allocate(per * std::max<int64_t>(ns, 1), "Ap", 8);
      ape_[1].allocate(per * std::max<int64_t>(ns, 1), "Ap", 8);
    }
    if (use_halo_ || ar3_) {
      apx_[0].allocate(L_.ext_len, "Ap", 8);
      apx_[1].allocate(L_.ext_len, "Ap", 8);
    }
  } else if (opt_.interleave == 1) {  // single-reduction form, {r, Ap} pairs, double-buffered by parity
    ra_[0].allocate(2 * L_.ext_len, "r", 8, 0, cap);
    ra_[1].allocate(2 * L_.ext_len, "r", 8, 0, cap);
  } else if (opt_.recurrence == 1) {  // single-reduction form: r and Ap are gathered -> ext layout, double-buffered
    r_.allocate(L_.ext_len, "r", 8, 0, cap);
    Ap_.allocate(L_.ext_len, "Ap", 8, 0, cap);
    Ap1_.allocate(L_.ext_len, "Ap", 8, 0, cap);
    r1_.allocate(L_.ext_len, "r", 8, 0, cap);
  } else {
    r_.allocate(L_.ext_len, "r", 8);
    Ap_.allocate(n, "Ap", 8);
  }
  p_[0].allocate(L_.ext_len, "p", 8, 0, cap);
  p_[1].allocate(L_.ext_len, "p", 8, 0, cap);
}

// Physical placement of the vector streams.  The same stream kernel on the same sizes runs at
// 4.7-5.45 TB/s depending on the allocation (stable per allocation, re-drawn by a new one), and
// within one allocation the relative offset of two read streams moves it by ~5 % (4 KiB and
// 1-3 MiB offsets faster than 0, 32 KiB or 256 KiB: profiles/r1_placement_probe.md); the CG
// benches show the same ~10 % spread from one process to the next.  Here the single-reduction
// pass (both parities, full work) is timed on `placement_tries` allocations of the vector set --
// each allocated while the earlier ones are still held, so it gets other memory -- times
// `placement_leads` start offsets of each vector inside its allocation (multiples of 4 KiB and
// 1 MiB), and the fastest combination is kept.  Vector contents are scratch until reset().
void GpuCgSolver::probe_placement_() {
  info_.placement_sets = 1;
  info_.placement_gain = 1.0;
  if (opt_.placement_tries <= 1 || opt_.recurrence != 1 || pmat_) return;
  trace::Range tr_("mcg.placement");
  auto bufs = vectors_();
  size_t set_bytes = 0;
  for (auto* b : bufs) set_bytes += b->bytes();
  const int leads = std::max(1, opt_.placement_leads);
  // start offset (doubles) of buffer i in lead trial t: trial 0 all zero, then pseudo-random
  // multiples of 4 KiB (0..7) + 1 MiB (0..3)
  auto lead_of = [&](int t, size_t i) -> size_t {
    if (t == 0 || bufs[i]->lead_capacity() < kLeadCap) return 0;
    uint32_t h = (uint32_t)(t * 16 + (int)i + 1) * 2654435761u;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    return ((size_t)(h & 7) * 4096 + (size_t)((h >> 3) & 3) * (1u << 20)) / sizeof(double);
  };
  auto set_leads = [&](int t) {
    for (size_t i = 0; i < bufs.size(); ++i)
      if (bufs[i]->get()) bufs[i]->relead(lead_of(t, i));
  };
  auto time_pairs = [&]() {
    // k = 0, 1: both parities, no convergence test (check = 0), so every launch does its work
    MCG_HIP(hipEventRecord(ev_t0_, s0_), "event record failed");
    for (int r = 0; r < 2; ++r) {
      enqueue_f1_(2, 0, 0);
      enqueue_f1_(3, 0, 0);
    }
    MCG_HIP(hipEventRecord(ev_t1_, s0_), "event record failed");
    MCG_HIP(hipEventSynchronize(ev_t1_), "event synchronize failed");
    float ms = 0.f;
    MCG_HIP(hipEventElapsedTime(&ms, ev_t0_, ev_t1_), "event elapsed failed");
    return ms;
  };
  // this set: warm once, then each lead trial; leaves the set at its best trial
  auto probe_set = [&](int& best_t) {
    enqueue_f1_(2, 0, 0);
    enqueue_f1_(3, 0, 0);
    float b = 0.f;
    for (int t = 0; t < leads; ++t) {
      if (leads > 1) set_leads(t);
      const float ms = time_pairs();
      info_.placement_worst_ms = std::max(info_.placement_worst_ms, (double)ms);
      if (t == 0 || ms < b) {
        b = ms;
        best_t = t;
      }
    }
    if (leads > 1) set_leads(best_t);
    return b;
  };
  info_.placement_worst_ms = 0.0;
  probing_ = true;
  struct Unprobe {
    bool& f;
    ~Unprobe() { f = false; }
  } unprobe{probing_};
  int best_t = 0;
  float best = probe_set(best_t);
  std::vector<std::vector<DeviceBuffer<double>>> held;
  for (int t = 1; t < opt_.placement_tries; ++t) {
    size_t free_b = 0, total_b = 0;
    MCG_HIP(hipMemGetInfo(&free_b, &total_b), "device memory query failed");
    if (free_b < set_bytes + set_bytes / 4 + ((size_t)1 << 30)) break;
    std::vector<DeviceBuffer<double>> prev(bufs.size());
    for (size_t i = 0; i < bufs.size(); ++i) prev[i].swap(*bufs[i]);
    allocate_vectors_();
    int bt = 0;
    const float ms = probe_set(bt);
    ++info_.placement_sets;
    if (ms < best) {
      best = ms;
      best_t = bt;
    } else {
      for (size_t i = 0; i < bufs.size(); ++i) prev[i].swap(*bufs[i]);  // keep the earlier set
    }
    held.push_back(std::move(prev));
  }
  info_.placement_peak_bytes = 0;
  for (auto& set : held)
    for (auto& b : set) info_.placement_peak_bytes += b.bytes() + b.lead_capacity() * sizeof(double);
  held.clear();
  info_.placement_best_ms = best;
  info_.placement_lead_trial = best_t;
  info_.placement_gain = best > 0.f ? info_.placement_worst_ms / best : 1.0;
  MCG_HIP(hipMemsetAsync(partials_.get(), 0, partials_.bytes(), s0_), "device memset failed");
  MCG_HIP(hipMemsetAsync(st_.get(), 0, sizeof(CgState), s0_), "device memset failed");
  MCG_HIP(hipStreamSynchronize(s0_), "device synchronize failed");
}

void GpuCgSolver::reset() {
  trace::Range tr_("mcg.reset");
  MCG_CHECK(setup_done_, "solver not set up");
  const int64_t n = L_.n_local();
  hipStream_t s = s0_;
  // a halo prefetched by the last iteration may still be sending / receiving rows of r, Ap and p
  // on s1_: order the memsets below after it (no write of s0_ may race the side stream's RCCL)
  join_halo_();
  MCG_HIP(hipMemsetAsync(x_.get(), 0, x_.bytes(), s), "device memset failed(x)");
  for (DeviceBuffer<double>* v : {&Ap_, &r_, &ra_[0], &ra_[1], &ape_[0], &ape_[1], &apx_[0], &apx_[1], &w_, &z_, &q_})
    if (v->bytes()) MCG_HIP(hipMemsetAsync(v->get(), 0, v->bytes(), s), "device memset failed(r)");
  MCG_HIP(hipMemsetAsync(p_[0].get(), 0, p_[0].bytes(), s), "device memset failed(p)");
  MCG_HIP(hipMemsetAsync(p_[1].get(), 0, p_[1].bytes(), s), "device memset failed(p)");
  // r = b  (CUDACG.cu:248; x0 = 0 so r0 = b - A x0 = b, and p0 = r0 is formed by K_A at k = 0)
  MCG_HIP(hipMemsetAsync(st_.get(), 0, sizeof(CgState), s), "device memset failed");
  if (opt_.recurrence == 2) {
    // pipelined: r_0 = b, w_0 = A r_0, {gamma_0, delta_0} all-reduced; p = s = z = 0
    MCG_HIP(hipMemcpyAsync(r_.get() + L_.own_off, b_.get(), n * sizeof(double), hipMemcpyDeviceToDevice, s),
            "vector copy failed(r)");
    if (use_halo_) {
      double* v[1] = {r_.get()};
      comm_->halo_exchange(L_, v, 1, s);
    }
    spmv_plain_(r_.get(), w_.get() + L_.own_off, s);
    kern::cg_pipe_dots(r_.get() + L_.own_off, w_.get() + L_.own_off, n, partials_.get(), pstride_, g_b_, st_.get(), 0, s);
    if (use_comm_) {
      comm_->allreduce_sum(st_.get()->red, 4, s);
      comm_->allreduce_sum(&st_.get()->rr_new, 1, s);  // rr0 stays this rank's b.b (rr0_local)
    }
  } else if (pmat_) {
    // U_0 forms r_0 = b - 0 * Ap and p_0 = r_0 + 0 * p: r = b, Ap = 0, p = 0
    MCG_HIP(hipMemcpyAsync(r_.get(), b_.get(), n * sizeof(double), hipMemcpyDeviceToDevice, s),
            "vector copy failed(r)");
  } else if (opt_.interleave == 1) {
    // iteration 0 reads the parity-1 pairs: {r_{-1}, Ap_{-1}} = {b, 0}
    kern::pack_pairs(b_.get(), reinterpret_cast<double2*>(ra_[1].get()) + L_.own_off, n, s);
  } else if (opt_.recurrence == 1) {
    // iteration 0 reads parity-1 buffers: r_{-1} = b, Ap_{-1} = 0, p_{-1} = 0
    MCG_HIP(hipMemsetAsync(r1_.get(), 0, r1_.bytes(), s), "device memset failed(r)");
    if (Ap1_.bytes()) MCG_HIP(hipMemsetAsync(Ap1_.get(), 0, Ap1_.bytes(), s), "device memset failed(Ap)");
    MCG_HIP(hipMemcpyAsync(r1_.get() + L_.own_off, b_.get(), n * sizeof(double), hipMemcpyDeviceToDevice, s),
            "vector copy failed(r)");
  } else {
    MCG_HIP(hipMemcpyAsync(r_.get() + L_.own_off, b_.get(), n * sizeof(double), hipMemcpyDeviceToDevice, s),
            "vector copy failed(r)");
  }
  if (opt_.recurrence != 2) {
    kern::dot_partials(b_.get(), b_.get(), n, partials_.get(), g_b_, s);
    kern::cg_reduce(partials_.get(), g_b_, st_.get(), kReduceInit, 1, opt_.tol, s);
    if (use_comm_) comm_->allreduce_sum(&st_.get()->rr_new, 1, s);
  }
  MCG_HIP(hipStreamSynchronize(s), "compute norm2 failed(r)");
  if (opt_.rtol > 0) {  // relative stopping: tol = rtol * ||b|| (kernels take tol by value: re-capture)
    double rr0 = 0.0;
    MCG_HIP(hipMemcpy(&rr0, &st_.get()->rr_new, sizeof(double), hipMemcpyDeviceToHost),
            "memcpy from device to host failed(state)");
    const double tol = opt_.rtol * std::sqrt(rr0);
    if (tol != opt_.tol) {
      drop_graphs_();
    }
    opt_.tol = tol;
  }
  k_ = 0;
  finalized_ = false;
  halo_ready_for_ = -1;
  ghosts_for_ = -1;
}

void GpuCgSolver::enqueue_spmv_(int k, int which, int final_mode) {
  const int first = (k == 0) ? 1 : 0;
  double* pold = p_[(k + 1) & 1].get();
  double* pnew = p_[k & 1].get();
  const TileRanges& tr = which == 1 ? tr_int_ : (which == 2 ? tr_bnd_ : tr_all_);
  const int grid = which == 1 ? g_int_ : (which == 2 ? g_bnd_ : g_all_);
  double* part = partials_.get() + (which == 2 ? bnd_base_ : 0);
  if (grid == 0) return;
  const int64_t n = L_.n_local();
  if (opt_.format == 1) {
    const SellDev A = sell_view();
    kern::cg_spmv_fused_sell(A, r_.get(), pold, pnew, x_.get(), Ap_.get(), L_.own_off, tr, part, grid, st_.get(),
                             opt_.tol, first, final_mode, info_.spmv_param,
                             (d16_ ? 4 : 0) |
                                 (c8_ ? 8 : 0),
                             s0_);
  } else if (info_.idx64) {
    CsrDev<int64_t> A{rp64_.get(), cols_.get(), vals_.get(), n};
    kern::cg_spmv_fused<int64_t>(A, r_.get(), pold, pnew, x_.get(), Ap_.get(), L_.own_off, tr, part, grid,
                                 st_.get(), opt_.tol, first, final_mode, info_.spmv_variant, info_.spmv_param,
                                 s0_);
  } else {
    CsrDev<int32_t> A{rp32_.get(), cols_.get(), vals_.get(), n};
    kern::cg_spmv_fused<int32_t>(A, r_.get(), pold, pnew, x_.get(), Ap_.get(), L_.own_off, tr, part, grid,
                                 st_.get(), opt_.tol, first, final_mode, info_.spmv_variant, info_.spmv_param,
                                 s0_);
  }
}

void GpuCgSolver::enqueue_f1_(int k, int which, int final_mode, bool fused_red) {
  // the placement probe times the steady-state passes (k = 2, 3) with no first-pass special case
  // and no convergence test, on scratch contents
  const int first = (k == 0 && !probing_) ? 1 : 0;
  const int check = (k >= 2 && !probing_) ? 1 : 0;  // the reference never tests r_0
  const TileRanges& tr = which == 1 ? tr_int_ : (which == 2 ? tr_bnd_ : tr_all_);
  const int grid = which == 1 ? g_int_ : (which == 2 ? g_bnd_ : g_all_);
  double* part = partials_.get() + (which == 2 ? bnd_base_ : 0);
  if (grid == 0) return;
  kern::RedCtl rc;
  if (fused_red) {
    MCG_CHECK(fused_red_ && !final_mode, "in-kernel reduction not set up");
    rc.cnt = red_cnt_.get();
    rc.lvl2 = red_l2_.get();
    rc.l2s = red_l2s_;
    rc.top = red_l2s_;
    rc.base = which == 2 ? bnd_base_ : 0;
    rc.ngroups = which == 0 ? red_groups_all_ : red_groups_split_;
    rc.check = check;
    rc.first = first;
  }
  const int64_t n = L_.n_local();
  const bool odd = (k & 1) != 0;
  DeviceBuffer<double>& r_new = odd ? r1_ : r_;
  DeviceBuffer<double>& r_old = odd ? r_ : r1_;
  DeviceBuffer<double>& ap_new = odd ? Ap1_ : Ap_;
  DeviceBuffer<double>& ap_old = odd ? Ap_ : Ap1_;
  kern::F1Vectors v{r_old.get(), ap_old.get(), p_[(k + 1) & 1].get(), r_new.get(), ap_new.get(), p_[k & 1].get(),
                    x_.get()};
  v.p_fix = p_[1].get();
  v.ext_len = L_.ext_len;
  if (opt_.interleave == 1) {
    v.ra_old = reinterpret_cast<const double2*>(ra_[(k + 1) & 1].get());
    v.ra_new = reinterpret_cast<double2*>(ra_[k & 1].get());
  }
  const SellDev S = sell_view();
  if (ar_) {
    MCG_CHECK(which == 0, "Ap-recomputing carry: one launch per iteration");
    v.ra_old = nullptr;
    v.ra_new = nullptr;
    v.ap_old = apx_[(k + 1) & 1].get();
    v.ap_new = apx_[k & 1].get();
    v.ape_old = ape_[(k + 1) & 1].get();
    v.ape_new = ape_[k & 1].get();
    if (p3_) {
      const int64_t ns2 = 2 * std::max<int64_t>((n + 63) / 64, 1);
      v.re_old = ape_[(k + 1) & 1].get() + ns2;
      v.re_new = ape_[k & 1].get() + ns2;
    }
    if (ar3_) {
      kern::cg_carry_ar3(2, info_.ar3_kw, S, v, L_.own_off, tr,
                         carry_lo2_, use_halo_, part, pstride_, grid, st_.get(), opt_.tol, first, check, k, final_mode,
                         s0_, rc, p3_);
      return;
    }
    // three-term even passes: operands 2 lines ahead (chains of 3 registers, renamed by the 3-step unroll)
    // operand prefetch depth in lines: 3 (2-D: 318 vs 301 it/s at 2); the three-term even passes 2
    // (their chains of 3 registers are renamed by the 3-step unroll, profiles/r2s6_p3_16384.md)
    const int depth = ((k & 1) == 0 && p3_) ? 2 : 3;
    kern::cg_carry_ar(dia4_.get() ? 4 : 2, info_.spmv_param, depth, S, v,
                      L_.own_off, tr, part, pstride_, grid, st_.get(), opt_.tol, first, check, k, final_mode, s0_, rc,
                      p3_, 3);
    return;
  }
  if (!final_mode && ((which == 0 && carry_all_) || (which == 1 && carry_int_))) {
    kern::cg_fused1_carry(c8_ ? 2 : 1, info_.spmv_param,
                          carry_lo2_ > 0 ? 1 : 3, carry_general_,
                          carry_lo2_, info_.carry_xchg, S, v, L_.own_off, tr, part, pstride_, grid, st_.get(),
                          opt_.tol, first, check, k, s0_, rc);
    return;
  }
  if (win_doubles_ > 0 && !final_mode) {
    kern::cg_fused1_win(d16_ ? 1 : 0, info_.spmv_param, S, v, L_.own_off, tr, win_.get(), win_doubles_, part,
                        pstride_, grid, st_.get(), opt_.tol, first, check, k, s0_, rc);
    return;
  }
  const int fmt = opt_.format == 1 ? (c8_ ? 4 : (d16_ ? 3 : 1)) : 0;
  if (info_.idx64)
    kern::cg_fused1<int64_t>(fmt, info_.spmv_param, CsrDev<int64_t>{rp64_.get(), cols_.get(), vals_.get(), n}, S, v,
                             L_.own_off, tr, part, pstride_, grid, st_.get(), opt_.tol, first, check, final_mode, k,
                             s0_, pipe_, rc);
  else
    kern::cg_fused1<int32_t>(fmt, info_.spmv_param, CsrDev<int32_t>{rp32_.get(), cols_.get(), vals_.get(), n}, S, v,
                             L_.own_off, tr, part, pstride_, grid, st_.get(), opt_.tol, first, check, final_mode, k,
                             s0_, pipe_, rc);
}

void GpuCgSolver::enqueue_halo_f1_(int k, hipStream_t s) {
  // ghosts read by iteration k: {r, Ap} (or r and Ap) and p of iteration k-1 (parity (k+1)&1)
  const bool odd = (k & 1) != 0;
  double* vecs[3] = {(odd ? r_ : r1_).get(), (odd ? Ap_ : Ap1_).get(), p_[(k + 1) & 1].get()};
  int nv = 3;
  static const int widths[2] = {2, 1};
  const int* w = nullptr;
  if (opt_.interleave == 1) {
    vecs[0] = ra_[(k + 1) & 1].get();
    vecs[1] = p_[(k + 1) & 1].get();
    nv = 2;
    w = widths;
  }
  if (ar_) vecs[1] = apx_[(k + 1) & 1].get();  // Ap of the ghost lines: the owners' stored first / last line
  if (p3_ && k > 0) {  // three-term form: a ghost line's r is recovered from its p_{k-1}, p_{k-2} (both
                       // received); iteration 0 (two-term kernel) reads r_{-1} = b of the ghosts
    vecs[0] = vecs[1];
    vecs[1] = vecs[2];
    nv = 2;
  }
  comm_->halo_exchange(L_, vecs, nv, s, w);
}

void GpuCgSolver::enqueue_split_spmv_(int k, int which, bool fused_red, int part) {
  const int first = (k == 0) ? 1 : 0;
  const int check = (k >= 2) ? 1 : 0;
  const TileRanges& tr = which == 1 ? tr_int_ : (which == 2 ? tr_bnd_ : tr_all_);
  const int grid = which == 1 ? g_int_ : (which == 2 ? g_bnd_ : g_all_);
  if (grid == 0) return;
  kern::RedCtl rc;
  if (fused_red && part != 1) {  // the local half (part 1) writes no partials
    rc.cnt = red_cnt_.get();
    rc.lvl2 = red_l2_.get();
    rc.l2s = red_l2s_;
    rc.top = red_l2s_;
    rc.base = which == 2 ? bnd_base_ : 0;
    rc.ngroups = which == 0 ? red_groups_all_ : red_groups_split_;
    rc.check = check;
    rc.first = first;
  }
  const int64_t n = L_.n_local();
  double* pp = partials_.get() + (which == 2 ? bnd_base_ : 0);
  if (tiles_) {
    MCG_CHECK(part == 0, "tiles: one SpMV launch per iteration");
    kern::cg_split_spmv_tiles(tiles_view(), p_[0].get(), r_.get(), Ap_.get(), L_.own_off, pp, pstride_, grid, st_.get(),
                              opt_.tol, first, check, s0_, rc);
    return;
  }
  const int fmt = opt_.format == 1 ? (aligned_ ? 6 : (c8_ ? 4 : (d16_ ? 3 : 1))) : (info_.spmv_variant == 2 ? 5 : 0);
  const SellDev S = sell_view();
  if (info_.idx64)
    kern::cg_split_spmv<int64_t>(fmt, info_.spmv_param, CsrDev<int64_t>{rp64_.get(), cols_.get(), vals_.get(), n}, S,
                                 p_[0].get(), r_.get(), Ap_.get(), L_.own_off, tr, pp, pstride_, grid, st_.get(),
                                 opt_.tol, first, check, s0_, rc, part);
  else
    kern::cg_split_spmv<int32_t>(fmt, info_.spmv_param, CsrDev<int32_t>{rp32_.get(), cols_.get(), vals_.get(), n}, S,
                                 p_[0].get(), r_.get(), Ap_.get(), L_.own_off, tr, pp, pstride_, grid, st_.get(),
                                 opt_.tol, first, check, s0_, rc, part);
}

void GpuCgSolver::enqueue_iteration_split_(int k) {
  trace::Range tr_("mcg.iteration.split");
  const int64_t n = L_.n_local();
  const bool fr = fused_red_;
  CgState* st = st_.get();
  double* pv[1] = {p_[0].get()};
  // U_k: x, r_k, p_k of the owned rows
  kern::cg_split_update(x_.get(), r_.get(), Ap_.get(), p_[0].get() + L_.own_off, n, st, opt_.tol, k == 0 ? 1 : 0,
                        k >= 2 ? 1 : 0, 0, partials_.get(), pstride_, g_b_, s0_);
  int np = g_all_;
  if (use_halo_ && opt_.overlap && !L_.allgather) {
    MCG_HIP(hipEventRecord(ev_r_, s0_), "event record failed");
    MCG_HIP(hipStreamWaitEvent(s1_, ev_r_, 0), "stream wait failed");
    comm_->halo_exchange(L_, pv, 1, s1_);
    MCG_HIP(hipEventRecord(ev_h_, s1_), "event record failed");
    enqueue_split_spmv_(k, 1, fr);  // interior rows || ghosts of p_k on the side stream
    MCG_HIP(hipStreamWaitEvent(s0_, ev_h_, 0), "stream wait failed");
    enqueue_split_spmv_(k, 2, fr);
    np = g_int_ + g_bnd_;
  } else if (ag_overlap_) {
    // all-gather of p_k on the side stream || the own-block slots of every row; then the rest
    MCG_HIP(hipEventRecord(ev_r_, s0_), "event record failed");
    MCG_HIP(hipStreamWaitEvent(s1_, ev_r_, 0), "stream wait failed");
    comm_->halo_exchange(L_, pv, 1, s1_);
    MCG_HIP(hipEventRecord(ev_h_, s1_), "event record failed");
    enqueue_split_spmv_(k, 2, fr, 1);
    MCG_HIP(hipStreamWaitEvent(s0_, ev_h_, 0), "stream wait failed");
    enqueue_split_spmv_(k, 2, fr, 2);
    np = g_int_ + g_bnd_;
  } else {
    if (use_halo_) comm_->halo_exchange(L_, pv, 1, s0_);
    // all-gather layout: no interior rows (g_int_ = 0), every row in the boundary launch
    const bool split = use_halo_ && opt_.overlap;
    enqueue_split_spmv_(k, split ? 2 : 0, fr);
    if (split) np = g_int_ + g_bnd_;
  }
  if (!fr) kern::cg_reduce_f1(partials_.get(), pstride_, np, st, 0, k >= 2 ? 1 : 0, k == 0 ? 1 : 0, opt_.tol, s0_);
  if (use_comm_) comm_->allreduce_sum(st->red, 4, s0_);
}

void GpuCgSolver::enqueue_iteration_f1_(int k) {
  if (pmat_) {
    enqueue_iteration_split_(k);
    return;
  }
  trace::Range tr_("mcg.iteration.single_reduction");
  int np = g_all_;
  const bool fr = fused_red_;
  if (halo_ahead_) {
    ensure_ghosts_(k);
    enqueue_f1_(k, 0, 0, fr);  // every owned row in one pass (the line-carry pass at P > 1 too)
    // the next iteration's ghosts are this pass's outputs, final now: exchange them on the side
    // stream while the all-reduce runs (the join sits in front of the next pass)
    MCG_HIP(hipEventRecord(ev_r_, s0_), "event record failed");
    MCG_HIP(hipStreamWaitEvent(s1_, ev_r_, 0), "stream wait failed");
    enqueue_halo_f1_(k + 1, s1_);
    MCG_HIP(hipEventRecord(ev_h_, s1_), "event record failed");
    ghosts_for_ = k + 1;
    halo_pending_ = true;
  } else if (use_halo_ && opt_.overlap) {
    if (halo_ready_for_ != k) {
      MCG_HIP(hipEventRecord(ev_r_, s0_), "event record failed");
      MCG_HIP(hipStreamWaitEvent(s1_, ev_r_, 0), "stream wait failed");
      enqueue_halo_f1_(k, s1_);
      MCG_HIP(hipEventRecord(ev_h_, s1_), "event record failed");
    }
    enqueue_f1_(k, 1, 0, fr);  // interior rows || halo on the side stream
    MCG_HIP(hipStreamWaitEvent(s0_, ev_h_, 0), "stream wait failed");
    enqueue_f1_(k, 2, 0, fr);  // boundary rows (its last arriver finishes the reduction)
    np = g_int_ + g_bnd_;
    halo_ready_for_ = -1;
    if (prefetch_halo_) {
      // the next iteration's ghosts are this iteration's outputs, final now: exchange them while
      // this iteration's reduction + all-reduce and the next interior pass run
      MCG_HIP(hipEventRecord(ev_r_, s0_), "event record failed");
      MCG_HIP(hipStreamWaitEvent(s1_, ev_r_, 0), "stream wait failed");
      enqueue_halo_f1_(k + 1, s1_);
      MCG_HIP(hipEventRecord(ev_h_, s1_), "event record failed");
      halo_ready_for_ = k + 1;
    }
  } else if (use_halo_) {
    enqueue_halo_f1_(k, s0_);
    enqueue_f1_(k, 0, 0, fr);
  } else {
    enqueue_f1_(k, 0, 0, fr);
  }
  CgState* st = st_.get();
  if (!fr) kern::cg_reduce_f1(partials_.get(), pstride_, np, st, 0, k >= 2 ? 1 : 0, k == 0 ? 1 : 0, opt_.tol, s0_);
  if (use_comm_) comm_->allreduce_sum(st->red, 4, s0_);
}

// y = A x over the owned rows (x in the ext layout, ghosts in place): the format's plain SpMV
void GpuCgSolver::spmv_plain_(const double* x_ext, double* y, hipStream_t s) {
  const int64_t n = L_.n_local();
  if (tiles_) {
    kern::spmv_tiles(tiles_view(), x_ext, y, g_all_, s);
  } else if (opt_.format == 1) {
    kern::spmv_sell(sell_view(), x_ext, y, s);
  } else if (info_.idx64) {
    kern::spmv_csr<int64_t>(CsrDev<int64_t>{rp64_.get(), cols_.get(), vals_.get(), n}, x_ext, y, s);
  } else {
    kern::spmv_csr<int32_t>(CsrDev<int32_t>{rp32_.get(), cols_.get(), vals_.get(), n}, x_ext, y, s);
  }
}

// Pipelined CG iteration k (cg_pipe.hip): the all-reduce of {gamma_k, delta_k} (left local by the
// previous update or by a residual replacement) runs on the side stream while S_k = A w_k runs on
// the compute stream; the update U_k joins it.
void GpuCgSolver::enqueue_iteration_pipe_(int k) {
  trace::Range tr_("mcg.iteration.pipelined");
  const int64_t n = L_.n_local();
  CgState* st = st_.get();
  // the all-reduce needs only U_{k-1}: forked after it onto the side stream, joined before U_k;
  // the longer of the two branches is enqueued first (pick_pipe_order_)
  const bool ar_side = use_comm_ && k > 0 && opt_.overlap && !comm_->serialized();
  if (use_comm_ && k > 0 && !ar_side) comm_->allreduce_sum(st->red, 4, s0_);  // reset() left k = 0's global
  if (ar_side) MCG_HIP(hipEventRecord(ev_r_, s0_), "event record failed");
  auto fork_ar = [&] {
    MCG_HIP(hipStreamWaitEvent(s1_, ev_r_, 0), "stream wait failed");
    comm_->allreduce_sum(st->red, 4, s1_);
    MCG_HIP(hipEventRecord(ev_h_, s1_), "event record failed");
  };
  if (ar_side && pipe_ar_first_) fork_ar();
  if (use_halo_) {  // ghosts of w_k for S_k
    double* v[1] = {w_.get()};
    comm_->halo_exchange(L_, v, 1, s0_);
  }
  spmv_plain_(w_.get(), q_.get(), s0_);  // S_k (|| the all-reduce)
  if (ar_side && !pipe_ar_first_) fork_ar();
  if (ar_side) MCG_HIP(hipStreamWaitEvent(s0_, ev_h_, 0), "stream wait failed");
  kern::RedCtl rc;
  rc.cnt = red_cnt_.get();
  rc.lvl2 = red_l2_.get();
  rc.l2s = red_l2s_;
  rc.top = red_l2s_;
  rc.base = 0;
  rc.ngroups = red_groups_b_;
  rc.check = k >= 1 ? 1 : 0;  // the reference never tests r_0
  rc.first = k == 0 ? 1 : 0;
  const int64_t o = L_.own_off;
  kern::PipeVectors v{x_.get(), r_.get() + o, w_.get() + o, p_[0].get() + o, Ap_.get() + o, z_.get(), q_.get()};
  kern::cg_pipe_update(v, n, partials_.get(), pstride_, g_b_, st, opt_.tol, s0_, rc);
  const int rr = std::abs(opt_.pipe_rr);
  if (rr > 0 && (k + 1) % rr == 0) {
    // replacement of the auxiliary recurrences: w = A r, s = A p, z = A s (their drift removed; r
    // stays the CG recurrence residual, as in the reference); pipe_rr < 0 also replaces r = b - A x
    if (opt_.pipe_rr < 0) {
      double* xv[1] = {xe_.get()};
      MCG_HIP(hipMemcpyAsync(xe_.get() + o, x_.get(), n * sizeof(double), hipMemcpyDeviceToDevice, s0_),
              "vector copy failed(x)");
      if (use_halo_) comm_->halo_exchange(L_, xv, 1, s0_);
      spmv_plain_(xe_.get(), q_.get(), s0_);
      kern::sub_vec(b_.get(), q_.get(), r_.get() + o, n, s0_);
    }
    double* rv[1] = {r_.get()};
    if (use_halo_) comm_->halo_exchange(L_, rv, 1, s0_);
    spmv_plain_(r_.get(), w_.get() + o, s0_);
    double* pv[1] = {p_[0].get()};
    if (use_halo_) comm_->halo_exchange(L_, pv, 1, s0_);
    spmv_plain_(p_[0].get(), Ap_.get() + o, s0_);
    double* sv[1] = {Ap_.get()};
    if (use_halo_) comm_->halo_exchange(L_, sv, 1, s0_);
    spmv_plain_(Ap_.get(), z_.get(), s0_);
    kern::cg_pipe_dots(r_.get() + o, w_.get() + o, n, partials_.get(), pstride_, g_b_, st, 1, s0_);
  }
}

void GpuCgSolver::enqueue_iteration_(int k) {
  trace::Range tr_("mcg.iteration");
  if (opt_.recurrence == 2) {
    enqueue_iteration_pipe_(k);
    return;
  }
  if (opt_.recurrence == 1) {
    enqueue_iteration_f1_(k);
    return;
  }
  const int first = (k == 0) ? 1 : 0;
  double* pold = p_[(k + 1) & 1].get();
  int np = g_all_;
  if (use_halo_) {
    double* vecs[2] = {r_.get(), pold};
    if (opt_.overlap) {
      MCG_HIP(hipEventRecord(ev_r_, s0_), "event record failed");
      MCG_HIP(hipStreamWaitEvent(s1_, ev_r_, 0), "stream wait failed");
      comm_->halo_exchange(L_, vecs, 2, s1_);
      MCG_HIP(hipEventRecord(ev_h_, s1_), "event record failed");
      enqueue_spmv_(k, 1, 0);
      MCG_HIP(hipStreamWaitEvent(s0_, ev_h_, 0), "stream wait failed");
      enqueue_spmv_(k, 2, 0);
      np = g_int_ + g_bnd_;
    } else {
      comm_->halo_exchange(L_, vecs, 2, s0_);
      enqueue_spmv_(k, 0, 0);
    }
  } else {
    enqueue_spmv_(k, 0, 0);
  }
  CgState* st = st_.get();
  kern::cg_reduce(partials_.get(), np, st, kReduceA, first, opt_.tol, s0_);
  if (use_comm_) comm_->allreduce_sum(&st->pAp, 1, s0_);
  kern::cg_update_r(r_.get() + L_.own_off, Ap_.get(), L_.n_local(), partials_.get(), g_b_, st, 1,
                    s0_);
  kern::cg_reduce(partials_.get(), g_b_, st, kReduceB, first, opt_.tol, s0_);
  if (use_comm_) comm_->allreduce_sum(&st->rr_new, 1, s0_);
}

void GpuCgSolver::join_halo_() {
  if (!halo_pending_) return;
  MCG_HIP(hipStreamWaitEvent(s0_, ev_h_, 0), "stream wait failed");
  halo_pending_ = false;
}

void GpuCgSolver::ensure_ghosts_(int k) {
  const bool have = ghosts_for_ == k;
  join_halo_();
  if (have) return;
  enqueue_halo_f1_(k, s0_);  // not prefetched (first iteration, after a reset / resume / profile)
  ghosts_for_ = k;
}

void GpuCgSolver::drop_graphs_() {
  for (int g = 0; g < 2; ++g) {
    if (graph_exec_[g]) (void)hipGraphExecDestroy(graph_exec_[g]);
    if (graph_[g]) (void)hipGraphDestroy(graph_[g]);
    graph_exec_[g] = nullptr;
    graph_[g] = nullptr;
  }
}

// Captures 2 (kind 0) or graph_iters (kind 1) iterations starting at an even k_.  The passes
// depend on k only through its parity (and k >= 2), so one capture replays for every even k_.
void GpuCgSolver::capture_pair_(int kind) {
  hipStream_t s = s0_;
  const int iters = kind == 0 ? 2 : opt_.graph_iters;
  // halo_ahead: a graph starts with its ghosts in place (joined before the launch) and ends by
  // joining the prefetch of its last iteration, so every replay sees the same host-side state
  if (halo_ahead_) ensure_ghosts_(k_);
  MCG_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal), "graph capture failed");
  try {
    for (int j = 0; j < iters; ++j) enqueue_iteration_(k_ + j);
    join_halo_();
  } catch (...) {
    hipGraph_t g = nullptr;
    (void)hipStreamEndCapture(s, &g);
    if (g) (void)hipGraphDestroy(g);
    ghosts_for_ = -1;
    halo_pending_ = false;
    throw;
  }
  ghosts_for_ = halo_ahead_ ? k_ : -1;  // nothing captured has run yet
  halo_pending_ = false;
  MCG_HIP(hipStreamEndCapture(s, &graph_[kind]), "graph capture failed");
  MCG_HIP(hipGraphInstantiate(&graph_exec_[kind], graph_[kind], nullptr, nullptr, 0), "graph instantiate failed");
}

void GpuCgSolver::run_iterations(int count) {
  MCG_CHECK(setup_done_, "solver not set up");
  const int glong = opt_.graph_iters > 2 ? opt_.graph_iters : 0;
  while (count > 0) {
    if (opt_.use_graph && k_ >= 2 && (k_ % 2) == 0 && count >= 2) {
      const int kind = glong && count >= glong ? 1 : 0;
      if (!graph_exec_[kind]) {
        try {
          capture_pair_(kind);
        } catch (const Error& e) {
          std::fprintf(stderr, "[mcg] graph capture unavailable (%s: %s); running eagerly\n", e.what(),
                       e.detail().c_str());
          (void)hipGetLastError();
          opt_.use_graph = false;
          ++info_.graph_fallbacks;
          continue;
        }
      }
      if (halo_ahead_) ensure_ghosts_(k_);
      const hipError_t le = (k_ == opt_.fail_graph_launch_at) ? hipErrorInvalidValue  // test hook
                                                              : hipGraphLaunch(graph_exec_[kind], s0_);
      if (le != hipSuccess) {
        (void)hipGetLastError();
        // Only errors that hipGraphLaunch reports while validating its arguments, before it enqueues
        // any node, leave the state untouched; anything else may have run part of the graph (x, r, p
        // updated twice on replay) and is fatal, as is every error on a multi-rank run.
        const bool nothing_ran = le == hipErrorInvalidValue || le == hipErrorInvalidResourceHandle ||
                                 le == hipErrorOutOfMemory;
        if (!nothing_ran || world_ > 1) MCG_HIP(le, "graph launch failed");
        std::fprintf(stderr, "[mcg] graph launch failed (%s); running eagerly\n", hipGetErrorString(le));
        MCG_HIP(hipStreamSynchronize(s0_), "device synchronize failed");  // earlier launches may still run
        drop_graphs_();
        opt_.use_graph = false;
        ++info_.graph_fallbacks;
        continue;
      }
      const int done = kind == 0 ? 2 : glong;
      k_ += done;
      count -= done;
      if (halo_ahead_) ghosts_for_ = k_;  // prefetched by the graph's last iteration and joined
    } else {
      if (k_ == opt_.inject_nan_at) inject_fault_(k_);
      enqueue_iteration_(k_);
      ++k_;
      --count;
    }
  }
}

// Fault-injection hook: poison the residual entry of this rank's first row
// with a NaN just before iteration k (the r the iteration reads).  The NaN
// reaches the global dot products, every rank latches "breakdown" at the same
// iteration, and the run ends instead of silently iterating on garbage.
void GpuCgSolver::inject_fault_(int k) {
  static const double nan = std::numeric_limits<double>::quiet_NaN();
  if (L_.n_local() == 0 || rank_ != 0) return;
  double* r = opt_.recurrence == 2 ? r_.get() + L_.own_off
              : pmat_ ? r_.get()
              : opt_.interleave == 1 ? ra_[(k + 1) & 1].get() + 2 * L_.own_off  // .x of the first owned pair
                                     : ((opt_.recurrence == 1 && (k & 1) == 0) ? r1_.get() : r_.get()) + L_.own_off;
  MCG_HIP(hipMemcpyAsync(r, &nan, sizeof(double), hipMemcpyHostToDevice, s0_), "fault injection failed");
}

void GpuCgSolver::finalize() {
  if (k_ == 0 || finalized_) return;
  finalized_ = true;  // the single-reduction catch-up of a pending x term must run once
  if (ar_ && use_halo_) ensure_ghosts_(k_);  // the final r_m recomputes Ap_{m-1} over the ghost lines too
  else join_halo_();
  if (opt_.recurrence == 2) {  // gamma_m of the last update, all-reduced, decides the flag
    if (use_comm_) comm_->allreduce_sum(st_.get()->red, 4, s0_);
    kern::cg_pipe_final(st_.get(), opt_.tol, s0_);
    return;
  }
  if (pmat_) {  // U in final mode: r_m, x_m and ||r_m||^2, then latch
    kern::cg_split_update(x_.get(), r_.get(), Ap_.get(), p_[0].get() + L_.own_off, L_.n_local(), st_.get(), opt_.tol,
                          0, k_ >= 2 ? 1 : 0, 1, partials_.get(), pstride_, g_b_, s0_);
    kern::cg_reduce_f1(partials_.get(), pstride_, g_b_, st_.get(), 1, k_ >= 2 ? 1 : 0, 0, opt_.tol, s0_);
    if (use_comm_) comm_->allreduce_sum(st_.get()->red, 4, s0_);
    kern::cg_reduce_f1(partials_.get(), pstride_, 0, st_.get(), 2, 0, 0, opt_.tol, s0_);
    return;
  }
  if (opt_.recurrence == 1) {
    // r_m = r_{m-1} - a Ap_{m-1}, x_m = x_{m-1} + a p_{m-1}, exact ||r_m||^2, then latch
    enqueue_f1_(k_, 0, 1);
    kern::cg_reduce_f1(partials_.get(), pstride_, g_all_, st_.get(), 1, k_ >= 2 ? 1 : 0, 0, opt_.tol, s0_);
    if (use_comm_) comm_->allreduce_sum(st_.get()->red, 4, s0_);
    kern::cg_reduce_f1(partials_.get(), pstride_, 0, st_.get(), 2, 0, 0, opt_.tol, s0_);
    return;
  }
  enqueue_spmv_(k_, 0, 1);  // pold = p_{k-1}: the deferred x += alpha p
  kern::cg_reduce(partials_.get(), 0, st_.get(), kReduceFinal, 0, opt_.tol, s0_);
}

// Drain both streams.  With a watchdog the wait is bounded like the solve's polls: a collective
// whose peer never arrives (a dead or diverged rank in a multi-GPU bench) ends in an error that
// names the stall, and the communicator is aborted, instead of a silent hang.
void GpuCgSolver::synchronize() {
  if (opt_.watchdog_seconds > 0) {
    MCG_HIP(hipEventRecord(ev_sync_[1], s1_), "event record failed");
    MCG_HIP(hipEventRecord(ev_sync_[0], s0_), "event record failed");
    wait_bounded_(ev_sync_[1]);
    wait_bounded_(ev_sync_[0]);
  }
  MCG_HIP(hipStreamSynchronize(s1_), "device synchronize failed");
  MCG_HIP(hipStreamSynchronize(s0_), "device synchronize failed");
  if (use_comm_) comm_->check_async();
}

// Host wait on a poll event.  With a watchdog it polls (checking RCCL async errors) and gives
// up after opt_.watchdog_seconds without the event completing: a hung peer or collective then
// surfaces as an error on every rank instead of a silent hang.
void GpuCgSolver::wait_bounded_(hipEvent_t ev) {
  if (opt_.watchdog_seconds <= 0) {
    MCG_HIP(hipEventSynchronize(ev), "event synchronize failed");
    return;
  }
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  for (int spin = 0;; ++spin) {
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return;
    if (q != hipErrorNotReady) MCG_HIP(q, "event synchronize failed");
    if (use_comm_) comm_->check_async();
    if (std::chrono::duration<double>(clk::now() - t0).count() > opt_.watchdog_seconds) {
      if (use_comm_) comm_->abort();
      fail("watchdog: no progress", "poll interval exceeded " + std::to_string(opt_.watchdog_seconds) + " s");
    }
    if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

CgResult GpuCgSolver::solve(bool resume) {
  trace::Range tr_("mcg.solve");
  if (!resume) reset();
  MCG_HIP(hipEventRecord(ev_t0_, s0_), "event record failed");
  const int every = std::max(1, opt_.check_every);
  int c = 0;
  int next_ckpt = opt_.checkpoint_every > 0 ? k_ + opt_.checkpoint_every : -1;
  while (k_ < opt_.maxit) {
    const int chunk = std::min(every, opt_.maxit - k_);
    run_iterations(chunk);
    MCG_HIP(hipMemcpyAsync(&host_st_[c & 1], st_.get(), sizeof(CgState), hipMemcpyDeviceToHost, s0_),
            "memcpy from device to host failed(state)");
    MCG_HIP(hipEventRecord(ev_poll_[c & 1], s0_), "event record failed");
    if (c > 0) {
      wait_bounded_(ev_poll_[(c - 1) & 1]);
      if (host_st_[(c - 1) & 1].done) break;
      if (use_comm_) comm_->check_async();
    }
    if (next_ckpt >= 0 && k_ >= next_ckpt && k_ < opt_.maxit) {
      save_checkpoint(opt_.checkpoint_path);  // synchronises: a consistent state after k_ iterations
      next_ckpt = k_ + opt_.checkpoint_every;
    }
    ++c;
  }
  finalize();
  MCG_HIP(hipEventRecord(ev_t1_, s0_), "event record failed");
  synchronize();
  return result();
}

// ---- checkpoint / resume ----------------------------------------------------
namespace {
constexpr char kCkptMagic[8] = {'M', 'C', 'G', 'C', 'K', 'P', 'T', '3'};
struct CkptHeader {
  char magic[8];
  int32_t rank, world, recurrence, format;
  int32_t pass_form, pad_;  // bit 0: Ap recomputed, bit 1: three-term (the vectors hold different state)
  int64_t n_local, ext_len, row_begin, k;
  int64_t n_global;
  uint64_t seed;
  int32_t kind, rhs;        // ProblemKind, RhsKind
  int64_t nnz_local;
  uint64_t fingerprint;     // problem_fingerprint(): the matrix (user CSR: rowptr / cols / vals) and b
};
}  // namespace

void GpuCgSolver::save_checkpoint(const std::string& prefix) {
  MCG_CHECK(setup_done_, "solver not set up");
  MCG_CHECK(!prefix.empty(), "checkpoint path not set");
  synchronize();
  const std::string path = prefix + ".rank" + std::to_string(rank_);
  const std::string tmp = path + ".tmp";
  std::FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) fail("checkpoint write failed", tmp);
  CkptHeader h{};
  std::memcpy(h.magic, kCkptMagic, 8);
  h.rank = rank_;
  h.world = world_;
  h.recurrence = opt_.recurrence;
  h.format = info_.format;
  h.pass_form = (ar_ ? 1 : 0) | (p3_ ? 2 : 0);
  h.n_local = L_.n_local();
  h.ext_len = L_.ext_len;
  h.row_begin = L_.row_begin;
  h.k = k_;
  h.n_global = L_.n_global;
  h.seed = spec_.seed;
  h.kind = (int32_t)spec_.kind;
  h.rhs = (int32_t)spec_.rhs;
  h.nnz_local = info_.nnz_local;
  h.fingerprint = fingerprint_;
  bool ok = std::fwrite(&h, sizeof(h), 1, f) == 1;
  std::vector<char> host;
  auto dump = [&](const void* dev, size_t bytes) {
    if (!ok || bytes == 0) return;
    host.resize(bytes);
    MCG_HIP(hipMemcpy(host.data(), dev, bytes, hipMemcpyDeviceToHost), "memcpy from device to host failed(ckpt)");
    ok = std::fwrite(host.data(), 1, bytes, f) == bytes;
  };
  dump(st_.get(), sizeof(CgState));
  for (DeviceBuffer<double>* b : {&x_, &r_, &r1_, &p_[0], &p_[1], &Ap_, &Ap1_, &ra_[0], &ra_[1], &ape_[0], &ape_[1],
                                  &apx_[0], &apx_[1], &w_, &z_, &q_})
    dump(b->get(), b->bytes());
  ok = (std::fclose(f) == 0) && ok;
  if (!ok || std::rename(tmp.c_str(), path.c_str()) != 0) fail("checkpoint write failed", path);
}

void GpuCgSolver::load_checkpoint(const std::string& prefix) {
  MCG_CHECK(setup_done_, "solver not set up");
  // nothing of an earlier solve may still run on either stream (a pending halo writes ghost rows)
  synchronize();
  join_halo_();
  const std::string path = prefix + ".rank" + std::to_string(rank_);
  std::FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) fail("checkpoint read failed", path);
  CkptHeader h{};
  bool ok = std::fread(&h, sizeof(h), 1, f) == 1 && std::memcmp(h.magic, kCkptMagic, 8) == 0;
  ok = ok && h.rank == rank_ && h.world == world_ && h.recurrence == opt_.recurrence && h.format == info_.format &&
       h.pass_form == ((ar_ ? 1 : 0) | (p3_ ? 2 : 0)) &&
       h.n_local == L_.n_local() && h.ext_len == L_.ext_len && h.row_begin == L_.row_begin &&
       h.n_global == L_.n_global && h.seed == spec_.seed && h.kind == (int32_t)spec_.kind &&
       h.rhs == (int32_t)spec_.rhs && h.nnz_local == info_.nnz_local && h.fingerprint == fingerprint_;
  if (!ok) {
    std::fclose(f);
    fail("checkpoint does not match this problem/layout", path);
  }
  std::vector<char> host;
  auto load = [&](void* dev, size_t bytes) {
    if (!ok || bytes == 0) return;
    host.resize(bytes);
    ok = std::fread(host.data(), 1, bytes, f) == bytes;
    if (ok) MCG_HIP(hipMemcpy(dev, host.data(), bytes, hipMemcpyHostToDevice), "memcpy from host to device failed(ckpt)");
  };
  load(st_.get(), sizeof(CgState));
  for (DeviceBuffer<double>* b : {&x_, &r_, &r1_, &p_[0], &p_[1], &Ap_, &Ap1_, &ra_[0], &ra_[1], &ape_[0], &ape_[1],
                                  &apx_[0], &apx_[1], &w_, &z_, &q_})
    load(b->get(), b->bytes());
  std::fclose(f);
  if (!ok) fail("checkpoint truncated", path);
  k_ = (int)h.k;
  finalized_ = false;
  halo_ready_for_ = -1;
  ghosts_for_ = -1;
}

std::vector<std::pair<std::string, double>> GpuCgSolver::phase_profile(int iters) {
  MCG_CHECK(setup_done_, "solver not set up");
  MCG_CHECK(opt_.recurrence == 1, "phase_profile: single-reduction form only");
  trace::Range tr_("mcg.phase_profile");
  synchronize();
  join_halo_();
  halo_ready_for_ = -1;
  ghosts_for_ = -1;
  // the first of the `iters` iterations is not timed when iters > 1: it is the first launch of kernels
  // the timed loop does not use (the separate reduce, the serialised halo), which HIP loads lazily
  // (~8 ms once, ~770 us per iteration on a 10-iteration mean)
  if (pmat_) {  // split pass: update | ghosts of p | [own-block SpMV half] | SpMV (+ in-kernel reduce) | all-reduce,
                // serialised (with ag_overlap_ the own-block half runs before the all-gather here, so both
                // halves and the all-gather are timed on their own)
    Event q[6];
    for (Event& v : q) v = Event(true, true);
    double acc[5] = {0, 0, 0, 0, 0};
    double* pv[1] = {p_[0].get()};
    const bool fr = fused_red_ && red_groups_all_ > 0;
    for (int it = 0; it < iters; ++it) {
      const int k = k_;
      MCG_HIP(hipEventRecord(q[0].get(), s0_), "event record failed");
      kern::cg_split_update(x_.get(), r_.get(), Ap_.get(), p_[0].get() + L_.own_off, L_.n_local(), st_.get(),
                            opt_.tol, k == 0 ? 1 : 0, k >= 2 ? 1 : 0, 0, partials_.get(), pstride_, g_b_, s0_);
      MCG_HIP(hipEventRecord(q[1].get(), s0_), "event record failed");
      if (use_halo_) comm_->halo_exchange(L_, pv, 1, s0_);
      MCG_HIP(hipEventRecord(q[2].get(), s0_), "event record failed");
      if (ag_overlap_) enqueue_split_spmv_(k, 0, false, 1);
      MCG_HIP(hipEventRecord(q[3].get(), s0_), "event record failed");
      enqueue_split_spmv_(k, 0, fr, ag_overlap_ ? 2 : 0);
      if (!fused_red_)
        kern::cg_reduce_f1(partials_.get(), pstride_, g_all_, st_.get(), 0, k >= 2 ? 1 : 0, k == 0 ? 1 : 0, opt_.tol,
                           s0_);
      MCG_HIP(hipEventRecord(q[4].get(), s0_), "event record failed");
      if (use_comm_) comm_->allreduce_sum(st_.get()->red, 4, s0_);
      MCG_HIP(hipEventRecord(q[5].get(), s0_), "event record failed");
      synchronize();
      for (int j = 0; j < 5 && (it > 0 || iters == 1); ++j) {
        float t = 0.f;
        MCG_HIP(hipEventElapsedTime(&t, q[j].get(), q[j + 1].get()), "event elapsed failed");
        acc[j] += t;
      }
      ++k_;
    }
    const int nt = iters > 1 ? iters - 1 : iters;
    const char* nm[5] = {"update", "halo", "spmv_local", "spmv", "allreduce"};
    std::vector<std::pair<std::string, double>> out;
    double tot = 0;
    for (int j = 0; j < 5; ++j) {
      out.emplace_back(nm[j], nt > 0 ? 1e3 * acc[j] / nt : 0.0);
      tot += acc[j];
    }
    out.emplace_back("iteration", nt > 0 ? 1e3 * tot / nt : 0.0);
    return out;
  }
  Event e[6], h[2];
  for (Event& v : e) v = Event(true, true);
  for (Event& v : h) v = Event(true, true);
  const char* names[] = {"interior_or_all", "halo_side_stream", "boundary_wait", "boundary", "reduce", "allreduce",
                         "iteration"};
  double acc[7] = {0, 0, 0, 0, 0, 0, 0};
  auto ms = [](const Event& a, const Event& b) {
    float t = 0.f;
    MCG_HIP(hipEventElapsedTime(&t, a.get(), b.get()), "event elapsed failed");
    return (double)t;
  };
  const bool split = split_;
  for (int it = 0; it < iters; ++it) {
    const int k = k_;
    MCG_HIP(hipEventRecord(e[0].get(), s0_), "event record failed");
    if (split) {
      MCG_HIP(hipStreamWaitEvent(s1_, e[0].get(), 0), "stream wait failed");
      MCG_HIP(hipEventRecord(h[0].get(), s1_), "event record failed");
      enqueue_halo_f1_(k, s1_);
      MCG_HIP(hipEventRecord(h[1].get(), s1_), "event record failed");
      enqueue_f1_(k, 1, 0);
      MCG_HIP(hipEventRecord(e[1].get(), s0_), "event record failed");
      MCG_HIP(hipStreamWaitEvent(s0_, h[1].get(), 0), "stream wait failed");
      MCG_HIP(hipEventRecord(e[2].get(), s0_), "event record failed");
      enqueue_f1_(k, 2, 0);
    } else {
      MCG_HIP(hipEventRecord(h[0].get(), s0_), "event record failed");
      if (use_halo_) enqueue_halo_f1_(k, s0_);  // serialised here, so it is timed on its own
      MCG_HIP(hipEventRecord(h[1].get(), s0_), "event record failed");
      enqueue_f1_(k, 0, 0);
      MCG_HIP(hipEventRecord(e[1].get(), s0_), "event record failed");
      MCG_HIP(hipEventRecord(e[2].get(), s0_), "event record failed");
    }
    MCG_HIP(hipEventRecord(e[3].get(), s0_), "event record failed");
    const int np = split ? g_int_ + g_bnd_ : g_all_;
    kern::cg_reduce_f1(partials_.get(), pstride_, np, st_.get(), 0, k >= 2 ? 1 : 0, k == 0 ? 1 : 0, opt_.tol, s0_);
    MCG_HIP(hipEventRecord(e[4].get(), s0_), "event record failed");
    if (use_comm_) comm_->allreduce_sum(st_.get()->red, 4, s0_);
    MCG_HIP(hipEventRecord(e[5].get(), s0_), "event record failed");
    synchronize();
    ++k_;
    if (it == 0 && iters > 1) continue;  // warm-up: first launches of the kernels only this profile uses
    acc[0] += split ? ms(e[0], e[1]) : ms(h[1], e[1]);
    acc[1] += ms(h[0], h[1]);
    acc[2] += ms(e[1], e[2]);
    acc[3] += ms(e[2], e[3]);
    acc[4] += ms(e[3], e[4]);
    acc[5] += ms(e[4], e[5]);
    acc[6] += ms(e[0], e[5]);
  }
  const int nt = iters > 1 ? iters - 1 : iters;
  std::vector<std::pair<std::string, double>> out;
  for (int q = 0; q < 7; ++q) out.emplace_back(names[q], nt > 0 ? 1e3 * acc[q] / nt : 0.0);
  return out;
}

CgResult GpuCgSolver::result() {
  synchronize();
  CgState st;
  MCG_HIP(hipMemcpy(&st, st_.get(), sizeof(CgState), hipMemcpyDeviceToHost), "memcpy from device to host failed(state)");
  CgResult r;
  r.iterations = st.done ? st.conv_iter : st.iter;
  r.converged = st.converged != 0;
  r.breakdown = st.breakdown != 0;
  r.beta_clamps = st.clamps;
  r.rr0_local = st.rr0;
  r.rnorm = std::sqrt(st.done ? st.rr_final : (opt_.recurrence >= 1 ? st.red[3] : st.rr_new));
  r.setup_seconds = setup_seconds_;
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, ev_t0_, ev_t1_) == hipSuccess) r.solve_seconds = ms * 1e-3;
  (void)hipGetLastError();
  return r;
}

std::vector<double> GpuCgSolver::x_local() {
  synchronize();
  std::vector<double> h(L_.n_local());
  if (!h.empty())
    MCG_HIP(hipMemcpy(h.data(), x_.get(), h.size() * sizeof(double), hipMemcpyDeviceToHost),
            "memcpy from device to host failed(x)");
  return h;
}

double GpuCgSolver::true_residual_norm() {
  trace::Range tr_("mcg.true_residual");
  synchronize();
  const int64_t n = L_.n_local();
  DeviceBuffer<double> xe(L_.ext_len, "x", 8), y(n, "Ap", 8), out(1, "scalar");
  hipStream_t s = s0_;
  MCG_HIP(hipMemsetAsync(xe.get(), 0, xe.bytes(), s), "device memset failed");
  MCG_HIP(hipMemcpyAsync(xe.get() + L_.own_off, x_.get(), n * sizeof(double), hipMemcpyDeviceToDevice, s),
          "vector copy failed(x)");
  if (use_halo_) {
    double* v[1] = {xe.get()};
    comm_->halo_exchange(L_, v, 1, s);
  }
  spmv_plain_(xe.get(), y.get(), s);
  kern::xpby(b_.get(), -1.0, y.get(), n, s);  // y = b - A x
  kern::dot_partials(y.get(), y.get(), n, partials_.get(), g_b_, s);
  kern::sum_partials(partials_.get(), g_b_, out.get(), s);
  if (use_comm_) comm_->allreduce_sum(out.get(), 1, s);
  double h = 0.0;
  MCG_HIP(hipMemcpyAsync(&h, out.get(), sizeof(double), hipMemcpyDeviceToHost, s), "memcpy from device to host failed");
  MCG_HIP(hipStreamSynchronize(s), "device synchronize failed");
  return std::sqrt(h);
}

}  // namespace mcg
