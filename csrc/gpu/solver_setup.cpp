// GpuCgSolver setup: the local matrix in the chosen storage (CSR / SELL-64 d16, c8, dia4, aligned /
// L2-segment tiles), the pass-form dispatch, vector allocation and the placement probe.  The iteration
// engine is in solver.cpp, checkpoint / diagnostics / results in solver_io.cpp.
#include "mcg/solver.hpp"

#include <algorithm>
#include <cstdlib>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <thread>
#include <unordered_set>

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

// SELL-64/aligned for a user matrix (per-slice offset unions): a slice's slots are the sorted union
// of its 64 rows' column offsets (ext column - the row's own ext column), each row's value at its
// offset's slot and 0.0 elsewhere, so every slot's 64 gathers are one contiguous run of p.  The
// entries keep their order (ascending offset = ascending column), so the row sums are CSR's.
// Returns the total slots (64 per slot of every slice); fills the arrays when `fill`.
int64_t aligned_unions(const HostCsr& A, int64_t own_off, bool fill, std::vector<int64_t>* slice_ptr,
                       std::vector<int32_t>* soffs, std::vector<double>* vals) {
  const int64_t n = A.n_rows, ns = (n + 63) / 64;
  int64_t total = 0;
  std::vector<int32_t> u;
  if (fill) {
    slice_ptr->assign(ns + 1, 0);
    soffs->clear();
    vals->clear();
  }
  for (int64_t sl = 0; sl < ns; ++sl) {
    u.clear();
    const int64_t r0 = sl * 64, r1 = std::min(n, r0 + 64);
    for (int64_t i = r0; i < r1; ++i)
      for (int64_t k = A.rowptr[i]; k < A.rowptr[i + 1]; ++k) u.push_back((int32_t)(A.cols[k] - (own_off + i)));
    std::sort(u.begin(), u.end());
    u.erase(std::unique(u.begin(), u.end()), u.end());
    const int64_t w = (int64_t)u.size();
    if (fill) {
      const int64_t base = (int64_t)vals->size();
      soffs->insert(soffs->end(), u.begin(), u.end());
      vals->resize(base + 64 * w, 0.0);
      for (int64_t i = r0; i < r1; ++i)
        for (int64_t k = A.rowptr[i]; k < A.rowptr[i + 1]; ++k) {
          const int32_t off = (int32_t)(A.cols[k] - (own_off + i));
          const int64_t j = std::lower_bound(u.begin(), u.end(), off) - u.begin();
          (*vals)[base + 64 * j + (i - r0)] += A.vals[k];  // duplicates were summed on input already
        }
      (*slice_ptr)[sl + 1] = base + 64 * w;
    }
    total += 64 * w;
  }
  return total;
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
  info_.interleave = opt_.form.interleave == 1;

  // ---- A: count -> scan -> fill (owned rows, ext-local columns) ----
  // generated families on the device; a user matrix (kind Csr) from its host rows
  DeviceBuffer<int64_t> rp64(n + 1, "A");
  HostCsr user;
  const bool is_user = spec_.kind == ProblemKind::Csr;
  // ---- irregular sparsity: L2-segment COO tiles (the split pass's SpMV) ----
  // auto: the scrambled random SPD, or a user matrix that is not a grid stencil on the all-gather
  // layout (its columns are scattered over the whole vector); the same decision on every rank
  // (the spec and the layout kind are global)
  // tiles: the scrambled family, and non-stencil user matrices whose columns are scattered -- on the
  // all-gather layout, or with >= 1/4 of the entries beyond kFarOffset of their row (a global
  // property of the matrix, so every rank decides the same)
  const bool scattered_user = is_user && stencil_line(spec_) == 0 && spec_.csr != nullptr &&
                              (L_.allgather ||
                               (spec_.csr->far > 0 && 4 * spec_.csr->far >= spec_.csr->rowptr[spec_.csr->n]));
  tiles_ = opt_.recurrence >= 1 && (opt_.form.pmat != 0 || opt_.recurrence == 2) && opt_.form.tiles != 0 &&
           (opt_.form.tiles == 1 || scrambled(spec_) || scattered_user);
  if (is_user) {
    user = build_local_csr(spec_, L_);
    // a banded user matrix whose slices share few offsets: SELL-64/aligned with per-slice offset
    // unions (the generated wide random SPD's layout), when the unions cost <= 1.6 slots per
    // nonzero; the same decision on every rank (it implies the split pass and its ghost vectors)
    if (opt_.format == 1 && !tiles_ && stencil_line(spec_) == 0 && opt_.recurrence == 1 && opt_.form.pmat != 0 &&
        opt_.form.sell_aligned != 0) {
      const int64_t slots = n > 0 ? aligned_unions(user, L_.own_off, false, nullptr, nullptr, nullptr) : 0;
      const int64_t unnz = user.nnz();
      // a matrix with a one-byte (value, offset) dictionary streams 1 B per entry on c8 (sellc8): keep it
      bool small_dict = false;
      if (c8_) {  // distinct (value bits, offset) pairs in a hash set, stopping at the 257th
        struct PairHash {
          size_t operator()(const std::pair<uint64_t, int32_t>& e) const {
            return (size_t)(e.first * 0x9E3779B97F4A7C15ull ^ (uint64_t)(uint32_t)e.second);
          }
        };
        std::unordered_set<std::pair<uint64_t, int32_t>, PairHash> seen;
        seen.reserve(512);
        small_dict = true;
        for (int64_t i = 0; i < n && small_dict; ++i)
          for (int64_t k = user.rowptr[i]; k < user.rowptr[i + 1] && small_dict; ++k) {
            uint64_t vb = 0;
            std::memcpy(&vb, &user.vals[k], sizeof(vb));
            seen.emplace(vb, (int32_t)(user.cols[k] - (L_.own_off + i)));
            small_dict = seen.size() <= 256;
          }
      }
      user_aligned_ = opt_.form.sell_aligned == 1 ||
                      (!small_dict && unnz > 0 && (double)slots <= 1.6 * (double)unnz);
      if (use_comm_ && world_ > 1) user_aligned_ = all_ranks_agree_(user_aligned_);
      info_.aligned_fill = unnz > 0 ? (double)slots / (double)unnz : 0.0;
    }
    if (opt_.format == 1 && !tiles_ && !user_aligned_ && opt_.form.sell_sigma != 0 && n > 64 && (opt_.form.sell_sigma > 0 || stencil_line(spec_) == 0)) {
      // SELL-C-sigma (int32 columns): the windows never mix interior and boundary slices (auto: not
      // for a detected grid stencil, whose rows stay in grid order for the line / plane carry)
      const int64_t sig = opt_.form.sell_sigma > 1 ? (opt_.form.sell_sigma + 63) / 64 * 64 : 4096;
      std::vector<int64_t> cuts;
      if (use_halo_ && opt_.overlap && !L_.allgather) {
        cuts.push_back(std::min<int64_t>(n, (L_.interior_begin + 63) / 64 * 64));
        cuts.push_back(std::max<int64_t>(0, L_.interior_end / 64 * 64));
      }
      std::vector<int32_t> perm;
      if (sigma_sort(user, sig, cuts, opt_.form.sell_sigma > 0, perm)) {
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
  info_.idx64 = nnz >= ((int64_t)1 << 31) - 64 || opt_.hooks.force_idx64;

  size_t matrix_bytes = 0;
  if (tiles_) {
    tgeo_ = kern::tiles_geometry(n, L_.ext_len, std::max(10, std::min(22, opt_.form.tile_seg_log2)));
    MCG_CHECK(tgeo_.G <= kern::kTileMaxSegments, "tiles: too many column segments (raise tile_seg_log2)");
    tptr_.allocate(tgeo_.nblocks * tgeo_.G + 1, "A");
    MCG_HIP(hipMemsetAsync(tptr_.get(), 0, tptr_.bytes(), s0_), "device memset failed(A)");
    tidx_.allocate(std::max<int64_t>(nnz, 1), "A", 64);
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
    kern::TilesOut to;
    to.tptr = tptr_.get();
    to.idx = tidx_.get();
    for (int fill = 0; fill < 2; ++fill) {
      if (fill) {
        tvals_.allocate(std::max<int64_t>(nnz, 1), "A", 64);
        to.vals = tvals_.get();
      }
      if (is_user) kern::tiles_build_csr(rp64.get(), tc.get(), tv.get(), n, tgeo_, to, fill, s0_);
      else kern::tiles_build_gen(spec_, L_.row_begin, n, L_.col_lo, L_.pad, rp64.get(), tgeo_, to, fill, s0_);
      if (!fill && ntp > 0) {  // tile sizes -> offsets
        DeviceBuffer<int64_t> tmp(kern::scan_tmp_elems(ntp), "A");
        kern::scan_inclusive_i64(tptr_.get() + 1, ntp, tmp.get(), s0_);
      }
      MCG_HIP(hipStreamSynchronize(s0_), "device synchronize failed(A)");
    }
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
    aligned_ = (spec_.kind == ProblemKind::RandomSPD && spec_.spread > 0 && !spec_.scramble && opt_.recurrence == 1 &&
                opt_.form.pmat != 0 && opt_.form.sell_aligned != 0 &&
                (opt_.form.sell_aligned == 1 || randspd_aligned_fill(spec_) <= 1.6)) ||
               user_aligned_;
    std::vector<int64_t> h_sp;
    std::vector<int32_t> h_so;
    std::vector<double> h_sv;
    if (user_aligned_) {  // per-slice offset unions, built on the host from the user's rows
      aligned_unions(user, L_.own_off, true, &h_sp, &h_so, &h_sv);
      MCG_HIP(hipMemcpy(slice_ptr_.get(), h_sp.data(), (ns + 1) * sizeof(int64_t), hipMemcpyHostToDevice),
              "memcpy from host to device failed(A)");
    } else if (aligned_) {
      kern::randspd_aligned_widths(spec_, L_.row_begin, n, slice_ptr_.get(), s0_);
    } else {
      kern::sell_slice_widths(rp64.get(), n, slice_ptr_.get(), s0_);
    }
    if (!user_aligned_) {  // widths -> slot offsets (the host-built unions come scanned)
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
    if (user_aligned_) {
      if (!h_so.empty()) {
        MCG_HIP(hipMemcpy(soffs_.get(), h_so.data(), h_so.size() * sizeof(int32_t), hipMemcpyHostToDevice),
                "memcpy from host to device failed(A)");
        MCG_HIP(hipMemcpy(vals_.get(), h_sv.data(), h_sv.size() * sizeof(double), hipMemcpyHostToDevice),
                "memcpy from host to device failed(A)");
      }
    } else if (aligned_) {
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
    if (!c8_ && !perm_.get() && !aligned_ && opt_.recurrence == 1 && opt_.form.window != 0 &&
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
      MCG_CHECK(opt_.form.window != 1 || fits, "windowed pass: a chunk's column window exceeds the LDS budget");
      if (fits && (opt_.form.window == 1 || dense_rows)) {
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
  pmat_ = opt_.recurrence == 1 && opt_.form.pmat != 0 &&
          (opt_.form.pmat == 1 || aligned_ || tiles_ || (win_doubles_ == 0 && !c8_ && (L_.allgather || nnz >= 32 * n)));
  // the pass form decides which ghost vectors are exchanged ({r, Ap} + p, or p alone): every rank
  // must take the same one, whatever its own rows look like
  if (use_comm_ && world_ > 1) pmat_ = all_ranks_agree_(pmat_);
  MCG_CHECK(!aligned_ || pmat_, "aligned SELL needs the split pass");
  MCG_CHECK(!tiles_ || pmat_ || opt_.recurrence == 2, "tiles need the split pass on every rank");
  info_.tiles = tiles_;
  info_.tile_segments = tiles_ ? tgeo_.G : 0;
  info_.tiles_tu = tiles_ ? tiles_view().tu : 0;
  if (pmat_) {
    opt_.form.interleave = 0;
    info_.interleave = false;
    prefetch_halo_ = false;
  }
  info_.pmat = pmat_;
  info_.allgather = L_.allgather;
  halo_ahead_ = opt_.form.halo_ahead != 0 && use_halo_ && opt_.overlap && !pmat_ && !L_.allgather && opt_.recurrence == 1;
  if (halo_ahead_) prefetch_halo_ = false;
  info_.halo_ahead = halo_ahead_;
  split_ = use_halo_ && opt_.overlap && !halo_ahead_;
  if (opt_.recurrence == 2) split_ = prefetch_halo_ = false;  // pipelined: the all-reduce is what overlaps
  // all-gather overlap: the own-block slots of each aligned slice are summed while p_k's all-gather
  // is in flight (aligned_ is decided from the spec and the layout is the same kind on every rank,
  // so every rank takes the same launches)
  ag_overlap_ = (aligned_ || tiles_) && pmat_ && use_halo_ && L_.allgather && opt_.overlap && opt_.form.ag_overlap != 0 &&
                n > 0;
  if (ag_overlap_ && tiles_) {
    // the segments wholly inside the own block [own_off, own_off + n) of p: final before the all-gather
    const int64_t S = (int64_t)1 << tgeo_.seg_shift;
    tg_lo_ = (int)std::min<int64_t>(tgeo_.G, (L_.own_off + S - 1) / S);
    tg_hi_ = (int)std::max<int64_t>(tg_lo_, std::min<int64_t>(tgeo_.G, (L_.own_off + n) / S));
    std::vector<int64_t> tp(tgeo_.nblocks * tgeo_.G + 1);
    MCG_HIP(hipMemcpy(tp.data(), tptr_.get(), tp.size() * sizeof(int64_t), hipMemcpyDeviceToHost),
            "memcpy from device to host failed(A)");
    int64_t loc = 0;
    for (int64_t b = 0; b < tgeo_.nblocks; ++b) loc += tp[b * tgeo_.G + tg_hi_] - tp[b * tgeo_.G + tg_lo_];
    info_.ag_local_frac = tp.back() > 0 ? (double)loc / (double)tp.back() : 0.0;
  } else if (ag_overlap_) {
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
  // tiles with the all-gather overlap run eagerly: replayed from a hipGraph the all-gather branch did
  // not start beside the own-segment half (a P = 8 share with a 2.3 ms all-gather: 18.6 it/s captured,
  // 19.3 eager = the same as with no all-gather at all, profiles/r4/c5ag); at ~50 ms an iteration the
  // launches cost nothing
  if (ag_overlap_ && tiles_) opt_.use_graph = false;

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
  pipe_ = opt_.form.pipeline != 0 && opt_.format == 1 && (d16_ || c8_) && opt_.form.interleave == 1 &&
          info_.max_row_len <= 8 && info_.spmv_param >= info_.max_row_len;
  MCG_CHECK(opt_.form.pipeline != 1 || pipe_, "pipelined pass needs SELL d16/c8, interleave and rows <= param <= 8");
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
    tile_ww_ = (opt_.form.tile_waves == 16 || opt_.form.tile_waves == 8) ? opt_.form.tile_waves : 4;
    MCG_CHECK(opt_.form.tile_waves == -1 || opt_.form.tile_waves == 4 || opt_.form.tile_waves == 8 ||
                  opt_.form.tile_waves == 16,
              "tile_waves: 4, 8 or 16 waves per workgroup");
    g_all_ = n > 0 ? kern::tiles_grid(ncu_, tile_ww_) : 0;
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
    // plain SELL-64 (int32 columns): a 3-D stencil whose +-plane offsets do not fit d16 and whose values
    // overflow c8 (variable coefficients at N >= 182) -- only the diav plane carry below can take it
    const bool plain3 = !d16_ && !c8_ && stencil_plane(spec_) > 0 && opt_.form.carry != 1;
    const bool ok = opt_.recurrence == 1 && opt_.format == 1 && (d16_ || c8_ || plain3) && opt_.form.interleave == 1 &&
                    win_doubles_ == 0 && info_.max_row_len <= 8 &&
                    info_.spmv_param >= info_.max_row_len && info_.spmv_param >= 4 && gl > 1 && gl % 64 == 0 &&
                    n % gl == 0 && L_.row_begin % gl == 0 && !perm_.get();
    MCG_CHECK(opt_.form.carry != 1 || ok,
              "line-carry pass needs SELL d16/c8, interleaved pairs, rows <= param <= 8 and whole 64-row grid lines");
    if (ok && opt_.form.carry != 0) {
      const int64_t S = gl / 64;
      // auto grid: 8 blocks per CU (two rounds of resident blocks, so CUs that finish early take more
      // jobs) when the launch has >= 4096 lines, else 4 (shorter runs would re-read their prologue
      // lines too often): 16384^2 509-516 vs 500-508 it/s, 4096^2 7224 vs 7028, a P = 8 rank's 2048
      // lines 3919 at 4 vs 3850 at 8 (profiles/r2s6_carry_grid.md)
      auto apply = [&](TileRanges& t, int& grid) {
        if (t.ntiles == 0 || t.nt0 != t.ntiles || t.b0 % S != 0 || t.nt0 % S != 0 || t.nt0 / S < 2) return false;
        t.strip = (int32_t)S;
        grid = ncu_ * (opt_.blocks_per_cu > 0 ? opt_.blocks_per_cu : (t.nt0 / S >= 4096 ? 8 : 4));
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
      // variable-coefficient 2-D 5-point stencil (no c8 dictionary: > 256 (value, offset) pairs):
      // SELL-64/diav, the per-row values streamed by the Ap-recomputing line carry
      if (!c8_ && carry_lo2_ == 0 && stencil_plane(spec_) == 0 && stencil_line(spec_) == gl &&
          info_.max_row_len <= 5 && opt_.form.carry_vc != 0 && opt_.form.ap_recompute != 0 && !split_ && n > 0 &&
          (n + gl) < ((int64_t)1 << 31)) {
        cv_len_ = n + gl;
        cv_.allocate(3 * cv_len_, "A", 64);
        if (kern::sell_to_diav(sell_view(), gl, cv_.get(), s0_)) {
          diav_ = true;
          carry_general_ = false;
        } else {
          cv_.release();
          cv_len_ = 0;
        }
      }
      // 3-D 7-point with variable coefficients: SELL-64/diav 3-D (four arrays, one plane in front) on
      // the plane carry's three-term lean loop (32-bit byte offsets: ranks below 2^29 rows)
      const int64_t ln3 = stencil_line(spec_);
      const int kwv = 8;  // the diav plane carry's blocks: 8 waves, 2 per SIMD
      if (!c8_ && !diav_ && stencil_plane(spec_) > 0 && ln3 >= 64 && ln3 % 64 == 0 && ln3 % kwv == 0 &&
          ln3 * ln3 == gl && info_.max_row_len <= 7 && opt_.form.carry_vc != 0 && opt_.form.ap_recompute != 0 &&
          opt_.form.p3 != 0 && !split_ && n > 0 && L_.ext_len < ((int64_t)1 << 29) && n + gl < ((int64_t)1 << 29)) {
        cv_len_ = n + gl;
        cv_.allocate(4 * cv_len_, "A", 64);
        if (kern::sell_to_diav(sell_view(), ln3, cv_.get(), s0_, gl)) {
          diav_ = diav3_ = true;
          carry_general_ = false;
          carry_lo2_ = (int32_t)ln3;
        } else {
          cv_.release();
          cv_len_ = 0;
        }
      }
      MCG_CHECK(opt_.form.carry_vc != 1 || diav_,
                "carry_vc: needs a symmetric 2-D 5-point / 3-D 7-point stencil without a c8 dictionary, ap_recompute "
                "on (3-D: p3 on, N a multiple of 64, ranks below 2^29 rows)");
      // auto: only the specialised pass (2-D stencils); with the slow path (3-D's +-N gathers) it
      // measured slower than the generic pass (288 vs 311 it/s at 512^3, profiles/sweep_carry.log).
      // Plain SELL-64 has no carry kernels of its own: only the diav conversion above makes it one
      const bool carry_ok = !plain3 || diav_;
      if (carry_ok && (opt_.form.carry == 1 || !carry_general_)) carry_all_ = apply(tr_all_, g_all_);
      if (carry_ok && split_ && (opt_.form.carry == 1 || !carry_general_)) carry_int_ = apply(tr_int_, g_int_);
    }
    info_.carry = carry_all_ || carry_int_;
    // Ap recomputed instead of stored: the specialised 2-D pass over every owned line in one launch
    // (with a split launch the boundary rows' generic pass would need the stored Ap); 3-D: the plane
    // carry with +-N through LDS, on SELL-64/dia4 only
    const bool ar_any = opt_.form.ap_recompute != 0 && carry_all_ && !carry_general_ && (c8_ || diav_) && !split_ &&
                        tr_all_.b0 == 0 && tr_all_.strip > 0;
    // blocks of 16 waves, 4 per SIMD (512^3: 714 vs 628 / 650-667 it/s at 4 / 8, profiles/r2_ar3_poisson512.md);
    // 3-D diav: 8 waves, 2 per SIMD (the streamed values need the registers; 557 vs 493 at 4, profiles/r4/vc)
    const int kw = diav3_ ? 8 : 16;
    const bool ar2 = ar_any && carry_lo2_ == 0 && info_.spmv_param <= 5;
    const bool ar3 = ar_any && carry_lo2_ > 0 && carry_lo2_ % 64 == 0 && info_.spmv_param <= 7 &&
                     (opt_.form.carry_dia != 0 || diav3_) && carry_lo2_ % kw == 0 && (int64_t)carry_lo2_ * carry_lo2_ == gl;
    MCG_CHECK(opt_.form.carry_dia != 1 || ar2 || ar3,
              "carry_dia needs the Ap-recomputing line / plane carry (ap_recompute)");
    if ((ar2 || ar3) && opt_.form.carry_dia != 0 && n > 0 && c8_) {  // SELL-64/dia4 from the c8 codes (replaces c4 + metadata)
      const int64_t ns = (n + 63) / 64;
      const int nslot = ar3 ? 7 : 5;
      dia4_.allocate(ns * 32 * nslot, "A", 256);
      dvals_.allocate(16, "A");
      const bool ok = kern::sell_to_dia4(sell_view(), (int)dict_offsets_.size(), (int64_t)tr_all_.strip * 64,
                                         ar3 ? (int64_t)carry_lo2_ : 0, dia4_.get(), dvals_.get(), s0_);
      MCG_CHECK(ok || opt_.form.carry_dia != 1, "carry_dia: the matrix is not a canonical 2-D 5-point / 3-D 7-point pattern");
      if (!ok) {
        dia4_.release();
        dvals_.release();
      } else if (opt_.form.dia_uniform != 0) {
        dpat_.allocate(ns, "A");
        const int64_t nu = kern::dia_patterns(dia4_.get(), dvals_.get(), ns, tr_all_.strip, nslot, dpat_.get(), s0_);
        info_.dia_uniform = ns > 0 ? (double)nu / (double)ns : 0.0;
      }
    }
    ar3_ = ar3 && (dia4_.get() != nullptr || diav3_);
    ar_ = ar2 || ar3_;
    // every rank takes the same pass form: it decides the vectors the halo carries ({r, Ap} pairs or
    // r / Ap / p) and their widths (one all-reduce of a flag at setup, like pmat)
    if (use_comm_ && world_ > 1 && !all_ranks_agree_(ar_) && ar_) {
      ar_ = ar3_ = false;
      dia4_.release();
      dvals_.release();
      dpat_.release();
      cv_.release();
      if (diav3_) {  // back to the d16 pass with the general carry (the 3-D stencil without the dictionary)
        carry_general_ = true;
        carry_lo2_ = 0;
        if (!d16_ && !c8_) carry_all_ = carry_int_ = info_.carry = false;  // plain SELL-64: the generic pass
      }
      diav_ = diav3_ = false;
      info_.dia_uniform = 0.0;
    }
    MCG_CHECK(opt_.form.ap_recompute != 1 || ar_,
              "ap_recompute needs the specialised line-carry pass over all lines (2-D: c8, <= 5 entries per row; "
              "3-D: dia4, N a multiple of 64)");
    // 4 waves per SIMD (one round of resident blocks; diav 3-D: 2).  Runs of planes per job column:
    // as many as make the jobs fill whole rounds of those blocks (a launch of 224 blocks over 256
    // jobs ran a second round for 32 of them: the 44 % that reserve_cus = 32 cost at 512^3,
    // profiles/r3_cumask_probe.md; 7 runs of 73 planes fill 8 rounds exactly)
    if (ar3_) {
      g_all_ = std::max(1, ncu_ * (diav3_ ? 8 : 16) / kw);
      const int64_t jpr = (int64_t)(carry_lo2_ / kw) * (carry_lo2_ / 64);
      // past 2^29 rows the lean runs keep their planes -3 .. end + 4 within 4 GiB of a per-run base
      const int64_t max_chunk = L_.ext_len >= ((int64_t)1 << 29) ? ((int64_t)1 << 32) / (gl * 8) - 8 : 0;
      tr_all_.runs3 = kern::carry3_runs(g_all_, jpr, n / gl, max_chunk);
    }
    info_.ar3_kw = ar3_ ? kw : 0;
    info_.ar3_runs = ar3_ ? tr_all_.runs3 : 0;
    info_.carry_xchg = info_.carry && carry_lo2_ > 0 &&
                       kern::carry_block_exchange_ok(info_.spmv_param, carry_lo2_, gl / 64);
  }
  if (ar_) {  // r and p in the plain ext layout (no {r, Ap} pairs); the pipelined generic pass reads pairs
    opt_.form.interleave = 0;
    pipe_ = false;
    info_.pipeline = false;
  }
  info_.ap_recompute = ar_;
  info_.interleave = opt_.form.interleave == 1;
  info_.dia4 = dia4_.get() != nullptr;
  // three-term form: the 2-D dia4 carry (the halo still carries r of the ghost lines: every rank
  // stores r on its first / last line in either form, so ranks need not agree on it)
  // auto: on for the 2-D line carry and the 3-D plane carry (whose three-term kernel spills a few
  // registers at 16-wave blocks and is still 15 % faster: profiles/r2s6_p3_16384.md)
  info_.diav = diav_;
  p3_ = ar_ && (info_.dia4 || diav_) && opt_.form.p3 != 0;
  // every rank takes the same form: it decides how many vectors the halo carries ({Ap, p} or {r, Ap, p})
  if (use_comm_ && world_ > 1 && !all_ranks_agree_(p3_)) p3_ = false;
  MCG_CHECK(opt_.form.p3 != 1 || p3_, "p3 needs the Ap-recomputing line / plane carry on SELL-64/dia4");
  info_.p3 = p3_;
  // lean-only three-term passes: every run of the launch takes the lean step, so the kernels
  // without the generic step run (cg_carry_ar.hip: LEAN = waves per SIMD the 2-D kernels are built
  // for; 3-D: LEAN); otherwise the generic kernels (no lean code: one kernel holding both measured
  // slower for each, profiles/r3/lean)
  lean_only_ = false;
  lean_depth_even_ = lean_depth_odd_ = 0;  // 0 = the lean kernels' default depth (3)
  if (p3_ && dpat_.get() != nullptr && n > 0 && tr_all_.strip > 0) {
    const int64_t nlines = (n + 63) / 64 / tr_all_.strip;
    int g = g_all_;
    if (!ar3_) {
      // 2-D: the largest grid of 16 / 8 / 4 blocks per CU whose runs keep >= 64 lines (shorter runs
      // re-read their prologue lines too often): 16384^2 16 per CU, 585.8 vs 581 it/s at 8; 4096^2
      // 4 per CU, 8592-8655 vs 7911-8484 at 8; a P = 8 share of 16384^2 8 per CU, within noise of 4
      // (profiles/r3/lean)
      int bpc_rule = 0;
      for (int bpc : {16, 8, 4}) {
        const int64_t waves = (int64_t)ncu_ * bpc * 4;  // 256-thread blocks
        if (nlines / std::max<int64_t>(1, waves / tr_all_.strip) >= 64) {
          g = ncu_ * bpc;
          bpc_rule = bpc;
          break;
        }
      }
      if (opt_.blocks_per_cu > 0) g = ncu_ * opt_.blocks_per_cu;  // fixed (tests: the generic pass's grid)
      // packed slice edges, the even passes on 5 or 6 blocks per CU (depth 3), the odd ones at depth 4 on
      // 4 (each on its own grid): r4 took it on the 4-blocks-per-CU grids (64-line runs: 4096^2 8441-8542
      // vs 8181-8188 it/s, profiles/r4/edge2); with three p buffers (p3buf) on every size below 2^29
      // rows: 16384^2 642-648 vs 612-615 on one grid of 16 per CU, a P = 8 share 4720 vs 4489, and 6 per
      // CU for the even passes where their runs keep >= 64 lines (the share 4826; 4096^2, 43-line runs:
      // 8346-8442 vs 8872-8982 at 5), profiles/r5/mix
      (void)bpc_rule;
      auto_mix_ = opt_.blocks_per_cu <= 0 && L_.ext_len < ((int64_t)1 << 29);
    }
    auto lean_ok = [&](int gg) {
      return kern::carry_lean_failures(dpat_.get(), tr_all_.strip, nlines, L_.ext_len, gg, ar3_ ? info_.ar3_kw : 0,
                                       ar3_ ? carry_lo2_ : 0, s0_, ar3_ ? tr_all_.runs3 : 0) == 0;
    };
    // the odd passes (x update paired in) on a grid of their own (auto_mix_): both grids' runs must qualify
    int go = g;
    if (auto_mix_) {
      const int64_t runs6 = std::max<int64_t>(1, (int64_t)ncu_ * 6 * 4 / tr_all_.strip);
      const int we = nlines / runs6 >= 64 ? 6 : 5;
      if (lean_ok(ncu_ * we) && lean_ok(ncu_ * 4)) {
        g = ncu_ * we;
        go = ncu_ * 4;
        lean_depth_even_ = opt_.hooks.lean_packed == 0 ? 0 : (we == 6 ? 15 : 13);
        lean_depth_odd_ = opt_.hooks.lean_packed == 0 ? 0 : 14;
      } else {
        auto_mix_ = false;
      }
    }
    const bool lean_all = lean_ok(g) && (go == g || lean_ok(go));
    // (at P > 1 too since r5: the r4 drift of a split rank next to a lean-only one was pass 0 running
    // on both launches, solver.cpp enqueue_pass_)
    if (!lean_all && !ar3_ && opt_.form.lean_split != 0 && !split_) {
      // some runs do not qualify: split the pass by run -- the lean kernels over the runs that do, the
      // generic ones over the rest, on the same grid (the same runs), when most runs qualify
      auto_mix_ = false;
      lean_depth_even_ = lean_depth_odd_ = 0;
      int64_t runs = 0, chunk = 0;
      kern::carry_jobs_host((int64_t)g * 4, tr_all_.strip, nlines, runs, chunk);
      const int64_t jobs = runs * tr_all_.strip;
      const int64_t fails = kern::carry_lean_failures(dpat_.get(), tr_all_.strip, nlines, L_.ext_len, g, 0, 0, s0_, 0);
      // auto: runs of >= 128 lines (each wave takes one run) -- 16384^2 (256-line runs) 548-557 it/s vs 514
      // all-generic with 3 changed rows; the 64-line runs of 4096^2 / 8192^2 lose (the few generic runs
      // sit on the critical path: 4855 vs 6816, 1819 vs 1938; profiles/r4/lsplit)
      const bool want = opt_.form.lean_split >= 1 || (2 * fails < jobs && chunk >= 128);
      // three p buffers on a split rank (T3 kernels, the packed-edge geometry: 4 blocks per CU): the lean launch
      // takes every lean stretch of its runs (whose lines match in the neighbouring columns too: it
      // recomputes their edge rows) and its first workgroups the ~3 lines around each odd slice, so it pays
      // on short runs as well (4096^2 with 3 odd rows: 8779 vs 6611 it/s on the generic kernels, uniform
      // 9715; profiles/r6/lsplit3): taken when at least 3/4 of the lines are lean, whatever the run length
      split_t3_lean_ = -1.0;
      if (opt_.form.p3buf != 0 && opt_.recurrence == 1 && info_.dia4 && !diav_ && opt_.blocks_per_cu <= 0 &&
          L_.ext_len < ((int64_t)1 << 29) && opt_.hooks.lean_packed != 0) {
        std::vector<int32_t> rng;
        if (kern::split_generic_ranges(dpat_.get(), tr_all_.strip, nlines, L_.ext_len, ncu_ * 4, 32, rng, s0_)) {
          int64_t glines = 0;
          for (size_t q = 0; q + 2 < rng.size(); q += 3) glines += rng[q + 2] - rng[q + 1];
          const double lean = 1.0 - (double)glines / (double)std::max<int64_t>(1, nlines * tr_all_.strip);
          if (opt_.form.lean_split >= 1 || lean >= 0.75) split_t3_lean_ = lean;
        }
      }
      if (jobs > 0 && ((want && fails < jobs) || split_t3_lean_ >= 0.0)) {
        lean_split_ = true;
        g_all_ = g;
        tr_int_ = tr_all_;
        tr_int_.lean_split = 1;
        tr_bnd_ = tr_all_;
        tr_bnd_.lean_split = 2;
        g_int_ = g_bnd_ = g;
        info_.lean_split = 1.0 - (double)fails / (double)jobs;
      }
    }
    if (lean_all) {
      lean_only_ = true;
      g_all_ = g;
      g_odd_ = go == g ? 0 : go;
      auto chunk_of = [&](int gg) {
        int64_t runs = 0, chunk = 0;
        kern::carry_jobs_host((int64_t)gg * 4, tr_all_.strip, nlines, runs, chunk);
        return (int32_t)chunk;
      };
      alt_chunk_even_ = g_odd_ > 0 ? chunk_of(g) : 0;
      alt_chunk_odd_ = g_odd_ > 0 ? chunk_of(go) : 0;
    }
  }
  if (p3_ && diav3_ && ar3_ && n > 0 && tr_all_.strip > 0 && opt_.form.dia_uniform != 0) {
    // 3-D diav: every run of the launch's job decomposition (k_cg_carry_ar3, tr_all_.runs3) >= 3 planes
    const int64_t ss = tr_all_.strip, nl = (n + 63) / 64 / ss;
    const int64_t jpr = (int64_t)(carry_lo2_ / info_.ar3_kw) * (carry_lo2_ / 64);
    const int64_t runs = tr_all_.runs3 > 0 ? tr_all_.runs3 : (g_all_ > jpr ? g_all_ / jpr : 1);
    const int64_t chunk = (nl + runs - 1) / runs;
    bool all = nl >= 4;
    for (int64_t r = 0; r < runs && all; ++r) {
      const int64_t l0 = r * chunk, l1 = std::min(nl, l0 + chunk);
      if (l0 < nl && l1 - l0 < 3) all = false;
    }
    lean_only_ = all;
    g_odd_ = 0;
  }
  if (p3_ && diav_ && !diav3_ && n > 0 && tr_all_.strip > 0 && opt_.form.dia_uniform != 0) {
    // diav: every run of >= 3 lines streams its coefficients in the lean loop (the same grids as the
    // dia4 2-D passes); checked here on the host from the launch's job decomposition
    const int64_t ss = tr_all_.strip, nlines = (n + 63) / 64 / ss;
    // every run of the launch must be >= 3 lines (within 4 GiB of byte offsets past 2^29 rows)
    auto all_lean = [&](int g) {
      const int64_t nw = (int64_t)g * 4, runs = nw > ss ? nw / ss : 1, chunk = (nlines + runs - 1) / runs;
      bool all = nlines >= 4 && L_.ext_len < ((int64_t)1 << 31) && (chunk + 8) * ss * 512 < ((int64_t)1 << 32);
      for (int64_t r = 0; r < runs && all; ++r) {
        const int64_t l0 = r * chunk, l1 = std::min(nlines, l0 + chunk);
        if (l0 < nlines && l1 - l0 < 3) all = false;
      }
      return all;
    };
    // the dia4 2-D grids (runs of >= 64 lines), else the largest smaller grid whose runs all qualify
    int g = 0;
    for (int bpc : {16, 8, 4})
      if (nlines / std::max<int64_t>(1, (int64_t)ncu_ * bpc * 4 / ss) >= 64) {
        g = ncu_ * bpc;
        break;
      }
    if (g == 0) g = g_all_;
    if (opt_.blocks_per_cu > 0) g = ncu_ * opt_.blocks_per_cu;
    for (int gg = g; gg >= 1 && !all_lean(gg); gg /= 2) g = gg / 2;
    if (g >= 1 && all_lean(g)) {
      lean_only_ = true;
      g_all_ = g;
      g_odd_ = 0;
    }
  }
  info_.lean_only = lean_only_;
  info_.lean_mix = auto_mix_ && lean_only_ && g_odd_ > 0 && opt_.hooks.lean_packed != 0;
  // three p buffers (PassForm::p3buf, T3 in cg_carry_ar.hip / cg_carry_ar3.hip): the lean three-term dia4
  // carries.  2-D: when every line's slices share one value pattern (a slice recomputes its
  // neighbours' edge rows with its own values); 2-D diav: r recovered, the edge rows' Ap stored.  3-D
  // (dia4 and diav): r recovered everywhere, the outer lines' and edge rows' Ap still stored.  Every rank the same (the in-kernel
  // halo maps the same buffer list on every rank)
  p3buf_ = false;
  if (opt_.form.p3buf != 0 && ar_ && p3_ && lean_only_ && !lean_split_ && opt_.recurrence == 1 && n > 0 &&
      tr_all_.strip > 0) {
    if (ar3_) p3buf_ = diav3_ || (info_.dia4 && dpat_.get() != nullptr);  // (diav: below 2^29 rows anyway)
    else if (info_.dia4 && !diav_ && dpat_.get() != nullptr)
      p3buf_ = kern::dia_lines_uniform(dpat_.get(), tr_all_.strip, (n + 63) / 64 / tr_all_.strip, s0_);
    else if (diav_) p3buf_ = L_.ext_len < ((int64_t)1 << 29);  // 2-D diav: r recovered, edge rows' Ap stored
  }
  // a split rank (r6): the lean T3 runs whose neighbouring columns match, the generic T3 kernels (edge rows
  // recomputed from their codes) over the rest
  // (on the packed-edge geometry only: its lean launch is the split kernel, COMBO, that takes the lean stretches)
  if (opt_.form.p3buf != 0 && ar_ && p3_ && lean_split_ && split_t3_lean_ >= 0.0 && opt_.recurrence == 1 && n > 0 &&
      opt_.blocks_per_cu <= 0 && L_.ext_len < ((int64_t)1 << 29) && opt_.hooks.lean_packed != 0)
    p3buf_ = true;
  if (use_comm_ && world_ > 1) p3buf_ = all_ranks_agree_(p3buf_);
  if (p3buf_ && lean_split_) {
    // the lean launch on the packed-edge kernels (EP, depth 4 at 4 waves per SIMD) over 4 blocks per CU for
    // both parities -- the lean-only odd passes' geometry; one grid, so one generic list serves both
    g_int_ = ncu_ * 4;  // (the packed-edge geometry: the p3buf condition above)
    lean_depth_even_ = lean_depth_odd_ = 14;
    // the lean launch takes every lean stretch of its runs, the generic launch only the lines around the odd
    // slices: a listed range (at most 32 lines) per wave, a small grid beside the lean launch
    const int64_t nlines = (n + 63) / 64 / tr_all_.strip;
    const int maxlen = opt_.hooks.gen_piece_lines > 0 ? opt_.hooks.gen_piece_lines : 32;
    std::vector<int32_t> rng;
    MCG_CHECK(kern::split_generic_ranges(dpat_.get(), tr_all_.strip, nlines, L_.ext_len, g_int_, maxlen, rng, s0_),
              "lean split: too many generic ranges");
    const int64_t ngen = (int64_t)rng.size() / 3;
    gen_list_.allocate(std::max<size_t>(rng.size(), 3), "generic runs");
    if (ngen > 0)
      MCG_HIP(hipMemcpy(gen_list_.get(), rng.data(), rng.size() * sizeof(int32_t), hipMemcpyHostToDevice),
              "memcpy from host to device failed(generic runs)");
    tr_int_.sub_ranges = tr_bnd_.sub_ranges = 1;
    tr_bnd_.gen_list = tr_int_.gen_list = gen_list_.get();
    tr_bnd_.ngen = tr_int_.ngen = (int32_t)ngen;
    g_bnd_ = (int)std::max<int64_t>(1, (ngen + 3) / 4);
    // default: one combined launch, the generic ranges' workgroups first (a second launch on the side stream
    // ran beside the lean one only when the graph put its branch on another hardware queue; on one stream
    // it added its whole ~22 us, profiles/r6/lsplit3); split_serial 0 / 1 keeps the two launches
    combo_ = ngen > 0 && opt_.hooks.split_serial < 0;
    if (combo_) {
      tr_int_.gen_blocks = (int32_t)(((ngen + 3) / 4 + 7) / 8 * 8);
      g_int_ += tr_int_.gen_blocks;
      g_bnd_ = 0;
    }
    int64_t glines = 0;
    for (int64_t q = 0; q < ngen; ++q) glines += rng[3 * q + 2] - rng[3 * q + 1];
    info_.lean_split = 1.0 - (double)glines / (double)std::max<int64_t>(1, nlines * tr_all_.strip);
  }
  MCG_CHECK(opt_.form.p3buf != 1 || p3buf_,
            "p3buf needs the lean three-term dia4 carry (2-D: one value pattern per line; 3-D: below 2^29 rows) on every rank");
  info_.p3buf = p3buf_;
  // in-kernel halo: the lean carries read their ghost lines / planes from the neighbours' rows and store
  // their own first / last ones write-through (carry_common.hpp PullBases), so an iteration from 2 on is
  // the pass + the all-reduce, no halo step.  The all-reduce orders the passes: a rank's pass k + 1
  // starts after every rank's pass k has finished (its sums are in the all-reduce), which is all the
  // pulled rows need -- p_{k-1} / Ap_{k-1} of the peer's first / last line sit in the buffers its pass k
  // does not write, and its pass k + 1 rewrites them only after this rank's pass k has contributed.
  // Every rank must take it (it decides the collectives of an iteration)
  {
    // (lean_split ranks too: their generic launch pulls and publishes like the lean one, cg_carry_ar.hip)
    const bool can = use_halo_ && ar_ && p3_ && (lean_only_ || lean_split_) && !L_.allgather && !pmat_ &&
                     opt_.recurrence == 1 && n > 0 && comm_ != nullptr &&
                     (comm_->maps_peers() || (opt_.form.halo_pull == 1 && !comm_->moves_data()));
    pull_ = opt_.form.halo_pull != 0 && can && (opt_.form.halo_pull == 1 || comm_->maps_peers());
    if (use_comm_ && world_ > 1) pull_ = all_ranks_agree_(pull_);
    MCG_CHECK(opt_.form.halo_pull != 1 || pull_,
              "halo_pull needs the lean line / plane carry on every rank (P > 1, a communicator that maps its peers)");
    info_.halo_pull = pull_;
  }
  // iterations that exchange a halo are captured only if the communicator's exchanges replay correctly
  // (the in-kernel halo's graphs hold none)
  if (use_halo_ && !pull_ && !comm_->halo_capturable()) opt_.use_graph = false;
  if (ar_ && !info_.dia4 && !diav_ && n > 0) {
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
  info_.graphs = opt_.use_graph;
  info_.grid_odd = g_odd_;
  info_.grid_b = g_b_;
  const bool split = split_ || lean_split_;
  fused_red_ = (opt_.recurrence == 1 && opt_.form.fused_reduce != 0) || opt_.recurrence == 2;
  auto groups = [](int g) { return (g + kern::kRedGroup - 1) / kern::kRedGroup; };
  // the boundary launch's partials start on a reduction-group boundary: round the interior grid up
  // (the extra blocks find no work in the grid-stride loops and contribute zero partials)
  // (lean_split: both launches keep the pass's grid -- the same runs -- and the boundary launch's
  // partials start at the next group boundary instead; the slots between are never read)
  if (split && fused_red_ && g_int_ > 0 && !lean_split_) g_int_ = groups(g_int_) * kern::kRedGroup;
  bnd_base_ = split ? ((fused_red_ && g_int_ > 0) ? groups(g_int_) * kern::kRedGroup : g_int_) : 0;
  const int np = std::max({g_all_, split ? bnd_base_ + g_bnd_ : 0, g_b_, g_odd_, 1});
  pstride_ = np + 64;
  partials_.allocate((size_t)pstride_ * (opt_.recurrence >= 1 ? 4 : 1), "partials");
  st_.allocate(1, "state");
  MCG_HIP(hipMemsetAsync(partials_.get(), 0, partials_.bytes(), s0_), "device memset failed");
  MCG_HIP(hipMemsetAsync(st_.get(), 0, sizeof(CgState), s0_), "device memset failed");
  if (fused_red_) {
    red_groups_all_ = groups(g_all_);
    red_groups_split_ = split ? groups(g_int_) + groups(g_bnd_) : 0;
    red_groups_b_ = groups(g_b_);  // the pipelined update's grid
    red_groups_odd_ = groups(g_odd_);
    red_l2s_ = std::max({red_groups_all_, red_groups_split_, red_groups_b_, red_groups_odd_, 1});
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
    // (diav 3-D: the four per-row value arrays, 32 B, instead of the codes)
    const double streamed = diav3_ ? 32.0 * n : (double)dia4_.bytes();
    info_.bytes_per_iter_model = streamed + ((p3_ ? 32.5 : 44.5) + (p3_ ? 24.0 : 16.0) / info_.ar3_kw) * n;
    info_.device_bytes = matrix_bytes + rp64_.bytes() + b_.bytes() + dia4_.bytes() + cv_.bytes();
    for (DeviceBuffer<double>* v : vectors_()) info_.device_bytes += v->bytes();
  } else if (ar_) {  // r rw, p rw 32 B; x rw 16 + p_{k-2} 8 every second pass = 12; edge Ap 0.25; + the codes it streams
    // dia4 codes; the three-term pass streams none over its lean runs (uniform slices)
    const double streamed = info_.dia4 ? (double)dia4_.bytes() * (p3_ ? 1.0 - info_.dia_uniform : 1.0)
                                       : (diav_ ? (diav3_ ? 32.0 : 24.0) * n : (double)matrix_bytes);
    // three-term form: p_{k-1}, p_{k-2} read, p_k written 24 B; x rw every second pass 8; edge r + Ap 0.5
    info_.bytes_per_iter_model = streamed + (p3_ ? 32.5 : 44.25) * n;
    info_.device_bytes = matrix_bytes + rp64_.bytes() + b_.bytes() + dia4_.bytes() + smeta_.bytes() + cv_.bytes();
    for (DeviceBuffer<double>* v : vectors_()) info_.device_bytes += v->bytes();
  }
  // vectors allocated with room for the placement probe's start offsets hold that headroom too
  for (DeviceBuffer<double>* v : vectors_()) info_.device_bytes += v->lead_capacity() * sizeof(double);
  probe_placement_();
  // the vectors a halo may carry, final now (after the placement probe): for a transport that maps
  // its peers' buffers (PeerHaloComm); the same list, in the same order, on every rank
  if (comm_ != nullptr) {
    if (use_halo_ && comm_->maps_peers()) xt_.allocate(L_.ext_len, "x", 8);
    halo_reg_.clear();
    for (DeviceBuffer<double>* b : {&r_, &r1_, &Ap_, &Ap1_, &p_[0], &p_[1], &ra_[0], &ra_[1], &apx_[0], &apx_[1], &w_, &xe_, &xt_,
                                    &p_[2]})
      if (b->get() != nullptr) halo_reg_.push_back(b->get());
    comm_->register_halo_buffers(halo_reg_, L_.own_off, L_.row_begin);
  }
  pull_mapped_ = false;
  if (opt_.recurrence == 2) pick_pipe_order_();
  setup_done_ = true;
  setup_seconds_ = std::chrono::duration<double>(clk::now() - t0).count();
}

// Pipelined CG: which branch of the fork after U_{k-1} -- S_k or the all-reduce -- is enqueued first.
// A graph runs a node's first-created child on the parent's queue and the others on helper queues,
// and a dependency across queues costs 5-11 us here (rocprofv3 kernel trace, profiles/
// r3_pipelined_cg.md), so the longer branch stays on the launch queue.  Both are timed once (3
// launches after a warm-up; the all-reduce is collective, so every rank times it at this point of
// setup, on a scratch buffer).  The order changes scheduling only, never the arithmetic, but every
// rank takes the same one (one all-reduce of the flag), so the halo and reduce communicators' kernels
// are enqueued in the same order everywhere.
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
  DeviceBuffer<double> scratch(4, "state");
  MCG_HIP(hipMemsetAsync(scratch.get(), 0, scratch.bytes(), s0_), "device memset failed");
  const double t_ar = time_us([&] { comm_->allreduce_sum(scratch.get(), 4, s0_); });
  MCG_HIP(hipStreamSynchronize(s0_), "device synchronize failed");
  pipe_ar_first_ = all_ranks_agree_(t_ar > t_s);
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
          &w_, &z_, &q_, &p_[2]};
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
  } else if (opt_.form.interleave == 1) {  // single-reduction form, {r, Ap} pairs, double-buffered by parity
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
  if (p3buf_) p_[2].allocate(L_.ext_len, "p", 8, 0, cap);
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
    // both parities, no convergence test (check = 0), so every launch does its work; three p buffers:
    // all six (parity, buffer rotation) combinations -- one rotation of the odd pass ran 15 % slower
    // than the other two on one box's allocation (2072 vs 1790 us, profiles/r5/final_prof), which
    // k = 2, 3 never time; probing all six: 651.5-652.2 vs 649.2-651.9 it/s (profiles/r5/probe6)
    MCG_HIP(hipEventRecord(ev_t0_, s0_), "event record failed");
    if (p3buf_) {
      for (int k = 2; k < 8; ++k) enqueue_f1_(k, 0, 0);
    } else {
      for (int r = 0; r < 2; ++r) {
        enqueue_f1_(2, 0, 0);
        enqueue_f1_(3, 0, 0);
      }
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

}  // namespace mcg
