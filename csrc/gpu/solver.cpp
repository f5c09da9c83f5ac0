// GpuCgSolver iteration engine: construction, reset, the per-recurrence iteration enqueue (two-
// reduction, single-reduction fused / carry / split, pipelined), hipGraph capture and replay, the
// bounded host waits, finalize and solve.  Setup is in solver_setup.cpp, checkpoint / diagnostics /
// results in solver_io.cpp.
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
    if (opt_.form.interleave < 0) opt_.form.interleave = ra_ok ? 1 : 0;
    MCG_CHECK(!opt_.form.interleave || ra_ok, "interleaved r/Ap layout needs the single-reduction recurrence on SELL");
  }
  use_comm_ = comm_ != nullptr && (world_ > 1 || opt_.force_comm);
  use_halo_ = use_comm_ && L_.has_halo();
  // one communicator for halo and all-reduce: every collective in one stream order on s0_
  if (use_comm_ && comm_->serialized()) opt_.overlap = false;
  if (use_comm_ && !comm_->graph_capturable()) opt_.use_graph = false;
  MCG_CHECK(opt_.graph_iters >= 2 && opt_.graph_iters % 2 == 0, "graph_iters must be even and >= 2");
  if (opt_.hooks.inject_nan_at >= 0) opt_.use_graph = false;  // the hook runs between eager iterations
  MCG_CHECK(opt_.recurrence >= -1 && opt_.recurrence <= 2, "recurrence must be -1 (auto), 0, 1 or 2 (pipelined)");
  // pipelined CG: a residual replacement every pipe_rr iterations is an eager step (no capture)
  if (opt_.recurrence == 2 && opt_.pipe_rr != 0) opt_.use_graph = false;
  // halo prefetch crosses iteration (and graph-launch) boundaries: eager runs only (and not for
  // the split pass, whose ghosts come from its own update kernel; decided in setup())
  prefetch_halo_ = use_halo_ && opt_.overlap && !opt_.use_graph && !L_.allgather;
  ncu_ = kern::num_cus();
  MCG_CHECK(opt_.reserve_cus >= 0 && opt_.reserve_cus <= ncu_ / 4, "reserve_cus must leave >= 3/4 of the CUs");
  if (opt_.reserve_cus > 0) {
    // withhold the top reserve_cus bits of the mask.  Bit i is CU slot i / 32 of shader engine (i / 8) % 4
    // of XCD i % 8 (__smid of a masked grid, profiles/r3_cumask_probe.md), so 32 withholds one CU per
    // shader engine: the dispatcher spreads a grid's blocks evenly over the XCDs and their SEs, and any
    // other count leaves some SE with fewer CUs for the same share of blocks
    std::vector<uint32_t> mask((ncu_ + 31) / 32, 0u);
    for (int i = 0; i < ncu_ - opt_.reserve_cus; ++i) mask[i / 32] |= 1u << (i % 32);
    s0_ = Stream::with_cu_mask(mask);  // (a blocking stream: the CU-mask create takes no flags, so it
                                       // also orders against the legacy null stream -- ordering only)
    ncu_ -= opt_.reserve_cus;
  } else {
    s0_ = Stream(true, 0);
  }
  s1_ = Stream(true, -1);  // comm stream at higher priority: halo kernels start first
  s2_ = Stream(true, -1);  // lean_split: the generic runs' launch beside the lean one
  ev_ls_[0] = Event(true);
  ev_ls_[1] = Event(true);
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
  if (s2_.get()) (void)hipStreamSynchronize(s2_);
  if (pull_host_) (void)hipHostFree(pull_host_);
}

void GpuCgSolver::reset() {
  trace::Range tr_("mcg.reset");
  MCG_CHECK(setup_done_, "solver not set up");
  // a halo prefetched by the last iteration may still be sending / receiving rows of r, Ap and p
  // on s1_: order the memsets below after it (no write of s0_ may race the side stream's RCCL)
  join_halo_();
  first_reset_checks_();  // (writes the p / apx lines and the state that reset_state_ clears)
  reset_state_();
}

void GpuCgSolver::first_reset_checks_() {
  if (pull_ && !pull_checked_) verify_pull_();
  if (!probed_) {
    probed_ = true;
    probe_transport_();
  }
}

void GpuCgSolver::reset_state_() {
  const int64_t n = L_.n_local();
  hipStream_t s = s0_;
  MCG_HIP(hipMemsetAsync(x_.get(), 0, x_.bytes(), s), "device memset failed(x)");
  for (DeviceBuffer<double>* v : {&Ap_, &r_, &ra_[0], &ra_[1], &ape_[0], &ape_[1], &apx_[0], &apx_[1], &w_, &z_, &q_})
    if (v->bytes()) MCG_HIP(hipMemsetAsync(v->get(), 0, v->bytes(), s), "device memset failed(r)");
  MCG_HIP(hipMemsetAsync(p_[0].get(), 0, p_[0].bytes(), s), "device memset failed(p)");
  MCG_HIP(hipMemsetAsync(p_[1].get(), 0, p_[1].bytes(), s), "device memset failed(p)");
  if (p_[2].bytes()) MCG_HIP(hipMemsetAsync(p_[2].get(), 0, p_[2].bytes(), s), "device memset failed(p)");
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
  } else if (opt_.form.interleave == 1) {
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
  pull_from_ = 2;
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
  // 2-D lean-only odd passes may run on a grid of their own (g_odd_, lean_bpc_odd)
  const bool odd_grid = which == 0 && g_odd_ > 0 && (k & 1) != 0 && !final_mode;
  const int grid = which == 1 ? g_int_ : (which == 2 ? g_bnd_ : (odd_grid ? g_odd_ : g_all_));
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
    rc.ngroups = which == 0 ? (odd_grid ? red_groups_odd_ : red_groups_all_) : red_groups_split_;
    rc.check = check;
    rc.first = first;
  }
  const int64_t n = L_.n_local();
  const bool odd = (k & 1) != 0;
  DeviceBuffer<double>& r_new = odd ? r1_ : r_;
  DeviceBuffer<double>& r_old = odd ? r_ : r1_;
  DeviceBuffer<double>& ap_new = odd ? Ap1_ : Ap_;
  DeviceBuffer<double>& ap_old = odd ? Ap_ : Ap1_;
  kern::F1Vectors v{r_old.get(), ap_old.get(), pbuf_(k - 1), r_new.get(), ap_new.get(), pbuf_(k), x_.get()};
  v.p_fix = p_[1].get();
  if (p3buf_) {  // three p buffers: p_k to a buffer this pass does not read (final mode reads p_{m-2} there)
    v.p_m2 = pbuf_(k - 2);
    if (final_mode) v.p_new = pbuf_(k - 2);
    for (int b = 0; b < 3; ++b) v.p_fix3[b] = p_[b].get();
  }
  v.ext_len = L_.ext_len;
  if (opt_.form.interleave == 1) {
    v.ra_old = reinterpret_cast<const double2*>(ra_[(k + 1) & 1].get());
    v.ra_new = reinterpret_cast<double2*>(ra_[k & 1].get());
  }
  const SellDev S = sell_view();
  if (ar_) {
    MCG_CHECK(which == 0 || lean_split_, "Ap-recomputing carry: one launch per iteration (lean_split: lean + generic runs)");
    // the launch runs the lean-only kernels: every run qualifies, or (lean_split) the lean half
    const bool lean_launch = lean_only_ || (lean_split_ && which == 1);
    // (lean_split: the generic launch runs on s2_, beside the lean one -- enqueue_pass_)
    const hipStream_t ls = (lean_split_ && which == 2 && opt_.hooks.split_serial <= 0) ? (hipStream_t)s2_ : (hipStream_t)s0_;
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
    if (pull_ && !probing_ && !final_mode) {  // in-kernel halo (carry_common.hpp PullBases)
      v.pull_pub = 1;
      if (k >= pull_from_) {
        MCG_CHECK(map_pull_(), "in-kernel halo: the peers' buffers are not mapped (attach the communicator)");
        const int pb = (k + 1) & 1;  // p_old / apx_old: the neighbours' pass k-1 outputs
        for (int sd = 0; sd < 2; ++sd) {
          v.pull_p[sd] = pull_p_[pidx_(k - 1)][sd];
          v.pull_ap[sd] = pull_ap_[pb][sd];
        }
      }
    }
    if (ar3_) {
      kern::cg_carry_ar3(2, info_.ar3_kw, S, v, L_.own_off, tr,
                         carry_lo2_, use_halo_, part, pstride_, grid, st_.get(), opt_.tol, first, check, k, final_mode,
                         s0_, rc, p3_, lean_only_);
      return;
    }
    // operand prefetch depth in lines: 3 (2-D: 318 vs 301 it/s at 2); the generic three-term even
    // passes 2 (their chains of 3 registers are renamed by the 3-step unroll, profiles/r2s6_p3_16384.md);
    // the lean ones 3 as well (4096^2 8191-8225 vs 8064-8084 it/s, 16384^2 586.4 vs 584.9,
    // profiles/r3/lean/README.md)
    const int ld = !lean_launch ? 0 : ((k & 1) != 0 ? lean_depth_odd_ : lean_depth_even_);
    if (g_odd_ > 0 && which == 0 && !final_mode) {
      // the two parities' runs differ: each pass also stores r on the other decomposition's run ends
      TileRanges ta = tr;
      ta.alt_chunk = (k & 1) != 0 ? alt_chunk_even_ : alt_chunk_odd_;
      kern::cg_carry_ar(dia4_.get() ? 4 : (cv_.get() ? 5 : 2), info_.spmv_param, ld > 0 ? ld : 3, S, v, L_.own_off, ta,
                        part, pstride_, grid, st_.get(), opt_.tol, first, check, k, final_mode, ls, rc, p3_, 3,
                        lean_launch);
      return;
    }
    const int depth = ((k & 1) == 0 && p3_ && !lean_launch) ? 2 : (lean_launch && ld > 0 ? ld : 3);
    kern::cg_carry_ar(dia4_.get() ? 4 : (cv_.get() ? 5 : 2), info_.spmv_param, depth, S, v,
                      L_.own_off, tr, part, pstride_, grid, st_.get(), opt_.tol, first, check, k, final_mode, ls, rc,
                      p3_, 3, lean_launch);
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
  double* vecs[3] = {(odd ? r_ : r1_).get(), (odd ? Ap_ : Ap1_).get(), pbuf_(k - 1)};
  int nv = 3;
  static const int widths[2] = {2, 1};
  const int* w = nullptr;
  if (opt_.form.interleave == 1) {
    vecs[0] = ra_[(k + 1) & 1].get();
    vecs[1] = pbuf_(k - 1);
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
  if (tiles_) {  // part 1 / 2: the own-block segments while p_k's all-gather is in flight / the rest
    kern::cg_split_spmv_tiles(tiles_view(), p_[0].get(), r_.get(), Ap_.get(), L_.own_off, pp, pstride_, grid, st_.get(),
                              opt_.tol, first, check, s0_, rc, part);
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
  if (use_halo_) comm_->halo_fence(s0_);  // U_k rewrites p_k's rows, which readers of exchange k-1 may still pull
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
    np = bnd_base_ + g_bnd_;
  } else if (ag_overlap_) {
    // all-gather of p_k on the side stream || the own-block slots of every row (tiles: the segments
    // inside the own block); then the rest
    MCG_HIP(hipEventRecord(ev_r_, s0_), "event record failed");
    MCG_HIP(hipStreamWaitEvent(s1_, ev_r_, 0), "stream wait failed");
    comm_->halo_exchange(L_, pv, 1, s1_);
    MCG_HIP(hipEventRecord(ev_h_, s1_), "event record failed");
    enqueue_split_spmv_(k, 2, fr, 1);
    MCG_HIP(hipStreamWaitEvent(s0_, ev_h_, 0), "stream wait failed");
    enqueue_split_spmv_(k, 2, fr, 2);
    np = bnd_base_ + g_bnd_;
  } else {
    if (use_halo_) comm_->halo_exchange(L_, pv, 1, s0_);
    // all-gather layout: no interior rows (g_int_ = 0), every row in the boundary launch
    const bool split = use_halo_ && opt_.overlap;
    enqueue_split_spmv_(k, split ? 2 : 0, fr);
    if (split) np = bnd_base_ + g_bnd_;
  }
  if (!fr) kern::cg_reduce_f1(partials_.get(), pstride_, np, st, 0, k >= 2 ? 1 : 0, k == 0 ? 1 : 0, opt_.tol, s0_);
  if (use_comm_) comm_->allreduce_sum(st->red, 4, s0_);
}

// one single-reduction pass over every owned row: one launch, or (lean_split) the lean kernels over
// the runs that qualify and then the generic ones over the rest, whose last arriver finishes the
// reduction.  Returns the number of block partials written.
int GpuCgSolver::enqueue_pass_(int k, bool fused_red) {
  // pass 0 (r_{-1} = b) runs the two-term generic kernel, which has no lean runs to leave to another
  // launch: one launch over every run.  (Two launches there each computed every run, so a split rank's
  // pass-0 sums came out doubled.  Harmless when every rank doubles -- alpha_0 and beta_0 are ratios of
  // the sums -- but a split rank next to a lean-only one all-reduced 2x + y: the r4 P > 1 drift,
  // profiles/r5/lsplit.)
  if (!lean_split_ || k == 0) {
    enqueue_f1_(k, 0, 0, fused_red);
    return (g_odd_ > 0 && (k & 1) != 0) ? g_odd_ : g_all_;
  }
  // the generic launch (few busy blocks: the runs that do not qualify) on the high-priority side
  // stream s2_ first, then the lean one on s0_: the generic runs overlap the lean pass instead of
  // following it.  The runs of one pass are independent (each reads the previous pass's vectors),
  // and the last arriver of either launch finishes the fused reduction.
  if (combo_) {  // one combined launch: the generic ranges' workgroups, then the lean ones (setup)
    enqueue_f1_(k, 1, 0, fused_red);
    return bnd_base_ + g_bnd_;
  }
  if (opt_.hooks.split_serial > 0) {  // the generic launch ahead of the lean one, one stream
    enqueue_f1_(k, 2, 0, fused_red);
    enqueue_f1_(k, 1, 0, fused_red);
    return bnd_base_ + g_bnd_;
  }
  MCG_HIP(hipEventRecord(ev_ls_[0], s0_), "event record failed");
  MCG_HIP(hipStreamWaitEvent(s2_, ev_ls_[0], 0), "stream wait failed");
  enqueue_f1_(k, 2, 0, fused_red);
  MCG_HIP(hipEventRecord(ev_ls_[1], s2_), "event record failed");
  enqueue_f1_(k, 1, 0, fused_red);
  MCG_HIP(hipStreamWaitEvent(s0_, ev_ls_[1], 0), "stream wait failed");
  return bnd_base_ + g_bnd_;
}

void GpuCgSolver::enqueue_iteration_f1_(int k) {
  if (pmat_) {
    enqueue_iteration_split_(k);
    return;
  }
  trace::Range tr_("mcg.iteration.single_reduction");
  int np = (g_odd_ > 0 && (k & 1) != 0) ? g_odd_ : g_all_;
  const bool fr = fused_red_;
  if (pull_) {
    // in-kernel halo: from pull_from_ on the pass reads its ghost lines from the neighbours' rows, so
    // the iteration is the pass and the all-reduce; before that (and for finalize) the ghosts are
    // exchanged in the serial order
    if (k >= pull_from_) {
      join_halo_();
      ghosts_for_ = -1;
    } else {
      ensure_ghosts_(k);
    }
    np = enqueue_pass_(k, fr);
  } else if (halo_ahead_) {
    ensure_ghosts_(k);
    np = enqueue_pass_(k, fr);  // every owned row in one pass (the line-carry pass at P > 1 too)
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
    np = bnd_base_ + g_bnd_;
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
    np = enqueue_pass_(k, fr);
  } else {
    np = enqueue_pass_(k, fr);
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
  if (use_halo_) comm_->halo_fence(s0_);  // the update rewrites w_, whose rows the readers may still pull
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
      np = bnd_base_ + g_bnd_;
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

// The in-kernel halo's pointers: for each p / apx buffer and side, the neighbour's buffer shifted so
// that this rank's ext index of a ghost row addresses the owner's copy of the same global row.  With a
// rehearsal communicator (no peers, no data moved) the rank's own first / last line stands in for the
// neighbours' (timing only, like NullComm's collectives).
// A layout or registration mismatch returns false like a missing mapping (verify_pull_ then turns the
// pull off on every rank through its agreement instead of one rank throwing before it).
bool GpuCgSolver::map_pull_() {
  if (pull_mapped_) return true;
  bool bad = false;
  auto idx = [&](const double* b) {
    auto it = std::find(halo_reg_.begin(), halo_reg_.end(), b);
    if (it == halo_reg_.end()) {
      bad = true;
      return (size_t)0;
    }
    return (size_t)(it - halo_reg_.begin());
  };
  const int64_t line = (int64_t)tr_all_.strip * 64;  // one grid line (2-D) / plane (3-D)
  for (int sd = 0; sd < 2; ++sd) {
    const HaloRange* h = nullptr;
    for (const HaloRange& r : L_.recvs)
      if (sd == 0 ? r.gbegin < L_.row_begin : r.gbegin >= L_.row_end) h = &r;
    for (int b = 0; b < 3; ++b) pull_p_[b][sd] = nullptr;
    for (int b = 0; b < 2; ++b) pull_ap_[b][sd] = nullptr;
    if (h == nullptr) continue;  // the first / last rank: no ghost on that side
    // the ghosts must be one whole line / plane next to the rank's rows
    if (h->count != line || !(sd == 0 ? h->gbegin + h->count == L_.row_begin : h->gbegin == L_.row_end)) return false;
    std::vector<double*> bufs;
    int64_t q_own = 0, q_rb = 0, src = 0;
    if (comm_->peer_view(h->peer, bufs, q_own, q_rb)) {
      if (bufs.size() != halo_reg_.size()) return false;  // the ranks registered different buffer lists
      src = q_own + (h->gbegin - q_rb);  // the owner's ext index of the first ghost row
    } else if (!comm_->moves_data() && opt_.hooks.pull_proxy == 1) {
      // rehearsal stand-in over PCIe: every pulled buffer's ghost line in pinned, coherent host memory
      // (5 buffers x 2 sides x one line), read by the pass's system-scope loads like a remote peer's rows
      if (pull_host_ == nullptr) {
        MCG_HIP(hipHostMalloc(reinterpret_cast<void**>(&pull_host_), (size_t)10 * line * sizeof(double),
                              hipHostMallocMapped | hipHostMallocCoherent),
                "host malloc failed(pull proxy)");
        std::memset(pull_host_, 0, (size_t)10 * line * sizeof(double));
      }
      const int64_t g0 = L_.ext_index(h->gbegin);
      for (int b = 0; b < 3; ++b)
        pull_p_[b][sd] = p_[b].bytes() ? pull_host_ + (int64_t)(5 * sd + b) * line - g0 : nullptr;
      for (int b = 0; b < 2; ++b) pull_ap_[b][sd] = pull_host_ + (int64_t)(5 * sd + 3 + b) * line - g0;
      continue;
    } else if (!comm_->moves_data()) {
      bufs = halo_reg_;  // rehearsal stand-in: this rank's own first / last line
      src = L_.own_off + (sd == 0 ? 0 : L_.n_local() - line);
    } else {
      return false;  // not mapped (a transport that was never attached, or whose mapping failed)
    }
    const int64_t shift = src - L_.ext_index(h->gbegin);
    for (int b = 0; b < 3; ++b)
      if (p_[b].bytes()) pull_p_[b][sd] = bufs[idx(p_[b].get())] + shift;
    for (int b = 0; b < 2; ++b) pull_ap_[b][sd] = bufs[idx(apx_[b].get())] + shift;
    if (bad) return false;  // a buffer the pass pulls was never registered
  }
  pull_mapped_ = true;
  return true;
}

// The in-kernel halo's check (the first reset, before the state is written; every rank takes part):
// each rank writes a pattern of its global row numbers into its first / last line of both p and both
// apx buffers, one all-reduce orders the ranks as the iterations will, and each rank reads its ghost
// lines back through the pull pointers with the pass's loads.  A rank that cannot map its peers, or
// reads a wrong value, turns it off on every rank: the halo is then exchanged, as before r5.  (A
// rehearsal communicator moves no data: its stand-in pointers are only mapped.)
void GpuCgSolver::verify_pull_() {
  pull_checked_ = true;
  const bool mapped = map_pull_();
  bool ok = all_ranks_agree_(mapped);
  if (ok && comm_->moves_data()) {
    const int64_t line = (int64_t)tr_all_.strip * 64, n = L_.n_local();
    DeviceBuffer<double>* bufs[5] = {&p_[0], &p_[1], &apx_[0], &apx_[1], &p_[2]};
    const int nb = p_[2].bytes() ? 5 : 4;
    std::vector<double> hv(line);
    auto pattern = [&](int64_t g0, int i) {
      for (int64_t t = 0; t < line; ++t) hv[t] = (double)(g0 + t) + 0.25 * i;
    };
    for (int i = 0; i < nb; ++i)
      for (int e = 0; e < 2 && n >= line; ++e) {
        const int64_t l0 = e == 0 ? 0 : n - line;
        pattern(L_.row_begin + l0, i);
        MCG_HIP(hipMemcpy(bufs[i]->get() + L_.own_off + l0, hv.data(), line * sizeof(double), hipMemcpyHostToDevice),
                "memcpy from host to device failed(pull check)");
      }
    MCG_HIP(hipDeviceSynchronize(), "device synchronize failed(pull check)");
    (void)all_ranks_agree_(true);  // every rank's pattern is in place (the order pass k -> pass k + 1 relies on)
    DeviceBuffer<double> got(line, "pull check");
    bool match = true;
    for (int sd = 0; sd < 2; ++sd)
      for (int i = 0; i < nb && pull_p_[0][sd] != nullptr; ++i) {
        const double* base = i == 4 ? pull_p_[2][sd] : (i < 2 ? pull_p_[i & 1][sd] : pull_ap_[i & 1][sd]);
        const int64_t g0 = sd == 0 ? L_.row_begin - line : L_.row_end;
        kern::pull_probe(base + L_.ext_index(g0), line, got.get(), s0_);
        MCG_HIP(hipMemcpyAsync(hv.data(), got.get(), line * sizeof(double), hipMemcpyDeviceToHost, s0_),
                "memcpy from device to host failed(pull check)");
        MCG_HIP(hipStreamSynchronize(s0_), "device synchronize failed(pull check)");
        for (int64_t t = 0; t < line && match; ++t) match = hv[t] == (double)(g0 + t) + 0.25 * i;
      }
    ok = all_ranks_agree_(match);
  }
  if (!ok) {
    if (rank_ == 0) std::fprintf(stderr, "[mcg] in-kernel halo check failed (peers not mapped, or a pulled row was wrong): "
                                         "the halo is exchanged instead\n");
    pull_ = false;
    info_.halo_pull = false;
    if (use_halo_ && !comm_->halo_capturable()) {
      drop_graphs_();
      opt_.use_graph = false;
      info_.graphs = false;
    }
  }
}

// Sum of n host doubles over the ranks (setup only: a device bounce through the communicator's
// all-reduce, then a sync).  Every rank gets the same bits, so a decision made from them is agreed.
void GpuCgSolver::allreduce_host_(double* v, int n) {
  if (!use_comm_ || !comm_->moves_data()) return;
  DeviceBuffer<double> d(n, "state");
  MCG_HIP(hipMemcpyAsync(d.get(), v, n * sizeof(double), hipMemcpyHostToDevice, s0_), "memcpy from host to device failed");
  comm_->allreduce_sum(d.get(), n, s0_);
  MCG_HIP(hipMemcpyAsync(v, d.get(), n * sizeof(double), hipMemcpyDeviceToHost, s0_), "memcpy from device to host failed");
  MCG_HIP(hipStreamSynchronize(s0_), "device synchronize failed");
}

namespace {
// the scalars of a run (every one the iterations wrote: equal bits = the same recurrence)
bool states_equal(const CgState& a, const CgState& b) {
  auto eq = [](double x, double y) { return std::memcmp(&x, &y, sizeof(double)) == 0; };
  bool ok = eq(a.rr_new, b.rr_new) && eq(a.rho, b.rho) && eq(a.pAp, b.pAp) && eq(a.a_prev, b.a_prev) &&
            eq(a.b_prev, b.b_prev) && a.iter == b.iter && a.done == b.done && a.breakdown == b.breakdown;
  for (int i = 0; i < 4; ++i) ok = ok && eq(a.red[i], b.red[i]);
  return ok;
}
bool states_close(const CgState& a, const CgState& b, double rel) {
  auto cl = [&](double x, double y) {
    if (std::isnan(x) || std::isnan(y)) return std::isnan(x) && std::isnan(y);
    return std::fabs(x - y) <= rel * std::max(std::fabs(x), std::fabs(y)) + 1e-300;
  };
  bool ok = cl(a.rr_new, b.rr_new) && cl(a.rho, b.rho) && cl(a.pAp, b.pAp) && a.iter == b.iter && a.done == b.done &&
            a.breakdown == b.breakdown;
  for (int i = 0; i < 4; ++i) ok = ok && cl(a.red[i], b.red[i]);
  return ok;
}
}  // namespace

// The transport probe (P > 1, the first reset, after verify_pull_): which halo and all-reduce the
// iterations use is chosen on the fabric the job runs on, from the same iterations timed both ways.
//   halo (halo_pull auto and verified): 2 + C untimed and C timed iterations from the same start with
//     the ghost lines pulled by the pass (PullBases) and with them exchanged before it (the
//     communicator's halo: RCCL's send/recv); C = the graph iterations of every replayed phase.  The
//     pulled run must end with the exchanged run's scalars bit for bit on every rank -- the real
//     test of the pull's ordering (a pass's write-through boundary stores -> kernel end -> the
//     all-reduce -> the neighbour's next pass), which verify_pull_'s memcpy'd pattern cannot be.
//   all-reduce (a mapped but unselected alternative, PeerHaloComm's IPC mailboxes): the same with the
//     halo chosen, its bounded wait cut to 10 s; it must match the first all-reduce's run to 1e-6
//     (the sums' order differs, RCCL's from rank order) with no time-out.
// Each rank's times and verdicts are summed over the ranks (one all-reduce on the first transport),
// so every rank takes the same choice from the mean times; info_.probe_* report them.  The state the
// arms leave is thrown away: reset_state_() follows.  Reference: the reduction sites CUDACG.cu:304,328
// and the SpMV's read of the neighbours' p, :288, which these transports carry.
void GpuCgSolver::probe_transport_() {
  info_.alt_allreduce = use_comm_ && comm_->alt_allreduce_in_use();
  // (not with a fault-injection hook armed: its iteration count refers to the real run)
  if (!use_comm_ || world_ < 2 || !comm_->moves_data() || opt_.transport_probe == 0 || opt_.hooks.inject_nan_at >= 0 ||
      opt_.hooks.fail_graph_launch_at >= 0)
    return;
  const bool halo_choice = pull_ && opt_.form.halo_pull == -1;  // (pull_ is agreed: the same on every rank)
  // the alternative all-reduce only if every rank mapped every mailbox (a rank whose mapping failed
  // must not leave the others running an arm it cannot)
  const bool ar_choice = all_ranks_agree_(comm_->alt_allreduce_ready() && !comm_->alt_allreduce_in_use());
  if (!halo_choice && !ar_choice) return;
  trace::Range tr_("mcg.transport_probe");
  const double tol0 = opt_.tol, rtol0 = opt_.rtol;
  const bool graph0 = opt_.use_graph;
  opt_.tol = -1.0;  // every probe iteration does its work (kernels take tol by value: fresh captures below)
  opt_.rtol = 0.0;
  const int cyc = graph0 ? (p3buf_ ? 3 : 1) * opt_.graph_iters : 16;
  struct Arm {
    double us = 0.0;
    CgState st{};
    bool timeout = false;
  };
  auto run_arm = [&](bool pull, bool alt) {
    Arm a;
    drop_graphs_();
    pull_ = pull;
    // (only a probed alternative is switched: a rehearsal's IPC all-reduce is its first and only one)
    if (ar_choice) comm_->use_alt_allreduce(alt);
    opt_.use_graph = graph0 && (pull || !use_halo_ || comm_->halo_capturable());
    reset_state_();
    run_iterations(2 + cyc);  // captures every graph the timed iterations replay
    MCG_HIP(hipEventRecord(ev_t0_, s0_), "event record failed");
    run_iterations(cyc);
    MCG_HIP(hipEventRecord(ev_t1_, s0_), "event record failed");
    if (alt) {  // (not synchronize(): its async check would throw on the time-out this arm may report)
      MCG_HIP(hipStreamSynchronize(s1_), "device synchronize failed");
      MCG_HIP(hipStreamSynchronize(s0_), "device synchronize failed");
    } else {
      synchronize();
    }
    float ms = 0.f;
    MCG_HIP(hipEventElapsedTime(&ms, ev_t0_, ev_t1_), "event elapsed time failed");
    a.us = 1e3 * (double)ms / cyc;
    MCG_HIP(hipMemcpy(&a.st, st_.get(), sizeof(CgState), hipMemcpyDeviceToHost), "memcpy from device to host failed(state)");
    if (alt) a.timeout = comm_->alt_allreduce_timed_out();
    if (ar_choice) comm_->use_alt_allreduce(false);
    return a;
  };
  info_.probe_ran = true;
  info_.probe_iters = cyc;
  const bool pull0 = pull_;  // without a halo choice: the configured halo (forced pull, or exchanged)
  bool pull = pull0;
  Arm best;
  {
    const Arm x = run_arm(halo_choice ? false : pull0, false);
    Arm p;
    if (halo_choice) p = run_arm(true, false);
    double v[3] = {x.us, halo_choice ? p.us : 0.0, halo_choice && !states_equal(p.st, x.st) ? 1.0 : 0.0};
    allreduce_host_(v, 3);
    if (halo_choice) {
      info_.probe_xchg_us = v[0] / world_;
      info_.probe_pull_us = v[1] / world_;
      info_.probe_pull_bitwise = v[2] == 0.0;
      pull = info_.probe_pull_bitwise && (opt_.hooks.probe_pick_halo >= 0 ? opt_.hooks.probe_pick_halo == 1
                                                                         : info_.probe_pull_us <= info_.probe_xchg_us);
      if (!info_.probe_pull_bitwise && rank_ == 0)
        std::fprintf(stderr, "[mcg] transport probe: the pulled run did not reproduce the exchanged one: the halo is exchanged\n");
    } else {
      (pull0 ? info_.probe_pull_us : info_.probe_xchg_us) = v[0] / world_;
    }
    best = pull && halo_choice ? p : x;
    best.us = pull ? info_.probe_pull_us : info_.probe_xchg_us;
  }
  bool alt = false;
  if (ar_choice) {
    const double budget0 = comm_->alt_allreduce_budget();
    comm_->set_alt_allreduce_budget(std::min(budget0, 10.0));
    const Arm a = run_arm(pull, true);
    double v[3] = {a.us, a.timeout ? 1.0 : 0.0, states_close(a.st, best.st, 1e-6) ? 0.0 : 1.0};
    allreduce_host_(v, 3);
    comm_->set_alt_allreduce_budget(budget0);
    info_.probe_alt_us = v[0] / world_;
    info_.probe_alt_timeout = v[1] != 0.0;
    info_.probe_alt_close = v[1] == 0.0 && v[2] == 0.0;
    alt = info_.probe_alt_close &&
          (opt_.hooks.probe_pick_ar >= 0 ? opt_.hooks.probe_pick_ar == 1 : info_.probe_alt_us < best.us);
    if (!info_.probe_alt_close && rank_ == 0)
      std::fprintf(stderr, "[mcg] transport probe: the alternative all-reduce %s: the first one is kept\n",
                   info_.probe_alt_timeout ? "timed out" : "did not reproduce the first one's sums");
  }
  drop_graphs_();
  pull_ = pull;
  info_.halo_pull = pull_;
  if (ar_choice) comm_->use_alt_allreduce(alt);
  info_.alt_allreduce = comm_->alt_allreduce_in_use();
  opt_.tol = tol0;
  opt_.rtol = rtol0;
  opt_.use_graph = graph0 && (pull_ || !use_halo_ || comm_->halo_capturable());
  info_.graphs = opt_.use_graph;
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
  for (int g = 0; g < 2; ++g)
    for (int ph = 0; ph < 3; ++ph) {
      if (graph_exec_[g][ph]) (void)hipGraphExecDestroy(graph_exec_[g][ph]);
      if (graph_[g][ph]) (void)hipGraphDestroy(graph_[g][ph]);
      graph_exec_[g][ph] = nullptr;
      graph_[g][ph] = nullptr;
    }
}

// Captures 2 (kind 0) or graph_iters (kind 1) iterations starting at an even k_.  The passes
// depend on k only through its parity (and k >= 2) -- with three p buffers also through k mod 3, the
// phase: one capture per (kind, phase) replays for every such k_.
void GpuCgSolver::capture_pair_(int kind, int phase) {
  hipStream_t s = s0_;
  const int iters = kind == 0 ? 2 : opt_.graph_iters;
  // halo_ahead: a graph starts with its ghosts in place (joined before the launch) and ends by
  // joining the prefetch of its last iteration, so every replay sees the same host-side state
  if (halo_ahead_ && !pull_) ensure_ghosts_(k_);
  MCG_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal), "graph capture failed");
  try {
    for (int j = 0; j < iters; ++j) enqueue_iteration_(k_ + j);
    join_halo_();
  } catch (...) {
    hipGraph_t g = nullptr;
    (void)hipStreamEndCapture(s, &g);
    if (g) (void)hipGraphDestroy(g);
    if (comm_ != nullptr) comm_->on_captured(false);
    ghosts_for_ = -1;
    halo_pending_ = false;
    throw;
  }
  ghosts_for_ = (halo_ahead_ && !pull_) ? k_ : -1;  // nothing captured has run yet
  halo_pending_ = false;
  const hipError_t ec = hipStreamEndCapture(s, &graph_[kind][phase]);
  if (comm_ != nullptr) comm_->on_captured(ec == hipSuccess);
  MCG_HIP(ec, "graph capture failed");
  MCG_HIP(hipGraphInstantiate(&graph_exec_[kind][phase], graph_[kind][phase], nullptr, nullptr, 0),
          "graph instantiate failed");
}

void GpuCgSolver::run_iterations(int count) {
  MCG_CHECK(setup_done_, "solver not set up");
  const int glong = opt_.graph_iters > 2 ? opt_.graph_iters : 0;
  while (count > 0) {
    if (opt_.use_graph && k_ >= 2 && (k_ % 2) == 0 && count >= 2 && (!pull_ || k_ >= pull_from_)) {
      const int kind = glong && count >= glong ? 1 : 0;
      const int phase = p3buf_ ? k_ % 3 : 0;
      if (!graph_exec_[kind][phase]) {
        try {
          capture_pair_(kind, phase);
        } catch (const Error& e) {
          std::fprintf(stderr, "[mcg] graph capture unavailable (%s: %s); running eagerly\n", e.what(),
                       e.detail().c_str());
          (void)hipGetLastError();
          opt_.use_graph = false;
          ++info_.graph_fallbacks;
          continue;
        }
      }
      if (halo_ahead_ && !pull_) ensure_ghosts_(k_);
      const hipError_t le = (k_ == opt_.hooks.fail_graph_launch_at) ? hipErrorInvalidValue  // test hook
                                                              : hipGraphLaunch(graph_exec_[kind][phase], s0_);
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
      if (halo_ahead_ && !pull_) ghosts_for_ = k_;  // prefetched by the graph's last iteration and joined
    } else {
      if (k_ == opt_.hooks.inject_nan_at) inject_fault_(k_);
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
              : opt_.form.interleave == 1 ? ra_[(k + 1) & 1].get() + 2 * L_.own_off  // .x of the first owned pair
                                     : ((opt_.recurrence == 1 && (k & 1) == 0) ? r1_.get() : r_.get()) + L_.own_off;
  // the three-term carries recover r from the two p's and read a stored r only past their runs' ends:
  // poison p_{k-1}, which pass k reads everywhere
  if (ar_ && p3_ && opt_.recurrence == 1) r = pbuf_(k - 1) + L_.own_off;
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
}  // namespace mcg
