// GpuCgSolver checkpoint / resume (v3 header with the problem fingerprint), the per-phase timing
// diagnostic, results and the true-residual check.
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
  h.pass_form = (ar_ ? 1 : 0) | (p3_ ? 2 : 0) | (p3buf_ ? 4 : 0);
  h.n_local = L_.n_local();
  h.ext_len = L_.ext_len;
  h.row_begin = L_.row_begin;
  h.k = k_;
  h.n_global = L_.n_global;
  h.seed = spec_.seed;
  h.kind = (int32_t)spec_.kind;
  h.rhs = (int32_t)spec_.rhs;
  h.nnz_local = info_.nnz_local;
  h.fingerprint = fingerprint();
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
                                  &apx_[0], &apx_[1], &w_, &z_, &q_, &p_[2]})
    dump(b->get(), b->bytes());
  ok = (std::fclose(f) == 0) && ok;
  if (!ok || std::rename(tmp.c_str(), path.c_str()) != 0) fail("checkpoint write failed", path);
}

void GpuCgSolver::load_checkpoint(const std::string& prefix) {
  MCG_CHECK(setup_done_, "solver not set up");
  // nothing of an earlier solve may still run on either stream (a pending halo writes ghost rows)
  synchronize();
  join_halo_();
  first_reset_checks_();  // (a resume without a reset: the in-kernel halo's check and the transport probe first)
  const std::string path = prefix + ".rank" + std::to_string(rank_);
  std::FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) fail("checkpoint read failed", path);
  CkptHeader h{};
  bool ok = std::fread(&h, sizeof(h), 1, f) == 1 && std::memcmp(h.magic, kCkptMagic, 8) == 0;
  ok = ok && h.rank == rank_ && h.world == world_ && h.recurrence == opt_.recurrence && h.format == info_.format &&
       h.pass_form == ((ar_ ? 1 : 0) | (p3_ ? 2 : 0) | (p3buf_ ? 4 : 0)) &&
       h.n_local == L_.n_local() && h.ext_len == L_.ext_len && h.row_begin == L_.row_begin &&
       h.n_global == L_.n_global && h.seed == spec_.seed && h.kind == (int32_t)spec_.kind &&
       h.rhs == (int32_t)spec_.rhs && h.nnz_local == info_.nnz_local && h.fingerprint == fingerprint();
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
                                  &apx_[0], &apx_[1], &w_, &z_, &q_, &p_[2]})
    load(b->get(), b->bytes());
  std::fclose(f);
  if (!ok) fail("checkpoint truncated", path);
  k_ = (int)h.k;
  pull_from_ = k_ + 2;  // in-kernel halo: the first two iterations exchange (their p_{k-2} ghost rows)
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
    // (split: the boundary launch's partials from bnd_base_; the slots between are never written, zero)
    const int np = split ? bnd_base_ + g_bnd_ : ((g_odd_ > 0 && (k & 1) != 0) ? g_odd_ : g_all_);
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
  // (a peer-mapping communicator moves registered buffers only: its x buffer, xt_)
  DeviceBuffer<double> xtmp(xt_.get() ? 0 : L_.ext_len, "x", 8), y(n, "Ap", 8), out(1, "scalar");
  double* xe = xt_.get() ? xt_.get() : xtmp.get();
  hipStream_t s = s0_;
  MCG_HIP(hipMemsetAsync(xe, 0, (size_t)L_.ext_len * sizeof(double), s), "device memset failed");
  MCG_HIP(hipMemcpyAsync(xe + L_.own_off, x_.get(), n * sizeof(double), hipMemcpyDeviceToDevice, s),
          "vector copy failed(x)");
  if (use_halo_) {
    double* v[1] = {xe};
    comm_->halo_exchange(L_, v, 1, s);
  }
  spmv_plain_(xe, y.get(), s);
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
