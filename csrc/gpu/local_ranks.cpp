// Emulate a P-rank run on ONE device: P host threads, each a full GpuCgSolver
// rank with a LocalComm (see comm.hpp).  Exercises the whole distributed path
// (row partition, halo plan, ghost layout, interior/boundary split with the
// side-stream overlap, collective placement, convergence latch agreement)
// against the same kernels the RCCL path runs.
#include "mcg/local_ranks.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>

#include "mcg/check.hpp"
#include "mcg/comm.hpp"
#include "mcg/solver.hpp"

namespace mcg {

LocalRunResult run_local_ranks(const ProblemSpec& spec, const CgOptions& opt, int world, int fixed_iters,
                               bool verify, int phase_iters) {
  MCG_CHECK(world >= 1, "invalid number of local ranks");
  int dev = 0;
  MCG_HIP(hipGetDevice(&dev), "Device Set failed");
  auto group = std::make_shared<LocalGroup>(world);
  LocalRunResult out;
  out.ranks.resize(world);
  std::vector<std::thread> ts;
  // setup-failure agreement before the first collective (a rank that threw must not
  // leave the others waiting at a LocalComm barrier)
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  bool any_failed = false;
  auto setup_barrier = [&](bool failed) {
    std::unique_lock<std::mutex> lk(m);
    any_failed = any_failed || failed;
    if (++arrived == world) cv.notify_all();
    else cv.wait(lk, [&] { return arrived == world; });
    return !any_failed;
  };
  for (int r = 0; r < world; ++r) {
    ts.emplace_back([&, r] {
      LocalRankResult& o = out.ranks[r];
      bool passed = false;
      try {
        MCG_HIP(hipSetDevice(dev), "Device Set failed");
        LocalComm comm(group, r);
        std::unique_ptr<GpuCgSolver> sp;
        try {
          sp.reset(new GpuCgSolver(spec, opt, r, world, &comm));
          sp->setup();
        } catch (...) {
          passed = true;
          setup_barrier(true);
          throw;
        }
        passed = true;
        if (!setup_barrier(false)) fail("another local rank failed during setup");
        GpuCgSolver& s = *sp;
        if (fixed_iters > 0) {
          s.reset();
          s.run_iterations(fixed_iters);
          if (phase_iters > 0) o.phases = s.phase_profile(phase_iters);
          s.finalize();
          o.res = s.result();
        } else {
          o.res = s.solve();
        }
        o.x = s.x_local();
        o.row_begin = s.layout().row_begin;
        o.carry = s.info().carry;
        o.ap_recompute = s.info().ap_recompute;
        o.lean_only = s.info().lean_only;
        o.lean_split = s.info().lean_split;
        o.p3 = s.info().p3;
        o.p3buf = s.info().p3buf;
        o.dia_uniform = s.info().dia_uniform;
        o.halo_pull = s.info().halo_pull;
        o.ag_overlap = s.info().ag_overlap;
        o.ag_local_frac = s.info().ag_local_frac;
        o.probe_ran = s.info().probe_ran;
        o.probe_pull_bitwise = s.info().probe_pull_bitwise;
        o.probe_pull_us = s.info().probe_pull_us;
        o.probe_xchg_us = s.info().probe_xchg_us;
        if (verify) o.true_rnorm = s.true_residual_norm();
      } catch (const Error& e) {
        o.error = std::string(e.what()) + ": " + e.detail();
        group->abort();
      } catch (const std::exception& e) {
        o.error = e.what();
        group->abort();
      }
      if (!passed) setup_barrier(true);
    });
  }
  for (auto& t : ts) t.join();
  std::string first;
  for (auto& o : out.ranks)
    if (!o.error.empty() && (first.empty() || first.find("another local rank failed") != std::string::npos))
      first = o.error;
  if (!first.empty()) fail("local rank failed", first);
  return out;
}

}  // namespace mcg
