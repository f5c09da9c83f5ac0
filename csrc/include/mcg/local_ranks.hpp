// P-rank emulation on one device (LocalComm); see csrc/gpu/local_ranks.cpp.
#pragma once

#include <string>
#include <vector>

#include "mcg/cg.hpp"
#include "mcg/problem.hpp"

namespace mcg {

struct LocalRankResult {
  CgResult res;
  std::vector<double> x;
  int64_t row_begin = 0;
  double true_rnorm = -1.0;
  bool ap_recompute = false;  // SolverInfo::ap_recompute of this rank
  bool lean_only = false;     // SolverInfo::lean_only of this rank
  double lean_split = 0.0;    // SolverInfo::lean_split of this rank
  bool p3 = false;            // SolverInfo::p3 (three-term carry form)
  bool p3buf = false;         // SolverInfo::p3buf (three p buffers)
  double dia_uniform = 0.0;   // SolverInfo::dia_uniform (fraction of uniform slices)
  bool halo_pull = false;     // SolverInfo::halo_pull of this rank
  bool carry = false;  // SolverInfo::carry of this rank (the line-carry pass ran on its interior)
  bool ag_overlap = false;     // SolverInfo::ag_overlap (own-block SpMV half || all-gather)
  double ag_local_frac = 0.0;  // SolverInfo::ag_local_frac
  bool probe_ran = false, probe_pull_bitwise = false;  // SolverInfo's transport probe
  double probe_pull_us = 0.0, probe_xchg_us = 0.0;
  std::vector<std::pair<std::string, double>> phases;  // phase_profile (mean us) when asked for
  std::string error;
};

struct LocalRunResult {
  std::vector<LocalRankResult> ranks;
};

// fixed_iters > 0: run exactly that many iterations (+ finalise) instead of solving to tol.
// A rank that throws aborts the LocalGroup: the others leave their barriers with an error.
// phase_iters > 0 (single-reduction form): afterwards, that many more iterations with hipEvents at
// every phase boundary on every rank (GpuCgSolver::phase_profile): the overlap rehearsal.
LocalRunResult run_local_ranks(const ProblemSpec& spec, const CgOptions& opt, int world, int fixed_iters = 0,
                               bool verify = false, int phase_iters = 0);

}  // namespace mcg
