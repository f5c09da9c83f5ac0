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
  bool carry = false;  // SolverInfo::carry of this rank (the line-carry pass ran on its interior)
  std::string error;
};

struct LocalRunResult {
  std::vector<LocalRankResult> ranks;
};

// fixed_iters > 0: run exactly that many iterations (+ finalise) instead of solving to tol.
// Note: an exception on one rank while others wait at a LocalComm barrier would hang;
// errors here are setup-time (allocation) errors, raised before any collective.
LocalRunResult run_local_ranks(const ProblemSpec& spec, const CgOptions& opt, int world, int fixed_iters = 0,
                               bool verify = false);

}  // namespace mcg
