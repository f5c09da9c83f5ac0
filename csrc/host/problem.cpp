#include "mcg/problem.hpp"

#include "mcg/check.hpp"

namespace mcg {

std::string problem_name(const ProblemSpec& s) {
  switch (s.kind) {
    case ProblemKind::Demo: return "demo";
    case ProblemKind::Poisson2D: return "poisson2d";
    case ProblemKind::Poisson3D: return "poisson3d";
    case ProblemKind::RandomSPD: return "randspd";
    case ProblemKind::Csr: return "csr";
  }
  return "?";
}

ProblemKind parse_problem_kind(const std::string& name) {
  if (name == "demo") return ProblemKind::Demo;
  if (name == "poisson2d" || name == "poisson-2d" || name == "2d") return ProblemKind::Poisson2D;
  if (name == "poisson3d" || name == "poisson-3d" || name == "3d") return ProblemKind::Poisson3D;
  if (name == "randspd" || name == "random-spd" || name == "random") return ProblemKind::RandomSPD;
  fail("unknown problem: " + name);
}

RhsKind parse_rhs_kind(const std::string& name) {
  if (name == "reference" || name == "ref") return RhsKind::Reference;
  if (name == "random" || name == "rand") return RhsKind::Random;
  if (name == "ones") return RhsKind::Ones;
  fail("unknown rhs: " + name);
}

}  // namespace mcg
