#include "mcg/problem.hpp"

#include <cstring>

#include "mcg/check.hpp"

namespace mcg {

std::string problem_name(const ProblemSpec& s) {
  switch (s.kind) {
    case ProblemKind::Demo: return "demo";
    case ProblemKind::Poisson2D: return s.coef ? "poisson2d-varcoef" : "poisson2d";
    case ProblemKind::Poisson3D: return s.coef ? "poisson3d-varcoef" : "poisson3d";
    case ProblemKind::RandomSPD: return s.scramble ? "randspd-scrambled" : "randspd";
    case ProblemKind::Csr: return "csr";
  }
  return "?";
}

namespace {
struct Fp {
  uint64_t h = 0x6A09E667F3BCC909ull;
  void add(uint64_t v) { h = mix64(h ^ (v + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2))); }
  void add_d(double d) {
    uint64_t u;
    std::memcpy(&u, &d, sizeof(u));
    add(u);
  }
};
}  // namespace

uint64_t problem_fingerprint(const ProblemSpec& s) {
  Fp f;
  f.add((uint64_t)s.kind);
  f.add((uint64_t)s.rhs);
  f.add(s.seed);
  if (s.kind == ProblemKind::Csr) {
    MCG_CHECK(s.csr != nullptr, "csr problem without a matrix");
    const CsrMatrix& A = *s.csr;
    f.add((uint64_t)A.n);
    for (int64_t i = 0; i <= A.n; ++i) f.add((uint64_t)A.rowptr[i]);
    for (int64_t k = 0; k < A.rowptr[A.n]; ++k) {
      f.add((uint64_t)A.cols[k]);
      f.add_d(A.vals[k]);
    }
    f.add(A.b ? 1 : 0);
    if (A.b)
      for (int64_t i = 0; i < A.n; ++i) f.add_d(A.b[i]);
    return f.h;
  }
  f.add((uint64_t)s.N);
  f.add((uint64_t)s.rows);
  f.add((uint64_t)s.band);
  f.add_d(s.density);
  f.add((uint64_t)s.spread);
  f.add((uint64_t)s.scramble);
  if (s.coef) f.add(0xC0EF0000ull + (uint64_t)s.coef);  // (absent for coef 0: older checkpoints stay valid)
  return f.h;
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
