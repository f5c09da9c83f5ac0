// Problem families ("models" of this framework): the linear systems A x = b that
// the CG solver is run on.  Every family is defined row-by-row by a pure function
// of the GLOBAL row index, usable on the host (CPU reference path, tests) and on
// the device (on-device generation of each rank's owned rows), so a matrix never
// has to exist in host memory and b does not depend on the number of ranks.
//
//   demo       the reference's hard-coded 3x3 system (CUDACG.cu:74-117,136-141):
//              A = [[3,0,2],[0,2,0],[2,0,1]], b = [3.5,1.5,2.0].  Symmetric
//              INDEFINITE (eigenvalues -0.236, 2, 4.236) — CG still reaches the
//              exact solution in 3 steps, which the reference's stdout pins.
//   poisson2d  5-point Dirichlet Laplacian on an N x N grid (4 / -1), n = N^2,
//              nnz = 5N^2 - 4N  (BASELINE.json configs 1-3).
//   poisson3d  7-point Dirichlet Laplacian on an N^3 grid (6 / -1),
//              nnz = 7N^3 - 6N^2 (BASELINE.json config 4).
//   randspd    symmetric, strictly diagonally dominant (hence SPD) banded matrix
//              with irregular row lengths: pair {a<b}, 0<b-a<=W, is present iff a
//              counter-based hash of the pair passes a density that varies per
//              1024-row region; value -w(a,b), w in (0,1]; diagonal = row length
//              (> sum |off-diagonal|).  BASELINE.json config 5.
#pragma once

#include <cmath>
#include <cstdint>
#include <string>

#if defined(__HIP__)
#define MCG_HD __host__ __device__
#else
#define MCG_HD
#endif

namespace mcg {

enum class ProblemKind : int { Demo = 0, Poisson2D = 1, Poisson3D = 2, RandomSPD = 3 };
enum class RhsKind : int { Reference = 0, Random = 1, Ones = 2 };

struct ProblemSpec {
  ProblemKind kind = ProblemKind::Demo;
  int64_t N = 3;           // grid edge for poisson2d/3d
  int64_t rows = 0;        // randspd: global rows
  int64_t band = 0;        // randspd: half bandwidth W (candidate offsets 1..W)
  double density = 0.5;    // randspd: mean probability that a candidate pair is present
  uint64_t seed = 1234;    // matrix + rhs seed
  RhsKind rhs = RhsKind::Reference;
};

// ---- counter-based hashing (SplitMix64 finaliser); identical on host/device ----
MCG_HD inline uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
MCG_HD inline double u01(uint64_t h) { return (double)(h >> 11) * 0x1.0p-53; }

MCG_HD inline int64_t global_rows(const ProblemSpec& s) {
  switch (s.kind) {
    case ProblemKind::Demo: return 3;
    case ProblemKind::Poisson2D: return s.N * s.N;
    case ProblemKind::Poisson3D: return s.N * s.N * s.N;
    case ProblemKind::RandomSPD: return s.rows;
  }
  return 0;
}

// Half-width of the column window: row i only touches columns in
// [i - lower_bw, i + upper_bw].  Drives the halo plan.
MCG_HD inline int64_t bandwidth(const ProblemSpec& s) {
  switch (s.kind) {
    case ProblemKind::Demo: return 2;
    case ProblemKind::Poisson2D: return s.N;
    case ProblemKind::Poisson3D: return s.N * s.N;
    case ProblemKind::RandomSPD: return s.band;
  }
  return 0;
}

// Natural partition granule: 1-D partitions of a stencil are aligned to whole
// grid lines (2-D) / planes (3-D) when possible.
MCG_HD inline int64_t partition_granule(const ProblemSpec& s) {
  switch (s.kind) {
    case ProblemKind::Poisson2D: return s.N;
    case ProblemKind::Poisson3D: return s.N * s.N;
    default: return 1;
  }
}

// randspd pair presence / weight.  a < b required.
MCG_HD inline double randspd_density(const ProblemSpec& s, int64_t a) {
  // per-1024-row region density factor in [0.25, 1.75] -> irregular row lengths
  const double f = 0.25 + 1.5 * u01(mix64(s.seed * 0x2545F4914F6CDD1Dull + (uint64_t)(a >> 10)));
  double q = s.density * f;
  return q > 1.0 ? 1.0 : q;
}
MCG_HD inline uint64_t pair_hash(const ProblemSpec& s, int64_t a, int64_t b) {
  return mix64(s.seed ^ mix64((uint64_t)a * 0x9E3779B97F4A7C15ull + (uint64_t)b));
}
MCG_HD inline bool randspd_present(const ProblemSpec& s, int64_t a, int64_t b) {
  return u01(pair_hash(s, a, b)) < randspd_density(s, a);
}
MCG_HD inline double randspd_weight(const ProblemSpec& s, int64_t a, int64_t b) {
  // (0,1]: reuse the low bits of the pair hash (independent of the presence test's high bits)
  return 1.0 - (double)(pair_hash(s, a, b) & 0xFFFFFull) * (1.0 / 1048576.0);
}

// Visit the entries of global row i in ascending column order: f(col, val).
// For randspd the diagonal value depends on the row length, which the caller
// passes in (from the count pass / rowptr); pass -1 to have it counted here.
template <class F>
MCG_HD inline void for_each_entry(const ProblemSpec& s, int64_t i, F&& f, int64_t rowlen = -1) {
  switch (s.kind) {
    case ProblemKind::Demo: {
      // CUDACG.cu:102-117 : val {3,2,2,2,1}, rowptr {0,2,3,5}, col {0,2,1,0,2}
      if (i == 0) { f(0, 3.0); f(2, 2.0); }
      else if (i == 1) { f(1, 2.0); }
      else { f(0, 2.0); f(2, 1.0); }
      return;
    }
    case ProblemKind::Poisson2D: {
      const int64_t N = s.N, ix = i % N, iy = i / N;
      if (iy > 0) f(i - N, -1.0);
      if (ix > 0) f(i - 1, -1.0);
      f(i, 4.0);
      if (ix < N - 1) f(i + 1, -1.0);
      if (iy < N - 1) f(i + N, -1.0);
      return;
    }
    case ProblemKind::Poisson3D: {
      const int64_t N = s.N, N2 = N * N;
      const int64_t ix = i % N, iy = (i / N) % N, iz = i / N2;
      if (iz > 0) f(i - N2, -1.0);
      if (iy > 0) f(i - N, -1.0);
      if (ix > 0) f(i - 1, -1.0);
      f(i, 6.0);
      if (ix < N - 1) f(i + 1, -1.0);
      if (iy < N - 1) f(i + N, -1.0);
      if (iz < N - 1) f(i + N2, -1.0);
      return;
    }
    case ProblemKind::RandomSPD: {
      const int64_t n = s.rows, W = s.band;
      if (rowlen < 0) {
        rowlen = 1;
        for (int64_t d = 1; d <= W; ++d) {
          if (i - d >= 0 && randspd_present(s, i - d, i)) ++rowlen;
          if (i + d < n && randspd_present(s, i, i + d)) ++rowlen;
        }
      }
      for (int64_t d = (W < i ? W : i); d >= 1; --d)
        if (randspd_present(s, i - d, i)) f(i - d, -randspd_weight(s, i - d, i));
      f(i, (double)rowlen);
      for (int64_t d = 1; d <= W && i + d < n; ++d)
        if (randspd_present(s, i, i + d)) f(i + d, -randspd_weight(s, i, i + d));
      return;
    }
  }
}

MCG_HD inline int64_t row_length(const ProblemSpec& s, int64_t i) {
  switch (s.kind) {
    case ProblemKind::Demo: return i == 1 ? 1 : 2;
    case ProblemKind::Poisson2D: {
      const int64_t N = s.N, ix = i % N, iy = i / N;
      return 1 + (iy > 0) + (ix > 0) + (ix < N - 1) + (iy < N - 1);
    }
    case ProblemKind::Poisson3D: {
      const int64_t N = s.N, N2 = N * N;
      const int64_t ix = i % N, iy = (i / N) % N, iz = i / N2;
      return 1 + (iz > 0) + (iy > 0) + (ix > 0) + (ix < N - 1) + (iy < N - 1) + (iz < N - 1);
    }
    case ProblemKind::RandomSPD: {
      int64_t len = 1;
      const int64_t n = s.rows, W = s.band;
      for (int64_t d = 1; d <= W; ++d) {
        if (i - d >= 0 && randspd_present(s, i - d, i)) ++len;
        if (i + d < n && randspd_present(s, i, i + d)) ++len;
      }
      return len;
    }
  }
  return 0;
}

// Right-hand side entry for global row i.
MCG_HD inline double rhs_value(const ProblemSpec& s, int64_t i) {
  switch (s.rhs) {
    case RhsKind::Reference: {
      if (s.kind == ProblemKind::Demo) return i == 0 ? 3.5 : (i == 1 ? 1.5 : 2.0);  // CUDACG.cu:138-140
      return 1.0;
    }
    case RhsKind::Random: return u01(mix64(s.seed ^ mix64((uint64_t)i + 0x51ED27ull)));
    case RhsKind::Ones: return 1.0;
  }
  return 0.0;
}

// Closed-form global nnz where available (-1 = must be counted).
inline int64_t closed_form_nnz(const ProblemSpec& s) {
  switch (s.kind) {
    case ProblemKind::Demo: return 5;
    case ProblemKind::Poisson2D: return 5 * s.N * s.N - 4 * s.N;
    case ProblemKind::Poisson3D: return 7 * s.N * s.N * s.N - 6 * s.N * s.N;
    default: return -1;
  }
}

std::string problem_name(const ProblemSpec& s);
ProblemKind parse_problem_kind(const std::string& name);
RhsKind parse_rhs_kind(const std::string& name);

}  // namespace mcg
