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
//              coef = 1 (both): heterogeneous diffusion -div(c grad u) with a seeded random
//              conductivity field: cell i has c_i in [0.1, 10) (0.1 + 9.9 u^3), the face between
//              neighbours i < j has k = 2 c_i c_j / (c_i + c_j) (harmonic mean) and a_ij = a_ji = -k, a
//              boundary face (Dirichlet) has k = c_i, and a_ii = the sum of the cell's face k's, so
//              the matrix is symmetric and diagonally dominant (strictly on the boundary rows): SPD,
//              with (almost) every off-diagonal value distinct.  coef = 0: every k = 1 (4 / -1, 6 / -1).
//   randspd    symmetric, strictly diagonally dominant (hence SPD) banded matrix
//              with irregular row lengths: pair {a<b}, 0<b-a<=W, is present iff a
//              counter-based hash of the pair passes a density that varies per
//              1024-row region; value -w(a,b), w in (0,1]; diagonal = row length
//              (> sum |off-diagonal|).  BASELINE.json config 5.
//              spread > 0 ("wide"): the W candidate offsets are not 1..W but W
//              distinct offsets d_0 < ... < d_{W-1} drawn over [1, spread] (one per
//              stratum of spread/W), so columns reach +-spread rows away — with
//              spread ~ n the sparsity is unstructured at every scale (the all-gather
//              ghost path), and each 64-row slice still reads 2W short runs of p.
//              Both are MULTI-DIAGONAL: every row draws from the same 2W offsets.
//              scramble = 1: the symmetric permutation P^T A P of that matrix, with P a
//              seeded bijection pi of [0, n) (Feistel network + cycle walking, O(1) per
//              index both ways): row i is base row pi(i) with every column c mapped to
//              pi^-1(c).  Still symmetric and strictly diagonally dominant (SPD), but
//              genuinely irregular: no two rows share an offset set, row lengths vary
//              with the base row's region, and every nonzero is a random column.
//   csr       a user matrix given as host CSR arrays (CsrMatrix view; Matrix
//              Market files, SciPy matrices) — the reference's own input form
//              (cusparseCreateCsr over rowptr/col/val, CUDACG.cu:93-117,213-216).
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

enum class ProblemKind : int { Demo = 0, Poisson2D = 1, Poisson3D = 2, RandomSPD = 3, Csr = 4 };

// Column offset beyond which a gather leaves an L2-sized neighbourhood of the row (2^16 doubles =
// 512 KiB of p): a user matrix with many such entries is "scattered" and takes the L2-segment tiles.
constexpr int64_t kFarOffset = (int64_t)1 << 16;

// Host CSR of a user matrix (global rows, 0-based, int64 row pointers and columns).  A view:
// the arrays are owned by the caller (HostMatrix, a NumPy array, ...).  Only host code reads
// it: a rank uploads its rows; the device generators never see this kind.
struct CsrMatrix {
  int64_t n = 0;
  const int64_t* rowptr = nullptr;  // n + 1
  const int64_t* cols = nullptr;    // rowptr[n]
  const double* vals = nullptr;
  const double* b = nullptr;        // optional right-hand side (n); null: the spec's rhs kind
  int64_t bw = 0;                   // max |i - j| over the stored entries
  int64_t far = 0;                  // entries with |i - j| > kFarOffset: gathers no SELL slice keeps in the L2
  // structured-grid stencil detected in the matrix (HostMatrix): every stored entry's column offset
  // is 0, +-1, +-line (2-D) or also +-plane = line^2 (3-D), and the rows are whole lines / planes;
  // 0 = none.  Lets a user matrix take the generated stencils' line / plane carry.
  int64_t line = 0, plane = 0;
};
enum class RhsKind : int { Reference = 0, Random = 1, Ones = 2 };

struct ProblemSpec {
  ProblemKind kind = ProblemKind::Demo;
  int64_t N = 3;           // grid edge for poisson2d/3d
  int64_t rows = 0;        // randspd: global rows
  int64_t band = 0;        // randspd: half bandwidth W (candidate offsets 1..W)
  double density = 0.5;    // randspd: mean probability that a candidate pair is present
  uint64_t seed = 1234;    // matrix + rhs seed
  RhsKind rhs = RhsKind::Reference;
  int64_t spread = 0;      // randspd: > 0 = wide candidate offsets over [1, spread] (see above)
  int scramble = 0;        // randspd: 1 = P^T A P with a seeded random permutation P (irregular)
  int coef = 0;            // poisson2d/3d: 0 = constant coefficients, 1 = random conductivity field
  const CsrMatrix* csr = nullptr;  // kind Csr: the matrix (host)
};

// ---- counter-based hashing (SplitMix64 finaliser); identical on host/device ----
MCG_HD inline uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
MCG_HD inline double u01(uint64_t h) { return (double)(h >> 11) * 0x1.0p-53; }

// ---- seeded bijection pi of [0, n) (scrambled random SPD) ----
// A 4-round balanced Feistel network on 2h-bit words (2^(2h) >= n, so the domain is < 4n) is a
// bijection of [0, 2^(2h)); cycle walking (re-apply until the value is < n) restricts it to a
// bijection of [0, n), and the inverse walks the inverse network the same way.  Both directions
// cost O(1) hashes per index (expected < 4 walks), on the host and on the device.
MCG_HD inline int perm_half_bits(int64_t n) {
  const int bits = n > 1 ? 64 - __builtin_clzll((unsigned long long)(n - 1)) : 1;
  return bits < 2 ? 1 : (bits + 1) / 2;
}
MCG_HD inline uint64_t feistel_key(uint64_t seed, int r) { return mix64(seed * 0xA24BAED4963EE407ull + (uint64_t)r); }
MCG_HD inline uint64_t feistel(uint64_t x, int h, uint64_t seed, bool inverse) {
  const uint64_t m = (1ull << h) - 1;
  uint64_t L = x >> h, R = x & m;
  if (!inverse) {
    for (int r = 0; r < 4; ++r) {  // (L, R) -> (R, L ^ f_r(R))
      const uint64_t t = L ^ (mix64(R ^ feistel_key(seed, r)) & m);
      L = R;
      R = t;
    }
  } else {
    for (int r = 3; r >= 0; --r) {  // (L', R') -> (R' ^ f_r(L'), L')
      const uint64_t t = R ^ (mix64(L ^ feistel_key(seed, r)) & m);
      R = L;
      L = t;
    }
  }
  return (L << h) | R;
}
// pi(i): the base row behind scrambled row i
MCG_HD inline int64_t scramble_fwd(const ProblemSpec& s, int64_t i) {
  const int h = perm_half_bits(s.rows);
  uint64_t x = (uint64_t)i;
  do x = feistel(x, h, s.seed ^ 0x5C4A3B1Du, false); while (x >= (uint64_t)s.rows);
  return (int64_t)x;
}
// pi^-1(c): the scrambled index of base row / column c
MCG_HD inline int64_t scramble_inv(const ProblemSpec& s, int64_t c) {
  const int h = perm_half_bits(s.rows);
  uint64_t x = (uint64_t)c;
  do x = feistel(x, h, s.seed ^ 0x5C4A3B1Du, true); while (x >= (uint64_t)s.rows);
  return (int64_t)x;
}
MCG_HD inline bool scrambled(const ProblemSpec& s) { return s.kind == ProblemKind::RandomSPD && s.scramble != 0; }

MCG_HD inline int64_t global_rows(const ProblemSpec& s) {
  switch (s.kind) {
    case ProblemKind::Demo: return 3;
    case ProblemKind::Poisson2D: return s.N * s.N;
    case ProblemKind::Poisson3D: return s.N * s.N * s.N;
    case ProblemKind::RandomSPD: return s.rows;
    case ProblemKind::Csr: return s.csr ? s.csr->n : 0;
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
    case ProblemKind::RandomSPD: return s.scramble ? (s.rows > 0 ? s.rows - 1 : 0) : (s.spread > 0 ? s.spread : s.band);
    case ProblemKind::Csr: return s.csr ? s.csr->bw : 0;
  }
  return 0;
}

// Natural partition granule: 1-D partitions of a stencil are aligned to whole
// grid lines (2-D) / planes (3-D) when possible.
MCG_HD inline int64_t partition_granule(const ProblemSpec& s) {
  switch (s.kind) {
    case ProblemKind::Poisson2D: return s.N;
    case ProblemKind::Poisson3D: return s.N * s.N;
    case ProblemKind::Csr: return s.csr && s.csr->plane > 0 ? s.csr->plane : (s.csr && s.csr->line > 0 ? s.csr->line : 1);
    default: return 1;
  }
}
// grid line length of a structured-grid stencil (generated, or detected in a user matrix); 0 = none
MCG_HD inline int64_t stencil_line(const ProblemSpec& s) {
  switch (s.kind) {
    case ProblemKind::Poisson2D:
    case ProblemKind::Poisson3D: return s.N;
    case ProblemKind::Csr: return s.csr ? s.csr->line : 0;
    default: return 0;
  }
}
// plane length (line^2) of a 3-D stencil; 0 = not 3-D
MCG_HD inline int64_t stencil_plane(const ProblemSpec& s) {
  switch (s.kind) {
    case ProblemKind::Poisson3D: return s.N * s.N;
    case ProblemKind::Csr: return s.csr ? s.csr->plane : 0;
    default: return 0;
  }
}

// poisson2d/3d coefficients (coef = 1): cell conductivity, and the conductivity of the face between
// cells a < b (or a boundary face of cell a: b = -1).  Only correctly rounded operations, written so
// that no compiler can contract them differently on the host and the device: every rank, the CPU
// path and the host CSR see the same bits, and k(a, b) is computed from the ordered pair, so a_ij
// and a_ji are the same double.
MCG_HD inline double cell_cond(const ProblemSpec& s, int64_t i) {
  const double u = u01(mix64((s.seed * 0x3C6EF372FE94F82Bull) ^ mix64((uint64_t)i + 0xC0EFull)));
  const double u3 = (u * u) * u;
  return fma(9.9, u3, 0.1);
}
MCG_HD inline double face_cond(const ProblemSpec& s, int64_t a, int64_t b) {
  if (s.coef == 0) return 1.0;
  const double ca = cell_cond(s, a);
  if (b < 0) return ca;
  const double cb = cell_cond(s, b);
  const double num = (2.0 * ca) * cb;
  return num / (ca + cb);
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
// candidate offset t (0 <= t < W), strictly increasing in t: 1..W (banded) or one offset per
// stratum [t * step, (t + 1) * step) of [1, spread] (wide)
MCG_HD inline int64_t randspd_offset(const ProblemSpec& s, int64_t t) {
  if (s.spread <= 0) return t + 1;
  const int64_t step = s.spread / s.band > 0 ? s.spread / s.band : 1;
  return t * step + 1 + (int64_t)(mix64(s.seed * 0xD1B54A32D192ED03ull + (uint64_t)t) % (uint64_t)step);
}

// randspd base matrix (not scrambled): row length and entries of row i in ascending column order
MCG_HD inline int64_t randspd_row_length(const ProblemSpec& s, int64_t i) {
  int64_t len = 1;
  const int64_t n = s.rows, W = s.band;
  for (int64_t t = 0; t < W; ++t) {
    const int64_t d = randspd_offset(s, t);
    if (i - d >= 0 && randspd_present(s, i - d, i)) ++len;
    if (i + d < n && randspd_present(s, i, i + d)) ++len;
  }
  return len;
}
template <class F>
MCG_HD inline void randspd_row(const ProblemSpec& s, int64_t i, F&& f, int64_t rowlen) {
  const int64_t n = s.rows, W = s.band;
  if (rowlen < 0) rowlen = randspd_row_length(s, i);
  for (int64_t t = W - 1; t >= 0; --t) {
    const int64_t d = randspd_offset(s, t);
    if (d <= i && randspd_present(s, i - d, i)) f(i - d, -randspd_weight(s, i - d, i));
  }
  f(i, (double)rowlen);
  for (int64_t t = 0; t < W; ++t) {
    const int64_t d = randspd_offset(s, t);
    if (i + d >= n) break;
    if (randspd_present(s, i, i + d)) f(i + d, -randspd_weight(s, i, i + d));
  }
}

// Visit the entries of global row i: f(col, val), in ascending column order except for the
// scrambled random SPD (base-row order: the mapped columns are unordered).
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
      if (s.coef == 0) {
        if (iy > 0) f(i - N, -1.0);
        if (ix > 0) f(i - 1, -1.0);
        f(i, 4.0);
        if (ix < N - 1) f(i + 1, -1.0);
        if (iy < N - 1) f(i + N, -1.0);
        return;
      }
      // faces in column order (north, west, east, south); a missing neighbour is a boundary face
      const double kn = face_cond(s, iy > 0 ? i - N : i, iy > 0 ? i : -1);
      const double kw = face_cond(s, ix > 0 ? i - 1 : i, ix > 0 ? i : -1);
      const double ke = face_cond(s, i, ix < N - 1 ? i + 1 : -1);
      const double ks = face_cond(s, i, iy < N - 1 ? i + N : -1);
      if (iy > 0) f(i - N, -kn);
      if (ix > 0) f(i - 1, -kw);
      f(i, ((kn + kw) + ke) + ks);
      if (ix < N - 1) f(i + 1, -ke);
      if (iy < N - 1) f(i + N, -ks);
      return;
    }
    case ProblemKind::Poisson3D: {
      const int64_t N = s.N, N2 = N * N;
      const int64_t ix = i % N, iy = (i / N) % N, iz = i / N2;
      if (s.coef == 0) {
        if (iz > 0) f(i - N2, -1.0);
        if (iy > 0) f(i - N, -1.0);
        if (ix > 0) f(i - 1, -1.0);
        f(i, 6.0);
        if (ix < N - 1) f(i + 1, -1.0);
        if (iy < N - 1) f(i + N, -1.0);
        if (iz < N - 1) f(i + N2, -1.0);
        return;
      }
      const double kb = face_cond(s, iz > 0 ? i - N2 : i, iz > 0 ? i : -1);
      const double kn = face_cond(s, iy > 0 ? i - N : i, iy > 0 ? i : -1);
      const double kw = face_cond(s, ix > 0 ? i - 1 : i, ix > 0 ? i : -1);
      const double ke = face_cond(s, i, ix < N - 1 ? i + 1 : -1);
      const double ks = face_cond(s, i, iy < N - 1 ? i + N : -1);
      const double kt = face_cond(s, i, iz < N - 1 ? i + N2 : -1);
      if (iz > 0) f(i - N2, -kb);
      if (iy > 0) f(i - N, -kn);
      if (ix > 0) f(i - 1, -kw);
      f(i, ((((kb + kn) + kw) + ke) + ks) + kt);
      if (ix < N - 1) f(i + 1, -ke);
      if (iy < N - 1) f(i + N, -ks);
      if (iz < N - 1) f(i + N2, -kt);
      return;
    }
    case ProblemKind::RandomSPD: {
      if (s.scramble)  // row pi(i) of the base matrix, its columns through pi^-1
        randspd_row(s, scramble_fwd(s, i), [&](int64_t c, double v) { f(scramble_inv(s, c), v); }, rowlen);
      else
        randspd_row(s, i, f, rowlen);
      return;
    }
    case ProblemKind::Csr: {
#if !defined(__HIP_DEVICE_COMPILE__)
      const CsrMatrix& A = *s.csr;
      for (int64_t k = A.rowptr[i]; k < A.rowptr[i + 1]; ++k) f(A.cols[k], A.vals[k]);
#endif
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
    case ProblemKind::RandomSPD: return randspd_row_length(s, s.scramble ? scramble_fwd(s, i) : i);
    case ProblemKind::Csr: {
#if !defined(__HIP_DEVICE_COMPILE__)
      return s.csr->rowptr[i + 1] - s.csr->rowptr[i];
#else
      return 0;
#endif
    }
  }
  return 0;
}

// Right-hand side entry for global row i.
MCG_HD inline double rhs_value(const ProblemSpec& s, int64_t i) {
  switch (s.rhs) {
    case RhsKind::Reference: {
      if (s.kind == ProblemKind::Demo) return i == 0 ? 3.5 : (i == 1 ? 1.5 : 2.0);  // CUDACG.cu:138-140
#if !defined(__HIP_DEVICE_COMPILE__)
      if (s.kind == ProblemKind::Csr && s.csr && s.csr->b) return s.csr->b[i];  // the user's b
#endif
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
    case ProblemKind::Csr: return s.csr ? s.csr->rowptr[s.csr->n] : 0;
    default: return -1;
  }
}

std::string problem_name(const ProblemSpec& s);
// 64-bit hash of everything that defines A and b: the family's parameters, and for a user matrix
// (kind csr) its rowptr / cols / vals and b (O(nnz) on the host).  Checkpoints record it so a
// resume against another matrix or right-hand side of the same size is refused.
uint64_t problem_fingerprint(const ProblemSpec& s);
ProblemKind parse_problem_kind(const std::string& name);
RhsKind parse_rhs_kind(const std::string& name);

}  // namespace mcg
