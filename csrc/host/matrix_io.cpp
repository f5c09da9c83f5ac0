#include "mcg/matrix.hpp"

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <fstream>
#include <numeric>
#include <sstream>

#include "mcg/check.hpp"

namespace mcg {

HostMatrix::HostMatrix(int64_t n, std::vector<int64_t> rowptr, std::vector<int64_t> cols, std::vector<double> vals,
                       std::vector<double> b)
    : rowptr_(std::move(rowptr)), cols_(std::move(cols)), vals_(std::move(vals)), b_(std::move(b)) {
  MCG_CHECK(n >= 0 && (int64_t)rowptr_.size() == n + 1, "csr: row pointers must have n + 1 entries");
  MCG_CHECK(rowptr_[0] == 0, "csr: row pointers must start at 0");
  for (int64_t i = 0; i < n; ++i) MCG_CHECK(rowptr_[i] <= rowptr_[i + 1], "csr: row pointers must not decrease");
  const int64_t nnz = rowptr_[n];
  MCG_CHECK((int64_t)cols_.size() == nnz && (int64_t)vals_.size() == nnz, "csr: cols / vals length != nnz");
  MCG_CHECK(b_.empty() || (int64_t)b_.size() == n, "csr: b length != n");
  MCG_CHECK(n < ((int64_t)1 << 31), "csr: more than 2^31 rows");
  int64_t bw = 0, far = 0;
  std::vector<std::pair<int64_t, double>> row;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t a = rowptr_[i], e = rowptr_[i + 1];
    bool sorted = true;
    for (int64_t k = a; k < e; ++k) {
      MCG_CHECK(cols_[k] >= 0 && cols_[k] < n, "csr: column index out of range");
      const int64_t d = cols_[k] > i ? cols_[k] - i : i - cols_[k];
      bw = std::max(bw, d);
      far += d > kFarOffset ? 1 : 0;
      if (k > a && cols_[k] < cols_[k - 1]) sorted = false;
    }
    if (!sorted) {  // the SpMV engines do not care; ascending order keeps the halo windows and tests simple
      row.clear();
      for (int64_t k = a; k < e; ++k) row.emplace_back(cols_[k], vals_[k]);
      std::sort(row.begin(), row.end(), [](auto& x, auto& y) { return x.first < y.first; });
      for (int64_t k = a; k < e; ++k) {
        cols_[k] = row[k - a].first;
        vals_[k] = row[k - a].second;
      }
    }
  }
  view_.n = n;
  view_.bw = bw;
  view_.far = far;
  detect_stencil_();
  bind_();
}

// structured-grid stencil: the distinct column offsets are {0, +-1, +-L} (2-D, n a multiple of L)
// or {0, +-1, +-L, +-L^2} (3-D, n a multiple of L^2), L >= 2 (CsrMatrix::line / plane)
void HostMatrix::detect_stencil_() {
  view_.line = view_.plane = 0;
  const int64_t n = view_.n;
  std::vector<int64_t> offs;
  for (int64_t i = 0; i < n; ++i)
    for (int64_t k = rowptr_[i]; k < rowptr_[i + 1]; ++k) {
      const int64_t d = cols_[k] - i;
      if (std::find(offs.begin(), offs.end(), d) == offs.end()) {
        offs.push_back(d);
        if (offs.size() > 7) return;
      }
    }
  auto has = [&](int64_t d) { return std::find(offs.begin(), offs.end(), d) != offs.end(); };
  int64_t far[2] = {0, 0};
  int nf = 0;
  for (int64_t d : offs) {
    if (d == 0 || d == 1 || d == -1) continue;
    if (d < 0) {
      if (!has(-d)) return;  // the offsets of a symmetric stencil come in pairs
      continue;
    }
    if (nf == 2) return;
    far[nf++] = d;
  }
  if (!has(1) || !has(-1) || nf == 0) return;
  if (nf == 1) {
    const int64_t L = far[0];
    if (L >= 2 && n % L == 0 && n / L >= 2) view_.line = L;
    return;
  }
  const int64_t L = std::min(far[0], far[1]), P = std::max(far[0], far[1]);
  if (L >= 2 && P == L * L && n % P == 0 && n / P >= 2) {
    view_.line = L;
    view_.plane = P;
  }
}

void HostMatrix::bind_() {
  view_.rowptr = rowptr_.data();
  view_.cols = cols_.data();
  view_.vals = vals_.data();
  view_.b = b_.empty() ? nullptr : b_.data();
}

void HostMatrix::set_rhs(std::vector<double> b) {
  MCG_CHECK(b.empty() || (int64_t)b.size() == view_.n, "rhs length != matrix rows");
  b_ = std::move(b);
  bind_();
}

bool HostMatrix::symmetric_pattern_and_values() const {
  const int64_t n = view_.n;
  for (int64_t i = 0; i < n; ++i)
    for (int64_t k = rowptr_[i]; k < rowptr_[i + 1]; ++k) {
      const int64_t j = cols_[k];
      auto b = cols_.begin() + rowptr_[j], e = cols_.begin() + rowptr_[j + 1];
      auto it = std::lower_bound(b, e, i);
      if (it == e || *it != i || vals_[it - cols_.begin()] != vals_[k]) return false;
    }
  return true;
}

ProblemSpec HostMatrix::spec(RhsKind rhs, uint64_t seed) const {
  ProblemSpec s;
  s.kind = ProblemKind::Csr;
  s.csr = &view_;
  s.rhs = rhs;
  s.seed = seed;
  s.N = 0;
  return s;
}

namespace {
std::string lower(std::string s) {
  for (char& c : s) c = (char)std::tolower((unsigned char)c);
  return s;
}
}  // namespace

HostMatrix* read_matrix_market(const std::string& path) {
  std::ifstream f(path);
  if (!f) fail("matrix read failed", path);
  std::string line;
  if (!std::getline(f, line)) fail("matrix read failed", path + ": empty file");
  std::istringstream hs(lower(line));
  std::string banner, object, format, field, symmetry;
  hs >> banner >> object >> format >> field >> symmetry;
  if (banner != "%%matrixmarket" || object != "matrix" || format != "coordinate")
    fail("matrix read failed", path + ": not a Matrix Market coordinate matrix");
  const bool pattern = field == "pattern";
  if (!(field == "real" || field == "integer" || pattern)) fail("matrix read failed", path + ": field " + field);
  const bool sym = symmetry == "symmetric", skew = symmetry == "skew-symmetric";
  if (!(sym || skew || symmetry == "general")) fail("matrix read failed", path + ": symmetry " + symmetry);
  while (std::getline(f, line))
    if (!line.empty() && line[0] != '%') break;
  int64_t nr = 0, nc = 0, ne = 0;
  {
    std::istringstream ss(line);
    if (!(ss >> nr >> nc >> ne)) fail("matrix read failed", path + ": bad size line");
  }
  if (nr != nc) fail("matrix read failed", path + ": matrix is not square");
  std::vector<int64_t> I, J;
  std::vector<double> V;
  I.reserve(sym || skew ? 2 * ne : ne);
  J.reserve(I.capacity());
  V.reserve(I.capacity());
  for (int64_t k = 0; k < ne; ++k) {
    int64_t i, j;
    double v = 1.0;
    if (!(f >> i >> j)) fail("matrix read failed", path + ": truncated entries");
    if (!pattern && !(f >> v)) fail("matrix read failed", path + ": truncated entries");
    if (i < 1 || i > nr || j < 1 || j > nc) fail("matrix read failed", path + ": index out of range");
    --i;
    --j;
    I.push_back(i);
    J.push_back(j);
    V.push_back(v);
    if ((sym || skew) && i != j) {
      I.push_back(j);
      J.push_back(i);
      V.push_back(skew ? -v : v);
    }
  }
  // COO -> CSR, duplicates summed
  const int64_t n = nr;
  std::vector<int64_t> order(I.size());
  std::iota(order.begin(), order.end(), (int64_t)0);
  std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return I[a] != I[b] ? I[a] < I[b] : J[a] < J[b]; });
  std::vector<int64_t> rowptr(n + 1, 0), cols;
  std::vector<double> vals;
  cols.reserve(order.size());
  vals.reserve(order.size());
  int64_t pi = -1, pj = -1;
  for (int64_t k : order) {
    if (I[k] == pi && J[k] == pj) {
      vals.back() += V[k];
      continue;
    }
    pi = I[k];
    pj = J[k];
    cols.push_back(J[k]);
    vals.push_back(V[k]);
    ++rowptr[I[k] + 1];
  }
  for (int64_t i = 0; i < n; ++i) rowptr[i + 1] += rowptr[i];
  return new HostMatrix(n, std::move(rowptr), std::move(cols), std::move(vals));
}

std::vector<double> read_vector(const std::string& path) {
  std::ifstream f(path);
  if (!f) fail("vector read failed", path);
  // Matrix Market: only the dense `array` format (one value per line, column-major) is a vector;
  // a `coordinate` file's lines are "i j v" and reading their first number would take the row
  // indices as values, so it is refused.  Without a banner: one value per line.
  std::vector<double> v;
  std::string line;
  bool header_done = false, mm = false, first = true;
  int64_t want = -1;
  while (std::getline(f, line)) {
    if (line.empty()) continue;
    if (first && line[0] == '%') {
      first = false;
      const std::string l = lower(line);
      if (l.rfind("%%matrixmarket", 0) == 0) {
        mm = true;
        std::istringstream ss(l);
        std::string banner, object, fmt, field;
        ss >> banner >> object >> fmt >> field;
        if (object != "matrix" || fmt != "array")
          fail("vector read failed", path + ": Matrix Market vector must be 'matrix array' (got '" + object + " " +
                                         fmt + "')");
        if (field == "complex") fail("vector read failed", path + ": complex vectors are not supported");
      }
      continue;
    }
    first = false;
    if (line[0] == '%') continue;
    std::istringstream ss(line);
    if (mm && !header_done) {  // "rows cols" of an array file: a column vector
      int64_t nr = 0, nc = 0;
      if (!(ss >> nr >> nc) || nr < 0 || nc != 1)
        fail("vector read failed", path + ": array size line must be 'rows 1'");
      want = nr;
      header_done = true;
      continue;
    }
    double x;
    if (ss >> x) v.push_back(x);
  }
  if (mm && !header_done) fail("vector read failed", path + ": missing size line");
  if (want >= 0 && (int64_t)v.size() != want)
    fail("vector read failed", path + ": " + std::to_string(v.size()) + " values, size line says " +
                                   std::to_string(want));
  return v;
}

}  // namespace mcg
