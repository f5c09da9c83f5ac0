// Native host unit tests (no GPU): generators, partition, halo plan, CPU CG.
// Built as build/test_host by the Makefile; run by tests/test_native_host.py.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <set>
#include <vector>

#include "mcg/cg.hpp"
#include "mcg/partition.hpp"
#include "mcg/problem.hpp"

using namespace mcg;

static int failures = 0;
#define EXPECT(c)                                                          \
  do {                                                                     \
    if (!(c)) {                                                            \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);    \
      ++failures;                                                          \
    }                                                                      \
  } while (0)

static ProblemSpec spec(ProblemKind k, int64_t N) {
  ProblemSpec s;
  s.kind = k;
  s.N = N;
  s.rhs = RhsKind::Random;
  return s;
}

static void test_nnz_formulas() {
  for (int64_t N : {1, 2, 3, 7, 16, 33}) {
    ProblemSpec s2 = spec(ProblemKind::Poisson2D, N);
    int64_t c = 0;
    for (int64_t i = 0; i < global_rows(s2); ++i) c += row_length(s2, i);
    EXPECT(c == closed_form_nnz(s2));
    ProblemSpec s3 = spec(ProblemKind::Poisson3D, N);
    c = 0;
    for (int64_t i = 0; i < global_rows(s3); ++i) c += row_length(s3, i);
    EXPECT(c == closed_form_nnz(s3));
  }
}

static void test_symmetry(const ProblemSpec& s) {
  std::map<std::pair<int64_t, int64_t>, double> m;
  const int64_t n = global_rows(s);
  for (int64_t i = 0; i < n; ++i) {
    int64_t prev = -1, cnt = 0;
    double diag = 0, off = 0;
    for_each_entry(s, i, [&](int64_t c, double v) {
      EXPECT(c > prev);  // ascending columns
      EXPECT(c >= 0 && c < n);
      EXPECT(std::llabs(c - i) <= bandwidth(s));
      prev = c;
      ++cnt;
      m[{i, c}] = v;
      if (c == i) diag = v; else off += std::fabs(v);
    });
    EXPECT(cnt == row_length(s, i));
    if (s.kind != ProblemKind::Demo) EXPECT(diag >= off);  // diagonal dominance
  }
  for (auto& kv : m) {
    auto it = m.find({kv.first.second, kv.first.first});
    EXPECT(it != m.end() && it->second == kv.second);
  }
}

static void test_partition_and_halo(const ProblemSpec& s, int P) {
  RowPartition part = partition_rows(s, P);
  EXPECT(part.offsets.front() == 0 && part.offsets.back() == global_rows(s));
  for (int r = 0; r < P; ++r) EXPECT(part.begin(r) <= part.end(r));
  std::vector<LocalLayout> L;
  for (int r = 0; r < P; ++r) L.push_back(make_layout(s, part, r));
  // every send has a matching recv on the peer, same global range, same order
  for (int r = 0; r < P; ++r) {
    EXPECT(L[r].own_off % 8 == 0);
    for (int q = 0; q < P; ++q) {
      if (q == r) continue;
      std::vector<HaloRange> s_rq, r_qr;
      for (auto& h : L[r].sends) if (h.peer == q) s_rq.push_back(h);
      for (auto& h : L[q].recvs) if (h.peer == r) r_qr.push_back(h);
      EXPECT(s_rq.size() == r_qr.size());
      for (size_t k = 0; k < s_rq.size() && k < r_qr.size(); ++k) {
        EXPECT(s_rq[k].gbegin == r_qr[k].gbegin);
        EXPECT(s_rq[k].count == r_qr[k].count);
      }
    }
    // every column of every owned row is owned or covered by exactly one recv
    std::set<int64_t> covered;
    for (auto& h : L[r].recvs)
      for (int64_t g = h.gbegin; g < h.gbegin + h.count; ++g) EXPECT(covered.insert(g).second);
    for (int64_t i = L[r].row_begin; i < L[r].row_end; ++i) {
      const bool interior = i - L[r].row_begin >= L[r].interior_begin && i - L[r].row_begin < L[r].interior_end;
      for_each_entry(s, i, [&](int64_t c, double) {
        const bool owned = c >= L[r].row_begin && c < L[r].row_end;
        EXPECT(owned || covered.count(c));
        if (interior) EXPECT(owned);
        EXPECT(L[r].ext_index(c) >= 0 && L[r].ext_index(c) < L[r].ext_len);
      });
    }
  }
}

static void test_cpu_demo_golden() {
  ProblemSpec s;  // demo
  CgOptions o;
  std::vector<double> x;
  CgResult r = cpu_cg(s, o, &x);
  EXPECT(r.iterations == 3);
  EXPECT(r.converged);
  char buf[64];
  const char* want[3] = {"0.500000", "0.750000", "1.000000"};
  for (int i = 0; i < 3; ++i) {
    std::snprintf(buf, sizeof buf, "%f", x[i]);
    EXPECT(std::string(buf) == want[i]);
  }
}

static void test_partitioned_matches(const ProblemSpec& s, int P) {
  CgOptions o;
  o.maxit = 60;
  o.tol = 1e-10;
  std::vector<double> x1, xp;
  CgResult a = cpu_cg(s, o, &x1);
  CgResult b = cpu_cg_partitioned(s, P, o, &xp);
  EXPECT(a.iterations == b.iterations);
  EXPECT(x1.size() == xp.size());
  double d = 0, m = 0;
  for (size_t i = 0; i < x1.size() && i < xp.size(); ++i) {
    d = std::max(d, std::fabs(x1[i] - xp[i]));
    m = std::max(m, std::fabs(x1[i]));
  }
  EXPECT(d <= 1e-9 * (1 + m));
}

int main() {
  test_nnz_formulas();
  test_symmetry(ProblemSpec{});
  test_symmetry(spec(ProblemKind::Poisson2D, 9));
  test_symmetry(spec(ProblemKind::Poisson3D, 5));
  ProblemSpec rs;
  rs.kind = ProblemKind::RandomSPD;
  rs.rows = 3000;
  rs.band = 40;
  rs.density = 0.3;
  test_symmetry(rs);
  for (int P : {1, 2, 3, 4, 8}) {
    test_partition_and_halo(spec(ProblemKind::Poisson2D, 16), P);
    test_partition_and_halo(spec(ProblemKind::Poisson3D, 8), P);
    test_partition_and_halo(rs, P);
  }
  test_partition_and_halo(spec(ProblemKind::Poisson2D, 4), 8);  // fewer grid lines than... n=16 rows
  test_partition_and_halo(ProblemSpec{}, 2);
  test_cpu_demo_golden();
  test_partitioned_matches(spec(ProblemKind::Poisson2D, 20), 3);
  test_partitioned_matches(spec(ProblemKind::Poisson3D, 9), 4);
  test_partitioned_matches(rs, 5);
  if (failures) {
    std::fprintf(stderr, "%d failures\n", failures);
    return 1;
  }
  std::printf("test_host: all passed\n");
  return 0;
}
