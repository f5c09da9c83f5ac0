// CPU reference path (BASELINE.json config 1: "single-process CPU reference
// path").  Mirrors the reference's operation sequence (CUDACG.cu:244-352)
// one-for-one so it doubles as the numerical oracle for the GPU solver.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <thread>

#include "mcg/cg.hpp"
#include "mcg/check.hpp"

namespace mcg {

namespace {

int pick_threads(int threads, int64_t rows) {
  if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
  threads = std::min<int>(threads, 16);
  if (rows < 65536) threads = 1;
  return threads;
}

template <class F>
void parallel_rows(int64_t n, int threads, F&& f) {
  if (threads <= 1) { f(0, n); return; }
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t) {
    const int64_t a = n * t / threads, b = n * (t + 1) / threads;
    ts.emplace_back([&f, a, b] { f(a, b); });
  }
  for (auto& t : ts) t.join();
}

double dot(const double* a, const double* b, int64_t n) {
  double s = 0.0;
  for (int64_t i = 0; i < n; ++i) s += a[i] * b[i];
  return s;
}

}  // namespace

HostCsr build_local_csr(const ProblemSpec& s, const LocalLayout& L, int threads) {
  HostCsr A;
  const int64_t n = L.n_local();
  A.n_rows = n;
  A.rowptr.assign(n + 1, 0);
  threads = pick_threads(threads, n);
  parallel_rows(n, threads, [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) A.rowptr[i + 1] = row_length(s, L.row_begin + i);
  });
  for (int64_t i = 0; i < n; ++i) A.rowptr[i + 1] += A.rowptr[i];
  A.cols.resize(A.nnz());
  A.vals.resize(A.nnz());
  parallel_rows(n, threads, [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) {
      int64_t k = A.rowptr[i];
      const int64_t len = A.rowptr[i + 1] - k;
      for_each_entry(s, L.row_begin + i, [&](int64_t c, double v) {
        A.cols[k] = (int32_t)L.ext_index(c);
        A.vals[k] = v;
        ++k;
      }, len);
    }
  });
  return A;
}

std::vector<double> build_rhs(const ProblemSpec& s, int64_t r0, int64_t r1) {
  std::vector<double> b(r1 - r0);
  for (int64_t i = r0; i < r1; ++i) b[i - r0] = rhs_value(s, i);
  return b;
}

void csr_spmv(const HostCsr& A, const double* x_ext, double* y) {
  const int threads = pick_threads(0, A.n_rows);
  parallel_rows(A.n_rows, threads, [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) {
      double s = 0.0;
      for (int64_t k = A.rowptr[i]; k < A.rowptr[i + 1]; ++k) s += A.vals[k] * x_ext[A.cols[k]];
      y[i] = s;
    }
  });
}

CgResult cpu_cg(const ProblemSpec& s, const CgOptions& opt, std::vector<double>* x_out,
                std::vector<double>* hist) {
  using clk = std::chrono::steady_clock;
  CgResult res;
  const auto t0 = clk::now();
  RowPartition part = partition_rows(s, 1);
  LocalLayout L = make_layout(s, part, 0);
  HostCsr A = build_local_csr(s, L);
  const int64_t n = L.n_local();
  std::vector<double> b = build_rhs(s, 0, n);
  std::vector<double> x(n, 0.0), r(n), p(L.ext_len, 0.0), Ap(n);
  double* pown = p.data() + L.own_off;
  const auto t1 = clk::now();
  res.setup_seconds = std::chrono::duration<double>(t1 - t0).count();

  // r = b ; p = b ; rho = nrm2(r)^2            (CUDACG.cu:248-266)
  std::copy(b.begin(), b.end(), r.begin());
  std::copy(b.begin(), b.end(), pown);
  double rho = std::sqrt(dot(r.data(), r.data(), n));
  const double tol = opt.rtol > 0 ? opt.rtol * rho : opt.tol;  // r0 = b
  rho = rho * rho;
  int it = 0;
  for (; it < opt.maxit;) {
    csr_spmv(A, p.data(), Ap.data());                          // :288
    const double tmp = dot(pown, Ap.data(), n);                // :304
    const double alpha = rho / tmp;                            // :311
    for (int64_t i = 0; i < n; ++i) x[i] += alpha * pown[i];   // :314
    for (int64_t i = 0; i < n; ++i) r[i] += -alpha * Ap[i];    // :321
    ++it;
    const double rhop = rho;                                   // :327
    rho = std::sqrt(dot(r.data(), r.data(), n));               // :328
    if (hist) hist->push_back(rho);
    if (!std::isfinite(rho)) { res.breakdown = true; break; }
    if (rho < tol) { res.converged = true; break; }            // :333
    rho = rho * rho;                                           // :336
    const double beta = rho / rhop;                            // :339
    for (int64_t i = 0; i < n; ++i) pown[i] = beta * pown[i];  // :342
    for (int64_t i = 0; i < n; ++i) pown[i] += r[i];           // :347
  }
  res.iterations = it;
  res.rnorm = res.converged || res.breakdown ? rho : std::sqrt(rho);
  res.solve_seconds = std::chrono::duration<double>(clk::now() - t1).count();
  if (x_out) *x_out = std::move(x);
  return res;
}

CgResult cpu_cg_partitioned(const ProblemSpec& s, int world, const CgOptions& opt,
                            std::vector<double>* x_out, std::vector<double>* hist) {
  using clk = std::chrono::steady_clock;
  CgResult res;
  const auto t0 = clk::now();
  RowPartition part = partition_rows(s, world, opt.halo_mode);
  struct Rank {
    LocalLayout L;
    HostCsr A;
    std::vector<double> x, r, p, Ap;
  };
  std::vector<Rank> R(world);
  for (int q = 0; q < world; ++q) {
    R[q].L = make_layout(s, part, q);
    R[q].A = build_local_csr(s, R[q].L, 1);
    const int64_t n = R[q].L.n_local();
    std::vector<double> b = build_rhs(s, R[q].L.row_begin, R[q].L.row_end);
    R[q].x.assign(n, 0.0);
    R[q].r = b;
    R[q].p.assign(R[q].L.ext_len, 0.0);
    std::copy(b.begin(), b.end(), R[q].p.begin() + R[q].L.own_off);
    R[q].Ap.assign(n, 0.0);
  }
  const auto t1 = clk::now();
  res.setup_seconds = std::chrono::duration<double>(t1 - t0).count();

  // halo: each recv range of rank q is copied from the owner's owned block
  auto halo = [&]() {
    for (int q = 0; q < world; ++q) {
      for (const HaloRange& h : R[q].L.recvs) {
        const Rank& src = R[h.peer];
        std::memcpy(R[q].p.data() + R[q].L.ext_index(h.gbegin),
                    src.p.data() + src.L.ext_index(h.gbegin), h.count * sizeof(double));
      }
    }
  };
  auto allreduce = [&](auto&& local) {  // fixed rank order
    double s = 0.0;
    for (int q = 0; q < world; ++q) s += local(R[q]);
    return s;
  };

  double rho = std::sqrt(allreduce([](Rank& k) { return dot(k.r.data(), k.r.data(), k.L.n_local()); }));
  const double tol = opt.rtol > 0 ? opt.rtol * rho : opt.tol;
  rho = rho * rho;
  int it = 0;
  for (; it < opt.maxit;) {
    halo();
    for (auto& k : R) csr_spmv(k.A, k.p.data(), k.Ap.data());
    const double tmp = allreduce([](Rank& k) {
      return dot(k.p.data() + k.L.own_off, k.Ap.data(), k.L.n_local()); });
    const double alpha = rho / tmp;
    for (auto& k : R) {
      const int64_t n = k.L.n_local();
      double* pown = k.p.data() + k.L.own_off;
      for (int64_t i = 0; i < n; ++i) k.x[i] += alpha * pown[i];
      for (int64_t i = 0; i < n; ++i) k.r[i] += -alpha * k.Ap[i];
    }
    ++it;
    const double rhop = rho;
    rho = std::sqrt(allreduce([](Rank& k) { return dot(k.r.data(), k.r.data(), k.L.n_local()); }));
    if (hist) hist->push_back(rho);
    if (!std::isfinite(rho)) { res.breakdown = true; break; }
    if (rho < tol) { res.converged = true; break; }
    rho = rho * rho;
    const double beta = rho / rhop;
    for (auto& k : R) {
      const int64_t n = k.L.n_local();
      double* pown = k.p.data() + k.L.own_off;
      for (int64_t i = 0; i < n; ++i) pown[i] = beta * pown[i] + k.r[i];
    }
  }
  res.iterations = it;
  res.rnorm = res.converged || res.breakdown ? rho : std::sqrt(rho);
  res.solve_seconds = std::chrono::duration<double>(clk::now() - t1).count();
  if (x_out) {
    x_out->clear();
    for (auto& k : R) x_out->insert(x_out->end(), k.x.begin(), k.x.end());
  }
  return res;
}

}  // namespace mcg
