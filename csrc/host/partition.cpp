#include "mcg/partition.hpp"

#include <algorithm>

#include "mcg/check.hpp"

namespace mcg {

namespace {
// randspd: nnz-balanced partition from the EXPECTED row lengths per 1024-row
// density region (the generator draws densities per region, so row lengths vary
// by up to 7x between regions; exact counting would cost 2W hashes per row).
RowPartition partition_randspd(const ProblemSpec& s, int world) {
  const int64_t n = s.rows, W = s.band, R = 1024;
  const int64_t nreg = (n + R - 1) / R;
  std::vector<double> q(nreg);
  for (int64_t g = 0; g < nreg; ++g) q[g] = randspd_density(s, g * R);
  // prefix of q over rows (region-constant) to average the density of a row window
  std::vector<double> qpre(nreg + 1, 0.0);
  for (int64_t g = 0; g < nreg; ++g) qpre[g + 1] = qpre[g] + q[g] * (double)std::min(R, n - g * R);
  auto qsum_rows = [&](int64_t a, int64_t b) {  // sum of q over rows [a, b)
    a = std::max<int64_t>(0, a);
    b = std::min(n, b);
    if (b <= a) return 0.0;
    const int64_t ga = a / R, gb = (b - 1) / R;
    if (ga == gb) return q[ga] * (double)(b - a);
    return q[ga] * (double)((ga + 1) * R - a) + (qpre[gb] - qpre[ga + 1]) + q[gb] * (double)(b - gb * R);
  };
  std::vector<int64_t> prefix(nreg + 1, 0);
  const double qmean = qpre[nreg] / (double)std::max<int64_t>(1, n);
  for (int64_t g = 0; g < nreg; ++g) {
    const int64_t r0 = g * R, r1 = std::min(n, r0 + R), mid = (r0 + r1) / 2;
    // pairs {i-d, i} use the density of i-d's region; pairs {i, i+d} that of i's (wide offsets:
    // the lower partners are spread over the whole matrix -> the mean density)
    // scrambled: a row is a random base row, every region has the mean length
    const double left = (s.spread > 0 || s.scramble) ? qmean * (double)W : qsum_rows(mid - W, mid);
    const double right = (s.scramble ? qmean : q[g]) * (double)std::min(W, n - 1 - mid);
    prefix[g + 1] = prefix[g] + (int64_t)((double)(r1 - r0) * (1.0 + left + right));
  }
  RowPartition pr = partition_by_weight(prefix, world);
  for (auto& o : pr.offsets) o = std::min(n, o * R);
  pr.offsets.back() = n;
  return pr;
}
}  // namespace

RowPartition partition_rows(const ProblemSpec& s, int world, int halo_mode) {
  MCG_CHECK(world >= 1, "invalid number of ranks");
  MCG_CHECK(s.kind != ProblemKind::Csr || s.csr != nullptr, "csr problem without a matrix");
  const int64_t n = global_rows(s);
  if (world > 1 && halo_mode != 0) {
    const int64_t other = n - (n + world - 1) / world;  // rows of the other ranks (equal blocks)
    if (halo_mode == 1 || 8 * bandwidth(s) >= 3 * other) {
      RowPartition p;
      p.allgather = true;
      p.block = ((n + world - 1) / world + 63) / 64 * 64;  // whole 64-row SELL slices per block
      p.offsets.resize(world + 1);
      for (int r = 0; r <= world; ++r) p.offsets[r] = std::min(n, (int64_t)r * p.block);
      return p;
    }
  }
  if (s.kind == ProblemKind::RandomSPD && world > 1 && n / 1024 >= world) return partition_randspd(s, world);
  // nnz + rows balanced (a user matrix with a detected grid stencil is split at whole lines / planes below)
  if (s.kind == ProblemKind::Csr && world > 1 && (partition_granule(s) <= 1 || n / partition_granule(s) < world)) {
    std::vector<int64_t> w(n + 1);
    for (int64_t i = 0; i <= n; ++i) w[i] = s.csr->rowptr[i] + i;
    return partition_by_weight(w, world);
  }
  int64_t g = partition_granule(s);
  if (g < 1 || n / g < world) g = 1;
  const int64_t units = (n + g - 1) / g;
  RowPartition p;
  p.offsets.resize(world + 1);
  for (int r = 0; r <= world; ++r) {
    const int64_t u = units * r / world;
    p.offsets[r] = std::min(n, u * g);
  }
  p.offsets[world] = n;
  return p;
}

RowPartition partition_by_weight(const std::vector<int64_t>& row_prefix, int world) {
  MCG_CHECK(world >= 1 && !row_prefix.empty(), "invalid weighted partition input");
  const int64_t n = (int64_t)row_prefix.size() - 1;
  const int64_t total = row_prefix.back();
  RowPartition p;
  p.offsets.resize(world + 1);
  p.offsets[0] = 0;
  for (int r = 1; r < world; ++r) {
    const int64_t target = (int64_t)((__int128)total * r / world);
    // first row boundary whose prefix >= target
    int64_t b = std::lower_bound(row_prefix.begin(), row_prefix.end(), target) - row_prefix.begin();
    b = std::max(b, p.offsets[r - 1]);
    p.offsets[r] = std::min(b, n);
  }
  p.offsets[world] = n;
  return p;
}

void column_window(const ProblemSpec& s, int64_t r0, int64_t r1, int64_t* lo, int64_t* hi) {
  const int64_t n = global_rows(s), bw = bandwidth(s);
  if (r1 <= r0) { *lo = r0; *hi = r0; return; }
  if (s.kind == ProblemKind::Csr) {  // the actual columns of the rows
    int64_t a = r0, b = r1 - 1;
    const CsrMatrix& A = *s.csr;
    for (int64_t k = A.rowptr[r0]; k < A.rowptr[r1]; ++k) {
      a = std::min(a, A.cols[k]);
      b = std::max(b, A.cols[k]);
    }
    *lo = a;
    *hi = b + 1;
    return;
  }
  *lo = std::max<int64_t>(0, r0 - bw);
  *hi = std::min<int64_t>(n, r1 + bw);
}

int64_t LocalLayout::halo_rows_in() const {
  int64_t t = 0;
  for (auto& h : recvs) t += h.count;
  return t;
}
int64_t LocalLayout::halo_rows_out() const {
  int64_t t = 0;
  for (auto& h : sends) t += h.count;
  return t;
}

static void intersect(int64_t a0, int64_t a1, int64_t b0, int64_t b1, int64_t* c0, int64_t* c1) {
  *c0 = std::max(a0, b0);
  *c1 = std::min(a1, b1);
}

LocalLayout make_layout(const ProblemSpec& s, const RowPartition& part, int rank) {
  const int P = part.world();
  MCG_CHECK(rank >= 0 && rank < P, "invalid rank");
  LocalLayout L;
  L.rank = rank;
  L.world = P;
  L.n_global = global_rows(s);
  L.row_begin = part.begin(rank);
  L.row_end = part.end(rank);
  if (part.allgather) {
    // ext = the whole vector in global order, P blocks of `block` rows (the last one padded):
    // own_off = rank * block, so an in-place all-gather of `block` rows fills every ghost
    L.allgather = true;
    L.block = part.block;
    L.col_lo = 0;
    L.col_hi = (int64_t)P * part.block;
    L.pad = 0;
    L.own_off = (int64_t)rank * part.block;  // = row_begin unless the rank is empty (rows ran out)
    L.ext_len = L.col_hi;
    L.interior_begin = L.interior_end = 0;
    if (P == 1) L.interior_end = L.n_local();
    for (int q = 0; q < P; ++q) {
      if (q == rank) continue;
      if (part.end(q) > part.begin(q)) L.recvs.push_back({q, part.begin(q), part.end(q) - part.begin(q)});
      if (L.n_local() > 0) L.sends.push_back({q, L.row_begin, L.n_local()});
    }
    return L;
  }
  column_window(s, L.row_begin, L.row_end, &L.col_lo, &L.col_hi);
  if (L.row_end <= L.row_begin) { L.col_lo = L.col_hi = L.row_begin; }
  L.col_lo = std::min(L.col_lo, L.row_begin);
  L.col_hi = std::max(L.col_hi, L.row_end);
  const int64_t ghost_lo = L.row_begin - L.col_lo;
  L.pad = (8 - ghost_lo % 8) % 8;
  L.own_off = L.pad + ghost_lo;
  L.ext_len = L.pad + (L.col_hi - L.col_lo);

  // interior rows: every column inside [row_begin, row_end)
  const int64_t bw = bandwidth(s);
  int64_t ib = (L.row_begin == 0) ? 0 : L.row_begin + bw;
  int64_t ie = (L.row_end == L.n_global) ? L.n_global : L.row_end - bw;
  ib = std::min(std::max(ib, L.row_begin), L.row_end);  // band wider than the block: no interior rows
  ie = std::min(ie, L.row_end);
  if (ie < ib) ie = ib;
  L.interior_begin = ib - L.row_begin;
  L.interior_end = ie - L.row_begin;

  // halo: what I receive = my ghost ranges ∩ peers' owned; what I send = my owned ∩ peers' ghosts
  for (int q = 0; q < P; ++q) {
    if (q == rank) continue;
    const int64_t q0 = part.begin(q), q1 = part.end(q);
    int64_t c0, c1;
    intersect(L.col_lo, L.row_begin, q0, q1, &c0, &c1);
    if (c1 > c0) L.recvs.push_back({q, c0, c1 - c0});
    intersect(L.row_end, L.col_hi, q0, q1, &c0, &c1);
    if (c1 > c0) L.recvs.push_back({q, c0, c1 - c0});

    int64_t qlo, qhi;
    column_window(s, q0, q1, &qlo, &qhi);
    if (q1 <= q0) continue;
    intersect(qlo, q0, L.row_begin, L.row_end, &c0, &c1);
    if (c1 > c0) L.sends.push_back({q, c0, c1 - c0});
    intersect(q1, qhi, L.row_begin, L.row_end, &c0, &c1);
    if (c1 > c0) L.sends.push_back({q, c0, c1 - c0});
  }
  return L;
}

}  // namespace mcg
