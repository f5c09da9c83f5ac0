// User matrices: host-owned global CSR (the reference's input form — a CSR triple handed to
// cusparseCreateCsr, CUDACG.cu:93-117,213-216) and a Matrix Market reader.
//
// A HostMatrix owns the arrays; ProblemSpec{kind = Csr, csr = &m.view()} points at them.  Every
// rank of a multi-GPU solve reads the whole matrix on the host and uploads only its own rows,
// with columns remapped into its ext layout (partition.hpp); the partition (nnz-balanced or
// all-gather) and the ghost plan come from the actual columns.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "mcg/problem.hpp"

namespace mcg {

class HostMatrix {
 public:
  HostMatrix() = default;
  // takes a 0-based CSR (row pointers n + 1, columns, values; b optional: empty = none);
  // validates shape and index ranges, sorts each row's columns, computes the bandwidth
  HostMatrix(int64_t n, std::vector<int64_t> rowptr, std::vector<int64_t> cols, std::vector<double> vals,
             std::vector<double> b = {});
  HostMatrix(const HostMatrix&) = delete;
  HostMatrix& operator=(const HostMatrix&) = delete;

  const CsrMatrix& view() const { return view_; }
  int64_t n() const { return view_.n; }
  int64_t nnz() const { return view_.rowptr ? view_.rowptr[view_.n] : 0; }
  bool symmetric_pattern_and_values() const;  // A == A^T (exact)
  const std::vector<double>& rhs() const { return b_; }
  void set_rhs(std::vector<double> b);  // length n (or empty: none)
  ProblemSpec spec(RhsKind rhs = RhsKind::Reference, uint64_t seed = 1234) const;

 private:
  void bind_();
  void detect_stencil_();  // CsrMatrix::line / plane
  std::vector<int64_t> rowptr_, cols_;
  std::vector<double> vals_, b_;
  CsrMatrix view_;
};

// Matrix Market "coordinate" files (real / integer / pattern; general / symmetric /
// skew-symmetric): duplicate entries are summed, symmetric storage is expanded to both
// triangles.  Throws mcg::Error on malformed input or a non-square matrix.
HostMatrix* read_matrix_market(const std::string& path);
// A dense vector from a Matrix Market "array" file or plain text (one value per line).
std::vector<double> read_vector(const std::string& path);

}  // namespace mcg
