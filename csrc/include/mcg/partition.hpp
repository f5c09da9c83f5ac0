// 1-D row partition and halo plan.
//
// The reference is single-GPU (cudaSetDevice(0), CUDACG.cu:87) and has no
// partitioning at all; BASELINE.json:5 asks for the matrix to be 1-D
// row-partitioned across the GPUs of a node with a boundary-row halo exchange.
//
// Layout of a rank's vectors that the SpMV gathers from (r and p):
//
//     ext = [ pad | ghost_lo | owned rows | ghost_hi ]
//            ^pad so that `own_off` is a multiple of 8 doubles (64 B)
//
// ghost_lo / ghost_hi are the contiguous global ranges [col_lo, row_begin) and
// [row_end, col_hi) of the rank's column window, so halo messages are sent
// straight out of the owner's owned block and received straight into the ghost
// block — no pack/unpack kernels.  Local CSR column indices are stored in ext
// coordinates (ext_index(global)).
#pragma once

#include <cstdint>
#include <vector>

#include "mcg/problem.hpp"

namespace mcg {

struct RowPartition {
  std::vector<int64_t> offsets;  // size P+1, offsets[0] = 0, offsets[P] = n
  // all-gather ghost layout: every rank owns `block` rows (the last one fewer) and the ghosts are
  // every other rank's rows, refreshed by one ncclAllGather of equal blocks per vector
  bool allgather = false;
  int64_t block = 0;
  int world() const { return (int)offsets.size() - 1; }
  int64_t begin(int r) const { return offsets[r]; }
  int64_t end(int r) const { return offsets[r + 1]; }
};

// Equal-rows partition, aligned to the problem's partition granule (grid lines
// for 2-D, planes for 3-D) whenever there are at least P granules; nnz-balanced for
// randspd and user CSR matrices.  halo_mode: 0 = column-window halo (contiguous
// ghost ranges, point-to-point), 1 = all-gather of equal row blocks, -1 = auto: the
// all-gather when a rank's column window covers >= 3/4 of the other ranks' rows
// (unstructured sparsity: p2p ranges would move nearly the whole vector anyway).
RowPartition partition_rows(const ProblemSpec& s, int world, int halo_mode = -1);
// nnz-balanced partition from per-row lengths (prefix sums), used for irregular matrices.
RowPartition partition_by_weight(const std::vector<int64_t>& row_prefix, int world);

struct HaloRange {
  int peer;        // other rank
  int64_t gbegin;  // first global row of the range
  int64_t count;   // number of rows
};

struct LocalLayout {
  int rank = 0, world = 1;
  int64_t n_global = 0;
  int64_t row_begin = 0, row_end = 0;  // owned global rows
  int64_t col_lo = 0, col_hi = 0;      // column window (global)
  int64_t pad = 0;                     // leading padding of the ext vectors
  int64_t ext_len = 0;                 // length of ext vectors
  int64_t own_off = 0;                 // ext index of row_begin
  int64_t interior_begin = 0;          // local row range whose columns are all owned
  int64_t interior_end = 0;
  bool allgather = false;  // ghosts = all other ranks' rows via all-gather (RowPartition::allgather)
  int64_t block = 0;       // rows per rank block of the all-gather (own_off = rank * block)
  std::vector<HaloRange> sends;  // owned ranges other ranks need (ascending peer, row)
  std::vector<HaloRange> recvs;  // ghost ranges filled from other ranks (ascending peer, row)

  int64_t n_local() const { return row_end - row_begin; }
  int64_t ext_index(int64_t g) const { return g - col_lo + pad; }
  bool has_halo() const { return !sends.empty() || !recvs.empty(); }
  int64_t halo_rows_in() const;
  int64_t halo_rows_out() const;
};

// Column window [lo, hi) touched by global rows [r0, r1).
void column_window(const ProblemSpec& s, int64_t r0, int64_t r1, int64_t* lo, int64_t* hi);

LocalLayout make_layout(const ProblemSpec& s, const RowPartition& part, int rank);

}  // namespace mcg
