// RCCL communicator over xGMI (one rank per GPU).
//
// The reference has no communication at all; the north star
// (BASELINE.json:5) moves the per-iteration global dot products and the
// boundary-row halo exchange onto RCCL.  Two communicators are used so the
// halo (side stream) and the scalar all-reduces (compute stream) can be in
// flight at the same time without sharing one communicator's FIFO:
//
//   reduce comm : ncclAllReduce(sum, f64) of the 8-byte CG scalars, in place
//                 on device memory (CgState::pAp / rr_new) — no host round trip
//   halo comm   : ncclSend/ncclRecv inside ncclGroupStart/End straight from the
//                 owner's owned block into the receiver's ghost block (the
//                 LocalLayout plan: contiguous ranges, no packing)
//
// Bootstrap needs only the two ncclUniqueIds to reach every rank: the Python
// layer ships them over the torch.distributed store (torchrun), the native CLI
// shares them between its per-GPU threads.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <string>
#include <vector>

#include "mcg/partition.hpp"

namespace mcg {

std::string unique_id_bytes();                    // ncclGetUniqueId -> 128 raw bytes
ncclUniqueId unique_id_from_bytes(const std::string& b);

class Comm {
 public:
  Comm(int rank, int world, const ncclUniqueId& reduce_id, const ncclUniqueId& halo_id);
  ~Comm();
  Comm(const Comm&) = delete;
  Comm& operator=(const Comm&) = delete;

  int rank() const { return rank_; }
  int world() const { return world_; }

  // in-place sum all-reduce of `count` doubles on `stream`
  void allreduce_sum(double* buf, size_t count, hipStream_t stream);
  // exchange the halo rows of every vector in `ext_vecs` (ext layout of `L`)
  void halo_exchange(const LocalLayout& L, double* const* ext_vecs, int nvec, hipStream_t stream);
  // generic device-buffer collectives used by gathers / tests
  void allgather_bytes(const void* send, void* recv, size_t bytes_per_rank, hipStream_t stream);
  void broadcast_bytes(void* buf, size_t bytes, int root, hipStream_t stream);
  // poll for asynchronous RCCL errors; throws mcg::Error
  void check_async();
  void abort();

 private:
  int rank_, world_;
  ncclComm_t reduce_ = nullptr;
  ncclComm_t halo_ = nullptr;
  bool aborted_ = false;
};

}  // namespace mcg
