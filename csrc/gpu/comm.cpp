#include "mcg/comm.hpp"

#include <dlfcn.h>

#include <algorithm>
#include <cstring>

#include "mcg/check.hpp"
#include "mcg/kernels.hpp"

namespace mcg {

int rccl_version() {
  int v = 0;
  if (ncclGetVersion(&v) != ncclSuccess) v = 0;
  return v;
}

// the shared object that provides ncclGetVersion in this process: the one every RCCL call binds to
std::string rccl_library() {
  Dl_info info{};
  if (dladdr(reinterpret_cast<void*>(&ncclGetVersion), &info) != 0 && info.dli_fname) return info.dli_fname;
  return "?";
}

std::string unique_id_bytes() {
  ncclUniqueId id;
  MCG_RCCL(ncclGetUniqueId(&id), "RCCL unique id failed");
  return std::string(id.internal, sizeof(id.internal));
}

ncclUniqueId unique_id_from_bytes(const std::string& b) {
  MCG_CHECK(b.size() == sizeof(ncclUniqueId), "bad RCCL unique id size");
  ncclUniqueId id;
  std::memcpy(id.internal, b.data(), sizeof(id.internal));
  return id;
}

Comm::Comm(int rank, int world, const ncclUniqueId& reduce_id, const ncclUniqueId& halo_id)
    : rank_(rank), world_(world) {
  MCG_CHECK(world >= 1 && rank >= 0 && rank < world, "invalid rank/world");
  MCG_RCCL(ncclCommInitRank(&reduce_, world, reduce_id, rank), "RCCL communicator init failed(reduce)");
  MCG_RCCL(ncclCommInitRank(&halo_, world, halo_id, rank), "RCCL communicator init failed(halo)");
}

Comm::Comm(int rank, int world, const ncclUniqueId& id) : rank_(rank), world_(world) {
  MCG_CHECK(world >= 1 && rank >= 0 && rank < world, "invalid rank/world");
  MCG_RCCL(ncclCommInitRank(&reduce_, world, id, rank), "RCCL communicator init failed(reduce)");
  halo_ = reduce_;
}

Comm::~Comm() {
  if (aborted_) return;
  if (halo_ && halo_ != reduce_) (void)ncclCommDestroy(halo_);
  if (reduce_) (void)ncclCommDestroy(reduce_);
}

void Comm::allreduce_sum(double* buf, size_t count, hipStream_t stream) {
  MCG_RCCL(ncclAllReduce(buf, buf, count, ncclFloat64, ncclSum, reduce_, stream), "RCCL allreduce failed");
}

void Comm::halo_exchange(const LocalLayout& L, double* const* ext_vecs, int nvec, hipStream_t stream,
                         const int* widths) {
  if (!L.has_halo()) return;
  if (L.allgather) {
    // unstructured sparsity: every rank's block to every rank, in place (own_off = rank * block,
    // the recv buffer is the whole ext vector); one collective per vector in one group
    MCG_RCCL(ncclGroupStart(), "RCCL group failed");
    for (int v = 0; v < nvec; ++v) {
      const int64_t w = widths ? widths[v] : 1;
      MCG_RCCL(ncclAllGather(ext_vecs[v] + w * L.own_off, ext_vecs[v], (size_t)(w * L.block), ncclFloat64, halo_,
                             stream),
               "RCCL allgather failed");
    }
    MCG_RCCL(ncclGroupEnd(), "RCCL group failed");
    return;
  }
  MCG_RCCL(ncclGroupStart(), "RCCL group failed");
  // Matching rule: for each (me, peer) pair both sides post their messages in the
  // same order — vector-major, then ascending global row (make_layout builds
  // sends/recvs in ascending order).
  for (int v = 0; v < nvec; ++v) {
    const int64_t w = widths ? widths[v] : 1;
    for (const HaloRange& h : L.sends)
      MCG_RCCL(ncclSend(ext_vecs[v] + w * L.ext_index(h.gbegin), (size_t)(w * h.count), ncclFloat64, h.peer, halo_,
                        stream),
               "RCCL halo send failed");
    for (const HaloRange& h : L.recvs)
      MCG_RCCL(ncclRecv(ext_vecs[v] + w * L.ext_index(h.gbegin), (size_t)(w * h.count), ncclFloat64, h.peer, halo_,
                        stream),
               "RCCL halo recv failed");
  }
  MCG_RCCL(ncclGroupEnd(), "RCCL group failed");
}

void Comm::sendrecv(const double* send, int to, double* recv, int from, size_t n, hipStream_t stream) {
  MCG_RCCL(ncclGroupStart(), "RCCL group failed");
  MCG_RCCL(ncclSend(send, n, ncclFloat64, to, halo_, stream), "RCCL halo send failed");
  MCG_RCCL(ncclRecv(recv, n, ncclFloat64, from, halo_, stream), "RCCL halo recv failed");
  MCG_RCCL(ncclGroupEnd(), "RCCL group failed");
}

void Comm::allgather_inplace(double* buf, size_t block, hipStream_t stream) {
  MCG_RCCL(ncclAllGather(buf + (size_t)rank_ * block, buf, block, ncclFloat64, halo_, stream),
           "RCCL allgather failed");
}

void DelayComm::allreduce_sum(double*, size_t, hipStream_t stream) {
  if (ar_us_ > 0) kern::spin(nullptr, ar_us_, fat_, 1, stream);
}

void DelayComm::halo_exchange(const LocalLayout& L, double* const* ext_vecs, int nvec, hipStream_t stream,
                              const int* widths) {
  if (!L.has_halo()) return;
  if (copy_) {  // the messages' bytes through the copy engines (source: the rank's own first rows)
    // the all-gather layout's blocks side by side (CopyFan); window halos' small copies in one queue:
    // fanned out over streams they took longer (a P = 8 share of 16384^2: 0.507 vs 0.301 ms an
    // iteration, profiles/r4/fan)
    // (a receive range longer than the rank's own rows -- the last rank of an all-gather layout, whose
    // block is short -- copies only as many rows as it owns: the source stays inside its rows)
    std::vector<CopyFan::Job> jobs;
    for (int v = 0; v < nvec; ++v) {
      const int64_t w = widths ? widths[v] : 1;
      for (const HaloRange& h : L.recvs)
        jobs.push_back({ext_vecs[v] + w * L.ext_index(h.gbegin), ext_vecs[v] + w * L.own_off,
                        (size_t)(w * std::min(h.count, L.n_local())) * sizeof(double), nullptr, 0});
    }
    if (L.allgather) {
      fan_->run(stream, jobs);
    } else {
      for (const CopyFan::Job& j : jobs)
        MCG_HIP(hipMemcpyAsync(j.dst, j.src, j.bytes, hipMemcpyDeviceToDeviceNoCU, stream), "halo copy failed");
    }
    return;
  }
  if (halo_us_ > 0) kern::spin(nullptr, halo_us_, fat_, 1, stream);
}

int Comm::count() const {
  int n = 0;
  MCG_RCCL(ncclCommCount(reduce_, &n), "RCCL comm count failed");
  return n;
}

void Comm::check_async() {
  for (ncclComm_t c : {reduce_, halo_}) {
    if (c == nullptr) continue;
    ncclResult_t async = ncclSuccess;
    MCG_RCCL(ncclCommGetAsyncError(c, &async), "RCCL async error query failed");
    if (async != ncclSuccess) {
      abort();
      fail("RCCL asynchronous error", ncclGetErrorString(async));
    }
  }
}

void Comm::abort() {
  if (aborted_) return;
  aborted_ = true;
  if (halo_ && halo_ != reduce_) (void)ncclCommAbort(halo_);
  if (reduce_) (void)ncclCommAbort(reduce_);
}

CopyFan::~CopyFan() {
  for (hipStream_t st : st_) (void)hipStreamDestroy(st);
  for (hipEvent_t ev : ev_) (void)hipEventDestroy(ev);
  if (fork_) (void)hipEventDestroy(fork_);
}

void CopyFan::run(hipStream_t stream, const std::vector<Job>& jobs) {
  auto issue = [](hipStream_t st, const Job& j) {
    if (j.wait_flag != nullptr)
      MCG_HIP(hipStreamWaitValue64(st, j.wait_flag, j.wait_value, hipStreamWaitValueEq, ~0ull), "copy fan: wait failed");
    if (j.bytes > 0) MCG_HIP(hipMemcpyAsync(j.dst, j.src, j.bytes, hipMemcpyDeviceToDeviceNoCU, st), "copy fan: copy failed");
  };
  // never inside a graph capture: captured stream memory operations do not keep their order on this
  // stack (ROCm 7.2, gfx950).  bench/streamop_capture.cpp isolates it: a captured hipStreamWaitValue64
  // node never completes, a captured hipStreamWriteValue64 node never lands (the producer waiting for it
  // hangs), while the same operations enqueued eagerly order correctly and captured NoCU copies /
  // kernels alone replay fine (profiles/r5/capture/streamop_capture.jsonl).  r4's "SIGSEGV at P = 2"
  // with forked branches and the wrong results of the serial captured form were both this: a solver
  // whose halo runs through these flags is not captured (PeerHaloComm::halo_capturable is false for the
  // copy-engine halo, so the solver stays eager there; the in-kernel halo needs no flags and captures).
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  MCG_HIP(hipStreamIsCapturing(stream, &cs), "copy fan: capture query failed");
  MCG_CHECK(cs == hipStreamCaptureStatusNone || !std::any_of(jobs.begin(), jobs.end(), [](const Job& j) { return j.wait_flag != nullptr; }),
            "copy fan: flag-ordered copies cannot be captured (bench/streamop_capture.cpp)");
  if (jobs.size() <= 1 || cs != hipStreamCaptureStatusNone) {
    for (const Job& j : jobs) issue(stream, j);
    return;
  }
  const size_t ns = std::min<size_t>(jobs.size(), kMaxStreams);
  if (fork_ == nullptr) MCG_HIP(hipEventCreateWithFlags(&fork_, hipEventDisableTiming), "copy fan: event create failed");
  while (st_.size() < ns) {
    hipStream_t st = nullptr;
    hipEvent_t ev = nullptr;
    MCG_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "copy fan: stream create failed");
    MCG_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "copy fan: event create failed");
    st_.push_back(st);
    ev_.push_back(ev);
  }
  MCG_HIP(hipEventRecord(fork_, stream), "copy fan: event record failed");
  for (size_t i = 0; i < ns; ++i) MCG_HIP(hipStreamWaitEvent(st_[i], fork_, 0), "copy fan: stream wait failed");
  for (size_t j = 0; j < jobs.size(); ++j) issue(st_[j % ns], jobs[j]);
  for (size_t i = 0; i < ns; ++i) {
    MCG_HIP(hipEventRecord(ev_[i], st_[i]), "copy fan: event record failed");
    MCG_HIP(hipStreamWaitEvent(stream, ev_[i], 0), "copy fan: stream wait failed");
  }
}

}  // namespace mcg
