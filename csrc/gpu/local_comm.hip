// LocalComm: P ranks as host threads of one process on one device (see comm.hpp).
//
// Ordering protocol (per call, all ranks in lockstep through host barriers):
//   all-reduce (parity p = call & 1):
//     wait every rank's ev_done[p] (its last read of staging[p], two calls ago)
//     copy buf -> staging[p][rank]; record ev_copy[p][rank]
//     barrier
//     wait every ev_copy[p][q]; sum staging[p][0..P) in rank order -> buf; record ev_done[p][rank]
//   halo: record ev_pre[rank]; publish (vecs, layout); barrier
//     for every recv range: wait ev_pre[peer]; D2D copy from the peer's owned block on the copy
//     engines (hipMemcpyDeviceToDeviceNoCU: the CU-free transport a real peer copy would use)
//     record ev_post[rank]; barrier; wait every ev_post[q] (no rank overwrites a
//     source block before every reader has copied it — RCCL send semantics)
// A rank re-records an event only after the next barrier, by which time every
// wait on its previous record has been issued, so no wait can see a later record.
#include <hip/hip_runtime.h>

#include "mcg/check.hpp"
#include "mcg/comm.hpp"

namespace mcg {

namespace {
__global__ __launch_bounds__(256) void k_sum_ranks(const double* __restrict__ staging, int P, size_t stride,
                                                   double* __restrict__ out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double s = 0.0;
  for (int q = 0; q < P; ++q) s += staging[q * stride + i];
  out[i] = s;
}
}  // namespace

LocalGroup::LocalGroup(int world, size_t max_allreduce) : world_(world), max_n_(max_allreduce) {
  MCG_CHECK(world >= 1, "invalid local group size");
  MCG_HIP(hipMalloc(&staging_, 2 * world * max_n_ * sizeof(double)), "device malloc failed(staging)");
  auto mk = [&](std::vector<hipEvent_t>& v) {
    v.resize(world);
    for (auto& e : v) MCG_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event create failed");
  };
  mk(ev_copy_[0]);
  mk(ev_copy_[1]);
  mk(ev_done_[0]);
  mk(ev_done_[1]);
  mk(ev_pre_);
  mk(ev_post_);
  halo_vecs_.assign(world, nullptr);
  halo_layouts_.assign(world, nullptr);
  reg_.assign(world, Reg{});
}

LocalGroup::~LocalGroup() {
  for (auto* v : {&ev_copy_[0], &ev_copy_[1], &ev_done_[0], &ev_done_[1], &ev_pre_, &ev_post_})
    for (auto e : *v) (void)hipEventDestroy(e);
  if (staging_) (void)hipFree(staging_);
}

void LocalGroup::barrier() {
  std::unique_lock<std::mutex> lk(m_);
  if (failed_) fail("another local rank failed");
  const int gen = gen_;
  if (++count_ == world_) {
    count_ = 0;
    ++gen_;
    cv_.notify_all();
    return;
  }
  cv_.wait(lk, [&] { return gen != gen_ || failed_; });
  if (gen == gen_) fail("another local rank failed");
}

void LocalGroup::abort() {
  std::lock_guard<std::mutex> lk(m_);
  failed_ = true;
  cv_.notify_all();
}

LocalComm::LocalComm(std::shared_ptr<LocalGroup> group, int rank) : group_(std::move(group)), rank_(rank) {
  MCG_CHECK(rank >= 0 && rank < group_->world(), "invalid local rank");
}

void LocalComm::allreduce_sum(double* buf, size_t count, hipStream_t stream) {
  LocalGroup& g = *group_;
  MCG_CHECK(count <= g.max_n_, "local all-reduce too large");
  const int P = g.world_;
  const int par = (int)(calls_++ & 1);
  double* stage = g.staging_ + (size_t)par * P * g.max_n_;
  if (calls_ > 2)
    for (int q = 0; q < P; ++q) MCG_HIP(hipStreamWaitEvent(stream, g.ev_done_[par][q], 0), "stream wait failed");
  MCG_HIP(hipMemcpyAsync(stage + (size_t)rank_ * g.max_n_, buf, count * sizeof(double), hipMemcpyDeviceToDevice,
                         stream),
          "local allreduce copy failed");
  MCG_HIP(hipEventRecord(g.ev_copy_[par][rank_], stream), "event record failed");
  g.barrier();
  for (int q = 0; q < P; ++q) MCG_HIP(hipStreamWaitEvent(stream, g.ev_copy_[par][q], 0), "stream wait failed");
  hipLaunchKernelGGL(k_sum_ranks, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, stream, stage, P, g.max_n_,
                     buf, count);
  MCG_HIP(hipGetLastError(), "local allreduce failed");
  MCG_HIP(hipEventRecord(g.ev_done_[par][rank_], stream), "event record failed");
}

// the in-kernel halo's peer views: each rank's buffers as registered (one process, plain pointers).  A
// solver asks for them at its first pulled pass, after every rank's setup registered (the all-reduces
// of reset() are host barriers in between)
void LocalComm::register_halo_buffers(const std::vector<double*>& bufs, int64_t own_off, int64_t row_begin) {
  LocalGroup& g = *group_;
  std::lock_guard<std::mutex> lk(g.m_);
  g.reg_[rank_] = LocalGroup::Reg{bufs, own_off, row_begin};
}

bool LocalComm::peer_view(int q, std::vector<double*>& bufs, int64_t& own_off, int64_t& row_begin) {
  LocalGroup& g = *group_;
  std::lock_guard<std::mutex> lk(g.m_);
  MCG_CHECK(q >= 0 && q < g.world_, "local peer view: invalid rank");
  const LocalGroup::Reg& r = g.reg_[q];
  if (r.bufs.empty()) return false;
  bufs = r.bufs;
  own_off = r.own_off;
  row_begin = r.row_begin;
  return true;
}

void LocalComm::halo_exchange(const LocalLayout& L, double* const* ext_vecs, int nvec, hipStream_t stream,
                              const int* widths) {
  LocalGroup& g = *group_;
  const int P = g.world_;
  MCG_HIP(hipEventRecord(g.ev_pre_[rank_], stream), "event record failed");
  g.halo_vecs_[rank_] = ext_vecs;
  g.halo_layouts_[rank_] = &L;
  g.barrier();
  for (const HaloRange& h : L.recvs) {
    MCG_HIP(hipStreamWaitEvent(stream, g.ev_pre_[h.peer], 0), "stream wait failed");
    const LocalLayout& Lp = *g.halo_layouts_[h.peer];
    for (int v = 0; v < nvec; ++v) {
      const int64_t w = widths ? widths[v] : 1;
      MCG_HIP(hipMemcpyAsync(ext_vecs[v] + w * L.ext_index(h.gbegin),
                             g.halo_vecs_[h.peer][v] + w * Lp.ext_index(h.gbegin), w * h.count * sizeof(double),
                             hipMemcpyDeviceToDeviceNoCU, stream),
              "local halo copy failed");
    }
  }
  MCG_HIP(hipEventRecord(g.ev_post_[rank_], stream), "event record failed");
  g.barrier();
  for (int q = 0; q < P; ++q) MCG_HIP(hipStreamWaitEvent(stream, g.ev_post_[q], 0), "stream wait failed");
}

}  // namespace mcg
