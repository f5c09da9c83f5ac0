// Communicators for the distributed CG solver (one rank = one GPU).
//
// The reference has no communication at all; the north star
// (BASELINE.json:5) moves the per-iteration global dot products and the
// boundary-row halo exchange onto RCCL over xGMI.
//
//   Comm (RCCL)   two communicators so the halo (side stream) and the scalar
//                 all-reduces (compute stream) can be in flight together (or, single-
//                 communicator mode, ONE communicator whose halo and all-reduce the solver
//                 issues in one stream order on the compute stream: serialized()):
//                 - reduce comm: ncclAllReduce(sum, f64) of the CG scalars, in place
//                   on device memory (CgState) — no host round trip
//                 - halo comm: ncclSend/ncclRecv inside ncclGroupStart/End straight
//                   from the owner's owned block into the receiver's ghost block
//                   (LocalLayout plan: contiguous ranges, no packing); for the
//                   all-gather layout (unstructured sparsity) one in-place
//                   ncclAllGather of equal row blocks per vector instead
//                 Bootstrap needs only the two ncclUniqueIds on every rank (the
//                 Python layer ships them over the torch.distributed store; the
//                 native CLI shares them between its per-GPU threads).
//   LocalComm     P ranks as host threads of ONE process sharing ONE device:
//                 all-reduce = D2D copies into a shared staging area + a fixed-order
//                 sum kernel; halo = D2D copies from the peer's owned block; stream
//                 ordering through events exchanged at host barriers.  RCCL refuses
//                 several ranks on one GPU, so this is how the multi-rank solver
//                 (partition, halo plan, interior/boundary split, overlap streams,
//                 collective placement) is exercised on a single MI355X.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "mcg/kernels.hpp"
#include "mcg/partition.hpp"

namespace mcg {

std::string unique_id_bytes();  // ncclGetUniqueId -> 128 raw bytes
int rccl_version();             // ncclGetVersion of the RCCL this process runs (e.g. 22606 = 2.26.6)
std::string rccl_library();     // path of the shared object that provides it
ncclUniqueId unique_id_from_bytes(const std::string& b);

// Several copy-engine copies (hipMemcpyDeviceToDeviceNoCU) at once: each on a stream of its own (up
// to kMaxStreams, then round robin), forked from and joined back to the caller's stream by events, so
// a graph captures them as branches.  One queue runs its copies one after another; a halo of 2 peers x
// 3 vectors of 128 KiB was 6 serial copies.  A job may first wait for a 64-bit flag (stream wait-value).
// Inside a graph capture (flag-free jobs only: captured wait / write-value nodes do not order on this
// stack, bench/streamop_capture.cpp) the copies stay on the caller's stream.
class CopyFan {
 public:
  static constexpr int kMaxStreams = 16;
  struct Job {
    void* dst;
    const void* src;
    size_t bytes;
    uint64_t* wait_flag;  // nullptr: no wait
    uint64_t wait_value;
  };
  CopyFan() = default;
  CopyFan(const CopyFan&) = delete;
  CopyFan& operator=(const CopyFan&) = delete;
  ~CopyFan();
  void run(hipStream_t stream, const std::vector<Job>& jobs);

 private:
  std::vector<hipStream_t> st_;
  std::vector<hipEvent_t> ev_;
  hipEvent_t fork_ = nullptr;
};

class Communicator {
 public:
  virtual ~Communicator() = default;
  virtual int rank() const = 0;
  virtual int world() const = 0;
  // in-place sum all-reduce of `count` doubles on `stream`
  virtual void allreduce_sum(double* buf, size_t count, hipStream_t stream) = 0;
  // exchange the halo rows of every vector in `ext_vecs` (ext layout of `L`);
  // `widths[v]` = doubles per row of vector v (nullptr: all 1; 2 = interleaved pairs)
  virtual void halo_exchange(const LocalLayout& L, double* const* ext_vecs, int nvec, hipStream_t stream,
                             const int* widths = nullptr) = 0;
  // poll for asynchronous errors; throws mcg::Error
  virtual void check_async() {}
  // whether the solver may capture this communicator's calls into a hipGraph
  virtual bool graph_capturable() const { return true; }
  // ... its halo exchanges too (the in-kernel halo's iterations hold none: only the all-reduce)
  virtual bool halo_capturable() const { return graph_capturable(); }
  // false for NullComm (per-rank timing rehearsal): setup-time agreements take this rank's own value
  virtual bool moves_data() const { return true; }
  // tear down outstanding collectives after a fatal error (watchdog)
  virtual void abort() {}
  // the caller is about to overwrite, on `stream`, rows it sent in its last halo exchange: wait until
  // every rank reading them has its copy.  A transport whose exchange returns before its readers have
  // copied (PeerHaloComm: the readers pull later, on their own streams) waits here; RCCL's send/recv
  // and LocalComm's copies complete in the exchange's stream order, so they have nothing to wait for
  virtual void halo_fence(hipStream_t) {}
  // true: halo and all-reduce share one communicator, so the solver must issue them in one stream
  // order (no side-stream halo; CgOptions::overlap is forced off)
  virtual bool serialized() const { return false; }
  // true: the halo moves its bytes with copy engines (no compute units), so it can run while a pass
  // holds every CU (r4's halo_hide split the pass around it; r5 removed that for the in-kernel halo)
  virtual bool halo_cu_free() const { return false; }
  // true: peer_view() will give the peers' buffers once every rank has set up (and, for processes,
  // attached): the solver may then read its ghost lines straight from them (PassForm::halo_pull)
  virtual bool maps_peers() const { return false; }
  // the solver's halo-exchanged vectors (every rank registers the same list in the same order, once
  // its buffers are final): a transport that maps its peers' memory needs them
  // (own_off / row_begin: where this rank's owned rows start in those ext vectors, and their first
  // global row)
  virtual void register_halo_buffers(const std::vector<double*>&, int64_t /*own_off*/, int64_t /*row_begin*/) {}
  // the in-kernel halo (GpuCgSolver pull_): rank q's registered buffers as this process addresses them
  // (IPC-mapped, or plain pointers of another thread) and where its owned rows start in them; false:
  // this transport cannot map its peers (RCCL alone, NullComm, DelayComm)
  virtual bool peer_view(int /*q*/, std::vector<double*>& /*bufs*/, int64_t& /*own_off*/, int64_t& /*row_begin*/) {
    return false;
  }
  // a graph capture holding this communicator's operations has ended (the solver calls it after
  // hipStreamEndCapture; kept = false: the capture failed and its graph is dropped): a transport whose
  // captured operations replay fixed values checks / rewinds its sequence here
  virtual void on_captured(bool /*kept*/) {}
  // A second all-reduce transport the solver's transport probe (GpuCgSolver::probe_transport_) may time
  // against the first at setup: PeerHaloComm's IPC mailboxes, once every rank's is mapped, next to an
  // inner communicator that moves data.  ready: both exist; use: route allreduce_sum to it (true) or to
  // the first (false); timed_out: its bounded wait gave up since the last call (the error is cleared);
  // budget: seconds that wait may last before it gives up
  virtual bool alt_allreduce_ready() const { return false; }
  virtual void use_alt_allreduce(bool) {}
  virtual bool alt_allreduce_in_use() const { return false; }
  virtual bool alt_allreduce_timed_out() { return false; }
  virtual void set_alt_allreduce_budget(double) {}
  virtual double alt_allreduce_budget() const { return 0.0; }
};

class Comm final : public Communicator {
 public:
  Comm(int rank, int world, const ncclUniqueId& reduce_id, const ncclUniqueId& halo_id);
  // single-communicator mode: halo and all-reduce on one communicator (serialized())
  Comm(int rank, int world, const ncclUniqueId& id);
  ~Comm() override;
  Comm(const Comm&) = delete;
  Comm& operator=(const Comm&) = delete;

  int rank() const override { return rank_; }
  int world() const override { return world_; }
  void allreduce_sum(double* buf, size_t count, hipStream_t stream) override;
  void halo_exchange(const LocalLayout& L, double* const* ext_vecs, int nvec, hipStream_t stream,
                     const int* widths = nullptr) override;
  void check_async() override;
  // ranks in the communicator as RCCL sees them (ncclCommCount)
  int count() const;
  bool serialized() const override { return halo_ == reduce_; }
  // one grouped point-to-point exchange on the halo communicator: send n doubles to `to`, receive
  // n doubles from `from` (either may be this rank: the loopback the 1-GPU tests capture in graphs)
  void sendrecv(const double* send, int to, double* recv, int from, size_t n, hipStream_t stream);
  // in-place all-gather of `block` doubles per rank on the halo communicator (buf: world * block)
  void allgather_inplace(double* buf, size_t block, hipStream_t stream);
  void abort() override;

 private:
  int rank_, world_;
  ncclComm_t reduce_ = nullptr;
  ncclComm_t halo_ = nullptr;
  bool aborted_ = false;
};

// Timing rehearsal of ONE rank of a P-rank run on a single GPU: the solver runs rank r's rows,
// ghost layout, interior / boundary launches, side-stream fork/join and graphs exactly as at P
// ranks, but the collectives move nothing (all-reduce: the local sums stay local; halo: no
// transfer, ghosts keep their values).  The numbers it computes are not the P-rank solve's; the
// time per iteration is the rank's own work without the communication latency.
class NullComm final : public Communicator {
 public:
  NullComm(int rank, int world) : rank_(rank), world_(world) {}
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  void allreduce_sum(double*, size_t, hipStream_t) override {}
  void halo_exchange(const LocalLayout&, double* const*, int, hipStream_t, const int* = nullptr) override {}
  bool moves_data() const override { return false; }

 private:
  int rank_, world_;
};

// Latency rehearsal: like NullComm, but every all-reduce and halo exchange costs a fixed
// device-side delay (a one-workgroup spin of `us` microseconds on the stream it is enqueued on),
// so the time an iteration spends waiting for a collective can be priced on one GPU.  `fat` spins
// with ~270 VGPRs per wave, RCCL's own kernel footprint (profiles/r3_corun_root_cause.md): such a
// wave cannot be placed next to a resident pass, the thin one (6 VGPRs) can.
class DelayComm final : public Communicator {
 public:
  // copy_halo: the halo is real copy-engine traffic of the layout's message sizes (each receive range
  // copied from this rank's own rows with hipMemcpyDeviceToDeviceNoCU: a timing stand-in for the
  // peer-to-peer copies, the ghosts get wrong values) instead of a spin
  DelayComm(int rank, int world, double allreduce_us, double halo_us, bool fat = false, bool copy_halo = false)
      : rank_(rank), world_(world), ar_us_(allreduce_us), halo_us_(halo_us), fat_(fat), copy_(copy_halo),
        fan_(std::make_unique<CopyFan>()) {}
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  void allreduce_sum(double*, size_t, hipStream_t stream) override;
  void halo_exchange(const LocalLayout& L, double* const*, int, hipStream_t stream, const int* = nullptr) override;
  bool moves_data() const override { return false; }
  bool halo_cu_free() const override { return copy_; }

 private:
  int rank_, world_;
  double ar_us_, halo_us_;
  bool fat_, copy_;
  std::unique_ptr<CopyFan> fan_;  // copy mode, all-gather layout: the blocks' copies side by side
};

// CU-free halo between the GPUs of one node (or processes / threads sharing one GPU): every rank
// maps its peers' halo buffers (IPC memory handles, exchanged out of band: attach()) and PULLS its
// ghost rows from the owners' rows with hipMemcpyAsync(..., hipMemcpyDeviceToDeviceNoCU) -- copy
// engines, no compute unit, so the copies run next to a pass that holds every CU
// (profiles/r4/corun: 2 x 128 KiB in 27-30 us beside the 16384^2 pass, RCCL 744 us).  Ordering
// without a host round trip: per peer two 64-bit flags in the RECEIVER's / OWNER's memory, written
// by stream memory operations (hipStreamWriteValue64) and waited on by the CP (hipStreamWaitValue64):
//   exchange s (value v(s) = 1 + s % 2, sense reversal; every rank makes the same calls):
//     for each rank q reading from me: wait done[q] == v(s - 1) (q copied my previous rows), then
//       write v(s) into q's ready[me] (my rows of this exchange are final: the call follows my pass)
//     for each rank q I read from: wait ready[q] == v(s), pull the ranges, write v(s) into q's done[me]
// The all-gather ghost layout (unstructured sparsity) takes the same path, every peer's block a range
// pulled on a stream of its own (CopyFan: several copy engines at once).
// The all-reduce goes to `inner` (RCCL, or NullComm in a one-GPU rehearsal), or, once
// attach_mailbox() has mapped every rank's mailbox, to the IPC all-reduce (ipc_allreduce.hip: each
// rank's sums written into every mailbox, a flag, a bounded wait, the slots summed in rank order) --
// which needs no RCCL, so P processes on ONE GPU run the real P-rank recurrence.
class PeerHaloComm final : public Communicator {
 public:
  PeerHaloComm(std::shared_ptr<Communicator> inner, int rank, int world);
  ~PeerHaloComm() override;
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  void allreduce_sum(double* buf, size_t count, hipStream_t stream) override;
  void halo_exchange(const LocalLayout& L, double* const* ext_vecs, int nvec, hipStream_t stream,
                     const int* widths = nullptr) override;
  void check_async() override;
  bool graph_capturable() const override { return inner_->graph_capturable() && capturable_; }
  // the copy-engine exchange replays from a hipGraph without its order: a 2-process solve with the
  // pulls captured drifts by 1.5e-2 in 40 iterations, eager it matches one rank to 1e-15
  // (bench/ipc_ranks.py --halo-pull 0, profiles/r5/capture; bench/streamop_capture.cpp)
  bool halo_capturable() const override { return graph_capturable() && (halo_inner_ ? inner_->halo_capturable() : false); }
  bool moves_data() const override { return ipc_ar_ || inner_->moves_data(); }
  void abort() override { inner_->abort(); }
  // the copy-engine halo never enters the inner communicator; with halo_via_inner it is the inner's
  bool serialized() const override { return halo_inner_ && inner_->serialized(); }
  bool halo_cu_free() const override { return !halo_inner_; }
  bool maps_peers() const override { return true; }
  // the mapping only (the in-kernel halo), the exchanges that remain (the first iterations, finalize,
  // the true residual) on the inner communicator's halo -- RCCL's send/recv: the P > 1 default, where
  // nothing but the pass's own pulled rows depends on the mapping
  void set_halo_via_inner(bool v) { halo_inner_ = v; }
  bool halo_via_inner() const { return halo_inner_; }
  void register_halo_buffers(const std::vector<double*>& bufs, int64_t own_off, int64_t row_begin) override;
  bool peer_view(int q, std::vector<double*>& bufs, int64_t& own_off, int64_t& row_begin) override;
  void on_captured(bool kept) override;
  void halo_fence(hipStream_t stream) override;
  // this rank's IPC handles (flags + registered buffers) as bytes, for an out-of-band all-gather
  std::string local_handles() const;
  // every rank's local_handles(), in rank order: map the peers' buffers (same process: plain pointers)
  void attach(const std::vector<std::string>& all);
  bool attached() const { return attached_; }
  void set_capturable(bool c) { capturable_ = c; }
  // test hook: the registered buffer list (device pointers) of rank q as mapped here
  std::vector<uintptr_t> peer_buffers(int q) const;
  // the IPC all-reduce: this rank's mailbox handle (the mailbox is allocated on this first use) for an
  // out-of-band all-gather, then every rank's, in rank order; from then on allreduce_sum runs through the
  // mailboxes (use_alt_allreduce(false) routes it back to the inner communicator)
  std::string mailbox_handle();
  void attach_mailbox(const std::vector<std::string>& all);
  bool ipc_allreduce() const { return ipc_ar_; }
  double ar_budget_seconds = 120.0;  // a peer that does not arrive for this long: error (check_async)
  bool alt_allreduce_ready() const override { return mb_attached_ && inner_->moves_data(); }
  void use_alt_allreduce(bool on) override { ipc_ar_ = on && mb_attached_; }
  bool alt_allreduce_in_use() const override { return ipc_ar_; }
  bool alt_allreduce_timed_out() override;
  void set_alt_allreduce_budget(double s) override { ar_budget_seconds = s; }
  double alt_allreduce_budget() const override { return ar_budget_seconds; }

 private:
  std::shared_ptr<Communicator> inner_;
  int rank_, world_;
  std::vector<double*> bufs_;
  uint64_t* flags_ = nullptr;  // [0, world): ready[q] (written by q), [world, 2 world): done[q]
  std::vector<std::vector<double*>> peer_bufs_;  // [q][i]
  std::vector<uint64_t*> peer_flags_;            // [q]
  int64_t own_off_ = 0, row_begin_ = 0;
  std::vector<int64_t> peer_own_off_, peer_row_begin_;
  std::vector<void*> opened_;                    // IPC mappings to close
  CopyFan fan_;                                  // the all-gather layout's pulls side by side
  double* mbox_ = nullptr;                       // uncached: [2][world][kIpcArMax] slots, then world + 1 u64 flags
  unsigned long long* err_host_ = nullptr;       // pinned, device-mapped error word of the IPC all-reduce
  kern::IpcMailboxes mb_;
  void ensure_mailbox_();
  bool mb_attached_ = false;  // every rank's mailbox mapped (attach_mailbox)
  bool ipc_ar_ = false;       // ... and the all-reduce runs through them
  bool halo_inner_ = false;
  long seq_ = 0;
  std::vector<int> last_readers_;  // the ranks that pull this rank's rows of exchange seq_
  long cap_n_ = 0;  // exchanges recorded by the capture in progress
  // A captured exchange replays the flag values of its capture, which continues the 1/2 alternation
  // only if every graph holds an even number of exchanges (the solver's graphs hold an even number
  // of iterations, one exchange each; on_captured() checks it).  Measured: stream write / wait value
  // and NoCU copies capture and replay (bench/gpu_run.py streamop)
  bool attached_ = false, capturable_ = true;
};

// Shared state of P in-process ranks on one device.
class LocalGroup {
 public:
  explicit LocalGroup(int world, size_t max_allreduce = 64);
  ~LocalGroup();
  int world() const { return world_; }
  // a rank failed: every rank waiting at (or later reaching) a barrier throws instead of waiting
  // for it forever (RCCL's ncclCommAbort, for threads)
  void abort();

 private:
  friend class LocalComm;
  void barrier();
  bool failed_ = false;
  int world_;
  size_t max_n_;
  double* staging_ = nullptr;  // [2 parities][world][max_n]
  std::vector<hipEvent_t> ev_copy_[2], ev_done_[2], ev_pre_, ev_post_;
  std::vector<double* const*> halo_vecs_;
  std::vector<const LocalLayout*> halo_layouts_;
  struct Reg {  // register_halo_buffers() of each rank (the in-kernel halo's peer views)
    std::vector<double*> bufs;
    int64_t own_off = 0, row_begin = 0;
  };
  std::vector<Reg> reg_;
  std::mutex m_;
  std::condition_variable cv_;
  int count_ = 0, gen_ = 0;
};

class LocalComm final : public Communicator {
 public:
  LocalComm(std::shared_ptr<LocalGroup> group, int rank);
  int rank() const override { return rank_; }
  int world() const override { return group_->world(); }
  void allreduce_sum(double* buf, size_t count, hipStream_t stream) override;
  void halo_exchange(const LocalLayout& L, double* const* ext_vecs, int nvec, hipStream_t stream,
                     const int* widths = nullptr) override;
  bool graph_capturable() const override { return false; }
  bool halo_cu_free() const override { return true; }  // hipMemcpyDeviceToDeviceNoCU (SDMA engines)
  bool maps_peers() const override { return true; }
  void register_halo_buffers(const std::vector<double*>& bufs, int64_t own_off, int64_t row_begin) override;
  bool peer_view(int q, std::vector<double*>& bufs, int64_t& own_off, int64_t& row_begin) override;

 private:
  std::shared_ptr<LocalGroup> group_;
  int rank_;
  long calls_ = 0;
};

}  // namespace mcg
