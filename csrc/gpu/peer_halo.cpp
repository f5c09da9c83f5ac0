// PeerHaloComm: the CU-free halo transport (comm.hpp).  Ghost rows are pulled from the owners'
// buffers with copy engines (hipMemcpyDeviceToDeviceNoCU), ordered by flags written and waited on
// with stream memory operations; the all-reduce is delegated to the wrapped communicator.
//
// The reference has no communication at all (CUDACG.cu is one process on device 0, :87); this is
// the north star's halo (the SpMV reads neighbours' p, CUDACG.cu:288), moved off the
// compute units so it can run beside the resident pass; the lean carries instead read these mapped rows
// themselves (PassForm::halo_pull, carry_common.hpp PullBases) and the copies serve the other passes.
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>

#include "mcg/check.hpp"
#include "mcg/comm.hpp"
#include "mcg/partition.hpp"

namespace mcg {

namespace {
constexpr uint64_t kBlobMagic = 0x4D4347504852ull;  // "MCGPHR"
struct Entry {  // one mapped allocation: this process's pointer, its IPC handle, the offset inside it
  uint64_t ptr;
  hipIpcMemHandle_t handle;
  int64_t offset;
};
void put(std::string& s, const void* p, size_t n) { s.append(reinterpret_cast<const char*>(p), n); }
template <class T>
T get(const std::string& s, size_t& at) {
  MCG_CHECK(at + sizeof(T) <= s.size(), "peer halo: truncated handle blob");
  T v;
  std::memcpy(&v, s.data() + at, sizeof(T));
  at += sizeof(T);
  return v;
}
Entry make_entry(void* p) {
  Entry e{};
  e.ptr = reinterpret_cast<uint64_t>(p);
  void* base = nullptr;
  size_t size = 0;
  MCG_HIP(hipMemGetAddressRange(reinterpret_cast<hipDeviceptr_t*>(&base), &size, p), "peer halo: address range failed");
  e.offset = static_cast<char*>(p) - static_cast<char*>(base);
  MCG_HIP(hipIpcGetMemHandle(&e.handle, base), "peer halo: IPC handle failed");
  return e;
}
// a peer's allocation as this process addresses it: the same process (threads, or one rank) uses the
// plain pointer (enabling peer access to another device), another process opens the IPC handle
void* map_entry(const Entry& e, bool same_process, int64_t pdev, std::vector<void*>& opened) {
  int dev = 0;
  MCG_HIP(hipGetDevice(&dev), "get device failed");
  if (same_process) {
    if (pdev != dev) {
      const hipError_t r = hipDeviceEnablePeerAccess((int)pdev, 0);
      if (r != hipSuccess && r != hipErrorPeerAccessAlreadyEnabled) MCG_HIP(r, "peer halo: peer access failed");
      (void)hipGetLastError();
    }
    return reinterpret_cast<void*>(e.ptr);
  }
  void* base = nullptr;
  MCG_HIP(hipIpcOpenMemHandle(&base, e.handle, hipIpcMemLazyEnablePeerAccess), "peer halo: IPC open failed");
  opened.push_back(base);
  return static_cast<char*>(base) + e.offset;
}
// who made a handle blob: a per-process random token, not the pid (with a PID namespace per rank two
// processes can share a pid, and a foreign pointer taken for a local one would fault the first pull)
int64_t process_token() {
  static const int64_t tok = [] {
    std::random_device rd;
    const uint64_t t = (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count();
    return (int64_t)((((uint64_t)rd() << 32) ^ rd() ^ (t * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)getpid() << 17)) |
                     1ull);
  }();
  return tok;
}
size_t mailbox_bytes(int world) {
  return (size_t)2 * world * kern::kIpcArMax * sizeof(double) + (size_t)(world + 1) * sizeof(unsigned long long);
}
}  // namespace

PeerHaloComm::PeerHaloComm(std::shared_ptr<Communicator> inner, int rank, int world)
    : inner_(std::move(inner)), rank_(rank), world_(world) {
  MCG_CHECK(inner_ != nullptr && world >= 1 && rank >= 0 && rank < world, "peer halo: invalid rank / world");
  MCG_HIP(hipMalloc(&flags_, 2 * world * sizeof(uint64_t)), "device malloc failed(peer halo flags)");
  // ready[q] = 0 (no exchange yet: never a value an exchange waits for); done[q] = 1, the value
  // exchange 1 waits for ("exchange 0 copied"), so every exchange waits, the first one included, and
  // a graph that captures the first exchange replays correctly as a later one
  std::vector<uint64_t> init(2 * world, 0);
  for (int q = 0; q < world; ++q) init[world + q] = 1;
  MCG_HIP(hipMemcpy(flags_, init.data(), init.size() * sizeof(uint64_t), hipMemcpyHostToDevice),
          "memcpy from host to device failed(peer halo flags)");
  peer_bufs_.assign(world, {});
  peer_flags_.assign(world, nullptr);
  peer_own_off_.assign(world, 0);
  peer_row_begin_.assign(world, 0);
  mb_.rank = rank;
  mb_.world = world;
}

// The IPC all-reduce's mailbox, allocated on first use (only a run that asks for the IPC all-reduce
// maps mailboxes): uncached device memory (every access goes to memory, so a flag a peer wrote over
// the fabric is never served from a stale cache line), zeroed: call counters start at 0
void PeerHaloComm::ensure_mailbox_() {
  if (mbox_ != nullptr) return;
  MCG_CHECK(world_ <= kern::kIpcMaxRanks, "peer halo: too many ranks for the IPC all-reduce mailboxes");
  // (MCG_IPC_MAILBOX=cached: plain hipMalloc memory, a diagnostic)
  const size_t mb_bytes = mailbox_bytes(world_);
  const char* mk = std::getenv("MCG_IPC_MAILBOX");
  const bool cached = mk != nullptr && std::string(mk) == "cached";
  if (cached || hipExtMallocWithFlags(reinterpret_cast<void**>(&mbox_), mb_bytes, hipDeviceMallocUncached) != hipSuccess) {
    (void)hipGetLastError();
    mbox_ = nullptr;
    MCG_HIP(hipMalloc(&mbox_, mb_bytes), "device malloc failed(ipc mailbox)");
  }
  MCG_HIP(hipMemset(mbox_, 0, mb_bytes), "device memset failed(ipc mailbox)");
  MCG_HIP(hipDeviceSynchronize(), "device synchronize failed(ipc mailbox)");  // zeroed before any peer maps it
  MCG_HIP(hipHostMalloc(reinterpret_cast<void**>(&err_host_), sizeof(unsigned long long),
                        hipHostMallocMapped | hipHostMallocCoherent),
          "host malloc failed(ipc all-reduce)");
  *err_host_ = 0;
  MCG_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&mb_.err), err_host_, 0), "host pointer mapping failed");
}

PeerHaloComm::~PeerHaloComm() {
  for (void* p : opened_) (void)hipIpcCloseMemHandle(p);
  if (flags_) (void)hipFree(flags_);
  if (mbox_) (void)hipFree(mbox_);
  if (err_host_) (void)hipHostFree(err_host_);
}

void PeerHaloComm::allreduce_sum(double* buf, size_t count, hipStream_t stream) {
  if (!ipc_ar_) {
    inner_->allreduce_sum(buf, count, stream);
    return;
  }
  kern::ipc_allreduce(buf, (int)count, mb_, ar_budget_seconds, stream);
}

void PeerHaloComm::check_async() {
  if (ipc_ar_ && err_host_ != nullptr && __atomic_load_n(err_host_, __ATOMIC_ACQUIRE) != 0) {
    fail("ipc all-reduce: a peer did not arrive", "waited " + std::to_string(ar_budget_seconds) + " s");
  }
  inner_->check_async();
}

bool PeerHaloComm::alt_allreduce_timed_out() {
  if (err_host_ == nullptr || __atomic_load_n(err_host_, __ATOMIC_ACQUIRE) == 0) return false;
  __atomic_store_n(err_host_, 0ull, __ATOMIC_RELEASE);
  return true;
}

std::string PeerHaloComm::mailbox_handle() {
  ensure_mailbox_();
  std::string s;
  const uint64_t magic = kBlobMagic + 1;
  const int64_t pid = process_token();
  int dev = 0;
  MCG_HIP(hipGetDevice(&dev), "get device failed");
  const int64_t d64 = dev;
  put(s, &magic, 8);
  put(s, &pid, 8);
  put(s, &d64, 8);
  const Entry e = make_entry(mbox_);
  put(s, &e, sizeof(Entry));
  return s;
}

void PeerHaloComm::attach_mailbox(const std::vector<std::string>& all) {
  MCG_CHECK((int)all.size() == world_, "ipc all-reduce: one mailbox handle per rank");
  ensure_mailbox_();
  const int64_t me = process_token();
  const size_t nslot = (size_t)2 * world_ * kern::kIpcArMax;
  for (int q = 0; q < world_; ++q) {
    double* mb = nullptr;
    if (q == rank_) {
      mb = mbox_;
    } else {
      size_t at = 0;
      const std::string& s = all[q];
      MCG_CHECK(get<uint64_t>(s, at) == kBlobMagic + 1, "ipc all-reduce: bad mailbox handle");
      const int64_t pid = get<int64_t>(s, at), pdev = get<int64_t>(s, at);
      mb = static_cast<double*>(map_entry(get<Entry>(s, at), pid == me, pdev, opened_));
    }
    mb_.slots[q] = mb;
    mb_.flags[q] = reinterpret_cast<unsigned long long*>(mb + nslot);
  }
  mb_attached_ = true;
  ipc_ar_ = true;
}

void PeerHaloComm::register_halo_buffers(const std::vector<double*>& bufs, int64_t own_off, int64_t row_begin) {
  bufs_ = bufs;
  own_off_ = own_off;
  row_begin_ = row_begin;
  attached_ = false;
}

std::string PeerHaloComm::local_handles() const {
  std::string s;
  const uint64_t magic = kBlobMagic;
  const int64_t pid = process_token(), nb = (int64_t)bufs_.size();
  int dev = 0;
  MCG_HIP(hipGetDevice(&dev), "get device failed");
  const int64_t d64 = dev;
  put(s, &magic, 8);
  put(s, &pid, 8);
  put(s, &d64, 8);
  put(s, &nb, 8);
  put(s, &own_off_, 8);
  put(s, &row_begin_, 8);
  const Entry f = make_entry(flags_);
  put(s, &f, sizeof(Entry));
  for (double* b : bufs_) {
    MCG_CHECK(b != nullptr, "peer halo: null halo buffer");
    const Entry e = make_entry(b);
    put(s, &e, sizeof(Entry));
  }
  return s;
}

void PeerHaloComm::attach(const std::vector<std::string>& all) {
  MCG_CHECK((int)all.size() == world_, "peer halo: one handle blob per rank");
  const int64_t me = process_token();
  auto map = [&](const Entry& e, int64_t pid, int64_t pdev) { return map_entry(e, pid == me, pdev, opened_); };
  for (int q = 0; q < world_; ++q) {
    if (q == rank_) {
      peer_flags_[q] = flags_;
      peer_bufs_[q] = bufs_;
      peer_own_off_[q] = own_off_;
      peer_row_begin_[q] = row_begin_;
      continue;
    }
    size_t at = 0;
    const std::string& s = all[q];
    MCG_CHECK(get<uint64_t>(s, at) == kBlobMagic, "peer halo: bad handle blob");
    const int64_t pid = get<int64_t>(s, at), pdev = get<int64_t>(s, at), nb = get<int64_t>(s, at);
    peer_own_off_[q] = get<int64_t>(s, at);
    peer_row_begin_[q] = get<int64_t>(s, at);
    MCG_CHECK(nb == (int64_t)bufs_.size(), "peer halo: ranks registered different buffer lists");
    peer_flags_[q] = static_cast<uint64_t*>(map(get<Entry>(s, at), pid, pdev));
    peer_bufs_[q].resize(nb);
    for (int64_t i = 0; i < nb; ++i) peer_bufs_[q][i] = static_cast<double*>(map(get<Entry>(s, at), pid, pdev));
  }
  attached_ = true;
}

void PeerHaloComm::on_captured(bool kept) {
  const long n = cap_n_;
  cap_n_ = 0;
  if (!kept) {  // the capture was abandoned: its exchanges never run, the sequence resumes before them
    seq_ -= n;
    return;
  }
  MCG_CHECK(n % 2 == 0, "peer halo: a graph must hold an even number of exchanges (its flag values replay)");
}

bool PeerHaloComm::peer_view(int q, std::vector<double*>& bufs, int64_t& own_off, int64_t& row_begin) {
  MCG_CHECK(q >= 0 && q < world_, "peer halo: invalid rank");
  if (!attached_) return false;
  bufs = peer_bufs_[q];
  own_off = peer_own_off_[q];
  row_begin = peer_row_begin_[q];
  return true;
}

// A single (not parity-alternating) exchanged buffer -- the pipelined pass's w, the split pass's p --
// is rewritten by its owner's next update before the owner's next exchange, whose wait on the done
// flags would come too late: the solver calls this first (torn ghost rows otherwise).
// The readers' done flags of exchange seq_ carry v(seq_); the next exchange waits for the same value.
void PeerHaloComm::halo_fence(hipStream_t stream) {
  if (halo_inner_) {
    inner_->halo_fence(stream);
    return;
  }
  if (seq_ == 0 || last_readers_.empty()) return;
  const uint64_t v = 1 + (uint64_t)(seq_ % 2);
  for (int q : last_readers_)
    MCG_HIP(hipStreamWaitValue64(stream, flags_ + world_ + q, v, hipStreamWaitValueEq, ~0ull), "peer halo: wait failed");
}

std::vector<uintptr_t> PeerHaloComm::peer_buffers(int q) const {
  std::vector<uintptr_t> v;
  for (double* p : peer_bufs_.at(q)) v.push_back(reinterpret_cast<uintptr_t>(p));
  return v;
}

void PeerHaloComm::halo_exchange(const LocalLayout& L, double* const* ext_vecs, int nvec, hipStream_t stream,
                                 const int* widths) {
  if (!L.has_halo()) return;
  if (halo_inner_) {
    inner_->halo_exchange(L, ext_vecs, nvec, stream, widths);
    return;
  }
  for (int k = 0; k < nvec; ++k)  // a vector outside the iteration's set (true residual's temporary x)
    if (std::find(bufs_.begin(), bufs_.end(), ext_vecs[k]) == bufs_.end()) {
      inner_->halo_exchange(L, ext_vecs, nvec, stream, widths);
      return;
    }
  MCG_CHECK(attached_, "peer halo: attach() the peers' handles before the first exchange");
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  MCG_HIP(hipStreamIsCapturing(stream, &cs), "peer halo: capture query failed");
  if (cs == hipStreamCaptureStatusActive) ++cap_n_;
  ++seq_;
  const uint64_t v = 1 + (uint64_t)(seq_ % 2), vprev = 1 + (uint64_t)((seq_ - 1) % 2);
  std::vector<int> readers, sources;
  for (const HaloRange& h : L.sends)
    if (std::find(readers.begin(), readers.end(), h.peer) == readers.end()) readers.push_back(h.peer);
  for (const HaloRange& h : L.recvs)
    if (std::find(sources.begin(), sources.end(), h.peer) == sources.end()) sources.push_back(h.peer);
  // my rows of this exchange are final (the call follows the pass on this stream): tell my readers,
  // once each has copied my rows of the previous exchange (which this exchange's pass overwrote a
  // buffer parity later: the wait protects the one after)
  for (int q : readers) {
    MCG_HIP(hipStreamWaitValue64(stream, flags_ + world_ + q, vprev, hipStreamWaitValueEq, ~0ull),
            "peer halo: wait failed");
    MCG_HIP(hipStreamWriteValue64(stream, peer_flags_[q] + rank_, v, 0), "peer halo: flag write failed");
  }
  last_readers_ = readers;
  // pull: the owner's rows for my ghost ranges, per vector, once the owner's rows are final
  std::vector<int> idx(nvec);
  for (int k = 0; k < nvec; ++k) {
    auto it = std::find(bufs_.begin(), bufs_.end(), ext_vecs[k]);
    MCG_CHECK(it != bufs_.end(), "peer halo: vector not registered");
    idx[k] = (int)(it - bufs_.begin());
  }
  // every pull (source peer x vector) after its owner's ready flag -- the all-gather layout's blocks on
  // copy streams of their own -- then, on `stream`, the done flags that let each owner reuse its rows
  std::vector<CopyFan::Job> jobs;
  for (int q : sources) {
    // the owner's ext index of global row g: its own block starts at own_off(q) with row_begin(q);
    // ghost ranges come from its owned rows, located through the owner's registered layout numbers
    bool any = false;
    for (const HaloRange& h : L.recvs) {
      if (h.peer != q) continue;
      for (int k = 0; k < nvec; ++k) {
        const int64_t w = widths ? widths[k] : 1;
        const int64_t src_row = peer_own_off_.at(q) + (h.gbegin - peer_row_begin_.at(q));
        jobs.push_back({ext_vecs[k] + w * L.ext_index(h.gbegin), peer_bufs_[q][idx[k]] + w * src_row,
                        (size_t)(w * h.count) * sizeof(double), flags_ + q, v});
        any = true;
      }
    }
    if (!any) jobs.push_back({nullptr, nullptr, 0, flags_ + q, v});  // no rows from q: still wait for it
  }
  if (L.allgather) {
    fan_.run(stream, jobs);  // whole blocks from every peer: several copy engines at once
  } else {
    // a window halo's few small copies in one queue (fanned out over streams they took longer:
    // profiles/r4/fan); each waits for its owner's flag first
    for (const CopyFan::Job& j : jobs) {
      MCG_HIP(hipStreamWaitValue64(stream, j.wait_flag, j.wait_value, hipStreamWaitValueEq, ~0ull), "peer halo: wait failed");
      if (j.bytes > 0)
        MCG_HIP(hipMemcpyAsync(j.dst, j.src, j.bytes, hipMemcpyDeviceToDeviceNoCU, stream), "peer halo: copy failed");
    }
  }
  for (int q : sources)
    MCG_HIP(hipStreamWriteValue64(stream, peer_flags_[q] + world_ + rank_, v, 0), "peer halo: flag write failed");
}

}  // namespace mcg
