// HIP runtime RAII: device buffers, pinned host buffers, streams, events.
//
// Replaces the reference's raw cudaMalloc/cudaFree + CLEANUP teardown
// (CUDACG.cu:10-33,119-186).  Every allocation happens at setup; the iteration
// loop allocates nothing (the reference cudaMalloc's an SpMV workspace every
// iteration and leaks it, CUDACG.cu:281).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <string>
#include <utility>
#include <vector>

#include "mcg/check.hpp"

namespace mcg {

template <typename T>
class DeviceBuffer {
 public:
  DeviceBuffer() = default;
  // `pad` extra elements are allocated (and zeroed) past `n`: the LDS-staged
  // SpMV stages 16-B chunks that may straddle the last element.
  DeviceBuffer(size_t n, const char* what, size_t pad = 0) { allocate(n, what, pad); }
  ~DeviceBuffer() { release(); }
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;
  DeviceBuffer(DeviceBuffer&& o) noexcept { swap(o); }
  DeviceBuffer& operator=(DeviceBuffer&& o) noexcept {
    if (this != &o) { release(); swap(o); }
    return *this;
  }

  // `lead` elements are skipped at the front (the buffer starts `lead` elements past the
  // allocation: staggers the base addresses of streams read at the same index); room is left
  // for leads up to `lead_cap` (relead())
  void allocate(size_t n, const char* what, size_t pad = 0, size_t lead = 0, size_t lead_cap = 0) {
    release();
    lead_cap = lead_cap > lead ? lead_cap : lead;
    const size_t bytes = (lead_cap + n + pad) * sizeof(T);
    if (bytes) {
      MCG_HIP(hipMalloc(&base_, bytes), std::string("device malloc failed(") + what + ")");
      ptr_ = base_ + lead;
      if (pad) MCG_HIP(hipMemset(ptr_ + n, 0, pad * sizeof(T)), "device memset failed");
    }
    n_ = n;
    pad_ = pad;
    cap_ = lead_cap;
  }
  // move the start within the allocation (contents are not kept; the pad is re-zeroed)
  void relead(size_t lead) {
    MCG_CHECK(base_ != nullptr && lead <= cap_, "buffer lead beyond its allocation");
    ptr_ = base_ + lead;
    if (pad_) MCG_HIP(hipMemset(ptr_ + n_, 0, pad_ * sizeof(T)), "device memset failed");
  }
  size_t lead_capacity() const { return cap_; }
  void release() {
    if (base_) (void)hipFree(base_);
    base_ = ptr_ = nullptr;
    n_ = pad_ = cap_ = 0;
  }
  T* get() const { return ptr_; }
  size_t size() const { return n_; }
  size_t bytes() const { return n_ * sizeof(T); }
  void swap(DeviceBuffer& o) noexcept {
    std::swap(base_, o.base_);
    std::swap(ptr_, o.ptr_);
    std::swap(n_, o.n_);
    std::swap(pad_, o.pad_);
    std::swap(cap_, o.cap_);
  }

 private:
  T* base_ = nullptr;
  T* ptr_ = nullptr;
  size_t n_ = 0, pad_ = 0, cap_ = 0;
};

template <typename T>
class PinnedBuffer {
 public:
  PinnedBuffer() = default;
  explicit PinnedBuffer(size_t n) {
    MCG_HIP(hipHostMalloc(&ptr_, n * sizeof(T), hipHostMallocDefault), "host malloc failed(pinned)");
    n_ = n;
  }
  ~PinnedBuffer() {
    if (ptr_) (void)hipHostFree(ptr_);
  }
  PinnedBuffer(const PinnedBuffer&) = delete;
  PinnedBuffer& operator=(const PinnedBuffer&) = delete;
  PinnedBuffer(PinnedBuffer&& o) noexcept {
    std::swap(ptr_, o.ptr_);
    std::swap(n_, o.n_);
  }
  PinnedBuffer& operator=(PinnedBuffer&& o) noexcept {
    std::swap(ptr_, o.ptr_);
    std::swap(n_, o.n_);
    return *this;
  }
  T* get() const { return ptr_; }
  T& operator[](size_t i) const { return ptr_[i]; }

 private:
  T* ptr_ = nullptr;
  size_t n_ = 0;
};

class Stream {
 public:
  Stream() = default;
  explicit Stream(bool create, int priority = 0) {
    if (create)
      MCG_HIP(hipStreamCreateWithPriority(&s_, hipStreamNonBlocking, priority), "stream create failed");
  }
  // a stream whose kernels run only on the CUs set in `mask` (32 CUs per word)
  static Stream with_cu_mask(const std::vector<uint32_t>& mask) {
    Stream st;
    MCG_HIP(hipExtStreamCreateWithCUMask(&st.s_, (uint32_t)mask.size(), mask.data()), "stream create failed");
    return st;
  }
  ~Stream() {
    if (s_) (void)hipStreamDestroy(s_);
  }
  Stream(const Stream&) = delete;
  Stream& operator=(const Stream&) = delete;
  Stream(Stream&& o) noexcept { std::swap(s_, o.s_); }
  Stream& operator=(Stream&& o) noexcept {
    std::swap(s_, o.s_);
    return *this;
  }
  hipStream_t get() const { return s_; }
  operator hipStream_t() const { return s_; }

 private:
  hipStream_t s_ = nullptr;
};

class Event {
 public:
  Event() = default;
  explicit Event(bool create, bool timing = false) {
    if (create)
      MCG_HIP(hipEventCreateWithFlags(&e_, timing ? hipEventDefault : hipEventDisableTiming),
              "event create failed");
  }
  ~Event() {
    if (e_) (void)hipEventDestroy(e_);
  }
  Event(const Event&) = delete;
  Event& operator=(const Event&) = delete;
  Event(Event&& o) noexcept { std::swap(e_, o.e_); }
  Event& operator=(Event&& o) noexcept {
    std::swap(e_, o.e_);
    return *this;
  }
  hipEvent_t get() const { return e_; }
  operator hipEvent_t() const { return e_; }

 private:
  hipEvent_t e_ = nullptr;
};

}  // namespace mcg
