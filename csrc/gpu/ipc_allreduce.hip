// IPC all-reduce: the CG scalars summed through peer-mapped mailboxes (PeerHaloComm::set_ipc_allreduce).
//
// The reference's two global reductions (CUDACG.cu:304 p.Ap, :328 ||r||) become one 32-byte
// all-reduce per iteration in the single-reduction form.  RCCL does it between GPUs; it refuses two
// ranks on one GPU, so the one-GPU pool could never run a real P-rank recurrence across processes.
// This kernel needs only memory every rank can map (IPC handles between processes, plain pointers
// between threads, xGMI between GPUs): one wave per call
//   1. writes this rank's `count` doubles into slot [parity][rank] of EVERY rank's mailbox (itself
//      included), at system scope (write-through);
//   2. after a barrier and a system-scope release fence, raises its flag in every mailbox: flag[rank]
//      = the call's sequence number;
//   3. waits (bounded by a wall-clock budget; a peer that never arrives sets the error word, the sums
//      come out NaN and the kernel ends) until every rank's flag in its own mailbox has reached the
//      sequence number, then acquires;
//   4. sums the slots in rank order (the same bits on every rank) into `buf`.
// The sequence number is a device counter (mailbox flag[world]), so a hipGraph replays the kernel
// correctly.  Slots alternate by the call's parity: a rank reaches call s + 2 only after every rank
// deposited for s + 1, which each did after reading call s's slots, so a slot is never overwritten
// while it is read.
#include <hip/hip_runtime.h>

#include "mcg/check.hpp"
#include "mcg/kernels.hpp"

namespace mcg {
namespace kern {
namespace {

typedef __attribute__((address_space(1))) unsigned long long ar_u64;

__device__ __forceinline__ void st_sys64(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store((ar_u64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ unsigned long long ld_sys64(const unsigned long long* p) {
  return __hip_atomic_load((ar_u64*)const_cast<unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(64) void k_ipc_allreduce(double* __restrict__ buf, int count, const IpcMailboxes mb,
                                                      long long budget_ticks) {
  const int t = threadIdx.x;
  const int P = mb.world, me = mb.rank;
  unsigned long long* my_flags = mb.flags[me];
  unsigned long long seq = 0;
  if (t == 0) seq = my_flags[P] + 1;  // this rank's call counter (only this kernel writes it)
  seq = __shfl(seq, 0, 64);
  if (seq >> 63) {  // an earlier call gave up waiting (the sticky bit below): fail at once, no waiting
    if (t < count) buf[t] = __builtin_nan("");
    return;
  }
  const int par = (int)(seq & 1);
  for (int e = t; e < P * count; e += 64) {
    const int q = e / count, i = e % count;
    unsigned long long* slot = (unsigned long long*)(mb.slots[q] + ((size_t)(par * P + me)) * kIpcArMax + i);
    st_sys64(slot, (unsigned long long)__double_as_longlong(buf[i]));
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: the deposits before any flag
  if (t < P) st_sys64(&mb.flags[t][me], seq);
  bool ok = true;
  if (t < P) {
    const long long t0 = wall_clock64();
    while (ld_sys64(&my_flags[t]) < seq) {
      if (wall_clock64() - t0 > budget_ticks) {
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(4);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  // a peer that did not arrive: the error word for the host, NaN sums so the solver's breakdown latch
  // stops every later iteration at once, and the call counter not advanced but marked failed (the
  // mailboxes are out of step: the run ends, or the transport probe drops them; every later call
  // returns NaN at once instead of waiting out its budget again)
  const bool all_ok = __syncthreads_and(ok) != 0;
  if (!all_ok) {
    if (t == 0) {
      st_sys64(mb.err, 1ull);
      my_flags[P] = (seq - 1) | (1ull << 63);  // sticky: every later call fails at once
    }
    if (t < count) buf[t] = __builtin_nan("");
    return;
  }
  if (t < count) {
    const double* mine = mb.slots[me] + (size_t)(par * P) * kIpcArMax + t;
    double s = 0.0;
    for (int q = 0; q < P; ++q) s += __longlong_as_double((long long)ld_sys64((const unsigned long long*)(mine + (size_t)q * kIpcArMax)));
    buf[t] = s;
  }
  if (t == 0) my_flags[P] = seq;
}

}  // namespace

void ipc_allreduce(double* buf, int count, const IpcMailboxes& mb, double budget_seconds, hipStream_t stream) {
  MCG_CHECK(count >= 1 && count <= kIpcArMax && mb.world >= 1 && mb.world <= kIpcMaxRanks && mb.err != nullptr,
            "ipc all-reduce: bad arguments");
  for (int q = 0; q < mb.world; ++q) MCG_CHECK(mb.slots[q] && mb.flags[q], "ipc all-reduce: mailbox not mapped");
  static long long khz = 0;  // the wall clock's rate (s_memrealtime), per process
  if (khz == 0) {
    int dev = 0, rate = 0;
    MCG_HIP(hipGetDevice(&dev), "get device failed");
    MCG_HIP(hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, dev), "device attribute failed");
    khz = rate > 0 ? rate : 100000;
  }
  const long long ticks = (long long)(budget_seconds * 1e3 * (double)khz);
  hipLaunchKernelGGL(k_ipc_allreduce, dim3(1), dim3(64), 0, stream, buf, count, mb, ticks);
  MCG_HIP(hipGetLastError(), "ipc all-reduce launch failed");
}

}  // namespace kern
}  // namespace mcg
